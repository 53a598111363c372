"""Variable-length Cmds through the payload heap on the CPU tier (the device
step code compiled for the host, tests/soa_cpu, with the engine's input
staging, rbe_host.h), against the oracle harness.

A Cmd longer than 16 bytes lives once in the engine's payload heap; every
replica's entry refers to it by (fingerprint, heap position), so Replicate
messages carry the reference, never the bytes.  Parity: every replica field
and the trace digest (which folds the Cmd fingerprint, oracle/harness.cpp
hash_entry) round by round; limitSize (entryutils.go:50-63) splits Replicates
by 128 + len(Cmd) per entry when MaxEntrySize is small.  The bytes read back
with rbe_get_entry_cmds are the ones the host pushed."""
import pytest

import oracle as O
from dragonboat_amd.engine import RBE_E_INVALID, RBE_E_STATE, EngineError, InputError
from heap_util import check_logs, mixed_cmd
from input_util import run_driven
from parity_util import C2, C3
from soa_cpu.soa import SoaCpu

DRIVEN = dict()


def _pair(kw, heap_bytes, **eng_more):
    eng = SoaCpu(trace=True, heap_bytes=heap_bytes, **dict(kw, **DRIVEN, **eng_more))
    return eng, O.Harness(**kw)


@pytest.mark.parametrize("name,kw,mes", [("C2", C2, 0), ("C2-small-batches", C2, 9000),
                                         ("C3", C3, 0)])
def test_mixed_size_proposals_parity(name, kw, mes):
    kw = dict(kw, n_groups=8, ext_inputs=True, max_entry_size=mes)
    ring = 128 if name == "C3" else 64
    eng, ref = _pair(kw, 64 << 20, ring=ring)
    pushed = set()

    def keep(ops):
        for kind, _, a in ops:
            if kind == "prop":
                pushed.update(c for _, c in a if len(c) > 16)

    d = run_driven(eng, ref, 150, seed=5, cmd=mixed_cmd, on_ops=keep, density=0.25)
    assert d is None, f"{name}: first divergence {d}"
    assert eng.faults()[0] == 0
    n = kw["n_replicas"]
    assert check_logs(eng, kw["n_groups"], n, ref.views(), ring, pushed) > 50


def test_heap_laps_report_compacted():
    """A heap smaller than the log window: entries whose bytes a later lap
    overwrote read as RBE_E_STATE (ErrCompacted); the protocol is unaffected."""
    kw = dict(C2, n_groups=4, ext_inputs=True)
    eng, ref = _pair(kw, 256 << 10)
    d = run_driven(eng, ref, 120, seed=9, cmd=lambda rng: rng.randbytes(4000), density=0.3)
    assert d is None, f"first divergence {d}"
    last = ref.views()[0].last_index
    with pytest.raises(EngineError, match=f"rc={RBE_E_STATE}"):
        eng.entry_cmds(0, max(1, last - 60), last)
    assert all(len(c) == 4000 for c in eng.entry_cmds(0, last, last) if c)


def test_heap_input_checks():
    eng = SoaCpu(trace=True, n_groups=2, n_replicas=3, ext_inputs=True, heap_bytes=64 << 10)
    with pytest.raises(InputError) as ei:  # more than a quarter of the heap
        eng.push_proposals([0], [[b"q" * (16 << 10 + 1)]])
    assert ei.value.rc == RBE_E_INVALID
    eng.push_proposals([0], [[b"q" * (16 << 10)]])
    eng.step()
    # a replica's batch may mix inline and heap Cmds
    eng.push_proposals([1, 2], [[b"a", b"b" * 300], [b"", b"c" * 17]])
    eng.step()
