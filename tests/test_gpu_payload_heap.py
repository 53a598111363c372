"""Variable-length Cmds on the HIP engine (cfg.heap_bytes, include/rbe.h):
mixed 0-16 B inline, 17-300 B and 1-4 KiB heap proposals pushed through
rbe_push_proposals (Peer.ProposeEntries, peer.go:117-123), against the oracle
harness round by round (every replica field and the trace digest, which folds
each heap Cmd's fingerprint).  A small MaxEntrySize makes limitSize
(entryutils.go:50-63) split Replicates and apply batches by 128 + len(Cmd).
The bytes read back with rbe_get_entry_cmds are the bytes the host pushed.
The CPU-tier twin is tests/test_payload_heap.py."""
import pytest

import oracle as O
from heap_util import check_logs, mixed_cmd
from input_util import run_driven
from parity_util import C2, C3

pytestmark = pytest.mark.gpu

DRIVEN = dict()


@pytest.mark.parametrize("name,kw,mes", [("C2", C2, 0), ("C2-small-batches", C2, 9000),
                                         ("C3", C3, 0)])
def test_gpu_mixed_size_proposals_parity(gpu_available, name, kw, mes):
    from dragonboat_amd.engine import Engine
    kw = dict(kw, n_groups=8, ext_inputs=True, max_entry_size=mes)
    ring = 128 if name == "C3" else 64
    eng = Engine(device=0, trace=True, heap_bytes=64 << 20, ring=ring, **dict(kw, **DRIVEN))
    ref = O.Harness(**kw)
    pushed = set()

    def keep(ops):
        for kind, _, a in ops:
            if kind == "prop":
                pushed.update(c for _, c in a if len(c) > 16)

    d = run_driven(eng, ref, 150, seed=5, cmd=mixed_cmd, on_ops=keep, density=0.25)
    assert d is None, f"{name}: first divergence {d}"
    assert eng.fault_summary()[0] == 0
    assert check_logs(eng, kw["n_groups"], kw["n_replicas"], ref.views(), ring, pushed) > 50
    # rbe_get_entries: the full length and the first 16 bytes of a heap Cmd
    v = ref.views()[0]
    ents = eng.entries(0, max(1, v.last_index - 10), v.last_index)
    cmds = eng.entry_cmds(0, max(1, v.last_index - 10), v.last_index)
    assert [e[3] for e in ents] == cmds
    eng.close()


def test_gpu_heap_laps_report_compacted(gpu_available):
    from dragonboat_amd.engine import Engine, EngineError, RBE_E_STATE
    kw = dict(C2, n_groups=4, ext_inputs=True)
    eng = Engine(device=0, trace=True, heap_bytes=256 << 10, **dict(kw, **DRIVEN))
    ref = O.Harness(**kw)
    d = run_driven(eng, ref, 120, seed=9, cmd=lambda rng: rng.randbytes(4000), density=0.3)
    assert d is None, f"first divergence {d}"
    last = ref.views()[0].last_index
    with pytest.raises(EngineError, match=f"rc={RBE_E_STATE}"):
        eng.entry_cmds(0, max(1, last - 60), last)
    eng.close()
