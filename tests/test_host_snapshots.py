"""Host-driven snapshots (cfg.snapshot_entries with cfg.ext_apply): the host's
state machine applies the committed entries, and its snapshot worker decides
when to snapshot and how far to compact (node.go:585-692 saveSnapshotRequired /
doSaveSnapshot / compactSnapshot, 849-866 compactLog), telling the engine with
rbe_snapshot_saved / rbe_compact.  The oracle harness's TestLogDB is driven the
same way (harness_snapshot_saved / harness_compact).  Isolated replicas fall
behind the leaders' compaction markers and come back by InstallSnapshot
(raft.go:684-697) carrying the host's snapshot.

Bar: every view field, the trace digest and the snapshot state equal the
oracle's every round, on the device step compiled for the host
(tests/soa_cpu); the GPU twin is tests/test_gpu_host_snapshots.py."""
import random

import pytest

import oracle as O
from input_util import apply_engine, apply_oracle, plan_round
from parity_util import C3, C3_HOT, counters_match, view_diff
from soa_cpu.soa import SoaCpu

HOST_SNAP = dict(ext_inputs=True, ext_apply=True, snapshot_entries=1)
DRIVE = dict()
CASES = {
    "C3": dict(C3, n_groups=16, **HOST_SNAP),
    "C3_HOT": dict(C3_HOT, n_groups=16, **HOST_SNAP),
    "C3_N7": dict(C3, n_groups=12, n_replicas=7, **HOST_SNAP),
}


def run_host_snapshots(eng, ref, rounds, seed=3, every=12, overhead=3, skip=(), density=0.15,
                       ready=0.0):
    """Lockstep with host input and a snapshot worker: a replica whose applied
    index passed its last snapshot by `every` entries snapshots there (term from
    the oracle's log, the host's LogDB), and some rounds later asks for a
    compaction to index - `overhead`.  With `ready` > 0 the apply queue fills
    and drains too (rbe_set_apply_ready, sometimes twice for one replica in a
    step: the last call wins), so one step's input can hold an applied index,
    a ready flag, a snapshot and a compaction for the same replica.  Returns
    (snapshots saved, compactions, snapshots restored from InstallSnapshot)."""
    rng = random.Random(seed)
    n = eng.cfg.n_replicas
    n_rep = eng.n_rep
    applied = [0] * n_rep
    last_ss = [0] * n_rep
    pend = {}
    saved = compacted = restored = 0
    for rnd in range(rounds):
        views = ref.views()
        ops = plan_round(rng, n_rep, n, rnd, views, True, density, applied, ready=ready)
        if ready:  # a second, later apply-queue report for some replicas
            ops += [("ready", r, rng.random() < 0.5) for kind, r, _ in list(ops)
                    if kind == "ready" and rng.random() < 0.3]
        apply_engine(eng, ops)
        apply_oracle(ref, ops)
        if rnd >= 30:
            for r in range(n_rep):
                if r in pend and rng.random() < 0.4:
                    to = pend.pop(r)
                    eng.compact([r], [to])
                    ref.compact(r, to)
                    compacted += 1
                elif applied[r] > last_ss[r] + every and rng.random() < 0.5:
                    idx = applied[r]
                    term = ref.log_term(r // n, r % n, idx)
                    if term == 0:
                        continue
                    eng.snapshot_saved([r], [idx], [term])
                    ref.snapshot_saved(r, idx, term)
                    last_ss[r] = idx
                    if idx > overhead:
                        pend[r] = idx - overhead
                    saved += 1
        eng.step()
        ref.step()
        ev, hv = eng.views(), ref.views()
        for i in range(n_rep):
            d = view_diff(ev[i], hv[i], skip)
            assert d is None, f"round {rnd} replica {i}: {d}"
        es = eng.snapshot_state()
        for i in range(n_rep):
            os_ = ref.snapshot_state(i)
            assert tuple(es[i]) == os_, f"round {rnd} replica {i}: {tuple(es[i])} != {os_}"
            if os_[2] > last_ss[i]:  # a snapshot the host did not save here: restored
                restored += 1
                last_ss[i] = os_[2]
    bad = counters_match(eng.counters(), ref.counters())
    assert not bad, f"counters differ {bad}"
    return saved, compacted, restored


@pytest.mark.parametrize("name", list(CASES))
def test_host_driven_snapshots(name):
    kw = CASES[name]
    eng = SoaCpu(trace=True, **kw, **DRIVE)
    ref = O.Harness(**kw)
    saved, compacted, restored = run_host_snapshots(eng, ref, 300)
    assert eng.faults()[0] == 0
    assert saved > 20 and compacted > 10, (saved, compacted)
    assert restored > 0, "no laggard was brought back by InstallSnapshot"


def test_host_driven_snapshots_untraced():
    kw = CASES["C3_HOT"]
    eng = SoaCpu(trace=False, **kw, **DRIVE)
    ref = O.Harness(**kw)
    run_host_snapshots(eng, ref, 200, skip=("digest",))
    assert eng.faults()[0] == 0


def test_host_driven_snapshots_apply_queue():
    """Applied indexes, apply-queue flags (twice for some replicas), snapshots
    and compactions for the same replicas in one step's input."""
    kw = CASES["C3_HOT"]
    eng = SoaCpu(trace=True, **kw, **DRIVE)
    ref = O.Harness(**kw)
    saved, compacted, _ = run_host_snapshots(eng, ref, 200, ready=0.5)
    assert eng.faults()[0] == 0
    assert saved > 10 and compacted > 5, (saved, compacted)


def test_host_snapshot_checks():
    from dragonboat_amd.engine import InputError, RBE_E_INVALID, RBE_E_STATE
    own = SoaCpu(trace=True, n_groups=2, n_replicas=3, snapshot_entries=8)
    with pytest.raises(InputError) as ei:  # the engine snapshots by itself without ext_apply
        own.snapshot_saved([0], [1], [1])
    assert ei.value.rc == RBE_E_STATE
    eng = SoaCpu(trace=True, n_groups=2, n_replicas=3, **HOST_SNAP)
    eng.run(30)
    eng.notify_applied([0], [3])
    eng.step()
    with pytest.raises(InputError) as ei:  # beyond the applied index
        eng.snapshot_saved([0], [4], [1])
    assert ei.value.rc == RBE_E_INVALID
    with pytest.raises(InputError) as ei:  # removed voters need cfg.membership
        eng.snapshot_saved([0], [3], [1], [0b100])
    assert ei.value.rc == RBE_E_INVALID
    eng.snapshot_saved([0], [3], [1])
    with pytest.raises(InputError) as ei:  # one per replica per step
        eng.snapshot_saved([0], [2], [1])
    assert ei.value.rc == RBE_E_STATE
    eng.compact([0], [2])
    eng.step()
    assert tuple(eng.snapshot_state()[0][:4]) == (2, 1, 3, 1)
