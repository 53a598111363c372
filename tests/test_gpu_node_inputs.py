"""The node-layer boundary on the HIP engine (libdragonboat_amd.so through the C
ABI) against the oracle harness, round by round: host-pushed proposal batches,
ReadIndex, leader transfer, Unreachable / SnapshotStatus reports, the state
machine's lagging applied index, rounds without a tick, and the seeded
leader-transfer schedule (the TimeoutNow path of raft.go:1712-1734 /
1906-1916).  The CPU-tier twin is tests/test_node_inputs.py."""
import pytest

import oracle as O
from input_util import run_driven
from parity_util import C2, C3, C4, MIXED, run_lockstep, counters_match

pytestmark = pytest.mark.gpu

EXTRA = {"C3": dict(), "C3_N7": dict(), "MIXED": dict()}
DRIVEN = dict()  # see tests/test_node_inputs.py
DRIVEN_BY_NAME = {"C3_N7": dict()}
N7 = ("C3_N7", dict(C3, n_groups=24, n_replicas=7))


def _pair(kw, name="", trace=True, **more):
    from dragonboat_amd.engine import Engine
    kw = dict(kw, **more)
    eng_kw = dict(kw)
    eng_kw.update(EXTRA.get(name, {}))
    if kw.get("ext_inputs"):
        eng_kw.update(DRIVEN)
        eng_kw.update(DRIVEN_BY_NAME.get(name, {}))
    return Engine(device=0, trace=trace, **eng_kw), O.Harness(**kw)


@pytest.mark.parametrize("name,kw", [("C2", C2), ("C3", C3), ("C4", C4), N7])
def test_gpu_driven_inputs_parity(gpu_available, name, kw):
    kw = dict(kw, n_groups=min(kw["n_groups"], 16))
    eng, ref = _pair(kw, name, ext_inputs=True)
    d = run_driven(eng, ref, 160, seed=7)
    assert d is None, f"{name}: first divergence {d}"
    assert eng.fault_summary()[0] == 0
    eng.close()


def test_gpu_driven_inputs_with_lagging_applied(gpu_available):
    kw = dict(C3, n_groups=12)
    eng, ref = _pair(kw, "C3", ext_inputs=True, ext_apply=True)
    d = run_driven(eng, ref, 200, seed=11, ext_apply=True)
    assert d is None, f"first divergence {d}"
    assert eng.fault_summary()[0] == 0
    eng.close()


def test_gpu_apply_ready_gate(gpu_available):
    """rbe_set_apply_ready toggled at random with a lagging applied index
    (tests/test_node_inputs.py::test_apply_ready_gate on the HIP engine)."""
    from dragonboat_amd.engine import Engine
    kw = dict(C2, n_groups=12, ext_inputs=True, ext_apply=True)
    # a held replica's unapplied entries must stay in the device window
    eng = Engine(device=0, trace=True, **dict(kw, **dict(DRIVEN)))
    ref = O.Harness(**kw)
    d = run_driven(eng, ref, 200, seed=13, ext_apply=True, ready=0.2)
    assert d is None, f"first divergence {d}"
    assert eng.fault_summary()[0] == 0
    eng.close()


@pytest.mark.parametrize("trace", [True, False])
def test_gpu_rounds_without_tick(gpu_available, trace):
    kw = dict(C4, n_groups=24)
    eng, ref = _pair(kw, trace=trace, ext_inputs=True)
    d = run_driven(eng, ref, 300, seed=3, tick_every=2, density=0.05,
                   skip=() if trace else ("digest",))
    assert d is None, f"first divergence {d}"
    eng.close()


@pytest.mark.parametrize("name,kw", [("C2", C2), ("C3", C3), ("MIXED", MIXED), N7])
def test_gpu_leader_transfer_schedule_parity(gpu_available, name, kw):
    kw = dict(kw, xfer_period=23, xfer_mod=2)
    eng, ref = _pair(kw, name)
    d = run_lockstep(eng, ref, 400, every=1)
    assert d is None, f"{name}: first divergence {d}"
    assert eng.fault_summary()[0] == 0
    bad = counters_match(eng.counters(), ref.counters())
    assert not bad, f"{name}: counters differ {bad}"
    assert ref.counters()["campaigns"] > kw["n_groups"]
    eng.close()


def test_gpu_update_flags_and_events(gpu_available):
    """rbe_get_updates carries the listener events and the Update flags
    (HasUpdate, FastApply) of the last step."""
    from dragonboat_amd import engine as E
    eng, ref = _pair(dict(n_groups=2, n_replicas=3), ext_inputs=True)
    for _ in range(30):
        eng.step()
        ref.step()
    ups, rv = eng.updates(), ref.views()
    for i in range(6):
        assert ups[i].events == rv[i].events
    leaders = [i for i in range(6) if rv[i].role == O.LEADER]
    eng.push_proposals(leaders, [[b"abc"]] * len(leaders))
    eng.step()
    ups = eng.updates()
    for i in leaders:
        u = ups[i]
        assert u.flags & E.UF_HAS_UPDATE
        assert u.save_lo <= u.save_hi  # the appended entry is to be saved
    eng.close()


@pytest.mark.parametrize("quiesce", [False, True])
def test_gpu_leader_inputs_fast_path(gpu_available, quiesce):
    """Host ReadIndexes and single inline proposals at leaders on the HIP
    engine (k_fast_both's leader step takes them), bit-exact with the oracle."""
    import random
    from dragonboat_amd.engine import Engine
    from input_util import apply_engine, apply_oracle, leader_inputs_round
    from parity_util import counters_match, view_diff
    kw = dict(n_groups=40, n_replicas=3, quiesce=quiesce, ext_inputs=True)
    eng = Engine(device=0, trace=True, **kw)
    ref = O.Harness(**kw)
    rng = random.Random(17)
    views = ref.views()
    for rnd in range(260):
        if rnd >= 60:
            ops = leader_inputs_round(rng, views, 3, rnd)
            apply_engine(eng, ops)
            apply_oracle(ref, ops)
        eng.step()
        ref.step()
        ev, views = eng.views(), ref.views()
        for i in range(len(views)):
            d = view_diff(ev[i], views[i])
            assert d is None, f"round {rnd} replica {i}: {d}"
    assert not counters_match(eng.counters(), ref.counters())
    eng.close()
