"""The spill tiers on the HIP engine (tests/test_spill.py is the CPU twin):
inputs the reference handles without limits — a 150-round isolation with
snapshots off, a node relaunched 500+ entries behind, a ReadIndex queue past
rq_cap, every list and queue of the planes overflowing — run bit-exact with
the oracle and fault-free with the engine's default capacities
(dragonboat_amd/csrc/rbe_spill.h)."""
import pytest

import oracle as O
from launch_util import restart
from parity_util import counters_match, run_lockstep
from test_spill import LONG_ISO, TINY

pytestmark = pytest.mark.gpu


def _check(eng, ref, rounds, skip=()):
    d = run_lockstep(eng, ref, rounds, every=1, skip=skip)
    assert d is None, f"first divergence {d}"
    n, bits = eng.fault_summary()
    assert n == 0, f"faults {bits:#x}"
    bad = counters_match(eng.counters(), ref.counters())
    assert not bad, f"counters differ {bad}"


@pytest.mark.parametrize("check_quorum", [True, False])
@pytest.mark.parametrize("mode", ["both", "full", "untraced"])
def test_gpu_long_isolation_cold_log(gpu_available, monkeypatch, check_quorum, mode):
    from dragonboat_amd.engine import Engine
    if mode == "full":
        monkeypatch.setenv("RBE_MODE", "full")
    kw = dict(LONG_ISO, check_quorum=check_quorum)
    trace = mode != "untraced"
    eng = Engine(device=0, trace=trace, **kw)
    ref = O.Harness(trace=trace, **kw)
    _check(eng, ref, 620, skip=() if trace else ("digest",))
    st = eng.spill_stats()
    assert st["oom"] == 0 and st["pool_pages_used"] > 0 and st["spill_peak_bytes"] > 0
    eng.close()


def test_gpu_relaunch_far_behind(gpu_available):
    from dragonboat_amd.engine import Engine
    kw = dict(n_groups=6, n_replicas=3, check_quorum=True, wl_enabled=True, wl_start_round=20,
              iso_period=600, iso_len=540, iso_mod=1)
    eng, ref = Engine(device=0, trace=True, **kw), O.Harness(**kw)
    assert run_lockstep(eng, ref, 600, every=20) is None
    isolated = [i for i, v in enumerate(ref.views()) if v.role == O.LEADER]
    assert len(isolated) == kw["n_groups"]
    assert run_lockstep(eng, ref, 540, every=20) is None
    views = ref.views()
    behind = min(max(views[g * 3 + k].last_index for k in range(3)) - views[r].last_index
                 for g, r in enumerate(isolated))
    assert behind > 500, behind
    restart(eng, ref, isolated, None)  # the whole LogDB through rbe_launch
    _check(eng, ref, 59)
    # the relaunched replicas' logs below the ring are readable at the boundary
    r = isolated[0]
    got = eng.entries(r, 1, 40)
    want = ref.persisted_entries(r, 1, 40)
    assert [(x[0], x[1]) for x in got] == [(e.index, e.term) for e in want]
    st = eng.spill_stats()
    assert st["pool_pages_used"] > 0 and st["spill_peak_bytes"] > 0 and st["oom"] == 0
    eng.close()


def test_gpu_readindex_queue_past_rq_cap(gpu_available):
    from dragonboat_amd.engine import Engine
    kw = dict(n_groups=4, n_replicas=3, check_quorum=True, wl_enabled=True,
              wl_start_round=20, wl_read_permille=0, wl_active_mod=4, iso_period=60,
              iso_len=30, iso_mod=1, ext_inputs=True)
    eng, ref = Engine(device=0, trace=True, rq_cap=8, **kw), O.Harness(**kw)
    assert run_lockstep(eng, ref, 60, every=1) is None
    leaders = [i for i, v in enumerate(ref.views()) if v.role == O.LEADER]
    longest = 0
    for rnd in range(12):
        for r in leaders:
            ctx = ((60 + rnd + 1) << 32 | (r + 1), 77 + rnd)
            eng.push_read_index([r], [ctx])
            ref.push(O.PUSH_READ, r, ctx[0], ctx[1])
        assert run_lockstep(eng, ref, 1, every=1) is None
        longest = max([longest] + [v.rq_count for v in eng.views()])
    assert longest > 8, f"the queue never passed rq_cap ({longest})"
    _check(eng, ref, 40)
    eng.close()


@pytest.mark.parametrize("caps", list(TINY))
@pytest.mark.parametrize("mode", ["both", "full"])
def test_gpu_lists_and_queues_past_capacity(gpu_available, monkeypatch, caps, mode):
    from dragonboat_amd.engine import Engine
    if mode == "full":
        monkeypatch.setenv("RBE_MODE", "full")
    kw = dict(n_groups=12, n_replicas=5, check_quorum=True, quiesce=True, wl_enabled=True,
              wl_start_round=25, wl_active_mod=2, wl_read_permille=500, iso_period=37,
              iso_len=20, iso_mod=2, seed=12345)
    eng = Engine(device=0, trace=True, **TINY[caps], **kw)
    ref = O.Harness(**kw)
    _check(eng, ref, 300)
    st = eng.spill_stats()
    assert st["spill_peak_bytes"] > 0 and st["pool_pages_used"] > 0 and st["oom"] == 0
    # the boundary reads the spilled lists and ReadyToReads: the collected
    # outputs of the last round equal the per-replica getters
    moff, msgs, roff, rtrs = eng.collect_outputs(0, eng.n_rep)
    for r in range(eng.n_rep):
        assert moff[r + 1] - moff[r] == len(eng.messages(r))
        assert roff[r + 1] - roff[r] == len(eng.ready_to_reads(r))
    eng.close()
