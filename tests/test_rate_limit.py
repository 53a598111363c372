"""Rate limiter on the engine (cfg.max_inmem_log_size; server/rate.go,
raft.go:660-683, 1779-1785, the inMemory size hooks of inmemory.go:139-246):
the device step logic compiled for the host (tests/soa_cpu) against the oracle
harness, round by round: views and trace digests (which fold every RateLimit
message with its Hint), Peer.RateLimited and rl.Get() of every replica.  The
oracle's limiter is pinned by the reference's own tests
(tests/test_oracle_rate.py)."""
import numpy as np
import pytest

import oracle as O
from parity_util import C2, C3_HOT, C4, ENGINE_EXTRA, MIXED, counters_match, run_lockstep
from soa_cpu.soa import SoaCpu

# limits around the in-memory window of these workloads (80 + 16 B per entry):
# small enough that replicas are limited often, and follower reports matter
CASES = {
    "C2": (C2, 300, 250),
    "C3_HOT": (C3_HOT, 400, 600),
    "C4": (C4, 400, 150),
    "MIXED": (MIXED, 500, 500),
    # InstallSnapshot restores (inMemory.restore: Set(0)) and LogDB compaction
    "C3_HOT_SNAP": (dict(C3_HOT, snapshot_entries=8, compaction_overhead=2), 400, 600),
    "C3_HOT_N7": (dict(C3_HOT, n_groups=24, n_replicas=7), 400, 600),
}


def _lockstep_rl(eng, ref, rounds, skip=()):
    limited_rounds = 0
    for rnd in range(rounds):
        d = run_lockstep(eng, ref, 1, every=1, skip=skip)
        assert d is None, f"round {rnd}: first divergence {d}"
        el, es = eng.rate_limited()
        rl, rs = ref.rate_limited()
        bad = np.nonzero(es != rs)[0]
        assert len(bad) == 0, (f"round {rnd}: in-memory size of replica {bad[0]}: "
                               f"engine {es[bad[0]]}, oracle {rs[bad[0]]}")
        bad = np.nonzero(el != rl)[0]
        assert len(bad) == 0, f"round {rnd}: RateLimited of replica {bad[0]} differs"
        limited_rounds += int(el.any())
    return limited_rounds


@pytest.mark.parametrize("mode", ["pipeline", "full_table"])
@pytest.mark.parametrize("name", list(CASES))
def test_rate_limiter_parity(name, mode):
    kw, rounds, limit = CASES[name]
    eng = SoaCpu(full_only=mode == "full_table", trace=True, max_inmem_log_size=limit, **kw,
                 **ENGINE_EXTRA.get(name.replace("_SNAP", ""), {}))
    ref = O.Harness(max_inmem_log_size=limit, **kw)
    limited = _lockstep_rl(eng, ref, rounds)
    assert limited > 0, "the limit never bit: the case tests nothing"
    n, bits = eng.faults()
    assert n == 0, f"faults {bits:#x}"
    bad = counters_match(eng.counters(), ref.counters())
    assert not bad, f"counters differ {bad}"


def test_rate_limiter_untraced():
    """The bench paths (no trace: lazy quiesced ticks, group sleep) keep the
    limiter's state exact."""
    kw, rounds, limit = CASES["C4"]
    eng = SoaCpu(trace=False, max_inmem_log_size=limit, **kw)
    ref = O.Harness(max_inmem_log_size=limit, **kw)
    assert _lockstep_rl(eng, ref, rounds, skip=("digest",)) > 0


def test_rate_limit_messages_reach_the_leader():
    """Followers report their in-memory size (RateLimit, Hint) every election
    timeout; the leader's limiter then counts the fresh reports."""
    kw = dict(C2, n_groups=8)
    eng = SoaCpu(trace=True, max_inmem_log_size=10**9, **kw)
    ref = O.Harness(max_inmem_log_size=10**9, **kw)
    _lockstep_rl(eng, ref, 120)
    # a huge limit is never reached, but the hooks still run
    el, es = eng.rate_limited()
    assert not el.any() and es.max() > 0


@pytest.mark.parametrize("name", ["C2", "C3"])
def test_rate_limiter_ext_commit(name):
    """Host-driven persistence (ext_commit): appliedLogTo runs inside the host's
    rbe_commit, which persists late or partly (tests/commit_util.py)."""
    from commit_util import run_commit_driven
    from parity_util import C3
    kw = dict({"C2": C2, "C3": C3}[name], n_groups=12, ext_inputs=True, ext_apply=True,
              ext_commit=True, max_inmem_log_size=400)
    eng = SoaCpu(trace=True, **kw)
    ref = O.Harness(**kw)
    # views and trace digests (RateLimit Hints) every round, the limiters at the end
    d, st = run_commit_driven(eng, ref, 160, seed=5)
    assert d is None, f"{name}: first divergence {d}"
    el, es = eng.rate_limited()
    rl, rs = ref.rate_limited()
    assert (es == rs).all() and (el == rl).all()
    assert eng.faults()[0] == 0
    assert st["committed"] > 100 and es.max() > 0, st


def relaunch_lagging_groups(eng, ref, rounds=90):
    """Relaunch whole groups whose replicas' commit lags their last index
    (rbe_launch: the in-memory log starts empty at last + 1,
    inMemory.init(lastIndex)), then keep the limiters in lockstep.  After the
    re-election a follower holds the new no-op in memory (over the limit) while
    its commit is still below the relaunched last index: its RateLimit Hint
    subtracts only the uncommitted entries the in-memory log holds,
    [max(committed + 1, markerIndex), last] (getUncommittedEntries,
    logentry.go:180-183, 205-211), not the LogDB's."""
    from launch_util import restart
    _lockstep_rl(eng, ref, 40)
    n = ref.n_replicas
    picks = []
    for g in range(len(ref.views()) // n):
        reps = list(range(g * n, (g + 1) * n))
        if all(ref.persisted(r)[2] < ref.persisted(r)[3] for r in reps):
            picks += reps
    assert len(picks) >= 3 * n, "too few groups with commit < last: the case tests nothing"
    restart(eng, ref, picks, 64)
    _lockstep_rl(eng, ref, rounds)
    return picks


def test_rate_limiter_after_relaunch():
    # a limit below one entry's in-memory size: every follower holding an entry is limited
    kw = dict(C2, n_groups=64)
    eng = SoaCpu(trace=True, max_inmem_log_size=50, **kw)
    ref = O.Harness(max_inmem_log_size=50, **kw)
    relaunch_lagging_groups(eng, ref)
    assert eng.faults()[0] == 0


def test_limiter_off_by_default():
    eng = SoaCpu(trace=True, **dict(C2, n_groups=4))
    with pytest.raises(Exception):
        eng.rate_limited()
