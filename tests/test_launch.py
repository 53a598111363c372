"""rbe_launch on the CPU tier (the device step compiled for the host,
tests/soa_cpu): replicas restarted from persisted state (pb.State + the log
tail from the oracle's LogDB) continue bit-exact with the oracle harness
restarting the same nodes through Peer.Launch over their LogDB (peer.go:64-86,
raft.go:234-289 newRaft/loadState, logentry.go:86-96: nothing applied yet, the
committed entries are applied again).  Covers a single replica, a group's
leader, whole groups, restarts with a lagging applied index (ext_apply) and
the batch checks."""
import pytest

import oracle as O
from input_util import run_driven
from launch_util import restart
from parity_util import C2, C3, run_lockstep
from soa_cpu.soa import SoaCpu


def _leaders(views):
    return [i for i, v in enumerate(views) if v.role == O.LEADER]


@pytest.mark.parametrize("name,kw,extra", [("C2", C2, {}), ("C3", C3, dict())])
def test_restart_continues_with_oracle(name, kw, extra):
    kw = dict(kw, n_groups=10)
    eng, ref = SoaCpu(trace=True, **dict(kw, **extra)), O.Harness(**kw)
    assert run_lockstep(eng, ref, 45, every=1) is None
    n = kw["n_replicas"]
    lead = _leaders(ref.views())
    picks = [1, lead[0], lead[1]] + list(range(5 * n, 6 * n))  # a follower, leaders, a group
    restart(eng, ref, sorted(set(picks)), extra.get("ring", 64))
    d = run_lockstep(eng, ref, 60, every=1)
    assert d is None, f"{name}: first divergence after restart {d}"
    assert eng.faults()[0] == 0
    # the restarted leaders' groups elected again
    assert ref.counters()["campaigns"] > 0


def test_restart_with_lagging_applied():
    kw = dict(C2, n_groups=8, ext_inputs=True, ext_apply=True)
    # a restarted replica applies its log again from index 1 (processed =
    # firstIndex - 1): the window must still hold it
    dr = dict()
    eng, ref = SoaCpu(trace=True, **dict(kw, **dr)), O.Harness(**kw)

    def hook(rnd):
        if rnd in (30, 52):
            restart(eng, ref, [0, 4, 8, 9, 10, 11] if rnd == 30 else [1, 2, 7], 256)

    d = run_driven(eng, ref, 80, seed=21, ext_apply=True, before_round=hook)
    assert d is None, f"first divergence after restart {d}"
    assert eng.faults()[0] == 0


def test_launch_batch_checks():
    from dragonboat_amd.engine import InputError
    eng = SoaCpu(trace=True, n_groups=2, n_replicas=3)
    eng.run(5)
    good = [(1, 0, 3, 3)], [[(1, 1, 1, b""), (2, 1, 1, b""), (3, 1, 1, b"")]]
    with pytest.raises(InputError):  # replica out of range
        eng.launch([6], *good)
    with pytest.raises(InputError):  # entries not ending at last_index
        eng.launch([0], [(1, 0, 3, 4)], good[1])
    with pytest.raises(InputError):  # commit past the log
        eng.launch([0], [(1, 0, 5, 3)], good[1])
    with pytest.raises(InputError):  # the same replica twice
        eng.launch([0, 0], good[0] * 2, good[1] * 2)
    eng.launch([0], *good)


def test_restart_untraced_group_sleep():
    """Untraced C4 (lazy quiesced ticks, group sleep): restarting replicas of
    sleeping groups wakes them; state stays equal to the oracle."""
    from parity_util import C4
    kw = dict(C4, n_groups=40, wl_start_round=10)
    eng, ref = SoaCpu(trace=False, **kw), O.Harness(**kw)
    assert run_lockstep(eng, ref, 40, every=1, skip=("digest",)) is None
    restart(eng, ref, [0, 1, 2, 30, 61, 100], 64)
    d = run_lockstep(eng, ref, 260, every=1, skip=("digest",))
    assert d is None, f"first divergence after restart {d}"
