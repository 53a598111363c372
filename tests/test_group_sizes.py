"""Every group size the engine is built for (N = 1..7 voting slots; rbe_types.h
kMaxN): the device step compiled for the host (tests/soa_cpu) against the
oracle harness, round by round, on C2-shaped replication, C3-shaped leader
isolation (elections, vote tally, conflicts and backtracking), C4-shaped
quiesced ReadIndex traffic and the membership schedule.  The reference has no
fixed group size (raft.go keeps remotes in a map); quorum is the majority of
the voters whatever their number (raft.go:366-416 numVotingMembers/quorum), so
even sizes (2, 4, 6) need a strict majority — a 2-node group cannot elect
without both, a 4-node group needs 3.  N = 3..5 take the steady-state fast
steps, the other sizes the full handler table for every replica-round."""
import pytest

import oracle as O
from parity_util import C2, C3, C4, counters_match, run_lockstep
from soa_cpu.soa import SoaCpu
from test_membership import CATCHUP, MEMB

SIZES = [1, 2, 3, 4, 5, 6, 7]


def shapes(n):
    return {
        "C2": (dict(C2, n_groups=16, n_replicas=n), {}, 150),
        "C3": (dict(C3, n_groups=16, n_replicas=n, iso_mod=2), dict(), 260),
        "C4": (dict(C4, n_groups=30, n_replicas=n, wl_active_mod=2), {}, 200),
    }


@pytest.mark.parametrize("shape", ["C2", "C3", "C4"])
@pytest.mark.parametrize("n", SIZES)
def test_group_size_parity(n, shape):
    kw, extra, rounds = shapes(n)[shape]
    eng = SoaCpu(trace=True, **kw, **extra)
    ref = O.Harness(**kw)
    d = run_lockstep(eng, ref, rounds, every=1)
    assert d is None, f"N={n} {shape}: first divergence {d}"
    assert eng.faults()[0] == 0
    bad = counters_match(eng.counters(), ref.counters())
    assert not bad, f"counters differ {bad}"
    c = ref.counters()
    assert c["committed"] > 0
    if shape == "C3" and n > 1:
        assert c["campaigns"] > kw["n_groups"], "the isolations forced no elections"


@pytest.mark.parametrize("n", [2, 4, 6, 7])
def test_group_size_untraced(n):
    """The bench paths (untraced: lazy quiesced ticks, group sleep)."""
    kw, extra, rounds = shapes(n)["C4"]
    eng = SoaCpu(trace=False, **kw, **extra)
    ref = O.Harness(**kw)
    assert run_lockstep(eng, ref, rounds, every=1, skip=("digest",)) is None


@pytest.mark.parametrize("n", [4, 6, 7])
def test_group_size_membership(n):
    kw = dict(C3, n_groups=12, n_replicas=n, **MEMB)
    eng = SoaCpu(trace=True, **kw, **CATCHUP)
    ref = O.Harness(**kw)
    seen = set()
    for _ in range(6):
        assert run_lockstep(eng, ref, 50, every=1) is None
        seen |= {v.removed for v in ref.views()}
    assert eng.faults()[0] == 0
    assert len(seen) > 2, seen


def test_group_size_limits():
    from dragonboat_amd.engine import Engine  # noqa: F401  (config builder only)
    with pytest.raises(Exception):
        SoaCpu(trace=True, n_groups=2, n_replicas=8)
    with pytest.raises(Exception):
        SoaCpu(trace=True, n_groups=2, n_replicas=0)


@pytest.mark.parametrize("n,nv", [(5, 3), (4, 1), (6, 3), (7, 4)])
def test_spare_slots_join(n, nv):
    """Groups that start with nv voters and n - nv spare slots: nodes that join
    later (started with no peers and an empty log, node.go:280-292) and take
    part once the membership schedule's AddNode for them is applied — the
    leader catches them up from index 1 (raft.go:1135-1157 addNode/setRemote)."""
    kw = dict(C3, n_groups=12, n_replicas=n, n_voters=nv, **MEMB)
    eng = SoaCpu(trace=True, **kw, **CATCHUP)
    ref = O.Harness(**kw)
    grew = False
    for _ in range(6):
        d = run_lockstep(eng, ref, 50, every=1)
        assert d is None, f"N={n} V={nv}: first divergence {d}"
        full = (1 << n) - 1
        voters = [bin(full & ~v.removed).count("1") for v in ref.views()]
        grew |= max(voters) > nv
    assert eng.faults()[0] == 0
    assert grew, "no group ever grew beyond its initial voters"
    bad = counters_match(eng.counters(), ref.counters())
    assert not bad, f"counters differ {bad}"


def test_spare_slots_need_membership():
    with pytest.raises(Exception):
        SoaCpu(trace=True, n_groups=2, n_replicas=5, n_voters=3)
