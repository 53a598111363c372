"""Membership change on the device (cfg.membership) on the CPU tier: the
device step compiled for the host (tests/soa_cpu) against the oracle
harness, round by round, every replica field (the removed-voter mask of each
replica's view included) and the trace digest.

Covered (reference internal/raft):
  * ProposeConfigChange at the leader (peer.go:126-135) → handleLeaderPropose
    with pendingConfigChange (raft.go:1587-1606; a second one is dropped for an
    empty entry, reportDroppedConfigChange 1983-1985);
  * the engine's state machine applying committed ConfigChange entries and
    handing them back at the next step (ApplyConfigChange, peer.go:138-149) →
    handleNodeConfigChange → addNode / removeNode (raft.go:1135-1198, 1537-1556);
  * quorum over the voters in tryCommit, vote tally, check-quorum, ReadIndex
    confirmation (raft.go:366-416, 886-907, 1060-1116);
  * a removed node: no elections (selfRemoved, raft.go:566-590, 1122-1133), a
    removed leader steps down, responses from non-members dropped (Peer.Handle,
    peer.go:186-198);
  * preLeaderPromotionHandleConfigChange (raft.go:1010-1018);
  * host-driven ApplyConfigChange / RejectConfigChange (ext_apply).
"""
import pytest

import oracle as O
from input_util import run_driven
from parity_util import C2, C3, MIXED, run_lockstep
from soa_cpu.soa import SoaCpu

# a voter added back is caught up from far behind in one Replicate: the entry
# arena and the in-memory window hold that many entries (the reference has no
# such capacities; the engine flags F_ARENA / F_WINDOW instead)
CATCHUP = dict()
EXTRA = {"C3": CATCHUP, "MIXED": CATCHUP, "C2": CATCHUP}
MEMB = dict(membership=True, cc_period=10, cc_mod=1)


def _removed_seen(ref, seen):
    for v in ref.views():
        seen.add(v.removed)


@pytest.mark.parametrize("name,kw", [("C2", C2), ("C3", C3), ("MIXED", MIXED)])
def test_membership_schedule_parity(name, kw):
    kw = dict(kw, n_groups=min(kw["n_groups"], 24), **MEMB)
    eng = SoaCpu(trace=True, **dict(kw, **EXTRA.get(name, {})))
    ref = O.Harness(**kw)
    seen = set()
    for _ in range(8):
        d = run_lockstep(eng, ref, 50, every=1)
        assert d is None, f"{name}: first divergence {d}"
        _removed_seen(ref, seen)
    assert eng.faults()[0] == 0
    assert len(seen) > 2, f"{name}: membership never changed {seen}"


def test_membership_full_table_only():
    kw = dict(C3, n_groups=16, **MEMB)
    eng = SoaCpu(trace=True, full_only=True, **dict(kw, **CATCHUP))
    ref = O.Harness(**kw)
    d = run_lockstep(eng, ref, 300, every=1)
    assert d is None, f"first divergence {d}"


def test_membership_untraced():
    kw = dict(C3, n_groups=16, **MEMB)
    eng = SoaCpu(trace=False, **dict(kw, **CATCHUP))
    ref = O.Harness(**kw)
    d = run_lockstep(eng, ref, 300, every=1, skip=("digest",))
    assert d is None, f"first divergence {d}"


def test_host_config_changes():
    """ext_apply: the host proposes config changes and applies / rejects the
    committed ones itself (rbe_propose_config_change / rbe_apply_config_change /
    rbe_reject_config_change), both sides driven identically."""
    import random
    kw = dict(C2, n_groups=6, ext_inputs=True, ext_apply=True, membership=True)
    eng = SoaCpu(trace=True, **dict(kw))
    ref = O.Harness(**kw)
    rng = random.Random(3)
    n = kw["n_replicas"]
    applied_cc = 0

    def hook(rnd):
        nonlocal applied_cc
        if rnd < 30:
            return
        views = ref.views()
        for r in range(eng.n_rep):
            u = rng.random()
            if u < 0.03:
                t, node = rng.choice((O.CC_ADD_NODE, O.CC_REMOVE_NODE)), rng.randrange(1, n + 1)
                eng.propose_config_change([r], [t], [node])
                ref.push(O.PUSH_CC_PROPOSE, r, t, node)
            elif u < 0.06 and views[r].removed != 0b111:
                t, node = rng.choice((O.CC_ADD_NODE, O.CC_REMOVE_NODE)), rng.randrange(0, n + 1)
                eng.apply_config_change([r], [node], [t])
                ref.push(O.PUSH_CC_APPLY, r, node, t)
                applied_cc += 1
            elif u < 0.07:
                eng.reject_config_change([r])
                ref.push(O.PUSH_CC_REJECT, r)

    d = run_driven(eng, ref, 200, seed=9, ext_apply=True, before_round=hook, density=0.1)
    assert d is None, f"first divergence {d}"
    assert applied_cc > 10


def test_membership_calls_refused():
    from dragonboat_amd.engine import InputError, RBE_E_INVALID, RBE_E_STATE
    eng = SoaCpu(trace=True, n_groups=2, n_replicas=3, ext_inputs=True)
    with pytest.raises(InputError) as ei:  # no membership configured
        eng.propose_config_change([0], [0], [1])
    assert ei.value.rc == RBE_E_STATE
    m = SoaCpu(trace=True, n_groups=2, n_replicas=3, ext_inputs=True, membership=True)
    with pytest.raises(InputError) as ei:  # node outside the group
        m.propose_config_change([0], [0], [4])
    assert ei.value.rc == RBE_E_INVALID
    with pytest.raises(InputError) as ei:  # the engine applies (no ext_apply)
        m.apply_config_change([0], [1], [0])
    assert ei.value.rc == RBE_E_STATE
    m.propose_config_change([0], [1], [2])
    with pytest.raises(InputError) as ei:  # one per replica per step
        m.propose_config_change([0], [0], [2])
    assert ei.value.rc == RBE_E_STATE
