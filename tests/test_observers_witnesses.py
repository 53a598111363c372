"""Observers and witnesses on the device (cfg.observer_slots / witness_slots
with cfg.membership): the device step compiled for the host (tests/soa_cpu)
against the oracle harness, round by round — every view field (each replica's
observers and witnesses included) and the trace digest.

Covered (reference internal/raft):
  * nodes that start as observers / witnesses (config.IsObserver / IsWitness,
    raft.go:270-281 → becomeObserver / becomeWitness) with no peers and an
    empty log;
  * the membership schedule at the leader: AddObserver, the observer's
    promotion by AddNode (raft.go:1135-1157 addNode: observer → remote,
    becomeFollower at the promoted node), AddWitness and RemoveNode of a
    witness (raft.go:1170-1213);
  * replication to them: r.nodes() fan-out order remotes → observers →
    witnesses (raft.go:390-402, 794-808); a witness gets MetadataEntries in
    place of everything but ConfigChanges (makeMetadataEntries, raft.go:
    742-756) and a witness snapshot (makeWitnessSnapshot, 699-707);
  * quorum over remotes + witnesses, observers outside it (raft.go:366-416
    numVotingMembers / votingMembers, tryCommit 1020-1043);
  * heartbeats to voting members, then observers (raft.go:834-846);
  * observers / witnesses never campaign (raft.go:577-581); the observer and
    witness handler rows (raft.go:2075-2097) — handleObserverReplicate etc.
    route to the follower handlers, ReadIndex at an observer forwards to the
    leader;
  * membership carried by snapshots and RestoreRemotes (raft.go:472-517) with
    observers and witnesses."""
import pytest

import oracle as O
from parity_util import C2, C3, run_lockstep
from soa_cpu.soa import SoaCpu
from test_membership import CATCHUP, MEMB

# (kwargs, rounds): slots 0..n_voters-1 voters, the rest observers / witnesses
OW_CASES = {
    # 3 voters, an observer (promoted later) and a witness (added, removed, re-added)
    "N5": (dict(C3, n_groups=16, n_replicas=5, n_voters=3, observer_slots=0b01000,
                witness_slots=0b10000, **MEMB), 400),
    # 2 voters and a witness: the witness holds the quorum of three
    "N3w": (dict(C2, n_groups=16, n_replicas=3, n_voters=2, witness_slots=0b100, **MEMB), 300),
    # 4 voters, an observer and a witness, leaders isolated every epoch
    "N6": (dict(C3, n_groups=12, n_replicas=6, n_voters=4, observer_slots=0b010000,
                witness_slots=0b100000, iso_mod=2, **MEMB), 400),
    # groups of 7: 5 voters, an observer and a witness in slot 6 (the slot whose
    # outbox word takes the sender's own place)
    "N7": (dict(C3, n_groups=10, n_replicas=7, n_voters=5, observer_slots=0b0100000,
                witness_slots=0b1000000, **MEMB), 400),
}
# engine sizes per case: in N7 the witness joins after ~370 rounds and catches up
# from index 1 in one Replicate, so the ring and the round's arena hold all of it
# (the default sizes fault it with F_ARENA, a capacity limit the reference lacks)
SIZES = {"N7": dict(CATCHUP)}


def _roles_seen(ref):
    obs = wit = 0
    for v in ref.views():
        obs |= v.observers
        wit |= v.witnesses
    return obs, wit


def run_ow(eng, ref, rounds, skip=()):
    obs = wit = promoted = 0
    full = (1 << eng.cfg.n_replicas) - 1
    for _ in range(rounds // 50):
        d = run_lockstep(eng, ref, 50, every=1, skip=skip)
        assert d is None, f"first divergence {d}"
        o, w = _roles_seen(ref)
        obs |= o
        wit |= w
        promoted = max(promoted, max(bin(~v.removed & ~v.observers & ~v.witnesses & full).count("1")
                                     for v in ref.views()))
    return obs, wit, promoted


@pytest.mark.parametrize("name", list(OW_CASES))
def test_observer_witness_schedule(name):
    kw, rounds = OW_CASES[name]
    eng = SoaCpu(trace=True, **kw, **SIZES.get(name, CATCHUP))
    ref = O.Harness(**kw)
    obs, wit, _ = run_ow(eng, ref, rounds)
    assert eng.faults()[0] == 0
    assert wit, "no witness ever joined"
    if kw.get("observer_slots"):
        assert obs, "no observer ever joined"
    c = ref.counters()
    assert c["committed"] > 0


def test_observer_promoted():
    """The observer slot's node is added as an observer and later promoted to a
    voter by AddNode: some replica sees it in raft.remotes."""
    kw, rounds = OW_CASES["N5"]
    eng = SoaCpu(trace=True, **kw, **CATCHUP)
    ref = O.Harness(**kw)
    promoted = False
    for _ in range(rounds // 50):
        assert run_lockstep(eng, ref, 50, every=1) is None
        promoted |= any(not (v.removed >> 3) & 1 for v in ref.views())
    assert promoted, "the observer was never promoted"


def test_observer_witness_full_table_only():
    kw, rounds = OW_CASES["N5"]
    eng = SoaCpu(trace=True, full_only=True, **kw, **CATCHUP)
    ref = O.Harness(**kw)
    assert run_lockstep(eng, ref, 300, every=1) is None


@pytest.mark.parametrize("name", ["N6", "N7"])
def test_observer_witness_untraced(name):
    kw, rounds = OW_CASES[name]
    eng = SoaCpu(trace=False, **kw, **SIZES.get(name, CATCHUP))
    ref = O.Harness(**kw)
    assert run_lockstep(eng, ref, rounds, every=1, skip=("digest",)) is None


@pytest.mark.parametrize("name", ["N5", "N7"])
def test_observer_witness_snapshots(name):
    """Snapshots and compaction with observers / witnesses in the membership:
    a node snapshot records them, InstallSnapshot carries them (a witness gets
    a witness snapshot), RestoreRemotes restores them."""
    from test_membership_snapshot import run_memb_snap
    kw = dict(OW_CASES[name][0], snapshot_entries=8, compaction_overhead=2, iso_mod=2)
    eng = SoaCpu(trace=True, **kw, **CATCHUP)
    ref = O.Harness(**kw)
    run_memb_snap(eng, ref, 400)
    assert eng.faults()[0] == 0
    seen = set()
    for i in range(len(ref.views())):
        seen.add(ref.snapshot_state(i)[7])
    assert any(s >> 8 for s in seen), f"no snapshot held an observer or witness {seen}"


def test_restore_remotes_roles():
    """The host's Peer.RestoreRemotes naming observers and witnesses
    (rbe_restore_remotes counts[3]) against PUSH_RESTORE on the harness."""
    import random
    kw = dict(C3, n_groups=8, n_replicas=5, ext_inputs=True, membership=True)
    eng = SoaCpu(trace=True, **kw, **CATCHUP)
    ref = O.Harness(**kw)
    rng = random.Random(11)
    n = 5
    calls = 0
    for rnd in range(240):
        if rnd > 30 and rnd % 40 == 0:
            views = ref.views()
            for r in range(eng.n_rep):
                if rng.random() < 0.3:
                    # the replica's own node stays a voter; a witness never becomes
                    # one (restoreRemotes panics, raft.go:476-481)
                    me = r % n + 1
                    wits = [x for x in range(1, n + 1) if (views[r].witnesses >> (x - 1)) & 1]
                    nodes = [x for x in range(1, n + 1) if x != me and x not in wits]
                    rng.shuffle(nodes)
                    nv = rng.randrange(1, len(nodes) + 1)
                    v = sorted(nodes[:nv] + [me])
                    rest = nodes[nv:] + wits
                    o = sorted(x for x in rest if rng.random() < 0.5)
                    w = sorted(x for x in rest if x not in o)
                    eng.restore_remotes([r], [v], [o], [w])
                    bits = lambda xs: sum(1 << (x - 1) for x in xs)  # noqa: E731
                    rem = bits(x for x in range(1, n + 1) if x not in v)
                    ref.push(O.PUSH_RESTORE, r, rem | bits(o) << 8 | bits(w) << 16)
                    calls += 1
        d = run_lockstep(eng, ref, 1, every=1)
        assert d is None, f"round {rnd}: {d}"
    assert eng.faults()[0] == 0
    assert calls > 10


def test_host_applies_roles():
    """ext_apply: the host proposes and applies AddObserver / AddWitness /
    AddNode / RemoveNode itself (rbe_propose_config_change /
    rbe_apply_config_change), both sides driven identically; only changes the
    reference's raft takes without panicking (raft.go:1135-1213) are applied."""
    import random
    from input_util import run_driven
    kw = dict(C2, n_groups=6, n_replicas=5, n_voters=3, observer_slots=0b01000,
              witness_slots=0b10000, ext_inputs=True, ext_apply=True, membership=True)
    eng = SoaCpu(trace=True, **dict(kw))
    ref = O.Harness(**kw)
    rng = random.Random(8)
    n = kw["n_replicas"]
    applied = seen = 0

    def hook(rnd):
        nonlocal applied, seen
        if rnd < 30:
            return
        views = ref.views()
        for r in range(eng.n_rep):
            seen |= (views[r].observers << 8) | views[r].witnesses
            u = rng.random()
            me = r % n + 1
            v = views[r]
            node = rng.choice([x for x in range(1, n + 1) if x != me])
            b = 1 << (node - 1)
            voter = not v.removed & b
            obs, wit = v.observers & b, v.witnesses & b
            if u < 0.03:
                t = rng.choice((O.CC_ADD_NODE, O.CC_ADD_OBSERVER, O.CC_ADD_WITNESS))
                eng.propose_config_change([r], [t], [node])
                ref.push(O.PUSH_CC_PROPOSE, r, t, node)
            elif u < 0.08:
                if obs:
                    t = rng.choice((O.CC_ADD_NODE, O.CC_REMOVE_NODE))
                elif wit:
                    t = O.CC_REMOVE_NODE
                elif voter:
                    if bin(~v.removed & ((1 << n) - 1)).count("1") <= 2:
                        continue
                    t = O.CC_REMOVE_NODE
                else:
                    t = rng.choice((O.CC_ADD_NODE, O.CC_ADD_OBSERVER, O.CC_ADD_WITNESS))
                eng.apply_config_change([r], [node], [t])
                ref.push(O.PUSH_CC_APPLY, r, node, t)
                applied += 1

    d = run_driven(eng, ref, 200, seed=4, ext_apply=True, before_round=hook, density=0.1)
    assert d is None, f"first divergence {d}"
    assert applied > 20
    assert seen >> 8 and seen & 0xFF, "no observer or no witness joined"
    assert eng.faults()[0] == 0


def test_host_cannot_put_a_node_in_two_sets():
    """ext_apply: an AddObserver of a voter, an AddWitness of a voter or an
    observer, an AddObserver of a witness would put one node in two of raft's
    maps (raft.go:1159-1180 checks only its own map), which a slot cannot
    hold: refused at the ABI with RBE_E_INVALID, nothing staged, no fault.
    A no-op re-add (AddObserver of an observer) is accepted."""
    from dragonboat_amd.engine import InputError, RBE_E_INVALID
    kw = dict(C2, n_groups=2, n_replicas=5, n_voters=3, observer_slots=0b01000,
              witness_slots=0b10000, ext_inputs=True, ext_apply=True, membership=True)
    eng = SoaCpu(trace=True, **dict(kw))
    eng.run(30)
    # node 4 (observer slot) becomes an observer at replica 0, node 5 a witness
    eng.apply_config_change([0], [4], [O.CC_ADD_OBSERVER])
    eng.step()
    eng.apply_config_change([0], [5], [O.CC_ADD_WITNESS])
    eng.step()
    v = eng.views()[0]
    assert v.observers == 0b01000 and v.witnesses == 0b10000, (v.observers, v.witnesses)
    for node, t in ((2, O.CC_ADD_OBSERVER), (3, O.CC_ADD_WITNESS), (4, O.CC_ADD_WITNESS),
                    (5, O.CC_ADD_OBSERVER)):
        with pytest.raises(InputError) as ei:
            eng.apply_config_change([0], [node], [t])
        assert ei.value.rc == RBE_E_INVALID, (node, t)
    eng.apply_config_change([0], [4], [O.CC_ADD_OBSERVER])  # already an observer: a no-op
    eng.step()
    v = eng.views()[0]
    assert v.observers == 0b01000 and v.witnesses == 0b10000
    assert eng.faults()[0] == 0
