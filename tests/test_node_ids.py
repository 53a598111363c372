"""Arbitrary node ids (rbe_set_node_ids): every group names its slots with its
own uint64 node ids (raft.Config.NodeID, pb.Message From/To), ascending with
the slots.  Inside the engine a node is its slot + 1, so the protocol — and the
trace digest — is the one the oracle harness runs with node ids 1..n; what
changes is every node id the boundary takes or returns: views and Updates
(vote, leader), messages in raftpb form (From, To, a RequestVote's or
LeaderTransfer's Hint), host inputs (leader-transfer targets, Unreachable /
SnapshotStatus nodes, ConfigChange nodes, RestoreRemotes voters, launch
votes) and the transport (rbe_get_outbox / rbe_push_messages, the wire
frames).  Checked on the device step compiled for the host (tests/soa_cpu):
an engine with random ids against the oracle (views mapped through the ids),
host input by id against input by slot, and engines that only talk through
the transport carrying ids."""
import random

import pytest

import oracle as O
from parity_util import C2, C3, view_diff
from soa_cpu.soa import SoaCpu
from test_membership import CATCHUP, MEMB


def random_ids(n_groups, n, seed=1):
    """ascending random node ids per group (some near 2^64, some small)"""
    rng = random.Random(seed)
    out = []
    for g in range(n_groups):
        hi = rng.choice((1 << 20, 1 << 40, (1 << 64) - 1))
        row = set()
        while len(row) < n:
            row.add(rng.randrange(1, hi))
        out.append(sorted(row))
    return out


def mapped(view, ids_row):
    """an oracle view (node ids 1..n) with its node ids mapped through ids_row"""
    m = O.ReplicaView()
    for f in O.VIEW_FIELDS:
        setattr(m, f, getattr(view, f))
    m.vote = ids_row[view.vote - 1] if view.vote else 0
    m.leader_id = ids_row[view.leader_id - 1] if view.leader_id else 0
    return m


def lockstep_ids(eng, ref, ids, n, rounds, skip=()):
    for rnd in range(rounds):
        eng.run(1)
        ref.run(1)
        ev, hv = eng.views(), ref.views()
        for i in range(len(hv)):
            d = view_diff(ev[i], mapped(hv[i], ids[i // n]), skip)
            assert d is None, f"round {rnd + 1} replica {i}: {d}"


ID_CASE = dict(C3, n_groups=12, iso_mod=2, xfer_period=7, xfer_mod=2, **MEMB)


def test_node_ids_protocol_unchanged():
    """Elections, leader transfers (RequestVote / LeaderTransfer hints),
    membership changes: the same protocol under any node ids."""
    n = ID_CASE["n_replicas"]
    ids = random_ids(ID_CASE["n_groups"], n)
    eng = SoaCpu(trace=True, **ID_CASE, **CATCHUP)
    eng.set_node_ids(0, ids)
    ref = O.Harness(**ID_CASE)
    lockstep_ids(eng, ref, ids, n, 300)
    assert eng.faults()[0] == 0
    c = ref.counters()
    assert c["campaigns"] > 20, c


def test_node_ids_spare_slots():
    """A slot beyond the initial voters is the id of a node that joins later."""
    kw = dict(C3, n_groups=10, n_replicas=5, n_voters=3, **MEMB)
    ids = random_ids(10, 5, seed=4)
    eng = SoaCpu(trace=True, **kw, **CATCHUP)
    eng.set_node_ids(0, ids)
    ref = O.Harness(**kw)
    lockstep_ids(eng, ref, ids, 5, 300)
    assert eng.faults()[0] == 0


def test_node_id_inputs():
    """Host input naming nodes by id (engine with ids) against the same input by
    slot id (engine without): identical protocol, round by round."""
    kw = dict(C2, n_groups=8, ext_inputs=True, ext_apply=True, membership=True)
    n = kw["n_replicas"]
    ids = random_ids(8, n, seed=9)
    a = SoaCpu(trace=True, **kw, **CATCHUP)
    a.set_node_ids(0, ids)
    b = SoaCpu(trace=True, **kw, **CATCHUP)
    rng = random.Random(5)
    applied = [0] * a.n_rep
    for rnd in range(220):
        views = b.views()
        for r in range(a.n_rep):
            row = ids[r // n]
            u = rng.random()
            node = rng.randrange(1, n + 1)
            if rnd < 25:
                pass
            elif u < 0.02:
                a.request_leader_transfer([r], [row[node - 1]])
                b.request_leader_transfer([r], [node])
            elif u < 0.04:
                a.report_unreachable([r], [row[node - 1]])
                b.report_unreachable([r], [node])
            elif u < 0.06:
                rej = rng.random() < 0.5
                a.report_snapshot_status([r], [row[node - 1]], [rej])
                b.report_snapshot_status([r], [node], [rej])
            elif u < 0.08:
                t = rng.choice((O.CC_ADD_NODE, O.CC_REMOVE_NODE))
                a.propose_config_change([r], [t], [row[node - 1]])
                b.propose_config_change([r], [t], [node])
            elif u < 0.10 and views[r].removed != (1 << n) - 1:
                t = rng.choice((O.CC_ADD_NODE, O.CC_REMOVE_NODE))
                a.apply_config_change([r], [row[node - 1]], [t])
                b.apply_config_change([r], [node], [t])
            elif u < 0.11:
                vs = sorted(rng.sample(range(1, n + 1), rng.randrange(1, n + 1)))
                a.restore_remotes([r], [[row[v - 1] for v in vs]])
                b.restore_remotes([r], [vs])
            applied[r] = max(applied[r], views[r].processed - rng.randrange(3))
        a.notify_applied(list(range(a.n_rep)), applied)
        b.notify_applied(list(range(b.n_rep)), applied)
        a.step()
        b.step()
        av, bv = a.views(), b.views()
        for i in range(a.n_rep):
            d = view_diff(av[i], mapped(bv[i], ids[i // n]))
            assert d is None, f"round {rnd} replica {i}: {d}"


def _owner(g, k, w):
    return (g + k) % w


def deliver_ids(engs, n, n_rep, ids):
    """transport_util.deliver with node ids on the wire of the outbox: the
    destination slot comes from the message's To id"""
    world = len(engs)
    batches = [([], [], [], []) for _ in range(world)]
    moved = 0
    for rank, e in enumerate(engs):
        for r in range(n_rep):
            g, k = divmod(r, n)
            if _owner(g, k, world) != rank:
                continue
            msgs, ents, cmds = e.outbox(r)
            ei = 0
            for m in msgs:
                ne = m.n_entries
                assert m.from_ == ids[g][k]
                dst = _owner(g, ids[g].index(m.to), world)
                if dst != rank:
                    gs, ms, es, cs = batches[dst]
                    gs.append(g)
                    ms.append(m)
                    es.extend(ents[ei:ei + ne])
                    cs.extend(cmds[ei:ei + ne])
                    moved += 1
                ei += ne
    for rank, e in enumerate(engs):
        e.push_messages(*batches[rank])
    return moved


@pytest.mark.parametrize("n", [5, 7])
@pytest.mark.parametrize("wire", [False, True])
def test_node_ids_over_the_transport(wire, n):
    """W = 2 engines whose cross-engine traffic carries node ids: raftpb
    messages (rbe_get_outbox / rbe_push_messages) or wire frames
    (rbe_wire_encode / rbe_wire_ingest); groups of 5 and of 7."""
    from transport_util import deliver_wire
    kw = dict(C3, n_groups=10, n_replicas=n, iso_mod=2, xfer_period=9, xfer_mod=2)
    n = kw["n_replicas"]
    ids = random_ids(10, n, seed=7)
    engs = []
    for rank in range(2):
        e = SoaCpu(trace=True, rep_world=2, rep_rank=rank, **kw, **CATCHUP)
        e.set_node_ids(0, ids)
        engs.append(e)
    ref = O.Harness(**kw)
    n_rep = len(ref.views())
    moved = 0
    for rnd in range(220):
        iso = [e.iso_leaders() for e in engs]
        if iso[0] is not None:
            bits = iso[0] | iso[1]
            for e in engs:
                e.set_iso_leaders(bits)
        for e in engs:
            e.step()
        ref.step()
        moved += deliver_wire(engs)[0] if wire else deliver_ids(engs, n, n_rep, ids)
        hv = ref.views()
        evs = [e.views() for e in engs]
        for r in range(n_rep):
            g, k = divmod(r, n)
            d = view_diff(evs[_owner(g, k, 2)][r], mapped(hv[r], ids[g]))
            assert d is None, f"round {rnd + 1} replica {r}: {d}"
    assert moved > 1000


def test_node_id_checks():
    from dragonboat_amd.engine import InputError, RBE_E_INVALID, RBE_E_STATE
    e = SoaCpu(trace=True, n_groups=3, n_replicas=3, ext_inputs=True)
    for bad in ([[0, 4, 9]], [[4, 4, 9]], [[4, 9, 4]]):  # NoNode, repeated
        with pytest.raises(InputError) as ei:
            e.set_node_ids(0, bad)
        assert ei.value.rc == RBE_E_INVALID
    with pytest.raises(InputError):  # past the groups
        e.set_node_ids(2, [[1, 2, 3], [4, 5, 6]])
    e.set_node_ids(1, [[10, 20, 30]])
    with pytest.raises(InputError) as ei:  # node 2 is not in group 1 any more
        e.request_leader_transfer([3], [2])
    assert ei.value.rc == RBE_E_INVALID
    e.request_leader_transfer([3], [20])
    e.request_leader_transfer([0], [2])  # group 0 keeps ids 1..3
    e.step()
    with pytest.raises(InputError) as ei:  # only before the first step
        e.set_node_ids(0, [[7, 8, 9]])
    assert ei.value.rc == RBE_E_STATE


# ---- runtime node ids (rbe_replace_node): a removed node's slot takes a new id
REPL_CASE = dict(C2, n_groups=6, n_replicas=3, membership=True, ext_inputs=True)
# per group: (slot, old id, new id) in order — remove node 3 and add node 9,
# then remove node 1 (the first leader) and add node 4
REPL_PLAN = ((2, 3, 9), (0, 1, 4))


def run_replacements(eng, ref, rounds, plan=REPL_PLAN, n=3):
    """Each group walks `plan`: propose RemoveNode(old) at its leader; once
    every replica applied it and nothing refers to the old node, both sides
    replace the slot (rbe_replace_node / Harness.replace must agree on when
    that is allowed), then propose AddNode(new) and wait until the new node has
    caught up.  Views (mapped through the current ids) equal the oracle's every
    round.  Returns per group the steps completed."""
    from dragonboat_amd.engine import InputError
    ng = len(eng.views()) // n
    ids = [[1, 2, 3] for _ in range(ng)]
    stage = [0] * ng          # index into plan (x2: 0 = remove, 1 = replace/add)
    phase = ["remove"] * ng   # remove -> wait_removed -> add -> wait_added
    refused = 0
    for rnd in range(rounds):
        hv = ref.views()
        for g in range(ng):
            if stage[g] >= len(plan):
                continue
            slot, old, new = plan[stage[g]]
            rows = [hv[g * n + k] for k in range(n)]
            lead = [k for k in range(n) if rows[k].role == O.LEADER]
            if phase[g] == "remove" and lead and rnd > 40:
                L = lead[0]
                eng.propose_config_change([g * n + L], [O.CC_REMOVE_NODE], [old])
                ref.push(O.PUSH_CC_PROPOSE, g * n + L, O.CC_REMOVE_NODE, slot + 1)
                phase[g] = "wait_removed"
            elif phase[g] == "wait_removed":
                ok_ref = ref.replace(g * n + slot)
                try:
                    eng.replace_node([g * n + slot], [new])
                    ok_eng = True
                except InputError:
                    ok_eng = False
                assert ok_eng == ok_ref, (rnd, g, "replace allowed", ok_eng, ok_ref)
                if ok_ref:
                    ids[g][slot] = new
                    phase[g] = "add"
                else:
                    refused += 1
            elif phase[g] == "add" and lead and lead[0] != slot:
                L = lead[0]
                eng.propose_config_change([g * n + L], [O.CC_ADD_NODE], [new])
                ref.push(O.PUSH_CC_PROPOSE, g * n + L, O.CC_ADD_NODE, slot + 1)
                phase[g] = "wait_added"
            elif phase[g] == "wait_added" and lead:
                lv = rows[lead[0]]
                # the new node counts at the leader and follows it (one
                # round behind on commits while proposals keep coming)
                if rows[slot].committed + 2 >= lv.committed and not (lv.removed >> slot) & 1:
                    stage[g] += 1
                    phase[g] = "remove"
        eng.step()
        ref.step()
        ev, hv = eng.views(), ref.views()
        for i in range(len(hv)):
            d = view_diff(ev[i], mapped(hv[i], ids[i // n]))
            assert d is None, f"round {rnd} replica {i}: {d}"
    return stage, refused


def test_replace_nodes_runtime_ids():
    """Remove node 3, add node 9 in its slot; remove node 1, add node 4: 300
    rounds, every view field and digest equal to the oracle's every round."""
    eng = SoaCpu(trace=True, **REPL_CASE, **CATCHUP)
    ref = O.Harness(**REPL_CASE)
    stage, refused = run_replacements(eng, ref, 300)
    assert eng.faults()[0] == 0
    assert all(s == len(REPL_PLAN) for s in stage), stage
    assert refused > 0, "the replacement was never refused while the group still knew the node"
    # the new ids are the nodes' ids at the boundary
    assert {v.leader_id for v in eng.views()} <= {2, 3, 4, 9}


def test_replace_node_checks():
    from dragonboat_amd.engine import InputError, RBE_E_INVALID, RBE_E_STATE
    eng = SoaCpu(trace=True, **REPL_CASE, **CATCHUP)
    eng.run(40)
    with pytest.raises(InputError) as ei:  # still a member everywhere
        eng.replace_node([2], [9])
    assert ei.value.rc == RBE_E_STATE
    with pytest.raises(InputError) as ei:  # the id of another slot of the group
        eng.replace_node([2], [1])
    assert ei.value.rc == RBE_E_INVALID
    with pytest.raises(InputError) as ei:  # node id 0
        eng.replace_node([2], [0])
    assert ei.value.rc == RBE_E_INVALID
    with pytest.raises(InputError) as ei:  # two slots of one group at once
        eng.replace_node([1, 2], [8, 9])
    assert ei.value.rc == RBE_E_STATE
    sched = SoaCpu(trace=True, **dict(REPL_CASE, **MEMB))
    with pytest.raises(InputError) as ei:  # a seeded schedule names slots
        sched.replace_node([2], [9])
    assert ei.value.rc == RBE_E_STATE
    plain = SoaCpu(trace=True, **C2)
    with pytest.raises(InputError) as ei:  # no membership change at all
        plain.replace_node([2], [9])
    assert ei.value.rc == RBE_E_STATE


def test_node_ids_any_order():
    """Node ids need not ascend with the slots: the canonical order is the
    slot order (any fixed order is one of the reference's map orders)."""
    n = ID_CASE["n_replicas"]
    ids = [list(reversed(row)) for row in random_ids(ID_CASE["n_groups"], n, seed=9)]
    eng = SoaCpu(trace=True, **ID_CASE, **CATCHUP)
    eng.set_node_ids(0, ids)
    ref = O.Harness(**ID_CASE)
    lockstep_ids(eng, ref, ids, n, 150)
    assert eng.faults()[0] == 0
