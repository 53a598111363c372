"""Arbitrary node ids on the HIP engine (rbe_set_node_ids); the CPU-tier twin
is tests/test_node_ids.py.  Besides the views, the device-side converters are
checked: rbe_collect_outputs / rbe_get_messages (From, To, node-id Hints) and
rbe_collect_updates / rbe_get_updates (vote, leader) of an engine with ids
equal those of an engine without, mapped through the ids."""
import pytest

import oracle as O
from test_membership import CATCHUP
from test_node_ids import ID_CASE, lockstep_ids, random_ids

pytestmark = pytest.mark.gpu


def test_gpu_node_ids_protocol_unchanged(gpu_available):
    from dragonboat_amd.engine import Engine
    n = ID_CASE["n_replicas"]
    ids = random_ids(ID_CASE["n_groups"], n)
    eng = Engine(device=0, trace=True, **ID_CASE, **CATCHUP)
    eng.set_node_ids(0, ids)
    ref = O.Harness(**ID_CASE)
    lockstep_ids(eng, ref, ids, n, 300)
    assert eng.fault_summary()[0] == 0
    eng.close()


def test_gpu_node_ids_outputs(gpu_available):
    from dragonboat_amd.engine import Engine
    n = ID_CASE["n_replicas"]
    ids = random_ids(ID_CASE["n_groups"], n, seed=3)
    a = Engine(device=0, trace=True, **ID_CASE, **CATCHUP)
    a.set_node_ids(0, ids)
    b = Engine(device=0, trace=True, **ID_CASE, **CATCHUP)

    def ext(g, x):
        return ids[g][x - 1] if x else 0

    node_hints = 0
    for rnd in range(200):
        a.step()
        b.step()
        offa, ma, _, _ = a.collect_outputs()
        offs, mb, _, _ = b.collect_outputs()
        assert len(ma) == len(mb) and list(offa) == list(offs)
        for r in range(a.n_rep):
            g = r // n
            for j in range(offs[r], offs[r + 1]):
                x, y = ma[j], mb[j]
                assert (x["to"], x["from_"]) == (ext(g, int(y["to"])), ext(g, int(y["from_"]))), (rnd, r)
                if y["type"] in (14, 23):  # RequestVote, LeaderTransfer (raft.pb.go:23-51)
                    assert x["hint"] == ext(g, int(y["hint"])), (rnd, r)
                    node_hints += y["hint"] != 0
                else:
                    assert x["hint"] == y["hint"]
        if rnd % 20 == 0:  # the per-replica getter too
            for r in range(0, a.n_rep, 7):
                g = r // n
                for x, y in zip(a.messages(r), b.messages(r)):
                    assert (x.to, x.from_) == (ext(g, y.to), ext(g, y.from_))
        ua, ub = a.updates(), b.updates()
        for r in range(a.n_rep):
            g = r // n
            assert ua[r].leader_id == ext(g, ub[r].leader_id) and ua[r].vote == ext(g, ub[r].vote)
        ra, upa = a.collect_updates()
        rb, upb = b.collect_updates()
        assert list(ra) == list(rb)
        for i, r in enumerate(rb):
            g = int(r) // n
            assert upa["leader_id"][i] == ext(g, int(upb["leader_id"][i]))
            assert upa["vote"][i] == ext(g, int(upb["vote"][i]))
    assert node_hints > 0, "no leader transfer carried a node id in its Hint"
    a.close()
    b.close()


def test_gpu_replace_nodes_runtime_ids(gpu_available):
    """rbe_replace_node on the HIP engine: remove node 3 and add node 9 in its
    slot, remove node 1 and add node 4; the device check (slot_referenced)
    allows it exactly when the oracle does, and every view equals the oracle's
    every round (CPU twin: test_node_ids.py)."""
    from dragonboat_amd.engine import Engine
    from test_node_ids import REPL_CASE, REPL_PLAN, run_replacements
    eng = Engine(device=0, trace=True, **REPL_CASE, **CATCHUP)
    ref = O.Harness(**REPL_CASE)
    stage, refused = run_replacements(eng, ref, 300)
    assert eng.fault_summary()[0] == 0
    assert all(s == len(REPL_PLAN) for s in stage) and refused > 0, (stage, refused)
    eng.close()


def test_gpu_node_ids_any_order(gpu_available):
    from dragonboat_amd.engine import Engine
    n = ID_CASE["n_replicas"]
    ids = [list(reversed(row)) for row in random_ids(ID_CASE["n_groups"], n, seed=9)]
    eng = Engine(device=0, trace=True, **ID_CASE, **CATCHUP)
    eng.set_node_ids(0, ids)
    ref = O.Harness(**ID_CASE)
    lockstep_ids(eng, ref, ids, n, 150)
    assert eng.fault_summary()[0] == 0
    eng.close()
