"""Pin the oracle's raft state machine (raft.go) against the reference's own
scenario and table tests (raft_etcd_test.go, raft_test.go, readindex_test.go),
vectors in tests/golden/raft.json.  These are the kernel groups of the device
engine: (1) ReplicateResp→tryCommit, (2) log matching, (3) vote tally,
(4) ReadIndex quorum, (5) ticks."""
import json
import os

import pytest

import oracle as O

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "raft.json")))


def _ents(pairs):
    return [O.Entry(index=i, term=t) for i, t in pairs]


def _db(pairs):
    db = O.LogDB()
    if pairs:
        db.append(_ents(pairs))
    return db


def _ents_with_config(node_id, terms):
    """entsWithConfig (raft_etcd_test.go:2788-2803)."""
    db = _db([(i + 1, t) for i, t in enumerate(terms)])
    r = O.Raft.new(node_id, (), election=5, heartbeat=1, logdb=db)
    r.reset(terms[-1])
    return r


# ---------------------------------------------------------------- kernel 1
@pytest.mark.parametrize("case", G["commit"]["cases"])
def test_commit(case):
    matches, logs, sm_term, exp = case
    db = _db(logs)
    db.set_state(term=sm_term)
    sm = O.Raft.new(1, [1], election=5, heartbeat=1, logdb=db)
    for j, m in enumerate(matches):
        sm.set_remote("remotes", j + 1, match=m, next=m + 1)
    sm.state = O.LEADER
    sm.try_commit()
    assert sm.committed == exp


@pytest.mark.parametrize("vals", G["sort_match_values"]["cases"])
def test_unrolled_bubble_sort_match_value(vals):
    sm = O.Raft.new(1, [1])
    sm.set_matched(vals)
    sm.sort_match_values()
    assert sm.matched() == sorted(vals)


@pytest.mark.parametrize("case", G["leader_append_resp"]["cases"])
def test_leader_append_resp(case):
    index, reject, wmatch, wnext, wnum, windex, wcommit = case
    sm = O.Raft.new(1, [1, 2, 3], logdb=_db(G["leader_append_resp"]["log"]))
    sm.become_candidate()
    sm.become_leader()
    sm.read_messages()
    sm.handle(O.msg(O.ReplicateResp, **{"from": 2}, log_index=index, term=sm.term,
                    reject=reject, hint=index))
    p = sm.remote(2)
    assert (p.match, p.next) == (wmatch, wnext)
    msgs = sm.read_messages()
    assert len(msgs) == wnum
    for m in msgs:
        assert (m.log_index, m.commit) == (windex, wcommit)


def test_bcast_beat():  # raft_etcd_test.go:1959-2016
    db = O.LogDB()
    assert db.apply_snapshot(O.Snapshot(index=1000, term=1, addresses=[1, 2, 3])) == O.ERR_OK
    sm = O.Raft.new(1, (), logdb=db)
    sm.term = 1
    sm.become_candidate()
    sm.become_leader()
    for i in range(10):
        sm.handle(O.msg(O.Propose, **{"from": 1}, to=1, entries=[O.Entry()]))
    sm.read_messages()
    r2, r3 = sm.remote(2), sm.remote(3)
    sm.set_remote("remotes", 2, match=5, next=6, state=r2.state, active=r2.active)
    sm.set_remote("remotes", 3, match=sm.last_index, next=sm.last_index + 1, state=r3.state,
                  active=r3.active)
    sm.handle(O.msg(O.LeaderHeartbeat))
    msgs = sm.read_messages()
    assert len(msgs) == 2
    want = {2: min(sm.committed, 5), 3: min(sm.committed, sm.last_index)}
    for m in msgs:
        assert m.type == O.Heartbeat and m.log_index == 0 and m.log_term == 0
        assert m.commit == want.pop(m.to)
        assert not m.entries


# ---------------------------------------------------------------- kernel 2
@pytest.mark.parametrize("case", G["handle_replicate"]["cases"])
def test_handle_mt_replicate(case):
    term, log_term, log_index, commit, ents, wlast, wcommit, wreject = case
    sm = O.Raft.new(1, [1], logdb=_db(G["handle_replicate"]["log"]))
    sm.become_follower(2, 0)
    sm.handle_direct("replicate", O.msg(O.Replicate, term=term, log_term=log_term,
                                        log_index=log_index, commit=commit,
                                        entries=_ents(ents)))
    assert (sm.last_index, sm.committed) == (wlast, wcommit)
    msgs = sm.read_messages()
    assert len(msgs) == 1 and msgs[0].reject == wreject


def test_follower_check_replicate():  # raft_etcd_paper_test.go:577-615
    ents = [(1, 1), (2, 2)]
    tests = [(0, 0, 1, False, 0), (ents[0][1], ents[0][0], 1, False, 0),
             (ents[1][1], ents[1][0], 2, False, 0), (ents[0][1], ents[1][0], ents[1][0], True, 2),
             (ents[1][1] + 1, ents[1][0] + 1, ents[1][0] + 1, True, 2)]
    for term, index, windex, wreject, wrejecthint in tests:
        db = _db(ents)
        r = O.Raft.new(1, [1, 2, 3], logdb=db)
        r.load_state_for_test = None
        r.committed = 1
        r.become_follower(2, 2)
        r.handle(O.msg(O.Replicate, **{"from": 2}, to=1, term=2, log_term=term, log_index=index))
        msgs = r.read_messages()
        assert len(msgs) == 1
        m = msgs[0]
        assert (m.from_, m.to, m.type, m.term, m.log_index, m.reject, m.hint) == (
            1, 2, O.ReplicateResp, 2, windex, wreject, wrejecthint)


# ---------------------------------------------------------------- kernel 3
@pytest.mark.parametrize("case", G["recv_request_vote"]["cases"])
def test_recv_msg_vote(case):
    state, li, lt, vote_for, wreject = case
    sm = O.Raft.new(1, [1, 2], logdb=_db(G["recv_request_vote"]["log"]))
    sm.state = G["recv_request_vote"]["states"][state]
    sm.vote = vote_for
    sm.handle(O.msg(O.RequestVote, **{"from": 2}, log_index=li, log_term=lt))
    msgs = sm.read_messages()
    assert len(msgs) == 1 and msgs[0].reject == wreject


@pytest.mark.parametrize("case", G["leader_election"]["cases"])
def test_leader_election(case):
    peers, wstate, wterm = case
    objs = []
    for i, p in enumerate(peers):
        if p is None:
            objs.append(None)
        elif p == "hole":
            objs.append(O.BlackHole())
        else:
            objs.append(_ents_with_config(i + 1, p))
    nt = O.Network(*objs)
    nt.send(O.msg(O.Election, **{"from": 1}, to=1))
    sm = nt.peers[1]
    assert (sm.state, sm.term) == (wstate, wterm)


def test_leader_cycle():  # raft_etcd_test.go:467-497
    nt = O.Network(None, None, None)
    for cid in (1, 2, 3):
        nt.send(O.msg(O.Election, **{"from": cid}, to=cid))
        for nid, sm in nt.peers.items():
            assert sm.state == (O.LEADER if nid == cid else O.FOLLOWER)


def test_dueling_candidates():  # raft_etcd_test.go:786-850
    a, b, c = (O.Raft.new(i, [1, 2, 3]) for i in (1, 2, 3))
    nt = O.Network(a, b, c)
    nt.cut(1, 3)
    nt.send(O.msg(O.Election, **{"from": 1}, to=1))
    nt.send(O.msg(O.Election, **{"from": 3}, to=3))
    assert a.state == O.LEADER and c.state == O.CANDIDATE
    nt.recover()
    nt.send(O.msg(O.Election, **{"from": 3}, to=3))
    for sm, wlast in ((a, 1), (b, 1), (c, 0)):
        assert (sm.state, sm.term, sm.last_index) == (O.FOLLOWER, 2, wlast)
    assert (a.committed, b.committed) == (1, 1)


def test_candidate_fallback():  # raft_etcd_paper_test.go:277-298
    for term in (1, 2):
        r = O.Raft.new(1, [1, 2, 3])
        r.handle(O.msg(O.Election, **{"from": 1}, to=1))
        assert r.state == O.CANDIDATE
        r.handle(O.msg(O.Replicate, **{"from": 2}, to=1, term=term))
        assert (r.state, r.term) == (O.FOLLOWER, term)


def test_handle_vote_resp():  # raft_test.go:1709-1725 (first response per voter counts)
    r = O.Raft.new(1, [1, 2, 3])
    r.become_candidate()
    assert r.handle_vote_resp(1, 0) == 1
    assert r.handle_vote_resp(2, 1) == 1
    assert r.handle_vote_resp(2, 0) == 1  # a repeated response is ignored
    assert r.handle_vote_resp(3, 0) == 2


# ---------------------------------------------------------------- kernel 4
def test_read_only_option_safe():
    a, b, c = (O.Raft.new(i, [1, 2, 3]) for i in (1, 2, 3))
    nt = O.Network(a, b, c)
    b.randomized_election_timeout = b.election_timeout + 1
    for _ in range(b.election_timeout):
        b.tick()
    nt.send(O.msg(O.Election, **{"from": 1}, to=1))
    assert a.state == O.LEADER
    sms = {1: a, 2: b, 3: c}
    for node, props, wri, lo, hi in G["read_only_option_safe"]["cases"]:
        for _ in range(props):
            nt.send(O.msg(O.Propose, **{"from": 1}, to=1, entries=[O.Entry()]))
        nt.send(O.msg(O.ReadIndex, **{"from": node}, to=node, hint=lo, hint_high=hi))
        r = sms[node]
        rtr = r.ready_to_read()
        assert rtr, node
        assert rtr[0] == (wri, lo, hi)
        r.clear_ready_to_read()


def _ctx(v):  # getTestSystemCtx (readindex_test.go:23-28)
    return (v, v + 1)


def test_read_index_leader_can_be_confirmed():  # readindex_test.go:125-162
    r = O.Raft.new(1, [1, 2, 3])
    ctx, ctx2, ctx3 = _ctx(10001), _ctx(10002), _ctx(10003)
    r.read_index_add(3, ctx2, 1)
    r.read_index_add(4, ctx, 3)
    r.read_index_add(5, ctx3, 2)
    assert r.read_index_confirm(ctx, 1, 3) == []
    ris = r.read_index_confirm(ctx, 3, 3)
    assert ris == [(4, 1) + ctx2, (4, 3) + ctx]
    assert len(r.read_index_queue()) == 1


def test_read_index_request_can_be_added():  # readindex_test.go:54-80
    r = O.Raft.new(1, [1, 2, 3])
    r.read_index_add(1, _ctx(10001), 1)
    r.read_index_add(2, _ctx(10002), 2)
    q = r.read_index_queue()
    assert len(q) == 2
    assert q[1][:4] == _ctx(10002) + (2, 2)


def test_read_index_same_ctx_can_not_be_added_twice():  # readindex_test.go:30-40
    r = O.Raft.new(1, [1, 2, 3])
    r.read_index_add(1, _ctx(10001), 1)
    r.read_index_add(2, _ctx(10001), 2)
    assert len(r.read_index_queue()) == 1


def test_read_index_checks_input_index():  # readindex_test.go:82-99
    r = O.Raft.new(1, [1, 2, 3])
    r.read_index_add(3, _ctx(10001), 1)
    r.read_index_add(5, _ctx(10002), 3)
    with pytest.raises(O.RaftPanic):
        r.read_index_add(4, _ctx(10003), 2)


def test_read_index_reset_after_state_change():  # readindex_test.go:164-174
    r = O.Raft.new(1, [1, 2, 3])
    r.read_index_add(3, _ctx(10001), 1)
    assert len(r.read_index_queue()) == 1
    r.reset(2)
    assert len(r.read_index_queue()) == 0


def test_leader_read_index_single_node():  # raft_test.go:2677-2701
    r = O.Raft.new(1, [1])
    r.become_candidate()
    r.become_leader()
    r.handle(O.msg(O.ReadIndex, **{"from": 1}, to=1, hint=12345, hint_high=12346))
    assert r.ready_to_read() == [(1, 12345, 12346)]


# ---------------------------------------------------------------- kernel 5
def test_follower_tick():
    r = O.Raft.new(1, [1, 2], election=5)
    r.become_follower(10, 2)
    for _ in range(9):
        assert not r.time_for_election()
        r.tick()
    msgs = r.read_messages()
    assert len(msgs) == 1 and msgs[0].type == O.RequestVote


def test_leader_tick():
    r = O.Raft.new(1, [1, 2], election=5)
    r.become_candidate()
    r.become_leader()
    r.read_messages()
    for _ in range(10):
        r.tick()
    msgs = r.read_messages()
    assert len(msgs) == 10 and all(m.type == O.Heartbeat for m in msgs)


def test_time_for_election():
    r = O.Raft.new(1, [1], election=5)
    assert 5 <= r.randomized_election_timeout < 10
    r.election_tick = r.randomized_election_timeout - 1
    assert not r.time_for_election()
    r.election_tick = r.randomized_election_timeout
    assert r.time_for_election()


def test_leader_checks_quorum_every_election_tick():
    r = O.Raft.new(1, [1, 2], election=5)
    r.become_candidate()
    r.become_leader()
    r.check_quorum = 1
    for _ in range(5):
        r.tick()
    assert r.state != O.LEADER


def test_quiesced_tick():
    r = O.Raft.new(1, [1, 2], election=5)
    r.become_candidate()
    r.become_leader()
    r.read_messages()
    for _ in range(200):
        r.quiesced_tick()
    assert not r.read_messages()
    r = O.Raft.new(1, [1, 2], election=5)
    r.become_follower(10, 2)
    for _ in range(200):
        r.quiesced_tick()
    assert not r.read_messages()


def test_leader_stepdown_when_quorum_lost():  # raft_etcd_test.go:1628-1643
    sm = O.Raft.new(1, [1, 2, 3], election=5, check_quorum=True)
    sm.become_candidate()
    sm.become_leader()
    for _ in range(sm.election_timeout + 1):
        sm.tick()
    assert sm.state == O.FOLLOWER


def test_leader_stepdown_when_quorum_active():  # raft_etcd_test.go:1610-1625
    sm = O.Raft.new(1, [1, 2, 3], election=5, check_quorum=True)
    sm.become_candidate()
    sm.become_leader()
    for _ in range(sm.election_timeout + 1):
        sm.handle(O.msg(O.HeartbeatResp, **{"from": 2}, term=sm.term))
        sm.tick()
    assert sm.state == O.LEADER
