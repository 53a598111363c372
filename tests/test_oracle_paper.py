"""Pin the oracle's log replication against the reference's Raft-paper tests
(raft_etcd_paper_test.go TestFollowerAppendEntries, TestLeaderSyncFollowerLog;
vectors in tests/golden/paper.json): the follower side of kernel group (2)
(matchTerm / getConflictIndex / tryAppend / merge) and the leader's
backtracking (decreaseTo → resend) that brings a divergent follower in line."""
import json
import os

import pytest

import oracle as O

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "paper.json")))


def _ents(pairs):
    return [O.Entry(index=i, term=t) for i, t in pairs]


def _db(pairs):
    db = O.LogDB()
    if pairs:
        db.append(_ents(pairs))
    return db


def _all(r):
    """getAllEntries (logentry_etcd_test.go:31-41)."""
    ents, err = r.log_entries(r.first_index)
    assert err == O.ERR_OK
    return [(e.index, e.term) for e in ents]


@pytest.mark.parametrize("case", G["follower_append_entries"]["cases"])
def test_follower_append_entries(case):
    li, lt, ents, want, want_unstable = case
    r = O.Raft.new(1, [1, 2, 3], 10, 1, logdb=_db(G["follower_append_entries"]["storage"]))
    r.become_follower(2, 2)
    r.handle(O.msg(O.Replicate, from_=2, to=1, term=2, log_term=lt, log_index=li,
                   entries=_ents(ents)))
    assert _all(r) == [tuple(x) for x in want]
    assert [(e.index, e.term) for e in r.log_entries_to_save()] == [tuple(x) for x in want_unstable]


def _ltoa(r):
    """ltoa (raft_etcd_test.go:88-95): committed, applied, all entries."""
    return (r.committed, r.processed, _all(r))


@pytest.mark.parametrize("fi", range(len(G["leader_sync_follower_log"]["followers"])))
def test_leader_sync_follower_log(fi):
    v = G["leader_sync_follower_log"]
    term = v["term"]
    lead = O.Raft.new(1, [1, 2, 3], 10, 1, logdb=_db(v["leader"]))
    lead.load_state(term, lead.last_index)
    follower = O.Raft.new(2, [1, 2, 3], 10, 1, logdb=_db(v["followers"][fi]))
    follower.load_state(term - 1, 0)
    nt = O.Network(lead, follower, O.BlackHole())
    nt.send(O.msg(O.Election, from_=1, to=1))
    nt.send(O.msg(O.RequestVoteResp, from_=3, to=1, term=term + 1))
    nt.send(O.msg(O.Propose, from_=1, to=1, entries=[O.Entry()]))
    assert _ltoa(lead) == _ltoa(follower)
    # the synced log is the leader's figure-7 log plus its no-op and the proposal
    assert _all(lead)[:10] == [tuple(x) for x in v["leader"]]
    assert lead.last_index == 12
