"""Pin the oracle's entryLog / inMemory (logentry.go, inmemory.go) against the
reference's logentry_test.go / logentry_etcd_test.go tables, transcribed as
vectors in tests/golden/log.json (entries are [index, term])."""
import json
import os

import pytest

import oracle as O

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "log.json")))


def _ents(pairs):
    return [O.Entry(index=i, term=t) for i, t in pairs]


def _log(spec):
    """newEntryLog(TestLogDB{spec.logdb}) + append(spec.append), via a bare raft."""
    db = O.LogDB()
    if spec.get("logdb"):
        db.append(_ents(spec["logdb"]))
    r = O.Raft.new(1, (), logdb=db)
    if spec.get("append"):
        r.log_append(_ents(spec["append"]))
    if "committed" in spec:
        r.committed = spec["committed"]
    return r


@pytest.mark.parametrize("case", G["match_term"]["cases"])
def test_match_term(case):
    idx, term, exp = case
    assert bool(_log(G["match_term"]).log_match_term(idx, term)) == exp


@pytest.mark.parametrize("name", ["up_to_date", "is_up_to_date"])
def test_up_to_date(name):
    spec = G[name]
    r = _log(spec)
    for idx, term, exp in spec["cases"]:
        assert bool(r.log_up_to_date(idx, term)) == exp, (name, idx, term)


@pytest.mark.parametrize("name", ["conflict_index", "find_conflict"])
def test_conflict_index(name):
    spec = G[name]
    for ents, exp in spec["cases"]:
        r = _log(spec)
        assert r.log_conflict_index(_ents(ents)) == exp, (name, ents)


def test_commit_to():
    spec = G["commit_to"]
    r = _log(spec)
    for to, exp in spec["steps"]:
        r.log_commit_to(to)
        assert r.committed == exp


def test_commit_to_unavailable_index_panics():  # logentry_test.go:532-556
    r = _log(G["commit_to"])
    with pytest.raises(O.RaftPanic):
        r.log_commit_to(8)


@pytest.mark.parametrize("case", G["append"]["cases"])
def test_append(case):
    ents, exp_last, exp_ents, exp_marker = case
    r = _log(G["append"])
    r.log_append(_ents(ents))
    assert r.last_index == exp_last
    got, err = r.log_entries(1)
    assert err == O.ERR_OK
    assert [(e.index, e.term) for e in got] == [tuple(x) for x in exp_ents]
    assert r.marker_index == exp_marker


@pytest.mark.parametrize("case", G["maybe_append"]["cases"])
def test_maybe_append(case):
    """handleReplicateMessage's log arm: matchTerm → tryAppend → commitTo(min)."""
    log_term, index, committed, ents, exp_last, exp_append, exp_commit, exp_panic = case
    r = _log(G["maybe_append"])
    glast, gappend = 0, False
    try:
        if r.log_match_term(index, log_term):
            gappend = True
            r.log_try_append(index, _ents(ents))
            glast = index + len(ents)
            r.log_commit_to(min(glast, committed))
    except O.RaftPanic:
        assert exp_panic
        return
    assert not exp_panic
    assert (glast, gappend, r.committed) == (exp_last, exp_append, exp_commit)
    if gappend and ents:
        got, err = r.log_get_entries(r.last_index - len(ents) + 1, r.last_index + 1)
        assert [(e.index, e.term) for e in got] == [tuple(x) for x in ents]
