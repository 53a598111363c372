"""Pin the oracle's remote (remote.go) against the reference's remote_test.go
tables, transcribed as vectors in tests/golden/remote.json."""
import json
import os

import pytest

import oracle as O

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "remote.json")))


@pytest.mark.parametrize("case", G["responded_to"]["cases"])
def test_responded_to(case):
    st, match, nxt, snap, exp_st, exp_next = case
    r = O.Remote(match=match, next=nxt, snapshot_index=snap, state=st)
    r.op("responded_to")
    assert (r.state, r.next) == (exp_st, exp_next)


@pytest.mark.parametrize("case", G["try_update"]["cases"])
def test_try_update(case):
    idx, paused, exp_match, exp_next, exp_paused, exp_updated = case
    init = G["try_update"]["init"]
    r = O.Remote(match=init["match"], next=init["next"])
    if paused:
        r.op("retry_to_wait")
    assert bool(r.op("try_update", idx)) == exp_updated
    assert (r.match, r.next) == (exp_match, exp_next)
    if exp_paused:
        assert r.state == O.REMOTE_WAIT


@pytest.mark.parametrize("case", G["decrease_to_replicate"]["cases"])
def test_decrease_to_in_replicate_state(case):
    match, nxt, rejected, exp_dec, exp_next = case
    r = O.Remote(match=match, next=nxt, state=O.REMOTE_REPLICATE)
    assert bool(r.op("decrease_to", rejected, G["decrease_to_replicate"]["last"])) == exp_dec
    assert r.next == exp_next


@pytest.mark.parametrize("case", G["decrease_to_not_replicate"]["cases"])
@pytest.mark.parametrize("state", G["decrease_to_not_replicate"]["states"])
def test_decrease_to_not_replicate_state(case, state):
    match, nxt, rejected, last, exp_dec, exp_next = case
    r = O.Remote(match=match, next=nxt, state=state)
    r.op("retry_to_wait")
    assert bool(r.op("decrease_to", rejected, last)) == exp_dec
    assert r.next == exp_next
    if exp_dec:
        assert r.state != O.REMOTE_WAIT


@pytest.mark.parametrize("case", G["is_paused"]["cases"])
def test_is_paused(case):
    st, exp = case
    assert bool(O.Remote(state=st).op("is_paused")) == exp


def test_is_paused_panics_on_invalid_state():  # remote_test.go:159-170
    with pytest.raises(O.RaftPanic):
        O.Remote(state=100).op("is_paused")


@pytest.mark.parametrize("case", G["become_retry"]["cases"])
def test_become_retry(case):
    st, match, snap, exp_next = case
    r = O.Remote(match=match, snapshot_index=snap, state=st)
    r.op("become_retry")
    assert r.next == exp_next and r.state == O.REMOTE_RETRY and r.snapshot_index == 0


@pytest.mark.parametrize("case", G["progress"]["cases"])
def test_progress(case):
    st, match, nxt, last, exp_next, exp_paused, exp_panic = case
    r = O.Remote(match=match, next=nxt, state=st)
    if exp_panic:
        with pytest.raises(O.RaftPanic):
            r.op("progress", last)
        return
    assert not r.op("is_paused")
    r.op("progress", last)
    assert r.next == exp_next and r.match == match
    assert bool(r.op("is_paused")) == exp_paused


@pytest.mark.parametrize("st", [O.REMOTE_REPLICATE, O.REMOTE_RETRY, O.REMOTE_SNAPSHOT])
def test_become_snapshot(st):  # remote_test.go:103-118
    r = O.Remote(match=10, next=11, state=st)
    r.op("become_snapshot", 12)
    assert (r.state, r.match, r.snapshot_index) == (O.REMOTE_SNAPSHOT, 10, 12)


def test_become_replication():  # remote_test.go:114-124
    r = O.Remote(match=10, next=11, state=O.REMOTE_RETRY)
    r.op("become_replicate")
    assert (r.state, r.match, r.next) == (O.REMOTE_REPLICATE, 10, 11)


def test_set_active():  # remote_test.go:46-63
    r = O.Remote()
    r.op("set_active")
    assert r.op("is_active")
    r.op("set_not_active")
    assert not r.op("is_active")


def test_try_update_cause_resume():  # remote_test.go:323-335
    r = O.Remote(next=5)
    r.op("retry_to_wait")
    r.op("decrease_to", 4, 4)
    assert r.state != O.REMOTE_WAIT
    r.op("retry_to_wait")
    r.op("try_update", 5)
    assert r.state != O.REMOTE_WAIT
