"""The node-layer boundary on the CPU tier: the device step code (rbe_step.h /
rbe_fast.h, compiled for the host in tests/soa_cpu) driven through the same
input staging as the HIP engine (rbe_host.h), against the oracle harness, round
by round, every replica field plus its trace digest and listener events.

Covers (include/rbe.h):
  * rbe_push_proposals (multi-entry batches, 0-16 B Cmd) / rbe_push_read_index
    at any replica: followers forward, candidates drop (ProposalDropped /
    ReadIndexDropped events), leaders append / queue — peer.go:117, 297;
  * rbe_request_leader_transfer (peer.go:106): LeaderTransfer → TimeoutNow →
    the target campaigns with the transfer hint (raft.go:1712-1734, 1906-1916);
  * rbe_report_unreachable / rbe_report_snapshot_status (peer.go:168, 177);
  * rbe_notify_applied with ext_apply: raft.applied lags processed, and
    hasConfigChangeToApply (committed > applied, raft.go:1460-1472) skips
    campaigns (CampaignSkipped);
  * RBE_STEP_NO_TICK rounds (a replica without an event makes no step);
  * the seeded leader-transfer schedule (xfer_period) of the harness.
"""
import pytest

import oracle as O
from input_util import run_driven
from parity_util import C2, C3, C4, MIXED, run_lockstep
from soa_cpu.soa import SoaCpu

EXTRA = {"C3": dict(), "C3_N7": dict(), "MIXED": dict()}


# Host-driven rounds put more traffic on one (sender, destination) stream than
# the lockstep workloads (a forwarded ReadIndex each triggers a heartbeat
# broadcast, every forwarded proposal a Replicate): the per-round message and
# entry capacities are raised so the test exercises the protocol, not F_OUTBOX.
DRIVEN = dict()
# a leader of 7 copies a range for each of six remotes in one round
DRIVEN_BY_NAME = {"C3_N7": dict()}


def _pair(kw, name="", **more):
    kw = dict(kw, **more)
    eng_kw = dict(kw)
    eng_kw.update(EXTRA.get(name, {}))
    if kw.get("ext_inputs"):
        eng_kw.update(DRIVEN)
        eng_kw.update(DRIVEN_BY_NAME.get(name, {}))
    return SoaCpu(trace=True, **eng_kw), O.Harness(**kw)


@pytest.mark.parametrize("name,kw", [("C2", C2), ("C3", C3), ("C4", C4),
                                     ("C3_N7", dict(C3, n_groups=24, n_replicas=7))])
def test_driven_inputs_parity(name, kw):
    kw = dict(kw, n_groups=min(kw["n_groups"], 16))
    eng, ref = _pair(kw, name, ext_inputs=True)
    d = run_driven(eng, ref, 160, seed=7)
    assert d is None, f"{name}: first divergence {d}"
    assert eng.faults()[0] == 0


def test_driven_inputs_with_lagging_applied():
    """ext_apply: the host reports an applied index 0-3 entries behind what it
    was handed; an election falls due while committed > applied is skipped."""
    kw = dict(C3, n_groups=12)
    eng, ref = _pair(kw, "C3", ext_inputs=True, ext_apply=True)
    d = run_driven(eng, ref, 200, seed=11, ext_apply=True)
    assert d is None, f"first divergence {d}"
    assert eng.faults()[0] == 0


@pytest.mark.parametrize("name,kw", [("C2", C2), ("C3", C3)])
def test_apply_ready_gate(name, kw):
    """rbe_set_apply_ready: while a node's apply queue is full
    (canHaveMoreEntriesToApply false, node.go:1002-1004) its Update carries no
    CommittedEntries (peer.go:329-331, HasUpdate 253-280); entries wait and are
    applied once it is ready again.  With a lagging applied index too."""
    kw = dict(kw, n_groups=12)
    eng, ref = _pair(kw, name, ext_inputs=True, ext_apply=True)
    # a held replica's unapplied entries must stay in the device window
    eng = SoaCpu(trace=True, **dict(kw, ext_inputs=True, ext_apply=True, **dict(DRIVEN)))
    d = run_driven(eng, ref, 200, seed=13, ext_apply=True, ready=0.2)
    assert d is None, f"{name}: first divergence {d}"
    assert eng.faults()[0] == 0


def test_campaign_skipped_while_applied_lags():
    """hasConfigChangeToApply (raft.go:1460-1472): with the state machine
    holding applied at 0, an election timeout skips the campaign and fires
    CampaignSkipped; once applied catches up the node campaigns."""
    kw = dict(n_groups=1, n_replicas=3)
    eng, ref = _pair(kw, ext_inputs=True, ext_apply=True)
    skipped = launched = 0
    for rnd in range(40):
        if rnd >= 25:  # the state machine catches up
            for r in range(3):
                v = ref.views()[r]
                eng.notify_applied([r], [v.processed])
                ref.push(O.PUSH_APPLIED, r, v.processed)
        eng.step()
        ref.step()
        ev, rv = eng.views(), ref.views()
        for i in range(3):
            assert ev[i].events == rv[i].events and ev[i].term == rv[i].term, (rnd, i)
            skipped += bool(rv[i].events & 4)
            launched += bool(rv[i].events & 2)
    assert skipped > 0 and launched > 0


@pytest.mark.parametrize("tick_every", [2, 3])
def test_rounds_without_tick(tick_every):
    kw = dict(C4, n_groups=24)
    eng, ref = _pair(kw, ext_inputs=True)
    d = run_driven(eng, ref, 300, seed=3, tick_every=tick_every, density=0.05)
    assert d is None, f"first divergence {d}"
    # untraced: lazy quiesced ticks must count ticks, not rounds
    eng2 = SoaCpu(trace=False, **dict(kw, ext_inputs=True))
    ref2 = O.Harness(**dict(kw, ext_inputs=True))
    d = run_driven(eng2, ref2, 300, seed=3, tick_every=tick_every, density=0.05,
                   skip=("digest",))
    assert d is None, f"untraced: first divergence {d}"


@pytest.mark.parametrize("name,kw", [("C2", C2), ("C3", C3), ("MIXED", MIXED),
                                     ("C3_N7", dict(C3, n_groups=24, n_replicas=7))])
def test_leader_transfer_schedule_parity(name, kw):
    """The seeded RequestLeaderTransfer schedule: transfers happen (TimeoutNow,
    a campaign with the transfer hint, a new leader) and every replica stays
    bit-exact with the oracle; also through the full handler table only."""
    kw = dict(kw, xfer_period=23, xfer_mod=2)
    eng, ref = _pair(kw, name)
    d = run_lockstep(eng, ref, 400, every=1)
    assert d is None, f"{name}: first divergence {d}"
    assert eng.faults()[0] == 0
    c = ref.counters()
    assert c["campaigns"] > kw["n_groups"], "the transfers never started a campaign"
    full, ref2 = SoaCpu(trace=True, full_only=True, **dict(kw, **EXTRA.get(name, {}))), O.Harness(**kw)
    d = run_lockstep(full, ref2, 200, every=1)
    assert d is None, f"{name} (full table only): first divergence {d}"


def test_transfer_moves_leadership():
    """RequestLeaderTransfer at the leader: the target becomes leader of the
    next term (raft.go:1712-1734 → TimeoutNow → handleFollowerTimeoutNow)."""
    kw = dict(n_groups=1, n_replicas=3)
    eng, ref = _pair(kw, ext_inputs=True)
    eng.run(30)
    ref.run(30)
    v = ref.views()
    lead = [i for i in range(3) if v[i].role == O.LEADER][0]
    target = (lead + 1) % 3 + 1
    eng.request_leader_transfer([lead], [target])
    ref.push(O.PUSH_XFER, lead, target)
    for _ in range(6):
        eng.step()
        ref.step()
    ev, rv = eng.views(), ref.views()
    assert rv[target - 1].role == O.LEADER and rv[target - 1].term == v[lead].term + 1
    for i in range(3):
        assert (ev[i].role, ev[i].term, ev[i].leader_id, ev[i].digest) == \
            (rv[i].role, rv[i].term, rv[i].leader_id, rv[i].digest)


def test_push_batches_are_all_or_nothing():
    from dragonboat_amd.engine import InputError, RBE_E_INVALID, RBE_E_STATE
    eng = SoaCpu(trace=True, n_groups=2, n_replicas=3, ext_inputs=True)
    with pytest.raises(InputError) as ei:  # a replica out of range stages nothing
        eng.push_proposals([0, 99], [[b"a"], [b"b"]])
    assert ei.value.rc == RBE_E_INVALID
    with pytest.raises(InputError) as ei:  # the same replica twice in one batch
        eng.push_read_index([1, 1], [(5, 0), (6, 0)])
    assert ei.value.rc == RBE_E_STATE
    eng.push_proposals([0], [[b"x" * 16]])
    with pytest.raises(InputError) as ei:  # a second batch for a replica this step
        eng.push_proposals([0], [[b"y"]])
    assert ei.value.rc == RBE_E_STATE
    with pytest.raises(InputError) as ei:  # Cmd > 16 bytes without a payload heap
        eng.push_proposals([1], [[b"z" * 17]])
    assert ei.value.rc == RBE_E_INVALID
    with pytest.raises(InputError):  # ctx.Low == 0 (requests.go:726)
        eng.push_read_index([2], [(0, 1)])
    with pytest.raises(InputError):  # transfer target outside the group
        eng.request_leader_transfer([2], [4])
    with pytest.raises(InputError):  # applied without ext_apply
        eng.notify_applied([0], [1])
    eng.step()
    eng.push_proposals([0], [[b"y"]])  # the next step takes a new batch
    # a failed batch is undone whole: records it created go, records an
    # earlier call staged keep their parts
    eng.push_proposals([4], [[b"p"]])
    with pytest.raises(InputError) as ei:
        eng.push_read_index([3, 4, 5, 3], [(7, 0)] * 4)
    assert ei.value.rc == RBE_E_STATE
    eng.push_read_index([3, 4, 5], [(7, 0)] * 3)
    with pytest.raises(InputError) as ei:
        eng.push_proposals([2, 5, 2], [[b"a"], [b"b"], [b"c"]])
    assert ei.value.rc == RBE_E_STATE
    eng.push_proposals([2, 5], [[b"a"], [b"b"]])
    with pytest.raises(InputError) as ei:
        eng.push_proposals([4], [[b"q"]])
    assert ei.value.rc == RBE_E_STATE


@pytest.mark.parametrize("quiesce", [False, True])
def test_leader_inputs_fast_path(quiesce):
    """Host ReadIndexes and single inline proposals at leaders (the node
    layer's steady traffic, bench c4h) take the fast leader step, bit-exact
    with the oracle; the full handler table sees only the rounds it would
    without input."""
    import random
    from input_util import apply_engine, apply_oracle, leader_inputs_round
    from parity_util import counters_match, view_diff
    kw = dict(n_groups=40, n_replicas=3, quiesce=quiesce, ext_inputs=True)
    eng = SoaCpu(trace=True, **kw)
    ref = O.Harness(**kw)
    rng = random.Random(17)
    views = ref.views()
    pushed = 0
    slow0 = None
    for rnd in range(260):
        if rnd >= 60:
            ops = leader_inputs_round(rng, views, 3, rnd)
            pushed += len(ops)
            apply_engine(eng, ops)
            apply_oracle(ref, ops)
        if rnd == 60:
            slow0 = eng.slow_total()
        eng.step()
        ref.step()
        ev, views = eng.views(), ref.views()
        for i in range(len(views)):
            d = view_diff(ev[i], views[i])
            assert d is None, f"round {rnd} replica {i}: {d}"
    assert not counters_match(eng.counters(), ref.counters())
    assert pushed > 3000
    # the 200 input rounds put ~4000 inputs at leaders; nearly all are stepped fast
    assert eng.slow_total() - slow0 < pushed // 10, (eng.slow_total() - slow0, pushed)
