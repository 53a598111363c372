"""Drive an engine (the HIP engine or the test-only host build) and the oracle
harness with the same host input, round by round: the node-layer calls of
handleEvents (node.go:1030-1067) — proposal batches, ReadIndex, leader
transfer, Unreachable / SnapshotStatus reports, the state machine's applied
index — plus rounds without a tick.  The schedule is a seeded function of the
round and of the state both sides already agree on (processed indexes), so
both receive identical input."""
from __future__ import annotations

import random

import oracle as O
from parity_util import counters_match, view_diff


def _cmd(rng):
    return bytes(rng.randrange(256) for _ in range(rng.randrange(17)))


def session_entry(rng, cmd):
    """A client proposal as requests.go:994-997 stamps it: Key, ClientID,
    SeriesID, RespondedTo (values below 2^49 and colfer's 9-byte form above),
    sometimes none (a NoOPSession proposal without a key)."""
    def v():
        u = rng.random()
        return 0 if u < 0.15 else (rng.randrange(1, 1 << 20) if u < 0.6 else
                                   rng.randrange(1 << 49, 1 << 64))
    e = O.Entry(type=rng.choice((0, 0, 2, 3)), cmd=cmd(rng))
    if rng.random() < 0.85:
        e.key, e.client_id, e.series_id, e.responded_to = v(), v(), v(), v()
    return e


def plan_round(rng, n_rep, n, rnd, views, ext_apply, density=0.3, applied=None, cmd=None,
               ready=0.0, session=False, props_only=False):
    """One round of host input: a list of (kind, replica, args).  `cmd(rng)`
    draws a proposal's Cmd (default: 0-16 bytes); `session` proposes whole
    raftpb.Entry values with session fields (session_entry); `props_only`
    draws proposals alone."""
    cmd = cmd or _cmd
    ops = []
    for r in range(n_rep):
        if rng.random() < density:
            if session:
                ops.append(("prop", r, [session_entry(rng, cmd)
                                        for _ in range(rng.randrange(1, 4))]))
            else:
                ops.append(("prop", r, [(rng.choice((0, 0, 2, 3)), cmd(rng))
                                        for _ in range(rng.randrange(1, 4))]))
        if props_only:
            continue
        if rng.random() < density:
            ops.append(("read", r, ((rnd + 1) << 32 | (r + 1), rng.randrange(1 << 40))))
        if rng.random() < density / 6:
            ops.append(("xfer", r, rng.randrange(1, n + 1)))
        if rng.random() < density / 8:
            ops.append(("unreach", r, rng.randrange(1, n + 1)))
        if rng.random() < density / 8:
            ops.append(("snapst", r, (rng.randrange(1, n + 1), rng.random() < 0.5)))
        if ext_apply:
            # the state machine lags the entries handed to it by 0-3 entries;
            # its applied index never moves backwards (node.go:911-913)
            v = max(applied[r], views[r].processed - rng.randrange(4))
            applied[r] = v
            ops.append(("applied", r, v))
        if ready and rng.random() < ready:
            # the node's apply queue fills up / drains (canHaveMoreEntriesToApply)
            ops.append(("ready", r, rng.random() < 0.6))
    return ops


def apply_engine(eng, ops):
    by = {}
    for kind, r, a in ops:
        by.setdefault(kind, []).append((r, a))
    if "prop" in by:
        eng.push_proposals([r for r, _ in by["prop"]], [a for _, a in by["prop"]])
    if "read" in by:
        eng.push_read_index([r for r, _ in by["read"]], [a for _, a in by["read"]])
    if "xfer" in by:
        eng.request_leader_transfer([r for r, _ in by["xfer"]], [a for _, a in by["xfer"]])
    if "unreach" in by:
        eng.report_unreachable([r for r, _ in by["unreach"]], [a for _, a in by["unreach"]])
    if "snapst" in by:
        eng.report_snapshot_status([r for r, _ in by["snapst"]], [a[0] for _, a in by["snapst"]],
                                   [a[1] for _, a in by["snapst"]])
    if "applied" in by:
        eng.notify_applied([r for r, _ in by["applied"]], [a for _, a in by["applied"]])
    if "ready" in by:
        eng.set_apply_ready([r for r, _ in by["ready"]], [a for _, a in by["ready"]])


def _oracle_entry(x):
    if isinstance(x, tuple):
        return O.Entry(type=x[0], cmd=x[1])
    return O.Entry(type=x.type, cmd=x.cmd, key=x.key, client_id=x.client_id,
                   series_id=x.series_id, responded_to=x.responded_to)


def apply_oracle(h, ops):
    for kind, r, a in ops:
        if kind == "prop":
            h.push(O.PUSH_PROPOSE, r, entries=[_oracle_entry(x) for x in a])
        elif kind == "read":
            h.push(O.PUSH_READ, r, a[0], a[1])
        elif kind == "xfer":
            h.push(O.PUSH_XFER, r, a)
        elif kind == "unreach":
            h.push(O.PUSH_UNREACH, r, a)
        elif kind == "snapst":
            h.push(O.PUSH_SNAPST, r, a[0], int(a[1]))
        elif kind == "applied":
            h.push(O.PUSH_APPLIED, r, a)
        elif kind == "ready":
            h.push(O.PUSH_APPLY_READY, r, int(a))


def run_driven(eng, ref, rounds, seed=1, tick_every=1, inputs=True, ext_apply=False,
               density=0.3, skip=(), cmd=None, on_ops=None, ready=0.0, before_round=None,
               session=False):
    """Step both `rounds` rounds with the same input; every `tick_every`-th
    round ticks, the others are RBE_STEP_NO_TICK rounds.  Returns the first
    divergence (round, replica, field, engine, oracle) or None."""
    rng = random.Random(seed)
    n = eng.cfg.n_replicas
    n_rep = eng.n_rep
    views = ref.views()
    applied = [0] * n_rep
    for rnd in range(rounds):
        if before_round:
            before_round(rnd)
            views = ref.views()
        if inputs:
            ops = plan_round(rng, n_rep, n, rnd, views, ext_apply, density, applied, cmd, ready,
                             session)
            if on_ops:
                on_ops(ops)
            apply_engine(eng, ops)
            apply_oracle(ref, ops)
        tick = (rnd % tick_every) == 0
        eng.step(tick=tick)
        ref.step(tick=tick)
        ev, views = eng.views(), ref.views()
        for i in range(n_rep):
            d = view_diff(ev[i], views[i], skip)
            if d is not None:
                return (rnd, i) + d
    bad = counters_match(eng.counters(), ref.counters())
    if bad:
        return ("counters", bad)
    return None


def leader_inputs_round(rng, views, n, rnd, density=0.5, read_share=0.9):
    """The node layer's steady traffic (bench c4h): at the leader of a share
    of the groups one ReadIndex, or one proposal of 0-16 bytes (a single
    inline entry, Application or Encoded)."""
    ops = []
    n_groups = len(views) // n
    for g in range(n_groups):
        if rng.random() >= density:
            continue
        lead = [g * n + k for k in range(n) if views[g * n + k].role == O.LEADER]
        if not lead:
            continue
        r = lead[0]
        if rng.random() < read_share:
            ops.append(("read", r, ((rnd + 1) << 32 | (r + 1), rng.randrange(1 << 40))))
        else:
            ops.append(("prop", r, [(rng.choice((0, 0, 2)), _cmd(rng))]))
    return ops
