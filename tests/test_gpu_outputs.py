"""rbe_collect_outputs on the HIP engine: the device-compacted batch of every
replica's Update.Messages and ReadyToReads (node.go:907-923 read for all nodes
at once) equals what the per-replica calls rbe_get_messages /
rbe_get_ready_to_reads return, round after round, for whole engines and for
replica sub-ranges; rounds that read at followers and leaders (C4) and
elections with rejections (C3) included."""
import numpy as np
import pytest

from parity_util import C2, C3, C4

pytestmark = pytest.mark.gpu

FIELDS = ("type", "reject", "to", "from_", "cluster_id", "term", "log_term", "log_index",
          "commit", "hint", "hint_high", "n_entries")


def _check(eng, first, count):
    moff, msgs, roff, rtrs = eng.collect_outputs(first, count)
    assert moff[0] == 0 and roff[0] == 0
    assert moff[-1] == len(msgs) and roff[-1] == len(rtrs)
    for i in range(count):
        ref = eng.messages(first + i)
        got = msgs[moff[i]:moff[i + 1]]
        assert len(got) == len(ref), (first + i, len(got), len(ref))
        for a, b in zip(got, ref):
            assert tuple(a[f] for f in FIELDS) == tuple(getattr(b, f) for f in FIELDS)
        rr = eng.ready_to_reads(first + i)
        gr = [tuple(x) for x in rtrs[roff[i]:roff[i + 1]].tolist()]
        assert gr == [tuple(x) for x in rr], (first + i, gr, rr)
    return len(msgs), len(rtrs)


@pytest.mark.parametrize("name,kw,extra", [("C2", C2, {}), ("C3", C3, dict()),
                                           ("C4", C4, {})])
def test_gpu_collect_outputs_match_per_replica(gpu_available, name, kw, extra):
    from dragonboat_amd.engine import Engine
    kw = dict(kw, n_groups=min(kw["n_groups"], 48))
    eng = Engine(device=0, trace=True, **dict(kw, **extra))
    nm = nr = 0
    for rnd in range(120):
        eng.step()
        if rnd % 7 == 3 or rnd > 110:
            a, b = _check(eng, 0, eng.n_rep)
            nm, nr = nm + a, nr + b
            _check(eng, 5, eng.n_rep - 11)  # a sub-range not aligned to groups or blocks
    assert nm > 0
    if name == "C4":
        assert nr > 0
    eng.close()


def test_gpu_collect_outputs_large(gpu_available):
    """A 200k-group C4 engine: offsets span several scan blocks' worth of lists."""
    from dragonboat_amd.engine import Engine
    eng = Engine(device=0, **dict(C4, n_groups=200_000))
    eng.run(260)
    moff, msgs, roff, rtrs = eng.collect_outputs()
    assert np.all(np.diff(moff.astype(np.int64)) >= 0) and moff[-1] == len(msgs)
    assert np.all(np.diff(roff.astype(np.int64)) >= 0) and roff[-1] == len(rtrs)
    assert len(msgs) > 10_000 and len(rtrs) > 1_000
    for r in (0, 1, 2, 99_999, 599_997, 599_999):
        assert moff[r + 1] - moff[r] == len(eng.messages(r))
        assert roff[r + 1] - roff[r] == len(eng.ready_to_reads(r))
    eng.close()


@pytest.mark.parametrize("name,kw,extra", [("C3", C3, dict()), ("C4", C4, {})])
def test_gpu_collect_updates_match_per_replica(gpu_available, name, kw, extra):
    """rbe_collect_updates returns exactly the replicas whose rbe_get_updates
    record has RBE_UF_HAS_UPDATE, ascending, each with the same record."""
    from dragonboat_amd import engine as E
    kw = dict(kw, n_groups=min(kw["n_groups"], 48))
    eng = E.Engine(device=0, trace=True, **dict(kw, **extra))
    seen = 0
    for rnd in range(120):
        eng.step()
        if rnd % 5 != 2 and rnd < 110:
            continue
        for first, count in ((0, eng.n_rep), (5, eng.n_rep - 11)):
            rep, ups = eng.collect_updates(first, count)
            full = np.frombuffer(bytes(eng.updates(first, count)), E.UPDATE_DTYPE)
            want = np.nonzero(full["flags"] & E.UF_HAS_UPDATE)[0]
            assert rep.tolist() == (want + first).tolist()
            assert ups.tobytes() == full[want].tobytes()
            seen += len(rep)
    assert seen > 0
    eng.close()


def test_gpu_collect_updates_large(gpu_available):
    """200k C4 groups: the compacted Updates span many scan blocks."""
    from dragonboat_amd import engine as E
    eng = E.Engine(device=0, **dict(C4, n_groups=200_000))
    eng.run(260)
    rep, ups = eng.collect_updates()
    full = np.frombuffer(bytes(eng.updates()), E.UPDATE_DTYPE)
    want = np.nonzero(full["flags"] & E.UF_HAS_UPDATE)[0]
    assert len(want) > 1000
    assert np.array_equal(rep, want.astype(np.uint64))
    assert ups.tobytes() == full[want].tobytes()
    eng.close()


@pytest.mark.parametrize("name,kw,extra", [("C3", C3, dict()), ("C4", C4, {})])
def test_gpu_collect_outputs_match_oracle(gpu_available, name, kw, extra):
    """rbe_collect_outputs against the oracle harness itself, not the engine's
    own getters: every sender's messages of the round, per destination, equal
    (type, from, to, term, log_term, log_index, commit, reject, hint, number
    of entries) the messages the oracle's network delivers to that destination
    from that sender next round (the Quiesce notice aside: it is not a
    Update.Messages entry in the engine's list form)."""
    import oracle as O
    from dragonboat_amd.engine import Engine
    kw = dict(kw, n_groups=min(kw["n_groups"], 40))
    eng = Engine(device=0, trace=True, **dict(kw, **extra))
    ref = O.Harness(**kw)
    n = kw["n_replicas"]
    checked = 0
    for rnd in range(150):
        eng.step()
        ref.step()
        if rnd % 3:
            continue
        moff, msgs, _, _ = eng.collect_outputs()
        for s in range(eng.n_rep):
            g, k = divmod(s, n)
            got = msgs[moff[s]:moff[s + 1]]
            for d in range(n):
                if d == k:
                    continue
                mine = [(int(m["type"]), int(m["from_"]), int(m["to"]), int(m["term"]),
                         int(m["log_term"]), int(m["log_index"]), int(m["commit"]),
                         int(m["reject"]), int(m["hint"]), int(m["n_entries"]))
                        for m in got if int(m["to"]) == d + 1]
                want = [t for t in ref.inbox(g * n + d, k) if t[0] != 21]
                assert mine == want, (rnd + 1, s, d, mine, want)
                checked += len(want)
    assert checked > 500
    eng.close()


@pytest.mark.parametrize("name,kw,extra", [("C2", C2, {}), ("C3", C3, dict()),
                                           ("C4", C4, {})])
def test_gpu_collect_step_matches(gpu_available, name, kw, extra):
    """rbe_collect_step: the Updates of rbe_collect_updates, and for exactly
    those replicas the messages / ReadyToReads of rbe_collect_outputs (every
    replica with outputs has an Update); with RBE_COLLECT_REMOTE_MSGS and one
    replica set per engine no message comes back (all are delivered on the
    device)."""
    from dragonboat_amd.engine import Engine
    kw = dict(kw, n_groups=min(kw["n_groups"], 48))
    eng = Engine(device=0, trace=True, **dict(kw, **extra))
    seen = [0, 0, 0, 0]
    for rnd in range(120):
        eng.step()
        first, count = (0, eng.n_rep) if rnd % 3 else (5, eng.n_rep - 9)
        rep, ups, moff, msgs, roff, rtrs = eng.collect_step(first, count)
        rep_u, ups_u = eng.collect_updates(first, count)
        assert list(rep) == list(rep_u)
        assert ups.tobytes() == ups_u.tobytes()
        om, allm, orr, allr = eng.collect_outputs(first, count)
        assert moff[-1] == len(msgs) and roff[-1] == len(rtrs)
        with_out = {first + i for i in range(count)
                    if om[i + 1] > om[i] or orr[i + 1] > orr[i]}
        assert with_out <= set(int(x) for x in rep), "outputs of a replica without an Update"
        for j, r in enumerate(rep):
            i = int(r) - first
            a, b = msgs[moff[j]:moff[j + 1]], allm[om[i]:om[i + 1]]
            assert a.tobytes() == b.tobytes(), (rnd, int(r))
            a, b = rtrs[roff[j]:roff[j + 1]], allr[orr[i]:orr[i + 1]]
            assert a.tobytes() == b.tobytes(), (rnd, int(r))
        assert len(msgs) == len(allm) and len(rtrs) == len(allr)
        r2, u2, mo2, m2, ro2, t2 = eng.collect_step(first, count, remote_only=True)
        assert len(m2) == 0 and list(r2) == list(rep) and t2.tobytes() == rtrs.tobytes()
        # RBE_COLLECT_SKIP_LOCAL: only the Updates with more than locally
        # delivered messages, the same records and ReadyToReads
        r3, u3, _, m3, ro3, t3 = eng.collect_step(first, count, remote_only=True, skip_local=True)
        keep = [j for j in range(len(rep)) if _actionable(ups[j])]
        assert list(r3) == [int(rep[j]) for j in keep], rnd
        assert u3.tobytes() == ups[keep].tobytes() and len(m3) == 0
        assert t3.tobytes() == rtrs.tobytes()  # every ReadyToRead is in a kept Update
        seen[3] += len(rep) - len(r3)
        seen[0] += len(rep)
        seen[1] += len(msgs)
        seen[2] += len(rtrs)
    assert seen[0] and seen[1] and seen[3], seen
    if name == "C4":
        assert seen[2], seen
    eng.close()


def _actionable(u):
    """An Update the node has work for besides its messages (RBE_COLLECT_SKIP_LOCAL)."""
    from dragonboat_amd import engine as E
    return bool(int(u["flags"]) & (E.UF_STATE_CHANGED | E.UF_SENT_QUIESCE | E.UF_SNAPSHOT |
                                   E.UF_APPLIED)) or \
        bool(u["events"] or u["n_ready_to_read"] or u["n_dropped_entries"] or
             u["n_dropped_read_indexes"] or u["save_lo"] <= u["save_hi"] or
             u["apply_lo"] <= u["apply_hi"])


def test_gpu_collect_untraced_group_sleep(gpu_available):
    """Untraced C4 (lazy quiesced ticks, group sleep): the collect passes skip
    the groups asleep after the round, and still return exactly the replicas
    whose rbe_get_updates record has an Update, round after round."""
    from dragonboat_amd import engine as E
    eng = E.Engine(device=0, trace=False, **dict(C4, n_groups=3000))
    seen = 0
    for rnd in range(300):
        eng.step()
        if rnd < 25:
            continue
        full = np.frombuffer(bytes(eng.updates()), E.UPDATE_DTYPE)
        want = np.nonzero(full["flags"] & E.UF_HAS_UPDATE)[0]
        rep, ups = eng.collect_updates()
        assert np.array_equal(rep, want.astype(np.uint64)), rnd
        assert ups.tobytes() == full[want].tobytes()
        rep2, ups2, _, _, _, _ = eng.collect_step()
        assert np.array_equal(rep2, rep) and ups2.tobytes() == ups.tobytes()
        seen += len(rep)
    assert seen > 1000
    eng.close()
