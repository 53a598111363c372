"""Whole raftpb.Entry values through the engine boundary (include/rbe.h
rbe_propose_entries, rbe_get_entries, rbe_get_outbox / rbe_push_messages,
rbe_wire_encode): the session fields Key / ClientID / SeriesID / RespondedTo
that requests.go:994-997 stamps on every client proposal, and Cmds of any
length, checked against the oracle harness's LogDB (its Entry carries every
field, oracle/raft_ref.h)."""
import wire as W

SESSION = ("key", "client_id", "series_id", "responded_to")


def check_entry_records(eng, ref, n_groups, n, ring, pushed=None):
    """Every replica's log window [max(1, last - ring + 1), last] equals the
    oracle's LogDB entry by entry: Index, Term, Type, session fields and the
    Cmd (the oracle hands back at most 64 Cmd bytes; `pushed` holds every
    whole Cmd the host proposed).  Returns the number of entries checked and
    how many of them carried session fields."""
    views = ref.views()
    checked = with_session = 0
    for r in range(n_groups * n):
        last = views[r].last_index
        lo = max(1, last - ring + 1)
        if last < lo:
            continue
        got = eng.entry_records(r, lo, last)
        exp = ref.persisted_entries(r, lo, last)
        for g, x in zip(got, exp):
            assert (g["index"], g["term"], g["type"]) == (x.index, x.term, x.type), (r, g, x)
            assert tuple(g[f] for f in SESSION) == tuple(getattr(x, f) for f in SESSION), (r, g["index"])
            assert g["cmd"][:64] == x.cmd[:64], (r, g["index"])
            if pushed is not None and len(g["cmd"]) > 16:
                assert g["cmd"] in pushed, (r, g["index"], len(g["cmd"]))
            checked += 1
            with_session += any(g[f] for f in SESSION)
    return checked, with_session


def check_outbox_decodes(eng, n_groups, n, gpb=0, deployment_id=0x5E55, bin_ver=210,
                         addrs=("a:1", "b:2", "c:3", "d:4", "e:5"), device_decode=False):
    """The engine's frames of the last round, decoded by the oracle's wire
    restatement (oracle/wire.py frames_decode), equal the engine's outbox
    records field by field, entries with session fields and whole Cmds
    included; with `device_decode` rbe_wire_decode must read the same records
    back on the device.  Returns (messages, entries with session fields,
    Propose messages with entries)."""
    got = eng.wire_encode(deployment_id, bin_ver, gpb, addrs[:n])
    stream = eng.wire_fetch(got)[0] if hasattr(eng, "wire_fetch") else got[0]
    out = {}
    for r in range(n_groups * n):
        g, k = divmod(r, n)
        msgs, ents, cmds = eng.outbox(r)
        ei = 0
        for m in msgs:
            es = []
            for _ in range(m.n_entries):
                e = ents[ei]
                es.append(dict(term=e.term, index=e.index, type=e.type, cmd=cmds[ei],
                               **{f: getattr(e, f) for f in SESSION}))
                ei += 1
            if m.type == W.INSTALL_SNAPSHOT:
                continue
            out.setdefault((k, m.to - 1), {}).setdefault(g, []).append((m, es))
    decoded = [W.batch_decode(p) for p in W.frames_decode(stream)]
    seen = ses = props = 0
    frames = iter(decoded)
    for k in range(n):
        for d in range(n):
            if d == k or (k, d) not in out:
                continue
            cells = out[(k, d)]
            gs = sorted(cells)
            for g0 in range(0, n_groups, gpb or n_groups):
                exp = [x for g in gs if g0 <= g < g0 + (gpb or n_groups) for x in cells[g]]
                if not exp:
                    continue
                batch = next(frames)
                assert batch["source_address"] == addrs[k]
                assert len(batch["requests"]) == len(exp)
                for (dm, dents), (m, es) in zip(batch["requests"], exp):
                    assert dm["type"] == m.type and dm["to"] == m.to and dm["from"] == m.from_
                    assert (dm["term"], dm["log_index"], dm["commit"]) == (m.term, m.log_index,
                                                                           m.commit)
                    assert len(dents) == len(es)
                    for de, e in zip(dents, es):
                        assert de == e, (de, e)
                        ses += any(e[f] for f in SESSION)
                    props += m.type == 7 and len(es) > 0
                    seen += 1
    assert next(frames, None) is None
    if device_decode and stream:
        dmsgs, dents, dcmd = eng.wire_decode(stream)
        exp_m = [req for b in decoded for req in b["requests"]]
        assert len(dmsgs) == len(exp_m)
        ei = ci = 0
        for m, (em, ee) in zip(dmsgs, exp_m):
            assert (m.type, m.to, m.from_, m.cluster_id, m.term, m.log_term, m.log_index,
                    m.commit, m.reject, m.hint, m.hint_high) == tuple(
                em[f] for f in ("type", "to", "from", "cluster_id", "term", "log_term",
                                "log_index", "commit", "reject", "hint", "hint_high"))
            assert m.n_entries == len(ee)
            for x in ee:
                e = dents[ei]
                ei += 1
                got = dict(term=e.term, index=e.index, type=e.type, cmd=dcmd[ci:ci + e.cmd_len],
                           **{f: getattr(e, f) for f in SESSION})
                ci += e.cmd_len
                assert got == x
    return seen, ses, props
