"""Expected transport frames of an engine's last round, built by the oracle's
wire restatement (oracle/wire.py) from the engine's own outbox records
(rbe_get_outbox, bit-exact with the oracle harness elsewhere), and the
comparison of decoded records with those records."""
import wire as W

INSTALL_SNAPSHOT = W.INSTALL_SNAPSHOT
ADDRS = ("node-1.example:26001", "node-2.example:26001", "node-3.example:26001",
         "node-4.example:26001", "node-5.example:26001", "node-6.example:26001",
         "node-7.example:26001")


def _msg_dict(m):
    return {"type": m.type, "to": m.to, "from": m.from_ if hasattr(m, "from_") else
            getattr(m, "from"), "cluster_id": m.cluster_id, "term": m.term,
            "log_term": m.log_term, "log_index": m.log_index, "commit": m.commit,
            "reject": m.reject, "hint": m.hint, "hint_high": m.hint_high}


SESSION = ("key", "client_id", "series_id", "responded_to")


def _ent_dict(e, cmd):
    d = {"term": e.term, "index": e.index, "type": e.type, "cmd": cmd}
    d.update({f: getattr(e, f) for f in SESSION})
    return d


def outbox_by_cell(eng, n_groups, n):
    """{(g, k, d): [(message dict, [entry dicts])]} of the last round, InstallSnapshot
    messages dropped; entries with their whole Cmds and session fields
    (rbe_get_outbox)."""
    cells, n_is = {}, 0
    for r in range(n_groups * n):
        g, k = divmod(r, n)
        msgs, ents, cmds = eng.outbox(r)
        ei = 0
        for m in msgs:
            es = []
            for _ in range(m.n_entries):
                es.append(_ent_dict(ents[ei], cmds[ei]))
                ei += 1
            if m.type == INSTALL_SNAPSHOT:
                n_is += 1
                continue
            cells.setdefault((g, k, m.to - 1), []).append((_msg_dict(m), es))
    return cells, n_is


def expected_stream(cells, n_groups, n, gpb, deployment_id, bin_ver, addrs=ADDRS):
    """The frames rbe_wire_encode must produce: pair-major (sender k, receiver d
    ascending, d != k), then group runs of gpb, empty batches left out."""
    out, frames = bytearray(), []
    gpb = gpb or n_groups
    for k in range(n):
        for d in range(n):
            if d == k:
                continue
            for g0 in range(0, n_groups, gpb):
                reqs = []
                for g in range(g0, min(n_groups, g0 + gpb)):
                    reqs += cells.get((g, k, d), [])
                if not reqs:
                    continue
                fb = W.frame(W.batch_bytes(reqs, deployment_id, addrs[k], bin_ver))
                frames.append((len(out), len(fb), g0, k, d, len(reqs)))
                out += fb
    return bytes(out), frames


def check_frames(stream, frames, exp_stream, exp_frames):
    got = [(f.offset, f.bytes, f.first_group, f.src, f.dst, f.n_messages) for f in frames]
    assert got == exp_frames
    assert stream == exp_stream


def check_decoded(msgs, ents, cmd, cells, n_groups, n, gpb):
    """rbe_wire_decode's records, in frame order, equal the outbox records."""
    exp = []
    gpb = gpb or n_groups
    for k in range(n):
        for d in range(n):
            if d == k:
                continue
            for g0 in range(0, n_groups, gpb):
                for g in range(g0, min(n_groups, g0 + gpb)):
                    exp += cells.get((g, k, d), [])
    assert len(msgs) == len(exp)
    ei, ci = 0, 0
    for m, (em, ee) in zip(msgs, exp):
        assert _msg_dict(m) == em
        assert m.n_entries == len(ee)
        for x in ee:
            e = ents[ei]
            ei += 1
            got = _ent_dict(e, cmd[ci:ci + e.cmd_len])
            ci += e.cmd_len
            assert got == x
            assert bytes(e.cmd[:min(16, e.cmd_len)]) == x["cmd"][:16]
    assert ei == len(ents) and ci == len(cmd)
