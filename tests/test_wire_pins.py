"""Pins of the wire-format restatement (oracle/wire.py) from the reference's
own tests, since the reference holds no byte vectors (no Go here):

  * Message / MessageBatch / Entry SizeUpperLimit bounds the marshaled size
    (raftpb/raft_test.go:244-386, getMaxSizedMsg: every u64 field max-valued —
    colfer's 9-byte form above 2^49 — 1 KiB Cmds, 1024 entries, a snapshot
    with a file path).  The reference's batch test holds 1024 such messages
    (1 GiB); the bound is additive per message, so 4 are used here.
  * requestHeader encode / decode / crc (internal/transport/tcp_test.go:23-88):
    round trip, a changed crc slot or size field is detected, an unknown
    method is refused.
"""
import wire as W

MAX64 = (1 << 64) - 1
MAX32 = (1 << 32) - 1


def _max_entry(cmd_len=1024):
    return dict(term=MAX64, index=MAX64, type=1, key=MAX64, client_id=MAX64, series_id=MAX64,
                responded_to=MAX64, cmd=bytes(cmd_len))


def _max_msg(n_ent=1024, cmd_len=1024):
    m = dict(type=4, to=MAX64, cluster_id=MAX64, term=MAX64, log_term=MAX64, log_index=MAX64,
             commit=MAX64, reject=True, hint=MAX64, hint_high=MAX64)
    m["from"] = MAX64
    snap = W.snapshot_bytes(MAX64, MAX64, "longfilepathisherexxxxxxxxxxxxxxxxx", MAX64)
    ents = [_max_entry(cmd_len) for _ in range(n_ent)]
    return m, ents, snap


def test_entry_size_upper_limit():  # raft_test.go:244-271
    for e in (_max_entry(1024), _max_entry(0), dict(), dict(cmd=bytes(1024))):
        assert len(W.entry_bytes(e)) <= W.entry_size_upper_limit(len(e.get("cmd", b"")))


def test_message_size_upper_limit():  # raft_test.go:348-357
    m, ents, snap = _max_msg()
    size = len(W.message_bytes(m, ents, snap))
    assert size <= W.message_size_upper_limit([1024] * 1024, snap)
    empty = dict(type=0, to=0, cluster_id=0, term=0, log_term=0, log_index=0, commit=0,
                 reject=False, hint=0, hint_high=0)
    empty["from"] = 0
    assert len(W.message_bytes(empty, [])) <= W.message_size_upper_limit([])


def test_message_batch_size_upper_limit():  # raft_test.go:359-386
    m, ents, snap = _max_msg(n_ent=64)
    addr = "longaddressisherexxxxxxxxxxxxxxxxxxxxxxxxx"
    mb = bytearray()
    for _ in range(4):
        b = W.message_bytes(m, ents, snap)
        mb.append(0x0A)
        W.put_varint(mb, len(b))
        mb += b
    W._field_varint(mb, 0x10, MAX64)
    a = addr.encode()
    mb.append(0x1A)
    W.put_varint(mb, len(a))
    mb += a
    W._field_varint(mb, 0x20, MAX32)
    bound = W.batch_size_upper_limit(addr, [W.message_size_upper_limit([1024] * 64, snap)] * 4)
    assert len(mb) <= bound
    assert len(W.batch_bytes([], 0, "", 0)) <= W.batch_size_upper_limit("", [])
    assert len(W.batch_bytes([], MAX64, addr + "x", MAX32)) <= W.batch_size_upper_limit(addr + "x", [])


def test_max_sized_message_round_trips():
    """The maximal values (9-byte colfer u64s, 10-byte varints) survive the
    restatement's encode → decode."""
    m, ents, snap = _max_msg(n_ent=3)
    got = W.message_decode(W.message_bytes(m, ents, snap))
    gm, gents = got[0], got[1]
    for f in ("to", "from", "cluster_id", "term", "log_term", "log_index", "commit", "hint",
              "hint_high"):
        assert gm[f] == MAX64, f
    assert len(gents) == 3 and all(e["key"] == MAX64 and e["responded_to"] == MAX64 and
                                   len(e["cmd"]) == 1024 for e in gents)


def test_request_header_round_trip():  # tcp_test.go:23-40
    h = W.request_header_encode(W.RAFT_TYPE, 1024, 1000)
    assert len(h) == W.HEADER_SIZE
    assert W.request_header_decode(h) == (W.RAFT_TYPE, 1024, 1000)


def test_request_header_crc_is_checked():  # tcp_test.go:42-72
    h = bytearray(W.request_header_encode(W.RAFT_TYPE, 1024, 1000))
    crc = int.from_bytes(h[10:14], "big")
    h[10:14] = ((crc + 1) & MAX32).to_bytes(4, "big")
    assert W.request_header_decode(bytes(h)) is None
    h[10:14] = crc.to_bytes(4, "big")
    assert W.request_header_decode(bytes(h)) is not None
    h[2:10] = (0).to_bytes(8, "big")
    assert W.request_header_decode(bytes(h)) is None


def test_invalid_method_is_reported():  # tcp_test.go:74-88
    assert W.request_header_decode(W.request_header_encode(1024, 1024, 1000)) is None
    assert W.request_header_decode(W.request_header_encode(W.SNAPSHOT_TYPE, 1, 2)) is not None
