"""Transport wire format on the GPU: rbe_wire_encode's frames equal, byte for
byte, the oracle's restatement (oracle/wire.py) of MessageBatch marshaling and
TCP framing applied to the engine's outbox records, and rbe_wire_decode reads
them back into exactly those records (crc32s checked on the device)."""
import random

import pytest

import wire as W
from parity_util import C2, C3, C4
from wire_util import ADDRS, check_decoded, check_frames, expected_stream, outbox_by_cell

pytestmark = pytest.mark.gpu


def _engine(**kw):
    from dragonboat_amd.engine import Engine
    return Engine(device=0, trace=True, **kw)


@pytest.mark.parametrize("name,kw,extra,gpb", [
    ("C2", C2, {}, 16), ("C3", C3, dict(), 0), ("C4", C4, {}, 7),
    ("C3_SNAP", dict(C3, check_quorum=False, snapshot_entries=20, compaction_overhead=5),
     dict(), 5),
    ("C3_N7", dict(C3, n_groups=20, n_replicas=7), dict(), 5)])
def test_gpu_wire_encode_decode(gpu_available, name, kw, extra, gpb):
    eng = _engine(**kw, **extra)
    n, G = kw["n_replicas"], kw["n_groups"]
    checked = 0
    for rnd in range(160):
        eng.run(1)
        if rnd % 9 and rnd < 150:
            continue
        cells, n_is = outbox_by_cell(eng, G, n)
        tot = eng.wire_encode(0xDB0A7, 210, gpb, ADDRS[:n])
        stream, frames = eng.wire_fetch(tot)
        exp, exp_frames = expected_stream(cells, G, n, gpb, 0xDB0A7, 210)
        check_frames(stream, frames, exp, exp_frames)
        assert tot[2] == sum(len(v) for v in cells.values()) and tot[3] == n_is
        msgs, ents, cmd = eng.wire_decode(stream)
        check_decoded(msgs, ents, cmd, cells, G, n, gpb)
        checked += tot[2]
    assert checked > 100
    eng.close()


def test_gpu_wire_heap_cmds(gpu_available):
    from heap_util import mixed_cmd
    kw = dict(C2, n_groups=8, ext_inputs=True, wl_enabled=False)
    eng = _engine(**kw, heap_bytes=8 << 20)
    n, G = 3, 8
    rng = random.Random(4)
    long_seen = 0
    for rnd in range(120):
        if rnd > 30:
            reps = [g * n + rng.randrange(n) for g in range(G)]
            eng.push_proposals(reps, [[mixed_cmd(rng)] for _ in reps])
        eng.run(1)
        cells, _ = outbox_by_cell(eng, G, n)
        tot = eng.wire_encode(1, 2, 3, ADDRS[:n])
        stream, frames = eng.wire_fetch(tot)
        exp, exp_frames = expected_stream(cells, G, n, 3, 1, 2)
        check_frames(stream, frames, exp, exp_frames)
        msgs, ents, cmd = eng.wire_decode(stream)
        check_decoded(msgs, ents, cmd, cells, G, n, 3)
        long_seen += sum(1 for e in ents if e.cmd_len > 16)
    assert long_seen > 20
    eng.close()


def test_gpu_wire_decode_rejects_corruption(gpu_available):
    from dragonboat_amd.engine import RBE_E_CORRUPT, EngineError
    eng = _engine(**C2)
    eng.run(40)
    tot = eng.wire_encode(5, 1, 0, ADDRS[:3])
    stream, frames = eng.wire_fetch(tot)
    assert len(frames) == 6
    for pos in (frames[2].offset + 5, frames[3].offset + 30, len(stream) - 1):
        bad = bytearray(stream)
        bad[pos] ^= 0x10
        with pytest.raises(EngineError) as ei:
            eng.wire_decode(bytes(bad))
        assert ei.value.rc == RBE_E_CORRUPT
    # the oracle reads the same frames
    assert len(W.frames_decode(stream)) == 6
    eng.close()


def test_gpu_wire_decode_dense_requests(gpu_available):
    """Requests shorter than 16 bytes (here empty Messages, valid protobuf)
    overflow the single-pass position slots: the decoder walks the frame again
    and still returns every request, in order (MessageBatch.Unmarshal)."""
    eng = _engine(**C2)
    eng.run(2)
    payload = b"\x0a\x00" * 100 + b"\x0a\x04\x08\x11\x10\x02" + b"\x10\x05\x1a\x01a\x20\x01"
    stream = W.frame(payload)
    msgs, ents, cmd = eng.wire_decode(stream)
    ref = W.batch_decode(W.frames_decode(stream)[0])["requests"]
    assert len(msgs) == len(ref) == 101 and not ents and not cmd
    assert [(m.type, m.to) for m in msgs] == [(r[0]["type"], r[0]["to"]) for r in ref]
    assert (msgs[-1].type, msgs[-1].to) == (0x11, 2)
    eng.close()


def test_gpu_wire_decode_max_sized_messages(gpu_available):
    """getMaxSizedMsg-shaped requests (raftpb/raft_test.go:319-346): every u64
    field max-valued (10-byte varints, colfer's 9-byte form), Entry session
    fields at 2^64-1 and just above 2^49, 1 KiB Cmds, an embedded Snapshot with
    a file path — decoded on the device exactly as oracle/wire.py reads them;
    a frame with an unknown method (tcp.go:93-112) is refused."""
    from dragonboat_amd.engine import RBE_E_CORRUPT, EngineError
    M = (1 << 64) - 1
    big = (1 << 49) + 12345
    msgs = []
    for i in range(6):
        m = dict(type=[12, 4, 13][i % 3], to=M - i, cluster_id=M, term=M, log_term=big,
                 log_index=M, commit=big + i, reject=i % 2 == 1, hint=M, hint_high=big)
        m["from"] = M - 7
        ents = [dict(term=M, index=big + j, type=j % 4, key=M, client_id=big, series_id=M - j,
                     responded_to=big + j, cmd=bytes((i + j + k) & 0xFF for k in range(1024)))
                for j in range(3 if i % 3 == 0 else 0)]
        snap = W.snapshot_bytes(M, M, "longfilepathisherexxxxxxxxxxxxxxxxx", M) if i == 1 else None
        msgs.append((m, ents, snap))
    payload = bytearray()
    for m, ents, snap in msgs:
        b = W.message_bytes(m, ents, snap)
        payload.append(0x0A)
        W.put_varint(payload, len(b))
        payload += b
    W._field_varint(payload, 0x10, M)
    payload += b"\x1a\x05node1"
    W._field_varint(payload, 0x20, (1 << 32) - 1)
    stream = W.frame(bytes(payload))
    eng = _engine(**C2)
    eng.run(2)
    dm, de, dcmd = eng.wire_decode(stream)
    ref = W.batch_decode(W.frames_decode(stream)[0])["requests"]
    assert len(dm) == len(ref) == 6
    ei, off = 0, 0
    for got, (rm, rents) in zip(dm, [(r[0], r[1]) for r in ref]):
        for f in ("type", "to", "cluster_id", "term", "log_term", "log_index", "commit", "hint",
                  "hint_high"):
            assert getattr(got, f) == rm[f], f
        assert got.from_ == rm["from"] and bool(got.reject) == bool(rm["reject"])
        assert got.n_entries == len(rents)
        for re_ in rents:
            e = de[ei]
            ei += 1
            for f in ("term", "index", "type", "key", "client_id", "series_id", "responded_to"):
                assert getattr(e, f) == re_[f], f
            assert e.cmd_len == len(re_["cmd"]) and dcmd[off:off + e.cmd_len] == re_["cmd"]
            off += e.cmd_len
    bad = W.MAGIC + W.request_header_encode(1024, len(payload), W.crc32(bytes(payload))) + bytes(payload)
    with pytest.raises(EngineError) as exc:
        eng.wire_decode(bad)
    assert exc.value.rc == RBE_E_CORRUPT
    eng.close()
