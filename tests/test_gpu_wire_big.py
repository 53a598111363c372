"""Big MessageBatch frames on the GPU: a frame longer than the engine's walk
threshold (RBE_WIRE_BIG, default 256 KiB) is walked by chunks — every byte
position's exit from its 8 KiB chunk by pointer doubling (k_wire_chunk_exit),
one hop per chunk along the true walk (k_wire_hop), the requests emitted per
chunk (k_wire_chunk_emit) — instead of one field at a time.  The records must
equal the oracle's decode (oracle/wire.py, MessageBatch.Unmarshal) and the
per-frame walk's, and malformed frames must be refused the same way."""
import os
import random

import pytest

import wire as W
from parity_util import C2
from wire_util import ADDRS, check_decoded, expected_stream, outbox_by_cell

pytestmark = pytest.mark.gpu


def _engine(big=None, **kw):
    from dragonboat_amd.engine import Engine
    old = os.environ.get("RBE_WIRE_BIG")
    if big is not None:
        os.environ["RBE_WIRE_BIG"] = str(big)
    try:
        return Engine(device=0, trace=True, **kw)
    finally:
        if big is not None:
            if old is None:
                del os.environ["RBE_WIRE_BIG"]
            else:
                os.environ["RBE_WIRE_BIG"] = old


def _records(dec):
    msgs, ents, cmd = dec
    return ([bytes(m) for m in msgs], [bytes(e) for e in ents], bytes(cmd))


@pytest.mark.parametrize("big,groups", [(4096, 3000), (1 << 18, 3000), (1 << 18, 12000)])
def test_gpu_wire_chunked_walk_equals_oracle(gpu_available, big, groups):
    """One frame per (sender, receiver) slot pair (gpb 0): 3,000 groups give
    frames of ~100-400 KB, every one walked by chunks at threshold 4 KiB;
    12,000 groups give frames over 256 KiB whose batches are scanned by
    segments and whose crc32s are taken by 64 KiB segments on encode."""
    kw = dict(C2, n_groups=groups)
    eng = _engine(big=big, **kw)
    n, G = 3, kw["n_groups"]
    checked = 0
    for rnd in range(60):
        eng.run(1)
        if rnd < 40 or rnd % 5:
            continue
        cells, _ = outbox_by_cell(eng, G, n)
        tot = eng.wire_encode(0xDB0A7, 210, 0, ADDRS[:n])
        stream, frames = eng.wire_fetch(tot)
        exp, _ = expected_stream(cells, G, n, 0, 0xDB0A7, 210)
        assert stream == exp
        assert max(f.bytes for f in frames) > 2 * 8192
        msgs, ents, cmd = eng.wire_decode(stream)
        check_decoded(msgs, ents, cmd, cells, G, n, 0)
        checked += tot[2]
    assert checked > 10000
    eng.close()


def _synthetic_payload(n_req, seed, tiny_every=0, split=False):
    """A MessageBatch payload of n_req requests drawn from a few Message
    templates (Replicate with entries, Heartbeat, ReplicateResp), every
    `tiny_every`-th one an empty Message (2 bytes), then the trailer; with
    `split`, (the first 3/4 of the requests, the rest with the trailer)."""
    rng = random.Random(seed)
    tmpl = []
    for i in range(16):
        m = dict(type=[1, 4, 5, 17][i % 4], to=1 + i % 3, cluster_id=rng.randrange(1 << 40),
                 term=rng.randrange(1, 1 << 20), log_term=rng.randrange(1 << 20),
                 log_index=rng.randrange(1 << 30), commit=rng.randrange(1 << 30),
                 reject=i % 5 == 0, hint=rng.randrange(1 << 10), hint_high=0)
        m["from"] = 1 + (i + 1) % 3
        ents = [dict(term=m["term"], index=m["log_index"] + j + 1, type=0, key=0, client_id=0,
                     series_id=0, responded_to=0, cmd=bytes(rng.randrange(256) for _ in range(16)))
                for j in range(i % 3)]
        b = W.message_bytes(m, ents, None)
        req = bytearray(b"\x0a")
        W.put_varint(req, len(b))
        tmpl.append(bytes(req + b))
    out = bytearray()
    head = b""
    for j in range(n_req):
        if j == n_req * 3 // 4:
            head = bytes(out)
            out = bytearray()
        out += b"\x0a\x00" if tiny_every and j % tiny_every == 0 else tmpl[rng.randrange(16)]
    W._field_varint(out, 0x10, 77)
    out += b"\x1a\x05node1"
    W._field_varint(out, 0x20, 210)
    return (head, bytes(out)) if split else head + bytes(out)


def test_gpu_wire_7mb_frame(gpu_available):
    """A 7 MB frame (~90k requests) through the chunked walk equals the
    per-frame walk's decode, request for request."""
    payload = _synthetic_payload(90_000, 5)
    assert len(payload) > 7_000_000
    stream = W.frame(payload)
    a, b = _engine(big=1 << 18, **C2), _engine(big=1 << 40, **C2)
    a.run(2)
    b.run(2)
    ra, rb = _records(a.wire_decode(stream)), _records(b.wire_decode(stream))
    assert len(ra[0]) == 90_000
    assert ra == rb
    a.close()
    b.close()


def test_gpu_wire_chunked_dense_and_malformed(gpu_available):
    """Requests of 2 bytes overflow the single-pass slots (the second walk
    re-emits them by chunks); a frame whose structure breaks inside a later
    chunk is refused with RBE_E_CORRUPT, as by the per-frame walk."""
    from dragonboat_amd.engine import RBE_E_CORRUPT, EngineError
    eng = _engine(big=1024, **C2)
    ref = _engine(big=1 << 40, **C2)
    eng.run(2)
    ref.run(2)
    dense = _synthetic_payload(20000, 9, tiny_every=1)  # 40 KB: 2,501 slots
    stream = W.frame(_synthetic_payload(3000, 9, tiny_every=3)) + W.frame(dense) + \
        W.frame(_synthetic_payload(50, 3))
    got = _records(eng.wire_decode(stream))
    assert got == _records(ref.wire_decode(stream))
    assert len(got[0]) == 23050
    head, tail = _synthetic_payload(4000, 11, split=True)
    assert len(head) > 4 * 8192
    for bad in (head + b"\x0b" + tail,                    # wire type 3 at a field boundary
                head + b"\x0a\xff\xff\xff\x7f" + tail,    # a length past the frame's end
                head + tail + b"\x0a",                    # a header cut by the end
                head + tail + b"\x10\x80\x80"):           # an unterminated varint
        for e in (eng, ref):
            with pytest.raises(EngineError) as ei:
                e.wire_decode(W.frame(bad))
            assert ei.value.rc == RBE_E_CORRUPT
    eng.close()
    ref.close()
