"""Transport wire format, CPU tier.

1. The oracle's restatement (oracle/wire.py) against the published algorithms'
   check values and an independent implementation (zlib's crc32), and by
   encode -> decode round trips (the reference holds no byte-level vectors for
   these types: parity of the byte layout is unpinned against reference bytes).
2. The device codec's per-cell functions (rbe_wire.h, compiled into the
   test-only host build) against the oracle: every round of a lockstep run,
   the frames equal byte for byte what the oracle builds from the engine's
   outbox records."""
import random
import zlib

import pytest

import wire as W
from parity_util import C2, C3, C4
from soa_cpu.soa import SoaCpu
from wire_util import ADDRS, check_frames, expected_stream, outbox_by_cell


def test_crc32_check_value_and_zlib():
    assert W.crc32(b"123456789") == 0xCBF43926  # the CRC-32/IEEE check value
    rng = random.Random(7)
    for n in (0, 1, 7, 64, 1000):
        b = bytes(rng.randrange(256) for _ in range(n))
        assert W.crc32(b) == zlib.crc32(b)


def test_crc32_combine():
    rng = random.Random(3)
    for _ in range(20):
        a = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 300)))
        b = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 300)))
        assert W.crc32_combine(W.crc32(a), W.crc32(b), len(b)) == W.crc32(a + b)


def test_varint_examples():
    for x, enc in ((0, b"\x00"), (1, b"\x01"), (150, b"\x96\x01"), (300, b"\xac\x02"),
                   (2**64 - 1, b"\xff" * 9 + b"\x01")):
        o = bytearray()
        W.put_varint(o, x)
        assert bytes(o) == enc and W.sov(x) == len(enc)
        assert W.get_varint(enc, 0) == (x, len(enc))


def test_colfer_entry_round_trip():
    rng = random.Random(11)
    for _ in range(200):
        e = {"term": rng.choice([0, 1, 2**20, 2**49 - 1, 2**49, 2**64 - 1]),
             "index": rng.choice([0, 5, 2**35, 2**63]), "type": rng.choice([0, 1, 2, 300]),
             "key": 0, "client_id": rng.choice([0, 77]), "series_id": 0, "responded_to": 0,
             "cmd": bytes(rng.randrange(256) for _ in range(rng.choice([0, 3, 16, 200])))}
        assert W.entry_decode(W.entry_bytes(e)) == e
    # absent fields encode to the bare terminator (raft_optimized.go:292-293)
    assert W.entry_bytes({}) == b"\x7f"


def test_message_batch_frame_round_trip():
    rng = random.Random(5)
    reqs = []
    for i in range(30):
        m = {"type": rng.randrange(27), "to": rng.randrange(1, 6), "from": rng.randrange(1, 6),
             "cluster_id": rng.randrange(2**40), "term": rng.randrange(100),
             "log_term": rng.randrange(100), "log_index": rng.randrange(2**33),
             "commit": rng.randrange(2**33), "reject": rng.randrange(2),
             "hint": rng.randrange(2**64), "hint_high": rng.randrange(2**64)}
        ents = [{"term": 3, "index": 10 + j, "type": 0, "key": 0, "client_id": 0,
                 "series_id": 0, "responded_to": 0, "cmd": bytes([j] * (j * 7))}
                for j in range(rng.randrange(4))]
        reqs.append((m, ents))
    payload = W.batch_bytes(reqs, 0x1234, "a:1", 210)
    st = W.frame(payload) + W.frame(W.batch_bytes(reqs[:1], 9, "b", 1))
    p1, p2 = W.frames_decode(st)
    b = W.batch_decode(p1)
    assert (b["deployment_id"], b["source_address"], b["bin_ver"]) == (0x1234, "a:1", 210)
    for (m, ents), (dm, de) in zip(reqs, b["requests"]):
        assert {k: dm[k] for k in m} == m and dm["snapshot"] == (0, 0)
        assert de == ents
    # a flipped payload bit and a flipped header bit are both caught
    bad = bytearray(st)
    bad[40] ^= 1
    with pytest.raises(ValueError):
        W.frames_decode(bytes(bad))
    bad = bytearray(st)
    bad[5] ^= 1
    with pytest.raises(ValueError):
        W.frames_decode(bytes(bad))


@pytest.mark.parametrize("name,kw,gpb", [("C2", C2, 16), ("C3", dict(C3), 0),
                                         ("C4", C4, 7),
                                         ("C3_N7", dict(C3, n_groups=20, n_replicas=7), 5)])
def test_host_build_frames_match_oracle(name, kw, gpb):
    eng = SoaCpu(trace=True, **kw)
    n, G = kw["n_replicas"], kw["n_groups"]
    for rnd in range(120):
        eng.run(1)
        if rnd % 7 and rnd < 110:
            continue
        cells, _ = outbox_by_cell(eng, G, n)
        stream, frames = eng.wire_encode(0xDB0A7, 210, gpb, ADDRS[:n])
        exp, exp_frames = expected_stream(cells, G, n, gpb, 0xDB0A7, 210)
        check_frames(stream, frames, exp, exp_frames)
        # and the oracle's decoder reads every request back
        got = sum(len(W.batch_decode(p)["requests"]) for p in W.frames_decode(stream))
        assert got == sum(len(v) for v in cells.values())


def test_host_build_frames_with_snapshots_and_heap_cmds():
    """InstallSnapshot messages are left out (snapshot stream) and Cmds longer
    than 16 bytes are encoded whole from the payload heap."""
    from heap_util import mixed_cmd
    kw = dict(C3, check_quorum=False, snapshot_entries=20, compaction_overhead=5,
              n_groups=8, ext_inputs=True, wl_enabled=False)
    eng = SoaCpu(trace=True, heap_bytes=8 << 20, **kw)
    n, G = kw["n_replicas"], kw["n_groups"]
    rng = random.Random(21)
    saw_is = saw_long = 0
    for rnd in range(260):
        if rnd > 30 and rnd % 2 == 0:
            reps = [g * n + rng.randrange(n) for g in range(G)]
            eng.push_proposals(reps, [[mixed_cmd(rng)] for _ in reps])
        eng.run(1)
        cells, n_is = outbox_by_cell(eng, G, n)
        saw_is += n_is
        saw_long += sum(1 for v in cells.values() for _, es in v for e in es
                        if len(e["cmd"]) > 16)
        stream, frames = eng.wire_encode(7, 210, 3, ADDRS[:n])
        exp, exp_frames = expected_stream(cells, G, n, 3, 7, 210)
        check_frames(stream, frames, exp, exp_frames)
    assert saw_is > 0 and saw_long > 0
