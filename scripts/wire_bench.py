"""Throughput of the device wire codec (rbe_wire_encode / rbe_wire_decode) on a
C2-shaped outbox: 1M groups x 3 replicas with one proposal per group per round
(each round's outbox: Replicate + responses), batches of 4096 groups per
(sender, receiver) slot pair.  Prints one JSON line.

Algorithmic bytes: encode reads each message record (64 B) and its entries
(32 B each) and writes the frame bytes; decode reads the frame bytes and writes
each message record (96 B rbe_message), entry (40 B rbe_entry) and Cmd byte."""
import argparse
import ctypes as C
import json
import sys
import time

sys.path.insert(0, ".")

from dragonboat_amd.engine import Engine, RbeEntry, RbeMessage  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=1_000_000)
    ap.add_argument("--gpb", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    eng = Engine(device=0, n_groups=a.groups, n_replicas=3, wl_enabled=True, wl_start_round=30,
                 ring=64, trace=False)
    eng.run(60)
    addrs = ("node-1:26001", "node-2:26001", "node-3:26001")
    tot = eng.wire_encode(1, 210, a.gpb, addrs)
    t0 = time.perf_counter()
    for _ in range(a.reps):
        tot = eng.wire_encode(1, 210, a.gpb, addrs)
    enc_s = (time.perf_counter() - t0) / a.reps
    stream, frames = eng.wire_fetch(tot)
    nmsg = tot[2]
    # the C call alone into preallocated buffers (no Python objects per record)
    cap = nmsg + 16
    msgs = (RbeMessage * cap)()
    ents = (RbeEntry * cap)()
    cmd = C.create_string_buffer(len(stream))
    src = C.create_string_buffer(stream, len(stream))
    nm, ne_, nc = C.c_uint32(), C.c_uint32(), C.c_uint64()

    def decode():
        rc = eng.lib.rbe_wire_decode(eng.h, src, len(stream), msgs, cap, C.byref(nm), ents, cap,
                                     C.byref(ne_), cmd, len(stream), C.byref(nc))
        assert rc == 0, rc

    decode()
    t0 = time.perf_counter()
    reps_d = max(1, a.reps)
    for _ in range(reps_d):
        decode()
    dec_s = (time.perf_counter() - t0) / reps_d
    assert nm.value == nmsg
    ne = ne_.value
    enc_alg = nmsg * 64 + ne * 32 + tot[0]
    dec_alg = tot[0] + nmsg * 96 + ne * 40 + nc.value
    print(json.dumps({
        "workload": f"C2 outbox {a.groups} groups x 3, {a.gpb} groups per batch",
        "frames": tot[1], "messages": nmsg, "entries": ne, "stream_bytes": tot[0],
        "encode_ms": enc_s * 1e3, "encode_msgs_per_s": nmsg / enc_s,
        "encode_alg_GBps": enc_alg / enc_s / 1e9,
        "decode_ms": dec_s * 1e3, "decode_msgs_per_s": nmsg / dec_s,
        "decode_alg_GBps": dec_alg / dec_s / 1e9,
        "note": "host wall clock around each call: includes the H2D copy of the input "
                "(decode), the D2H copy of the records and two stream syncs"}))


if __name__ == "__main__":
    main()
