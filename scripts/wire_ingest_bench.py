"""Transport hop as bytes at scale (diagnostic for profiles/, not the bench
line): two engines on one GPU (rep_world = 2, replica k of group g on engine
(g + k) % 2) step a C2-shaped workload (steady replication, one 16 B proposal
per group per round); after every round each engine encodes its frames for
the other (rbe_wire_encode + rbe_wire_fetch to host memory, as a transport
would write them on a socket) and the other ingests them (rbe_wire_ingest:
H2D, decode, checks, sort, scatter into the inbox planes).  Prints one JSON
line with per-round times and volumes; run under rocprofv3 --stats for the
kernel split.  The stream goes through pinned host buffers (a transport's
socket buffers would be registered the same way), and frames hold
--gpb groups each (the reference's transport batches up to 64 MB per
connection, transport.go:511-538; one block walks each frame's top level)."""
import argparse
import ctypes as C
import json
import sys
import os
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dragonboat_amd.engine import (Engine, RbeWireIngestStats, _check,  # noqa: E402
                                   wire_config)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=100_000)
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--gpb", type=int, default=512, help="groups per frame")
    a = ap.parse_args()
    kw = dict(n_groups=a.groups, n_replicas=3, wl_enabled=True, wl_start_round=20,
              maxm=8, ecap=16)
    engs = [Engine(device=0, trace=False, rep_world=2, rep_rank=r, **kw) for r in range(2)]
    hip = C.CDLL("libamdhip64.so")
    cap = 1 << 28
    bufs = []
    for _ in range(2):  # pinned host buffers (hipHostMalloc)
        ptr = C.c_void_p()
        assert hip.hipHostMalloc(C.byref(ptr), C.c_size_t(cap), 0) == 0
        bufs.append(ptr)
    t = {"step": 0.0, "encode": 0.0, "fetch": 0.0, "ingest": 0.0}
    vol = {"bytes": 0, "frames": 0, "messages": 0, "entries": 0}

    def hop(timed):
        for e in engs:
            t0 = time.perf_counter()
            e.step()
            e.sync()
            if timed:
                t["step"] += time.perf_counter() - t0
        sizes = []
        for r, e in enumerate(engs):
            t0 = time.perf_counter()
            tot = (C.c_uint64 * 4)()
            wc = wire_config(groups_per_batch=a.gpb, dst_rank=1 - r)
            _check(e.lib.rbe_wire_encode(e.h, C.byref(wc), tot), "rbe_wire_encode")
            e.sync()
            t1 = time.perf_counter()
            assert tot[0] <= cap
            _check(e.lib.rbe_wire_fetch(e.h, bufs[r], cap, None, 0),
                   "rbe_wire_fetch")
            t2 = time.perf_counter()
            sizes.append(tot[0])
            if timed:
                t["encode"] += t1 - t0
                t["fetch"] += t2 - t1
        for r, e in enumerate(engs):
            t0 = time.perf_counter()
            st = RbeWireIngestStats()
            _check(e.lib.rbe_wire_ingest(e.h, bufs[1 - r], sizes[1 - r],
                                         C.byref(st)), "rbe_wire_ingest")
            if timed:
                t["ingest"] += time.perf_counter() - t0
                vol["bytes"] += sizes[1 - r]
                vol["frames"] += st.frames
                vol["messages"] += st.messages
                vol["entries"] += st.entries

    for _ in range(a.warmup):
        hop(False)
    for _ in range(a.rounds):
        hop(True)
    R = a.rounds
    faults = [e.fault_summary()[0] for e in engs]
    c = [e.counters() for e in engs]
    print(json.dumps({
        "groups": a.groups, "replicas": 3, "engines": 2, "rounds": R, "groups_per_frame": a.gpb,
        "ms_per_round": {k: v * 1e3 / R for k, v in t.items()},
        "per_round": {k: v / R for k, v in vol.items()},
        "ingest_gbs": vol["bytes"] / max(1e-12, t["ingest"]) / 1e9,
        "committed": sum(x["committed"] for x in c), "faulty_replicas": sum(faults)}),
        flush=True)
    for e in engs:
        e.close()


if __name__ == "__main__":
    main()
