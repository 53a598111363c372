"""One big MessageBatch frame through rbe_wire_decode (diagnostic for
profiles/, not the bench line): a ~7-8 MB frame of ~90k requests (the
synthetic payload of tests/test_gpu_wire_big.py), decoded with the chunked
walk (default threshold) and with the per-frame walk (threshold above the
frame), wall time of the rbe_wire_decode call (H2D of the stream, the
device decode, D2H of the records into preallocated host buffers) per call
over --reps calls after one warm-up."""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]

import wire as W  # noqa: E402
from test_gpu_wire_big import _synthetic_payload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--requests", type=int, default=90_000)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from dragonboat_amd.engine import Engine, RbeEntry, RbeMessage
    stream = W.frame(_synthetic_payload(a.requests, 5))
    out = {"frame_bytes": len(stream), "requests": a.requests}
    cap, ecap, ccap = a.requests + 16, 4 * a.requests, 64 * a.requests
    msgs, ents = (RbeMessage * cap)(), (RbeEntry * ecap)()
    cmd = C.create_string_buffer(ccap)
    nm, ne, nc = C.c_uint32(), C.c_uint32(), C.c_uint64()
    for name, big in (("chunked", None), ("per_frame", 1 << 40)):
        if big is not None:
            os.environ["RBE_WIRE_BIG"] = str(big)
        eng = Engine(device=0, trace=False, n_groups=64, n_replicas=3)
        os.environ.pop("RBE_WIRE_BIG", None)
        eng.run(2)

        def call():
            rc = eng.lib.rbe_wire_decode(eng.h, stream, len(stream), msgs, cap, C.byref(nm), ents,
                                         ecap, C.byref(ne), cmd, ccap, C.byref(nc))
            assert rc == 0 and nm.value == a.requests, (rc, nm.value)
        call()
        reps = a.reps if big is None else 1
        t0 = time.perf_counter()
        for _ in range(reps):
            call()
        out[name + "_ms"] = (time.perf_counter() - t0) * 1e3 / reps
        eng.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
