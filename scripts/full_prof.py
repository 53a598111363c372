"""Diagnostic: what the slowest waves of k_full_list hold, from the
RBE_FULL_PROF build (build/full_prof.so):

    scripts/build_variant.sh build/full_prof.so -DRBE_FULL_PROF
    RBE_LIB=$PWD/build/full_prof.so python scripts/full_prof.py c3

Each record is one wave iteration of the general step: its wall-clock span
(s_memrealtime, 100 MHz), its active lanes, the classes of its lanes, a class
being (role before, role after, any inbound message), and the most inbound
and outbound messages of one of its lanes."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from dragonboat_amd import engine as E  # noqa: E402

lib = E.load_library(os.environ["RBE_LIB"])
lib.rbe_debug_full_prof.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]
w = sys.argv[1] if len(sys.argv) > 1 else "c3"
kw, settle, _ = bench.WORKLOADS[w]
eng = E.Engine(**dict(kw))
eng.run(settle)
eng.sync()
cap = 1 << 20
buf = np.zeros((cap, 4), np.uint64)
n = C.c_uint64()
lib.rbe_debug_full_prof(eng.h, buf.ctypes.data, cap, C.byref(n))  # allocates, clears
rounds = 20
ms = eng.profile_rounds(rounds)
lib.rbe_debug_full_prof(eng.h, buf.ctypes.data, cap, C.byref(n))
m = min(n.value, cap)
rec = buf[:m]
dt = rec[:, 0].astype(np.float64) * 10e-3  # us
ROLES = "FCLOW"
names = {}
for q in range(128):
    rb, ra, inb = q >> 4, (q >> 1) & 7, q & 1
    if rb < 5 and ra < 5:
        names[q] = f"{ROLES[rb]}->{ROLES[ra]}{'+in' if inb else ''}"
print(f"{w}: {rounds} rounds, kernel split (ms/round) {[round(x / rounds, 4) for x in ms]}")
lanes = (rec[:, 3] & np.uint64(0xFF)).astype(np.int64)
mx_in = ((rec[:, 3] >> np.uint64(8)) & np.uint64(0xFFFF)).astype(np.int64)
mx_out = ((rec[:, 3] >> np.uint64(24)) & np.uint64(0xFFFF)).astype(np.int64)
print(f"wave iterations {m} ({m / rounds:.0f}/round), lanes/iter {lanes.mean():.1f}, "
      f"span us: mean {dt.mean():.2f} p50 {np.median(dt):.2f} p99 {np.percentile(dt, 99):.2f} "
      f"max {dt.max():.2f}")
stats = []
for q, nm in names.items():
    has = ((rec[:, 1] >> np.uint64(q)) & np.uint64(1)) if q < 64 else \
        ((rec[:, 2] >> np.uint64(q - 64)) & np.uint64(1))
    has = has.astype(bool)
    if has.any():
        stats.append((dt[has].sum(), nm, int(has.sum()), dt[has].mean(), dt[has].max()))
stats.sort(reverse=True)
print(f"{'class':14s} {'waves':>8s} {'sum us':>10s} {'mean':>8s} {'max':>8s}")
for s, nm, c, mu, mx in stats[:20]:
    print(f"{nm:14s} {c:8d} {s:10.1f} {mu:8.2f} {mx:8.2f}")
# waves holding a single class: the per-class cost without mixing
single = []
for q, nm in names.items():
    lo = np.uint64(1 << q) if q < 64 else np.uint64(0)
    hi = np.uint64(1 << (q - 64)) if q >= 64 else np.uint64(0)
    only = (rec[:, 1] == lo) & (rec[:, 2] == hi)
    if only.any():
        single.append((dt[only].mean(), nm, int(only.sum())))
single.sort(reverse=True)
print("single-class waves:", [(nm, round(mu, 2), c) for mu, nm, c in single[:12]])
# span against the busiest lane's message counts
for lo, hi in ((0, 2), (2, 5), (5, 10), (10, 20), (20, 1 << 16)):
    sel = (mx_in >= lo) & (mx_in < hi)
    if sel.any():
        print(f"max inbound {lo:3d}-{hi:5d}: waves {int(sel.sum()):6d} span mean {dt[sel].mean():8.2f} "
              f"max out mean {mx_out[sel].mean():6.1f} lanes {lanes[sel].mean():5.1f}")
order = np.argsort(-dt)[:10]
print("slowest:", [(round(float(dt[i]), 1), int(lanes[i]), int(mx_in[i]), int(mx_out[i])) for i in order])
