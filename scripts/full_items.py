"""Diagnostic: where the general steps longer than 20 us spend their time, from
the RBE_FULL_ITEM_PROF build (build/full_items.so):

    scripts/build_variant.sh build/full_items.so -DRBE_FULL_ITEM_PROF
    RBE_LIB=$PWD/build/full_items.so python scripts/full_items.py c3

Per record (rbe_step.h step_replica): total wall time, before the event loop,
inbox messages, local events and ticks, the deferred fan-out after each
event, the rest (after the loop: the step's stores), the longest inbox message
and its type, inbox messages handled, messages sent, role before / after."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from dragonboat_amd import engine as E  # noqa: E402

lib = E.load_library(os.environ["RBE_LIB"])
lib.rbe_debug_full_items.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]
w = sys.argv[1] if len(sys.argv) > 1 else "c3"
kw, settle, _ = bench.WORKLOADS[w]
eng = E.Engine(**dict(kw))
eng.run(settle)
eng.sync()
cap = 1 << 19
buf = np.zeros((cap, 8), np.uint64)
n = C.c_uint64()
lib.rbe_debug_full_items(eng.h, buf.ctypes.data, cap, C.byref(n))  # allocates
lib.rbe_debug_full_items(eng.h, buf.ctypes.data, cap, C.byref(n))  # clears
rounds = 20
ms = eng.profile_rounds(rounds)
lib.rbe_debug_full_items(eng.h, buf.ctypes.data, cap, C.byref(n))
m = min(n.value, cap)
r = buf[:m]
us = lambda x: x.astype(np.float64) * 10e-3  # noqa: E731  (100 MHz ticks)
tot, pre, inb, loc, fan = (us(r[:, i]) for i in range(5))
mx = us(r[:, 5] & np.uint64((1 << 48) - 1))
mxt = (r[:, 5] >> np.uint64(48)).astype(np.int64)
nin = (r[:, 6] & np.uint64(0xFFFF)).astype(np.int64)
nout = ((r[:, 6] >> np.uint64(16)) & np.uint64(0xFFFF)).astype(np.int64)
rb = ((r[:, 6] >> np.uint64(32)) & np.uint64(0xFF)).astype(np.int64)
ra = ((r[:, 6] >> np.uint64(40)) & np.uint64(0xFF)).astype(np.int64)
rest = tot - pre - inb - loc - fan
print(f"{w}: {rounds} rounds, kernel split ms/round {[round(x / rounds, 4) for x in ms]}")
print(f"steps > 20 us: {m} ({m / rounds:.0f}/round)")
if m:
    print(f"total us: mean {tot.mean():.1f} p50 {np.median(tot):.1f} p99 {np.percentile(tot, 99):.1f} "
          f"max {tot.max():.1f}")
    print(f"share of the time: pre {pre.sum() / tot.sum():.2f} inbox {inb.sum() / tot.sum():.2f} "
          f"local {loc.sum() / tot.sum():.2f} fan-out {fan.sum() / tot.sum():.2f} "
          f"after {rest.sum() / tot.sum():.2f}")
    k = nin > 0
    print(f"us per inbox message (steps with any): {(inb[k] / nin[k]).mean():.2f}; "
          f"messages in / out per step: {nin.mean():.1f} / {nout.mean():.1f}")
    names = {12: "Rep", 13: "RepR", 14: "Vote", 15: "VoteR", 16: "Snap", 17: "HB", 18: "HBR",
             19: "RI", 20: "RIR", 7: "Prop", 21: "Qui", 23: "Xfer", 24: "TNow"}
    types, cnt = np.unique(mxt, return_counts=True)
    print("longest message's type:", {names.get(int(t), int(t)): int(c) for t, c in zip(types, cnt)})
    top = np.argsort(-tot)[:15]
    print(f"{'total':>7s} {'pre':>6s} {'inbox':>7s} {'local':>6s} {'fan':>6s} {'after':>6s} "
          f"{'maxmsg':>7s} type  in  out role")
    for i in top:
        print(f"{tot[i]:7.1f} {pre[i]:6.1f} {inb[i]:7.1f} {loc[i]:6.1f} {fan[i]:6.1f} {rest[i]:6.1f} "
              f"{mx[i]:7.1f} {names.get(int(mxt[i]), int(mxt[i])):>4} {nin[i]:3d} {nout[i]:4d} "
              f"{rb[i]}->{ra[i]}")
