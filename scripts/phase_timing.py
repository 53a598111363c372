"""Diagnostic: per-phase wave time of the fast steps (s_memtime stamps) from
the RBE_PHASE_TIMING build (build/libdragonboat_amd_phase.so).

    scripts/build_variant.sh build/libdragonboat_amd_phase.so -DRBE_PHASE_TIMING
    python scripts/phase_timing.py c4
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from dragonboat_amd import engine as E  # noqa: E402

lib = E.load_library(os.path.join(ROOT, "build", "libdragonboat_amd_phase.so"))
E._lib = lib
lib.rbe_debug_phases.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
w = sys.argv[1] if len(sys.argv) > 1 else "c4"
kw, settle, _ = bench.WORKLOADS[w]
kw = dict(kw)
if len(sys.argv) > 2:
    kw["n_groups"] = int(sys.argv[2])
eng = E.Engine(**kw)
eng.run(settle)
eng.sync()
o = (C.c_uint64 * 24)()
lib.rbe_debug_phases(eng.h, o)
rounds = 20
ms = eng.profile_rounds(rounds)
lib.rbe_debug_phases(eng.h, o)
names = {0: ["gather1", "gather2", "inbox+read", "tick+propose", "scatter+finish"],
         1: ["gather1", "gather2", "inbox", "-", "tick+finish"],
         2: ["groups", "loads", "classify+reserve", "lds-fill", "copy-out", "counters"]}
for role, rn in ((0, "leader"), (1, "follower"), (2, "triage")):
    n = o[role * 8 + 7]
    if not n:
        continue
    parts = [f"{names[role][i]}={o[role * 8 + i] / n:.0f}" for i in range(len(names[role]))
             if names[role][i] != "-"]
    print(f"{w} {rn}: waves={n / rounds:.0f}/round cycles/wave: " + " ".join(parts))
    tot, rt = o[role * 8 + 6] / n, o[role * 8 + 5] / n
    if rt and role < 2:
        print(f"    wave t0->t5: {tot:.0f} cycles, {rt * 0.01:.2f} us realtime, "
              f"clock {tot / (rt * 0.01) / 1e3:.2f} GHz")
print("kernel ms per round:", [round(x / rounds, 4) for x in ms], eng.kernel_names())
