"""Diagnostic: the untraced MIXED membership-snapshot case on the HIP engine
against the host build and the oracle, round by round; on the first
divergence print the group's views (both engines and the oracle) for the
rounds before it."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import oracle as O  # noqa: E402
from dragonboat_amd.engine import Engine  # noqa: E402
from parity_util import view_diff  # noqa: E402
from soa_cpu.soa import SoaCpu  # noqa: E402
from test_membership_snapshot import CASES  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "MIXED"
trace = len(sys.argv) > 2 and sys.argv[2] == "trace"
kw, extra, rounds = CASES[name]
g_eng = Engine(device=0, trace=trace, **kw, **extra)
s_eng = SoaCpu(trace=trace, **kw, **extra)
ref = O.Harness(**kw)
n = kw["n_replicas"]
hist = []
F = ["role", "term", "vote", "leader_id", "committed", "last_index", "processed", "removed",
     "election_tick", "q_tick", "raft_quiesce"]
for rnd in range(rounds):
    g_eng.run(1)
    s_eng.run(1)
    ref.run(1)
    gv, sv, hv = g_eng.views(), s_eng.views(), ref.views()
    gs, ss = g_eng.snapshot_state(), s_eng.snapshot_state()
    hist.append((gv, sv, hv, gs, ss))
    hist = hist[-8:]
    bad = [i for i in range(len(hv)) if view_diff(gv[i], sv[i], ("digest",)) or
           tuple(gs[i]) != tuple(ss[i])]
    if bad:
        i0 = bad[0]
        g = i0 // n
        print(f"round {rnd + 1}: GPU differs from host build at replicas {bad[:10]}:",
              view_diff(gv[i0], sv[i0], ("digest",)), tuple(gs[i0]), tuple(ss[i0]))
        print("host vs oracle:", view_diff(sv[i0], hv[i0], ("digest",)))
        for back, (a, b, c, sa, sb) in enumerate(hist):
            print(f"-- round {rnd + 2 - len(hist) + back}")
            for i in range(g * n, g * n + n):
                for tag, v in (("G", a[i]), ("S", b[i]), ("O", c[i])):
                    print(" ", tag, i, {f: getattr(v, f) for f in F}, "match",
                          list(v.match)[:n], "next", list(v.next)[:n])
                print("   snap G", tuple(sa[i]), "S", tuple(sb[i]))
        sys.exit(1)
print("no divergence in", rounds, "rounds")
