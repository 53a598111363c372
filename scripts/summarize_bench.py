"""Print a one-line summary (and the per-kernel split) of a bench.py JSON line."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
tag = sys.argv[2] if len(sys.argv) > 2 else ""
r = d["roofline"]
print(f"{tag}: ms/step {d['ms_per_step']:.3f}  Gsteps/s {d['value'] / 1e9:.3f}  "
      f"commit/s {d['committed_entries_per_s']:.3g}  reads/s {d['read_confirmations_per_s']:.3g}  "
      f"dom {r['kernel']} {r['avg_launch_us']:.1f}us frac {r['frac']:.4f}  "
      f"round frac {d['round'].get('frac', float('nan')):.4f}  faulty {d['faulty_replicas']}")
if "exchange" in d:
    print(f"    exchange {d['exchange']}")
for k in d["round"]["kernels"]:
    print(f"    {k['kernel']:20s} {k['avg_us']:9.1f} us  {k['alg_bytes_per_launch'] / 1e6:9.2f} MB  "
          f"{k['achieved_gbs']:8.1f} GB/s")
