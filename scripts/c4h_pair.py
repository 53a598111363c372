"""Summary of the c4h bench lines of one GPU pass (pipelined and serial)."""
import json
import sys

for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    b = d["boundary"]
    print(f.split("/")[-1], round(d["ms_per_step"], 3),
          {k: (round(v, 3) if isinstance(v, float) else v) for k, v in b.items() if k != "read_back"})
