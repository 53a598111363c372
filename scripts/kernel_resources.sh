#!/bin/bash
# Per-kernel resources of the gfx950 engine build: code length, VGPRs/AGPRs,
# SGPRs, scratch and occupancy, from the compiler's own assembly comments.
#   bash scripts/kernel_resources.sh [extra hipcc flags...]
# The assembly stays in build/temps/ for reading.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/build/temps
mkdir -p "$OUT"
cd "$OUT"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared --save-temps "$@" \
  -DRBE_SINGLE_TU -o "$OUT/libtmp.so" "$ROOT/dragonboat_amd/csrc/rbe_engine.hip" 2>/dev/null
S=$(ls "$OUT"/*gfx950*.s | head -1)
python3 - "$S" <<'EOF'
import re
import subprocess
import sys
cur = None
rows = []
for line in open(sys.argv[1]):
    m = re.match(r"^(_Z[^:\s]+):", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    if cur is None:
        continue
    for key, pat in (("code", r"; codeLenInByte = (\d+)"), ("vgpr", r"; NumVgprs: (\d+)"),
                     ("agpr", r"; NumAgprs: (\d+)"), ("sgpr", r"; NumSgprs: (\d+)"),
                     ("scratch", r"; ScratchSize: (\d+)"), ("occ", r"; Occupancy: (\d+)")):
        m = re.search(pat, line)
        if m:
            cur[key] = int(m.group(1))
for r in rows:
    if "code" not in r:
        continue
    dn = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
    print(f"{r['code']:8d} B  vgpr {r.get('vgpr', 0):3d} agpr {r.get('agpr', 0):3d} "
          f"sgpr {r.get('sgpr', 0):3d} scratch {r.get('scratch', 0):5d} occ {r.get('occ', 0)}  "
          f"{dn[:100]}")
EOF
