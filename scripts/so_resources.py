"""Per-kernel VGPRs / scratch / LDS of a built engine library, read from the
gfx950 code object's metadata notes (no rebuild; scripts/kernel_resources.sh
is the full --save-temps variant).   python3 scripts/so_resources.py lib.so [filter]"""
import re
import subprocess
import sys
import tempfile

lib = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
blob = open(lib, "rb").read()
starts = [m.start() for m in re.finditer(b"__CLANG_OFFLOAD_BUNDLE__", blob)]
if not starts:
    sys.exit("no offload bundle in " + lib)
notes = ""
with tempfile.TemporaryDirectory() as d:
    # one bundle per translation unit (rbe_engine.hip, rbe_round.hip per N and trace)
    for k, i in enumerate(starts):
        fb = f"{d}/fat{k}.bin"
        open(fb, "wb").write(blob[i:starts[k + 1] if k + 1 < len(starts) else len(blob)])
        co = f"{d}/co{k}.o"
        r = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--type=o",
                            "--unbundle", f"--input={fb}", f"--output={co}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"], capture_output=True)
        if r.returncode == 0:
            notes += subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", co],
                                    capture_output=True, text=True).stdout
cur = {}
rows = []
for line in notes.splitlines():
    line = line.strip()
    m = re.match(r"- \.agpr_count:\s+(\d+)", line) or re.match(r"\.agpr_count:\s+(\d+)", line)
    for key in ("agpr_count", "group_segment_fixed_size", "private_segment_fixed_size",
                "vgpr_count", "sgpr_count", "name"):
        mm = re.match(r"-?\s*\." + key + r":\s+(\S+)", line)
        if mm:
            if key == "agpr_count" and cur:
                rows.append(cur)
                cur = {}
            cur[key] = mm.group(1)
if cur:
    rows.append(cur)
for r in rows:
    n = r.get("name", "?")
    if flt in n:
        print(f"vgpr {r.get('vgpr_count'):>4} agpr {r.get('agpr_count'):>3} scratch "
              f"{r.get('private_segment_fixed_size'):>5} lds {r.get('group_segment_fixed_size'):>6}  {n}")
