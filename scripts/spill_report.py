"""Per-kernel code size and scratch traffic of an engine object or library:
VGPR / AGPR / scratch bytes (code object notes) and the count of
scratch_load / scratch_store instructions and calls in each named kernel's
disassembly.   python3 scripts/spill_report.py lib.so|obj.o [kernel-substring ...]"""
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin/"
path = sys.argv[1]
keys = sys.argv[2:] or ["k_fast_both", "k_full_list", "k_triage"]
blob = open(path, "rb").read()
starts = [m.start() for m in re.finditer(b"__CLANG_OFFLOAD_BUNDLE__", blob)]
with tempfile.TemporaryDirectory() as d:
    for k, i in enumerate(starts):
        fb, co = f"{d}/f{k}.bin", f"{d}/c{k}.o"
        open(fb, "wb").write(blob[i:starts[k + 1] if k + 1 < len(starts) else len(blob)])
        if subprocess.run([LLVM + "clang-offload-bundler", "--type=o", "--unbundle", f"--input={fb}",
                           f"--output={co}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"],
                          capture_output=True).returncode:
            continue
        syms = subprocess.run([LLVM + "llvm-objdump", "-t", co], capture_output=True,
                              text=True).stdout
        for line in syms.splitlines():
            parts = line.split()
            if not parts or ".text" not in line:
                continue
            name = parts[-1]
            m = re.search(r"\.text\s+([0-9a-fA-F]+)", line)
            size = int(m.group(1), 16) if m else 0
            if not name.startswith("_ZN3rbe") or not any(x in name for x in keys):
                continue
            dis = subprocess.run([LLVM + "llvm-objdump", "-d", f"--disassemble-symbols={name}", co],
                                 capture_output=True, text=True).stdout
            sl, ss = dis.count("scratch_load"), dis.count("scratch_store")
            calls = dis.count("s_swappc")
            print(f"{size:8d} B  scratch ld {sl:5d} st {ss:5d}  calls {calls:3d}  {name[:90]}")
