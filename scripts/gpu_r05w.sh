#!/bin/bash
# Round 5: deferred Replicate sends in the general step — the whole GPU suite,
# then an A/B against the build without them (RBE_NO_DEFER) on C3 / C3s / C2s / C4.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05w_tests.log 2>&1
echo "tests ok $(( $(date +%s) - S ))s: $(tail -1 gpurun_out/r05w_tests.log)"
for rep in 1 2; do
for lib in build/libdragonboat_amd_nodefer.so dragonboat_amd/libdragonboat_amd.so; do
  for w in c3 c3s c2s c4; do
    RBE_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --also "" --steps 100 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err
    python3 scripts/summarize_bench.py gpurun_out/ab.json "$(basename $lib) $w" | head -4 | tr '\n' ' ' | sed 's/  */ /g'; echo
  done
done
done
