#!/bin/bash
# The general step's inbox head in LDS (RBE_FULL_INPF = 2, 4, 6 messages per
# lane, global_load_lds before the first store): the GPU suite on the K=4 build,
# then C3 A/B pairs against the default library.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RBE_LIB=$PWD/build/inpf4.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/inpf_tests.log 2>&1
echo "inpf4 gpu tests ok"; tail -1 gpurun_out/inpf_tests.log
for rep in 1 2; do
  for lib in dragonboat_amd/libdragonboat_amd.so build/inpf2.so build/inpf4.so build/inpf6.so; do
    RBE_LIB=$PWD/$lib timeout -k 10 200 python bench.py --workload c3 --no-cpu-baseline --also "" \
      --steps 100 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err
    python3 scripts/summarize_bench.py gpurun_out/ab.json "$(basename $lib) c3 #$rep" | grep -E "ms/step|k_full_list"
  done
done
