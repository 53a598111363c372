#!/bin/bash
# Round 4: host-input fast path (GPU tests), the c4h line, the k_full_list wave
# profile on C3 (diagnostic build).  Each GPU step has its own limit.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 300 python -u -m pytest tests/test_gpu_node_inputs.py tests/test_gpu_outputs.py tests/test_gpu_payload_heap.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_inputs.log 2>&1 || { tail -30 gpurun_out/gpu_inputs.log; exit 1; }
echo "input tests ok $(( $(date +%s) - S ))s"; tail -1 gpurun_out/gpu_inputs.log
timeout -k 10 300 python -u bench.py --workload c4h --steps 50 --warmup 5 > gpurun_out/bench_c4h.json 2> gpurun_out/bench_c4h.err || { tail -20 gpurun_out/bench_c4h.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_c4h.json').read().strip().splitlines()[-1]);print('c4h', d['ms_per_step'], d['boundary'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4h -o run -- python3 bench.py --workload c4h --steps 30 --warmup 5 > gpurun_out/prof_c4h.log 2>&1 || { tail -20 gpurun_out/prof_c4h.log; exit 1; }
echo "prof ok $(( $(date +%s) - S ))s"
RBE_LIB=$PWD/build/full_prof.so timeout -k 10 300 python -u scripts/full_prof.py c3 > gpurun_out/full_prof_c3.log 2>&1 || { tail -20 gpurun_out/full_prof_c3.log; exit 1; }
cat gpurun_out/full_prof_c3.log
echo "all ok $(( $(date +%s) - S ))s"
