#!/bin/bash
# Round 4: rbe_collect_step GPU test, the C5 full-size rehearsal, then the
# host-driven C4 line with the sparse read-back and with every message, and a
# kernel trace of the former.  Each GPU step has its own limit.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 300 python -u -m pytest tests/test_gpu_outputs.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_outputs.log 2>&1 || { tail -30 gpurun_out/gpu_outputs.log; exit 1; }
echo "outputs tests ok $(( $(date +%s) - S ))s"; tail -1 gpurun_out/gpu_outputs.log
timeout -k 10 300 python -u bench.py --workload c4h --steps 50 --warmup 5 > gpurun_out/bench_c4h.json 2> gpurun_out/bench_c4h.err || { tail -20 gpurun_out/bench_c4h.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_c4h.json').read().strip().splitlines()[-1]);print('c4h', d['ms_per_step'], d['boundary'])"
timeout -k 10 300 python -u bench.py --workload c4h --steps 50 --warmup 5 --c4h-all-msgs > gpurun_out/bench_c4h_all.json 2> gpurun_out/bench_c4h_all.err || { tail -20 gpurun_out/bench_c4h_all.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_c4h_all.json').read().strip().splitlines()[-1]);print('c4h all', d['ms_per_step'], d['boundary'])"
echo "c4h ok $(( $(date +%s) - S ))s"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4h -o run -- python3 bench.py --workload c4h --steps 30 --warmup 5 > gpurun_out/prof_c4h.log 2>&1 || { tail -20 gpurun_out/prof_c4h.log; exit 1; }
echo "prof ok $(( $(date +%s) - S ))s"
timeout -k 10 600 python -u -m pytest tests/test_gpu_c5_rehearsal.py -m gpu -x -v --timeout 580 --timeout-method thread > gpurun_out/gpu_c5r.log 2>&1 || { tail -30 gpurun_out/gpu_c5r.log; exit 1; }
echo "c5 rehearsal ok $(( $(date +%s) - S ))s"; tail -1 gpurun_out/gpu_c5r.log
