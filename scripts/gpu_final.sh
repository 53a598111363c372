#!/bin/bash
# Round-end evidence on one GPU box for the library in the tree: smoke, the
# whole -m gpu suite, the default bench line (CPU baseline included), its
# rocprofv3 kernel-trace summary, the PMC passes (FETCH_SIZE, WRITE_SIZE, L2
# read/write requests) of the same command, and the C3 and host-driven C4
# lines.  Each GPU step has its own limit; the first failure ends the call.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
echo "smoke ok $(( $(date +%s) - S ))s"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "gpu tests ok $(( $(date +%s) - S ))s"; tail -1 gpurun_out/gpu_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "bench ok $(( $(date +%s) - S ))s"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --also "" > gpurun_out/prof.log 2>&1
echo "rocprof ok $(( $(date +%s) - S ))s"
WORKLOADS="c4" bash scripts/pmc_traffic.sh
echo "pmc ok $(( $(date +%s) - S ))s"
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum -d gpurun_out/pmc_c4_REQ -o run --output-format csv -- python3 bench.py --workload c4 --steps 10 --warmup 2 --prof-rounds 10 --no-cpu-baseline --also "" > gpurun_out/pmc_c4_REQ.log 2>&1
echo "pmc req ok $(( $(date +%s) - S ))s"
timeout -k 10 300 python -u bench.py --workload c3 --no-cpu-baseline --also "" > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err
echo "c3 ok $(( $(date +%s) - S ))s"
timeout -k 10 300 python -u bench.py --workload c4h --steps 50 --warmup 5 > gpurun_out/bench_c4h.json 2> gpurun_out/bench_c4h.err
echo "c4h ok $(( $(date +%s) - S ))s"
