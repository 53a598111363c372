#!/bin/bash
# Round-5 end evidence for the library in the tree: smoke, the whole -m gpu
# suite, the default bench line (both CPU baselines) and the driver's 20-step
# command, the rocprofv3 kernel-trace summary of the bench, the PMC passes
# (FETCH_SIZE, WRITE_SIZE; L2 request counts), the C3 and host-driven C4
# lines.  Each GPU step has its own limit; the first failure ends the call.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_final
mkdir -p $O
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "smoke ok $(( $(date +%s) - S ))s"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "gpu tests ok $(( $(date +%s) - S ))s"; tail -1 $O/gpu_tests.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
echo "bench ok $(( $(date +%s) - S ))s"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver20.json 2> $O/bench_driver20.err
echo "bench20 ok $(( $(date +%s) - S ))s"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --also "" > $O/prof.log 2>&1
echo "rocprof ok $(( $(date +%s) - S ))s"
WORKLOADS="c4" bash scripts/pmc_traffic.sh
cp gpurun_out/traffic_c4.json $O/traffic_c4.json
echo "pmc ok $(( $(date +%s) - S ))s"
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum -d $O/pmc_c4_REQ -o run --output-format csv -- python3 bench.py --workload c4 --steps 10 --warmup 2 --prof-rounds 10 --no-cpu-baseline --also "" > $O/pmc_c4_REQ.log 2>&1
echo "pmc req ok $(( $(date +%s) - S ))s"
timeout -k 10 300 python -u bench.py --workload c3 --no-cpu-baseline --also "" > $O/bench_c3.json 2> $O/bench_c3.err
echo "c3 ok $(( $(date +%s) - S ))s"
timeout -k 10 300 python -u bench.py --workload c4h --steps 50 --warmup 5 > $O/bench_c4h.json 2> $O/bench_c4h.err
echo "c4h ok $(( $(date +%s) - S ))s"
