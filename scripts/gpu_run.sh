#!/bin/bash
# One GPU-box runner for every measurement of a round (replaces the per-call
# scripts of earlier rounds):
#   gpurun -- bash scripts/gpu_run.sh OUT STEP [STEP ...]
# OUT is a directory under gpurun_out/; the steps run in order, each under its
# own time limit, and the first failure ends the call:
#   smoke      __graft_entry__.smoke()
#   spill      tests/test_gpu_spill.py (the spill tiers on the HIP engine)
#   suite      the whole -m gpu suite
#   bench      bench.py as the driver runs it (20 steps), then the default run
#   prof       rocprofv3 kernel trace + stats of the default bench (C4 only)
#   c4h        the host-driven round, pipelined and serial
#   c5         the replica-per-GPU rehearsal (2 ranks on the one GPU, gloo), counted and fixed
#   pmc        HBM traffic counters of the default bench (scripts/pmc_traffic.sh)
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
shift
mkdir -p "$O"
export TMPDIR=/tmp
S=$(date +%s)
for step in "$@"; do
  case $step in
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1 ||
        { tail -20 "$O/smoke.txt"; exit 1; } ;;
    spill)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_spill.py -x -v --timeout 300 \
        --timeout-method thread > "$O/gpu_spill.log" 2>&1 ||
        { grep -E "FAILED|Error" "$O/gpu_spill.log" | head -20; tail -30 "$O/gpu_spill.log"; exit 1; }
      tail -1 "$O/gpu_spill.log" ;;
    suite)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 \
        --timeout-method thread > "$O/gpu_tests.log" 2>&1 ||
        { grep -E "FAILED|Error" "$O/gpu_tests.log" | head -20; tail -30 "$O/gpu_tests.log"; exit 1; }
      tail -1 "$O/gpu_tests.log" ;;
    bench)
      timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$O/bench_driver20.json" \
        2> "$O/bench_driver20.err"
      python3 scripts/summarize_bench.py "$O/bench_driver20.json" driver20
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --also "" > "$O/bench_default.json" \
        2> "$O/bench_default.err"
      python3 scripts/summarize_bench.py "$O/bench_default.json" default ;;
    prof)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" \
        -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --also "" \
        > "$GRAFT_REPO_ROOT/$O/bench_prof.json" 2> "$GRAFT_REPO_ROOT/$O/bench_prof.err") ;;
    c4h)
      timeout -k 10 400 python -u bench.py --workload c4h --steps 50 --warmup 5 --no-cpu-baseline \
        > "$O/bench_c4h.json" 2> "$O/bench_c4h.err"
      timeout -k 10 400 python -u bench.py --workload c4h --steps 50 --warmup 5 --no-cpu-baseline \
        --c4h-serial > "$O/bench_c4h_serial.json" 2> "$O/bench_c4h_serial.err"
      python3 scripts/c4h_pair.py "$O/bench_c4h.json" "$O/bench_c4h_serial.json" ;;
    c5)
      # two ranks sharing the box's one GPU, the exchange staged through gloo
      for mode in "" "--xchg-fixed"; do
        tag=${mode:+_fixed}
        timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
          --master-addr 127.0.0.1 --master-port 29533 bench.py --workload c5 --xchg-gloo $mode \
          --groups ${C5_GROUPS:-100000} --steps 30 --warmup 5 --prof-rounds 10 \
          > "$O/bench_c5$tag.json" 2> "$O/bench_c5$tag.err" || { tail -30 "$O/bench_c5$tag.err"; exit 1; }
        python3 scripts/summarize_bench.py "$O/bench_c5$tag.json" "c5$tag"
      done ;;
    pmc)
      timeout -k 10 600 bash scripts/pmc_traffic.sh ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
  echo "$step ok $(( $(date +%s) - S ))s"
done
