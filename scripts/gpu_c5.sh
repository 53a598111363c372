#!/bin/bash
# Replica-per-GPU (C5) on a one-GPU box: the parity tests (W processes on
# cuda:0, gloo), then a two-rank bench rehearsal with host-staged exchange.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_replica.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_replica.log 2>&1 || { tail -40 gpurun_out/gpu_replica.log; exit 1; }
tail -3 gpurun_out/gpu_replica.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --workload c5 --xchg-gloo --groups ${C5_GROUPS:-100000} --steps 30 --warmup 5 --prof-rounds 10 > gpurun_out/bench_c5_gloo.json 2> gpurun_out/bench_c5_gloo.err || { tail -30 gpurun_out/bench_c5_gloo.err; exit 1; }
python3 scripts/summarize_bench.py gpurun_out/bench_c5_gloo.json c5 || cat gpurun_out/bench_c5_gloo.json
