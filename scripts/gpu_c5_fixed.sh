#!/bin/bash
# C5 rehearsal on one GPU (2 ranks on cuda:0, gloo staging): the counted and
# the fixed-capacity exchange back to back.  Each step has its own limit.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for mode in "" "--xchg-fixed"; do
  tag=${mode:+_fixed}
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --workload c5 --xchg-gloo $mode --groups ${C5_GROUPS:-100000} --steps 30 --warmup 5 --prof-rounds 10 > gpurun_out/bench_c5$tag.json 2> gpurun_out/bench_c5$tag.err || { tail -30 gpurun_out/bench_c5$tag.err; exit 1; }
  python3 scripts/summarize_bench.py gpurun_out/bench_c5$tag.json "c5$tag" || cat gpurun_out/bench_c5$tag.json
done
