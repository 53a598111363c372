#!/bin/bash
# Round 5: C5's replica-per-GPU round at its per-GPU size (500k groups per rank),
# two ranks sharing the one GPU of the box, the exchange staged through gloo
# (a rehearsal of the RCCL path: same packing, same fixed-capacity layout):
# the fixed exchange (no host count read) and the counted one.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05_c5
export TMPDIR=/tmp
for mode in fixed counted; do
  extra=""; [ $mode = fixed ] && extra="--xchg-fixed"
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2953${#mode} bench.py --workload c5 --gpus 2 --xchg-gloo $extra --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05_c5/c5_w2_$mode.json 2> gpurun_out/r05_c5/c5_w2_$mode.err
  echo "$mode: $(tail -c 1500 gpurun_out/r05_c5/c5_w2_$mode.json)"
done
