#!/bin/bash
# The at-scale wire hop only (scripts/wire_ingest_bench.py), timed and under
# rocprofv3 --stats (csv).
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/wire_ingest_bench.py --groups ${GROUPS_:-100000} --gpb ${GPB:-512} \
  > gpurun_out/ingest_bench.json 2> gpurun_out/ingest_bench.err
echo "bench ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ingest -o run --output-format csv -- \
  python3 scripts/wire_ingest_bench.py --groups ${GROUPS_:-100000} --gpb ${GPB:-512} --rounds 10 --warmup 30 \
  > gpurun_out/prof_ingest.log 2>&1
echo "prof ok"
