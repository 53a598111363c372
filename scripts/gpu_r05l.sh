#!/bin/bash
# Round 5: ingest evidence on the final wire code (tests, the 512-group and
# one-frame-per-pair ingest workloads, the 7 MB decode, rocprof splits) and the
# per-phase wave cycles of k_triage (RBE_PHASE_TIMING build).
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05_ingest
export TMPDIR=/tmp
O=gpurun_out/r05_ingest
S=$(date +%s)
timeout -k 10 600 python -u -m pytest tests/test_gpu_wire_big.py tests/test_gpu_wire.py tests/test_gpu_wire_ingest.py -x -q --timeout 300 --timeout-method thread > $O/gpu_wire_tests.log 2>&1
echo "tests ok $(( $(date +%s) - S ))s"; tail -1 $O/gpu_wire_tests.log
for g in 512 100000; do
  timeout -k 10 300 python -u scripts/wire_ingest_bench.py --gpb $g > $O/ingest_gpb$g.json 2> $O/ingest_gpb$g.err
  echo "ingest gpb=$g"; cat $O/ingest_gpb$g.json
done
RBE_INGEST_EXACT=1 timeout -k 10 300 python -u scripts/wire_ingest_bench.py --gpb 512 > $O/ingest_gpb512_exact.json 2> $O/exact.err
echo "exact"; cat $O/ingest_gpb512_exact.json
timeout -k 10 200 python -u scripts/wire_big_bench.py > $O/decode_7mb.json 2> $O/decode_7mb.err
echo "big"; cat $O/decode_7mb.json
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_decode_7mb -o big -- python3 $GRAFT_REPO_ROOT/scripts/wire_big_bench.py --reps 3 > $GRAFT_REPO_ROOT/$O/prof_decode_7mb.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_ingest_gpb512 -o ing -- python3 $GRAFT_REPO_ROOT/scripts/wire_ingest_bench.py --gpb 512 > $GRAFT_REPO_ROOT/$O/prof_ingest.log 2>&1
cd $GRAFT_REPO_ROOT
echo "prof ok $(( $(date +%s) - S ))s"
timeout -k 10 200 python -u scripts/phase_timing.py c4 > gpurun_out/r05l_phase_c4.log 2>&1
echo "phase"; cat gpurun_out/r05l_phase_c4.log
