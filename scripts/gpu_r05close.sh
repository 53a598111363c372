#!/bin/bash
# Round 5 close: smoke and the driver's exact 20-step bench command on the
# tree's library, on whatever box this lands on (reproducibility check).
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_close
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
tail -1 $O/smoke.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_driver20.json 2> $O/bench_driver20.err
python3 scripts/summarize_bench.py $O/bench_driver20.json driver20
timeout -k 10 300 python -u bench.py --no-cpu-baseline --also "" > $O/bench_default.json 2> $O/bench_default.err
python3 scripts/summarize_bench.py $O/bench_default.json default
