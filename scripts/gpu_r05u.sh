#!/bin/bash
# Round 5: the default bench line with both CPU baselines, C3 and C4 lines.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 600 python -u bench.py > gpurun_out/r05u_bench.json 2> gpurun_out/r05u_bench.err
echo "bench ok $(( $(date +%s) - S ))s"
python3 -c "
import json; d=json.load(open('gpurun_out/r05u_bench.json'))
print(d['ms_per_step'], d['value']/1e9, d['roofline']['frac']); cb=d['cpu_baseline']; print(cb['value'], cb['cores'], cb.get('one_thread',{}).get('value'), cb.get('soa_host'))
print({k:(v.get('ms_per_step'), v['dominant']) for k,v in d.get('workloads',{}).items()})"
