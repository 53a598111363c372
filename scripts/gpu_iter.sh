set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -5 | tee gpurun_out/gpu_tests.log
for w in c4 c2m c2; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --workload $w --no-cpu-baseline 2>&1 | grep metric | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w', 'ms/step %.3f'%d['ms_per_step'], 'Gsteps/s %.3f'%(d['value']/1e9), 'commit/s %.3g'%d['committed_entries_per_s'], 'frac %.4f'%d['roofline']['frac'], 'faulty', d['faulty_replicas'])" | tee -a gpurun_out/bench_iter.log
done
RBE_MODE=full timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --workload c4 --no-cpu-baseline 2>&1 | grep metric | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4-fullmode', 'ms/step %.3f'%d['ms_per_step'])" | tee -a gpurun_out/bench_iter.log
