set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 100 --warmup 10 2>&1 | tee gpurun_out/bench_c4.log
timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --workload c2m --no-cpu-baseline 2>&1 | tee gpurun_out/bench_c2m.log
timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --workload c2 --no-cpu-baseline 2>&1 | tee gpurun_out/bench_c2.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/prof_c4.log 2>&1
echo done
