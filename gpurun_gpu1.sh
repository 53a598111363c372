set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tee gpurun_out/smoke.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/gpu_tests.log
