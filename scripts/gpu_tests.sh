set -o pipefail
cd $GRAFT_REPO_ROOT
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "pytest exit $?"
tail -30 gpurun_out/gpu_tests.log
