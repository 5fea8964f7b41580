set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; echo "pytest exit $?"; tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u bench.py --docs ${DOCS:-4096} --steps 3 --warmup 1 --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err; echo "bench exit $?"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
