set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && echo tests-ok && \
timeout -k 10 400 python -u scripts/bench_config3.py --docs ${C3DOCS:-8192} > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err && echo c3-ok && cat gpurun_out/bench_c3.json && \
timeout -k 10 300 python -u scripts/bench_config4.py --docs ${C4DOCS:-32768} > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err && echo c4-ok && cat gpurun_out/bench_c4.json
echo "exit $?"; tail -3 gpurun_out/gpu_tests.log
