# GPU tests, then the secondary config lines (config 3 at 65,536 documents, config 4 at 125,000)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && echo tests-ok && tail -1 gpurun_out/gpu_tests.log && \
timeout -k 10 200 python scripts/pub_time.py 4096 && \
timeout -k 10 400 python -u scripts/bench_config3.py > gpurun_out/config3.json 2> gpurun_out/config3.err && echo c3-ok && cat gpurun_out/config3.json && \
timeout -k 10 500 python -u scripts/bench_config4.py > gpurun_out/config4.json 2> gpurun_out/config4.err && echo c4-ok && cat gpurun_out/config4.json
