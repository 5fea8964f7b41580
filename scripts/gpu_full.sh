# Round evidence: GPU tests, the default bench line (CPU baseline + text leg), a kernel-trace
# profile of the bench, and the PMC passes (SQ + HBM) of one clean k_replay launch.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && echo tests-ok && tail -1 gpurun_out/gpu_tests.log && \
timeout -k 10 400 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err && echo bench-ok && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ktrace -o ktrace --output-format csv -- python bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.err && echo ktrace-ok && \
DOCS=8192 bash scripts/gpu_pmc_all.sh
