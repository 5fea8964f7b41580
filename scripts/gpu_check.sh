# Quick iteration: all GPU tests, then a kernel-trace profile of a short bench (no CPU leg).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && echo tests-ok && tail -1 gpurun_out/gpu_tests.log && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ktrace -o ktrace --output-format csv -- python bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.err && echo ktrace-ok && \
cut -c1-160 gpurun_out/ktrace/ktrace_kernel_stats.csv | head -6 && python -c "import json; d=json.load(open('gpurun_out/bench.json')); print(d['ms_per_step'], d['value']/1e9)"
