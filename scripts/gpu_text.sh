set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_text.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_text.log 2>&1 && echo text-ok && \
timeout -k 10 400 python -u bench.py --no-cpu > gpurun_out/bench_text.json 2> gpurun_out/bench_text.err && cat gpurun_out/bench_text.json && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ktrace_m -o ktrace --output-format csv -- python bench.py --no-cpu --steps 2 --warmup 1 > gpurun_out/ktrace_m.log 2>&1 && echo ktrace-ok
