# Round-end evidence: all GPU tests, smoke(), the default bench line (with CPU baseline and the
# materialize leg), and a kernel-trace profile of the bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && echo tests-ok && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo smoke-ok && \
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && echo bench-ok && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ktrace -o ktrace --output-format csv -- python bench.py --no-cpu --no-stated-size --steps 2 --warmup 1 > gpurun_out/ktrace.log 2>&1 && echo ktrace-ok && \
{ [ "${SINGLE:-1}" != 1 ] || { timeout -k 10 400 python -u scripts/bench_single.py > gpurun_out/single.jsonl 2> gpurun_out/single.err && echo single-ok; }; }
