# Publish iteration: GPU tests, k_publish wall time at 8,192 AP documents, a short bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests$TAG.log 2>&1 && echo tests-ok && tail -1 gpurun_out/gpu_tests$TAG.log && \
timeout -k 10 150 python scripts/pub_time.py 8192 > gpurun_out/pub_time$TAG.txt 2>&1 && cat gpurun_out/pub_time$TAG.txt && \
timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/bench$TAG.json 2> gpurun_out/bench$TAG.err && echo bench-ok && \
python -c "import json; d=json.load(open('gpurun_out/bench$TAG.json')); print('value', d['value']/1e9, 'ms', d['ms_per_step'], 'replay', d['roofline']['kernel_ms'], 'parity', d['parity_ok'], d['queries_ok'])"
