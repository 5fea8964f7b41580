# One optimisation iteration on the GPU: the GPU tests, the micro-path SQ profile (TAG) and a
# short bench (no CPU leg).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests$TAG.log 2>&1 && echo tests-ok && tail -1 gpurun_out/gpu_tests$TAG.log && \
TAG=$TAG bash scripts/gpu_micro_paths.sh && \
timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/bench$TAG.json 2> gpurun_out/bench$TAG.err && echo bench-ok && \
python -c "import json; d=json.load(open('gpurun_out/bench$TAG.json')); print('value', d['value']/1e9, 'ms', d['ms_per_step'], 'replay', d['roofline']['kernel_ms'], 'parity', d['parity_ok'], d['queries_ok'])"
