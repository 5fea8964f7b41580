# Round 3: GPU tests, AP A/B (base vs new), config 5 at 1,024 docs with both libraries (bench line)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-v7}
B=text-crdt-rust_amd/build
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1; rc=$?
tail -1 gpurun_out/gpu_tests_$TAG.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_$TAG.log | head -20; exit 1; }
for L in $B/libcrdt_gpu_base.so $B/libcrdt_gpu.so $B/libcrdt_gpu_base.so $B/libcrdt_gpu.so; do
  echo -n "ap8192 $(basename $L) "
  CRDT_GPU_LIB=$L timeout -k 10 120 python scripts/prof_replay.py --docs 8192 --clean | tail -1 || exit 1
done
for L in $B/libcrdt_gpu_base.so $B/libcrdt_gpu.so; do
  CRDT_GPU_LIB=$L timeout -k 10 300 python -u scripts/bench_config5.py --docs 1024 --no-cpu > gpurun_out/c5ab_$(basename $L).json 2> /dev/null && \
  python -c "import json; d=json.load(open('gpurun_out/c5ab_$(basename $L).json')); print('c5-1024 $(basename $L)', d['value']/1e6, 'M ops/s', d['kernels_ms'], d['parity_ok'])" || exit 1
done
