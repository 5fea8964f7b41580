# Round 4 A/B on one box: (optionally) the GPU tests on the new library, then alternating clean
# k_replay launches of the base and new libraries on 8,192 automerge-paper remote documents, and
# (EXTRA=1) config 5 (1,024 docs), config 4 (16,384 docs) and kevin (one document + 64).
# usage: TAG=v1 TESTS=1 EXTRA=0 [LIBS="a.so b.so"] bash scripts/gpu_r4_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-v1}
B=text-crdt-rust_amd/build
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1; rc=$?
  tail -1 gpurun_out/gpu_tests_$TAG.log
  [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_$TAG.log | head -20; exit 1; }
fi
LIBS=${LIBS:-"libcrdt_gpu_base.so libcrdt_gpu.so"}
for L in $LIBS $LIBS; do
  L=$B/$L
  echo -n "ap8192 $(basename $L) "
  CRDT_GPU_LIB=$L timeout -k 10 120 python scripts/prof_replay.py --docs 8192 --clean | tail -1 || exit 1
done
if [ "${EXTRA:-0}" = 1 ]; then
for L in $B/libcrdt_gpu_base.so $B/libcrdt_gpu.so; do
  N=$(basename $L .so)
  CRDT_GPU_LIB=$L timeout -k 10 300 python -u scripts/bench_config5.py --docs 1024 --no-cpu > gpurun_out/ab_c5_$N.json 2> /dev/null && \
  python -c "import json; d=json.load(open('gpurun_out/ab_c5_$N.json')); print('c5-1024 $N', round(d['value']/1e6, 2), 'M ops/s', d['kernels_ms'], d['parity_ok'])" || exit 1
  CRDT_GPU_LIB=$L timeout -k 10 300 python -u scripts/bench_config4.py --docs 16384 --cpu-seconds 0.5 > gpurun_out/ab_c4_$N.json 2> /dev/null && \
  python -c "import json; d=json.load(open('gpurun_out/ab_c4_$N.json')); print('c4-16384 $N', round(d['value']/1e9, 3), 'G ops/s', d['kernels_ms'], d['parity_ok'])" || exit 1
  CRDT_GPU_LIB=$L timeout -k 10 300 python -u scripts/bench_kevin.py --docs 64 --reps 2 > gpurun_out/ab_kevin_$N.json 2> /dev/null && \
  python -c "import json; d=json.load(open('gpurun_out/ab_kevin_$N.json')); print('kevin $N', d['single_doc']['k_replay_ms'], 'ms', d['batch']['ops_per_s']/1e9, 'G ops/s @64', d['parity_ok'])" || exit 1
done
fi
