# Iteration: all GPU tests (incl. the two-level root), AP A/B vs the round-2 library
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
OLD=text-crdt-rust_amd/build/libcrdt_gpu_r2.so
NEW=text-crdt-rust_amd/build/libcrdt_gpu.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=8 > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -12 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/gpu_tests.log | head -20; exit 1; }
C3=text-crdt-rust_amd/build/libcrdt_gpu_c3.so
for L in $OLD $C3 $NEW $OLD $C3 $NEW; do
  echo -n "ap8192 $(basename $L) "
  CRDT_GPU_LIB=$L timeout -k 10 120 python scripts/prof_replay.py --docs 8192 --clean | tail -1 || exit 1
done
