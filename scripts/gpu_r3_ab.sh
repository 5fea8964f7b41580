# Round 3 A/B: GPU tests with the new library, AP replay base vs new (8,192 docs, twice each),
# then (MICRO=1) the SQ micro-path counts of the new library.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-v5}
OLD=text-crdt-rust_amd/build/libcrdt_gpu_base.so
NEW=text-crdt-rust_amd/build/libcrdt_gpu.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1; rc=$?
tail -1 gpurun_out/gpu_tests_$TAG.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_$TAG.log | head -20; exit 1; }
for L in $OLD $NEW $OLD $NEW; do
  echo -n "ap8192 $(basename $L) "
  CRDT_GPU_LIB=$L timeout -k 10 120 python scripts/prof_replay.py --docs 8192 --clean | tail -1 || exit 1
done
for L in $OLD $NEW; do
  echo -n "c5-1024 $(basename $L) "
  CRDT_GPU_LIB=$L timeout -k 10 200 python scripts/prof_replay.py --docs 1024 --config5 --clean | tail -1 || exit 1
done
[ -z "$MICRO" ] || TAG=_$TAG bash scripts/gpu_micro_paths.sh
