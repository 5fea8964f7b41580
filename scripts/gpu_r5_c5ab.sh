# Round 5: GPU tests of the product library, then an A/B of LIBS on config 5 (C5DOCS documents,
# prof_replay.py --config5) and automerge-paper (8,192), same box.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B=text-crdt-rust_amd/build
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_gpu_tests_${V:-v4}.log 2>&1
  rc=$?; echo tests rc=$rc; tail -1 gpurun_out/r5_gpu_tests_${V:-v4}.log
  [ $rc -le 1 ] || exit $rc
fi
for L in $LIBS; do
  echo -n "c5 ${C5DOCS:-8192} $L "; CRDT_GPU_LIB=$B/$L timeout -k 10 300 python scripts/prof_replay.py --docs ${C5DOCS:-8192} --config5 --clean | tail -1 || exit 1
done
for L in $LIBS; do
  echo -n "ap 8192 $L "; CRDT_GPU_LIB=$B/$L timeout -k 10 120 python scripts/prof_replay.py --docs 8192 --clean | tail -1 || exit 1
done
