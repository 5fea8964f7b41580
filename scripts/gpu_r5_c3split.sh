# Round 5: GPU tests, then a same-box A/B of LIBS on config 3 (65,536 mixed local documents, no
# fit) and on rustcode / sveltecomponent local at 8,192 documents (prof_replay.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B=text-crdt-rust_amd/build
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_gpu_tests_${V:-v9}.log 2>&1
  rc=$?; echo tests rc=$rc; tail -1 gpurun_out/r5_gpu_tests_${V:-v9}.log
  [ $rc -le 1 ] || exit $rc
fi
for L in $LIBS; do
  echo -n "c3 65536 $L "; CRDT_GPU_LIB=$B/$L timeout -k 10 300 python scripts/prof_replay.py --docs 65536 --config3 --clean --no-fit | tail -1 || exit 1
done
for t in rustcode sveltecomponent; do
  for L in $LIBS; do
    echo -n "$t 8192 $L "; CRDT_GPU_LIB=$B/$L timeout -k 10 200 python scripts/prof_replay.py --docs 8192 --local --trace $t --clean | tail -1 || exit 1
  done
done
