# Round 5: GPU tests, then a same-box A/B of LIBS on automerge-paper (8,192, two reps), config 4
# (16,384 documents x 20,000 generated ops) and config 3 (65,536, no fit): clean k_replay launches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B=text-crdt-rust_amd/build
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_gpu_tests_${V:-v11}.log 2>&1
  rc=$?; echo tests rc=$rc; tail -1 gpurun_out/r5_gpu_tests_${V:-v11}.log
  [ $rc -le 1 ] || exit $rc
fi
for rep in 1 2; do
  for L in $LIBS; do
    echo -n "ap 8192 $L "; CRDT_GPU_LIB=$B/$L timeout -k 10 120 python scripts/prof_replay.py --docs 8192 --clean | tail -1 || exit 1
  done
done
for L in $LIBS; do
  echo -n "c4 16384 $L "; CRDT_GPU_LIB=$B/$L timeout -k 10 200 python scripts/prof_replay.py --docs 16384 --random 20000 --clean | tail -1 || exit 1
done
for L in $LIBS; do
  echo -n "c3 65536 $L "; CRDT_GPU_LIB=$B/$L timeout -k 10 300 python scripts/prof_replay.py --docs 65536 --config3 --clean --no-fit | tail -1 || exit 1
done
