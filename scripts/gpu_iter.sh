# Iteration check: all GPU tests, A/B of the replay against the round-2 library (AP remote,
# 8,192 documents), config 4 at 16,384 documents with both libraries.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
OLD=text-crdt-rust_amd/build/libcrdt_gpu_r2.so
NEW=text-crdt-rust_amd/build/libcrdt_gpu.so
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/gpu_tests.log | head -20; exit 1; }
for rep in 1 2; do
  for L in $OLD $NEW; do
    echo -n "ap8192 $(basename $L) "
    CRDT_GPU_LIB=$L timeout -k 10 120 python scripts/prof_replay.py --docs 8192 --clean | tail -1 || exit 1
  done
done
for L in $OLD $NEW; do
  echo "c4 $(basename $L)"
  CRDT_GPU_LIB=$L timeout -k 10 300 python scripts/bench_config4.py --docs ${C4DOCS:-16384} --steps 2 --check-docs 16 --cpu-seconds 2 > gpurun_out/c4_$(basename $L).json 2>gpurun_out/c4_$(basename $L).err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/c4_$(basename $L).json')); print({k: d.get(k) for k in ('value','ms_per_step','parity_ok')}, d.get('replay_ms'))"
done
