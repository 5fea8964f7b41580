# Iteration: GPU tests, AP A/B vs the round-2 library, config 5 (1,024 docs) with the memory layout
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
OLD=text-crdt-rust_amd/build/libcrdt_gpu_r2.so
NEW=text-crdt-rust_amd/build/libcrdt_gpu.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log
grep -E "PASSED|FAILED" gpurun_out/gpu_tests.log | grep -E "kevin|api|config5" 
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/gpu_tests.log | head -20; exit 1; }
for L in $OLD $NEW $OLD $NEW; do
  echo -n "ap8192 $(basename $L) "
  CRDT_GPU_LIB=$L timeout -k 10 120 python scripts/prof_replay.py --docs 8192 --clean | tail -1 || exit 1
done
CRDT_DEBUG_MEM=1 timeout -k 10 600 python -u scripts/bench_config5.py --cpu-seconds 5 > gpurun_out/c5_${TAG:-v2}.json 2> gpurun_out/c5_${TAG:-v2}.err && echo c5-ok && tail -3 gpurun_out/c5_${TAG:-v2}.err && \
python -c "import json; d=json.load(open('gpurun_out/c5_${TAG:-v2}.json')); print(d['value']/1e9, d['ms_per_step'], d['kernels_ms'], d['roofline']['frac'], d['parity_ok'], d['config']['hbm_bytes_per_doc'])"
