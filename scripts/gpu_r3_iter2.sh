# Round-3 iteration: GPU tests, AP A/B (base vs new library, 8,192 docs), query-kernel A/B, and the
# HBM passes (FETCH_SIZE, WRITE_SIZE) over one clean AP k_replay launch of the new library.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-v4}
OLD=text-crdt-rust_amd/build/libcrdt_gpu_base.so
NEW=text-crdt-rust_amd/build/libcrdt_gpu.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1; rc=$?
tail -1 gpurun_out/gpu_tests_$TAG.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_$TAG.log | head -20; exit 1; }
for L in $OLD $NEW $OLD $NEW; do
  echo -n "ap8192 $(basename $L) "
  CRDT_GPU_LIB=$L timeout -k 10 120 python scripts/prof_replay.py --docs 8192 --clean | tail -1 || exit 1
done
timeout -k 10 300 python -u scripts/bench_queries.py > gpurun_out/queries_$TAG.json 2> gpurun_out/queries_$TAG.err && echo queries-ok && cat gpurun_out/queries_$TAG.err | grep -v amdgpu.ids || exit 1
R="--kernel-include-regex k_replay"
P="python scripts/prof_replay.py --docs 8192 --clean"
timeout -s KILL 150 rocprofv3 $R --pmc FETCH_SIZE -d gpurun_out/pmc_fetch$TAG -o f --output-format csv -- $P > gpurun_out/pmcf$TAG.log 2>&1 && echo fetch-ok && \
timeout -s KILL 150 rocprofv3 $R --pmc WRITE_SIZE -d gpurun_out/pmc_write$TAG -o w --output-format csv -- $P > gpurun_out/pmcw$TAG.log 2>&1 && echo write-ok && \
python scripts/traffic_from_pmc.py 8192 gpurun_out/traffic_k_replay.json k_replay $TAG "automerge-paper remote, one clean launch"
