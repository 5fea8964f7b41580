# Round-3 iteration: GPU tests, AP A/B (base vs new library, 8,192 docs), kevin at the reference
# size, then (EXTRA=1) the materialize HBM passes, config 5 at 4,096 docs and SQ passes over one
# clean config-5 launch.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-v3}
OLD=text-crdt-rust_amd/build/libcrdt_gpu_base.so
NEW=text-crdt-rust_amd/build/libcrdt_gpu.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1; rc=$?
tail -1 gpurun_out/gpu_tests_$TAG.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_$TAG.log | head -20; exit 1; }
for L in $OLD $NEW $OLD $NEW; do
  echo -n "ap8192 $(basename $L) "
  CRDT_GPU_LIB=$L timeout -k 10 120 python scripts/prof_replay.py --docs 8192 --clean | tail -1 || exit 1
done
timeout -k 10 300 python -u scripts/bench_kevin.py > gpurun_out/kevin_$TAG.json 2> gpurun_out/kevin_$TAG.err && echo kevin-ok || exit 1
timeout -k 10 300 python -u scripts/bench_queries.py > gpurun_out/queries_$TAG.json 2> gpurun_out/queries_$TAG.err && echo queries-ok || exit 1
[ -z "$PROF" ] || bash scripts/gpu_prof_paths.sh || exit 1
[ -n "$EXTRA" ] || exit 0
R="--kernel-include-regex k_replay"
P="python scripts/prof_replay.py --docs 1024 --clean --config5"
DOCS=8192 bash scripts/gpu_pmc_mat.sh && \
timeout -k 10 400 python -u scripts/bench_config5.py --docs 4096 > gpurun_out/c5_4096_$TAG.json 2> gpurun_out/c5_4096_$TAG.err && echo c5-ok && \
timeout -s KILL 150 rocprofv3 $R --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES SQ_INSTS_BRANCH -d gpurun_out/c5pmc1 -o pmc1 --output-format csv -- $P > gpurun_out/c5pmc1.log 2>&1 && echo pmc1-ok && \
timeout -s KILL 150 rocprofv3 $R --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA -d gpurun_out/c5pmc2 -o pmc2 --output-format csv -- $P > gpurun_out/c5pmc2.log 2>&1 && echo pmc2-ok
