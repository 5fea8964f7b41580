# Per-path attribution of k_replay with the diagnostic builds (built in-tree beforehand):
# libcrdt_gpu_prof.so (-DCRDT_PROF: cycles / calls / txns per fast path, delete-call parts) and
# libcrdt_gpu_profloop.so (-DCRDT_PROF -DCRDT_PROF_LOOP: parts of the delete runs' leaf-split loop).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B=text-crdt-rust_amd/build
OUT=gpurun_out/prof_paths_${TAG:-r4}.txt
: > $OUT
if [ -f $B/libcrdt_gpu_prof.so ]; then
  CRDT_GPU_LIB=$B/libcrdt_gpu_prof.so timeout -k 10 200 python scripts/prof_paths.py 4096 >> $OUT 2>&1 || exit 1
fi
if [ -f $B/libcrdt_gpu_profloop.so ]; then
  PROF_LOOP=1 CRDT_GPU_LIB=$B/libcrdt_gpu_profloop.so timeout -k 10 200 python scripts/prof_paths.py 4096 >> $OUT 2>&1 || exit 1
fi
cat $OUT
