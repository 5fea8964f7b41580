# apply_txn's cycles by part on config 5 (diagnostic -DCRDT_PROF -DCRDT_PROF_TXN build, in-tree beforehand)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/prof_c5_${TAG:-r4}.txt
PROF_TXN=1 CRDT_GPU_LIB=text-crdt-rust_amd/build/libcrdt_gpu_proftxn.so timeout -k 10 300 python scripts/prof_paths.py ${DOCS:-1024} config5 > $OUT 2>&1 || exit 1
if [ -f text-crdt-rust_amd/build/libcrdt_gpu_proftxn2.so ]; then
  PROF_TXN2=1 CRDT_GPU_LIB=text-crdt-rust_amd/build/libcrdt_gpu_proftxn2.so timeout -k 10 300 python scripts/prof_paths.py ${DOCS:-1024} config5 >> $OUT 2>&1 || exit 1
fi
if [ -f text-crdt-rust_amd/build/libcrdt_gpu_prof.so ]; then
  KEVIN_OPS=5000000 CRDT_GPU_LIB=text-crdt-rust_amd/build/libcrdt_gpu_prof.so timeout -k 10 300 python scripts/prof_paths.py 4 kevin >> $OUT 2>&1 || exit 1
fi
cat $OUT
