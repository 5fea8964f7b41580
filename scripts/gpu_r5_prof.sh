# Round 5: s_memtime cycle attribution (diagnostic -DCRDT_PROF builds, made in-tree beforehand):
# per-path cycles of the forward / backward delete-run micro workloads and of AP, and apply_txn's
# parts on config 5 (-DCRDT_PROF_TXN).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/r5_prof_paths.txt
: > $OUT
for m in wire:data/micro/fd200.rtx.gz wire:data/micro/bs200.rtx.gz wire:data/micro/base.rtx.gz remote; do
  CRDT_GPU_LIB=text-crdt-rust_amd/build/libcrdt_gpu_prof.so timeout -k 10 200 python scripts/prof_paths.py 2048 $m >> $OUT 2>&1 || exit 1
done
PROF_TXN=1 CRDT_GPU_LIB=text-crdt-rust_amd/build/libcrdt_gpu_proftxn.so timeout -k 10 300 python scripts/prof_paths.py 4096 config5 >> $OUT 2>&1 || exit 1
cat $OUT
