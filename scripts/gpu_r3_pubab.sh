# A/B of the publish step: the library vs a diagnostic build without the digest's hashing.
set -o pipefail
cd $GRAFT_REPO_ROOT
B=text-crdt-rust_amd/build
for L in $B/libcrdt_gpu.so $B/libcrdt_gpu_ab.so $B/libcrdt_gpu.so $B/libcrdt_gpu_ab.so; do
  echo -n "ap8192 $(basename $L) "
  CRDT_GPU_LIB=$L timeout -k 10 120 python scripts/prof_replay.py --docs 8192 --clean | tail -1 || exit 1
done
