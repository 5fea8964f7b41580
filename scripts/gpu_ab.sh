# A/B replay timing of builds on the same box (alternating, clean single-launch replays).
# usage: LIBS="a.so b.so" DOCS="2048 8192" bash scripts/gpu_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
LIBS=${LIBS:-"text-crdt-rust_amd/build/libcrdt_gpu_old.so text-crdt-rust_amd/build/libcrdt_gpu.so"}
for D in ${DOCS:-8192}; do
  for rep in 1 2; do
    for L in $LIBS; do
      echo -n "$D $(basename $L) "
      CRDT_GPU_LIB=$L timeout -k 10 120 python scripts/prof_replay.py --docs $D --clean ${ARGS:-} | tail -1 || exit 1
    done
  done
done
