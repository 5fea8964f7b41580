# Same-box A/B of two builds (LIBS), alternating, on the workloads in WL (as gpu_ab_env.sh):
# clean single-launch replays (scripts/prof_replay.py), digests printed for equality.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
LIBS=${LIBS:-"text-crdt-rust_amd/build/libcrdt_gpu.so text-crdt-rust_amd/build/libcrdt_gpu_nt.so"}
for w in ${WL:-ap c4}; do
  case $w in
    ap) ARGS="--docs 8192 --clean";;
    c4) ARGS="--docs 16384 --random 20000 --clean";;
    c4b) ARGS="--docs 125000 --random 20000 --clean";;
    apl) ARGS="--docs 8192 --local --clean";;
    c3) ARGS="--docs 65536 --config3 --clean --no-fit";;
    c5) ARGS="--docs 4096 --config5 --clean";;
    c5d) ARGS="";;  # config 5 at 8,192 documents with their own histories (scripts/bench_config5.py)
    j1) ARGS="--docs 2048 --clean --wire data/micro/jump1.rtx.gz";;
    d1) ARGS="--docs 2048 --clean --wire data/micro/del1.rtx.gz";;
  esac
  for rep in 1 2; do
    for L in $LIBS; do
      echo -n "$w $(basename $L) "
      if [ $w = c5d ]; then
        CRDT_GPU_LIB=$L timeout -k 10 400 python scripts/bench_config5.py --docs 8192 --steps 2 --no-cpu --check-docs 8 | python -c "
import json, sys; d = json.loads(sys.stdin.read().strip().splitlines()[-1])
print('k_replay_ms %.1f publish_ms %.1f value %.4g parity %s' % (d['kernels_ms']['k_replay'], d['kernels_ms']['k_publish'], d['value'], d['parity_ok']))" || exit 1
      else
        CRDT_GPU_LIB=$L timeout -k 10 300 python scripts/prof_replay.py $ARGS | tail -1 || exit 1
      fi
    done
  done
done
