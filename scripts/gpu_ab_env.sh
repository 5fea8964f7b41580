# Same-box A/B of one library under two environments (ENV_A vs ENV_B, e.g. CRDT_NO_SHAPES=1 vs
# nothing), alternating, on the workloads in WL (ap = automerge-paper remote at 8,192 documents,
# c4 = config 4 generated ops at 16,384, c3 = config 3 local corpus at 65,536, c5 = config 5 at
# 4,096): clean single-launch replays (scripts/prof_replay.py), digests printed for equality.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ENV_A=${ENV_A:-CRDT_NO_SHAPES=1}
ENV_B=${ENV_B:-CRDT_NO_SHAPES=0}
for w in ${WL:-ap c4}; do
  case $w in
    ap) ARGS="--docs 8192 --clean";;
    c4) ARGS="--docs 16384 --random 20000 --clean";;
    c3) ARGS="--docs 65536 --config3 --clean --no-fit";;
    c5) ARGS="--docs 4096 --config5 --clean";;
    j1) ARGS="--docs 2048 --clean --wire data/micro/jump1.rtx.gz";;
    d1) ARGS="--docs 2048 --clean --wire data/micro/del1.rtx.gz";;
  esac
  for rep in 1 2; do
    for E in "$ENV_A" "$ENV_B"; do
      echo -n "$w [$E] "
      env $E timeout -k 10 300 python scripts/prof_replay.py $ARGS | tail -1 || exit 1
    done
  done
done
