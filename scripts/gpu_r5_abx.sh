# Round 5: same-box A/B of LIBS on automerge-paper (8,192, two reps) and config 3 (65,536 mixed
# local documents, no fit), clean k_replay launches (prof_replay.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
B=text-crdt-rust_amd/build
for rep in 1 2; do
  for L in $LIBS; do
    echo -n "ap 8192 $L "; CRDT_GPU_LIB=$B/$L timeout -k 10 120 python scripts/prof_replay.py --docs 8192 --clean | tail -1 || exit 1
  done
done
for L in $LIBS; do
  echo -n "c3 65536 $L "; CRDT_GPU_LIB=$B/$L timeout -k 10 300 python scripts/prof_replay.py --docs 65536 --config3 --clean --no-fit | tail -1 || exit 1
done
