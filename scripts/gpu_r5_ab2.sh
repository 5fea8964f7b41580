# Round 5 A/B of LIBS on automerge-paper (8,192 documents) and on the backspace / forward-delete
# micro workloads (2,048 documents), clean k_replay launches, same box.
set -o pipefail
cd $GRAFT_REPO_ROOT
B=text-crdt-rust_amd/build
for rep in 1 2; do
  for L in $LIBS; do
    echo -n "ap 8192 $L "; CRDT_GPU_LIB=$B/$L timeout -k 10 120 python scripts/prof_replay.py --docs 8192 --clean | tail -1 || exit 1
  done
done
for w in bs200 fd200 bs10; do
  for L in $LIBS; do
    echo -n "$w 2048 $L "; CRDT_GPU_LIB=$B/$L timeout -k 10 120 python scripts/prof_replay.py --docs 2048 --clean --wire data/micro/$w.rtx.gz | tail -1 || exit 1
  done
done
