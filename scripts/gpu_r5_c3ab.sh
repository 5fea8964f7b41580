# Round 5: config 3 (65,536 mixed local documents, shared record streams) A/B of LIBS on one box,
# clean k_replay launches (prof_replay.py --config3), then the config-3 line of the product.
set -o pipefail
cd $GRAFT_REPO_ROOT
B=text-crdt-rust_amd/build
for rep in 1 2; do
  for L in $LIBS; do
    echo -n "c3 65536 $L "; CRDT_GPU_LIB=$B/$L timeout -k 10 300 python scripts/prof_replay.py --docs 65536 --config3 --clean | tail -1 || exit 1
  done
done
