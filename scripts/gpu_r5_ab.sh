# Round 5 A/B (one box): clean k_replay launches of LIBS (lib:docs pairs) on automerge-paper
# remote (config 2) and, with C5=1, on config 5 (prof_replay.py --config5) at C5DOCS documents.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
B=text-crdt-rust_amd/build
for rep in 1 2; do
  for LD in ${LIBS}; do
    L=${LD%%:*}; D=${LD##*:}
    echo -n "ap $D $L "
    CRDT_GPU_LIB=$B/$L timeout -k 10 120 python scripts/prof_replay.py --docs $D --clean | tail -1 || exit 1
  done
done
if [ -n "$C5" ]; then
  for L in ${C5LIBS}; do
    echo -n "c5 ${C5DOCS:-4096} $L "
    CRDT_GPU_LIB=$B/$L timeout -k 10 300 python scripts/prof_replay.py --docs ${C5DOCS:-4096} --config5 --clean | tail -1 || exit 1
  done
fi
echo done
