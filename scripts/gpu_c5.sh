# Config 5 lines on one box (round RN): the SURVEY §8(d) shape with one history per document (C++
# generator, no shared streams) at DOCS documents, then round 5's shape (8 config5_wire histories
# shared by every document) at 8,192 for a same-box A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=${V:-v1}
RN=${RN:-r06}
for D in ${DOCS:-8192}; do
  timeout -k 10 900 python -u scripts/bench_config5.py --docs $D > gpurun_out/${RN}_bench_config5_${D}_distinct_$V.json 2> gpurun_out/${RN}_bench_config5_${D}_distinct_$V.err || exit 1
  echo c5-$D-ok
done
if [ -z "$NOAB" ]; then
  timeout -k 10 600 python -u scripts/bench_config5.py --docs 8192 --gen py --distinct 8 --share > gpurun_out/${RN}_bench_config5_8192_shared8_$V.json 2> gpurun_out/${RN}_bench_config5_8192_shared8_$V.err || exit 1
  echo c5-shared8-ok
fi
