# SQ instruction counts of one clean k_replay launch per micro workload (data/micro, made by
# tests/golden/make_micro.py): base document P, and P + 20,000 ops of one shape.  Per-op costs =
# (X - base) / 20,000 (scripts/micro_summary.py).  One rocprofv3 --pmc run per workload.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/micro
D=${DOCS:-2048}
TAG=${TAG:-}
for W in ${WLS:-base typing jump10 jump1 bs10 del1 bs200 fd200}; do
  timeout -s KILL 120 rocprofv3 --kernel-include-regex k_replay --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_LDS SQ_WAVES SQ_INSTS_BRANCH \
    -d gpurun_out/micro/$W$TAG -o m --output-format csv -- python scripts/prof_replay.py --docs $D --clean --wire data/micro/$W.rtx.gz > gpurun_out/micro/$W$TAG.log 2>&1 || exit 1
  echo $W-ok
done
timeout -s KILL 120 rocprofv3 --kernel-include-regex k_replay --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_LDS SQ_WAVES SQ_INSTS_BRANCH \
  -d gpurun_out/micro/ap$TAG -o m --output-format csv -- python scripts/prof_replay.py --docs $D --clean > gpurun_out/micro/ap$TAG.log 2>&1 || exit 1
python scripts/micro_summary.py $D "$TAG" | tee gpurun_out/micro/summary$TAG.txt
