# Round-end evidence in one call: GPU tests, smoke, the default bench line (CPU baseline included),
# a kernel-trace profile of the bench, then the PMC passes over one clean k_replay launch.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_final.sh && DOCS=${DOCS:-8192} bash scripts/gpu_pmc_all.sh
