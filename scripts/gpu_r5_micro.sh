# Round 5: micro-path SQ counts (scripts/gpu_micro_paths.sh) for WLS, then the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
WLS=${WLS:-"base bs200 fd200"} TAG=${TAG:-_r5b} bash scripts/gpu_micro_paths.sh || exit 1
