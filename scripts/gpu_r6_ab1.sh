# Round-6 shape instances: GPU tests, then the same-box A/B of CRDT_NO_SHAPES=1 (every stream in the
# general instance) against the shape instances (scripts/gpu_ab_env.sh) -> profiles/r06_ab_shapes.txt.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_gpu_tests_v2.log 2>&1; rc=$?; echo tests rc=$rc; tail -2 gpurun_out/r06_gpu_tests_v2.log; [ $rc -le 1 ] || exit $rc
WL="ap c4 j1 d1" bash scripts/gpu_ab_env.sh > gpurun_out/r06_ab_shapes.txt 2>&1; rc=$?; cat gpurun_out/r06_ab_shapes.txt; exit $rc
