# Publish timing at one build over the A/B workloads (scripts/gpu_ab_libs.sh with one library):
# profiles/r06_digest_on_request.txt and r06_publish_branchfree.txt were made this way.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_gpu_tests_v5.log 2>&1; rc=$?; echo tests rc=$rc; tail -2 gpurun_out/r06_gpu_tests_v4.log; [ $rc -le 1 ] || exit $rc
LIBS="text-crdt-rust_amd/build/libcrdt_gpu.so" WL="ap c4 c4b c5 j1" bash scripts/gpu_ab_libs.sh > gpurun_out/r06_publish_branchfree.txt 2>&1; rc=$?; cat gpurun_out/r06_publish_branchfree.txt; exit $rc
