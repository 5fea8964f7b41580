# Frontier heads in context lanes: the new GPU tests (wide frontiers then local txns, per-document
# config-5 histories), then a same-box A/B against the previous build on config 5 (per-document
# histories) and automerge-paper.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "wide_frontier or per_document or config5" > gpurun_out/r06_gpu_tests_frontier.log 2>&1 && echo tests-ok || { tail -30 gpurun_out/r06_gpu_tests_frontier.log; exit 1; }
LIBS="text-crdt-rust_amd/build/libcrdt_gpu_base.so text-crdt-rust_amd/build/libcrdt_gpu.so" WL="${WL:-c5d ap}" bash scripts/gpu_ab_libs.sh > gpurun_out/r06_ab_frontier_lanes.txt 2>&1; rc=$?; cat gpurun_out/r06_ab_frontier_lanes.txt; exit $rc
