# Same-box A/B: recent-window agent-run search (seq_to_order) against the previous build, config 5
# with per-document histories.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
LIBS="text-crdt-rust_amd/build/libcrdt_gpu_base.so text-crdt-rust_amd/build/libcrdt_gpu.so" WL="${WL:-c5d}" bash scripts/gpu_ab_libs.sh > gpurun_out/r06_ab_arun_recent.txt 2>&1; rc=$?; cat gpurun_out/r06_ab_arun_recent.txt; exit $rc
