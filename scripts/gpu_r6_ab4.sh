# Same-box A/B: integrate's concurrent-sibling shortcut (no origin_left lookup when it is the new
# item's own) against the previous build: config 5 per-document histories and automerge-paper.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
LIBS="text-crdt-rust_amd/build/libcrdt_gpu_base.so text-crdt-rust_amd/build/libcrdt_gpu.so" WL="${WL:-c5d ap}" bash scripts/gpu_ab_libs.sh > gpurun_out/r06_ab_sibling_shortcut.txt 2>&1; rc=$?; cat gpurun_out/r06_ab_sibling_shortcut.txt; exit $rc
