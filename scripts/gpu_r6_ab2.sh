# Local-only shape instance: GPU tests, then the same-box A/B against the previous build
# (scripts/gpu_ab_libs.sh) -> profiles/r06_ab_local_shape.txt.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_gpu_tests_v3.log 2>&1; rc=$?; echo tests rc=$rc; tail -2 gpurun_out/r06_gpu_tests_v3.log; [ $rc -le 1 ] || exit $rc
LIBS="text-crdt-rust_amd/build/libcrdt_gpu_base.so text-crdt-rust_amd/build/libcrdt_gpu.so" WL="apl c3 ap" bash scripts/gpu_ab_libs.sh > gpurun_out/r06_ab_local_shape.txt 2>&1; rc=$?; cat gpurun_out/r06_ab_local_shape.txt; exit $rc
