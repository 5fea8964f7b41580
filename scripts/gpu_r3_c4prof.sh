# Config-4 path attribution (-DCRDT_PROF diagnostic build): where a generated op's cycles go.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CRDT_GPU_LIB=text-crdt-rust_amd/build/libcrdt_gpu_prof.so timeout -k 10 200 python scripts/prof_paths.py 8192 random > gpurun_out/prof_paths_c4.txt 2>&1; rc=$?
cat gpurun_out/prof_paths_c4.txt
exit $rc
