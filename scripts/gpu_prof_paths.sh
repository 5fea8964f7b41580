# Per-path attribution of k_replay (diagnostic -DCRDT_PROF build, built in-tree beforehand).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CRDT_GPU_LIB=text-crdt-rust_amd/build/libcrdt_gpu_prof.so timeout -k 10 200 python scripts/prof_paths.py 4096 > gpurun_out/prof_paths.txt 2>&1 && \
CRDT_GPU_LIB=text-crdt-rust_amd/build/libcrdt_gpu_prof.so timeout -k 10 200 python scripts/prof_paths.py 4096 local >> gpurun_out/prof_paths.txt 2>&1
cat gpurun_out/prof_paths.txt
