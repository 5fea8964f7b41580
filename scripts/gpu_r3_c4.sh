# Config 4 (generated random edits) diagnostics: path attribution (-DCRDT_PROF build), then the SQ
# and HBM PMC passes of one clean k_replay launch over 16,384 documents x 20,000 ops.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
CRDT_GPU_LIB=text-crdt-rust_amd/build/libcrdt_gpu_prof.so timeout -k 10 200 python scripts/prof_paths.py 8192 random > gpurun_out/prof_paths_c4.txt 2>&1 && cat gpurun_out/prof_paths_c4.txt && \
DOCS=16384 TAG=c4 P="python scripts/prof_replay.py --docs 16384 --random 20000 --clean" bash scripts/gpu_pmc_all.sh && \
python scripts/sq_summary.py gpurun_out/sq_c4.json 16384 20000 c4 && cat gpurun_out/sq_c4.json && \
python scripts/traffic_from_pmc.py 16384 gpurun_out/traffic_c4.json k_replay c4 "config4 16384 docs x 20000 generated ops, one clean launch" && cat gpurun_out/traffic_c4.json
