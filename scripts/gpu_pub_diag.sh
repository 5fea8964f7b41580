# k_publish breakdown at 8,192 AP documents: wall time with and without the order->span index
# sweeps (PUB_NO_INDEX build), and one SQ PMC pass over the publish kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
D=${DOCS:-8192}
timeout -k 10 150 python scripts/pub_time.py $D > gpurun_out/pub_diag.txt 2>&1 && \
CRDT_GPU_LIB=text-crdt-rust_amd/build/libcrdt_gpu_noidx.so timeout -k 10 150 python scripts/pub_time.py $D >> gpurun_out/pub_diag.txt 2>&1 && \
timeout -s KILL 150 rocprofv3 --kernel-include-regex k_publish --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -d gpurun_out/pubpmc -o p --output-format csv -- python scripts/pub_time.py $D > gpurun_out/pubpmc.log 2>&1 && echo pmc-ok
