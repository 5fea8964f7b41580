# Round 3: kevin at the reference size (512 docs), replicated-staging interning both ways, the
# k_materialize HBM passes on the bench's per-document content, config 5 at 4,096 docs, and SQ
# passes over one clean config-5 launch (1,024 docs).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-v2}
R="--kernel-include-regex k_replay"
P="python scripts/prof_replay.py --docs 1024 --clean --config5"


DOCS=8192 bash scripts/gpu_pmc_mat.sh && \
timeout -k 10 400 python -u scripts/bench_config5.py --docs 4096 > gpurun_out/c5_4096_$TAG.json 2> gpurun_out/c5_4096_$TAG.err && echo c5-ok && \
timeout -s KILL 150 rocprofv3 $R --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES SQ_INSTS_BRANCH -d gpurun_out/c5pmc1 -o pmc1 --output-format csv -- $P > gpurun_out/c5pmc1.log 2>&1 && echo pmc1-ok && \
timeout -s KILL 150 rocprofv3 $R --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA -d gpurun_out/c5pmc2 -o pmc2 --output-format csv -- $P > gpurun_out/c5pmc2.log 2>&1 && echo pmc2-ok
