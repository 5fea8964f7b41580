set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=${DOCS:-256}
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES SQ_INSTS_BRANCH -d gpurun_out/pmc1 -o pmc1 --output-format csv -- python scripts/prof_replay.py --docs $D > gpurun_out/pmc1.log 2>&1 && echo pmc1-ok && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SMEM_NORM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA -d gpurun_out/pmc2 -o pmc2 --output-format csv -- python scripts/prof_replay.py --docs $D > gpurun_out/pmc2.log 2>&1 && echo pmc2-ok
echo done
