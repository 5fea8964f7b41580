# SQ counter passes (one per run, <= 8 SQ counters each) over ONE clean k_replay launch.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=${DOCS:-4096}
R="--kernel-include-regex k_replay"
timeout -s KILL 120 rocprofv3 $R --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES SQ_INSTS_BRANCH -d gpurun_out/pmc1 -o pmc1 --output-format csv -- python scripts/prof_replay.py --docs $D --clean > gpurun_out/pmc1.log 2>&1 && echo pmc1-ok && \
timeout -s KILL 120 rocprofv3 $R --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA -d gpurun_out/pmc2 -o pmc2 --output-format csv -- python scripts/prof_replay.py --docs $D --clean > gpurun_out/pmc2.log 2>&1 && echo pmc2-ok && \
timeout -s KILL 120 rocprofv3 $R --pmc SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT SQ_IFETCH -d gpurun_out/pmc3 -o pmc3 --output-format csv -- python scripts/prof_replay.py --docs $D --clean > gpurun_out/pmc3.log 2>&1 && echo pmc3-ok
echo done
