set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES -d gpurun_out/pmc1 -o pmc1 --output-format csv -- python scripts/prof_replay.py --docs 64 > gpurun_out/pmc1.log 2>&1; echo "pmc1 $?"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_INST_CYCLES_VMEM_RD SQ_INSTS_FLAT SQ_BUSY_CYCLES -d gpurun_out/pmc2 -o pmc2 --output-format csv -- python scripts/prof_replay.py --docs 64 > gpurun_out/pmc2.log 2>&1; echo "pmc2 $?"
