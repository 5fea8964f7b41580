# PMC passes over ONE clean k_replay launch (config 2, DOCS docs): three SQ passes (<= 8 SQ
# counters each) and the two HBM passes (FETCH_SIZE, WRITE_SIZE in separate runs), each its own
# rocprofv3 --pmc run with only the kernel trace (no runtime / sys trace).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
D=${DOCS:-4096}
TAG=${TAG:-}
R=${R:-"--kernel-include-regex k_replay"}
P=${P:-"python scripts/prof_replay.py --docs $D --clean"}
PT=${PT:-150}  # seconds per pass
timeout -s KILL $PT rocprofv3 $R --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES SQ_INSTS_BRANCH -d gpurun_out/pmc1$TAG -o pmc1 --output-format csv -- $P > gpurun_out/pmc1$TAG.log 2>&1 && echo pmc1-ok && \
timeout -s KILL $PT rocprofv3 $R --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA -d gpurun_out/pmc2$TAG -o pmc2 --output-format csv -- $P > gpurun_out/pmc2$TAG.log 2>&1 && echo pmc2-ok && \
timeout -s KILL $PT rocprofv3 $R --pmc SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT SQ_IFETCH -d gpurun_out/pmc3$TAG -o pmc3 --output-format csv -- $P > gpurun_out/pmc3$TAG.log 2>&1 && echo pmc3-ok && \
timeout -s KILL $PT rocprofv3 $R --pmc FETCH_SIZE -d gpurun_out/pmc_fetch$TAG -o f --output-format csv -- $P > gpurun_out/pmcf$TAG.log 2>&1 && echo fetch-ok && \
timeout -s KILL $PT rocprofv3 $R --pmc WRITE_SIZE -d gpurun_out/pmc_write$TAG -o w --output-format csv -- $P > gpurun_out/pmcw$TAG.log 2>&1 && echo write-ok || exit 1
echo done
