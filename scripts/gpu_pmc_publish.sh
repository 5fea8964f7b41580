# SQ instruction counters of k_publish (one pass, AP 8,192 documents, the last dispatch = the clean
# publish) and the publish time of two builds (LIBS) A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 150 rocprofv3 --kernel-include-regex k_publish --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES SQ_INSTS_BRANCH -d gpurun_out/pmc_pub -o pmcpub --output-format csv -- python scripts/prof_replay.py --docs 8192 --clean > gpurun_out/pmc_pub.log 2>&1 && echo pmc-ok
