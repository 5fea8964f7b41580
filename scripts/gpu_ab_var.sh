# A/B replay of several builds on the same box (AP remote 8,192 docs; config 4 16,384 docs), then
# SQ passes of one clean config-4 launch of the current build.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
B=text-crdt-rust_amd/build
for rep in 1 2; do
  for L in ${LIBS:-r2 nogen nospan ""}; do
    F=$B/libcrdt_gpu${L:+_$L}.so
    echo -n "ap $L "; CRDT_GPU_LIB=$F timeout -k 10 120 python scripts/prof_replay.py --docs 8192 --clean | tail -1 || exit 1
  done
done
for L in ${LIBS:-r2 nogen nospan ""}; do
  F=$B/libcrdt_gpu${L:+_$L}.so
  echo -n "c4 $L "; CRDT_GPU_LIB=$F timeout -k 10 120 python scripts/prof_replay.py --docs 16384 --random 20000 --clean | tail -1 || exit 1
done
R="--kernel-include-regex k_replay"
P="python scripts/prof_replay.py --docs 16384 --random 20000 --clean"
timeout -s KILL 150 rocprofv3 $R --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES SQ_INSTS_BRANCH -d gpurun_out/pmc1_c4 -o pmc1 --output-format csv -- $P > gpurun_out/pmc1_c4.log 2>&1 && echo pmc1-ok && \
timeout -s KILL 150 rocprofv3 $R --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA -d gpurun_out/pmc2_c4 -o pmc2 --output-format csv -- $P > gpurun_out/pmc2_c4.log 2>&1 && echo pmc2-ok && \
timeout -s KILL 150 rocprofv3 $R --pmc SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT SQ_IFETCH -d gpurun_out/pmc3_c4 -o pmc3 --output-format csv -- $P > gpurun_out/pmc3_c4.log 2>&1 && echo pmc3-ok
echo done
