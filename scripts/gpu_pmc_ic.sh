set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
grep -o "SQC_[A-Z_0-9]*\|SQ_IFETCH[A-Z_]*\|SQ_INST_LEVEL[A-Z_]*\|SQ_WAIT[A-Z_]*\|SQ_LEVEL[A-Z_]*" gpurun_out/counters.txt | sort -u > gpurun_out/counters_sq.txt || true
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAVES -d gpurun_out/pmc4 -o pmc4 --output-format csv -- python scripts/prof_replay.py --docs 256 > gpurun_out/pmc4.log 2>&1 && echo pmc4-ok
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INST_LEVEL_VMEM SQ_WAVES -d gpurun_out/pmc5 -o pmc5 --output-format csv -- python scripts/prof_replay.py --docs 256 > gpurun_out/pmc5.log 2>&1 && echo pmc5-ok
echo done
