# Instruction-cache counters of ONE clean k_replay launch (config 2, DOCS docs).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
D=${DOCS:-8192}
TAG=${TAG:-}
rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
timeout -s KILL 150 rocprofv3 --kernel-include-regex k_replay --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAVES SQ_IFETCH SQ_WAIT_INST_ANY \
  -d gpurun_out/pmc_ic$TAG -o ic --output-format csv -- python scripts/prof_replay.py --docs $D --clean > gpurun_out/pmc_ic$TAG.log 2>&1 && echo ic-ok
python - <<PY
import csv, glob
agg = {}
for f in glob.glob("gpurun_out/pmc_ic$TAG/**/*counter_collection.csv", recursive=True):
    rows = [r for r in csv.DictReader(open(f)) if "k_replay" in r.get("Kernel_Name", "")]
    last = max(int(r["Dispatch_Id"]) for r in rows)
    for r in rows:
        if int(r["Dispatch_Id"]) == last:
            agg[r["Counter_Name"]] = agg.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
print(agg)
h, m = agg.get("SQC_ICACHE_HITS", 0), agg.get("SQC_ICACHE_MISSES", 0)
print("icache miss rate", m / max(h + m, 1))
PY
grep -o "SQC_[A-Z_0-9]*" gpurun_out/counters.txt | sort -u | tr '\n' ' '
