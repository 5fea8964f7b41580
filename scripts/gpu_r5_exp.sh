# Round 5 experiments: same-box A/B of clean k_replay launches (8,192 AP documents) for the
# libraries in LIBS, plus a WRITE_SIZE and a FETCH_SIZE pass of each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
LIBS=${LIBS:-"text-crdt-rust_amd/build/libcrdt_gpu_base.so text-crdt-rust_amd/build/libcrdt_gpu.so"}
D=${DOCS:-8192}
for rep in 1 2; do
  for L in $LIBS; do
    echo -n "$D $(basename $L) "
    CRDT_GPU_LIB=$L timeout -k 10 120 python scripts/prof_replay.py --docs $D --clean ${ARGS:-} | tail -1 || exit 1
  done
done
if [ -n "$PMC" ]; then
  for L in $LIBS; do
    T=$(basename $L .so)
    CRDT_GPU_LIB=$L timeout -s KILL 150 rocprofv3 --kernel-include-regex k_replay --pmc WRITE_SIZE -d gpurun_out/pmcw_$T -o w --output-format csv -- python scripts/prof_replay.py --docs $D --clean ${ARGS:-} > gpurun_out/pmcw_$T.log 2>&1 || exit 1
    CRDT_GPU_LIB=$L timeout -s KILL 150 rocprofv3 --kernel-include-regex k_replay --pmc FETCH_SIZE -d gpurun_out/pmcf_$T -o f --output-format csv -- python scripts/prof_replay.py --docs $D --clean ${ARGS:-} > gpurun_out/pmcf_$T.log 2>&1 || exit 1
    python - <<PY
import csv, glob
def last(pat, c):
    rows = []
    for f in glob.glob(pat, recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_replay" in r["Kernel_Name"] and r["Counter_Name"] == c:
                rows.append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    return sorted(rows)[-1][1]
w = last("gpurun_out/pmcw_$T/**/*counter_collection.csv", "WRITE_SIZE")
f = last("gpurun_out/pmcf_$T/**/*counter_collection.csv", "FETCH_SIZE")
print("$T", "write GB", round(w * 1024 / 1e9, 2), "fetch x2 GB", round(f * 2048 / 1e9, 2))
PY
  done
fi
echo done
