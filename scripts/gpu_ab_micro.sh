# A/B of two builds on the same box: clean replay time at DOCS docs (AP remote) and the SQ
# instruction counts per op of the B build's AP replay (micro-path harness row "ap").
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/micro
A=${A:-text-crdt-rust_amd/build/libcrdt_gpu_old.so}
B=${B:-text-crdt-rust_amd/build/libcrdt_gpu.so}
LIBS="$A $B" DOCS=${DOCS:-8192} bash scripts/gpu_ab.sh || exit 1
for L in $A $B; do
  T=$(basename $L .so)
  CRDT_GPU_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-include-regex k_replay --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_LDS SQ_WAVES SQ_INSTS_BRANCH \
    -d gpurun_out/micro/ap_$T -o m --output-format csv -- python scripts/prof_replay.py --docs 2048 --clean > gpurun_out/micro/ap_$T.log 2>&1 || exit 1
done
python - <<PY
import csv, glob
for t in ("$(basename $A .so)", "$(basename $B .so)"):
    agg = {}
    for f in glob.glob(f"gpurun_out/micro/ap_{t}/**/*counter_collection.csv", recursive=True):
        rows = [r for r in csv.DictReader(open(f)) if "k_replay" in r.get("Kernel_Name", "")]
        last = max(int(r["Dispatch_Id"]) for r in rows)
        for r in rows:
            if int(r["Dispatch_Id"]) == last:
                agg[r["Counter_Name"]] = agg.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ops = 2048 * 259778
    print(t, {k[9:].lower(): round(v / ops, 2) for k, v in agg.items() if k.startswith("SQ_INSTS")})
PY
