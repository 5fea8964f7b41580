# Memory latency / translation counters of ONE clean k_replay launch at two occupancies.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for D in 2048 8192; do
timeout -s KILL 150 rocprofv3 --kernel-include-regex k_replay --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum \
  -d gpurun_out/pmc_lat_a$D -o a --output-format csv -- python scripts/prof_replay.py --docs $D --clean > gpurun_out/pmc_lat_a$D.log 2>&1 && echo a$D-ok || exit 1
timeout -s KILL 150 rocprofv3 --kernel-include-regex k_replay --pmc TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_STALL_MULTI_MISS_sum \
  -d gpurun_out/pmc_lat_b$D -o b --output-format csv -- python scripts/prof_replay.py --docs $D --clean > gpurun_out/pmc_lat_b$D.log 2>&1 && echo b$D-ok || exit 1
done
python - <<'PY'
import csv, glob
for D in (2048, 8192):
    agg = {}
    for f in glob.glob(f"gpurun_out/pmc_lat_[ab]{D}/**/*counter_collection.csv", recursive=True):
        rows = [r for r in csv.DictReader(open(f)) if "k_replay" in r.get("Kernel_Name", "")]
        last = max(int(r["Dispatch_Id"]) for r in rows)
        for r in rows:
            if int(r["Dispatch_Id"]) == last:
                agg[r["Counter_Name"]] = agg.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                agg["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    print(D, agg)
    g = lambda k: agg.get(k, agg.get(k.replace("_sum", ""), 0.0))
    m, h = g("TCP_UTCL1_TRANSLATION_MISS_sum"), g("TCP_UTCL1_TRANSLATION_HIT_sum")
    print(D, "utcl1 miss rate", m / max(m + h, 1), "read lat", g("TCP_TCC_READ_REQ_LATENCY_sum") / max(g("TCP_TCC_READ_REQ_sum"), 1),
          "write lat", g("TCP_TCC_WRITE_REQ_LATENCY_sum") / max(g("TCP_TCC_WRITE_REQ_sum"), 1))
PY
