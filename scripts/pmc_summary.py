"""Summarise rocprofv3 PMC csv files for the replay kernel: per-wave and per-op figures."""
import csv, glob, sys
ops = int(sys.argv[1]) if len(sys.argv) > 1 else 259778
agg = {}
for f in sorted(glob.glob("gpurun_out/pmc*/pmc*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "k_replay" not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]] = agg.get(r["Counter_Name"], 0) + float(r["Counter_Value"])
w = agg.get("SQ_WAVES", 1)
for k in sorted(agg):
    print(f"{k:28s} total {agg[k]:.4g}  per-wave {agg[k]/w:.4g}  per-op {agg[k]/w/ops:.2f}")
