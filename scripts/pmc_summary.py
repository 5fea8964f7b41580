"""Summarise rocprofv3 PMC csv files for the LAST k_replay dispatch of each pass (the clean
single launch of prof_replay.py --clean): totals, per wave and per op."""
import csv, glob, sys
ops = int(sys.argv[1]) if len(sys.argv) > 1 else 259778
agg = {}
for f in sorted(glob.glob("gpurun_out/pmc*/**/*counter_collection.csv", recursive=True)):
    last = {}
    for r in csv.DictReader(open(f)):
        if not r.get("Kernel_Name") or "k_replay" not in r["Kernel_Name"]:
            continue
        key = r["Counter_Name"]
        did = int(r["Dispatch_Id"])
        if key not in last or did > last[key][0]:
            last[key] = (did, 0.0)
        if did == last[key][0]:
            last[key] = (did, last[key][1] + float(r["Counter_Value"]))
    for k, (_, v) in last.items():
        agg[k] = v
w = agg.get("SQ_WAVES", 1)
for k in sorted(agg):
    print(f"{k:28s} total {agg[k]:.4g}  per-wave {agg[k]/w:.4g}  per-op {agg[k]/w/ops:.2f}")
