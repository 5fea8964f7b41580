"""Per-op instruction costs of each micro workload (scripts/gpu_micro_paths.sh): SQ counters of the
last k_replay dispatch, (workload - base) / 20,000 ops, per wave (= per document)."""
import csv
import glob
import sys

docs = int(sys.argv[1])
tag = sys.argv[2] if len(sys.argv) > 2 else ""
N = 20000
KEYS = ("SQ_INSTS_SALU", "SQ_INSTS_VALU", "SQ_INSTS_BRANCH", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_FLAT")


def load(w):
    agg, ns = {}, 0
    for f in glob.glob(f"gpurun_out/micro/{w}{tag}/**/*counter_collection.csv", recursive=True):
        rows = [r for r in csv.DictReader(open(f)) if "k_replay" in r.get("Kernel_Name", "")]
        last = max(int(r["Dispatch_Id"]) for r in rows)
        for r in rows:
            if int(r["Dispatch_Id"]) == last:
                agg[r["Counter_Name"]] = agg.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return agg, ns


base, bns = load("base")
print(f"{'workload':8s} {'all':>7s} " + " ".join(f"{k[9:].lower():>8s}" for k in KEYS) + "   ns/op(launch)")
b = {k: base.get(k, 0) / docs for k in KEYS}
print(f"{'base/op':8s} {sum(b.values()) / 50000:7.1f} " + " ".join(f"{b[k] / 50000:8.1f}" for k in KEYS) + f"   {bns / 50000:.1f}")
for w in ("typing", "jump10", "jump1", "bs10", "del1", "bs200", "fd200"):
    a, ns = load(w)
    d = {k: (a.get(k, 0) - base.get(k, 0)) / docs / N for k in KEYS}
    print(f"{w:8s} {sum(d.values()):7.1f} " + " ".join(f"{d[k]:8.1f}" for k in KEYS) + f"   {(ns - bns) / N:.1f}")
a, ns = load("ap")
if a:  # automerge-paper remote, whole replay (259,778 ops), no base subtracted
    d = {k: a.get(k, 0) / docs / 259778 for k in KEYS}
    print(f"{'ap':8s} {sum(d.values()):7.1f} " + " ".join(f"{d[k]:8.1f}" for k in KEYS) + f"   {ns / 259778:.1f}")
