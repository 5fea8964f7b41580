"""Per-launch HBM traffic of the clean (last) k_replay dispatch from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE; KB units).  gfx950 correction per MI355X_MICROARCH.md 'HBM': FETCH_SIZE
reports half of the bytes of wide coalesced reads -> doubled; WRITE_SIZE taken as is.  Writes
profiles/traffic_k_replay.json (read by bench.py)."""
import csv
import glob
import json
import sys

docs = int(sys.argv[1])
out = sys.argv[2] if len(sys.argv) > 2 else "profiles/traffic_k_replay.json"
kernel = sys.argv[3] if len(sys.argv) > 3 else "k_replay"
tag = sys.argv[4] if len(sys.argv) > 4 else ""
workload = sys.argv[5] if len(sys.argv) > 5 else "automerge-paper remote, one clean launch"


def last_value(pattern, counter):
    rows = []
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
                rows.append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    rows.sort()
    return rows[-1][1], len(rows)


fetch_kb, nf = last_value(f"gpurun_out/pmc_fetch{tag}/**/*counter_collection.csv", "FETCH_SIZE")
write_kb, nw = last_value(f"gpurun_out/pmc_write{tag}/**/*counter_collection.csv", "WRITE_SIZE")
res = {
    "kernel": kernel + "<32>", "docs": docs, "workload": workload,
    "fetch_size_kb": fetch_kb, "write_size_kb": write_kb,
    "hbm_bytes_per_launch": fetch_kb * 1024 * 2 + write_kb * 1024,
    "correction": "FETCH_SIZE x2 (gfx950 wide-read half count), WRITE_SIZE x1",
    "dispatches_seen": [nf, nw],
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
