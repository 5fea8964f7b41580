"""Per-launch HBM traffic of the clean (LAST) dispatch of a kernel from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE; KB units).  gfx950 correction per MI355X_MICROARCH.md 'HBM': FETCH_SIZE
reports half of the bytes of wide coalesced reads -> doubled; WRITE_SIZE taken as is.

usage: python scripts/traffic_from_pmc.py DOCS OUT.json KERNEL TAG "WORKLOAD LABEL"
The workload label is required (bench.py reads a traffic file only when its label and document
count match the line it reports).  `dispatches_seen` counts the kernel's dispatches in each pass:
prof_replay.py --clean runs the growth launches first, then ONE clean launch, which is the last."""
import csv
import glob
import json
import sys

if len(sys.argv) != 6:
    sys.exit(__doc__)
docs, out, kernel, tag, workload = int(sys.argv[1]), sys.argv[2], sys.argv[3], sys.argv[4], sys.argv[5]


def last_value(pattern, counter):
    rows = []
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
                rows.append((int(r["Dispatch_Id"]), float(r["Counter_Value"]), int(r["Grid_Size"]) // 64))
    rows.sort()
    return rows[-1], len(rows)


(fid, fetch_kb, fwaves), nf = last_value(f"gpurun_out/pmc_fetch{tag}/**/*counter_collection.csv", "FETCH_SIZE")
(wid, write_kb, wwaves), nw = last_value(f"gpurun_out/pmc_write{tag}/**/*counter_collection.csv", "WRITE_SIZE")
assert fwaves == wwaves == docs, (fwaves, wwaves, docs)
res = {
    "kernel": kernel + "<32>", "docs": docs, "workload": workload,
    "fetch_size_kb": fetch_kb, "write_size_kb": write_kb,
    "fetch_bytes": fetch_kb * 1024 * 2, "write_bytes": write_kb * 1024,
    "hbm_bytes_per_launch": fetch_kb * 1024 * 2 + write_kb * 1024,
    "correction": "FETCH_SIZE x2 (gfx950 wide-read half count), WRITE_SIZE x1",
    "dispatch": "the last dispatch of the kernel in each pass (the clean launch)", "grid_waves": fwaves,
    "dispatches_seen": [nf, nw],
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
