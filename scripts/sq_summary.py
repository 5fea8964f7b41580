"""Summarise the SQ PMC passes of ONE clean k_replay launch (scripts/gpu_pmc_all.sh) into a
profiles/ JSON: counter totals of the LAST dispatch of the kernel in each pass (the clean launch:
prof_replay.py --clean replays once more after the growth launches), instructions per op and per
wave, and issue utilisation.

usage: python scripts/sq_summary.py OUT.json DOCS OPS_PER_DOC TAG "WORKLOAD LABEL"
The workload label is required (it names what the passes ran: no default, so a record cannot
inherit another workload's label).  SQ counters on gfx950 count per wave-instruction;
SQ_WAVE_CYCLES / SQ_BUSY_CYCLES are in the SQ clock.  WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~=
WAVE_CYCLES (MI355X_MICROARCH.md, PMC slots).  `grid_waves` is the dispatch's grid / 64; SQ_WAVES
above it means waves were counted twice (e.g. a context save / restore of a long dispatch), which
the record then says."""
import csv
import os
import glob
import json
import sys

if len(sys.argv) != 6:
    sys.exit(__doc__)
out, docs, ops_doc, tag, workload = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5]
kernel = os.environ.get("SQ_KERNEL", "k_replay")
agg, meta, seen = {}, {}, {}
for f in sorted(glob.glob(f"gpurun_out/pmc[123]{tag}/**/*counter_collection.csv", recursive=True)):
    rows = [r for r in csv.DictReader(open(f)) if kernel in r.get("Kernel_Name", "")]
    ids = sorted({int(r["Dispatch_Id"]) for r in rows})
    last = ids[-1]
    seen[os.path.basename(os.path.dirname(f)) or f] = {"dispatches": len(ids), "last": last}
    for r in rows:
        if int(r["Dispatch_Id"]) == last:
            agg[r["Counter_Name"]] = agg.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            meta = {"vgpr": int(r["VGPR_Count"]), "sgpr": int(r["SGPR_Count"]), "lds_block": int(r["LDS_Block_Size"]),
                    "grid_threads": int(r["Grid_Size"]), "workgroup": int(r["Workgroup_Size"]),
                    "kernel_ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])}
ops = docs * ops_doc
grid_waves = meta.get("grid_threads", 64 * docs) // 64
waves = agg.get("SQ_WAVES", docs)
inst = {k: agg[k] for k in agg if k.startswith("SQ_INSTS_")}
total_inst = sum(agg.get(k, 0) for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                                         "SQ_INSTS_SMEM", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH", "SQ_INSTS_FLAT"))
wc = agg.get("SQ_WAVE_CYCLES", 0)
res = {
    "kernel": kernel + "<32>", "docs": docs, "ops_per_doc": ops_doc, "workload": workload,
    "dispatch": "the last dispatch of the kernel in each pass (the clean launch); earlier ones are the growth launches",
    "passes": seen, "launch": meta, "grid_waves": grid_waves, "sq_waves": waves,
    "waves_note": None if waves == grid_waves == docs else
    f"SQ_WAVES {waves:.0f} vs {grid_waves} waves in the grid ({docs} documents): waves counted more than once "
    f"(a long dispatch's context save / restore); per-wave ratios below use the grid's waves",
    "counters": agg,
    "per_op": {k.replace("SQ_INSTS_", "").lower(): v / ops for k, v in inst.items()},
    "instructions_per_op": total_inst / ops,
    "ratios": {
        "active_inst_any / wave_cycles": agg.get("SQ_ACTIVE_INST_ANY", 0) / wc if wc else None,
        "wait_any / wave_cycles": agg.get("SQ_WAIT_ANY", 0) / wc if wc else None,
        "wait_inst_any / wave_cycles": agg.get("SQ_WAIT_INST_ANY", 0) / wc if wc else None,
        "active_inst_sca / wave_cycles": agg.get("SQ_ACTIVE_INST_SCA", 0) / wc if wc else None,
        "active_inst_valu / wave_cycles": agg.get("SQ_ACTIVE_INST_VALU", 0) / wc if wc else None,
        "salu_insts / all_insts": agg.get("SQ_INSTS_SALU", 0) / total_inst if total_inst else None,
        "valu_insts / all_insts": agg.get("SQ_INSTS_VALU", 0) / total_inst if total_inst else None,
        "wave_cycles_per_wave": wc / grid_waves if grid_waves else None,
        "busy_cycles": agg.get("SQ_BUSY_CYCLES"),
    },
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
