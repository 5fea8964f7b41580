"""Per-dispatch durations of the k_replay / k_publish instances in a rocprofv3 kernel trace, grouped by
kernel and grid size, so that the trace's average for the bench's own launches (8,192 documents =
524,288 threads) can be set beside the bench line's HIP-event `kernel_ms` (the stats file's
per-kernel average mixes the config-2, stated-size and corpus launches).
usage: python scripts/ktrace_dispatches.py gpurun_out/ktrace/ktrace_kernel_trace.csv"""
import collections
import csv
import sys

groups = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "k_replay" not in n and "k_publish" not in n:
        continue
    name = n.split("(")[0].replace("void ", "")
    groups[(name, int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
print(f"{'kernel':32s} {'threads':>9s} {'docs':>7s} {'launches':>8s} {'avg ms':>9s} {'min ms':>9s} {'max ms':>9s}")
for (name, g), v in sorted(groups.items()):
    print(f"{name:32s} {g:9d} {g // 64:7d} {len(v):8d} {sum(v) / len(v):9.3f} {min(v):9.3f} {max(v):9.3f}")
