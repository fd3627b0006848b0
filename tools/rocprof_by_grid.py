"""Per-(kernel, grid size) duration statistics from a rocprofv3 --kernel-trace CSV, so that a
kernel launched at several sizes (bench.py's one-batch forward() references: 32 frames; the
pipeline's group launches: G * 32 frames) can be compared with the in-bench HIP-event mean of
the launches of one size.

usage: python tools/rocprof_by_grid.py <kernel_trace.csv> <out.csv>"""
import csv
import sys
from collections import defaultdict


def main(src, out):
    acc = defaultdict(list)
    for r in csv.DictReader(open(src)):
        name = r["Kernel_Name"]
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        acc[(name, grid, int(r["Stream_Id"]))].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    rows = sorted(acc.items(), key=lambda kv: -sum(kv[1]))
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Grid_Size", "Stream_Id", "Calls", "AverageNs", "MinNs", "MaxNs", "TotalDurationNs"])
        for (name, grid, sid), d in rows:
            w.writerow([name, grid, sid, len(d), sum(d) / len(d), min(d), max(d), sum(d)])
    for (name, grid, sid), d in rows[:14]:
        print(f"{name[:70]:70s} grid {grid:>10d} stream {sid:>2d} calls {len(d):4d} avg {sum(d) / len(d) / 1e6:8.3f} ms")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
