"""Per-kernel duration summary from a rocprofv3 kernel trace, split by launch size.

  python tools/trace_split.py run_kernel_trace.csv OUT.csv

bench.py launches every stage twice per step size: the timed steps as `--groups` slices (S/groups
scans per launch) and the per-stage timing pass as one launch of all S scans.  rocprofv3's
--stats file averages both; this split lets the full-S launches be compared with bench.py's
per-launch stage times (stages_ms, roofline.launch_ms).
"""
import collections
import csv
import sys


def main():
    src, out = sys.argv[1], sys.argv[2]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(src)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        if name.startswith("__amd"):
            continue
        grid = int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1)
        acc[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "workgroups", "calls", "avg_us", "min_us", "max_us"])
        for (name, grid), v in sorted(acc.items()):
            w.writerow([name, grid, len(v), round(sum(v) / len(v), 2), round(min(v), 2), round(max(v), 2)])
            print("%-24s wg=%6d calls=%3d avg %9.2f us  min %9.2f  max %9.2f" % (
                name, grid, len(v), sum(v) / len(v), min(v), max(v)))


if __name__ == "__main__":
    main()
