"""Per-kernel duration summary from a rocprofv3 kernel trace of bench.py, split by bench phase.

  python tools/trace_split.py run_kernel_trace.csv OUT.csv [--steps K] [--warmup W]

bench.py runs the W + K steps twice: first the throughput pass (the timed region; with lag 1 and one
slice, k_publish / k_lm run on an internal stream concurrently with the next scan's front end, so a
kernel's duration there includes sharing the GPU), then the per-stage timing pass (one stream, stages
in sequence) whose last K launches give bench.py's stages_ms, and for k_project / k_fa_prep the
roofline pass (R back-to-back pairs, --roofline-reps) that gives roofline.launch_ms.  rocprofv3's
--stats file averages all passes; this split reports them apart, so the timing pass can be compared
with the bench line.  Launches are assigned to the passes in time order, per kernel (each kernel runs
once per step in each pass).
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("out")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--roofline-reps", type=int, default=20, help="bench.py's back-to-back roofline launches")
    a = ap.parse_args()
    per = a.steps + a.warmup
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(a.trace)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        if name.startswith("__amd") or "rocprim" in name:
            continue
        grid = int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1)
        acc[(name, grid)].append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    rows = []
    for (name, grid), v in sorted(acc.items()):
        v.sort()
        d = [x for _, x in v]
        if len(d) == 2 * per:  # throughput pass, then the timing pass (measured: its last K)
            parts = (("throughput_pass", d[a.warmup:per]), ("timing_pass", d[per + a.warmup:]))
        elif len(d) == 2 * per + a.roofline_reps:  # + the roofline pass (k_project / k_fa_prep)
            parts = (("throughput_pass", d[a.warmup:per]), ("timing_pass", d[per + a.warmup:2 * per]),
                     ("roofline_pass", d[2 * per:]))
        else:
            parts = (("all", d),)
        for phase, x in parts:
            rows.append([name, grid, phase, len(x), round(sum(x) / len(x), 2), round(min(x), 2), round(max(x), 2)])
    with open(a.out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "workgroups", "phase", "calls", "avg_us", "min_us", "max_us"])
        for r in rows:
            w.writerow(r)
            print("%-24s wg=%6d %-16s calls=%3d avg %9.2f us  min %9.2f  max %9.2f" % tuple(r))


if __name__ == "__main__":
    main()
