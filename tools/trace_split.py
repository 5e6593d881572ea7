"""Per-kernel duration summary from a rocprofv3 kernel trace of bench.py, split by bench pass.

  python tools/trace_split.py run_kernel_trace.csv OUT.csv [--steps K] [--warmup W] [--roofline-reps R]
      [--passes throughput,probe,timing]

Run bench.py under the profiler with --no-alt-order --roofline-streams 0 --no-c5, so every launch of a
given (kernel, grid) belongs to the one C3 batch.  bench.py then runs the W + K steps three times --
the throughput pass (the timed region), the probe pass (events around the projection and smoothness
stages: roofline.in_pipeline) and the per-stage timing pass (one stream, stages in sequence: stages_ms)
-- and then launches the roofline pair (projection kernels + k_fa_prep4) R times back to back
(roofline.launch_ms).  rocprofv3's --stats file averages all of them; this split reports them apart.
Launches are assigned to the passes in time order, per (kernel, grid): every kernel of the step runs
once per step in each pass (the pipeline is flushed at the end of each pass, so the lagged LM and
publish launches of a pass's scans stay inside it).  A (kernel, grid) whose count does not fit is
reported whole ("all").  The roofline rows' mean is what bench.py's roofline.launch_ms times with events.
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
    ap.add_argument("--passes", default="throughput,probe,timing")
    a = ap.parse_args()
    per = a.steps + a.warmup
    names = a.passes.split(",")
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(a.trace)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        if name.startswith("__amd") or "rocprim" in name:
            continue
        grid = int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1) * int(r.get("Grid_Size_Z", 1) or 1) // max(
            int(r["Workgroup_Size_X"]) * int(r.get("Workgroup_Size_Y", 1) or 1) * int(r.get("Workgroup_Size_Z", 1) or 1), 1)
        acc[(name, grid)].append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    rows = []
    pair = collections.defaultdict(float)
    for (name, grid), v in sorted(acc.items()):
        v.sort()
        d = [x for _, x in v]
        npass = len(names)
        if len(d) in (npass * per, npass * per + a.roofline_reps):
            parts = [("%s_pass" % nm, d[i * per + a.warmup:(i + 1) * per]) for i, nm in enumerate(names)]
            if len(d) > npass * per:
                parts.append(("roofline_pass", d[npass * per:]))
        else:
            parts = [("all", d)]
        for phase, x in parts:
            avg = sum(x) / len(x)
            rows.append([name, grid, phase, len(x), round(avg, 2), round(min(x), 2), round(max(x), 2)])
            if phase == "roofline_pass":
                pair["roofline_pass"] += avg
    with open(a.out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "workgroups", "phase", "calls", "avg_us", "min_us", "max_us"])
        for r in rows:
            w.writerow(r)
            print("%-28s wg=%7d %-16s calls=%3d avg %9.2f us  min %9.2f  max %9.2f" % tuple(r))
    if pair:
        print("roofline pair (sum of the roofline_pass means): %.2f us" % pair["roofline_pass"])


if __name__ == "__main__":
    main()
