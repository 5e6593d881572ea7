"""Timeline of the throughput pass from a rocprofv3 kernel trace of bench.py (--no-alt-order).

  python tools/timeline.py run_kernel_trace.csv [--steps K] [--warmup W] [--pass 0]

Prints, per step of the timed region, each kernel's start and end relative to the step's k_project
start (microseconds), so it shows which launch a step waits for: e.g. whether k_publish(k-2) starts
at k_voxel(k-2)'s end (the VoxelGrid on the critical path) or at k_lm(k-3)'s.  The throughput pass
is the first W + K launches of k_project (k_pw_scatter in the wide layout; bench.py's later passes
follow it).
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.trace)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        if name.startswith("__amd") or "rocprim" in name:
            continue
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    first = next(r[2] for r in rows if r[2] == "k_project" or r[2].startswith("k_pw_scatter"))
    proj = [r for r in rows if r[2] == first]  # the layout of the throughput pass (the first launches)
    per = a.steps + a.warmup
    starts = [p[0] for p in proj[:per + 1]]
    t_end = proj[per][0] if len(proj) > per else rows[-1][1]
    sel = [r for r in rows if starts[0] <= r[0] < t_end]
    for k in range(a.warmup, per):
        t0 = starts[k]
        t1 = starts[k + 1] if k + 1 < len(starts) else t_end
        print("step %2d  k_project at %.1f us, next step +%.1f us" % (k, (t0 - starts[0]) / 1e3, (t1 - t0) / 1e3))
        for s, e, n in sel:
            if t0 <= s < t1:
                print("   %-28s %8.1f .. %8.1f  (%7.1f)" % (n, (s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3))


if __name__ == "__main__":
    main()
