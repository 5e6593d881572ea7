"""Summarise rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE, collected in separate runs as
MI355X_MICROARCH.md prescribes) into per-kernel means per dispatch.

  python tools/pmc_summarize.py FETCH_DIR WRITE_DIR OUT.json --workload "..." [--streams S]

HBM bytes per dispatch = 2 * FETCH_SIZE + WRITE_SIZE (counter unit KiB): on gfx950 FETCH_SIZE
reports half of the bytes of 16-B-per-lane coalesced reads (the guide's calibration); other access
widths are uncalibrated, so the figure is an estimate for the gather / byte-wide parts of a kernel.
The counters include Infinity-Cache hits (memory-side L2 requests), so a working set below 256 MiB
reads as traffic even when it never reaches HBM.
"""
import argparse
import collections
import csv
import glob
import json
import os


def per_kernel(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    assert files, "no counter_collection.csv under %s" % d
    acc = collections.defaultdict(lambda: [0.0, set()])
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            acc[name][0] += float(r["Counter_Value"])
            acc[name][1].add((f, r["Dispatch_Id"]))
    return {k: (v[0] / len(v[1]), len(v[1])) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("out")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--streams", type=int, default=256)
    ap.add_argument("--note", default="", help="what was run (free text)")
    a = ap.parse_args()
    fe = per_kernel(a.fetch_dir, "FETCH_SIZE")
    wr = per_kernel(a.write_dir, "WRITE_SIZE")
    out = {"workload": a.workload, "streams": a.streams, "note": a.note, "unit": "bytes per dispatch",
           "formula": "2*FETCH_SIZE + WRITE_SIZE (KiB counters x 1024); gfx950 FETCH_SIZE halves 16-B reads",
           "kernels": {}}
    for k in sorted(set(fe) | set(wr)):
        if k.startswith("__amd"):
            continue
        f, nf = fe.get(k, (0.0, 0))
        w, nw = wr.get(k, (0.0, 0))
        out["kernels"][k] = {"fetch_kib": round(f, 1), "write_kib": round(w, 1), "dispatches": [nf, nw],
                             "hbm_bytes": int((2 * f + w) * 1024)}
    json.dump(out, open(a.out, "w"), indent=1)
    for k, v in out["kernels"].items():
        print("%-28s fetch %10.0f KiB  write %10.0f KiB  -> %.1f MB" % (k, v["fetch_kib"], v["write_kib"],
                                                                      v["hbm_bytes"] / 1e6))


if __name__ == "__main__":
    main()
