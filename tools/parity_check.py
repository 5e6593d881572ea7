"""Diagnostic: run the GPU front end and the CPU oracle side by side on a synthetic sequence and print
every difference (projection bit-exact, features bit-exact, transforms within tolerance).

  python tools/parity_check.py [--kind vlp16|hdl64] [--scans N] [--seq S]
"""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lego-loam-bor_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import lego_amd as L  # noqa: E402
from lego_amd import _abi as A  # noqa: E402
import oracle as O  # noqa: E402

PROJ_KEYS = ["segmented_cloud", "outlier_cloud", "scan_msg", "start_ring_index", "end_ring_index",
             "start_orientation", "end_orientation", "orientation_diff", "segmented_cloud_ground_flag",
             "segmented_cloud_col_ind", "segmented_cloud_range", "label_mat", "ground_mat", "range_mat"]
FEAT_KEYS = ["sharp_ind", "less_sharp_ind", "flat_ind", "sharp", "less_sharp", "flat", "less_flat"]


def same(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    if a.shape != b.shape:
        return False
    if a.dtype.kind == "f":
        return np.array_equal(a.view(np.uint32 if a.itemsize == 4 else np.uint64),
                              b.astype(a.dtype).view(np.uint32 if a.itemsize == 4 else np.uint64))
    return np.array_equal(a, b)


def describe(k, a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    if a.shape != b.shape:
        return "%s: shape %s vs %s" % (k, a.shape, b.shape)
    d = np.argwhere(~((a == b) | (np.isnan(a) & np.isnan(b)) if a.dtype.kind == "f" else (a == b)))
    return "%s: %d diffs, first at %s: gpu=%s ref=%s" % (k, len(d), d[:3].tolist(), a[tuple(d[0])] if len(d) else None,
                                                        b[tuple(d[0])] if len(d) else None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="vlp16")
    ap.add_argument("--scans", type=int, default=8)
    ap.add_argument("--seq", type=int, default=0)
    args = ap.parse_args()
    params = L.params_vlp16() if args.kind == "vlp16" else L.params_hdl64()
    cfg = A.synth_cfg(args.kind)
    fe = L.Frontend(params)
    orc = O.Oracle(params)
    bad = 0
    for k in range(args.scans):
        pts = A.synth_scan(cfg, args.seq, k)
        t0 = time.time()
        pg = fe.cloud_handler(pts)
        fg = fe.feature_association()
        t1 = time.time()
        pr = orc.cloud_handler(pts)
        fr = orc.feature_association()
        t2 = time.time()
        diffs = []
        for key in PROJ_KEYS:
            if not same(pg[key], pr[key]):
                diffs.append(describe(key, pg[key], pr[key]))
        for key in FEAT_KEYS:
            if not same(fg[key], fr[key]):
                diffs.append(describe(key, fg[key], fr[key]))
        dc = np.abs(fg["transform_cur"] - fr["transform_cur"]).max()
        ds = np.abs(fg["transform_sum"] - fr["transform_sum"]).max()
        print("scan %d M=%d sharp=%d lsharp=%d flat=%d lflat=%d st=%#x/%#x it=%d,%d/%d,%d |dcur|=%.2e |dsum|=%.2e "
              "gpu %.1f ms cpu %.1f ms" % (k, len(pg["segmented_cloud"]), len(fg["sharp"]), len(fg["less_sharp"]),
                                           len(fg["flat"]), len(fg["less_flat"]), fg["status"], fr["status"],
                                           fg["lm_iter_surf"], fg["lm_iter_corner"], fr["lm_iter_surf"],
                                           fr["lm_iter_corner"], dc, ds, (t1 - t0) * 1e3, (t2 - t1) * 1e3))
        for d in diffs:
            print("   DIFF", d)
        bad += len(diffs) + (dc > 1e-4)
    print("RESULT", "OK" if bad == 0 else "MISMATCH %d" % bad)


if __name__ == "__main__":
    main()
