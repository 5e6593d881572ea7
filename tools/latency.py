"""One scan in flight (BASELINE config C2's mode, on synthetic VLP-16 sweeps): per-scan latency of the
single-context drop-in, lego_cloud_handler + lego_feature_association with host buffers in and out,
i.e. what a rosbag replay through the C-ABI sees.

  python tools/latency.py [--scans 60] [--warmup 5] [--voxel-order 0|1]

Prints one JSON line: mean / median / p99 per-scan latency (ms) and the resulting scans/s.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lego-loam-bor_amd"))
import lego_amd as L  # noqa: E402
from lego_amd import _abi as A  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scans", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--seq", type=int, default=5)
    ap.add_argument("--voxel-order", type=int, default=0, choices=(0, 1),
                    help="0 = libstdc++ introsort tie order (reference-exact), 1 = stable order")
    args = ap.parse_args()
    params = L.params_vlp16(voxel_tie_order=args.voxel_order)
    cfg = A.synth_cfg("vlp16")
    n = args.warmup + args.scans
    scans = [np.ascontiguousarray(A.synth_scan(cfg, args.seq, k), dtype=np.float32) for k in range(n)]
    lib = L.lib()
    fe = L.Frontend(params)
    pout, aout = A.LegoProjectionOut(), A.LegoAssociationOut()
    t_ih, t_fa = [], []
    for k in range(n):
        pts = scans[k]
        t0 = time.perf_counter()
        rc = lib.lego_cloud_handler(fe.h, pts.ctypes.data, pts.shape[0], 16, 0, 4, 8, C.byref(pout))
        t1 = time.perf_counter()
        rc |= lib.lego_feature_association(fe.h, C.byref(aout))
        t2 = time.perf_counter()
        assert rc == 0, rc
        if k >= args.warmup:
            t_ih.append(t1 - t0)
            t_fa.append(t2 - t1)
    tot = np.array(t_ih) + np.array(t_fa)
    fe.close()
    print(json.dumps({"mode": "one scan in flight (single-context C-ABI, host buffers in/out)",
                      "scans": args.scans, "voxel_tie_order": args.voxel_order, "cloud_handler_ms": round(1e3 * float(np.mean(t_ih)), 3),
                      "feature_association_ms": round(1e3 * float(np.mean(t_fa)), 3),
                      "scan_ms_mean": round(1e3 * float(tot.mean()), 3),
                      "scan_ms_median": round(1e3 * float(np.median(tot)), 3),
                      "scan_ms_p99": round(1e3 * float(np.percentile(tot, 99)), 3),
                      "scans_per_s": round(1.0 / float(tot.mean()), 1)}))


if __name__ == "__main__":
    main()
