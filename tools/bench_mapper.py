"""Measure the native mapping thread (lego_mapper_*, lego_amd.Mapper): per-cycle latency of one
sequence on one GPU vs the same loop on the CPU oracle.

The AssociationOut stream comes from the product front end (lego_amd.Frontend) over a synthetic VLP-16
sequence; every emitted record (every 5th scan, mapping_frequency_divider) is one mapping cycle.  Each
Mapper.step is synchronous (host clouds in, transformAftMapped out), so the wall time of a step is the
cycle's latency, host logic, copies and the three device operations included.  The CPU baseline runs
the same cycles through lego_amd.mapping.MapSequence around the oracle's operations (single thread),
which also gives the parity figure (max |delta transformAftMapped| over all cycles).

  python tools/bench_mapper.py [--scans 151] [--seq 3] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lego-loam-bor_amd"), os.path.join(REPO, "tests"), os.path.join(REPO, "oracle")]

LEGO_ST_EMITTED = 0x080


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scans", type=int, default=151)
    ap.add_argument("--seq", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default="")
    ap.add_argument("--detail", action="store_true")
    args = ap.parse_args()

    import lego_amd as LA
    from lego_amd import _abi as A
    from lego_amd import mapping as M

    fe = LA.Frontend(LA.params_vlp16())
    cfg = A.synth_cfg("vlp16")
    assocs = []
    for k in range(args.scans):
        fe.cloud_handler(A.synth_scan(cfg, args.seq, k))
        a = fe.feature_association()
        if a["status"] & LEGO_ST_EMITTED:
            assocs.append(a)
    fe.close()
    C = len(assocs)

    best = None
    for _ in range(args.reps):  # each rep a fresh mapper over the whole sequence
        mp = LA.Mapper(max_map_points=200000, max_key_points=20_000_000)
        ms, poses, ran, infos = [], [], 0, []
        for a in assocs:
            t0 = time.perf_counter()
            t, info = mp.step(a["corner_last"], a["surf_last"], a["outlier_last"],
                             M.odometry_to_transform(a["odom_orientation"], a["odom_position"]))
            ms.append((time.perf_counter() - t0) * 1e3)
            poses.append(t)
            infos.append(info.copy())
            ran += int(info[0] == 1)
        keys = len(mp.key_poses())
        mp.close()
        if best is None or np.mean(ms) < np.mean(best[0]):
            best = (ms, poses, ran, keys, infos)
    ms, poses, ran, keys, infos = best

    import oracle as O
    sq = M.MapSequence(associate=O.associate_to_map, odometry=O.odometry_to_transform)
    from test_gpu_mapping_loop import mapping_step_oracle
    cpu_ms, dmax, per_cycle = [], 0.0, []
    for a, t, ig in zip(assocs, poses, infos):
        t0 = time.perf_counter()
        (_, _, ir), = mapping_step_oracle([sq], [a])
        cpu_ms.append((time.perf_counter() - t0) * 1e3)
        d = float(np.abs(sq.t_aft - t).max())
        dmax = max(dmax, d)
        per_cycle.append([d, [int(x) for x in ig], [int(x) for x in ir]])

    res = {
        "what": "MapOptimization::run loop body (loop closure off), one sequence, synchronous steps",
        "sequence": {"sensor": "vlp16 synthetic", "seq": args.seq, "scans": args.scans, "cycles": C,
                     "cycles_with_lm": ran, "key_frames": keys},
        "gpu": {"ms_per_cycle_mean": round(float(np.mean(ms)), 3), "ms_per_cycle_median": round(float(np.median(ms)), 3),
                "ms_per_cycle_max": round(float(np.max(ms)), 3), "cycles_per_s": round(1e3 / float(np.mean(ms)), 1),
                "first_cycle_ms": round(ms[0], 3)},
        "cpu_baseline": {"kind": "port", "cores": 1, "ms_per_cycle_mean": round(float(np.mean(cpu_ms)), 3),
                         "cycles_per_s": round(1e3 / float(np.mean(cpu_ms)), 2)},
        "parity_max_abs_delta_transform": dmax,
    }
    if args.detail:
        res["per_cycle"] = per_cycle  # [max |delta|, GPU info, oracle info]
    line = json.dumps(res)
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
