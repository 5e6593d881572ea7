"""Regenerate the golden fixtures in tests/golden/ (run in the build container).

The reference has no tests and no fixtures and cannot be built here (§8c), so these
vectors are produced by the CPU oracle (oracle/, a restatement of the reference's path) on the
deterministic synthetic sweeps.  They pin the oracle and the GPU path against regressions; they
do not by themselves pin the oracle to the reference (see DESIGN.md §Parity status).

  python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "lego-loam-bor_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
from lego_amd import _abi as A  # noqa: E402
import oracle as O  # noqa: E402

PROJ_HASH = ["segmented_cloud", "outlier_cloud", "scan_msg", "start_ring_index", "end_ring_index",
             "segmented_cloud_ground_flag", "segmented_cloud_col_ind", "segmented_cloud_range", "label_mat",
             "ground_mat", "range_mat"]
FEAT_HASH = ["sharp_ind", "less_sharp_ind", "flat_ind", "sharp", "less_sharp", "flat", "less_flat"]

NOISE_FREE = {"range_noise": 0.0, "az_jitter_deg": 0.0, "roll_pitch_noise_deg": 0.0}
# (name, sensor kind, synth overrides, sequence, number of scans, fp_mode)
CASES = [
    ("vlp16_seq0", "vlp16", {}, 0, 6, 0),
    ("vlp16_seq7", "vlp16", {}, 7, 3, 0),
    ("vlp16_noisefree_seq3", "vlp16", NOISE_FREE, 3, 3, 0),
    ("hdl64_seq0", "hdl64", {}, 0, 2, 0),
    # fp_mode 1: the unqualified libm calls in double (the Indigo / Kinetic toolchains)
    ("vlp16_seq0_fp1", "vlp16", {}, 0, 6, 1),
    ("vlp16_noisefree_seq3_fp1", "vlp16", NOISE_FREE, 3, 3, 1),
    ("hdl64_seq0_fp1", "hdl64", {}, 0, 2, 1),
]


def params_for(kind, fp_mode=0):
    p = A.LegoParams()
    if kind == "vlp16":
        vals = (16, 1800, 7, -15.0, 15.0, 0.0, 0.1, 5, 3, 60.0, 0.1, 0.1, 5.0, 5, 0)
    else:
        vals = (64, 2048, 55, -24.8, 2.0, 0.0, 0.1, 5, 3, 60.0, 0.1, 0.1, 5.0, 5, 0)
    for (name, _), v in zip(A.LegoParams._fields_, vals):
        setattr(p, name, v)
    p.fp_mode = fp_mode
    return p


def h(a):
    a = np.ascontiguousarray(a)
    return hashlib.sha256(a.tobytes()).hexdigest()[:24]


def run_case(kind, over, seq, nscans, fp_mode=0):
    params = params_for(kind, fp_mode)
    cfg = A.synth_cfg(kind, **over)
    orc = O.Oracle(params)
    rows = []
    for k in range(nscans):
        pts = A.synth_scan(cfg, seq, k)
        pr = orc.cloud_handler(pts)
        fa = orc.feature_association()
        row = {"scan": k, "n_points": int(len(pts)), "input": h(pts)}
        row.update({"p_" + key: h(pr[key]) for key in PROJ_HASH})
        row.update({"f_" + key: h(fa[key]) for key in FEAT_HASH})
        row["M"] = int(len(pr["segmented_cloud"]))
        row["n_sharp"] = int(len(fa["sharp"]))
        row["n_flat"] = int(len(fa["flat"]))
        row["n_less_flat"] = int(len(fa["less_flat"]))
        row["status"] = int(fa["status"])
        row["transform_cur"] = [float(x) for x in fa["transform_cur"]]
        row["transform_sum"] = [float(x) for x in fa["transform_sum"]]
        rows.append(row)
    return rows, pts, pr, fa


def main():
    out = {"generator": "oracle/lego_oracle.cpp via tests/golden/make_golden.py", "cases": {}}
    for name, kind, over, seq, n, fp_mode in CASES:
        rows, pts, pr, fa = run_case(kind, over, seq, n, fp_mode)
        out["cases"][name] = {"kind": kind, "synth": over, "seq": seq, "fp_mode": fp_mode, "scans": rows}
        print(name, [(r["M"], r["n_sharp"], r["n_flat"], hex(r["status"])) for r in rows])
    with open(os.path.join(HERE, "golden_oracle.json"), "w") as f:
        json.dump(out, f, indent=1)
    # full arrays of one VLP-16 scan (first scan of vlp16_seq0) for element-wise diagnostics
    params = params_for("vlp16")
    cfg = A.synth_cfg("vlp16")
    orc = O.Oracle(params)
    pts = A.synth_scan(cfg, 0, 0)
    pr = orc.cloud_handler(pts)
    fa = orc.feature_association()
    np.savez_compressed(os.path.join(HERE, "vlp16_seq0_scan0.npz"), points=pts, label_mat=pr["label_mat"],
                        ground_mat=pr["ground_mat"], start_ring_index=pr["start_ring_index"],
                        end_ring_index=pr["end_ring_index"], segmented_cloud_col_ind=pr["segmented_cloud_col_ind"],
                        sharp_ind=fa["sharp_ind"], less_sharp_ind=fa["less_sharp_ind"], flat_ind=fa["flat_ind"])


if __name__ == "__main__":
    main()
