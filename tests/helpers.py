"""Shared helpers for the parity tests: bit-exact comparison of projection / feature outputs."""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")

PROJ_KEYS = ["segmented_cloud", "outlier_cloud", "scan_msg", "start_ring_index", "end_ring_index",
             "start_orientation", "end_orientation", "orientation_diff", "segmented_cloud_ground_flag",
             "segmented_cloud_col_ind", "segmented_cloud_range", "label_mat", "ground_mat", "range_mat"]
FEAT_KEYS = ["sharp_ind", "less_sharp_ind", "flat_ind", "sharp", "less_sharp", "flat", "less_flat"]
# 6-DoF tolerance stated by north_star (rad / m)
TF_TOL = 1e-4


def bits_equal(a, b):
    """Bit-exact equality (floats compared by bit pattern; NaN == NaN with the same payload)."""
    a = np.asarray(a)
    b = np.asarray(b)
    if a.shape != b.shape:
        return False
    if a.dtype.kind == "f":
        w = {2: np.uint16, 4: np.uint32, 8: np.uint64}[a.itemsize]
        return np.array_equal(np.ascontiguousarray(a).view(w), np.ascontiguousarray(b.astype(a.dtype)).view(w))
    return np.array_equal(a, b)


def diff_report(keys, got, ref):
    bad = []
    for k in keys:
        if not bits_equal(got[k], ref[k]):
            g, r = np.asarray(got[k]), np.asarray(ref[k])
            if g.shape != r.shape:
                bad.append("%s: shape %s vs %s" % (k, g.shape, r.shape))
            else:
                ne = np.argwhere(g != r) if g.dtype.kind != "f" else np.argwhere(~((g == r) | (np.isnan(g) & np.isnan(r))))
                bad.append("%s: %d elements differ, first %s" % (k, len(ne), ne[:3].tolist()))
    return bad


def load_golden():
    with open(os.path.join(GOLDEN, "golden_oracle.json")) as f:
        return json.load(f)


def golden_case(name):
    return load_golden()["cases"][name]
