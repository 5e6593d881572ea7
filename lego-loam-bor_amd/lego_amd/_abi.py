"""ctypes mirror of include/lego_frontend.h (the C-ABI) and of the synthetic-sweep generator.

Only plain ctypes here: the product library (liblego_frontend.so) and the synthetic generator
(liblego_synth.so) are loaded from this package's directory, where build.py puts them.
"""
import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_FRONTEND = os.environ.get("LEGO_FRONTEND_LIB", os.path.join(PKG_DIR, "liblego_frontend.so"))
LIB_SYNTH = os.path.join(PKG_DIR, "liblego_synth.so")

LEGO_OK, LEGO_EINVAL, LEGO_ENOMEM, LEGO_EDEVICE, LEGO_ENOTSUP, LEGO_EEMPTY = 0, -1, -2, -3, -4, -5

ST_INIT = 0x001
ST_LM_SKIPPED = 0x002
ST_DEGENERATE = 0x004
ST_STALE_TREE = 0x008
ST_FWD_OOB = 0x010
ST_NN_TIE = 0x020
ST_STALE_IND_OOB = 0x040
ST_EMITTED = 0x080
ST_VOXEL_OVERFLOW = 0x100
ST_DEGEN_UB = 0x200
ST_TIE_UNRESOLVED = 0x400  # a 1-NN tie the device kd-tree could not resolve (stack overflow): not nanoflann's
# bits that mark reference undefined behaviour given defined behaviour here, or a result not pinned to the
# reference (NN_TIE alone is resolved as nanoflann does)
ST_UB_MASK = ST_STALE_TREE | ST_FWD_OOB | ST_STALE_IND_OOB | ST_DEGEN_UB | ST_TIE_UNRESOLVED
S2M_ST_TIE_UNRESOLVED = 0x20


class LegoParams(C.Structure):
    _fields_ = [
        ("num_vertical_scans", C.c_int32),
        ("num_horizontal_scans", C.c_int32),
        ("ground_scan_index", C.c_int32),
        ("vertical_angle_bottom", C.c_float),
        ("vertical_angle_top", C.c_float),
        ("sensor_mount_angle", C.c_float),
        ("scan_period", C.c_float),
        ("segment_valid_point_num", C.c_int32),
        ("segment_valid_line_num", C.c_int32),
        ("segment_theta", C.c_float),
        ("edge_threshold", C.c_float),
        ("surf_threshold", C.c_float),
        ("nearest_feature_search_distance", C.c_float),
        ("mapping_frequency_divider", C.c_int32),
        ("fp_mode", C.c_int32),
        ("voxel_tie_order", C.c_int32),
    ]


class LegoPoint(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float), ("intensity", C.c_float)]


P = C.POINTER


class LegoProjectionOut(C.Structure):
    _fields_ = [
        ("n_segmented", C.c_int32),
        ("n_outlier", C.c_int32),
        ("n_scan", C.c_int32),
        ("segmented_cloud", P(LegoPoint)),
        ("outlier_cloud", P(LegoPoint)),
        ("scan_msg", P(LegoPoint)),
        ("start_ring_index", P(C.c_int32)),
        ("end_ring_index", P(C.c_int32)),
        ("start_orientation", C.c_float),
        ("end_orientation", C.c_float),
        ("orientation_diff", C.c_float),
        ("segmented_cloud_ground_flag", P(C.c_uint8)),
        ("segmented_cloud_col_ind", P(C.c_uint32)),
        ("segmented_cloud_range", P(C.c_float)),
        ("label_mat", P(C.c_int32)),
        ("ground_mat", P(C.c_int8)),
        ("range_mat", P(C.c_float)),
    ]


class LegoAssociationOut(C.Structure):
    _fields_ = [
        ("status", C.c_int32),
        ("n_sharp", C.c_int32),
        ("n_less_sharp", C.c_int32),
        ("n_flat", C.c_int32),
        ("n_less_flat", C.c_int32),
        ("corner_points_sharp", P(LegoPoint)),
        ("corner_points_less_sharp", P(LegoPoint)),
        ("surf_points_flat", P(LegoPoint)),
        ("surf_points_less_flat", P(LegoPoint)),
        ("sharp_ind", P(C.c_int32)),
        ("less_sharp_ind", P(C.c_int32)),
        ("flat_ind", P(C.c_int32)),
        ("transform_cur", C.c_float * 6),
        ("transform_sum", C.c_float * 6),
        ("odom_orientation", C.c_double * 4),
        ("odom_position", C.c_double * 3),
        ("lm_iter_surf", C.c_int32),
        ("lm_iter_corner", C.c_int32),
        ("n_corner_last", C.c_int32),
        ("n_surf_last", C.c_int32),
        ("n_outlier_last", C.c_int32),
        ("cloud_corner_last", P(LegoPoint)),
        ("cloud_surf_last", P(LegoPoint)),
        ("cloud_outlier_last", P(LegoPoint)),
    ]


class LegoSynthCfg(C.Structure):
    _fields_ = [
        ("V", C.c_int32), ("H", C.c_int32),
        ("elev_bottom_deg", C.c_float), ("elev_top_deg", C.c_float),
        ("sensor_height", C.c_float),
        ("base_seed", C.c_int32),
        ("dropout", C.c_float),
        ("range_noise", C.c_float),
        ("az_jitter_deg", C.c_float),
        ("max_range", C.c_float),
        ("speed", C.c_float),
        ("yaw_rate_deg", C.c_float),
        ("roll_pitch_noise_deg", C.c_float),
        ("scan_period", C.c_float),
    ]


def _arr(ptr, n, dtype):
    """Copy n elements behind a ctypes pointer into a numpy array (empty when n == 0)."""
    if n <= 0 or not ptr:
        return np.zeros((0,), dtype=dtype)
    return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dtype, copy=True)


def _pts(ptr, n):
    if n <= 0 or not ptr:
        return np.zeros((0, 4), dtype=np.float32)
    raw = C.cast(ptr, P(C.c_float))
    return np.ctypeslib.as_array(raw, shape=(n * 4,)).reshape(n, 4).copy()


def projection_to_dict(out, V, H):
    n = out.n_segmented
    d = {
        "segmented_cloud": _pts(out.segmented_cloud, n),
        "outlier_cloud": _pts(out.outlier_cloud, out.n_outlier),
        "scan_msg": _pts(out.scan_msg, out.n_scan),
        "start_ring_index": _arr(out.start_ring_index, V, np.int32),
        "end_ring_index": _arr(out.end_ring_index, V, np.int32),
        "start_orientation": np.float32(out.start_orientation),
        "end_orientation": np.float32(out.end_orientation),
        "orientation_diff": np.float32(out.orientation_diff),
        "segmented_cloud_ground_flag": _arr(out.segmented_cloud_ground_flag, n, np.uint8),
        "segmented_cloud_col_ind": _arr(out.segmented_cloud_col_ind, n, np.uint32),
        "segmented_cloud_range": _arr(out.segmented_cloud_range, n, np.float32),
    }
    if out.label_mat:
        d["label_mat"] = _arr(out.label_mat, V * H, np.int32).reshape(V, H)
    if out.ground_mat:
        d["ground_mat"] = _arr(out.ground_mat, V * H, np.int8).reshape(V, H)
    if out.range_mat:
        d["range_mat"] = _arr(out.range_mat, V * H, np.float32).reshape(V, H)
    return d


def association_to_dict(out):
    return {
        "status": int(out.status),
        "sharp": _pts(out.corner_points_sharp, out.n_sharp),
        "less_sharp": _pts(out.corner_points_less_sharp, out.n_less_sharp),
        "flat": _pts(out.surf_points_flat, out.n_flat),
        "less_flat": _pts(out.surf_points_less_flat, out.n_less_flat),
        "sharp_ind": _arr(out.sharp_ind, out.n_sharp, np.int32),
        "less_sharp_ind": _arr(out.less_sharp_ind, out.n_less_sharp, np.int32),
        "flat_ind": _arr(out.flat_ind, out.n_flat, np.int32),
        "transform_cur": np.array(out.transform_cur[:], dtype=np.float32),
        "transform_sum": np.array(out.transform_sum[:], dtype=np.float32),
        "odom_orientation": np.array(out.odom_orientation[:], dtype=np.float64),
        "odom_position": np.array(out.odom_position[:], dtype=np.float64),
        "lm_iter_surf": int(out.lm_iter_surf),
        "lm_iter_corner": int(out.lm_iter_corner),
        "corner_last": _pts(out.cloud_corner_last, out.n_corner_last),
        "surf_last": _pts(out.cloud_surf_last, out.n_surf_last),
        "outlier_last": _pts(out.cloud_outlier_last, out.n_outlier_last),
    }


def projection_from_dict(d, keep):
    """Build a LegoProjectionOut pointing at numpy arrays (kept alive in `keep`)."""
    out = LegoProjectionOut()

    def ptr(name, dtype, ctype):
        a = np.ascontiguousarray(d[name], dtype=dtype)
        keep.append(a)
        return a.ctypes.data_as(P(ctype))

    seg = np.ascontiguousarray(d["segmented_cloud"], dtype=np.float32).reshape(-1, 4)
    out.n_segmented = seg.shape[0]
    keep.append(seg)
    out.segmented_cloud = seg.ctypes.data_as(P(LegoPoint))
    outl = np.ascontiguousarray(d["outlier_cloud"], dtype=np.float32).reshape(-1, 4)
    keep.append(outl)
    out.n_outlier = outl.shape[0]
    out.outlier_cloud = outl.ctypes.data_as(P(LegoPoint))
    sm = np.ascontiguousarray(d.get("scan_msg", np.zeros((0, 4), np.float32)), dtype=np.float32).reshape(-1, 4)
    keep.append(sm)
    out.n_scan = sm.shape[0]
    out.scan_msg = sm.ctypes.data_as(P(LegoPoint))
    out.start_ring_index = ptr("start_ring_index", np.int32, C.c_int32)
    out.end_ring_index = ptr("end_ring_index", np.int32, C.c_int32)
    out.start_orientation = float(d["start_orientation"])
    out.end_orientation = float(d["end_orientation"])
    out.orientation_diff = float(d["orientation_diff"])
    out.segmented_cloud_ground_flag = ptr("segmented_cloud_ground_flag", np.uint8, C.c_uint8)
    out.segmented_cloud_col_ind = ptr("segmented_cloud_col_ind", np.uint32, C.c_uint32)
    out.segmented_cloud_range = ptr("segmented_cloud_range", np.float32, C.c_float)
    return out


# ---------------------------------------------------------------------------------------------
# synthetic generator
# ---------------------------------------------------------------------------------------------
_synth = None


def synth_lib():
    global _synth
    if _synth is None:
        lib = C.CDLL(LIB_SYNTH)
        lib.lego_synth_vlp16.argtypes = [P(LegoSynthCfg)]
        lib.lego_synth_hdl64.argtypes = [P(LegoSynthCfg)]
        lib.lego_synth_scan.argtypes = [P(LegoSynthCfg), C.c_int, C.c_int, P(C.c_float), C.c_int]
        lib.lego_synth_scan.restype = C.c_int
        lib.lego_synth_batch.argtypes = [P(LegoSynthCfg), C.c_int, P(C.c_int), P(C.c_int), P(C.c_float),
                                         P(C.c_int64), C.c_int, P(C.c_int), C.c_int]
        lib.lego_synth_batch.restype = C.c_int
        _synth = lib
    return _synth


def synth_cfg(kind="vlp16", **over):
    cfg = LegoSynthCfg()
    lib = synth_lib()
    if kind == "vlp16":
        lib.lego_synth_vlp16(C.byref(cfg))
    elif kind == "hdl64":
        lib.lego_synth_hdl64(C.byref(cfg))
    else:
        raise ValueError(kind)
    for k, v in over.items():
        setattr(cfg, k, v)
    return cfg


def synth_scan(cfg, seq, scan):
    cap = cfg.V * cfg.H
    buf = np.zeros((cap, 4), dtype=np.float32)
    n = synth_lib().lego_synth_scan(C.byref(cfg), seq, scan, buf.ctypes.data_as(P(C.c_float)), cap)
    if n < 0:
        raise RuntimeError("synth capacity")
    return buf[:n].copy()


def synth_batch(cfg, seqs, scans, nthreads=0):
    """Scans (seqs[i], scans[i]) into one padded array [n, V*H, 4]; returns (points, counts)."""
    n = len(seqs)
    cap = cfg.V * cfg.H
    out = np.zeros((n, cap, 4), dtype=np.float32)
    offs = (np.arange(n, dtype=np.int64) * cap)
    counts = np.zeros(n, dtype=np.int32)
    s = np.ascontiguousarray(seqs, dtype=np.int32)
    k = np.ascontiguousarray(scans, dtype=np.int32)
    rc = synth_lib().lego_synth_batch(C.byref(cfg), n, s.ctypes.data_as(P(C.c_int)), k.ctypes.data_as(P(C.c_int)),
                                      out.ctypes.data_as(P(C.c_float)), offs.ctypes.data_as(P(C.c_int64)), cap,
                                      counts.ctypes.data_as(P(C.c_int)), int(nthreads))
    if rc != 0:
        raise RuntimeError("synth batch failed")
    return out, counts
