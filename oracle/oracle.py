"""ctypes wrapper of the CPU oracle (oracle/liblego_oracle.so).

TEST INFRASTRUCTURE ONLY: loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
always as the checker or the CPU baseline, never as the product path.
"""
import ctypes as C
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liblego_oracle.so")
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "lego-loam-bor_amd"))
from lego_amd import _abi as A  # noqa: E402

P = C.POINTER


def build(force=False):
    srcs = [os.path.join(HERE, f) for f in ("lego_oracle.cpp", "s2m_oracle.cpp")]
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(f) for f in srcs):
        subprocess.check_call(["make", "-C", HERE, "liblego_oracle.so"])


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB)
        L.oracle_create.argtypes = [P(A.LegoParams)]
        L.oracle_create.restype = C.c_void_p
        L.oracle_destroy.argtypes = [C.c_void_p]
        L.oracle_cloud_handler.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                           P(A.LegoProjectionOut)]
        L.oracle_feature_association.argtypes = [C.c_void_p, P(A.LegoAssociationOut)]
        L.oracle_feature_association_from.argtypes = [C.c_void_p, P(A.LegoProjectionOut), P(A.LegoAssociationOut)]
        L.oracle_smoothness.argtypes = [C.c_void_p, C.c_int, P(C.c_float), P(C.c_int64)]
        L.oracle_lm_flags.argtypes = [C.c_void_p, P(C.c_int32), P(C.c_int32)]
        L.oracle_set_lm_state.argtypes = [C.c_void_p, P(C.c_float), P(C.c_float), C.c_int32, P(C.c_float), C.c_int32,
                                          P(C.c_float), C.c_int32, C.c_int32]
        L.oracle_std_sort.argtypes = [P(C.c_uint32), P(C.c_int32), C.c_int, C.c_int]
        L.oracle_atan2f.argtypes = [C.c_float, C.c_float]
        L.oracle_atan2f.restype = C.c_float
        L.oracle_asinf.argtypes = [C.c_float]
        L.oracle_asinf.restype = C.c_float
        _lib = L
    return _lib


class Oracle:
    """One sequence: the reference's ImageProjection + FeatureAssociation, restated on the CPU."""

    def __init__(self, params):
        self.params = params
        self.V = params.num_vertical_scans
        self.H = params.num_horizontal_scans
        self.h = lib().oracle_create(C.byref(params))
        if not self.h:
            raise ValueError("oracle_create failed")

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_destroy(self.h)
            self.h = None

    def cloud_handler(self, pts):
        import numpy as np
        pts = np.ascontiguousarray(pts, dtype=np.float32).reshape(-1, 4)
        out = A.LegoProjectionOut()
        rc = lib().oracle_cloud_handler(self.h, pts.ctypes.data, pts.shape[0], 16, 0, 4, 8, C.byref(out))
        if rc != 0:
            raise RuntimeError("oracle_cloud_handler rc=%d" % rc)
        return A.projection_to_dict(out, self.V, self.H)

    def feature_association(self, proj=None):
        out = A.LegoAssociationOut()
        if proj is None:
            rc = lib().oracle_feature_association(self.h, C.byref(out))
        else:
            keep = []
            pin = A.projection_from_dict(proj, keep)
            rc = lib().oracle_feature_association_from(self.h, C.byref(pin), C.byref(out))
        if rc != 0:
            raise RuntimeError("oracle_feature_association rc=%d" % rc)
        return A.association_to_dict(out)

    def feature_association_with_state(self, proj, cur, tsum, degenerate, corner_last, surf_last, tree_stale):
        """feature_association(proj) starting from the given LM state (oracle_set_lm_state)."""
        import numpy as np
        f = lambda a, k: np.ascontiguousarray(np.asarray(a, np.float32).reshape(-1, k))  # noqa: E731
        c6, s6, cl, sl = f(cur, 6), f(tsum, 6), f(corner_last, 4), f(surf_last, 4)
        fp = lambda a: a.ctypes.data_as(P(C.c_float))  # noqa: E731
        rc = lib().oracle_set_lm_state(self.h, fp(c6), fp(s6), int(degenerate), fp(cl), len(cl), fp(sl), len(sl),
                                       int(tree_stale))
        if rc != 0:
            raise RuntimeError("oracle_set_lm_state rc=%d" % rc)
        return self.feature_association(proj)

    def lm_flags(self):
        """(isDegenerate, kd-trees stale) after the last feature_association."""
        d, t = C.c_int32(), C.c_int32()
        lib().oracle_lm_flags(self.h, C.byref(d), C.byref(t))
        return d.value, t.value

    def smoothness(self, k):
        v = C.c_float()
        i = C.c_int64()
        lib().oracle_smoothness(self.h, k, C.byref(v), C.byref(i))
        return v.value, i.value


def std_sort(keys, vals, is_float):
    """libstdc++ std::sort of (key, val) by key only; keys as uint32 bit patterns."""
    import numpy as np
    k = np.ascontiguousarray(keys, dtype=np.uint32).copy()
    v = np.ascontiguousarray(vals, dtype=np.int32).copy()
    lib().oracle_std_sort(k.ctypes.data_as(P(C.c_uint32)), v.ctypes.data_as(P(C.c_int32)), len(k), int(is_float))
    return k, v


# ---- scan-to-map LM (oracle/s2m_oracle.cpp) ----------------------------------------------------------
def _f32(a, cols=4):
    import numpy as np
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32).reshape(-1, cols))


def scan2map(corner, surf, corner_map, surf_map, transform, degenerate=0):
    """MapOptimization::scan2MapOptimization restated: returns (transform[6], degenerate, info[4])."""
    import numpy as np
    L = lib()
    c, s, cm, sm = (_f32(a) for a in (corner, surf, corner_map, surf_map))
    t = np.ascontiguousarray(np.asarray(transform, dtype=np.float32).copy())
    dg = C.c_int32(int(degenerate))
    info = np.zeros(4, np.int32)
    fp = lambda a: a.ctypes.data_as(P(C.c_float))  # noqa: E731
    L.oracle_scan2map(fp(c), len(c), fp(s), len(s), fp(cm), len(cm), fp(sm), len(sm), fp(t), C.byref(dg),
                      info.ctypes.data_as(P(C.c_int32)))
    return t, dg.value, info


def eig3(A):
    import numpy as np
    A = np.ascontiguousarray(np.asarray(A, np.float32).reshape(9))
    ev = np.zeros(3, np.float32)
    V = np.zeros(9, np.float32)
    lib().oracle_eig3(A.ctypes.data_as(P(C.c_float)), ev.ctypes.data_as(P(C.c_float)), V.ctypes.data_as(P(C.c_float)))
    return ev, V.reshape(3, 3)


def qr_solve(A, b):
    import numpy as np
    A = np.ascontiguousarray(np.asarray(A, np.float32))
    b = np.ascontiguousarray(np.asarray(b, np.float32).reshape(-1))
    x = np.zeros(A.shape[1], np.float32)
    f = {(5, 3): lib().oracle_qr53, (6, 6): lib().oracle_qr66}[A.shape]
    f(A.ctypes.data_as(P(C.c_float)), b.ctypes.data_as(P(C.c_float)), x.ctypes.data_as(P(C.c_float)))
    return x


def knn5(cloud, queries):
    """(indices [n,5], sq dists [n,5], flags [n]: bit 0 = 5th closer than 1, bit 1 = distance tie)."""
    import numpy as np
    m, q = _f32(cloud), _f32(queries)
    ind = np.zeros((len(q), 5), np.int32)
    d = np.zeros((len(q), 5), np.float32)
    fl = np.zeros(len(q), np.int32)
    lib().oracle_knn5(m.ctypes.data_as(P(C.c_float)), len(m), q.ctypes.data_as(P(C.c_float)), len(q),
                      ind.ctypes.data_as(P(C.c_int32)), d.ctypes.data_as(P(C.c_float)), fl.ctypes.data_as(P(C.c_int32)))
    return ind, d, fl


def knn_tree(cloud, queries, k=1):
    """nanoflann k-NN restated (oracle/nanoflann_restated.h): (indices [m, k], squared distances [m, k])."""
    import numpy as np
    c, q = _f32(cloud), _f32(queries)
    idx = np.zeros((len(q), k), np.int32)
    d = np.zeros((len(q), k), np.float32)
    lib().oracle_knn_tree(c.ctypes.data_as(P(C.c_float)), len(c), q.ctypes.data_as(P(C.c_float)), len(q), int(k),
                          idx.ctypes.data_as(P(C.c_int32)), d.ctypes.data_as(P(C.c_float)))
    return idx, d


def voxel_grid(points, leaf, stable=True):
    """pcl::VoxelGrid::filter restated (oracle/lego_oracle.cpp): (output (M, 4) float32, status bits)."""
    import numpy as np
    p = _f32(points)
    out = np.zeros((max(len(p), 1), 4), np.float32)
    n_out = C.c_int(0)
    L = lib()
    L.oracle_voxel_grid.restype = C.c_int
    st = L.oracle_voxel_grid(p.ctypes.data_as(P(C.c_float)), len(p), C.c_float(leaf), int(bool(stable)),
                             out.ctypes.data_as(P(C.c_float)), C.byref(n_out))
    return out[:n_out.value].copy(), st


def scan2map_debug(corner, surf, corner_map, surf_map, transform, degenerate=0, max_iters=10):
    """scan2map with at most max_iters LM iterations; also returns the last iteration's rows (8 floats a
    query, lego_test_s2m_debug's layout)."""
    import numpy as np
    arrs = [_f32(a) for a in (corner, surf, corner_map, surf_map)]
    t = np.ascontiguousarray(np.asarray(transform, np.float32).reshape(6).copy())
    dg = C.c_int32(int(degenerate))
    info = np.zeros(4, np.int32)
    rows = np.zeros((len(arrs[0]) + len(arrs[1]), 8), np.float32)
    args = []
    for a in arrs:
        args += [a.ctypes.data_as(P(C.c_float)), len(a)]
    lib().oracle_scan2map_debug(*args, t.ctypes.data_as(P(C.c_float)), C.byref(dg), info.ctypes.data_as(P(C.c_int32)),
                                int(max_iters), rows.ctypes.data_as(P(C.c_float)))
    return t, dg.value, info, rows


def odometry_to_transform(orientation, position):
    """OdometryToTransform restated (utility.h:96-110): transformSum from the odometry message."""
    import numpy as np
    q = np.ascontiguousarray(np.asarray(orientation, np.float64).reshape(4))
    p = np.ascontiguousarray(np.asarray(position, np.float64).reshape(3))
    t = np.zeros(6, np.float32)
    lib().oracle_odometry_to_transform(q.ctypes.data_as(P(C.c_double)), p.ctypes.data_as(P(C.c_double)),
                                       t.ctypes.data_as(P(C.c_float)))
    return t


def associate_to_map(t_sum, t_bef, t_aft):
    """MapOptimization::transformAssociateToMap restated (mapOptmization.cpp:264-387): transformTobeMapped."""
    import numpy as np
    a = [np.ascontiguousarray(np.asarray(t, np.float32).reshape(6)) for t in (t_sum, t_bef, t_aft)]
    out = np.zeros(6, np.float32)
    lib().oracle_associate_to_map(*[x.ctypes.data_as(P(C.c_float)) for x in a + [out]])
    return out


def transform_cloud(points, pose):
    """MapOptimization::transformPointCloud restated: pose = (roll, pitch, yaw, x, y, z)."""
    import numpy as np
    p = _f32(points)
    out = np.zeros_like(p)
    q = np.ascontiguousarray(np.asarray(pose, np.float32).reshape(6))
    lib().oracle_transform_cloud(p.ctypes.data_as(P(C.c_float)), len(p), q.ctypes.data_as(P(C.c_float)),
                                 out.ctypes.data_as(P(C.c_float)))
    return out
