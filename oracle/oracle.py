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
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(os.path.join(HERE, "lego_oracle.cpp")):
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
