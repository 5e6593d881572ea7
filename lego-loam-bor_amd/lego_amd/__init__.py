"""lego_amd — Python view of the MI355X LeGO-LOAM-BOR front end (C-ABI in include/lego_frontend.h).

The product is liblego_frontend.so (HIP kernels for gfx950).  This module only binds it with ctypes;
there is no Python or CPU fallback: if the library is missing, or no HIP device is present, the
constructors raise.

  Frontend  — one sequence: cloud_handler() (ImageProjection::cloudHandler) and
              feature_association() (one FeatureAssociation::runFeatureAssociation iteration).
  Batch     — S independent sequences advanced one scan per step on device-resident input.
  ScanToMap — MapOptimization::scan2MapOptimization for many problems at once (include/lego_s2m.h).
"""
import ctypes as C
import os

import numpy as np

from . import _abi as A
from ._abi import (LegoAssociationOut, LegoParams, LegoPoint, LegoProjectionOut, association_to_dict,  # noqa: F401
                   projection_from_dict, projection_to_dict)

P = C.POINTER
_lib = None


class LegoMapTransformIo(C.Structure):
    """lego_map_transform_io (include/lego_s2m.h)."""
    _fields_ = [(n, C.c_void_p) for n in ("in_", "in_off", "in_n", "pose", "out", "out_off")]


class LegoMapVoxelIo(C.Structure):
    """lego_map_voxel_io (include/lego_s2m.h)."""
    _fields_ = [(n, C.c_void_p) for n in ("in_", "in_off", "in_n", "leaf", "out", "out_off", "out_n", "status")]


class LegoS2mIo(C.Structure):
    """lego_s2m_io (include/lego_s2m.h): device pointers of a batch of scan-to-map problems."""
    _fields_ = [(n, C.c_void_p) for c in ("corner", "surf", "corner_map", "surf_map")
                for n in (c, c + "_off", c + "_n")] + [("transform", C.c_void_p), ("degenerate", C.c_void_p),
                                                       ("info", C.c_void_p)]


class LegoError(RuntimeError):
    pass


def lib():
    """Load liblego_frontend.so from this package directory (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(A.LIB_FRONTEND):
            raise LegoError("liblego_frontend.so not built: run python lego-loam-bor_amd/build.py")
        try:  # torch first: its HIP runtime (loaded RTLD_GLOBAL) then serves this library as well, so the
            import torch  # noqa: F401  process has one runtime and torch's tensors / streams interoperate
        except ImportError:
            pass
        L = C.CDLL(A.LIB_FRONTEND)
        L.lego_abi_version.restype = C.c_int32
        L.lego_params_vlp16.argtypes = [P(LegoParams)]
        L.lego_params_hdl64.argtypes = [P(LegoParams)]
        L.lego_params_validate.argtypes = [P(LegoParams)]
        L.lego_params_load_yaml.argtypes = [C.c_char_p, P(LegoParams)]
        L.lego_test_libm_d.argtypes = [P(C.c_double), P(C.c_double), P(C.c_double), C.c_int32, C.c_int32]
        L.lego_device_count.restype = C.c_int32
        L.lego_ctx_create.argtypes = [P(LegoParams), C.c_int32, P(C.c_void_p)]
        L.lego_ctx_destroy.argtypes = [C.c_void_p]
        L.lego_cloud_handler.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                         C.c_int32, P(LegoProjectionOut)]
        L.lego_feature_association.argtypes = [C.c_void_p, P(LegoAssociationOut)]
        L.lego_feature_association_from.argtypes = [C.c_void_p, P(LegoProjectionOut), P(LegoAssociationOut)]
        L.lego_test_set_lm_state.argtypes = [C.c_void_p, P(C.c_float), P(C.c_float), C.c_int32, C.c_void_p, C.c_int32,
                                             C.c_void_p, C.c_int32, C.c_int32]
        L.lego_batch_create.argtypes = [P(LegoParams), C.c_int32, C.c_int32, C.c_int32, P(C.c_void_p)]
        L.lego_batch_destroy.argtypes = [C.c_void_p]
        L.lego_batch_step.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.lego_batch_sync.argtypes = [C.c_void_p]
        L.lego_batch_flush.argtypes = [C.c_void_p]
        L.lego_batch_read.argtypes = [C.c_void_p, C.c_int32, P(LegoProjectionOut), P(LegoAssociationOut)]
        L.lego_batch_read_poses.argtypes = [C.c_void_p, P(C.c_float), P(C.c_int32)]
        L.lego_batch_reset.argtypes = [C.c_void_p]
        L.lego_batch_stage_times.argtypes = [C.c_void_p, P(C.c_float)]
        L.lego_batch_set_timing.argtypes = [C.c_void_p, C.c_int32]
        L.lego_batch_time_hbm_stages.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                                                 C.c_void_p, C.c_void_p, C.c_void_p, P(C.c_float)]
        L.lego_batch_set_groups.argtypes = [C.c_void_p, C.c_int32]
        L.lego_batch_set_lag.argtypes = [C.c_void_p, C.c_int32]
        L.lego_batch_set_probe.argtypes = [C.c_void_p, C.c_int32]
        L.lego_batch_set_trajectory.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
        L.lego_batch_time_voxel.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, P(C.c_float)]
        L.lego_batch_probe_times.argtypes = [C.c_void_p, P(C.c_float), P(C.c_int32)]
        L.lego_batch_set_wide.argtypes = [C.c_void_p, C.c_int32]
        L.lego_batch_wide.argtypes = [C.c_void_p]
        L.lego_batch_lag.argtypes = [C.c_void_p]
        L.lego_batch_read_counts.argtypes = [C.c_void_p, P(C.c_int32)]
        L.lego_batch_state_size.argtypes = [C.c_void_p, P(C.c_size_t)]
        L.lego_batch_save_state.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_size_t]
        L.lego_batch_load_state.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_size_t]
        L.lego_ctx_state_size.argtypes = [C.c_void_p, P(C.c_size_t)]
        L.lego_ctx_save_state.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.lego_ctx_load_state.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.lego_test_sort.argtypes = [P(C.c_uint32), P(C.c_int32), C.c_int32, C.c_int32]
        L.lego_test_libm.argtypes = [P(C.c_float), P(C.c_float), P(C.c_float), C.c_int32, C.c_int32]
        L.lego_test_project_cells.argtypes = [P(LegoParams), P(C.c_float), C.c_int32, P(C.c_int32), P(C.c_int32)]
        L.lego_s2m_create.argtypes = [C.c_int32, C.c_int32, C.c_int32, P(C.c_void_p)]
        L.lego_s2m_destroy.argtypes = [C.c_void_p]
        L.lego_s2m_run.argtypes = [C.c_void_p, C.c_int32, P(LegoS2mIo), C.c_void_p]
        L.lego_s2m_run_host.argtypes = [C.c_void_p] + [C.c_void_p, C.c_int32] * 4 + [P(C.c_float), P(C.c_int32),
                                                                                  P(C.c_int32)]
        L.lego_map_transform.argtypes = [C.c_void_p, C.c_int32, P(LegoMapTransformIo), C.c_void_p]
        L.lego_map_voxel.argtypes = [C.c_void_p, C.c_int32, P(LegoMapVoxelIo), C.c_void_p]
        L.lego_s2m_set_layout.argtypes = [C.c_void_p, C.c_int32]
        L.lego_s2m_set_voxel_tie_order.argtypes = [C.c_void_p, C.c_int32]
        L.lego_mapper_set_voxel_tie_order.argtypes = [C.c_void_p, C.c_int32]
        L.lego_mapper_create.argtypes = [C.c_int32, C.c_int32, C.c_int64, P(C.c_void_p)]
        L.lego_mapper_destroy.argtypes = [C.c_void_p]
        L.lego_mapper_step.argtypes = [C.c_void_p] + [C.c_void_p, C.c_int32] * 3 + [P(C.c_float), P(C.c_float),
                                                                                    P(C.c_int32)]
        L.lego_mapper_key_poses.argtypes = [C.c_void_p, P(C.c_float), C.c_int32, P(C.c_int32)]
        L.lego_map_associate.argtypes = [P(C.c_float)] * 4
        L.lego_map_odometry_to_transform.argtypes = [P(C.c_double), P(C.c_double), P(C.c_float)]
        _lib = L
    return _lib


def _check(rc, what):
    if rc != 0:
        raise LegoError("%s failed: rc=%d" % (what, rc))


def params_vlp16(**over):
    p = LegoParams()
    lib().lego_params_vlp16(C.byref(p))
    for k, v in over.items():
        setattr(p, k, v)
    return p


def params_from_yaml(path, **over):
    """lego_params from the reference's loam_config.yaml (lego_params_load_yaml)."""
    p = LegoParams()
    lib().lego_params_vlp16(C.byref(p))
    _check(lib().lego_params_load_yaml(os.fsencode(path), C.byref(p)), "lego_params_load_yaml(%s)" % path)
    for k, v in over.items():
        setattr(p, k, v)
    return p


def params_hdl64(**over):
    p = LegoParams()
    lib().lego_params_hdl64(C.byref(p))
    for k, v in over.items():
        setattr(p, k, v)
    return p


def device_count():
    return int(lib().lego_device_count())


def _save_state(size_fn, save_fn, h, *s):
    n = C.c_size_t()
    _check(size_fn(h, C.byref(n)), "state_size")
    buf = np.zeros(n.value, np.uint8)
    _check(save_fn(h, *s, buf.ctypes.data, n.value), "save_state")
    return buf.tobytes()


def _load_state(load_fn, h, data, *s):
    buf = np.frombuffer(bytes(data), np.uint8).copy()
    _check(load_fn(h, *s, buf.ctypes.data, buf.size), "load_state")


class Frontend:
    """One sequence on one GPU: the drop-in for the reference's ImageProjection + FeatureAssociation."""

    def __init__(self, params=None, device=0):
        self.params = params if params is not None else params_vlp16()
        self.V = self.params.num_vertical_scans
        self.H = self.params.num_horizontal_scans
        h = C.c_void_p()
        _check(lib().lego_ctx_create(C.byref(self.params), int(device), C.byref(h)), "lego_ctx_create")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            lib().lego_ctx_destroy(self.h)
            self.h = None

    __del__ = close

    def cloud_handler(self, pts, point_step=16, off=(0, 4, 8)):
        """ImageProjection::cloudHandler on an (N, 4) float32 x,y,z,intensity array (or raw bytes)."""
        if isinstance(pts, np.ndarray):
            pts = np.ascontiguousarray(pts, dtype=np.float32).reshape(-1, 4)
            n, ptr = pts.shape[0], pts.ctypes.data
        else:
            raise TypeError("pts must be a numpy array")
        out = LegoProjectionOut()
        _check(lib().lego_cloud_handler(self.h, ptr, n, point_step, off[0], off[1], off[2], C.byref(out)),
               "lego_cloud_handler")
        return projection_to_dict(out, self.V, self.H)

    def feature_association(self, proj=None):
        out = LegoAssociationOut()
        if proj is None:
            _check(lib().lego_feature_association(self.h, C.byref(out)), "lego_feature_association")
        else:
            keep = []
            pin = projection_from_dict(proj, keep)
            _check(lib().lego_feature_association_from(self.h, C.byref(pin), C.byref(out)),
                   "lego_feature_association_from")
        return association_to_dict(out)

    def save_state(self):
        """Checkpoint of the sequence's FeatureAssociation state (lego_ctx_save_state) as bytes."""
        return _save_state(lib().lego_ctx_state_size, lib().lego_ctx_save_state, self.h)

    def load_state(self, data):
        """Resume from a checkpoint (lego_ctx_load_state); the next scans continue as the saved sequence's."""
        _load_state(lib().lego_ctx_load_state, self.h, data)

    def set_lm_state(self, transform_cur, transform_sum, degenerate, corner_last, surf_last, tree_stale):
        """Test hook (lego_test_set_lm_state): the LM state the next association starts from."""
        f = lambda a, k: np.ascontiguousarray(np.asarray(a, np.float32).reshape(-1, k))  # noqa: E731
        cur, sm, cl, sl = f(transform_cur, 6), f(transform_sum, 6), f(corner_last, 4), f(surf_last, 4)
        fp = C.POINTER(C.c_float)
        _check(lib().lego_test_set_lm_state(self.h, cur.ctypes.data_as(fp), sm.ctypes.data_as(fp), int(degenerate),
                                            cl.ctypes.data, len(cl), sl.ctypes.data, len(sl), int(tree_stale)),
               "lego_test_set_lm_state")


class Batch:
    """S independent sequences advanced one scan per step (device-resident input)."""

    def __init__(self, params, n_streams, max_points, device=0):
        self.params = params
        self.S = int(n_streams)
        self.V = params.num_vertical_scans
        self.H = params.num_horizontal_scans
        h = C.c_void_p()
        _check(lib().lego_batch_create(C.byref(params), int(device), self.S, int(max_points), C.byref(h)),
               "lego_batch_create")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            lib().lego_batch_destroy(self.h)
            self.h = None

    __del__ = close

    def step(self, d_points, d_offsets, d_counts, stream=0):
        """Device pointers (ints): lego_point array, int64 offsets[S], int32 counts[S]; async on `stream`."""
        _check(lib().lego_batch_step(self.h, C.c_void_p(d_points), C.c_void_p(d_offsets), C.c_void_p(d_counts),
                                     C.c_void_p(stream)), "lego_batch_step")

    def sync(self):
        _check(lib().lego_batch_sync(self.h), "lego_batch_sync")

    def flush(self):
        """Enqueue the pending work of the last steps (LM / lessFlat publish; asynchronous)."""
        _check(lib().lego_batch_flush(self.h), "lego_batch_flush")

    def reset(self):
        _check(lib().lego_batch_reset(self.h), "lego_batch_reset")

    def save_state(self, s):
        """Checkpoint of stream s's FeatureAssociation state (lego_batch_save_state) as bytes."""
        return _save_state(lib().lego_batch_state_size, lib().lego_batch_save_state, self.h, C.c_int32(int(s)))

    def load_state(self, s, data):
        """Stream s resumes from a checkpoint (lego_batch_load_state; any stream of a batch of the same sensor)."""
        _load_state(lib().lego_batch_load_state, self.h, data, C.c_int32(int(s)))

    def set_timing(self, on=True):
        _check(lib().lego_batch_set_timing(self.h, 1 if on else 0), "lego_batch_set_timing")

    def set_groups(self, groups):
        """Launch the streams as `groups` slices on separate HIP streams (overlapping kernel tails)."""
        _check(lib().lego_batch_set_groups(self.h, int(groups)), "lego_batch_set_groups")

    def time_voxel(self, reps=10, stream=0):
        """Mean ms of the last step's VoxelGrid launch, alone on the device (lego_batch_time_voxel)."""
        ms = C.c_float()
        _check(lib().lego_batch_time_voxel(self.h, int(reps), C.c_void_p(stream or None), C.byref(ms)),
               "lego_batch_time_voxel")
        return ms.value

    def set_trajectory(self, d_traj_ptr, max_scans):
        """Per-scan odometry record (lego_batch_set_trajectory): a device array of S * max_scans * 12
        float32 (transformCur, transformSum after each association); (0, 0) stops recording."""
        _check(lib().lego_batch_set_trajectory(self.h, C.c_void_p(d_traj_ptr or None), int(max_scans)),
               "lego_batch_set_trajectory")

    def set_probe(self, on=True):
        """Events around the projection and smoothness stages of every overlap-schedule step."""
        _check(lib().lego_batch_set_probe(self.h, int(bool(on))), "lego_batch_set_probe")

    def probe_times(self):
        """(projection ms, smoothness ms, steps): mean in-pipeline durations since set_probe; clears them."""
        ms = (C.c_float * 2)()
        n = C.c_int32()
        _check(lib().lego_batch_probe_times(self.h, ms, C.byref(n)), "lego_batch_probe_times")
        return float(ms[0]), float(ms[1]), int(n.value)

    def set_lag(self, lag):
        """Pipeline depth: 0 = a step runs its own scan's LM, 1 = the previous scan's, 2 = the one before,
        -1 automatic (the default)."""
        _check(lib().lego_batch_set_lag(self.h, int(lag)), "lego_batch_set_lag")

    def lag(self):
        """The pipeline depth in effect: 0, 1 or 2 (set_lag)."""
        return int(lib().lego_batch_lag(self.h))

    def set_wide(self, mode):
        """Projection / segmentation layout: 1 wide (many workgroups a scan), 0 one workgroup a scan
        (LDS images), 2 one-workgroup projection + wide segmentation, -1 automatic."""
        _check(lib().lego_batch_set_wide(self.h, int(mode)), "lego_batch_set_wide")

    def wide(self):
        """The layout in effect: 0, 1 or 2 (set_wide)."""
        return int(lib().lego_batch_wide(self.h))

    def counts(self):
        """[S, 7] int32: segmented, outlier, scan_msg, sharp, less sharp, flat, less flat counts."""
        out = np.zeros((self.S, 7), dtype=np.int32)
        _check(lib().lego_batch_read_counts(self.h, out.ctypes.data_as(P(C.c_int32))), "lego_batch_read_counts")
        return out

    def time_hbm_stages(self, d_points, d_offsets, d_counts, d_offsets_alt=0, d_counts_alt=0, reps=20, stream=0):
        """Mean ms of one projection + smoothness pair, `reps` launches back to back on the inputs of
        the last step (the same device arrays; the projections alternate with a second input set when
        given); the batch's results are unchanged."""
        ms = C.c_float()
        _check(lib().lego_batch_time_hbm_stages(self.h, int(reps), C.c_void_p(d_points), C.c_void_p(d_offsets),
                                                C.c_void_p(d_counts), C.c_void_p(d_offsets_alt or None),
                                                C.c_void_p(d_counts_alt or None), C.c_void_p(stream), C.byref(ms)),
               "lego_batch_time_hbm_stages")
        return ms.value

    def stage_times(self):
        ms = (C.c_float * 6)()
        _check(lib().lego_batch_stage_times(self.h, ms), "lego_batch_stage_times")
        return list(ms)

    def read(self, s):
        po, ao = LegoProjectionOut(), LegoAssociationOut()
        _check(lib().lego_batch_read(self.h, int(s), C.byref(po), C.byref(ao)), "lego_batch_read")
        return projection_to_dict(po, self.V, self.H), association_to_dict(ao)

    def poses(self):
        out = np.zeros((self.S, 12), dtype=np.float32)
        st = np.zeros(self.S, dtype=np.int32)
        _check(lib().lego_batch_read_poses(self.h, out.ctypes.data_as(P(C.c_float)), st.ctypes.data_as(P(C.c_int32))),
               "lego_batch_read_poses")
        return out, st


class ScanToMap:
    """MapOptimization's scan-to-map LM (scan2MapOptimization, mapOptmization.cpp:1315-1332) on the GPU.

    run_host(): one problem from host clouds, as the reference's mapping thread calls it per scan.
    run():      many problems from device arrays (lego_s2m_io), one workgroup each.
    """

    def __init__(self, max_problems=1, max_map_points=200000, device=0):
        h = C.c_void_p()
        _check(lib().lego_s2m_create(int(device), int(max_problems), int(max_map_points), C.byref(h)),
               "lego_s2m_create")
        self.h = h
        self.max_problems = int(max_problems)

    def close(self):
        if getattr(self, "h", None):
            lib().lego_s2m_destroy(self.h)
            self.h = None

    __del__ = close

    def run_host(self, corner, surf, corner_map, surf_map, transform, degenerate=0):
        """Returns (transform[6] float32, degenerate, info[4] int32)."""
        arrs = [np.ascontiguousarray(np.asarray(a, np.float32).reshape(-1, 4)) for a in (corner, surf, corner_map,
                                                                                          surf_map)]
        t = np.ascontiguousarray(np.asarray(transform, np.float32).reshape(6).copy())
        dg = C.c_int32(int(degenerate))
        info = np.zeros(4, np.int32)
        args = []
        for a in arrs:
            args += [C.c_void_p(a.ctypes.data), len(a)]
        _check(lib().lego_s2m_run_host(self.h, *args, t.ctypes.data_as(P(C.c_float)), C.byref(dg),
                                       info.ctypes.data_as(P(C.c_int32))), "lego_s2m_run_host")
        return t, dg.value, info

    def run(self, n, io, stream=0):
        """n problems described by a LegoS2mIo of device pointers; asynchronous on `stream`."""
        _check(lib().lego_s2m_run(self.h, int(n), C.byref(io), C.c_void_p(stream)), "lego_s2m_run")

    def set_layout(self, layout):
        """lego_s2m_run's launch layout: 0 a workgroup a problem, 1 latency, -1 automatic (<= 16: latency)."""
        _check(lib().lego_s2m_set_layout(self.h, int(layout)), "lego_s2m_set_layout")

    def map_transform(self, n, io, stream=0):
        """transformPointCloud of n parts (LegoMapTransformIo of device pointers); asynchronous."""
        _check(lib().lego_map_transform(self.h, int(n), C.byref(io), C.c_void_p(stream)), "lego_map_transform")

    def map_voxel(self, n, io, stream=0):
        """pcl::VoxelGrid::filter of n clouds (LegoMapVoxelIo of device pointers); asynchronous (tie order 1;
        order 0 synchronizes `stream` once per device-wide sort level)."""
        _check(lib().lego_map_voxel(self.h, int(n), C.byref(io), C.c_void_p(stream)), "lego_map_voxel")

    def set_voxel_tie_order(self, order):
        """map_voxel's tie order: 0 (default) PCL's std::sort permutation (the reference), 1 std::stable_sort's."""
        _check(lib().lego_s2m_set_voxel_tie_order(self.h, int(order)), "lego_s2m_set_voxel_tie_order")


class Mapper:
    """MapOptimization's mapping thread (mapOptmization.cpp:1521-1570, loop closure off) for one
    sequence: step() takes one AssociationOut's clouds and transformSum and returns transformAftMapped;
    the key frames' downsampled clouds stay in device memory (lego_mapper_*, include/lego_s2m.h)."""

    def __init__(self, max_map_points=200000, max_key_points=50_000_000, device=0, voxel_tie_order=0):
        h = C.c_void_p()
        _check(lib().lego_mapper_create(int(device), int(max_map_points), int(max_key_points), C.byref(h)),
               "lego_mapper_create")
        self.h = h
        _check(lib().lego_mapper_set_voxel_tie_order(self.h, int(voxel_tie_order)), "lego_mapper_set_voxel_tie_order")

    def close(self):
        if getattr(self, "h", None):
            lib().lego_mapper_destroy(self.h)
            self.h = None

    __del__ = close

    def step(self, corner_last, surf_last, outlier_last, transform_sum):
        """transform_sum: the mapping thread's transformSum (OdometryToTransform of the odometry message,
        lego_amd.mapping.odometry_to_transform).  Returns (transformAftMapped[6] float32, info[4] int32 as
        lego_s2m_run's)."""
        arrs = [np.ascontiguousarray(np.asarray(a, np.float32).reshape(-1, 4)) for a in (corner_last, surf_last,
                                                                                          outlier_last)]
        ts = np.ascontiguousarray(np.asarray(transform_sum, np.float32).reshape(6))
        out = np.zeros(6, np.float32)
        info = np.zeros(4, np.int32)
        args = []
        for a in arrs:
            args += [C.c_void_p(a.ctypes.data), len(a)]
        _check(lib().lego_mapper_step(self.h, *args, ts.ctypes.data_as(P(C.c_float)), out.ctypes.data_as(P(C.c_float)),
                                      info.ctypes.data_as(P(C.c_int32))), "lego_mapper_step")
        return out, info

    def key_poses(self):
        """cloudKeyPoses6D as an (n, 6) float32 array of (roll, pitch, yaw, x, y, z)."""
        n = C.c_int32()
        _check(lib().lego_mapper_key_poses(self.h, None, 0, C.byref(n)), "lego_mapper_key_poses")
        out = np.zeros((max(n.value, 1), 6), np.float32)
        _check(lib().lego_mapper_key_poses(self.h, out.ctypes.data_as(P(C.c_float)), n.value, C.byref(n)),
               "lego_mapper_key_poses")
        return out[:n.value]
