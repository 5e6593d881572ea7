"""Host-side assembly of scan-to-map problems (the caller's side of include/lego_s2m.h).

MapOptimization (mapOptmization.cpp) prepares the four clouds scan2MapOptimization works on before
calling it; ScanToMap takes them ready-made.  This module restates that preparation in simplified
form, for examples, tests and benchmarks:

  * pointAssociateToMap (:412-426) in numpy float32, used to put key frames into the map frame
    (the reference's transformPointCloud, :428-508, with the key pose in the same Euler convention);
  * a VoxelGrid stand-in (one centroid per occupied leaf, in leaf order) for the map and scan
    downsampling (:71-73 leaves 0.2 / 0.4 m; :988-1025);
  * build_problem(): the surrounding map from the previous key frames' corner / surf + outlier clouds
    (the loop-closure-disabled path of extractSurroundingKeyFrames, :915-995, with every earlier frame
    inside the search radius taken as a key frame) and the current scan's downsampled clouds
    (downsampleCurrentScan, :999-1026).

The clouds' exact values do not matter to the parity tests, which feed the same arrays to the GPU
and to the oracle; only their realism does.
"""
import numpy as np


def associate_to_map(points, t):
    """pointAssociateToMap of an (N, 4) float32 cloud with transform t[6] (roll, pitch, yaw, x, y, z)."""
    p = np.asarray(points, np.float32).reshape(-1, 4)
    t = np.asarray(t, np.float32)
    cr, sr = np.float32(np.cos(t[0])), np.float32(np.sin(t[0]))
    cp, sp = np.float32(np.cos(t[1])), np.float32(np.sin(t[1]))
    cy, sy = np.float32(np.cos(t[2])), np.float32(np.sin(t[2]))
    x1 = cy * p[:, 0] - sy * p[:, 1]
    y1 = sy * p[:, 0] + cy * p[:, 1]
    z1 = p[:, 2]
    y2 = cr * y1 - sr * z1
    z2 = sr * y1 + cr * z1
    out = np.empty_like(p)
    out[:, 0] = cp * x1 + sp * z2 + t[3]
    out[:, 1] = y2 + t[4]
    out[:, 2] = -sp * x1 + cp * z2 + t[5]
    out[:, 3] = p[:, 3]
    return out


def voxel_downsample(points, leaf):
    """One centroid (x, y, z, intensity) per occupied leaf^3 voxel, in ascending voxel order."""
    p = np.asarray(points, np.float32).reshape(-1, 4)
    if len(p) == 0:
        return p.copy()
    inv = np.float32(1.0 / leaf)
    ijk = np.floor(p[:, :3] * inv).astype(np.int64)
    ijk -= ijk.min(axis=0)
    dims = ijk.max(axis=0) + 1
    key = ijk[:, 0] + ijk[:, 1] * dims[0] + ijk[:, 2] * dims[0] * dims[1]
    order = np.argsort(key, kind="stable")
    key_s = key[order]
    starts = np.flatnonzero(np.r_[True, key_s[1:] != key_s[:-1]])
    sums = np.add.reduceat(p[order].astype(np.float64), starts, axis=0)
    cnt = np.diff(np.r_[starts, len(key_s)]).astype(np.float64)
    return (sums / cnt[:, None]).astype(np.float32)


def build_problem(frames, k, n_keys=10, perturb=(0.002, 0.002, 0.004, 0.03, 0.01, 0.03)):
    """Scan-to-map problem for frame k of a sequence.

    frames: list of dicts with "corner_last", "surf_last", "outlier_last" ((N, 4) float32, the scan-end
    frame) and "transform_sum" (6 floats): e.g. AssociationOut records of lego_amd.Frontend / Batch.
    The map holds frames max(0, k - n_keys) .. k-1 put into the map frame by their transform_sum; the
    initial guess is frame k's transform_sum plus `perturb`.  Returns a dict of the four clouds and
    the initial transform.
    """
    lo = max(0, k - n_keys)
    cm = [associate_to_map(frames[j]["corner_last"], frames[j]["transform_sum"]) for j in range(lo, k)]
    sm = [associate_to_map(np.concatenate([frames[j]["surf_last"], frames[j]["outlier_last"]]),
                           frames[j]["transform_sum"]) for j in range(lo, k)]
    corner_map = voxel_downsample(np.concatenate(cm), 0.2)
    surf_map = voxel_downsample(np.concatenate(sm), 0.4)
    f = frames[k]
    corner = voxel_downsample(f["corner_last"], 0.2)
    surf_total = np.concatenate([voxel_downsample(f["surf_last"], 0.4), voxel_downsample(f["outlier_last"], 0.4)])
    surf = voxel_downsample(surf_total, 0.4)
    t0 = np.asarray(f["transform_sum"], np.float32) + np.asarray(perturb, np.float32)
    return {"corner": corner, "surf": surf, "corner_map": corner_map, "surf_map": surf_map,
            "transform": t0.astype(np.float32)}
