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


# ---- the same preparation on the GPU (lego_map_transform / lego_map_voxel) ---------------------------
SCAN_CLOUDS = ("corner", "surf", "corner_map", "surf_map")


def _parts(frames, k, n_keys):
    """The clouds build_problem assembles, as (key-frame parts, current-scan clouds)."""
    lo = max(0, k - n_keys)
    corner_parts = [(frames[j]["corner_last"], frames[j]["transform_sum"]) for j in range(lo, k)]
    surf_parts = []
    for j in range(lo, k):  # per key frame: its surf cloud, then its outlier cloud (:909-913, :982-986)
        surf_parts += [(frames[j]["surf_last"], frames[j]["transform_sum"]),
                       (frames[j]["outlier_last"], frames[j]["transform_sum"])]
    f = frames[k]
    return corner_parts, surf_parts, (f["corner_last"], f["surf_last"], f["outlier_last"])


def prepare_gpu(s2m, sequences, k, n_keys=10, perturb=(0.002, 0.002, 0.004, 0.03, 0.01, 0.03), stream=0,
                events=None):
    """GPU version of build_problem for many sequences at once: the scan-to-map problem of scan k of
    every sequence (a list of AssociationOut-like records per sequence), built on the device with
    lego_map_transform (key frames into the map frame, concatenated) and lego_map_voxel (the
    reference's leaves; downsampleCurrentScan's surf total = VoxelGrid(VoxelGrid(surf) ++
    VoxelGrid(outlier))).  Two launches of each, one host read of the first VoxelGrid's counts.

    Returns (io, keep, transform, degenerate, info, views): a LegoS2mIo for ScanToMap.run, the tensors
    behind it, the transform / degenerate / info tensors it points at, and the VoxelGrid outputs
    (for tests).  events = (start, end) torch.cuda.Events are recorded around the device work (after the
    key frames' upload; including the count read between the two VoxelGrid launches).
    """
    cparts, sparts, scans = zip(*[_parts(seq, k, n_keys) for seq in sequences])
    t0 = np.stack([np.asarray(seq[k]["transform_sum"], np.float32) + np.asarray(perturb, np.float32)
                   for seq in sequences]).astype(np.float32)
    return prepare_parts_gpu(s2m, cparts, sparts, scans, t0, stream=stream, events=events)


def prepare_parts_gpu(s2m, cparts, sparts, scans, t0, degenerate=None, stream=0, events=None):
    """prepare_gpu on explicit inputs, per problem p: cparts[p] / sparts[p] = [(cloud, key pose), ...]
    (the surrounding key frames' corner clouds; their surf and outlier clouds, frame by frame), scans[p]
    = (corner, surf, outlier) of the current scan, t0[p] = transformTobeMapped before the optimisation,
    degenerate[p] = isDegenerate."""
    import torch
    from . import LegoMapTransformIo, LegoMapVoxelIo, LegoS2mIo
    P_ = len(scans)
    dev = "cuda"
    f32 = lambda a: np.ascontiguousarray(np.asarray(a, np.float32).reshape(-1, 4))  # noqa: E731

    # 1. key-frame parts of every problem: corner map parts, then surf map parts
    parts = [(f32(c), t) for pp in cparts for (c, t) in pp] + [(f32(c), t) for pp in sparts for (c, t) in pp]
    n_c = [sum(len(f32(c)) for c, _ in pp) for pp in cparts]
    n_s = [sum(len(f32(c)) for c, _ in pp) for pp in sparts]
    sizes = np.array([len(a) for a, _ in parts], np.int32)
    in_off = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    raw = torch.from_numpy(np.concatenate([a for a, _ in parts]) if len(parts) else np.zeros((1, 4), np.float32)).to(dev)
    poses = torch.from_numpy(np.stack([np.asarray(t, np.float32) for _, t in parts]) if parts
                             else np.zeros((1, 6), np.float32)).to(dev)
    # concatenated outputs: problem p's corner map raw cloud, then (after all of them) surf map raw clouds
    map_raw = torch.empty((max(1, int(sizes.sum())), 4), dtype=torch.float32, device=dev)
    keep = [raw, poses, map_raw]
    t_io = LegoMapTransformIo()
    t_in_off = torch.from_numpy(in_off).to(dev)
    t_in_n = torch.from_numpy(sizes).to(dev)
    keep += [t_in_off, t_in_n]
    t_io.in_, t_io.in_off, t_io.in_n, t_io.pose = raw.data_ptr(), t_in_off.data_ptr(), t_in_n.data_ptr(), poses.data_ptr()
    t_io.out, t_io.out_off = map_raw.data_ptr(), t_in_off.data_ptr()  # parts land next to each other
    sc = [f32(x) for tri in scans for x in tri]  # per problem: corner, surf, outlier
    scan_raw = torch.from_numpy(np.concatenate(sc) if sc else np.zeros((1, 4), np.float32)).to(dev)
    sc_n = np.array([len(a) for a in sc], np.int32)
    if events is not None:
        events[0].record()
    if parts:
        s2m.map_transform(len(parts), t_io, stream)

    # 2. VoxelGrid: corner maps (0.2), surf maps (0.4), the scans' corner (0.2), surf (0.4), outlier (0.4)
    sc_off = np.concatenate([[0], np.cumsum(sc_n)[:-1]]).astype(np.int64)
    # the voxel inputs as (base tensor, offset) pairs: map clouds live in map_raw, scans in scan_raw
    c_off = np.concatenate([[0], np.cumsum(n_c)[:-1]]).astype(np.int64)
    s_off = int(sum(n_c)) + np.concatenate([[0], np.cumsum(n_s)[:-1]]).astype(np.int64)
    # one input base for the launch: map_raw ++ scan_raw
    both = torch.cat([map_raw[:int(sizes.sum())], scan_raw[:int(sc_n.sum())]]) if sizes.sum() or sc_n.sum() \
        else torch.zeros((1, 4), dtype=torch.float32, device=dev)
    base_sc = int(sizes.sum())
    v_off = np.concatenate([c_off, s_off, base_sc + sc_off]).astype(np.int64)
    v_n = np.concatenate([n_c, n_s, sc_n]).astype(np.int32)
    leaf = np.concatenate([np.full(P_, 0.2), np.full(P_, 0.4),
                           np.tile(np.array([0.2, 0.4, 0.4]), P_)]).astype(np.float32)
    nv = len(v_n)
    v_out = torch.empty((max(1, int(v_n.sum())), 4), dtype=torch.float32, device=dev)
    out_off = np.concatenate([[0], np.cumsum(v_n)[:-1]]).astype(np.int64)
    tens = {n: torch.from_numpy(a).to(dev) for n, a in (("off", v_off), ("n", v_n), ("leaf", leaf), ("oo", out_off))}
    out_n = torch.zeros(nv, dtype=torch.int32, device=dev)
    status = torch.zeros(nv, dtype=torch.int32, device=dev)
    keep += [scan_raw, both, v_out, out_n, status] + list(tens.values())
    v_io = LegoMapVoxelIo()
    v_io.in_, v_io.in_off, v_io.in_n, v_io.leaf = both.data_ptr(), tens["off"].data_ptr(), tens["n"].data_ptr(), \
        tens["leaf"].data_ptr()
    v_io.out, v_io.out_off, v_io.out_n, v_io.status = v_out.data_ptr(), tens["oo"].data_ptr(), out_n.data_ptr(), \
        status.data_ptr()
    s2m.map_voxel(nv, v_io, stream)
    on = out_n.cpu().numpy()  # the one host read: where the surf total clouds start

    # 3. surf total = VoxelGrid(surf DS ++ outlier DS) of each scan (leaf 0.4)
    i_sd = 2 * P_ + 3 * np.arange(P_) + 1  # the scans' surf DS entries; outlier DS follows each
    tot_n = (on[i_sd] + on[i_sd + 1]).astype(np.int32)
    tot_off = np.concatenate([[0], np.cumsum(tot_n)[:-1]]).astype(np.int64)
    tot_raw = torch.empty((max(1, int(tot_n.sum())), 4), dtype=torch.float32, device=dev)
    # concatenation by the identity transform (cos 0 = 1, sin 0 = 0: every coordinate copied exactly)
    cat_in_off = np.stack([out_off[i_sd], out_off[i_sd + 1]], 1).reshape(-1).astype(np.int64)
    cat_n = np.stack([on[i_sd], on[i_sd + 1]], 1).reshape(-1).astype(np.int32)
    cat_out_off = np.stack([tot_off, tot_off + on[i_sd]], 1).reshape(-1).astype(np.int64)
    ident = torch.zeros((2 * P_, 6), dtype=torch.float32, device=dev)
    ct = {n: torch.from_numpy(a).to(dev) for n, a in (("io", cat_in_off), ("n", cat_n), ("oo", cat_out_off))}
    keep += [tot_raw, ident] + list(ct.values())
    c_io = LegoMapTransformIo()
    c_io.in_, c_io.in_off, c_io.in_n, c_io.pose = v_out.data_ptr(), ct["io"].data_ptr(), ct["n"].data_ptr(), \
        ident.data_ptr()
    c_io.out, c_io.out_off = tot_raw.data_ptr(), ct["oo"].data_ptr()
    s2m.map_transform(2 * P_, c_io, stream)
    t2 = {n: torch.from_numpy(a).to(dev) for n, a in (("off", tot_off), ("n", tot_n),
                                                       ("leaf", np.full(P_, 0.4, np.float32)))}
    tot_out = torch.empty_like(tot_raw)
    tot_on = torch.zeros(P_, dtype=torch.int32, device=dev)
    tot_st = torch.zeros(P_, dtype=torch.int32, device=dev)
    keep += [tot_out, tot_on, tot_st] + list(t2.values())
    v2 = LegoMapVoxelIo()
    v2.in_, v2.in_off, v2.in_n, v2.leaf = tot_raw.data_ptr(), t2["off"].data_ptr(), t2["n"].data_ptr(), \
        t2["leaf"].data_ptr()
    v2.out, v2.out_off, v2.out_n, v2.status = tot_out.data_ptr(), t2["off"].data_ptr(), tot_on.data_ptr(), \
        tot_st.data_ptr()
    s2m.map_voxel(P_, v2, stream)
    if events is not None:
        events[1].record()

    # 4. the scan-to-map io: corner map / surf map / scan corner from the first VoxelGrid, surf total from the second
    oo = torch.from_numpy(out_off).to(dev)
    keep.append(oo)
    io = LegoS2mIo()
    co, cn = oo[2 * P_::3].contiguous(), out_n[2 * P_::3].contiguous()
    keep += [co, cn]
    io.corner, io.corner_off, io.corner_n = v_out.data_ptr(), co.data_ptr(), cn.data_ptr()
    io.surf, io.surf_off, io.surf_n = tot_out.data_ptr(), t2["off"].data_ptr(), tot_on.data_ptr()
    cmo, cmn = oo[:P_].contiguous(), out_n[:P_].contiguous()
    smo, smn = oo[P_:2 * P_].contiguous(), out_n[P_:2 * P_].contiguous()
    keep += [cmo, cmn, smo, smn]
    io.corner_map, io.corner_map_off, io.corner_map_n = v_out.data_ptr(), cmo.data_ptr(), cmn.data_ptr()
    io.surf_map, io.surf_map_off, io.surf_map_n = v_out.data_ptr(), smo.data_ptr(), smn.data_ptr()
    tr = torch.from_numpy(np.ascontiguousarray(np.asarray(t0, np.float32).reshape(P_, 6))).to(dev)
    dg = (torch.from_numpy(np.asarray(degenerate, np.int32)).to(dev) if degenerate is not None
          else torch.zeros(P_, dtype=torch.int32, device=dev))
    info = torch.zeros((P_, 4), dtype=torch.int32, device=dev)
    keep += [tr, dg, info]
    io.transform, io.degenerate, io.info = tr.data_ptr(), dg.data_ptr(), info.data_ptr()
    views = {"v_out": v_out, "out_off": out_off, "out_n": out_n, "tot_out": tot_out, "tot_off": tot_off,
             "tot_n": tot_on, "status": status, "tot_status": tot_st}
    return io, keep, tr, dg, info, views


# ---- MapOptimization's mapping loop around the GPU operations ---------------------------------------
def odometry_to_transform(orientation, position):
    """OdometryToTransform (utility.h:96-110): the mapping thread's transformSum from the odometry
    message (AssociationOut.laser_odometry: orientation x, y, z, w and position; the assoc dicts'
    odom_orientation / odom_position), through tf's getRPY in double.  Product library
    (lego_map_odometry_to_transform)."""
    import ctypes as C
    import lego_amd as LA
    q = np.ascontiguousarray(np.asarray(orientation, np.float64).reshape(4))
    p = np.ascontiguousarray(np.asarray(position, np.float64).reshape(3))
    t = np.zeros(6, np.float32)
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
    LA._check(LA.lib().lego_map_odometry_to_transform(dp(q), dp(p), t.ctypes.data_as(C.POINTER(C.c_float))),
              "lego_map_odometry_to_transform")
    return t


def transform_associate_to_map(tSum, tBef, tAft):
    """transformAssociateToMap (mapOptmization.cpp:264-387): the odometry increment since the last mapping
    step applied to the last mapped pose; returns transformTobeMapped.  Runs in the product library
    (lego_map_associate: float, the float libm the reference's build calls)."""
    import ctypes as C
    import lego_amd as LA
    S, B, A = [np.ascontiguousarray(np.asarray(t, np.float32).reshape(6)) for t in (tSum, tBef, tAft)]
    T = np.zeros(6, np.float32)
    fp = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))  # noqa: E731
    LA._check(LA.lib().lego_map_associate(fp(S), fp(B), fp(A), fp(T)), "lego_map_associate")
    return T


def voxel_grid_small(points, leaf):
    """pcl::VoxelGrid::applyFilter for small clouds on the host (the 1 m key-pose filter, :78, :930-931):
    float32 leaf indices, float32 sums in point order (stable tie order), ascending leaf order."""
    p = np.asarray(points, np.float32).reshape(-1, 4)
    if len(p) == 0:
        return p.copy()
    inv = np.float32(1.0) / np.float32(leaf)
    mn, mx = p[:, :3].min(0), p[:, :3].max(0)
    min_b = np.floor(mn * inv).astype(np.int64)
    div = np.floor(mx * inv).astype(np.int64) - min_b + 1
    ijk = (np.floor(p[:, :3] * inv) - min_b.astype(np.float32)).astype(np.int64)
    key = ijk[:, 0] + ijk[:, 1] * div[0] + ijk[:, 2] * div[0] * div[1]
    out = []
    for kv in np.unique(key):
        acc = np.zeros(4, np.float32)
        idx = np.flatnonzero(key == kv)
        for i in idx:
            acc = (acc + p[i]).astype(np.float32)
        out.append((acc / np.float32(len(idx))).astype(np.float32))
    return np.array(out, np.float32)


class MapSequence:
    """MapOptimization::run (mapOptmization.cpp:1521-1570) for one sequence, loop closure off (the
    reference's default, loam_config.yaml:24), host side: transformAssociateToMap,
    extractSurroundingKeyFrames (:915-995: key poses within 50 m, their 1 m VoxelGrid, the existing
    key-frame list kept in the reference's order), the inputs of downsampleCurrentScan, and after the
    scan-to-map LM transformUpdate and saveKeyFramesAndFactor (:1335-1478).  GTSAM is left out: with no
    loop closure its graph is a chain whose optimum is the inserted pose itself, so the key pose is
    transformAftMapped (the reference's Rot3 round trip aside).  The clouds' transforms and VoxelGrids
    and the LM run batched over many sequences (MappingBatch)."""

    RADIUS = 50.0  # surrounding_keyframe_search_radius (loam_config.yaml:27)

    def __init__(self, associate=None, odometry=None):
        self._associate = associate or transform_associate_to_map  # tests pass the oracle's
        self._odometry = odometry or odometry_to_transform
        z = lambda: np.zeros(6, np.float32)  # noqa: E731
        self.t_sum, self.t_tobe, self.t_bef, self.t_aft = z(), z(), z(), z()
        self.key_pos = []       # cloudKeyPoses3D: (x, y, z, index)
        self.key_pose6 = []     # cloudKeyPoses6D as (roll, pitch, yaw, x, y, z)
        self.key_clouds = []    # (corner DS, surf DS, outlier DS) per key frame, lidar frame
        self.existing = []      # surroundingExistingKeyPosesID
        self.cur_pos = np.zeros(3, np.float32)
        self.prev_pos = np.zeros(3, np.float32)
        self.degenerate = 0
        self.cycles = 0

    def begin(self, assoc):
        """One AssociationOut: returns (corner parts, surf parts, scan clouds, transformTobeMapped)."""
        self.t_sum = self._odometry(assoc["odom_orientation"], assoc["odom_position"])  # OdometryToTransform (:1540)
        self.t_tobe = self._associate(self.t_sum, self.t_bef, self.t_aft)
        if self.key_pos:  # extractSurroundingKeyFrames, loop closure off (:915-995)
            kp = np.array(self.key_pos, np.float32)
            d = ((kp[:, 0] - self.cur_pos[0]) ** 2 + (kp[:, 1] - self.cur_pos[1]) ** 2) + (kp[:, 2] - self.cur_pos[2]) ** 2
            sel = np.flatnonzero(d < np.float32(self.RADIUS * self.RADIUS))
            sel = sel[np.argsort(d[sel], kind="stable")]  # radiusSearch, sorted by distance
            ds = voxel_grid_small(kp[sel], 1.0)
            ids = [int(x) for x in ds[:, 3]]
            self.existing = [i for i in self.existing if i in ids]
            for i in ids:
                if i not in self.existing:
                    self.existing.append(i)
        corner_parts = [(self.key_clouds[i][0], self.key_pose6[i]) for i in self.existing]
        surf_parts = []
        for i in self.existing:
            surf_parts += [(self.key_clouds[i][1], self.key_pose6[i]), (self.key_clouds[i][2], self.key_pose6[i])]
        scan = (assoc["corner_last"], assoc["surf_last"], assoc["outlier_last"])
        return corner_parts, surf_parts, scan, self.t_tobe.copy()

    def end(self, transform, degenerate, info, scan_ds):
        """After the LM: scan_ds = (corner DS, surf DS, outlier DS) of the current scan."""
        self.t_tobe = np.asarray(transform, np.float32).copy()
        self.degenerate = int(degenerate)
        if info[0] == 1:  # transformUpdate (:389-395), inside scan2MapOptimization's gate
            self.t_bef = self.t_sum.copy()
            self.t_aft = self.t_tobe.copy()
        # saveKeyFramesAndFactor (:1335-1478) without GTSAM
        self.cur_pos = self.t_aft[3:6].copy()
        dd = self.prev_pos - self.cur_pos
        moved = float(np.sqrt(dd[0] * dd[0] + dd[1] * dd[1] + dd[2] * dd[2])) >= 0.3  # float distance vs double 0.3
        self.cycles += 1
        if not moved and self.key_pos:
            return
        self.prev_pos = self.cur_pos.copy()
        # the first key frame is the prior at transformTobeMapped (:1361-1376), later ones the chain's
        # estimate at transformAftMapped (:1381-1406, :1424-1426)
        pose = (self.t_tobe if not self.key_pos else self.t_aft).copy()
        self.key_pos.append((pose[3], pose[4], pose[5], float(len(self.key_pos))))
        self.key_pose6.append(pose)
        if len(self.key_pos) > 1:  # :1447-1459
            self.t_tobe = self.t_aft.copy()
        self.key_clouds.append(tuple(np.asarray(c, np.float32).reshape(-1, 4).copy() for c in scan_ds))


def mapping_step_gpu(s2m, seqs, assocs, stream=0):
    """One mapping cycle of every sequence in `seqs` (MapSequence) on its AssociationOut: the key
    frames' transforms and all VoxelGrids (lego_map_transform / lego_map_voxel) and the scan-to-map LM
    (lego_s2m_run) in batched launches.  Returns the per-sequence (transform, degenerate, info)."""
    import torch
    begun = [sq.begin(a) for sq, a in zip(seqs, assocs)]
    cparts, sparts, scans, t0 = zip(*begun)
    io, keep, tr, dg, info, v = prepare_parts_gpu(s2m, cparts, sparts, scans, np.stack(t0),
                                                  degenerate=[sq.degenerate for sq in seqs], stream=stream)
    s2m.run(len(seqs), io, stream)
    torch.cuda.synchronize()
    P_ = len(seqs)
    vo, oo, on = v["v_out"].cpu().numpy(), v["out_off"], v["out_n"].cpu().numpy()
    t, d, inf = tr.cpu().numpy(), dg.cpu().numpy(), info.cpu().numpy()
    for p, sq in enumerate(seqs):
        b = 2 * P_ + 3 * p  # the scan's corner, surf, outlier DS
        ds = tuple(vo[oo[b + i]:oo[b + i] + on[b + i]] for i in range(3))
        sq.end(t[p], d[p], inf[p], ds)
    return [(t[p], int(d[p]), inf[p]) for p in range(P_)]
