"""GPU parity of the map-side cloud preparation (include/lego_s2m.h: lego_map_transform, lego_map_voxel).

MapOptimization builds the clouds scan2MapOptimization consumes with transformPointCloud
(mapOptmization.cpp:443-473) and pcl::VoxelGrid (leaves :71-78; extractSurroundingKeyFrames :857-996,
downsampleCurrentScan :999-1026).  Bar: bit-exact against the oracle's restatements (VoxelGrid in both
tie orders: PCL's std::sort permutation, the reference's, and std::stable_sort's), then the whole
GPU-prepared problem through the scan-to-map LM within 1e-4 of the oracle-prepared one.
"""
import numpy as np
import pytest

import oracle as O
from lego_amd import _abi as A
from lego_amd import mapping as M

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def s2m(gpu):
    import lego_amd as LA
    m = LA.ScanToMap(max_problems=8, max_map_points=120000, device=gpu)
    yield m
    m.close()


def _frames(seq, n):
    import lego_amd as LA
    orc = O.Oracle(LA.params_vlp16())
    cfg = A.synth_cfg("vlp16")
    out = []
    for k in range(n):
        orc.cloud_handler(A.synth_scan(cfg, seq, k))
        out.append(orc.feature_association())
    return out


@pytest.fixture(scope="module")
def sequences():
    return [_frames(seq, 6) for seq in (2, 5, 9)]


def _gpu_voxel(s2m, clouds, leaves):
    import torch
    import lego_amd as LA
    cl = [np.ascontiguousarray(np.asarray(c, np.float32).reshape(-1, 4)) for c in clouds]
    n = np.array([len(c) for c in cl], np.int32)
    off = np.concatenate([[0], np.cumsum(n)[:-1]]).astype(np.int64)
    flat = torch.from_numpy(np.concatenate(cl) if n.sum() else np.zeros((1, 4), np.float32)).cuda()
    t_off, t_n = torch.from_numpy(off).cuda(), torch.from_numpy(n).cuda()
    leaf = torch.from_numpy(np.asarray(leaves, np.float32)).cuda()
    out = torch.zeros((max(1, int(n.sum())), 4), dtype=torch.float32, device="cuda")
    out_n = torch.zeros(len(cl), dtype=torch.int32, device="cuda")
    st = torch.zeros(len(cl), dtype=torch.int32, device="cuda")
    io = LA.LegoMapVoxelIo()
    io.in_, io.in_off, io.in_n, io.leaf = flat.data_ptr(), t_off.data_ptr(), t_n.data_ptr(), leaf.data_ptr()
    io.out, io.out_off, io.out_n, io.status = out.data_ptr(), t_off.data_ptr(), out_n.data_ptr(), st.data_ptr()
    s2m.map_voxel(len(cl), io)
    torch.cuda.synchronize()
    o, on, so = out.cpu().numpy(), out_n.cpu().numpy(), st.cpu().numpy()
    return [(o[off[i]:off[i] + max(on[i], 0)], int(on[i]), int(so[i])) for i in range(len(cl))]


@pytest.mark.parametrize("order", [0, 1])
def test_voxel_matches_oracle(s2m, sequences, order):
    s2m.set_voxel_tie_order(order)
    fr = sequences[0]
    rng = np.random.default_rng(11)
    big = np.concatenate([M.associate_to_map(np.concatenate([f["surf_last"], f["outlier_last"]]), f["transform_sum"])
                          for f in fr[:5]])
    clouds = [fr[3]["corner_last"], fr[3]["surf_last"], fr[3]["outlier_last"], big,
              rng.uniform(-20, 20, (5000, 4)).astype(np.float32),  # sparse: mostly single-point leaves
              np.repeat(rng.uniform(-1, 1, (50, 4)).astype(np.float32), 40, axis=0),  # 40 copies per point
              np.zeros((0, 4), np.float32), rng.uniform(-1, 1, (1, 4)).astype(np.float32)]
    for leaf in (0.2, 0.4, 1.0):
        got = _gpu_voxel(s2m, clouds, [leaf] * len(clouds))
        for c, (o, on, st) in zip(clouds, got):
            ref, rst = O.voxel_grid(c, leaf, stable=order == 1)
            assert st == rst and on == len(ref), (leaf, len(c), on, len(ref))
            assert np.array_equal(o.view(np.int32), ref.view(np.int32)), (leaf, len(c))


@pytest.mark.parametrize("order", [0, 1])
def test_voxel_both_sort_layouts(s2m, sequences, order):
    """Order 1: few clouds take one device-wide radix sort (64-bit cloud|leaf keys), many clouds rocPRIM's
    segmented sort; order 0: one range list over all clouds.  The same clouds give the oracle's output."""
    s2m.set_voxel_tie_order(order)
    fr = sequences[1]
    rng = np.random.default_rng(17)
    base = [fr[4]["corner_last"], fr[4]["surf_last"], np.zeros((0, 4), np.float32),
            np.repeat(rng.uniform(-1, 1, (30, 4)).astype(np.float32), 7, axis=0)]
    many = base + [rng.uniform(-5, 5, (int(rng.integers(0, 300)), 4)).astype(np.float32) for _ in range(66)]
    for clouds in (base, many):  # 4 clouds: device-wide; 70 clouds: segmented
        got = _gpu_voxel(s2m, clouds, [0.4] * len(clouds))
        for c, (o, on, st) in zip(clouds, got):
            ref, rst = O.voxel_grid(c, 0.4, stable=order == 1)
            assert st == rst and on == len(ref) and np.array_equal(o.view(np.int32), ref.view(np.int32)), len(clouds)


@pytest.mark.parametrize("order", [0, 1])
def test_voxel_limits(s2m, order):
    s2m.set_voxel_tie_order(order)
    rng = np.random.default_rng(12)
    wide = rng.uniform(-1000, 1000, (2000, 4)).astype(np.float32)  # 1e-3 leaves: indices overflow int32
    huge = np.zeros((130000, 4), np.float32)                       # above max_map_points
    got = _gpu_voxel(s2m, [wide, huge], [1e-3, 0.2])
    ref, rst = O.voxel_grid(wide, 1e-3, stable=order == 1)
    assert got[0][2] == rst == 0x100 and got[0][1] == len(wide)    # LEGO_ST_VOXEL_OVERFLOW: copied
    assert np.array_equal(got[0][0], ref)
    assert got[1][1] == -1


@pytest.mark.parametrize("order", [0, 1])
def test_voxel_overflow_then_normal_clouds(s2m, sequences, order):
    """An overflowing cloud (PCL's int32 leaf-index warning path: copied unfiltered) FOLLOWED by normal
    clouds, through the few-clouds layout (one device-wide sort of cloud|leaf keys): the later clouds'
    sorted ranges must not shift, so each equals the oracle (the overflowed slots once
    sorted past every cloud)."""
    s2m.set_voxel_tie_order(order)
    fr = sequences[2]
    rng = np.random.default_rng(21)
    wide = rng.uniform(-1000, 1000, (3000, 4)).astype(np.float32)
    clouds = [wide, fr[3]["corner_last"], fr[3]["surf_last"], np.repeat(rng.uniform(-1, 1, (40, 4)).astype(np.float32),
                                                                         5, axis=0), wide[:500]]
    leaves = [1e-3, 0.2, 0.4, 0.4, 1e-3]
    got = _gpu_voxel(s2m, clouds, leaves)
    for c, leaf, (o, on, st) in zip(clouds, leaves, got):
        ref, rst = O.voxel_grid(c, leaf, stable=order == 1)
        assert st == rst and on == len(ref), (leaf, len(c), on, len(ref), st, rst)
        assert np.array_equal(o.view(np.int32), ref.view(np.int32)), (leaf, len(c))
    assert got[0][2] == 0x100 and got[4][2] == 0x100


@pytest.mark.parametrize("order", [0, 1])
def test_voxel_keys_past_2_31(s2m, order):
    """Leaf indices of 2^31 and above: PCL's overflow gate multiplies the truncated extents
    (dx = (max - min) / leaf + 1 = 1290 per axis, 1290^3 < 2^31 - 1: not flagged), while the indices use
    floor(max / leaf) - floor(min / leaf) + 1 = 1291 per axis, so the largest leaf index is ~2.15e9.
    The std::sort-order path's per-range sort takes keys below 2^31 - 1 and ranks such ranges first."""
    s2m.set_voxel_tie_order(order)
    rng = np.random.default_rng(31)
    lo, hi = 0.005, 12.904  # leaf 0.01: lo / leaf = 0.5, hi / leaf = 1290.4, (hi - lo) / leaf = 1289.9
    corners = np.array([[x, y, z, 1.0] for x in (lo, hi) for y in (lo, hi) for z in (lo, hi)], np.float32)
    def cloud(n):
        near_hi = hi - rng.uniform(0, 0.05, (n // 3, 3))  # top voxels: keys past 2^31
        near_lo = lo + rng.uniform(0, 0.05, (n // 3, 3))
        mid = rng.uniform(lo, hi, (n - 2 * (n // 3), 3))
        p = np.concatenate([near_hi, near_lo, mid])
        p = np.concatenate([p, rng.uniform(0, 1, (len(p), 1))], 1).astype(np.float32)
        p = np.concatenate([corners, p, p[: n // 4]])  # repeated points: ties
        return p[rng.permutation(len(p))]
    clouds = [cloud(1500), cloud(6000), cloud(40000)]
    got = _gpu_voxel(s2m, clouds, [0.01] * len(clouds))
    for c, (o, on, st) in zip(clouds, got):
        ref, rst = O.voxel_grid(c, 0.01, stable=order == 1)
        assert rst == 0, "the cloud must pass PCL's overflow gate"
        assert st == rst and on == len(ref), (len(c), on, len(ref))
        assert np.array_equal(o.view(np.int32), ref.view(np.int32)), len(c)


def test_voxel_std_order_key_sequences(s2m):
    """voxel_tie_order 0 on clouds whose leaf indices are chosen key sequences (points at x = key + 0.5, leaf 1):
    tie-heavy random keys up to 100k points (several device-wide levels, then one wave a range), sorted,
    reversed, organ-pipe and run sequences, and the introsort adversary (ranges longer than 2,048 reaching
    the depth limit: the device-wide heap sort), each against the oracle's std::sort VoxelGrid; the
    intensities differ per point, so any other summation order shows."""
    import os
    import subprocess
    import tempfile
    s2m.set_voxel_tie_order(0)
    rng = np.random.default_rng(31)

    def cloud(keys):
        keys = np.asarray(keys, np.int64)
        p = np.zeros((len(keys), 4), np.float32)
        p[:, 0] = keys + 0.5
        p[:, 3] = rng.uniform(0, 100, len(keys)).astype(np.float32)
        return p
    seqs = [rng.integers(0, d, n) for n, d in [(3000, 5), (20000, 300), (100000, 2000), (60000, 60000), (2049, 2),
                                                 (4096, 1)]]
    i = np.arange(30000)
    seqs += [i, i[::-1], np.minimum(i, 30000 - i), i // 7, (i * 7919) % 4001]
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "ia")
        subprocess.check_call(["g++", "-std=c++17", "-O2", "-I" + os.path.join(repo, "lego-loam-bor_amd", "csrc"),
                               os.path.join(repo, "tests", "native", "introsort_adversary.cpp"), "-o", exe])
        for n, c in [(3000, 1), (8192, 2), (50000, 1)]:
            out = subprocess.run([exe, str(n), str(c)], stdout=subprocess.PIPE, universal_newlines=True, check=True)
            seqs.append(np.array(out.stdout.split(), dtype=np.int64))
    clouds = [cloud(k) for k in seqs]
    for batch in (clouds[:6], clouds[6:]):
        got = _gpu_voxel(s2m, batch, [1.0] * len(batch))
        for c, (o, on, st) in zip(batch, got):
            ref, rst = O.voxel_grid(c, 1.0, stable=False)
            assert st == rst and on == len(ref), (len(c), on, len(ref))
            assert np.array_equal(o.view(np.int32), ref.view(np.int32)), len(c)


def test_transform_matches_oracle(s2m, sequences):
    import torch
    import lego_amd as LA
    fr = sequences[1]
    parts = [(fr[j][c], fr[j]["transform_sum"]) for j in range(1, 5) for c in ("corner_last", "surf_last")]
    cl = [np.ascontiguousarray(p[0], np.float32) for p in parts]
    n = np.array([len(c) for c in cl], np.int32)
    off = np.concatenate([[0], np.cumsum(n)[:-1]]).astype(np.int64)
    flat = torch.from_numpy(np.concatenate(cl)).cuda()
    poses = torch.from_numpy(np.stack([np.asarray(p[1], np.float32) for p in parts])).cuda()
    t_off, t_n = torch.from_numpy(off).cuda(), torch.from_numpy(n).cuda()
    out = torch.zeros_like(flat)
    io = LA.LegoMapTransformIo()
    io.in_, io.in_off, io.in_n, io.pose = flat.data_ptr(), t_off.data_ptr(), t_n.data_ptr(), poses.data_ptr()
    io.out, io.out_off = out.data_ptr(), t_off.data_ptr()
    s2m.map_transform(len(cl), io)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    for i, (c, t) in enumerate(parts):
        ref = O.transform_cloud(c, t)
        assert np.array_equal(o[off[i]:off[i] + n[i]].view(np.int32), ref.view(np.int32)), i


def _oracle_problem(frames, k, n_keys=10, perturb=(0.002, 0.002, 0.004, 0.03, 0.01, 0.03), order=0):
    """build_problem with the oracle's transformPointCloud and VoxelGrid (in the given tie order)."""
    cparts, sparts, (c, s, o) = M._parts(frames, k, n_keys)
    cm = np.concatenate([O.transform_cloud(x, t) for x, t in cparts])
    sm = np.concatenate([O.transform_cloud(x, t) for x, t in sparts])
    vg = lambda x, leaf: O.voxel_grid(x, leaf, stable=order == 1)[0]  # noqa: E731
    return {"corner_map": vg(cm, 0.2), "surf_map": vg(sm, 0.4), "corner": vg(c, 0.2),
            "surf": vg(np.concatenate([vg(s, 0.4), vg(o, 0.4)]), 0.4),
            "transform": (np.asarray(frames[k]["transform_sum"], np.float32) + np.asarray(perturb, np.float32))}


@pytest.mark.parametrize("order", [0, 1])
def test_prepared_problems_match_oracle(s2m, sequences, order):
    import torch
    s2m.set_voxel_tie_order(order)
    k = 5
    io, keep, tr, dg, info, v = M.prepare_gpu(s2m, sequences, k)
    torch.cuda.synchronize()
    P_ = len(sequences)
    vo, oo, on = v["v_out"].cpu().numpy(), v["out_off"], v["out_n"].cpu().numpy()
    to, toff, tn = v["tot_out"].cpu().numpy(), v["tot_off"], v["tot_n"].cpu().numpy()
    refs = [_oracle_problem(seq, k, order=order) for seq in sequences]
    for p, ref in enumerate(refs):
        got = {"corner_map": vo[oo[p]:oo[p] + on[p]], "surf_map": vo[oo[P_ + p]:oo[P_ + p] + on[P_ + p]],
               "corner": vo[oo[2 * P_ + 3 * p]:oo[2 * P_ + 3 * p] + on[2 * P_ + 3 * p]],
               "surf": to[toff[p]:toff[p] + tn[p]]}
        for name, a in got.items():
            assert np.array_equal(a.view(np.int32), ref[name].view(np.int32)), (p, name, len(a), len(ref[name]))
    s2m.run(P_, io)
    torch.cuda.synchronize()
    t_gpu, i_gpu = tr.cpu().numpy(), info.cpu().numpy()
    for p, ref in enumerate(refs):
        t_ref, dg_ref, i_ref = O.scan2map(ref["corner"], ref["surf"], ref["corner_map"], ref["surf_map"], ref["transform"])
        assert np.abs(t_gpu[p] - t_ref).max() <= 1e-4, (p, t_gpu[p], t_ref)
        assert i_gpu[p][1] == i_ref[1] and (i_gpu[p][3] & ~1) == (i_ref[3] & ~1)
