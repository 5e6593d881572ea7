"""CPU tests of the scan-to-map oracle (oracle/s2m_oracle.cpp) and of the C-ABI surface of lego_s2m.h.

The oracle restates MapOptimization::scan2MapOptimization (mapOptmization.cpp:1315-1332); the GPU
path (tests/test_gpu_s2m.py) is checked against it.  Here: its restated pieces on their own
(kNN-5 pinned against the reference's vendored nanoflann; the Eigen restatements against numpy
double-precision answers), and whole problems built from the FA oracle's AssociationOut records.
"""
import ctypes as C
import os
import struct
import subprocess

import numpy as np
import pytest

import oracle as O
from lego_amd import _abi as A
from lego_amd import mapping as M

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def frames():
    """AssociationOut records of one synthetic VLP-16 sequence (FA oracle)."""
    import lego_amd as LA
    orc = O.Oracle(LA.params_vlp16())
    cfg = A.synth_cfg("vlp16")
    out = []
    for k in range(8):
        orc.cloud_handler(A.synth_scan(cfg, 1, k))
        out.append(orc.feature_association())
    return out


def test_eig3_restatement_is_an_eigendecomposition():
    rng = np.random.default_rng(3)
    for _ in range(200):
        X = rng.normal(size=(5, 3)).astype(np.float32) * rng.uniform(0.01, 3.0, size=3).astype(np.float32)
        A3 = np.cov(X.T, bias=True).astype(np.float32)
        ev, V = O.eig3(A3)
        ref = np.linalg.eigvalsh(A3.astype(np.float64))
        assert np.all(np.diff(ev) >= 0)  # ascending, as SelfAdjointEigenSolver
        np.testing.assert_allclose(ev, ref, rtol=1e-4, atol=1e-6 * max(1.0, ref[-1]))
        np.testing.assert_allclose(V.T @ V, np.eye(3), atol=2e-6)
        np.testing.assert_allclose(A3 @ V, V * ev, atol=2e-5 * max(1.0, ref[-1]))
    # diagonal and already-tridiagonal inputs take the v1norm2 <= min branch
    ev, V = O.eig3(np.diag([3.0, 1.0, 2.0]).astype(np.float32))
    np.testing.assert_array_equal(ev, [1.0, 2.0, 3.0])
    np.testing.assert_array_equal(np.abs(V), np.array([[0, 0, 1], [1, 0, 0], [0, 1, 0]], np.float32))


def test_qr_restatement_solves():
    rng = np.random.default_rng(4)
    for _ in range(100):
        A5 = rng.normal(size=(5, 3)).astype(np.float32)
        b5 = -np.ones(5, np.float32)
        ref = np.linalg.lstsq(A5.astype(np.float64), b5.astype(np.float64), rcond=None)[0]
        np.testing.assert_allclose(O.qr_solve(A5, b5), ref, rtol=1e-4, atol=1e-5)
        B = rng.normal(size=(8, 6)).astype(np.float32)
        A6 = (B.T @ B).astype(np.float32)
        b6 = rng.normal(size=6).astype(np.float32)
        ref = np.linalg.solve(A6.astype(np.float64), b6.astype(np.float64))
        np.testing.assert_allclose(O.qr_solve(A6, b6), ref, rtol=2e-3, atol=2e-3 * np.abs(ref).max())
    # rank-deficient plane fit (collinear points): the pivots below threshold give zeros, no NaN
    A5 = np.array([[1, 2, 3], [2, 4, 6], [3, 6, 9], [4, 8, 12], [5, 10, 15]], np.float32)
    x = O.qr_solve(A5, -np.ones(5, np.float32))
    assert np.all(np.isfinite(x))


def _brute_knn5(cloud, q):
    d = ((q[:, None, 0] - cloud[None, :, 0]) ** 2 + (q[:, None, 1] - cloud[None, :, 1]) ** 2) + (q[:, None, 2] - cloud[None, :, 2]) ** 2
    order = np.lexsort((np.broadcast_to(np.arange(len(cloud)), d.shape), d), axis=1)[:, :6]
    return order, np.take_along_axis(d, order, axis=1)


def test_knn5_matches_brute_force(frames):
    pr = M.build_problem(frames, 6)
    cloud = pr["surf_map"]
    rng = np.random.default_rng(5)
    q = np.concatenate([cloud[rng.integers(0, len(cloud), 300)] + rng.normal(0, 0.2, (300, 4)).astype(np.float32),
                        rng.uniform(-40, 40, (50, 4)).astype(np.float32)]).astype(np.float32)
    ind, dist, fl = O.knn5(cloud, q)
    bo, bd = _brute_knn5(cloud.astype(np.float32), q.astype(np.float32))
    ok = bd[:, 4] < 1.0
    np.testing.assert_array_equal((fl & 1) != 0, ok)
    assert ok.sum() > 100
    untied = ok & ((fl & 2) == 0)
    np.testing.assert_array_equal(ind[untied], bo[untied, :5])
    assert np.array_equal(dist[ok].view(np.int32), bd[ok, :5].astype(np.float32).view(np.int32))
    # a duplicated point: equal distances are flagged as a tie and ordered as nanoflann's tree orders them
    _, d0 = _brute_knn5(cloud[:500], cloud[:500])
    i = int(np.argmax(d0[:, 5] < 1.0))
    assert d0[i, 5] < 1.0
    dup = np.concatenate([cloud, cloud[i:i + 1]])
    ind, dist, fl = O.knn5(dup, cloud[i:i + 1])
    ti, td = O.knn_tree(dup, cloud[i:i + 1], 5)
    assert fl[0] == 3 and sorted(ind[0, :2].tolist()) == [i, len(cloud)]
    np.testing.assert_array_equal(ind[0], ti[0])


def test_knn5_pin_nanoflann(frames):
    """The oracle's kNN-5 equals the reference's vendored nanoflann 1.3.0 nearestKSearch(k = 5) (built
    from /root/reference into oracle/_ref) wherever the 5th is within the 1 m ball, exact distance ties
    included (a duplicated map resolves every query's ties by nanoflann's visit order)."""
    if not os.path.exists("/root/reference/LeGO-LOAM/include/lego_loam/nanoflann.hpp"):
        pytest.skip("reference sources not mounted here")
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"])
    exe = os.path.join(REPO, "oracle", "_ref", "nanoflann_pin")
    pr = M.build_problem(frames, 6)
    rng = np.random.default_rng(6)
    dupmap = np.repeat(pr["corner_map"], 2, axis=0)
    for cloud, scan in ((pr["surf_map"], pr["surf"]), (pr["corner_map"], pr["corner"]), (dupmap, pr["corner"])):
        q = M.associate_to_map(scan, pr["transform"])[:600]
        q = np.concatenate([q, cloud[rng.integers(0, len(cloud), 200)] + rng.normal(0, 0.1, (200, 4)).astype(np.float32)])
        xyz = np.ascontiguousarray(cloud[:, :3], np.float32)
        qq = np.ascontiguousarray(q[:, :3], np.float32)
        blob = struct.pack("<i", len(xyz)) + xyz.tobytes() + struct.pack("<i", len(qq)) + qq.tobytes()
        out = subprocess.run([exe, "5"], input=blob, stdout=subprocess.PIPE, check=True).stdout
        res = np.frombuffer(out, dtype=np.dtype([("i", "<i4"), ("d", "<f4")])).reshape(len(qq), 5)
        ind, dist, fl = O.knn5(cloud, q)
        use = (fl & 1) != 0
        assert use.sum() > 100
        np.testing.assert_array_equal(ind[use], res["i"][use])
        assert np.array_equal(dist[use].view(np.int32), res["d"][use].view(np.int32))
        # the gate: nanoflann's 5th distance < 1.0 exactly where the oracle found 5 in the ball
        np.testing.assert_array_equal((fl & 1) != 0, res["d"][:, 4] < 1.0)


def test_scan2map_oracle_converges(frames):
    for k in (3, 7):
        pr = M.build_problem(frames, k)
        t, dg, info = O.scan2map(pr["corner"], pr["surf"], pr["corner_map"], pr["surf_map"], pr["transform"])
        assert info[0] == 1 and 1 <= info[1] <= 10 and info[2] > 1000
        assert info[3] & 0x08  # LEGO_S2M_ST_CONVERGED
        assert dg == 0
        assert np.all(np.isfinite(t))
        # the perturbed guess is pulled back toward the sequence's odometry
        assert np.abs(t - frames[k]["transform_sum"]).sum() < np.abs(pr["transform"] - frames[k]["transform_sum"]).sum()


def test_scan2map_oracle_gates(frames):
    pr = M.build_problem(frames, 5)
    # :1316 map gate: corner map <= 10 points -> nothing runs, transform untouched
    t, dg, info = O.scan2map(pr["corner"], pr["surf"], pr["corner_map"][:10], pr["surf_map"], pr["transform"])
    assert info[0] == 0 and info[3] == 0x10 and np.array_equal(t, pr["transform"])
    # :1208 fewer than 50 correspondences: no update in any iteration
    t, dg, info = O.scan2map(pr["corner"][:5], pr["surf"][:20], pr["corner_map"], pr["surf_map"], pr["transform"])
    assert info[0] == 1 and info[1] == 10 and info[3] & 0x04 and np.array_equal(t, pr["transform"])


def test_s2m_abi_exports():
    """liblego_frontend.so exports every entry point include/lego_s2m.h declares (no GPU needed)."""
    import re
    hdr = open(os.path.join(REPO, "include", "lego_s2m.h")).read()
    names = set(re.findall(r"\b(lego_(?:s2m|map|mapper)_\w+)\s*\(", hdr))
    assert names == {"lego_s2m_create", "lego_s2m_destroy", "lego_s2m_run", "lego_s2m_run_host", "lego_s2m_set_layout",
                     "lego_map_transform",
                     "lego_map_voxel", "lego_map_associate", "lego_map_odometry_to_transform", "lego_mapper_create",
                     "lego_mapper_destroy",
                     "lego_mapper_step", "lego_mapper_key_poses", "lego_s2m_set_voxel_tie_order",
                     "lego_mapper_set_voxel_tie_order"}
    assert "lego_test_s2m_debug" in hdr
    names.add("lego_test_s2m_debug")
    lib = C.CDLL(A.LIB_FRONTEND)
    for n in names:
        assert hasattr(lib, n), n


def test_voxel_grid_stable_oracle_matches_python():
    """The oracle's VoxelGrid with std::stable_sort's tie order (the map-side order) against a direct
    Python restatement of PCL's applyFilter: float32 leaf indices, float32 sums in point order."""
    rng = np.random.default_rng(13)
    pts = np.concatenate([rng.uniform(-3, 3, (400, 4)), np.repeat(rng.uniform(-3, 3, (30, 4)), 5, axis=0)]).astype(np.float32)
    rng.shuffle(pts)
    for leaf in (0.2, 0.4, 1.0):
        got, st = O.voxel_grid(pts, leaf, stable=True)
        inv = np.float32(1.0) / np.float32(leaf)
        mn, mx = pts[:, :3].min(0), pts[:, :3].max(0)
        min_b = np.floor(mn * inv).astype(np.int64)
        div = np.floor(mx * inv).astype(np.int64) - min_b + 1
        ijk = (np.floor(pts[:, :3] * inv) - min_b.astype(np.float32)).astype(np.int64)
        key = ijk[:, 0] + ijk[:, 1] * div[0] + ijk[:, 2] * div[0] * div[1]
        out = []
        for kv in np.unique(key):
            s_ = np.zeros(4, np.float32)
            idx = np.flatnonzero(key == kv)
            for i in idx:
                s_ = (s_ + pts[i]).astype(np.float32)
            out.append((s_ / np.float32(len(idx))).astype(np.float32))
        ref = np.array(out, np.float32)
        assert st == 0 and np.array_equal(got.view(np.int32), ref.view(np.int32)), leaf


def test_associate_to_map_matches_oracle():
    """transformAssociateToMap: the product's host function (lego_map_associate, used by the mapping
    loop) bit-exact to the oracle's restatement (float, the float libm) on random poses."""
    from lego_amd import mapping as M
    rng = np.random.default_rng(21)
    for _ in range(300):
        t = rng.uniform(-1, 1, (3, 6)).astype(np.float32)
        t[:, 3:] *= 50
        got = M.transform_associate_to_map(t[0], t[1], t[2])
        ref = O.associate_to_map(t[0], t[1], t[2])
        assert np.array_equal(got.view(np.int32), ref.view(np.int32)), (t, got, ref)
    z = np.zeros(6, np.float32)
    assert np.array_equal(M.transform_associate_to_map(z, z, z), z)



def test_odometry_to_transform_matches_oracle():
    """OdometryToTransform (utility.h:96-110): the product's host function (lego_map_odometry_to_transform,
    the mapping thread's transformSum) bit-exact to the oracle's restatement of tf's getRPY, including
    gimbal-locked and non-unit quaternions; and it inverts publishOdometry's quaternion to within float
    rounding."""
    from lego_amd import mapping as M
    rng = np.random.default_rng(23)
    qs = list(rng.normal(size=(400, 4)))
    for r, p, y in rng.uniform(-1.5, 1.5, (200, 3)):  # publishOdometry's quaternion of transformSum
        hy, hp, hr = -y * 0.5, -r * 0.5, p * 0.5  # roll = t[2], pitch = -t[0], yaw = -t[1]
        cy, sy, cp, sp, cr, sr = np.cos(hy), np.sin(hy), np.cos(hp), np.sin(hp), np.cos(hr), np.sin(hr)
        qx, qy = sr * cp * cy - cr * sp * sy, cr * sp * cy + sr * cp * sy
        qz, qw = cr * cp * sy - sr * sp * cy, cr * cp * cy + sr * sp * sy
        q = np.array([-qy, -qz, qx, qw])
        qs.append(q)
        t = M.odometry_to_transform(q, [1.0, 2.0, 3.0])
        assert np.allclose(t, [r, y, p, 1, 2, 3], atol=2e-6), (r, p, y, t)
    qs += [np.array([0.0, 0.0, np.sqrt(0.5), np.sqrt(0.5)]), np.array([0.5, 0.5, 0.5, 0.5]),
           np.array([0.0, 0.0, 0.0, 1.0])]
    for q in qs:
        pos = rng.normal(size=3) * 100
        got, ref = M.odometry_to_transform(q, pos), O.odometry_to_transform(q, pos)
        assert np.array_equal(got.view(np.int32), ref.view(np.int32)), (q, got, ref)


def test_normal_equation_order_gap(tmp_path):
    """Eigen's float GEMM order for matAt * matA (featureAssociation.cpp:861-862, mapOptmization.cpp:1258-1259)
    cannot be restated without Eigen, so the oracle and the product sum float products in double (FA) or in
    k_s2m's fixed lane order (scan-to-map).  This measures how far a second model of the reference's order,
    float accumulators in row order (oracle_set_float_normal_equations), moves the results: FA odometry over
    a 30-scan sequence and the scan-to-map transform of 6 problems.  Reported (LEGO_REPORT_DIR or the test's
    tmp dir); asserted only to stay far inside the north-star 1e-4 for a single solve's scale of change."""
    import json
    import lego_amd as LA
    L = O.lib()
    cfg = A.synth_cfg("vlp16")
    scans = [A.synth_scan(cfg, 2, k) for k in range(30)]
    runs = {}
    try:
        for mode in (0, 1):
            L.oracle_set_float_normal_equations(mode)
            orc = O.Oracle(LA.params_vlp16())
            sums, frames = [], []
            for p in scans:
                orc.cloud_handler(p)
                fr = orc.feature_association()
                sums.append(np.asarray(fr["transform_sum"], np.float64))
                frames.append(fr)
            s2m = []
            for k in (4, 9, 14, 19, 24, 29):
                pr = M.build_problem(frames[:k + 1], k)
                t, dg, info = O.scan2map(pr["corner"], pr["surf"], pr["corner_map"], pr["surf_map"], pr["transform"])
                s2m.append(np.asarray(t, np.float64))
            runs[mode] = (np.array(sums), np.array(s2m))
    finally:
        L.oracle_set_float_normal_equations(0)
    fa_gap = np.abs(runs[0][0] - runs[1][0]).max(axis=1)
    s2m_gap = np.abs(runs[0][1] - runs[1][1]).max(axis=1)
    report = {"fa_transform_sum_gap_per_scan": [float(x) for x in fa_gap],
              "fa_first_scan_over_1e-6": int(np.argmax(fa_gap > 1e-6)) if (fa_gap > 1e-6).any() else None,
              "s2m_transform_gap_per_problem": [float(x) for x in s2m_gap]}
    out = os.environ.get("LEGO_REPORT_DIR", str(tmp_path))
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "normal_equation_order_gap.json"), "w") as f:
        json.dump(report, f, indent=1)
    print(json.dumps(report))
    assert np.all(np.isfinite(fa_gap)) and np.all(np.isfinite(s2m_gap))
    assert fa_gap.max() < 1e-2 and s2m_gap.max() < 1e-2  # same trajectory, not a divergence


def _associate_double_libm(S, B, A):
    """transformAssociateToMap (mapOptmization.cpp:264-387) as a GCC 4.8 / 5 build evaluates it
    (lego_params.fp_mode 1): unqualified sin / cos / asin / atan2 on floats are the double functions, each
    expression evaluated in double and rounded where it is stored to a float."""
    import math
    f = np.float32
    d = lambda x: float(x)  # noqa: E731
    c, s = math.cos, math.sin
    S, B, A = [[f(v) for v in t] for t in (S, B, A)]
    x1 = f(c(d(S[1])) * d(f(B[3] - S[3])) - s(d(S[1])) * d(f(B[5] - S[5])))
    y1 = f(B[4] - S[4])
    z1 = f(s(d(S[1])) * d(f(B[3] - S[3])) + c(d(S[1])) * d(f(B[5] - S[5])))
    y2 = f(c(d(S[0])) * d(y1) + s(d(S[0])) * d(z1))
    z2 = f(-s(d(S[0])) * d(y1) + c(d(S[0])) * d(z1))
    inc3 = f(c(d(S[2])) * d(x1) + s(d(S[2])) * d(y2))
    inc4 = f(-s(d(S[2])) * d(x1) + c(d(S[2])) * d(y2))
    inc5 = z2
    tr = [f(g(d(v))) for v in (S[0], S[1], S[2], B[0], B[1], B[2], A[0], A[1], A[2]) for g in (s, c)]
    sbcx, cbcx, sbcy, cbcy, sbcz, cbcz, sblx, cblx, sbly, cbly, sblz, cblz, salx, calx, saly, caly, salz, calz = tr
    p1 = salx * sblx + calx * cblx * salz * sblz + calx * calz * cblx * cblz
    p2 = calx * calz * (cbly * sblz - cblz * sblx * sbly) - calx * salz * (cbly * cblz + sblx * sbly * sblz) + \
        cblx * salx * sbly
    p3 = calx * salz * (cblz * sbly - cbly * sblx * sblz) - calx * calz * (sbly * sblz + cbly * cblz * sblx) + \
        cblx * cbly * salx
    srx = -sbcx * p1 - cbcx * sbcy * p2 - cbcx * cbcy * p3
    T = [f(0)] * 6
    T[0] = f(-math.asin(d(srx)))
    q1, q2 = caly * calz + salx * saly * salz, caly * salz - calz * salx * saly
    q3, q4 = saly * salz + caly * calz * salx, calz * saly - caly * salx * salz
    srycrx = sbcx * (cblx * cblz * q2 - cblx * sblz * q1 + calx * saly * sblx) - \
        cbcx * cbcy * (q1 * (cblz * sbly - cbly * sblx * sblz) + q2 * (sbly * sblz + cbly * cblz * sblx) -
                       calx * cblx * cbly * saly) + \
        cbcx * sbcy * (q1 * (cbly * cblz + sblx * sbly * sblz) + q2 * (cbly * sblz - cblz * sblx * sbly) +
                       calx * cblx * saly * sbly)
    crycrx = sbcx * (cblx * sblz * q4 - cblx * cblz * q3 + calx * caly * sblx) + \
        cbcx * cbcy * (q3 * (sbly * sblz + cbly * cblz * sblx) + q4 * (cblz * sbly - cbly * sblx * sblz) +
                       calx * caly * cblx * cbly) - \
        cbcx * sbcy * (q3 * (cbly * sblz - cblz * sblx * sbly) + q4 * (cbly * cblz + sblx * sbly * sblz) -
                       calx * caly * cblx * sbly)
    T[1] = f(math.atan2(d(srycrx) / c(d(T[0])), d(crycrx) / c(d(T[0]))))
    srzcrx = (cbcz * sbcy - cbcy * sbcx * sbcz) * p3 - (cbcy * cbcz + sbcx * sbcy * sbcz) * p2 + cbcx * sbcz * p1
    crzcrx = (cbcy * sbcz - cbcz * sbcx * sbcy) * p2 - (sbcy * sbcz + cbcy * cbcz * sbcx) * p3 + cbcx * cbcz * p1
    T[2] = f(math.atan2(d(srzcrx) / c(d(T[0])), d(crzcrx) / c(d(T[0]))))
    x1 = f(c(d(T[2])) * d(inc3) - s(d(T[2])) * d(inc4))
    y1 = f(s(d(T[2])) * d(inc3) + c(d(T[2])) * d(inc4))
    z1 = inc5
    y2 = f(c(d(T[0])) * d(y1) - s(d(T[0])) * d(z1))
    z2 = f(s(d(T[0])) * d(y1) + c(d(T[0])) * d(z1))
    T[3] = f(d(A[3]) - (c(d(T[1])) * d(x1) + s(d(T[1])) * d(z2)))
    T[4] = f(A[4] - y2)
    T[5] = f(d(A[5]) - (-s(d(T[1])) * d(x1) + c(d(T[1])) * d(z2)))
    return np.array(T, np.float32)


def test_mapping_half_is_fp_mode_0():
    """The mapping half implements lego_params.fp_mode 0 only (include/lego_s2m.h): no
    lego_s2m / lego_map / lego_mapper entry point takes an fp_mode, and transformAssociateToMap
    (lego_map_associate, the mapping loop's) is the float-libm evaluation bit for bit, which a GCC 4.8 / 5
    build's double-libm evaluation (fp_mode 1) is not on a measurable share of poses."""
    import re
    from lego_amd import mapping as M
    hdr = open(os.path.join(REPO, "include", "lego_s2m.h")).read()
    decls = re.findall(r"int\s+lego_(?:s2m|map|mapper)_\w+\s*\([^;]*\);", hdr)
    assert decls and not any("fp_mode" in d for d in decls)
    rng = np.random.default_rng(5)
    differ = 0
    for _ in range(400):
        t = rng.uniform(-1, 1, (3, 6)).astype(np.float32)
        t[:, 3:] *= 50
        got = M.transform_associate_to_map(t[0], t[1], t[2])
        assert np.array_equal(got.view(np.int32), O.associate_to_map(t[0], t[1], t[2]).view(np.int32))
        differ += not np.array_equal(got.view(np.int32), _associate_double_libm(t[0], t[1], t[2]).view(np.int32))
    assert differ >= 20, differ  # the two libm models are distinguishable: the test discriminates
