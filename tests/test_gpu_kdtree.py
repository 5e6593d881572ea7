"""Exact 1-NN distance ties on the device: the LM's grid search finds the nearest
distance; when several Last-cloud points share it, k_lm builds nanoflann's tree and re-runs nanoflann's
search, so the reference's first-visited point is chosen.  Checked against the oracle's restated
nanoflann (itself pinned to the reference's vendored nanoflann.hpp by test_nanoflann_pin):
* the device tree + search on tie-heavy clouds (lattices, duplicated points, mirrored pairs);
* the whole LM with Last clouds whose every point is duplicated (every 1-NN is a tie), injected into
  GPU and oracle alike (lego_test_set_lm_state), both libm models.
"""
import ctypes as C

import numpy as np
import pytest

import helpers as Hs
import lego_amd as L
from lego_amd import _abi as A

pytestmark = pytest.mark.gpu


def _dev_knn(cloud4, q4, k):
    cloud4, q4 = np.ascontiguousarray(cloud4, np.float32), np.ascontiguousarray(q4, np.float32)
    idx = np.zeros((len(q4), k), np.int32)
    d = np.zeros((len(q4), k), np.float32)
    fp, ip = C.POINTER(C.c_float), C.POINTER(C.c_int32)
    rc = L.lib().lego_test_kd_knn(cloud4.ctypes.data_as(fp), len(cloud4), q4.ctypes.data_as(fp), len(q4), k,
                                  idx.ctypes.data_as(ip), d.ctypes.data_as(fp))
    assert rc == 0
    return idx, d


def _frames(params, seq, n):
    import oracle as O
    orc = O.Oracle(params)
    cfg = A.synth_cfg("vlp16")
    out = []
    for k in range(n):
        pr = orc.cloud_handler(A.synth_scan(cfg, seq, k))
        out.append((pr, orc.feature_association(), orc.lm_flags()))
    return out


@pytest.mark.parametrize("k", [1, 5])
def test_device_tree_matches_nanoflann_restatement(gpu, k):
    import oracle as O
    import test_oracle_cpu as T
    fr = _frames(L.params_vlp16(), 0, 2)[1][1]
    rng = np.random.default_rng(0)
    pad = lambda a: np.concatenate([a, np.zeros((len(a), 1), np.float32)], 1)  # noqa: E731
    ties = 0
    for name, xyz, q in T._tie_clouds(rng, fr):
        c4, q4 = pad(np.asarray(xyz, np.float32)), pad(np.asarray(q, np.float32))
        gi, gd = _dev_knn(c4, q4, k)
        oi, od = O.knn_tree(c4, q4, k)
        np.testing.assert_array_equal(gi, oi, err_msg=name)
        assert Hs.bits_equal(gd, od), name
        d = ((q4[:, None, :3] - c4[None, :, :3]) ** 2).sum(-1)
        ties += int(((d == d.min(1, keepdims=True)).sum(1) > 1).sum())
    assert ties > 300


@pytest.mark.parametrize("fp_mode", [0, 1])
def test_lm_with_duplicated_last_clouds(gpu, fp_mode):
    """Every Last-cloud point twice (every 1-NN an exact tie between i and i + n, and the rings'
    index order kept): the GPU LM equals the oracle's, whose 1-NN is nanoflann's."""
    import oracle as O
    params = L.params_vlp16(fp_mode=fp_mode)
    run = _frames(params, 13, 5)
    fe = L.Frontend(params)
    orc = O.Oracle(params)
    tied = 0
    for k, (pr, fr_src, flags) in enumerate(run):
        if k > 0:
            p = run[k - 1][1]
            cl = np.repeat(p["corner_last"], 2, axis=0)  # i, i: ring order (intensity) preserved
            sl = np.repeat(p["surf_last"], 2, axis=0)
            dg, stale = run[k - 1][2]
            fe.set_lm_state(p["transform_cur"], p["transform_sum"], dg, cl, sl, stale)
            orc_state = (p["transform_cur"], p["transform_sum"], dg, cl, sl, stale)
        else:
            orc_state = None
        fg = fe.feature_association(pr)
        if orc_state is None:
            fo = orc.feature_association(pr)
        else:
            fo = orc.feature_association_with_state(pr, *orc_state)
        assert not Hs.diff_report(Hs.FEAT_KEYS, fg, fo), k
        assert fg["status"] == fo["status"], (k, hex(fg["status"]), hex(fo["status"]))
        assert (fg["lm_iter_surf"], fg["lm_iter_corner"]) == (fo["lm_iter_surf"], fo["lm_iter_corner"]), k
        np.testing.assert_allclose(fg["transform_cur"], fo["transform_cur"], atol=Hs.TF_TOL, rtol=0)
        tied += int(bool(fg["status"] & A.ST_NN_TIE)) if hasattr(A, "ST_NN_TIE") else int(bool(fg["status"] & 0x20))
    fe.close()
    assert tied >= 3  # the tie path ran
