"""Checkpoint / resume of a stream's FeatureAssociation state (lego_batch_save_state / load_state,
lego_ctx_save_state / load_state; featureAssociation.h:70-115 plus the persistent smoothness vectors whose
stale entries the next scan reads).  Property: a stream resumed from a checkpoint — in another
batch, on another stream index — produces bit for bit what the uninterrupted stream produces, and both match
the oracle's uninterrupted sequence."""
import numpy as np
import pytest

import helpers as Hs
import lego_amd as L
from lego_amd import _abi as A
from test_gpu_parity import oracle_for

pytestmark = pytest.mark.gpu

S, K0, K1 = 4, 5, 3  # streams; scans before the checkpoint; scans after it


def _same(fa, fb):
    assert not Hs.diff_report(Hs.FEAT_KEYS, fa, fb)
    for k in ("transform_cur", "transform_sum", "corner_last", "surf_last", "outlier_last"):
        assert Hs.bits_equal(fa[k], fb[k]), k
    assert fa["status"] == fb["status"]
    assert (fa["lm_iter_surf"], fa["lm_iter_corner"]) == (fb["lm_iter_surf"], fb["lm_iter_corner"])
    np.testing.assert_array_equal(fa["odom_orientation"], fb["odom_orientation"])


@pytest.mark.parametrize("order", [0, 1])
def test_batch_checkpoint_resumes_exactly(gpu, order):
    import torch
    params = L.params_vlp16(voxel_tie_order=order)
    cfg = A.synth_cfg("vlp16")
    cap = params.num_vertical_scans * params.num_horizontal_scans
    K = K0 + K1
    seqs = np.repeat(np.arange(S, dtype=np.int32)[None, :] + 300, K, 0).reshape(-1)
    scans = np.repeat(np.arange(K, dtype=np.int32)[:, None], S, 1).reshape(-1)
    pts, cnt = A.synth_batch(cfg, seqs, scans)
    d_pts = torch.from_numpy(pts).cuda()
    d_off = torch.from_numpy((np.arange(K * S, dtype=np.int64) * cap).reshape(K, S)).cuda()
    d_cnt = torch.from_numpy(cnt.reshape(K, S).astype(np.int32)).cuda()
    st = torch.cuda.current_stream().cuda_stream
    a = L.Batch(params, S, cap)
    for k in range(K0):
        a.step(d_pts.data_ptr(), d_off[k].data_ptr(), d_cnt[k].data_ptr(), st)
    ckpt = [a.save_state(s) for s in range(S)]
    ref = []
    for k in range(K0, K):
        a.step(d_pts.data_ptr(), d_off[k].data_ptr(), d_cnt[k].data_ptr(), st)
        a.sync()
        ref.append([a.read(s)[1] for s in range(S)])
    a.close()
    # a fresh batch, the checkpoints loaded on permuted streams, fed the same scans in that permutation
    perm = [2, 0, 3, 1]
    b = L.Batch(params, S, cap)
    for j in range(S):
        b.load_state(j, ckpt[perm[j]])
    off_p = torch.from_numpy((np.arange(K * S, dtype=np.int64) * cap).reshape(K, S)[:, perm].copy()).cuda()
    cnt_p = torch.from_numpy(cnt.reshape(K, S)[:, perm].astype(np.int32).copy()).cuda()
    for i, k in enumerate(range(K0, K)):
        b.step(d_pts.data_ptr(), off_p[k].data_ptr(), cnt_p[k].data_ptr(), st)
        b.sync()
        for j in range(S):
            _same(b.read(j)[1], ref[i][perm[j]])
    b.close()
    # and the resumed sequence is the oracle's uninterrupted one
    orc = oracle_for(params)
    for k in range(K):
        orc.cloud_handler(pts[k * S + 1, :cnt[k * S + 1]])
        fr = orc.feature_association()
    np.testing.assert_allclose(ref[-1][1]["transform_sum"], fr["transform_sum"], atol=Hs.TF_TOL, rtol=0)


def test_ctx_checkpoint_resumes_exactly_and_rejects_other_sensor(gpu):
    params = L.params_vlp16()
    cfg = A.synth_cfg("vlp16")
    fe = L.Frontend(params)
    scans = [A.synth_scan(cfg, 7, k) for k in range(6)]
    for k in range(4):
        fe.cloud_handler(scans[k])
        fe.feature_association()
    ck = fe.save_state()
    ref = []
    for k in range(4, 6):
        fe.cloud_handler(scans[k])
        ref.append(fe.feature_association())
    fe.close()
    fe2 = L.Frontend(params)
    fe2.load_state(ck)
    for i, k in enumerate(range(4, 6)):
        fe2.cloud_handler(scans[k])
        _same(fe2.feature_association(), ref[i])
    fe2.close()
    hdl = L.Frontend(L.params_hdl64())
    with pytest.raises(L.LegoError):
        hdl.load_state(ck)
    with pytest.raises(L.LegoError):
        hdl.load_state(ck[:100])
    hdl.close()
