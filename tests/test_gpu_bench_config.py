"""The exact configuration bench.py times, against the oracle.

bench.py's headline builds Batch(S = 256 VLP-16 sequences) with voxel_tie_order 0 and
bench.configure_batch: lag 1, lego_batch_set_wide(-1) (at 256 scans: the wide layout for order 0, the
one-workgroup layout for order 1), one caller
stream; W warm-up steps, flush, K timed steps, flush.  The same batch here, with every scan's
odometry recorded on the device (lego_batch_set_trajectory, which does not change the schedule): each of
the 256 streams' transformCur / transformSum after every scan within 1e-4 of an independent oracle run
(featureAssociation.cpp:1213-1270, 1286-1298), and exact parity of the last scan (projection, features,
Last clouds) on a sample of streams.  The stable order (bench.py's other_voxel_tie_order) runs the same way,
and so does the double libm model (fp_mode 1, shorter: its register-capped k_lm<512, 384, true, 4> runs only
with more than half a scan a CU in flight, which no other fp_mode 1 test reaches).
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import bench
import helpers as Hs
import lego_amd as L
from lego_amd import _abi as A
from test_gpu_parity import assert_scan_parity, oracle_for

pytestmark = pytest.mark.gpu

S, W, K = 256, 3, 6


def _oracle_sequence(params, pts, cnt, s, W=W, K=K):
    orc = oracle_for(params)
    traj, last = [], None
    for k in range(W + K):
        pr = orc.cloud_handler(pts[k * S + s, :cnt[k * S + s]])
        fr = orc.feature_association()
        traj.append(np.concatenate([fr["transform_cur"], fr["transform_sum"]]))
        last = (pr, fr)
    return np.array(traj, np.float64), last


@pytest.mark.parametrize("order,wide,fp_mode", [(0, 1, 0), (1, 0, 0), (0, 1, 1)])
def test_bench_schedule_matches_oracle(gpu, order, wide, fp_mode):
    import torch
    W, K = (3, 6) if fp_mode == 0 else (1, 3)
    params = L.params_vlp16(voxel_tie_order=order, fp_mode=fp_mode)
    cfg = A.synth_cfg("vlp16")
    cap = params.num_vertical_scans * params.num_horizontal_scans
    seqs = np.repeat(np.arange(S, dtype=np.int32)[None, :], W + K, 0).reshape(-1)  # bench.py's sequences 0 .. S-1
    scans = np.repeat(np.arange(W + K, dtype=np.int32)[:, None], S, 1).reshape(-1)
    pts, cnt = A.synth_batch(cfg, seqs, scans)
    d_pts = torch.from_numpy(pts).cuda()
    d_off = torch.from_numpy((np.arange((W + K) * S, dtype=np.int64) * cap).reshape(W + K, S)).cuda()
    d_cnt = torch.from_numpy(cnt.reshape(W + K, S).astype(np.int32)).cuda()
    b = L.Batch(params, S, cap)
    lag = bench.configure_batch(b, order)
    assert lag == 1 and b.wide() == wide  # the schedule the bench line reports at 256 streams
    traj = torch.zeros((S, W + K, 12), dtype=torch.float32, device="cuda")
    b.set_trajectory(traj.data_ptr(), W + K)
    stream = torch.cuda.current_stream()
    for k in range(W):  # bench.timed(): warm-up, flush, timed steps, flush
        b.step(d_pts.data_ptr(), d_off[k].data_ptr(), d_cnt[k].data_ptr(), stream.cuda_stream)
    b.flush()
    torch.cuda.synchronize()
    for k in range(W, W + K):
        b.step(d_pts.data_ptr(), d_off[k].data_ptr(), d_cnt[k].data_ptr(), stream.cuda_stream)
    b.flush()
    torch.cuda.synchronize()
    got = traj.cpu().numpy().astype(np.float64)
    poses, status = b.poses()
    assert np.all((status & A.ST_UB_MASK) == 0)
    with ThreadPoolExecutor(8) as ex:  # the oracle's ctypes calls release the GIL
        ref = list(ex.map(lambda s: _oracle_sequence(params, pts, cnt, s, W, K), range(S)))
    worst = max(float(np.abs(got[s] - ref[s][0]).max()) for s in range(S))
    exact = sum(int(np.array_equal(got[s].astype(np.float32), ref[s][0].astype(np.float32))) for s in range(S))
    print("order %d fp_mode %d: %d streams x %d scans, max |d pose| %.3g, %d streams bit-identical" % (
        order, fp_mode, S, W + K, worst, exact))
    assert worst <= Hs.TF_TOL
    np.testing.assert_array_equal(got[:, -1].astype(np.float32), poses)
    for s in (0, 101, 202, S - 1):  # exact parity of the last scan on a sample
        pg, fg = b.read(s)
        pr, fr = ref[s][1]
        assert_scan_parity((order, fp_mode, s), pg, pr, fg, fr)
    b.close()
