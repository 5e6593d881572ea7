"""Few-stream latency probe (C5's per-rank workload): S sequences as the streams of one
batch, K scans each, bench.configure_batch's schedule, every step timed between two events on the step
stream (host wall time beside it).  With a kernel trace (rocprofv3 --kernel-trace) the timeline shows
which chain a step waits for.   python tools/few_streams.py [S] [K] [order] [lag] [wide]"""
import os
import sys
import time

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "lego-loam-bor_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
import lego_amd as L  # noqa: E402
from lego_amd import _abi as A  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 10
K = int(sys.argv[2]) if len(sys.argv) > 2 else 60
order = int(sys.argv[3]) if len(sys.argv) > 3 else 0
lag = None if len(sys.argv) <= 4 or sys.argv[4] == "auto" else int(sys.argv[4])
wide = int(sys.argv[5]) if len(sys.argv) > 5 else -1
params = L.params_vlp16(voxel_tie_order=order)
cfg = A.synth_cfg("vlp16")
cap = params.num_vertical_scans * params.num_horizontal_scans
seqs = np.repeat(np.arange(S, dtype=np.int32)[None, :] + 5000, K, 0).reshape(-1)
scans = np.repeat(np.arange(K, dtype=np.int32)[:, None], S, 1).reshape(-1)
pts, cnt = A.synth_batch(cfg, seqs, scans, nthreads=16)
d_pts = torch.from_numpy(pts).cuda()
d_off = torch.from_numpy((np.arange(K * S, dtype=np.int64) * cap).reshape(K, S)).cuda()
d_cnt = torch.from_numpy(cnt.reshape(K, S).astype(np.int32)).cuda()
b = L.Batch(params, S, cap)
eff = bench.configure_batch(b, order, lag, wide)
st = torch.cuda.current_stream()
torch.cuda.synchronize()
host = []
t0 = time.perf_counter()
for k in range(K):
    h0 = time.perf_counter()
    b.step(d_pts.data_ptr(), d_off[k].data_ptr(), d_cnt[k].data_ptr(), st.cuda_stream)
    host.append(time.perf_counter() - h0)
b.flush()
torch.cuda.synchronize()
el = time.perf_counter() - t0
print("S=%d K=%d order=%d lag=%d wide=%d: %.3f ms/step, %.1f scans/s; host enqueue %.1f us/step (median)" % (
    S, K, order, eff, b.wide(), 1e3 * el / K, S * K / el, 1e6 * float(np.median(host))))
b.close()
