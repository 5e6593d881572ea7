"""Projection-only timing of library variants (round 6 A/B of the wide projection): a fresh Batch (no
step: the smoothness launch of the timed pair has no segmented points to read), S scans of synthetic
input resident in HBM, the wide projection launched back to back by lego_batch_time_hbm_stages
(alternating two input sets).   LEGO_FRONTEND_LIB=... python tools/proj_time.py [kind] [S] [wide]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lego-loam-bor_amd"))
import torch  # noqa: E402

import lego_amd as L  # noqa: E402
from lego_amd import _abi as A  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "vlp16"
S = int(sys.argv[2]) if len(sys.argv) > 2 else 256
wide = int(sys.argv[3]) if len(sys.argv) > 3 else 1
params = L.params_vlp16() if kind == "vlp16" else L.params_hdl64()
cfg = A.synth_cfg(kind)
cap = params.num_vertical_scans * params.num_horizontal_scans
seqs = np.tile(np.arange(S, dtype=np.int32), 2)
scans = np.repeat(np.arange(2, dtype=np.int32), S)
pts, cnt = A.synth_batch(cfg, seqs, scans, nthreads=16)
d_pts = torch.from_numpy(pts.reshape(-1, 4)).cuda()
offs = torch.from_numpy((np.arange(2 * S, dtype=np.int64) * cap).reshape(2, S)).cuda()
cnts = torch.from_numpy(cnt.reshape(2, S).astype(np.int32)).cuda()
b = L.Batch(params, S, cap)
b.set_wide(wide)
st = torch.cuda.current_stream().cuda_stream
ms = [b.time_hbm_stages(d_pts.data_ptr(), offs[1].data_ptr(), cnts[1].data_ptr(), offs[0].data_ptr(),
                        cnts[0].data_ptr(), reps=20, stream=st) for _ in range(5)]
bytes_proj = S * (16 * float(cnt.mean()) + 20 * cap)
print("%s %s S=%d wide=%d proj_ms %.4f (min of 5: %s) -> %.2f TB/s projection-only" % (
    os.path.basename(os.environ.get("LEGO_FRONTEND_LIB", "default")), kind, S, wide, min(ms),
    " ".join("%.4f" % m for m in ms), bytes_proj / (min(ms) * 1e-3) / 1e12))
b.close()
# diagnostic builds (-DLG_PWS_STATS): k_pw_slice / k_pw_fix category counts over all launches above
try:
    import ctypes as C
    lib = L.lib()
    st8 = (C.c_uint64 * 8)()
    if hasattr(lib, "lego_debug_pws_stats") and lib.lego_debug_pws_stats(st8, 0) == 0:
        print("pws stats: fallback slices %d, band slices %d, owned %d, empty %d, contested %d, incomplete %d, "
              "rescan blocks %d" % tuple(st8[:7]))
except Exception as e:  # noqa: BLE001
    print("pws stats unavailable:", e)
