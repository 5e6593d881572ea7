"""Diagnostic: per-scan timing of k_lm (profile build) — what sets the launch's slowest scans.

  python lego-loam-bor_amd/build.py --profile
  LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so python tools/lm_log.py [S] [order] [kind]

Runs S streams for a few pipelined steps (bench.py's schedule) and reads the last k_lm launch's per-block
log (lego_debug_lm_log): duration (100 MHz real-time counter), the shader cycles of each loop's grid build,
searches and iteration blocks (thread 0's stamps), the iteration counts and the cloud sizes.
"""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lego-loam-bor_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import lego_amd as L  # noqa: E402
from lego_amd import _abi as A  # noqa: E402
import bench  # noqa: E402

COLS = ["build_s", "build_c", "search_s", "search_c", "iter_s", "iter_c"]


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    order = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    kind = sys.argv[3] if len(sys.argv) > 3 else "vlp16"
    steps = 8
    params = (L.params_vlp16 if kind == "vlp16" else L.params_hdl64)(voxel_tie_order=order)
    cfg = A.synth_cfg(kind)
    cap = params.num_vertical_scans * params.num_horizontal_scans
    seqs = np.repeat(np.arange(S)[None, :], steps, 0).reshape(-1)
    scans = np.repeat(np.arange(steps)[:, None], S, 1).reshape(-1)
    pts, cnt = A.synth_batch(cfg, seqs, scans, nthreads=16)
    d_pts = torch.from_numpy(pts).cuda()
    offs = torch.from_numpy((np.arange(S * steps, dtype=np.int64) * cap).reshape(steps, S)).cuda()
    cnts = torch.from_numpy(cnt.reshape(steps, S).astype(np.int32)).cuda()
    b = L.Batch(params, S, cap)
    bench.configure_batch(b, order)
    lib = L.lib()
    lib.lego_debug_lm_log.argtypes = [C.POINTER(C.c_uint64), C.c_int32]
    st = torch.cuda.current_stream().cuda_stream
    for k in range(steps):
        b.step(d_pts.data_ptr(), offs[k].data_ptr(), cnts[k].data_ptr(), st)
    b.sync()
    lg = np.zeros(S * 16, np.uint64)
    assert lib.lego_debug_lm_log(lg.ctypes.data_as(C.POINTER(C.c_uint64)), S) == 0
    lg = lg.reshape(S, 16).astype(np.int64)
    t0, t1 = lg[:, 0], lg[:, 1]
    dur = (t1 - t0) / 100.0  # us
    start = (t0 - t0.min()) / 100.0
    cyc = lg[:, 2:8].astype(np.float64)
    tot_cyc = cyc.sum(1)
    ghz = np.median(tot_cyc / np.maximum(dur, 1e-3)) / 1e3  # cycles a us -> GHz (phases cover most of a scan)
    print("S %d order %d %s: last k_lm launch span %.1f us; scan us mean %.1f p50 %.1f p90 %.1f max %.1f; "
          "start p50 %.1f max %.1f; phase clock ~%.2f GHz (median phases/duration)" % (
              S, order, kind, (t1.max() - t0.min()) / 100.0, dur.mean(), *np.percentile(dur, [50, 90]), dur.max(),
              np.median(start), start.max(), ghz))
    us = cyc / 2400.0  # shader cycles at 2.4 GHz
    print("mean us: " + "  ".join("%s %.1f" % (c, us[:, i].mean()) for i, c in enumerate(COLS)))
    print("iterations surf / corner mean %.2f / %.2f; flat / sharp queries %.0f / %.0f; surf / lessSharp Last %.0f / %.0f"
          % tuple(lg[:, 8:14].mean(0)))
    top = np.argsort(-(start + dur))[:12]
    print("latest-ending scans: start, dur (us), phases (us at 2.4 GHz), it_s it_c, nq_flat nq_sharp, n_surf n_lsharp")
    for i in top:
        print("  %6.1f %6.1f  %s  %2d %2d  %4d %4d  %5d %4d" % (start[i], dur[i], " ".join("%6.1f" % x for x in us[i]),
                                                             *lg[i, 8:14]))
    r = np.corrcoef(np.vstack([dur, us.T, lg[:, 9]]))[0, 1:]
    print("corr(duration, phase): " + "  ".join("%s %.2f" % (c, v) for c, v in zip(COLS + ["it_c"], r)))
    b.close()


if __name__ == "__main__":
    main()
