"""Diagnostic: per-ring timing of k_voxel (profile build) — which rings set a launch's time.

  python lego-loam-bor_amd/build.py --profile
  LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so python tools/ring_log.py [S] [order] [kind]

Runs S streams for a few pipelined steps (bench.py's schedule), then logs (a) the last in-pipeline VoxelGrid
launch and (b) the same launch alone on the device (lego_batch_time_voxel, reps = 1).  Stamps: the 100 MHz real-time
counter (s_memrealtime; the shader clock differs between XCDs).  Prints the ring-time distribution, the launch span,
the slowest rings (size, start offset, duration) and how late rings start (dispatch rounds).
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


def read_log(lib, nb):
    out = np.zeros(nb * 4, np.uint64)
    rc = lib.lego_debug_ring_log(out.ctypes.data_as(C.POINTER(C.c_uint64)), nb)
    assert rc == 0, rc
    return out.reshape(nb, 4)


def report(tag, lg, tick_per_us):
    t0 = lg[:, 0].astype(np.int64)
    t1 = lg[:, 1].astype(np.int64)
    n = (lg[:, 2] & 0xffffffff).astype(np.int64)
    base = t0.min()
    start = (t0 - base) / tick_per_us
    dur = (t1 - t0) / tick_per_us
    span = (t1.max() - base) / tick_per_us
    print("== %s: span %.1f us; ring us mean %.1f p50 %.1f p90 %.1f p99 %.1f max %.1f; start p50 %.1f p90 %.1f max %.1f"
          % (tag, span, dur.mean(), *np.percentile(dur, [50, 90, 99]), dur.max(), *np.percentile(start, [50, 90]),
             start.max()))
    end = start + dur
    top = np.argsort(-end)[:12]
    print("   latest-ending rings: (n, start us, duration us)")
    for i in top:
        print("     n %5d  start %7.1f  dur %7.1f  end %7.1f" % (n[i], start[i], dur[i], end[i]))
    for lo, hi in ((0, 256), (256, 512), (512, 1024), (1024, 1400), (1400, 4096)):
        m = (n >= lo) & (n < hi)
        if m.any():
            print("   n in [%4d, %4d): %5d rings, dur mean %7.1f max %7.1f us" % (lo, hi, m.sum(), dur[m].mean(),
                                                                                 dur[m].max()))
    return span


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
    lib.lego_debug_ring_log.argtypes = [C.POINTER(C.c_uint64), C.c_int32]
    st = torch.cuda.current_stream().cuda_stream
    for k in range(steps):
        b.step(d_pts.data_ptr(), offs[k].data_ptr(), cnts[k].data_ptr(), st)
    b.sync()
    nb = S * params.num_vertical_scans
    pipe = read_log(lib, nb)
    ms = b.time_voxel(reps=1, stream=st)
    alone = read_log(lib, nb)
    tick_per_us = 100.0  # s_memrealtime
    print("S %d order %d %s: alone launch %.3f ms (hipEvents); log span %.3f ms" % (
        S, order, kind, ms, float(alone[:, 1].max() - alone[:, 0].min()) / tick_per_us / 1e3))
    report("in pipeline (last step)", pipe, tick_per_us)
    report("alone", alone, tick_per_us)
    b.close()


if __name__ == "__main__":
    main()
