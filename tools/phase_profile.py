"""Diagnostic: per-phase shader-cycle totals of k_extract / k_lm from the -DLG_PROFILE build.

  python lego-loam-bor_amd/build.py --profile
  LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so python tools/phase_profile.py

Stamps cost time themselves: read the SHARES, not absolute kernel times.
"""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lego-loam-bor_amd"))
import torch  # noqa: E402
import lego_amd as L  # noqa: E402
from lego_amd import _abi as A  # noqa: E402

NAMES = {0: "x:load+sort seg", 1: "x:sharp greedy", 2: "x:flat greedy", 3: "x:lessflat list", 4: "x:voxel total",
         5: "x:voxel sort", 6: "  sort:wave partitions", 7: "  sort:heap fallback", 11: "  sort:final insertion",
         12: "  seg: global load", 13: "  seg: sort", 8: "lm:transform sel", 9: "lm:search", 10: "lm:coeff+reduce",
         15: "lm:solve (thread 0)", 16: "lm:build grid", 17: "lm:surf loop", 18: "lm:corner loop",
         20: "p:init winner", 21: "p:scatter", 22: "p:reduce+orient", 23: "p:columns",
         36: "  sort:heap pops", 37: "lm:  grid nn", 38: "lm:  ring scans",
         32: "f:tile distort", 33: "f:tile LDS load", 34: "f:occl flags", 35: "f:smooth+picked",
         40: "lm:  it surf rows (w0)", 41: "lm:  it corner rows (w0)", 42: "lm:  it reduce (w0)",
         43: "lm:  it solve (w0)", 46: "lm:  corner nn", 47: "lm:  corner scans", 48: "lm:corner stage",
         25: "s:init parents", 26: "s:edges+unite", 27: "s:find roots", 28: "s:sizes+rank+label", 29: "s:compaction", 31: "s:distortion"}


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    order = int(sys.argv[2]) if len(sys.argv) > 2 else 1  # voxel_tie_order (bench default 1)
    kind = sys.argv[3] if len(sys.argv) > 3 else "vlp16"
    steps = 4
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
    prof = (C.c_uint64 * 256)()
    lib = L.lib()
    lib.lego_debug_prof.argtypes = [C.POINTER(C.c_uint64), C.c_int32]
    for k in range(steps):
        if k == 1:
            b.sync()
            lib.lego_debug_prof(prof, 1)
        b.step(d_pts.data_ptr(), offs[k].data_ptr(), cnts[k].data_ptr(), torch.cuda.current_stream().cuda_stream)
    b.sync()
    rc = lib.lego_debug_prof(prof, 0)
    assert rc == 0, rc
    tot = sum(prof[i] for i in NAMES if i < 17 or i >= 20)
    nsteps = steps - 1
    print("segments sorted via the tie path: %d per step (of %d segments)" % (prof[14] / nsteps, S * 16 * 6))
    print("rings waiting for their scan's first pass: %d per step (of %d rings)" % (prof[30] / nsteps, S * 16))
    for i, nm in NAMES.items():
        print("%-20s %14.0f cycles/step  (%5.1f%%)  per ring-wave %.0f  per stream %.0f  max one %.0f" % (
            nm, prof[i] / nsteps, 100.0 * prof[i] / max(tot, 1), prof[i] / nsteps / (S * 16), prof[i] / nsteps / S,
            prof[192 + i]))


    print("heap-sort fallbacks %d per step" % (prof[24] / nsteps))
    print("LM solves per scan: surf %.2f corner %.2f" % (prof[44] / nsteps / S, prof[45] / nsteps / S))
    V = params.num_vertical_scans
    print("per-ring extract wave cycles (mean / max over streams), ring 63 = first pass:")
    for r in list(range(V)) + [63]:
        if prof[128 + r]:
            print("  ring %2d  mean %9.0f  max %9.0f" % (r, prof[64 + r] / nsteps / S, prof[128 + r]))


if __name__ == "__main__":
    main()
