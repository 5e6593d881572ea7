"""Host model (round 5): points a surf / corner 1-NN query visits in the pruned uniform grid at several cell
sizes (the dense LDS table forces 3.34 m cells on a ~100 m scene).  Usage: python tools/analysis/nn_grid_model.py vlp16 2
"""
import sys, numpy as np
sys.path[:0] = ["/root/repo/lego-loam-bor_amd", "/root/repo/oracle", "/root/repo/tests"]
import lego_amd as L
from lego_amd import _abi as A
import oracle as O
kind = sys.argv[1]
params = (L.params_vlp16 if kind == "vlp16" else L.params_hdl64)(voxel_tie_order=0)
cfg = A.synth_cfg(kind)
def t2s(p, cur):
    s = 10 * (p[:, 3] - np.floor(p[:, 3]))
    rx, ry, rz = s * cur[0], s * cur[1], s * cur[2]; tx, ty, tz = s * cur[3], s * cur[4], s * cur[5]
    x1 = np.cos(rz) * (p[:, 0] - tx) + np.sin(rz) * (p[:, 1] - ty)
    y1 = -np.sin(rz) * (p[:, 0] - tx) + np.cos(rz) * (p[:, 1] - ty)
    z1 = p[:, 2] - tz
    y2 = np.cos(rx) * y1 + np.sin(rx) * z1; z2 = -np.sin(rx) * y1 + np.cos(rx) * z1
    return np.stack([np.cos(ry) * x1 - np.sin(ry) * z2, y2, np.sin(ry) * x1 + np.cos(ry) * z2], 1)
def grid_cost(last, sel, cs0, maxcells, dims=3):
    lo = last.min(0); hi = last.max(0); cs = cs0
    while True:
        dim = ((hi - lo) / cs).astype(int) + 1
        if dims == 2: dim[2] = 1
        if np.prod(dim) <= maxcells: break
        cs *= 2
    R = 1 if cs >= 3 * cs0 else 2 if cs >= 1.5 * cs0 else 3
    cell = np.clip(np.floor((last - lo) / cs).astype(int), 0, dim - 1)
    if dims == 2: cell[:, 2] = 0
    from collections import defaultdict
    cnt = defaultdict(int)
    for c in map(tuple, cell): cnt[c] += 1
    tot_pts = []; tot_cells = []
    for q in sel:
        d = ((last - q) ** 2).sum(1); best = min(d.min(), 25.0)
        qc = np.floor((q - lo) / cs).astype(int)
        if dims == 2: qc[2] = 0
        npts = 0; ncell = 0
        for k in range(R + 1):
            if k >= 2 and ((k - 1) * cs) ** 2 > best: break
            rng = range(-k, k + 1)
            for dz in (rng if dims == 3 else [0]):
                for dy in rng:
                    for dx in rng:
                        if max(abs(dx), abs(dy), abs(dz)) != k: continue
                        c = (qc[0] + dx, qc[1] + dy, qc[2] + dz)
                        if c not in cnt: continue
                        if k > 0:
                            clo = lo + np.array(c) * cs; chi = clo + cs
                            e = np.maximum(np.maximum(clo - q, q - chi), 0)
                            if dims == 2: e[2] = 0
                            if (e ** 2).sum() > best: continue
                        npts += cnt[c]; ncell += 1
        tot_pts.append(npts); tot_cells.append(ncell)
    return cs, np.prod(dim), np.mean(tot_pts), np.percentile(tot_pts, 90), np.max(tot_pts), np.mean(tot_cells)
for seq in range(int(sys.argv[2])):
    orc = O.Oracle(params); prev = None
    for k in range(4):
        orc.cloud_handler(A.synth_scan(cfg, seq, k)); fr = orc.feature_association()
        if k == 3:
            for nm, lastk, qk in (("surf", "surf_last", "flat"), ("corner", "corner_last", "sharp")):
                last = np.asarray(prev[lastk]).reshape(-1, 4)[:, :3].astype(np.float64)
                sel = t2s(np.asarray(fr[qk]).reshape(-1, 4), np.asarray(fr["transform_cur"], np.float64))
                print(nm, "n", len(last), "q", len(sel), "bbox", np.round(last.max(0) - last.min(0), 1))
                for cs0, mc, dims in ((5.01/3, 8191 if nm == "surf" else 2047, 3), (5.01/3, 2**15, 3), (5.01/3, 2**17, 3), (0.5, 2**20, 3)):
                    print("   cs0 %.2f maxcells %6d: cs %.2f cells %6d  pts/query mean %.0f p90 %.0f max %.0f cells/query %.1f" % ((cs0, mc) + grid_cost(last, sel, cs0, mc, dims)))
        prev = fr
