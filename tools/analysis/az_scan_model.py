"""Host model (round 5): how far the azimuth bound would prune the surf scans, on the oracle's own clouds.
For each flat query of a scan (TransformToStart with the scan's final transformCur, a close stand-in for the
searches' pointSel), the brute-force 2nd / 3rd points, and how many points an exact azimuth walk would have
to visit before rho * sin(angle) exceeds the best distance.  Usage: python tools/analysis/az_scan_model.py vlp16 8
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
stats = []
for seq in range(int(sys.argv[2])):
    orc = O.Oracle(params); prev = None
    for k in range(4):
        orc.cloud_handler(A.synth_scan(cfg, seq, k)); fr = orc.feature_association()
        if k == 3 and prev is not None:
            last = np.asarray(prev["surf_last"]).reshape(-1, 4); q = np.asarray(fr["flat"]).reshape(-1, 4)
            sel = t2s(q, np.asarray(fr["transform_cur"], np.float64)); nq = len(q)
            ring = last[:, 3].astype(np.int64); az = np.arctan2(last[:, 1], last[:, 0])
            for i in range(nq):
                d = ((last[:, :3] - sel[i]) ** 2).sum(1); c = int(np.argmin(d))
                if d[c] >= 25: continue
                r0 = ring[c]; rho = np.hypot(sel[i, 0], sel[i, 1]); aq = np.arctan2(sel[i, 1], sel[i, 0])
                fwd = c + 1 < min(nq, len(last))
                m2 = (ring == r0) & (np.arange(len(last)) < c); m3 = (ring == r0 - 1) | (ring == r0 - 2)
                b2 = d[m2].min() if m2.any() else 25.0; b3 = d[m3].min() if m3.any() else 25.0
                b2 = min(b2, 25.0); b3 = min(b3, 25.0)
                da = np.abs((az - aq + np.pi) % (2 * np.pi) - np.pi)
                def need(mask, b):
                    a = np.arcsin(min(1.0, np.sqrt(b) / max(rho, 1e-9)))
                    return int((mask & (da <= a)).sum()), int(mask.sum())
                n2, t2 = need(m2, b2); n3, t3 = need(m3, b3)
                brute = int(((ring >= r0 - 2) & (np.arange(len(last)) < c)).sum())
                stats.append((fwd, rho, np.sqrt(b2), np.sqrt(b3), n2, t2, n3, t3, brute, len(last)))
        prev = fr
S = np.array(stats, float)
print("queries", len(S), "fwd-nonempty %.3f" % S[:, 0].mean(), "Last size %.0f" % S[:, 9].mean())
print("rho median %.1f; pt2 dist median %.2f (25 means none: %.2f); pt3 dist median %.2f (none %.2f)" % (
    np.median(S[:, 1]), np.median(S[:, 2]), (S[:, 2] >= 5).mean(), np.median(S[:, 3]), (S[:, 3] >= 5).mean()))
for c, nm in ((4, "pt2 needed"), (5, "pt2 total"), (6, "pt3 needed"), (7, "pt3 total"), (8, "brute range")):
    print("%-12s mean %7.1f  p50 %6.0f  p90 %6.0f  max %6.0f" % (nm, S[:, c].mean(), *np.percentile(S[:, c], [50, 90, 100])))
