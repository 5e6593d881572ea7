"""Host model (round 5): libstdc++ introsort on VoxelGrid keys dumped by the oracle (LEGO_ORACLE_DUMP_VOXEL_KEYS):
per ring the partition work, the depth-limit heap-sort sizes, and which rings are costly.
  LEGO_ORACLE_DUMP_VOXEL_KEYS=/tmp/k.bin (oracle run) ; python tools/analysis/introsort_model.py /tmp/k.bin
"""
import sys, numpy as np
def read(fn):
    b = np.fromfile(fn, np.uint32); i = 0; rings = []
    while i < len(b):
        n = int(b[i]); rings.append(b[i+1:i+1+n].astype(np.int64)); i += 1 + n
    return rings
def lg(n): return n.bit_length() - 1
def sim(a):
    a = list(a); st = {"part": 0, "nparts": 0, "heap": [], "small": 0}
    def med3(r, x, y, z):
        ax, ay, az = a[x], a[y], a[z]
        if ax < ay:
            if ay < az: a[r], a[y] = a[y], a[r]
            elif ax < az: a[r], a[z] = a[z], a[r]
            else: a[r], a[x] = a[x], a[r]
        elif ax < az: a[r], a[x] = a[x], a[r]
        elif ay < az: a[r], a[z] = a[z], a[r]
        else: a[r], a[y] = a[y], a[r]
    def part(f, l, p):
        while True:
            while a[f] < a[p]: f += 1
            l -= 1
            while a[p] < a[l]: l -= 1
            if not (f < l): return f
            a[f], a[l] = a[l], a[f]; f += 1
    def loop(f, l, d):
        while l - f > 16:
            if d == 0:
                st["heap"].append(l - f); a[f:l] = sorted(a[f:l]); return
            d -= 1
            med3(f, f + 1, f + (l - f) // 2, l - 1)
            st["part"] += l - f; st["nparts"] += 1
            if l - f <= 64: st["small"] += 1
            c = part(f + 1, l, f)
            loop(c, l, d); l = c
    if len(a) > 1: loop(0, len(a), 2 * lg(len(a)))
    return st
rings = read(sys.argv[1])
rows = []
for r in rings:
    s = sim(r)
    rows.append((len(r), s["part"], s["nparts"], sum(s["heap"]), max(s["heap"] or [0]), len(s["heap"]), len(np.unique(r))))
R = np.array(rows)
print("rings", len(R), "n mean %.0f max %d" % (R[:,0].mean(), R[:,0].max()))
print("rings with heap fallback: %d (%.0f%%); heap len mean(when) %.0f, max %d" % ((R[:,5]>0).sum(), 100*(R[:,5]>0).mean(), R[R[:,5]>0,3].mean(), R[:,4].max()))
order = np.argsort(-R[:,4])
print("top 15 by max heap range: n, part positions, nparts, heap total, heap max, nheap, distinct")
for i in order[:15]: print(R[i])
# cost model: partitions ~ positions/64 chunks * c1 ; heap ~ total*log2 * c2
cost = R[:,1] / 64.0 * 1.0 + R[:,3] * np.log2(np.maximum(R[:,3], 2)) * 0.12
print("corr(n, cost) %.2f" % np.corrcoef(R[:,0], cost)[0,1])
top = np.argsort(-cost)[:40]
print("rank of the 40 costliest rings by size:", sorted([int((R[:,0] > R[i,0]).sum()) for i in top]))
