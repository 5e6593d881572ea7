"""The level-synchronous formulation of libstdc++'s introsort that k_voxel (lvl_sort, lego_wavesort.h) and
the map clouds' VoxelGrid (k_vxs_*, lego_s2m.hip) run, as a position-level numpy model, against the host's
std::sort (oracle.std_sort) on tie-heavy, structured and adversarial key sequences.

The model is the algorithm's argument, checked on the CPU:
  * all ranges of one recursion level partition together (their order does not change the result), each
    with depth limit 2 floor(log2 n) - level;
  * a range [f, l) with the median-of-3 pivot at f: left stops lf(p) = !(key < pivot), right stops
    rf(p) = !(pivot < key) for p in (f, l); A(p) = #lf in (f, p), B(p) = #rf in (p, l), D = A - B
    (non-decreasing in p): a left stop is swapped iff D < 0, a right stop iff D > 0, the k-th of each kind
    with each other; the cut is the first p with (lf and D >= 0) or (rf and D > 0);
  * ranges longer than 16 at depth 0 are heap-sorted (__partial_sort); __final_insertion_sort is the
    stable order by key of the post-partition array.
(The device code's register / wave mechanics are checked on the GPU: test_device_level_sort_matches_libstdcxx,
test_voxel_std_order_key_sequences.)"""
import os
import subprocess

import numpy as np

import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _heap_sort(k, v, f, l):  # __partial_sort(first, last, last): __make_heap + __sort_heap (stl_heap.h)
    def adjust(first, hole, n, vk, vv):
        top = second = hole
        while second < (n - 1) // 2:
            second = 2 * (second + 1)
            if k[first + second] < k[first + second - 1]:
                second -= 1
            k[first + hole], v[first + hole] = k[first + second], v[first + second]
            hole = second
        if (n & 1) == 0 and second == (n - 2) // 2:
            second = 2 * (second + 1)
            k[first + hole], v[first + hole] = k[first + second - 1], v[first + second - 1]
            hole = second - 1
        parent = (hole - 1) // 2
        while hole > top and k[first + parent] < vk:
            k[first + hole], v[first + hole] = k[first + parent], v[first + parent]
            hole, parent = parent, (parent - 1) // 2
        k[first + hole], v[first + hole] = vk, vv
    n = l - f
    if n >= 2:
        for parent in range((n - 2) // 2, -1, -1):
            adjust(f, parent, n, k[f + parent], v[f + parent])
    last = l
    while last - f > 1:
        last -= 1
        vk, vv = k[last], v[last]
        k[last], v[last] = k[f], v[f]
        adjust(f, 0, last - f, vk, vv)


def level_sort(keys):
    n = len(keys)
    k = np.array(keys, np.int64)
    v = np.arange(n)
    if n <= 1:
        return k, v
    starts = np.zeros(n + 1, bool)
    starts[0] = starts[n] = True
    d0 = 2 * (n.bit_length() - 1)
    for t in range(d0 + 1):
        sp = np.flatnonzero(starts)
        first = np.repeat(sp[:-1], np.diff(sp))
        last = np.repeat(sp[1:], np.diff(sp))
        act = (last - first) > 16
        if not act.any():
            break
        if t == d0:  # depth limit
            kl, vl = list(k), list(v)
            for f, l in zip(sp[:-1], sp[1:]):
                if l - f > 16:
                    _heap_sort(kl, vl, f, l)
            k, v = np.array(kl), np.array(vl)
            break
        for f, l in zip(sp[:-1], sp[1:]):  # __move_median_to_first(f, f + 1, mid, l - 1)
            if l - f <= 16:
                continue
            x, y, z = f + 1, f + (l - f) // 2, l - 1
            if k[x] < k[y]:
                s = y if k[y] < k[z] else (z if k[x] < k[z] else x)
            else:
                s = x if k[x] < k[z] else (z if k[y] < k[z] else y)
            k[[f, s]], v[[f, s]] = k[[s, f]], v[[s, f]]
        pos = np.arange(n)
        pv = k[first]
        inner = act & (pos > first)
        lf, rf = inner & (k >= pv), inner & (k <= pv)
        cl, cr = np.concatenate([[0], np.cumsum(lf)]), np.concatenate([[0], np.cumsum(rf)])
        D = (cl[pos] - cl[first]) - (cr[last] - cr[pos + 1])
        swl, swr = lf & (D < 0), rf & (D > 0)
        cand = (lf & (D >= 0)) | (rf & (D > 0))
        nk, nv = k.copy(), v.copy()
        for f, l in zip(sp[:-1], sp[1:]):
            if l - f <= 16:
                continue
            L = np.flatnonzero(swl[f:l]) + f          # left stops in rank order
            R = (np.flatnonzero(swr[f:l]) + f)[::-1]  # right stops in rank order (from the right)
            assert len(L) == len(R) and 2 * len(L) < l - f
            nk[L], nv[L], nk[R], nv[R] = k[R], v[R], k[L], v[L]
            c = np.flatnonzero(cand[f:l])
            assert len(c) and f < f + c[0] < l
            starts[f + c[0]] = True
        k, v = nk, nv
    o = np.argsort(k, kind="stable")
    return k[o], v[o]


def _check(keys):
    keys = np.asarray(keys, np.uint32)
    ek, ev = O.std_sort(keys, np.arange(len(keys), dtype=np.int32), 0)
    gk, gv = level_sort(keys.astype(np.int64))
    assert np.array_equal(gk, ek.astype(np.int64)) and np.array_equal(gv, ev), len(keys)


def test_level_sort_model_matches_libstdcxx():
    rng = np.random.default_rng(3)
    for n in [0, 1, 2, 16, 17, 40, 65, 300, 1000, 2048, 5000]:
        for distinct in [1, 2, 7, 60, 10 ** 6]:
            _check(rng.integers(0, distinct, n))
    for n in [129, 1500, 4096]:
        i = np.arange(n)
        for keys in [i, n - i, np.minimum(i, n - i), i % 37, i // 9, (i > n // 3).astype(np.int64)]:
            _check(keys)
    rec = np.load(os.path.join(REPO, "tools", "data", "voxel_keys_heavy.npz"))  # recorded VoxelGrid rings
    for name in rec.files:
        _check(rec[name])


def test_level_sort_model_on_adversary(tmp_path):
    """libstdc++'s median-of-3 killer: ranges reach the depth limit (heap sort)."""
    exe = str(tmp_path / "ia")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-I" + os.path.join(REPO, "lego-loam-bor_amd", "csrc"),
                           os.path.join(HERE, "native", "introsort_adversary.cpp"), "-o", exe])
    for n, c in [(500, 1), (700, 2), (3000, 1), (3000, 2)]:
        out = subprocess.run([exe, str(n), str(c)], stdout=subprocess.PIPE, universal_newlines=True, check=True)
        _check(np.array(out.stdout.split(), dtype=np.int64))
