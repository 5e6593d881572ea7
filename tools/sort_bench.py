"""Diagnostic: kernel time of the device std::sort emulation on recorded voxel-key sets.

  LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so python tools/sort_bench.py

tools/data/voxel_keys_heavy.npz holds VoxelGrid key sequences of single rings recorded from the CPU
oracle on synthetic VLP-16 scans (c110 drives libstdc++'s introsort into a 1309-element heap-sort
fallback; c10 is an ordinary ring).  Each set is sorted by 1 block (latency) and by 256*11 blocks
(one per wave slot of the chip, throughput), by the streaming emulation (k_voxel's) and the
level-synchronous one (voxel_std_sort).  An optional .npz of recorded rings adds their totals.
"""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lego-loam-bor_amd"))
import lego_amd as L  # noqa: E402


def main():
    lib = L.lib()
    lib.lego_debug_sort_bench.argtypes = [C.POINTER(C.c_uint32), C.c_int32, C.c_int32, C.POINTER(C.c_float)]
    d = np.load(os.path.join(REPO, "tools", "data", "voxel_keys_heavy.npz"))
    sets = [(name, np.ascontiguousarray(d[name].astype(np.uint32))) for name in d.files]
    if len(sys.argv) > 1:  # recorded rings of whole scans (tools/voxel_keys.py)
        r = np.load(sys.argv[1])
        sets += [("r%d" % i, np.ascontiguousarray(r["keys"][r["off"][i]:r["off"][i + 1]].astype(np.uint32)))
                 for i in range(len(r["off"]) - 1)]
    tot = {}
    for name, k in sets:
        for blocks in (1, 256 * 11):
            for algo, sign in (("stream", 1), ("level", -1)):
                ms = C.c_float()
                rc = lib.lego_debug_sort_bench(k.ctypes.data_as(C.POINTER(C.c_uint32)), len(k), sign * blocks,
                                               C.byref(ms))
                assert rc == 0, rc
                tot[(algo, blocks)] = tot.get((algo, blocks), 0.0) + ms.value
                if not name.startswith("r"):
                    print("%-5s n=%5d blocks=%5d %-6s %.3f ms" % (name, len(k), blocks, algo, ms.value))
    for (algo, blocks), v in sorted(tot.items()):
        print("total over %d sets: %-6s blocks=%5d %.3f ms" % (len(sets), algo, blocks, v))


if __name__ == "__main__":
    main()
