"""Diagnostic: kernel time of the device std::sort emulation on recorded voxel-key sets.

  LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so python tools/sort_bench.py

tools/data/voxel_keys_heavy.npz holds VoxelGrid key sequences of single rings recorded from the CPU
oracle on synthetic VLP-16 scans (c110 drives libstdc++'s introsort into a 1309-element heap-sort
fallback; c10 is an ordinary ring).  Each set is sorted by 1 block (latency) and by 256*11 blocks
(one per wave slot of the chip, throughput), with the stack emulation (wave_std_sort) and the
level-synchronous one (lvl_sort).
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
    lib.lego_debug_sort_bench.argtypes = [C.POINTER(C.c_uint32), C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_float)]
    lib.lego_debug_prof.argtypes = [C.POINTER(C.c_uint64), C.c_int32]
    d = np.load(os.path.join(REPO, "tools", "data", "voxel_keys_heavy.npz"))
    for name in d.files:
        k = np.ascontiguousarray(d[name].astype(np.uint32))
        for mode in (0,):
            for blocks in (1, 4096):  # 4096: C3's rings a step (16 a CU)
                ms = C.c_float()
                prof = (C.c_uint64 * 256)()
                lib.lego_debug_prof(prof, 1)
                rc = lib.lego_debug_sort_bench(k.ctypes.data_as(C.POINTER(C.c_uint32)), len(k), blocks, mode,
                                               C.byref(ms))
                lib.lego_debug_prof(prof, 0)
                if blocks == 1 and rc == 0:  # phase split of the one copy (shader cycles; the bench may run it more than once)
                    print("      phases (max one, cycles): partitions %d  heap fallback %d  heap pops %d  final %d" % (
                        prof[192 + 6], prof[192 + 7], prof[192 + 36], prof[192 + 11]))
                if rc != 0:
                    print("%-5s n=%5d mode %d: rc %d" % (name, len(k), mode, rc))
                    continue
                print("%-5s n=%5d %-12s blocks=%5d  %.3f ms" % (
                    name, len(k), ("stack", "level", "stack+blkins", "window only", "bitonic only")[mode], blocks, ms.value))


if __name__ == "__main__":
    main()
