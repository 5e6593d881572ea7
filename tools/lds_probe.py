"""Diagnostic: which LDS sizes let 11 (10, 12) one-wave blocks share a CU (profile build).
  LEGO_FRONTEND_LIB=lego-loam-bor_amd/lego_amd/liblego_frontend_prof.so python tools/lds_probe.py"""
import ctypes as C
import os
import sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lego-loam-bor_amd"))
import lego_amd as L  # noqa: E402

lib = L.lib()
lib.lego_debug_lds_probe.argtypes = [C.c_int32, C.c_int32, C.POINTER(C.c_float)]
for per_cu in (10, 11, 12):
    for b in (13312, 13824, 14336, 14592, 14848, 14900, 15360):
        ms = C.c_float()
        lib.lego_debug_lds_probe(b, 256 * per_cu, C.byref(ms))
        print("blocks/CU %2d  LDS %6d B: %.3f ms" % (per_cu, b, ms.value), flush=True)
