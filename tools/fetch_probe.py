"""Counter calibration run (under rocprofv3 --pmc FETCH_SIZE): k_project's read patterns over the bench's
C3 input size, each mode launched REPS times.  Prints the algorithmic bytes per launch per mode."""
import ctypes as C
import sys

import torch

sys.path.insert(0, "lego-loam-bor_amd")
import lego_amd as L  # noqa: E402

S, N, REPS = 256, 26553, 5
pts = torch.randn(S * N, 4, device="cuda", dtype=torch.float32) * 20
offs = torch.arange(S, device="cuda", dtype=torch.int64) * N
cnts = torch.full((S,), N, device="cuda", dtype=torch.int32)
out = torch.zeros(S * 1024, device="cuda", dtype=torch.float32)
lib = L.lib()
lib.lego_debug_fetch_probe.argtypes = [C.c_int32, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
for mode in (0, 1, 2):
    for _ in range(REPS):
        assert lib.lego_debug_fetch_probe(mode, S, pts.data_ptr(), offs.data_ptr(), cnts.data_ptr(), out.data_ptr(),
                                          C.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
    torch.cuda.synchronize()
    print("mode %d: %d points x 16 B = %.1f MB per launch (x%d)" % (mode, S * N, S * N * 16 / 1e6, 2 if mode == 2 else 1))
