/* lego_debug.h — diagnostic entry points of the PROFILE build only (liblego_frontend_prof.so, built by
 * `python lego-loam-bor_amd/build.py --profile` with -DLG_PROFILE).  The shipped liblego_frontend.so exports
 * none of these symbols and contains none of their kernels (k_sort_bench, k_fetch_probe, k_lds_probe).
 * Used by tools/ (phase_profile.py, ring_log.py, lm_log.py, sort_bench.py, lds_probe.py, fetch_probe.py). */
#ifndef LEGO_DEBUG_H
#define LEGO_DEBUG_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* Diagnostic phase timers (shader cycles summed over waves). */
int  lego_debug_prof(uint64_t* out256, int32_t reset);
/* k_voxel's per-block log of its last launch: {start, end, n | ring id << 32, slot}, the
 * stamps from the 100 MHz real-time counter, 4 words a block. */
int  lego_debug_ring_log(uint64_t* out, int32_t n_blocks);
/* k_lm's per-block log of its last launch: {start, end (100 MHz real time), shader
 * cycles of the surf / corner grid builds, searches and iteration blocks, surf / corner iterations,
 * flat / sharp queries, surf / lessSharp Last sizes, 2 unused}, 16 words a block. */
int  lego_debug_lm_log(uint64_t* out, int32_t n_blocks);
/* Kernel time of `blocks` concurrent one-wave copies of the device sort of h_keys;
 * mode 0 the stack emulation, 1 the level-synchronous one (n <= 2048). */
int  lego_debug_sort_bench(const uint32_t* h_keys, int32_t n, int32_t blocks, int32_t mode, float* ms);
/* LDS co-residency probe: mean ms of `blocks`
 * one-wave blocks that each hold `bytes` of LDS and sleep ~20 us. */
int  lego_debug_lds_probe(int32_t bytes, int32_t blocks, float* ms);
/* Counter calibration: k_project's input read
 * patterns (mode 0 12-byte buffer loads, 1 16-byte loads, 2 both passes) over S scans of device points
 * (offs / cnts as lego_batch_run's), out[S * 1024]. */
int  lego_debug_fetch_probe(int32_t mode, int32_t S, const void* pts, const int64_t* offs, const int32_t* cnts,
                            float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* LEGO_DEBUG_H */
