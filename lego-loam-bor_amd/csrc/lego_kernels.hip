// lego_kernels.hip — gfx950 kernels for LeGO-LOAM-BOR's per-scan front end + two-step LM.
//
// One launch per stage for ALL streams (sequences) of a batch; the stage -> kernel map:
//   k_project     ImageProjection::resetParameters/findStartEndAngle/projectPointCloud/groundRemoval
//                 (imageProjection.cpp:107-150, 234-249, 178-224, 254-346)  — workgroup per scan
//   k_segment     cloudSegmentation + labelComponents (imageProjection.cpp:352-496) as union-find
//                 connected components + raster-order compaction — workgroup per scan
//   k_fa_prep     FeatureAssociation::adjustDistortion / calculateSmoothness / markOccludedPoints
//                 (featureAssociation.cpp:161-262) + adjustOutlierCloud (:1273-1283)
//   k_extract     extractFeatures (:265-383) incl. PCL VoxelGrid per ring — one wave per ring
//   k_concat      ring-ordered concatenation of the per-ring feature clouds
//   k_lm          updateTransformation (:1213-1235) with both LM loops, integrateTransformation
//                 (:1241-1270), publishOdometry (:1286-1306), publishCloudsLast (:1329-1383)
//                 — one persistent workgroup per scan pair
// Compile with -ffp-contract=off (see lego_device.h).
#include <float.h>
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "../../include/lego_frontend.h"
#include "lego_device.h"
#include "lego_kdtree.h"
#include "lego_introsort.h"

using namespace lg;

#define DEG_TO_RAD_D (M_PI / 180.0)

// ---- diagnostic phase timers (build with -DLG_PROFILE; never in the shipped library) -----------
#ifdef LG_PROFILE
// 256 logical slots ([0,32) phases, [64+r] / [128+r] per-ring sum / max, [192+i] phase max), each in
// 64 copies picked by block index so that the timer atomics do not serialise on one address.
__device__ unsigned long long g_prof[256 * 64];
#define PROF_SLOT(i) g_prof[(size_t)(i) * 64 + (blockIdx.x & 63)]
// k_voxel's ring log of its last launch (profile build): per block {start, end, n | ring << 32, scan}
__device__ unsigned long long g_ring_log[65536 * 4];
// k_lm's per-scan log of its last launch (profile build): {start, end (real time), phase cycles [6],
// surf / corner iterations, flat / sharp queries, surf / lessSharp Last sizes}
__device__ unsigned long long g_lm_log[4096 * 16];
#define PROF_LM(i, t0) do { if (threadIdx.x == 0) L.plog[i] += __builtin_amdgcn_s_memtime() - (t0); } while (0)
#define PROF_T(v) unsigned long long v = __builtin_amdgcn_s_memtime()
#define PROF_ADD(slot, t0)                                           \
  do {                                                               \
    if ((threadIdx.x & 63) == 0) {                                   \
      const unsigned long long dt_ = __builtin_amdgcn_s_memtime() - (t0); \
      atomicAdd(&PROF_SLOT(slot), dt_);                              \
      atomicMax(&PROF_SLOT(192 + (slot)), dt_);                      \
    }                                                                \
  } while (0)
#else
#define PROF_T(v) do {} while (0)
#define PROF_ADD(slot, t0) do {} while (0)
#define PROF_LM(i, t0) do {} while (0)
#endif

#include "lego_wavesort.h"  // heap_sort_wave, lvl_sort (after the phase-timer macros it uses)
using namespace lgws;

// ============================================================================================
// block / wave helpers
// ============================================================================================
LG_DEVICE int lane_id() { return threadIdx.x & 63; }
LG_DEVICE int wave_id() { return threadIdx.x >> 6; }
LG_DEVICE int popc_below(unsigned long long m) {
  return __popcll(m & ((1ull << lane_id()) - 1ull));
}

// Raw buffer access: a load whose byte offset is >= num_records returns 0 and touches no memory,
// which makes per-lane predicated loads branch-free (no wait inside a divergent branch).
LG_DEVICE __amdgpu_buffer_rsrc_t buffer_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
LG_DEVICE float4 buffer_load_f4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  const i32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
  return make_float4(__int_as_float(v.x), __int_as_float(v.y), __int_as_float(v.z), __int_as_float(v.w));
}
LG_DEVICE float3 buffer_load_f3(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  typedef int i32x3 __attribute__((ext_vector_type(3)));
  const i32x3 v = __builtin_amdgcn_raw_buffer_load_b96(r, (int)off, 0, 0);
  return make_float3(__int_as_float(v.x), __int_as_float(v.y), __int_as_float(v.z));
}
LG_DEVICE float buffer_load_f1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __int_as_float((int)__builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
}

LG_DEVICE unsigned long long shfl64(unsigned long long v, int l) {
  return ((unsigned long long)(unsigned)__shfl((int)(v >> 32), l) << 32) | (unsigned)__shfl((int)(unsigned)v, l);
}

template <typename T>
LG_DEVICE T wave_min(T v) {
  for (int o = 32; o > 0; o >>= 1) {
    T u = __shfl_xor(v, o);
    v = u < v ? u : v;
  }
  return v;
}
template <typename T>
LG_DEVICE T wave_max(T v) {
  for (int o = 32; o > 0; o >>= 1) {
    T u = __shfl_xor(v, o);
    v = u > v ? u : v;
  }
  return v;
}
LG_DEVICE int wave_or(int v) {
  for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o);
  return v;
}
template <typename T>
LG_DEVICE T wave_sum(T v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Block-wide exclusive scan of two booleans (any block size that is a multiple of 64, <= 1024).
// scratch: >= 2*16+2 ints of LDS.
LG_DEVICE void block_scan2(bool p1, bool p2, int* scratch, int& ex1, int& ex2, int& tot1, int& tot2) {
  const int nw = blockDim.x >> 6;
  unsigned long long b1 = __ballot(p1), b2 = __ballot(p2);
  int w = wave_id();
  if (lane_id() == 0) {
    scratch[w] = __popcll(b1);
    scratch[16 + w] = __popcll(b2);
  }
  __syncthreads();
  int o1 = 0, o2 = 0, t1 = 0, t2 = 0;
  for (int k = 0; k < nw; ++k) {
    int a = scratch[k], b = scratch[16 + k];
    if (k < w) { o1 += a; o2 += b; }
    t1 += a; t2 += b;
  }
  ex1 = o1 + popc_below(b1);
  ex2 = o2 + popc_below(b2);
  tot1 = t1;
  tot2 = t2;
  __syncthreads();
}

LG_DEVICE int block_min_int(int v, int* scratch) {
  v = wave_min(v);
  if (lane_id() == 0) scratch[wave_id()] = v;
  __syncthreads();
  int r = scratch[0];
  for (int k = 1; k < (int)(blockDim.x >> 6); ++k) r = min(r, scratch[k]);
  __syncthreads();
  return r;
}
LG_DEVICE int block_max_int(int v, int* scratch) {
  v = wave_max(v);
  if (lane_id() == 0) scratch[wave_id()] = v;
  __syncthreads();
  int r = scratch[0];
  for (int k = 1; k < (int)(blockDim.x >> 6); ++k) r = max(r, scratch[k]);
  __syncthreads();
  return r;
}

// ---- projection cell of a point: exact (glibc-faithful) and fast-with-margin ------------------
// projectPointCloud (imageProjection.cpp:186-207): row = int((asin(z / range) + ang_bottom) /
// ang_res_y), col = int(-round((atan2(x, y) - pi/2) / ang_res_x) + H/2) (wrapped), range >= 0.1.
// Returns the cell (row * H + col) or -1 (rejected).
LG_DEVICE int proj_cell_exact(const LgParams& P, float4 p) {
  const float range = sqrtf(p.x * p.x + p.y * p.y + p.z * p.z);
  const float verticalAngle = asinf_g(p.z / range);
  const int rowIdn = (int)((verticalAngle + P.ang_bottom) / P.ang_res_y);
  if (rowIdn < 0 || rowIdn >= P.V) return -1;
  const float horizonAngle = atan2f_g(p.x, p.y);
  int columnIdn = (int)(-round(((double)horizonAngle - M_PI_2) / (double)P.ang_res_x) + P.H * 0.5);
  if (columnIdn >= P.H) columnIdn -= P.H;
  if (columnIdn < 0 || columnIdn >= P.H) return -1;
  if ((double)range < 0.1) return -1;
  return rowIdn * P.H + columnIdn;
}

// atan(a) on [0, 1]: a * P(a^2), P a degree-8 least-squares fit; |error| < 1e-7 evaluated in float
LG_DEVICE float atan01_poly(float a) {
  const float s = a * a;
  float p = 0.0024571234825998545f;
  p = p * s + -0.014402952045202255f;
  p = p * s + 0.03978383168578148f;
  p = p * s + -0.07235082238912582f;
  p = p * s + 0.10499055683612823f;
  p = p * s + -0.14161258935928345f;
  p = p * s + 0.1998591125011444f;
  p = p * s + -0.33332598209381104f;
  p = p * s + 0.9999998807907104f;
  return a * p;
}

// The same decisions without the libm restatements, from approximations whose errors are bounded
// far below the margins: the row from a reciprocal-sqrt and fdlibm's small-argument asin polynomial
// (|v - v_exact| < 1e-4 row units; margin 2e-3), the column from a polynomial atan2 (< 2e-6 rad,
// i.e. < 1e-3 column units with the rounding of the scaled angle; margin 4e-3 from the .5 rounding
// boundary), the range test from |p|^2 against [0.0099, 0.0101].  Returns the cell, -1 (rejected) or
// -2: too close to a decision boundary to tell, the exact path decides.  The margins hold for
// ang_res_y >= 0.1 deg and ang_res_x >= 0.1 deg (lg_fast_projection checks them).
// kLayout: the cell as row * H + col (0), col * V + row (1: the wide winner image) or row << 16 | col (2)
template <int kLayout = 0>
LG_DEVICE int proj_cell_fast(const LgParams& P, float4 p) {
  const float d2 = p.x * p.x + p.y * p.y + p.z * p.z;
  if (!(d2 > 0.0101f)) return d2 < 0.0099f ? -1 : -2;
  const float t = p.z * __builtin_amdgcn_rsqf(d2);
  if (!(fabsf(t) < 0.49f)) return -2;
  const float tt = t * t;
  const float w = tt * (1.666675248e-1f + tt * (7.495297643e-2f + tt * (4.547037598e-2f + tt * (2.417951451e-2f + tt * 4.216630880e-2f))));
  const float va = t + t * w;
  const float v = (va + P.ang_bottom) * P.inv_res_y;
  const float mr = 2e-3f;
  const int r0 = (int)(v - mr), r1 = (int)(v + mr);
  if (r0 != r1) return -2;
  if (r0 < 0 || r0 >= P.V) return -1;
  // horizonAngle = atan2(x, y)
  const float ax = fabsf(p.y), ay = fabsf(p.x);
  const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
  if (!(mx > 0.f)) return -2;
  float h = atan01_poly(mn * __builtin_amdgcn_rcpf(mx));
  if (ay > ax) h = 1.57079637f - h;
  if (p.y < 0.f) h = 3.14159274f - h;
  if (p.x < 0.f) h = -h;
  const float q = (h - 1.57079637f) * P.inv_res_x;
  const float fq = floorf(q), fr = q - fq;
  if (fabsf(fr - 0.5f) < 4e-3f) return -2;
  const int k = (int)fq + (fr > 0.5f ? 1 : 0);  // round(q), q not near a half
  // (int)(-k + H * 0.5) in double: the real (H - 2k) / 2 truncated toward zero, as C++ int division
  int columnIdn = (P.H - 2 * k) / 2;
  if (columnIdn >= P.H) columnIdn -= P.H;
  if (columnIdn < 0 || columnIdn >= P.H) return -1;
  return kLayout == 1 ? columnIdn * P.V + r0 : kLayout == 2 ? (r0 << 16) | columnIdn : r0 * P.H + columnIdn;
}

// groundRemoval's test (imageProjection.cpp:276-285): (double)(va - mount) <= 10 deg with va =
// std::atan2(dZ, sqrt(s2)), s2 = dX*dX + dY*dY + dZ*dZ in float: atan2f(dZ, sqrtf(s2)) with the float
// overloads (fp_mode 0); with ::sqrt(double) (fp_mode 1) the std::atan2(float, double) overload
// promotes, va = (float)atan2(double(dZ), sqrt(double(s2))).  r = sqrt(s2) >= |dZ|, so the angle lies
// in [-pi/4, pi/4].  A pair with an empty cell (NaN) is never ground (atan2 of a NaN is NaN in both
// models).  A polynomial atan (error < 1e-6 rad with the reciprocal) decides every pair farther than
// 1e-5 rad from the threshold in both models; the rest, and r == 0, take the glibc-faithful path of
// the model.
__attribute__((noinline)) __device__ bool ground_pair_exact(float dZ, float s2, float mount, int fp1) {  // one copy
  const float va = fp1 ? (float)atan2_d((double)dZ, sqrt((double)s2)) : atan2f_g(dZ, sqrtf(s2));
  return (double)(va - mount) <= 10 * DEG_TO_RAD_D;
}
LG_DEVICE bool ground_pair(float dZ, float s2, float mount, int fp1) {
  // an empty cell (nanPoint) on either side: every model's angle is NaN and the test false
  if (__builtin_isnan(dZ) || __builtin_isnan(s2)) return false;
  const double thr = 10 * DEG_TO_RAD_D;
  const float r = sqrtf(s2);
  if (r > 0.f && r < FLT_MAX) {
    float h = atan01_poly(fminf(fabsf(dZ) * __builtin_amdgcn_rcpf(r), 1.f));
    const float d = (dZ < 0.f ? -h : h) - mount;
    if (d < (float)thr - 1e-5f) return true;
    if (d > (float)thr + 1e-5f) return false;
  }
  return ground_pair_exact(dZ, s2, mount, fp1);
}

// ============================================================================================
// k_project: reset + findStartEndAngle + projectPointCloud + groundRemoval + 2-D scan candidates
// ============================================================================================
// The reference's scatter "later input point overwrites earlier ones in the same cell"
// (imageProjection.cpp:214-222) is an atomicMax of the input index per cell, followed by a
// column-parallel gather that writes every cell (so resetParameters' fill is fused in).
#define PQ_CAP 128  // per-wave queue of undecided points: < 64 before an append of <= 64
// The exact path for the 64 queued points q[0, 64) (lane l takes q[l]).  Out of line: it runs for
// ~0.3% of the points, and one copy of the libm restatements serves every call site.
// (The projection constants go by value: a reference into the kernel arguments would be copied to
// the stack for the call.)
__attribute__((noinline)) __device__ int proj_cell_exact_ni(float ang_bottom, float res_x, float res_y, int V, int H,
                                                          float4 p) {  // one out-of-line copy
  LgParams P;
  P.ang_bottom = ang_bottom;
  P.ang_res_x = res_x;
  P.ang_res_y = res_y;
  P.V = V;
  P.H = H;
  return proj_cell_exact(P, p);
}
// cell (row-major, or -1) -> column-major index j * V + i (wide mode's winner image)
LG_DEVICE int cell_cm(int c, int V, int H) {
  if (c < 0) return c;
  const int i = c / H;
  return (c - i * H) * V + i;
}
__attribute__((noinline)) __device__ void proj_drain_cm(float ang_bottom, float res_x, float res_y, int V, int H,
                                                        const float4* in, const int* q, unsigned* winner,
                                                        unsigned tag) {
  LgParams P;
  P.ang_bottom = ang_bottom;
  P.ang_res_x = res_x;
  P.ang_res_y = res_y;
  P.V = V;
  P.H = H;
  const int i = q[lane_id()];
  const int c = cell_cm(proj_cell_exact(P, in[i]), V, H);
  if (c >= 0) atomicMax(&winner[c], tag | (unsigned)i);
}
__attribute__((noinline)) __device__ void proj_drain(float ang_bottom, float res_x, float res_y, int V, int H,
                                                     const float4* in, const int* q, int* winner) {
  LgParams P;
  P.ang_bottom = ang_bottom;
  P.ang_res_x = res_x;
  P.ang_res_y = res_y;
  P.V = V;
  P.H = H;
  const int i = q[lane_id()];
  const int c = proj_cell_exact(P, in[i]);
  if (c >= 0) atomicMax(&winner[c], i);
}
// Column pass of column j: the lane walks the rows bottom-up.  Each chunk of CR rows first reads its
// CR winners and gathers their points (unconditional loads, all in flight together), then writes
// range / cloud cells, the ground pairs (i-1, i) of groundRemoval (:271-285), and row i-1's ground
// flag and 2-D scan candidate (:312-330) as soon as pair (i-1, i) has settled it.
template <int CR>
LG_DEVICE void proj_column(const LgParams& P, const LgBufs& B, int s, int j, const int* winner, const float4* src0,
                           float* range, float4* cloud, int8_t* ground) {
  const int V = P.V, H = P.H;
  const float qnan = __int_as_float(0x7fc00000);
  unsigned long long gmask = 0ull;
  float4 prev = make_float4(0.f, 0.f, 0.f, 0.f);
  float prev_r = 0.f;
  float min_range = 1000.f;
  int id_min = -1;
  const double jfrac = (double)(float)j / 10000.0;
  auto scan = [&](int i, float r, float Z) {  // 2-D scan (:312-330), row i final
    const int c = i * H + j;
    const int g = (int)((gmask >> i) & 1ull);
    ground[c] = (int8_t)g;
    if (g != 1 && (double)Z > 0.4 && (double)Z < 1.2 && r < 40.f && r < min_range) {
      min_range = r;
      id_min = c;
    }
  };
  for (int i0 = 0; i0 < V; i0 += CR) {
    int w[CR];
    float4 pk[CR];
#pragma unroll
    for (int u = 0; u < CR; ++u) w[u] = (i0 + u < V) ? winner[(i0 + u) * H + j] : -1;
#pragma unroll
    for (int u = 0; u < CR; ++u) pk[u] = src0[w[u] >= 0 ? w[u] : 0];
#pragma unroll
    for (int u = 0; u < CR; ++u) {
      const int i = i0 + u;
      if (i >= V) continue;  // (not `break`: the loop must stay unrollable, pk[] in registers)
      const int c = i * H + j;
      float4 q;
      float r;
      if (w[u] >= 0) {
        const float4 p = pk[u];
        r = sqrtf(p.x * p.x + p.y * p.y + p.z * p.z);
        q = make_float4(p.x, p.y, p.z, (float)((double)(float)i + jfrac));
      } else {
        r = FLT_MAX;
        q = make_float4(qnan, qnan, qnan, 0.f);  // nanPoint: PCL default intensity 0
      }
      st_nt(&range[c], r);  // streaming stores: the input lines stay in L2 for the gathers
      st_nt(&cloud[c], q);
      if (i >= 1 && i <= P.G) {  // pair (i-1, i): groundRemoval :271-285
        const float dX = q.x - prev.x, dY = q.y - prev.y, dZ = q.z - prev.z;
        if (ground_pair(dZ, dX * dX + dY * dY + dZ * dZ, P.mount, P.fp1)) gmask |= (3ull << (i - 1));
      }
      if (i >= 1) scan(i - 1, prev_r, prev.z);
      prev = q;
      prev_r = r;
    }
  }
  scan(V - 1, prev_r, prev.z);
  B.scan_cand[(size_t)s * H + j] = (min_range < 1000.f) ? id_min : -1;
}

// findStartEndAngle (:234-249) from the first / last finite point (thread 0)
LG_DEVICE void proj_orient(const LgParams& P, const LgBufs& B, int s, const float4* in, int fmin, int fmax) {
  float so = 0.f, eo = 0.f, od = 0.f;
  if (fmax >= 0) {
    float4 a = in[fmin], b = in[fmax];
    so = -atan2f_g(a.y, a.x);
    eo = (float)(-(double)atan2f_g(b.y, b.x) + 2 * M_PI);
    if ((double)(eo - so) > 3 * M_PI) eo = (float)((double)eo - 2 * M_PI);
    else if ((double)(eo - so) < M_PI) eo = (float)((double)eo + 2 * M_PI);
    od = eo - so;
  }
  B.orient[s * 4 + 0] = so;
  B.orient[s * 4 + 1] = eo;
  B.orient[s * 4 + 2] = od;
  B.orient[s * 4 + 3] = (float)(fmax >= 0);
  B.fe_state[2 * s] = (fmax >= 0) ? LEGO_OK : LEGO_EEMPTY;
}

// k_project's body (one 1,024-thread workgroup a scan; smem: the dynamic LDS, lg_lds_projection)
LG_DEVICE void project_lds(const LgParams& P, const LgBufs& B, const float4* __restrict__ pts,
                           const int64_t* __restrict__ offs, const int32_t* __restrict__ cnts, int* smem) {
  const int s = P.s0 + blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  const int V = P.V, H = P.H, VH = P.VH;
  int* scratch = smem;                 // 64 ints
  int* winner = smem + 64;  // LDS image: V*H ints
  const float4* in = pts + offs[s];
  const int n = cnts[s];
  // the first batch's point loads go out before the LDS image reset (see below)
  constexpr int kU = 8;
  const __amdgpu_buffer_rsrc_t rin = buffer_rsrc(in, (uint32_t)n * 16u);
  float3 pk[kU];
#pragma unroll
  for (int u = 0; u < kU; ++u) pk[u] = buffer_load_f3(rin, (uint32_t)(tid + u * nt) * 16u);
  PROF_T(t_p0);
  for (int c = tid; c < VH; c += nt) winner[c] = -1;
  __syncthreads();
  PROF_ADD(20, t_p0);
  PROF_T(t_p1);
  int fmin = 0x7fffffff, fmax = -1;
  // The points' x, y, z (12-byte buffer loads; the input intensity is not used) in batches of kU per
  // lane, the next batch's loads issued before the current batch is processed.  Lanes past n load
  // nothing (buffer range check).  Cells come from the fast path; the few points it cannot decide
  // queue per wave and take the exact path 64 at a time.
  int* queue = smem + 64 + VH + wave_id() * PQ_CAP;  // PQ_CAP ints per wave
  int qn = 0;
  for (int i0 = tid; i0 < n; i0 += nt * kU) {
    float3 nx[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) nx[u] = buffer_load_f3(rin, (uint32_t)(i0 + (kU + u) * nt) * 16u);
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = i0 + u * nt;
      const float4 p = make_float4(pk[u].x, pk[u].y, pk[u].z, 0.f);
      int c = -1;
      if (i < n && isfinite_f(p.x) && isfinite_f(p.y) && isfinite_f(p.z)) {  // removeNaNFromPointCloud
        fmin = min(fmin, i);
        fmax = max(fmax, i);
        c = P.fast_proj ? proj_cell_fast(P, p) : proj_cell_exact_ni(P.ang_bottom, P.ang_res_x, P.ang_res_y, V, H, p);
        if (c >= 0) atomicMax(&winner[c], i);
      }
      const unsigned long long amb = __ballot(c == -2);
      if (c == -2) queue[qn + popc_below(amb)] = i;
      qn += __popcll(amb);
      if (qn >= 64) {  // wave-uniform, rare: the oldest 64 take the exact path
        proj_drain(P.ang_bottom, P.ang_res_x, P.ang_res_y, V, H, in, queue + qn - 64, winner);
        qn -= 64;
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) pk[u] = nx[u];
  }
  if (qn > 0) {  // the rest (< 64): lanes past qn repeat entry 0 (the same max, harmless)
    if (lane_id() >= qn) queue[lane_id()] = queue[0];
    proj_drain(P.ang_bottom, P.ang_res_x, P.ang_res_y, V, H, in, queue, winner);
  }
  PROF_ADD(21, t_p1);
  PROF_T(t_p2);
  // first / last finite point: per-wave results now, combined by thread 0 after the column pass
  // (findStartEndAngle's result is not needed before then; no extra barrier)
  fmin = wave_min(fmin);
  fmax = wave_max(fmax);
  if (lane_id() == 0) {
    scratch[wave_id()] = fmin;
    scratch[32 + wave_id()] = fmax;
  }
  __syncthreads();
  PROF_ADD(22, t_p2);
  PROF_T(t_p3);
  // Column pass: one lane per column (proj_column)
  float* range = B.range + (size_t)s * VH;
  float4* cloud = B.cloud + (size_t)s * VH;
  int8_t* ground = B.ground + (size_t)s * VH;
  const float4* src0 = n > 0 ? in : cloud;  // any readable address for empty cells (value unused)
  for (int j = tid; j < H; j += nt) proj_column<16>(P, B, s, j, winner, src0, range, cloud, ground);
  PROF_ADD(23, t_p3);
  if (tid == 0) {
    for (int w = 1; w < (nt >> 6); ++w) {
      fmin = min(fmin, scratch[w]);
      fmax = max(fmax, scratch[32 + w]);
    }
    proj_orient(P, B, s, in, fmin, fmax);
  }
}

// ============================================================================================
// Wide mode (large images: HDL-64E's 64 x 2048; few scans in flight): each scan's projection and
// segmentation spread over many workgroups instead of one, with the per-scan state in HBM.
// ============================================================================================
// k_pw_scatter: grid (point chunks of PW_PTS, scans).  "Later point wins" is a device-scope
// atomicMax of the input index into the scan's winner image; each entry carries the launch's tag
// (P.wtag: a launch counter 1..15 in the top 4 bits, the index in the low 28), so entries of earlier
// launches are smaller than any of this one and read as empty by k_pw_columns, and the image needs no
// reset between launches (the host zeroes it when the counter wraps).  The first / last finite
// point go to proj_mm by atomicMin / Max.  The
// image is column-major (cell (i, j) at j * V + i): one firing's lasers are consecutive points and
// land in consecutive words, so a wave's atomics touch a few cache lines instead of one per lane.
// kNB batches of 8 points a lane per workgroup: 4 when many scans are in flight (fewer, longer
// workgroups stream the input with the next batch's loads in flight), 1 for few scans (more
// workgroups a scan).
#ifndef LG_PW_SLICE  // the shipped wide projection: scatter + column pass
#define PW_NT 256
#define PW_PTS (PW_NT * 8)  // points a batch
template <int kNB>
__global__ __launch_bounds__(PW_NT) void k_pw_scatter(LgParams P, LgBufs B, const float4* __restrict__ pts,
                                                      const int64_t* __restrict__ offs,
                                                      const int32_t* __restrict__ cnts) {
  __shared__ int queue_all[(PW_NT / 64) * PQ_CAP];
  const int s = P.s0 + blockIdx.y, tid = threadIdx.x;
  const int V = P.V, H = P.H;
  const int n = cnts[s];
  const int c0 = blockIdx.x * PW_PTS * kNB;
  if (c0 >= n) return;
  unsigned* winner = (unsigned*)B.winner + (size_t)s * P.VH;
  const unsigned tag = P.wtag;
  const float4* in = pts + offs[s];
  const __amdgpu_buffer_rsrc_t rin = buffer_rsrc(in, (uint32_t)n * 16u);
  int* queue = queue_all + wave_id() * PQ_CAP;
  int qn = 0;
  int fmin = 0x7fffffff, fmax = -1;
  constexpr int kU = 8;
  // the batches' loads double-buffered: batch b + 1's go out before batch b is processed
  float3 pk[kU];
#pragma unroll
  for (int u = 0; u < kU; ++u) pk[u] = buffer_load_f3(rin, (uint32_t)(c0 + u * PW_NT + tid) * 16u);
  for (int b = 0; b < kNB; ++b) {
    const int i0 = c0 + b * kU * PW_NT;
    if (i0 >= n) break;
    float3 nx[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) nx[u] = buffer_load_f3(rin, (uint32_t)(i0 + (kU + u) * PW_NT + tid) * 16u);
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = i0 + u * PW_NT + tid;
      const float4 p = make_float4(pk[u].x, pk[u].y, pk[u].z, 0.f);
      int c = -1;
      if (i < n && isfinite_f(p.x) && isfinite_f(p.y) && isfinite_f(p.z)) {  // removeNaNFromPointCloud
        fmin = min(fmin, i);
        fmax = max(fmax, i);
        c = P.fast_proj ? proj_cell_fast<1>(P, p)
                        : cell_cm(proj_cell_exact_ni(P.ang_bottom, P.ang_res_x, P.ang_res_y, V, H, p), V, H);
        if (c >= 0) atomicMax(&winner[c], tag | (unsigned)i);
      }
      const unsigned long long amb = __ballot(c == -2);
      if (c == -2) queue[qn + popc_below(amb)] = i;
      qn += __popcll(amb);
      if (qn >= 64) {
        proj_drain_cm(P.ang_bottom, P.ang_res_x, P.ang_res_y, V, H, in, queue + qn - 64, winner, tag);
        qn -= 64;
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) pk[u] = nx[u];
  }
  if (qn > 0) {
    if (lane_id() >= qn) queue[lane_id()] = queue[0];
    proj_drain_cm(P.ang_bottom, P.ang_res_x, P.ang_res_y, V, H, in, queue, winner, tag);
  }
  fmin = wave_min(fmin);
  fmax = wave_max(fmax);
  if (lane_id() == 0 && fmax >= 0) {
    atomicMin(&B.proj_mm[2 * s], fmin);
    atomicMax(&B.proj_mm[2 * s + 1], fmax);
  }
}

#endif  // !LG_PW_SLICE

// The column pass of one column j from its cells' points, NQ lanes a column, R rows a lane (V <= R * NQ):
// lane q of the column holds rows Rq .. Rq + R - 1, pk[u] the x, y, z of row Rq + u (NaN for an empty
// cell, nanPoint) and bit u of hm whether that row has a point.  Writes the range / cloud / ground cells
// and the 2-D scan candidate of the column when `col` (lanes with !col take part in the shuffles only).
// The pair (Rq - 1, Rq) of groundRemoval (:271-285) is settled by lane q with lane q - 1's last point
// (shuffled up), and its result for row 16q - 1 goes back down; the 2-D scan candidate (:312-330) is the
// (range, row) minimum over the lanes, which is what the sequential bottom-up scan with a strict `<` picks.
template <int NQ, int R = 16>
LG_DEVICE void pw_column_emit(const LgParams& P, const LgBufs& B, int s, int j, int q, bool col, const float3 (&pk)[R],
                              unsigned hm) {
  const int V = P.V, H = P.H, VH = P.VH, i0 = R * q;
  float* range = B.range + (size_t)s * VH;
  float4* cloud = B.cloud + (size_t)s * VH;
  int8_t* ground = B.ground + (size_t)s * VH;
  const double jfrac = (double)(float)j / 10000.0;
  // groundRemoval (:271-285): pair (i-1, i) for 1 <= i <= G marks both rows
  unsigned gm = 0u;  // bit u: row i0 + u
  float3 below = make_float3(0.f, 0.f, 0.f);
  if constexpr (NQ > 1) {
    below.x = __shfl_up(pk[R - 1].x, 1, NQ);
    below.y = __shfl_up(pk[R - 1].y, 1, NQ);
    below.z = __shfl_up(pk[R - 1].z, 1, NQ);
  }
  bool down = false;  // pair (i0 - 1, i0) marks row i0 - 1, lane q - 1's last row
  if (NQ > 1 && q > 0 && i0 <= P.G && col && i0 < V) {
    const float dX = pk[0].x - below.x, dY = pk[0].y - below.y, dZ = pk[0].z - below.z;
    if (ground_pair(dZ, dX * dX + dY * dY + dZ * dZ, P.mount, P.fp1)) {
      gm |= 1u;
      down = true;
    }
  }
#pragma unroll
  for (int u = 1; u < R; ++u) {
    const int i = i0 + u;
    if (col && i < V && i <= P.G) {
      const float dX = pk[u].x - pk[u - 1].x, dY = pk[u].y - pk[u - 1].y, dZ = pk[u].z - pk[u - 1].z;
      if (ground_pair(dZ, dX * dX + dY * dY + dZ * dZ, P.mount, P.fp1)) gm |= 3u << (u - 1);
    }
  }
  if constexpr (NQ > 1) {
    const int dn = __shfl_down((int)down, 1, NQ);
    if (q + 1 < NQ && dn) gm |= 1u << (R - 1);
  }
  float min_range = 1000.f;
  int id_min = 0x7fffffff;
  if (col) {
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const int i = i0 + u;
      if (i >= V) continue;
      const int c = i * H + j;
      const float3 p = pk[u];
      const bool h = (hm >> u) & 1u;
      const float r = h ? sqrtf(p.x * p.x + p.y * p.y + p.z * p.z) : FLT_MAX;
      st_nt(&range[c], r);
      st_nt(&cloud[c], make_float4(p.x, p.y, p.z, h ? (float)((double)(float)i + jfrac) : 0.f));  // nanPoint: 0
      const int g = (int)((gm >> u) & 1u);
      ground[c] = (int8_t)g;
      if (g != 1 && (double)p.z > 0.4 && (double)p.z < 1.2 && r < 40.f && r < min_range) {  // 2-D scan (:312-330)
        min_range = r;
        id_min = c;
      }
    }
  }
  if constexpr (NQ > 1) {
#pragma unroll
    for (int o = 1; o < NQ; o <<= 1) {
      const float o_r = __shfl_xor(min_range, o, NQ);
      const int o_c = __shfl_xor(id_min, o, NQ);
      if (o_r < min_range || (o_r == min_range && o_c < id_min)) {
        min_range = o_r;
        id_min = o_c;
      }
    }
  }
  if (col && q == 0) B.scan_cand[(size_t)s * H + j] = (min_range < 1000.f) ? id_min : -1;
}

// findStartEndAngle (:234-249) of scan s from proj_mm, which is left reset for the next launch
LG_DEVICE void pw_orient(const LgParams& P, const LgBufs& B, int s, const float4* in) {
  const int fmin = B.proj_mm[2 * s], fmax = B.proj_mm[2 * s + 1];
  B.proj_mm[2 * s] = 0x7fffffff;
  B.proj_mm[2 * s + 1] = -1;
  proj_orient(P, B, s, in, fmin, fmax);
}

#ifdef LG_PW_SLICE
// ---- the wide projection in one read of the input (round 6; built with -DLG_PW_SLICE, not shipped) ------
// Measured against the shipped scatter + column pass (tools/proj_time.py): correct (every wide
// parity test) but slower: 0.15 vs 0.11 ms for 256 VLP-16 scans, 1.0 vs 0.55 ms for HDL-64E.
// k_pw_slice: grid (slices of PWS_NT * kU consecutive input points, scans).  The input is in firing order
// (azimuth-major), so a slice's points land in a narrow band of columns.  A slice resolves "later point
// wins" (imageProjection.cpp:214-222) for its own points in an LDS image of that band (atomicMax of the
// point's slot), keeps its points' x, y, z in LDS, and runs the column pass (pw_column_emit) of every
// band column it touched: range / cloud / ground cells, the 2-D scan candidate.  Each point is read from
// HBM once and each cell of an uncontested column written once.  Whether another slice also touched a
// column is only known after every slice ran: each slice counts its touch in colcnt[column] (+1), and
// publishes its band winners to the scan's winner image W (tagged atomicMax as k_pw_scatter) for the
// PW_EDGE columns at either end of its band (+0x1000: "published"), where consecutive slices meet, and
// for its whole band if it is the scan's first or last slice (the seam of the sweep).  A slice whose
// band does not fit (input not in firing order) publishes every point to W and marks its columns
// (bit 31).  k_pw_fix then settles every column: touched by exactly one band slice -> done; by none ->
// empty cells; otherwise rebuilt from W, or, when a band slice touched it without publishing it (a
// second sweep over the same azimuth), from a rescan of the scan's input for that column block.
#define PWS_NT 256
#define PW_EDGE 4  // band columns at either end of a slice published to the winner image

// The exact path for 64 queued slots of a slice (lane l takes q[l]): the point read from the input, its
// cell as row << 16 | col (or -1) into pcell.
__attribute__((noinline)) __device__ void proj_drain_slot(float ang_bottom, float res_x, float res_y, int V, int H,
                                                          const float4* in, int c0, const int* q, int* pcell) {
  LgParams P;
  P.ang_bottom = ang_bottom;
  P.ang_res_x = res_x;
  P.ang_res_y = res_y;
  P.V = V;
  P.H = H;
  const int k = q[lane_id()];
  const float4 p = in[c0 + k];
  const int c = proj_cell_exact(P, make_float4(p.x, p.y, p.z, 0.f));
  pcell[k] = c < 0 ? -1 : ((c / H) << 16) | (c - (c / H) * H);
}

#ifdef LG_PWS_STATS  // diagnostic builds only: [0] fallback slices [1] band slices [2] owned [3] empty
                     // [4] contested complete [5] incomplete columns [6] rescan blocks
__device__ unsigned long long g_pws[8];
#define PWS_STAT(i, v) atomicAdd(&g_pws[i], (unsigned long long)(v))
#else
#define PWS_STAT(i, v) do {} while (0)
#endif

// k_pw_slice's LDS.  VM: rows (V <= VM); NBC: band columns held (a wider band: input out of firing order).
template <int kU, int VM, int NBC>
struct PwSliceLds {
  static constexpr int PS = PWS_NT * kU;  // points a slice
  static constexpr int NW = PWS_NT / 64;
  static constexpr int VS = VM + 1;       // band image column stride (rows, then the touched flag)
  int pcell[PS];                          // the slice's cells, row << 16 | col (-1: none)
  int bwin[NBC * VS];                     // band image: winning slot a cell (-1: empty); [k * VS + VM]: touched
  unsigned gbits[NBC * 2];                // ground rows of a band column (groundRemoval's pairs)
  unsigned long long scan[NBC];           // 2-D scan candidate of a band column: range bits << 32 | cell
  int queue[NW * PQ_CAP];
  int red[4 * NW];
};

#ifndef LG_PWS_WPE
#define LG_PWS_WPE 5
#endif
#define LG_PWS_ATTR __attribute__((amdgpu_waves_per_eu(LG_PWS_WPE)))
template <int kU, int VM, int NBC>
__global__ __launch_bounds__(PWS_NT) LG_PWS_ATTR void k_pw_slice(LgParams P, LgBufs B, const float4* __restrict__ pts,
                                                                 const int64_t* __restrict__ offs,
                                                                 const int32_t* __restrict__ cnts) {
  using Lds = PwSliceLds<kU, VM, NBC>;
  constexpr int PS = Lds::PS, NW = Lds::NW, VS = Lds::VS;
  __shared__ Lds L;
  const int s = P.s0 + blockIdx.y, tid = threadIdx.x;
  const int V = P.V, H = P.H;
  const int n = cnts[s];
  const int c0 = blockIdx.x * PS;
  if (c0 >= n) return;
  const float4* in = pts + offs[s];
  const __amdgpu_buffer_rsrc_t rin = buffer_rsrc(in, (uint32_t)n * 16u);
  int* queue = L.queue + wave_id() * PQ_CAP;
  int qn = 0, fmin = 0x7fffffff, fmax = -1;
  {
    float3 pk[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) pk[u] = buffer_load_f3(rin, (uint32_t)(c0 + u * PWS_NT + tid) * 16u);
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int slot = u * PWS_NT + tid, i = c0 + slot;
      const float4 p = make_float4(pk[u].x, pk[u].y, pk[u].z, 0.f);
      int c = -1;
      if (i < n && isfinite_f(p.x) && isfinite_f(p.y) && isfinite_f(p.z)) {  // removeNaNFromPointCloud
        fmin = min(fmin, i);
        fmax = max(fmax, i);
        if (P.fast_proj) {
          c = proj_cell_fast<2>(P, p);
        } else {
          c = proj_cell_exact_ni(P.ang_bottom, P.ang_res_x, P.ang_res_y, V, H, p);
          c = c < 0 ? -1 : ((c / H) << 16) | (c - (c / H) * H);
        }
      }
      L.pcell[slot] = c;
      const unsigned long long amb = __ballot(c == -2);
      if (c == -2) queue[qn + popc_below(amb)] = slot;
      qn += __popcll(amb);
      if (qn >= 64) {  // wave-uniform, rare: the oldest 64 take the exact path
        proj_drain_slot(P.ang_bottom, P.ang_res_x, P.ang_res_y, V, H, in, c0, queue + qn - 64, L.pcell);
        qn -= 64;
      }
    }
  }
  if (qn > 0) {  // the rest (< 64): lanes past qn repeat entry 0 (the same write, harmless)
    if (lane_id() >= qn) queue[lane_id()] = queue[0];
    proj_drain_slot(P.ang_bottom, P.ang_res_x, P.ang_res_y, V, H, in, c0, queue, L.pcell);
  }
  fmin = wave_min(fmin);
  fmax = wave_max(fmax);
  if (lane_id() == 0 && fmax >= 0) {  // findStartEndAngle's first / last finite point (k_pw_fix settles it)
    atomicMin(&B.proj_mm[2 * s], fmin);
    atomicMax(&B.proj_mm[2 * s + 1], fmax);
  }
  __syncthreads();
#if defined(LG_PWS_CUT) && LG_PWS_CUT == 1
  return;
#endif
  // The band: the slice's column range, directly or rotated by half a turn (a slice across the column
  // wrap), whichever is narrower.  jr = (j + Hr) mod H, j = (jr + Hh) mod H.
  const int Hh = H / 2, Hr = H - Hh;
  int m0 = 0x7fffffff, x0 = -1, m1 = 0x7fffffff, x1 = -1;
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const int c = L.pcell[u * PWS_NT + tid];
    if (c >= 0) {
      const int j = c & 0xffff, jr = j < Hh ? j + Hr : j - Hh;
      m0 = min(m0, j); x0 = max(x0, j);
      m1 = min(m1, jr); x1 = max(x1, jr);
    }
  }
  m0 = wave_min(m0); x0 = wave_max(x0); m1 = wave_min(m1); x1 = wave_max(x1);
  if (lane_id() == 0) {
    L.red[4 * wave_id()] = m0; L.red[4 * wave_id() + 1] = x0; L.red[4 * wave_id() + 2] = m1; L.red[4 * wave_id() + 3] = x1;
  }
  __syncthreads();
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    m0 = min(m0, L.red[4 * w]); x0 = max(x0, L.red[4 * w + 1]);
    m1 = min(m1, L.red[4 * w + 2]); x1 = max(x1, L.red[4 * w + 3]);
  }
  if (x0 < 0) return;  // no point of the slice has a cell (block-uniform)
  const bool rot = x1 - m1 < x0 - m0;
  const int base = rot ? m1 : m0, bw = (rot ? x1 - m1 : x0 - m0) + 1;
  unsigned* W = (unsigned*)B.winner + (size_t)s * P.VH;
  int* colcnt = B.colcnt + (size_t)s * H;
  const unsigned tag = P.wtag;
  if (tid == 0) PWS_STAT(bw > NBC ? 0 : 1, 1);
  if (bw > NBC) {  // not in firing order: every point to the winner image, its columns marked
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int c = L.pcell[u * PWS_NT + tid];
      if (c < 0) continue;
      const int j = c & 0xffff;
      atomicMax(&W[j * V + (c >> 16)], tag | (unsigned)(c0 + u * PWS_NT + tid));
      atomicOr(&colcnt[j], (int)0x80000000);
    }
    return;
  }
  for (int e = tid; e < bw * VS; e += PWS_NT) {
    const int k = e / VS;
    L.bwin[e] = (e - k * VS == VM) ? 0 : -1;
  }
  for (int k = tid; k < bw; k += PWS_NT) {
    L.gbits[2 * k] = 0u;
    L.gbits[2 * k + 1] = 0u;
    L.scan[k] = ~0ull;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const int c = L.pcell[u * PWS_NT + tid];
    if (c < 0) continue;
    const int j = c & 0xffff;
    const int k = (rot ? (j < Hh ? j + Hr : j - Hh) : j) - base;
    atomicMax(&L.bwin[k * VS + (c >> 16)], u * PWS_NT + tid);  // later point wins
    L.bwin[k * VS + VM] = 1;                                  // touched
  }
  __syncthreads();
#if defined(LG_PWS_CUT) && LG_PWS_CUT == 2
  return;
#endif
  auto colof = [&](int k) {
    const int jv = base + k;
    return rot ? (jv + Hh < H ? jv + Hh : jv + Hh - H) : jv;
  };
  const float qnan = __int_as_float(0x7fc00000);
  // groundRemoval (:271-285): the pairs (r, r + 1), r < G, of every touched band column, in strips of 8 rows
  // a lane (the winners' points read again from the input, which this workgroup has just read: L2)
  const int G = P.G, nstrip = (G + 7) >> 3;
  for (int e = tid; e < nstrip * bw; e += PWS_NT) {
    const int st = e / bw, k = e - st * bw, r0 = st << 3;
    if (!L.bwin[k * VS + VM]) continue;
    float3 q[9];
    unsigned hm = 0u;
#pragma unroll
    for (int u = 0; u < 9; ++u) {
      const int r = r0 + u;
      const int w = (r <= G && r < V) ? L.bwin[k * VS + r] : -1;
      hm |= (unsigned)(w >= 0) << u;
      q[u] = buffer_load_f3(rin, w >= 0 ? (uint32_t)(c0 + w) * 16u : 0xffffffffu);
    }
    unsigned long long g = 0ull;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int r = r0 + u;
      if (r < G && ((hm >> u) & 3u) == 3u) {  // (a pair with an empty cell is never ground)
        const float dX = q[u + 1].x - q[u].x, dY = q[u + 1].y - q[u].y, dZ = q[u + 1].z - q[u].z;
        if (ground_pair(dZ, dX * dX + dY * dY + dZ * dZ, P.mount, P.fp1)) g |= 3ull << r;
      }
    }
    if ((unsigned)g) atomicOr(&L.gbits[2 * k], (unsigned)g);
    if ((unsigned)(g >> 32)) atomicOr(&L.gbits[2 * k + 1], (unsigned)(g >> 32));
  }
  __syncthreads();
  // every cell of the touched band columns, row-major over the band (a row's consecutive columns in
  // consecutive lanes): range / cloud / ground, the 2-D scan candidate (:312-330) by a 64-bit LDS min of
  // (range, cell) — the sequential bottom-up scan with a strict `<` keeps the lowest row of equal ranges
  float* range = B.range + (size_t)s * P.VH;
  float4* cloud = B.cloud + (size_t)s * P.VH;
  int8_t* ground = B.ground + (size_t)s * P.VH;
  {
    constexpr int EM = (VM * NBC + PWS_NT - 1) / PWS_NT;  // cells a lane at most
    const int nc = V * bw;
    int wv[EM];
    float3 p3[EM];
#pragma unroll
    for (int t = 0; t < EM; ++t) {  // every gather in flight at once (one round trip)
      const int e = tid + t * PWS_NT;
      const int i = e / bw, k = e - i * bw;
      wv[t] = (e < nc && L.bwin[k * VS + VM]) ? L.bwin[k * VS + i] : -2;  // -2: not a cell of a touched column
      p3[t] = buffer_load_f3(rin, wv[t] >= 0 ? (uint32_t)(c0 + wv[t]) * 16u : 0xffffffffu);
    }
#pragma unroll
    for (int t = 0; t < EM; ++t) {
      if (wv[t] == -2) continue;
      const int e = tid + t * PWS_NT;
      const int i = e / bw, k = e - i * bw;
      const int j = colof(k), c = i * H + j;
      const bool h = wv[t] >= 0;
      const float4 pc = h ? make_float4(p3[t].x, p3[t].y, p3[t].z, (float)((double)(float)i + (double)(float)j / 10000.0))
                          : make_float4(qnan, qnan, qnan, 0.f);  // nanPoint: intensity 0
      const float r = h ? sqrtf(p3[t].x * p3[t].x + p3[t].y * p3[t].y + p3[t].z * p3[t].z) : FLT_MAX;
      const int g = (int)((L.gbits[2 * k + (i >> 5)] >> (i & 31)) & 1u);
      st_nt(&range[c], r);
      st_nt(&cloud[c], pc);
      ground[c] = (int8_t)g;
      if (g != 1 && (double)pc.z > 0.4 && (double)pc.z < 1.2 && r < 40.f)
        atomicMin(&L.scan[k], ((unsigned long long)__float_as_uint(r) << 32) | (unsigned)c);
    }
  }
  __syncthreads();
  // per touched column: the scan candidate, its touch, and (at the band's ends, the scan's first / last
  // slice) its winners to W
  for (int k = tid; k < bw; k += PWS_NT) {
    if (!L.bwin[k * VS + VM]) continue;
    const int j = colof(k);
    const unsigned long long sc = L.scan[k];
    B.scan_cand[(size_t)s * H + j] = sc == ~0ull ? -1 : (int)(unsigned)sc;
    const bool pub = k < PW_EDGE || k >= bw - PW_EDGE || c0 == 0 || c0 + PS >= n;
    atomicAdd(&colcnt[j], pub ? 0x1001 : 1);
    if (pub)
      for (int i = 0; i < V; ++i) {
        const int w = L.bwin[k * VS + i];
        if (w >= 0) atomicMax(&W[j * V + i], tag | (unsigned)(c0 + w));
      }
  }
}

// k_pw_fix: grid (column blocks, scans), NQ lanes a column: reads and clears each column's colcnt and
// settles the columns k_pw_slice left open: empty columns (no point) get their empty cells; contested
// columns are rebuilt from the winner image W (each winner's point gathered from the input, as
// k_pw_columns did for every column), or, where a band slice touched a column without publishing it,
// from the winners of a rescan of the whole scan's input into the block's columns (LDS).  Block (0, s)
// settles findStartEndAngle.
template <int NQ, int PC_NT, int CPL>
__global__ __launch_bounds__(PC_NT) void k_pw_fix(LgParams P, LgBufs B, const float4* __restrict__ pts,
                                                  const int64_t* __restrict__ offs, const int32_t* __restrict__ cnts) {
  constexpr int NC = PC_NT / NQ;  // columns a workgroup pass; CPL passes (every colcnt read up front)
  constexpr int VS = 16 * NQ + 1;
  __shared__ unsigned wl[NC * VS];
  const int s = P.s0 + blockIdx.y, tid = threadIdx.x;
  const int V = P.V, H = P.H;
  const int jj = tid / NQ, q = tid % NQ, i0 = 16 * q;
  int* colcnt = B.colcnt + (size_t)s * H;
  static_assert(CPL >= 1 && CPL <= 4, "up to four column passes a workgroup");
  unsigned v4[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int rep = 0; rep < CPL; ++rep) {
    const int j = (blockIdx.x * CPL + rep) * NC + jj;
    v4[rep] = (j < H && q == 0) ? (unsigned)colcnt[j] : 0u;
  }
#pragma unroll
  for (int rep = 0; rep < CPL; ++rep) {
    const int j = (blockIdx.x * CPL + rep) * NC + jj;
    if (j < H && q == 0) colcnt[j] = 0;
    if constexpr (NQ > 1) v4[rep] = (unsigned)__shfl((int)v4[rep], lane_id() & ~(NQ - 1));
  }
  const int n = cnts[s];
  const float4* in = pts + offs[s];
  const __amdgpu_buffer_rsrc_t rin = buffer_rsrc(in, (uint32_t)n * 16u);
  const float qnan = __int_as_float(0x7fc00000);
#pragma unroll 1
  for (int rep = 0; rep < CPL; ++rep) {
    const int jb = (blockIdx.x * CPL + rep) * NC, j = jb + jj;
    const bool col = j < H;  // (whole lane groups: NQ divides 64)
    const unsigned v = rep == 0 ? v4[0] : rep == 1 ? v4[1] : rep == 2 ? v4[2] : v4[3];
    const unsigned t = v & 0xfffu, pb = (v >> 12) & 0xfffu;
    const bool owned = (v >> 31) == 0u && t == 1u;  // one band slice, which wrote the column
    const bool need = v != 0u && !owned;             // contested: rebuilt here
    const bool incomplete = need && pb != t;         // a band slice touched it without publishing it
    if (col && q == 0) PWS_STAT(owned ? 2 : v == 0u ? 3 : incomplete ? 5 : 4, 1);
    const int any_inc = __syncthreads_or(incomplete);
    const int any_work = __syncthreads_or(col && !owned);
    if (!any_work) continue;  // (block-uniform)
    if (tid == 0 && any_inc) PWS_STAT(6, 1);
    if (any_inc) {  // rare: the block's winners from every point of the scan (exact cells)
      for (int e = tid; e < NC * VS; e += PC_NT) wl[e] = 0u;
      __syncthreads();
      for (int i = tid; i < n; i += PC_NT) {
        const float3 p3 = buffer_load_f3(rin, (uint32_t)i * 16u);
        if (!(isfinite_f(p3.x) && isfinite_f(p3.y) && isfinite_f(p3.z))) continue;
        const int c = proj_cell_exact_ni(P.ang_bottom, P.ang_res_x, P.ang_res_y, V, H, make_float4(p3.x, p3.y, p3.z, 0.f));
        if (c < 0) continue;
        const int r = c / H, jc = c - r * H;
        if (jc >= jb && jc < jb + NC) atomicMax(&wl[(jc - jb) * VS + r], P.wtag | (unsigned)i);
      }
      __syncthreads();
    }
    const unsigned* W = (const unsigned*)B.winner + (size_t)s * P.VH + (size_t)(col ? j : 0) * V;
    float3 pk[16];
    unsigned hm = 0u;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int i = i0 + u;
      unsigned w = 0u;
      if (need && i < V) w = any_inc ? wl[jj * VS + i] : W[i];
      const bool h = (w & 0xf0000000u) == P.wtag;
      hm |= (unsigned)h << u;
      pk[u] = buffer_load_f3(rin, h ? (w & 0x0fffffffu) * 16u : 0xffffffffu);
    }
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (!((hm >> u) & 1u)) pk[u] = make_float3(qnan, qnan, qnan);
    pw_column_emit<NQ>(P, B, s, j, q, col && !owned, pk, hm);
    if (any_inc) __syncthreads();  // wl is reused by the next pass
  }
  if (blockIdx.x == 0 && tid == 0) pw_orient(P, B, s, in);  // findStartEndAngle (:234-249)
}
#endif  // LG_PW_SLICE

#ifndef LG_PW_SLICE
// k_pw_columns: grid (column blocks of PW_NT, scans), one lane per column: the column pass of
// k_project over the scan's winner image in HBM (each cell read once; entries without this launch's
// tag are empty cells).  labelComponents' initial state is k_sw_local's.  Block (0, s) settles
// findStartEndAngle from proj_mm.
// NQ lanes a column (pw_column_emit).  PC_NT lanes a workgroup
// (256; 128 for V <= 16, so that one scan still spreads over many workgroups), PC_NT / NQ columns, the
// workgroup's columns of the column-major winner image staged in LDS with a
// (V + 1)-word column stride.  Many small workgroups keep more waves in flight than one lane a column
// walking all rows (each lane has one chunk of 16 gathers to wait for, not V / 16 in turn).
template <int NQ, int PC_NT>
__global__ __launch_bounds__(PC_NT) void k_pw_columns(LgParams P, LgBufs B, const float4* __restrict__ pts,
                                                      const int64_t* __restrict__ offs,
                                                      const int32_t* __restrict__ cnts) {
  constexpr int NC = PC_NT / NQ;  // columns a workgroup
  __shared__ int wl[NC * (16 * NQ + 1)];
  const int s = P.s0 + blockIdx.y, tid = threadIdx.x;
  const int V = P.V, H = P.H, VH = P.VH, VS = V + 1;
  {
    const int* wsrc = B.winner + (size_t)s * VH + (size_t)blockIdx.x * NC * V;
    const int nw = min(NC, H - (int)blockIdx.x * NC) * V;
    if ((V & 3) == 0) {  // 16-byte aligned, 4 words of one column at a time
      const int4* wg = (const int4*)wsrc;
      for (int q4 = tid; q4 < (nw >> 2); q4 += PC_NT) {
        const int4 v = wg[q4];
        const int e = 4 * q4, jj = e / V, i = e - jj * V;
        int* d = wl + jj * VS + i;
        d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
      }
    } else {
      for (int e = tid; e < nw; e += PC_NT) {
        const int jj = e / V;
        wl[jj * VS + e - jj * V] = wsrc[e];
      }
    }
  }
  __syncthreads();
  const int n = cnts[s];
  const float4* in = pts + offs[s];
  const float qnan = __int_as_float(0x7fc00000);
  const __amdgpu_buffer_rsrc_t rin = buffer_rsrc(in, (uint32_t)n * 16u);
  const int jj = tid / NQ, q = tid % NQ, i0 = 16 * q;
  const int j = blockIdx.x * NC + jj;
  const bool col = j < H;  // (whole lane groups: NQ divides 64)
  float3 pk[16];  // x, y, z of the cell's point; NaN for an empty cell (nanPoint)
  unsigned hm = 0u;  // bit u: row i0 + u has a point
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const unsigned v = (col && i0 + u < V) ? (unsigned)wl[jj * VS + i0 + u] : 0u;
    const bool h = (v & 0xf0000000u) == P.wtag;
    hm |= (unsigned)h << u;
    pk[u] = buffer_load_f3(rin, h ? (v & 0x0fffffffu) * 16u : 0xffffffffu);
  }
#pragma unroll
  for (int u = 0; u < 16; ++u)
    if (!((hm >> u) & 1u)) pk[u] = make_float3(qnan, qnan, qnan);
  pw_column_emit<NQ>(P, B, s, j, q, col, pk, hm);
  if (blockIdx.x == 0 && tid == 0) pw_orient(P, B, s, in);  // findStartEndAngle (:234-249)
}
#endif  // !LG_PW_SLICE

// ============================================================================================
// k_segment: labelComponents as connected components
// ============================================================================================
// BFS from every unlabelled cell in raster order (imageProjection.cpp:354-356, 412-496) labels the
// connected components of the symmetric edge relation "tang > tan(theta)" over 4-neighbour cells
// (vertical clamp, horizontal wrap) among cells with label 0 (not ground, valid range).  The BFS
// seed is the component's minimum raster index, feasible components are numbered 1,2,... in seed
// order, infeasible ones get 999999, and the line count excludes the seed's own row unless another
// member shares it (:469).  Reproduced with lock-free union-find (hook larger root onto smaller:
// the root is the component minimum = the seed), per-root size and non-seed row mask, and a
// raster-order block scan over feasible roots.
// labelComponents' edge test (imageProjection.cpp:457-465) between cells of ranges ra, rb; horiz:
// alpha = _ang_resolution_X (same row), else _ang_resolution_Y.  tang = d2 * sin(alpha) / (d1 - d2 *
// cos(alpha)) in float (fp_mode 0) or in double, rounded to the float tang (fp_mode 1).
LG_DEVICE bool seg_edge(const LgParams& P, float ra, float rb, bool horiz) {
  float d1 = (ra < rb) ? rb : ra;  // std::max(from, this)
  float d2 = (rb < ra) ? rb : ra;  // std::min(from, this)
  float tang;
  if (P.fp1) {
    const double sA = horiz ? P.sinXd : P.sinYd, cA = horiz ? P.cosXd : P.cosYd;
    tang = (float)((double)d2 * sA / ((double)d1 - (double)d2 * cA));
  } else {
    const float sA = horiz ? P.sinX : P.sinY, cA = horiz ? P.cosX : P.cosY;
    tang = (d2 * sA / (d1 - d2 * cA));
  }
  return tang > P.theta_thr;
}

template <typename PT>
LG_DEVICE int uf_find(PT parent, int x) {
  int p = parent[x];
  while (p != x) {
    x = p;
    p = parent[x];
  }
  return x;
}

template <typename PT>
LG_DEVICE void uf_unite(PT parent, int a, int b) {
  bool done;
  do {
    a = uf_find(parent, a);
    b = uf_find(parent, b);
    if (a < b) {
      int old = atomicMin(&parent[b], a);
      done = (old == b);
      b = old;
    } else if (b < a) {
      int old = atomicMin(&parent[a], b);
      done = (old == a);
      a = old;
    } else {
      done = true;
    }
  } while (!done);
}

// ECL-CC style (Jaiganesh & Burtscher): parent[v] <= v always; the find halves the path it walks
// (each store replaces a parent by one of its ancestors, so concurrent finds and hooks stay valid)
// and a root is hooked under the smaller root with a CAS, retried from the value found.
template <typename PT>
LG_DEVICE int uf_rep(PT parent, int x) {
  int curr = parent[x];
  if (curr != x) {
    int prev = x, next;
    while (curr > (next = parent[curr])) {
      parent[prev] = next;
      prev = curr;
      curr = next;
    }
  }
  return curr;
}

template <typename PT>
LG_DEVICE void uf_unite_rep(PT parent, int a, int b) {
  int ra = uf_rep(parent, a), rb = uf_rep(parent, b);
  while (ra != rb) {
    if (ra > rb) { const int t = ra; ra = rb; rb = t; }
    const int old = atomicCAS(&parent[rb], rb, ra);  // hook root rb under ra
    if (old == rb) break;
    rb = uf_rep(parent, old);
  }
}

// Raster-order compaction without block-wide scans: wave w owns the contiguous cells
// [w*L, w*L + L) (L a multiple of 64; one ring per wave for VLP-16), counts its two predicates with
// ballots, publishes the totals in wt[] (2 * waves ints of LDS), and after one barrier knows its
// exclusive offsets.  pred(c, p1, p2) is evaluated twice (count pass, then emit pass);
// emit(c, p1, p2, k1, k2) gets the raster-order output positions.  Returns the two totals.
template <typename Pred, typename Emit>
LG_DEVICE int2 wave_raster_compact(int n, int* wt, Pred pred, Emit emit) {
  const int lane = lane_id(), w = wave_id(), nw = (int)(blockDim.x >> 6);
  const int L = ((n + nw - 1) / nw + 63) & ~63;
  const int lo = min(w * L, n), hi = min(lo + L, n);
  int c1 = 0, c2 = 0;
  for (int base = lo; base < hi; base += 64) {
    const int c = base + lane;
    bool p1 = false, p2 = false;
    if (c < hi) pred(c, p1, p2);
    c1 += __popcll(__ballot(p1));
    c2 += __popcll(__ballot(p2));
  }
  if (lane == 0) { wt[w] = c1; wt[nw + w] = c2; }
  __syncthreads();
  int o1 = 0, o2 = 0, t1 = 0, t2 = 0;
  for (int k = 0; k < nw; ++k) {
    const int a = wt[k], b = wt[nw + k];
    if (k < w) { o1 += a; o2 += b; }
    t1 += a;
    t2 += b;
  }
  for (int base = lo; base < hi; base += 64) {
    const int c = base + lane;
    bool p1 = false, p2 = false;
    if (c < hi) pred(c, p1, p2);
    const unsigned long long m1 = __ballot(p1), m2 = __ballot(p2);
    if (c < hi) emit(c, p1, p2, o1 + popc_below(m1), o2 + popc_below(m2));
    o1 += __popcll(m1);
    o2 += __popcll(m2);
  }
  __syncthreads();  // wt[] reusable, emits visible block-wide
  return make_int2(t1, t2);
}

LG_DEVICE float ori_branch1(float ori, float so) {
  if ((double)ori < (double)so - M_PI / 2) ori = (float)((double)ori + 2 * M_PI);
  else if ((double)ori > (double)so + M_PI * 3 / 2) ori = (float)((double)ori - 2 * M_PI);
  return ori;
}
LG_DEVICE float ori_branch2(float ori, float eo) {
  ori = (float)((double)ori + 2 * M_PI);
  if ((double)ori < (double)eo - M_PI * 3 / 2) ori = (float)((double)ori + 2 * M_PI);
  else if ((double)ori > (double)eo + M_PI / 2) ori = (float)((double)ori - 2 * M_PI);
  return ori;
}

// adjustDistortion (featureAssociation.cpp:161-197) over the segmented cloud seg_pts[0, M) ->
// seg_fa.  halfPassed switches after the first point whose branch-1 orientation passes start + pi
// (index h).  Tiles of nt * FP_U points run in point order: while h is not yet known, a tile's raw
// orientations also give its first switching point (one block min); point i uses branch 1 iff
// i <= h, so a tile before h's tile is all branch 1 and one after it all branch 2.  Loads are
// unconditional (index clamped) and issued together.  Block-uniform; scratch >= 16 ints.
#define FP_U 8
// fp_mode 1's orientation, (float)(-atan2(double y, double x)): out of line (one copy) — inlined FP_U times, the
// double atan2 restatement set the register peak of k_sw_finish / k_segment_lds (38 / 18 VGPRs spilled) in
// either mode
__device__ __attribute__((noinline)) float neg_atan2_d(float y, float x) { return (float)(-atan2_d((double)y, (double)x)); }
LG_DEVICE void distort_segmented(const LgParams& P, const LgBufs& B, int s, int M, int* scratch) {
  const int tid = threadIdx.x, nt = blockDim.x;
  const float so = B.orient[s * 4 + 0], eo = B.orient[s * 4 + 1], od = B.orient[s * 4 + 2];
  const float4* __restrict__ seg = B.seg_pts + (size_t)s * P.VH;
  float4* __restrict__ fa = B.seg_fa + (size_t)s * P.VH;
  int h = 0x7fffffff;
  for (int t0 = 0; t0 < M; t0 += nt * FP_U) {
    float4 pk[FP_U];
    float ori[FP_U];
#pragma unroll
    for (int u = 0; u < FP_U; ++u) pk[u] = seg[min(t0 + u * nt + tid, M - 1)];
#pragma unroll
    for (int u = 0; u < FP_U; ++u)  // float ori = -atan2(point.x, point.z): point.x = y, point.z = x (:172)
      ori[u] = P.fp1 ? neg_atan2_d(pk[u].y, pk[u].x) : -atan2f_g(pk[u].y, pk[u].x);
    if (h == 0x7fffffff) {
      int hc = 0x7fffffff;
#pragma unroll
      for (int u = 0; u < FP_U; ++u) {
        const int i = t0 + u * nt + tid;
        if (i < M && (double)(ori_branch1(ori[u], so) - so) > M_PI) hc = min(hc, i);
      }
      h = block_min_int(hc, scratch);
    }
#pragma unroll
    for (int u = 0; u < FP_U; ++u) {
      const int i = t0 + u * nt + tid;
      const float4 p = pk[u];
      const float o = (i <= h) ? ori_branch1(ori[u], so) : ori_branch2(ori[u], eo);
      const float relTime = (o - so) / od;
      const float inten = (float)(int)p.w + P.scan_period * relTime;
      if (i < M) fa[i] = make_float4(p.y, p.z, p.x, inten);
    }
  }
}

// ---- k_segment (LDS path: V <= 16, V*H <= SEG_VH_MAX) ----------------------------------------
// One 16-bit LDS word per cell carries the whole labelling state (57.6 KB for VLP-16, so the kernel
// co-resides with k_lm's 66 KB on a CU):
//   cell index (< 0x7ffe)    eligible cell: union-find parent, after path compression its root
//   SEG_GND / SEG_EMPTY      ground cell / no return (label -1, :293-300)
//   SEG_FLAG | payload       a root: its member count (seed included); then, for 5 <= count < 30, the
//                            pending flag and the rows its non-seed members occupy relative to the
//                            seed's (bit d: d rows below, d = 0..SEG_DMAX, the last bit for any
//                            deeper); finally its label (k + 1 in seed raster order, or SEG_LBAD for
//                            999999)
// A component's rows form an interval that starts at its seed's row (edges join cells of one row or
// of adjacent rows, and the seed is its first cell in raster order), so lineCountFlag's count of
// distinct non-seed rows (:466-470) is bit 0 plus the deepest d present: exact while
// segment_valid_line_num <= SEG_DMAX (lg_lds_segment).  LDS atomics are 32-bit: a half-word's CAS / add / or operates on its word
// (the other half is never changed; counts stay below 0x8000, so an add never carries across).
// Global reads are batched (SEG_U cells per lane per round, all loads issued before use).
#define SEG_GND 0x7ffe
#define SEG_EMPTY 0x7fff
#define SEG_FLAG 0x8000
#define SEG_PEND 0x2000
#define SEG_FEAS 0x4000
#define SEG_LBAD 0x7fff   // label payload of an infeasible root (999999)
#define SEG_DMAX 12       // row bits 0..12 of a pending root (below SEG_PEND)
#define SEG_VH_MAX 32765  // cell indices stay below SEG_GND
#define SEG_U 8
#define SEG_ROUNDS 4  // 4 * 1024 * SEG_U = 32768 >= V*H on this path

LG_DEVICE bool seg_eligible(int8_t g, float r) { return g != 1 && r != FLT_MAX; }  // _label_mat == 0

// half-word LDS atomics through the containing 32-bit word
LG_DEVICE unsigned* h16_word(uint16_t* p, int i) { return (unsigned*)p + (i >> 1); }
LG_DEVICE int h16_shift(int i) { return (i & 1) << 4; }
LG_DEVICE int cas16(uint16_t* p, int i, int expected, int desired) {  // returns the value found
  unsigned* w = h16_word(p, i);
  const int sh = h16_shift(i);
  unsigned old = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  while (true) {
    const int cur = (int)((old >> sh) & 0xffffu);
    if (cur != expected) return cur;
    const unsigned nw = (old & ~(0xffffu << sh)) | ((unsigned)desired << sh);
    const unsigned got = atomicCAS(w, old, nw);
    if (got == old) return expected;
    old = got;
  }
}
LG_DEVICE void uf_unite_rep16(uint16_t* parent, int a, int b) {  // uf_unite_rep on half-words
  int ra = uf_rep(parent, a), rb = uf_rep(parent, b);
  while (ra != rb) {
    if (ra > rb) { const int t = ra; ra = rb; rb = t; }
    const int old = cas16(parent, rb, rb, ra);  // hook root rb under ra
    if (old == rb) break;
    rb = uf_rep(parent, old);
  }
}

// k_segment_lds's body (one 1,024-thread workgroup a scan; smem: 64 ints + V*H half-words)
LG_DEVICE void segment_lds(const LgParams& P, const LgBufs& B, int* smem) {
  const int s = P.s0 + blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  const int V = P.V, H = P.H, VH = P.VH, G = P.G;
  int* scratch = smem;  // 64 ints
  uint16_t* parent = (uint16_t*)(smem + 64);
  const float* __restrict__ range = B.range + (size_t)s * VH;
  const int8_t* __restrict__ ground = B.ground + (size_t)s * VH;
  const float4* __restrict__ cloud = B.cloud + (size_t)s * VH;
  int32_t* __restrict__ label = B.label + (size_t)s * VH;

  // ---- pass 1: the edges of every cell to its smaller-index neighbours: up (c - H), the horizontal
  // wrap ((i, 0) for j = H - 1) and left (c - 1).  parent starts at the smallest connected one
  // (ECL-CC's initialisation: short trees from the start); the other edges are united in pass 2.
  PROF_T(t_s0);
  unsigned ebits[SEG_ROUNDS];
#pragma unroll
  for (int rd = 0; rd < SEG_ROUNDS; ++rd) {
    ebits[rd] = 0u;
    const int cb = rd * nt * SEG_U;
    if (cb >= VH) continue;
    float r0[SEG_U], ru[SEG_U], rw[SEG_U], rl[SEG_U];
    int8_t g0[SEG_U], gu[SEG_U], gw[SEG_U], gl[SEG_U];
#pragma unroll
    for (int u = 0; u < SEG_U; ++u) {
      const int c = min(cb + u * nt + tid, VH - 1);
      const int i = c / H, j = c - i * H;
      const int cu = i > 0 ? c - H : c, cw = j == H - 1 ? i * H : c, cl = j > 0 ? c - 1 : c;
      r0[u] = range[c]; ru[u] = range[cu]; rw[u] = range[cw]; rl[u] = range[cl];
      g0[u] = ground[c]; gu[u] = ground[cu]; gw[u] = ground[cw]; gl[u] = ground[cl];
    }
#pragma unroll
    for (int u = 0; u < SEG_U; ++u) {
      const int c = cb + u * nt + tid;
      if (c >= VH) continue;
      const int i = c / H, j = c - i * H;
      const bool e0 = seg_eligible(g0[u], r0[u]);
      // the predicate is symmetric in its two ranges (d1 = max, d2 = min), as the BFS's is
      const bool eu = e0 && i > 0 && seg_eligible(gu[u], ru[u]) && seg_edge(P, r0[u], ru[u], false);
      const bool ew = e0 && j == H - 1 && H > 1 && seg_eligible(gw[u], rw[u]) &&
                      seg_edge(P, r0[u], rw[u], true);
      const bool el = e0 && j > 0 && seg_eligible(gl[u], rl[u]) && seg_edge(P, r0[u], rl[u], true);
      int p0 = c;
      unsigned rest = 0u;  // bit0 up, bit1 wrap, bit2 left: edges left for pass 2
      if (eu) p0 = c - H;
      if (ew) { if (p0 == c) p0 = i * H; else rest |= 2u; }
      if (el) { if (p0 == c) p0 = c - 1; else rest |= 4u; }
      parent[c] = (uint16_t)(e0 ? p0 : (g0[u] == 1 ? SEG_GND : SEG_EMPTY));
      ebits[rd] |= rest << (3 * u);
    }
  }
  __syncthreads();
  PROF_ADD(25, t_s0);
  // ---- pass 2: union the remaining edges (hook the larger root under the smaller: the root of a
  // component is its minimum cell, the BFS seed) --------------------------------------------------
  PROF_T(t_s1);
#pragma unroll
  for (int rd = 0; rd < SEG_ROUNDS; ++rd) {
    unsigned m = ebits[rd];
    while (m) {
      const int b = __ffs(m) - 1;
      m &= m - 1u;
      const int c = rd * nt * SEG_U + (b / 3) * nt + tid;
      const int i = c / H;
      const int k = b % 3;
      const int o = k == 0 ? c - H : (k == 1 ? i * H : c - 1);
      uf_unite_rep16(parent, c, o);
    }
  }
  __syncthreads();
  PROF_ADD(26, t_s1);
  // ---- pass 3: every eligible cell points at its root.  Only a cell's own word is written (a find
  // that halved other cells' paths here could overwrite a root already stored by their owner).
  PROF_T(t_s2);
  for (int c = tid; c < VH; c += nt) {
    const int p = parent[c];
    if (p < SEG_GND && p != c) parent[c] = (uint16_t)uf_find(parent, p);
  }
  __syncthreads();
  PROF_ADD(27, t_s2);
  // ---- pass 4: per-root size (seed included) and rows of the non-seed members (:466-470) ---------
  PROF_T(t_s3);
  for (int c = tid; c < VH; c += nt)
    if (parent[c] == c) parent[c] = (uint16_t)(SEG_FLAG | 1);
  __syncthreads();
  for (int c = tid; c < VH; c += nt) {
    const int r = parent[c];
    if (r < SEG_GND) atomicAdd(h16_word(parent, r), 1u << h16_shift(r));
  }
  __syncthreads();
  // count >= 30: feasible; < seg_valid_pt: not; otherwise the rows decide (pending)
  for (int c = tid; c < VH; c += nt) {
    const int a = parent[c];
    if (a & SEG_FLAG) {
      const int cnt = a & 0x7fff;
      parent[c] = (uint16_t)(SEG_FLAG | (cnt >= 30 ? SEG_FEAS : (cnt >= P.seg_valid_pt ? SEG_PEND : 0)));
    }
  }
  __syncthreads();
  for (int c = tid; c < VH; c += nt) {
    const int r = parent[c];
    if (r < SEG_GND && (parent[r] & SEG_PEND)) {
      const int d = c / H - r / H;  // >= 0: the seed is the component's first cell in raster order
      atomicOr(h16_word(parent, r), (1u << min(d, SEG_DMAX)) << h16_shift(r));
    }
  }
  __syncthreads();
  // feasible roots numbered in raster order of their seed (the BFS's _label_count++)
  wave_raster_compact(
      VH, scratch,
      [&](int c, bool& feas, bool& isroot) {
        const int a = parent[c];
        isroot = (a & SEG_FLAG) != 0;
        if (isroot) {
          // distinct non-seed rows: the seed's row (bit 0) + the rows below it up to the deepest
          const int lines = (a & 1) + (31 - __clz((a & ((2 << SEG_DMAX) - 2)) | 1));
          feas = (a & SEG_FEAS) || ((a & SEG_PEND) && lines >= P.seg_valid_line);
        }
      },
      [&](int c, bool feas, bool isroot, int k, int) {
        if (isroot) parent[c] = (uint16_t)(SEG_FLAG | (feas ? k + 1 : SEG_LBAD));
      });
  PROF_ADD(28, t_s3);
  // ---- pass 5: label image + cloudSegmentation's raster-order compaction (:358-396) -------------
  PROF_T(t_s4);
  float4* __restrict__ seg_pts = B.seg_pts + (size_t)s * VH;
  float* __restrict__ seg_range = B.seg_range + (size_t)s * VH;
  uint32_t* __restrict__ seg_col = B.seg_col + (size_t)s * VH;
  uint8_t* __restrict__ seg_ground = B.seg_ground + (size_t)s * VH;
  float4* __restrict__ outlier = B.outlier + (size_t)s * VH;
  float4* __restrict__ outlier_fa = B.outlier_fa + (size_t)s * VH;
  int32_t* __restrict__ ring_start = B.ring_start + (size_t)s * V;
  int32_t* __restrict__ ring_end = B.ring_end + (size_t)s * V;
  // adjustOutlierCloud (fa.cpp:1273-1283) runs in publishCloudsLast, i.e. not on the
  // initialisation scan (:1414-1416): the state read here is the one FeatureAssociation will see
  const bool swap_axes = B.fe_state[2 * s + 1] > 0;  // not the initialisation scan (:1414-1416)
  auto cell_label = [&](int c, int& lab, bool& gnd) {
    const int v = parent[c];
    gnd = v == SEG_GND;
    if (v == SEG_GND || v == SEG_EMPTY) {
      lab = -1;
    } else {
      const int l = ((v & SEG_FLAG) ? v : (int)parent[v]) & 0x7fff;
      lab = l == SEG_LBAD ? 999999 : l;
    }
  };
  auto classify = [&](int c, int lab, bool gnd, bool& pseg, bool& pout) {
    const int i = c / H, j = c - i * H;
    pseg = pout = false;
    if (lab > 0 || gnd) {
      if (lab == 999999) pout = (i > G && j % 5 == 0);
      else if (!(gnd && (j % 5 != 0 && j > 5 && j < H - 5))) pseg = true;
    }
  };
  const int lane = lane_id(), w = wave_id(), nw = (int)(nt >> 6);
  const int L = ((VH + nw - 1) / nw + 63) & ~63;
  const int lo = min(w * L, VH), hi = min(lo + L, VH);
  int c1 = 0, c2 = 0;
  for (int base = lo; base < hi; base += 64) {  // count pass (LDS only) + label image
    const int c = base + lane;
    bool p1 = false, p2 = false;
    if (c < hi) {
      int lab;
      bool gnd;
      cell_label(c, lab, gnd);
      label[c] = lab;
      classify(c, lab, gnd, p1, p2);
    }
    c1 += __popcll(__ballot(p1));
    c2 += __popcll(__ballot(p2));
  }
  if (lane == 0) { scratch[w] = c1; scratch[nw + w] = c2; }
  __syncthreads();
  int o1 = 0, o2 = 0, nseg = 0, nout = 0;
  for (int k = 0; k < nw; ++k) {
    const int a = scratch[k], b = scratch[nw + k];
    if (k < w) { o1 += a; o2 += b; }
    nseg += a;
    nout += b;
  }
  // emit pass: kCU chunks of 64 cells per batch; the cloud / range loads are buffer loads whose
  // offset is out of range for cells that are not emitted (they return 0 without a memory access)
  constexpr int kCU = 8;
  const __amdgpu_buffer_rsrc_t rs_cloud = buffer_rsrc(cloud, (uint32_t)VH * 16u);
  const __amdgpu_buffer_rsrc_t rs_range = buffer_rsrc(range, (uint32_t)VH * 4u);
  for (int base = lo; base < hi; base += 64 * kCU) {
    float4 pc[kCU];
    float rc[kCU];
    bool ps[kCU], po[kCU], pg[kCU];
#pragma unroll
    for (int u = 0; u < kCU; ++u) {
      const int c = base + 64 * u + lane;
      ps[u] = po[u] = pg[u] = false;
      if (c < hi) {
        int lab;
        cell_label(c, lab, pg[u]);
        classify(c, lab, pg[u], ps[u], po[u]);
      }
      pc[u] = buffer_load_f4(rs_cloud, (ps[u] || po[u]) ? (uint32_t)c * 16u : 0xffffffffu);
      rc[u] = buffer_load_f1(rs_range, ps[u] ? (uint32_t)c * 4u : 0xffffffffu);
    }
#pragma unroll
    for (int u = 0; u < kCU; ++u) {
      const int c = base + 64 * u + lane;
      const bool p1 = ps[u], p2 = po[u], gnd = pg[u];
      const unsigned long long m1 = __ballot(p1), m2 = __ballot(p2);
      if (c < hi) {
        const int i = c / H, j = c - i * H;
        const int k1 = o1 + popc_below(m1), k2 = o2 + popc_below(m2);
        if (j == 0) {  // k1 = segmented points before this ring
          ring_start[i] = k1 - 1 + 5;
          if (i > 0) ring_end[i - 1] = k1 - 1 - 5;
        }
        if (p1) {
          seg_pts[k1] = pc[u];
          seg_range[k1] = rc[u];
          seg_col[k1] = (uint32_t)j;
          seg_ground[k1] = (uint8_t)gnd;
        }
        if (p2) {
          const float4 p = pc[u];
          outlier[k2] = p;
          outlier_fa[k2] = swap_axes ? make_float4(p.y, p.z, p.x, p.w) : p;
        }
      }
      o1 += __popcll(m1);
      o2 += __popcll(m2);
    }
  }
  __syncthreads();
  if (tid == 0) ring_end[V - 1] = nseg - 1 - 5;
  // 2-D scan compaction (column order): each wave's columns read their candidate once and gather the
  // scan points with all loads in flight, then one barrier gives the waves' offsets
  const int32_t* cand = B.scan_cand + (size_t)s * H;
  float4* scan = B.scan_msg + (size_t)s * H;
  int nscan = 0;
  {
    constexpr int kJ = 4;  // 64 * kJ columns a round (one round a wave with 1,024 threads)
    const int Lc = ((H + nw - 1) / nw + 63) & ~63;
    const int jlo = min(w * Lc, H), jhi = min(jlo + Lc, H);
    int cnt_w = 0;
    for (int jb = jlo + 64 * kJ; jb < jhi; jb += 64) {  // columns past the first round: counted first
      const int j = jb + lane;
      cnt_w += __popcll(__ballot(j < jhi && cand[j] >= 0));
    }
    int cj[kJ];
#pragma unroll
    for (int u = 0; u < kJ; ++u) {
      const int j = jlo + 64 * u + lane;
      cj[u] = (j < jhi) ? cand[j] : -1;
    }
    float4 pc[kJ];
#pragma unroll
    for (int u = 0; u < kJ; ++u) {
      pc[u] = buffer_load_f4(rs_cloud, cj[u] >= 0 ? (uint32_t)cj[u] * 16u : 0xffffffffu);
      cnt_w += __popcll(__ballot(cj[u] >= 0));
    }
    if (lane == 0) scratch[w] = cnt_w;
    __syncthreads();
    int off = 0;
    for (int k = 0; k < nw; ++k) {
      const int a = scratch[k];
      if (k < w) off += a;
      nscan += a;
    }
    for (int jb = jlo; jb < jhi; jb += 64 * kJ) {
      if (jb > jlo) {  // later rounds (fewer than 16 waves)
#pragma unroll
        for (int u = 0; u < kJ; ++u) {
          const int j = jb + 64 * u + lane;
          cj[u] = (j < jhi) ? cand[j] : -1;
        }
#pragma unroll
        for (int u = 0; u < kJ; ++u) pc[u] = buffer_load_f4(rs_cloud, cj[u] >= 0 ? (uint32_t)cj[u] * 16u : 0xffffffffu);
      }
#pragma unroll
      for (int u = 0; u < kJ; ++u) {
        const unsigned long long m = __ballot(cj[u] >= 0);
        if (cj[u] >= 0) scan[off + popc_below(m)] = pc[u];
        off += __popcll(m);
      }
    }
    __syncthreads();  // scratch reusable
  }
  PROF_ADD(29, t_s4);
  PROF_T(t_s5);
  distort_segmented(P, B, s, nseg, scratch);
  PROF_ADD(31, t_s5);
  if (tid == 0) {
    int32_t* cnt = B.counts + (size_t)s * CNT_N;
    cnt[CNT_M] = nseg;
    cnt[CNT_OUTLIER] = nout;
    cnt[CNT_SCAN] = nscan;
  }
}

#ifndef LG_KP_ATTR
#define LG_KP_ATTR
#endif
__global__ __launch_bounds__(1024) LG_KP_ATTR void k_project(LgParams P, LgBufs B, const float4* __restrict__ pts,
                                                  const int64_t* __restrict__ offs,
                                                  const int32_t* __restrict__ cnts) {
  extern __shared__ __attribute__((aligned(16))) int smem[];
  project_lds(P, B, pts, offs, cnts, smem);
}
__global__ __launch_bounds__(1024) void k_segment_lds(LgParams P, LgBufs B) {
  extern __shared__ __attribute__((aligned(16))) int smem[];
  segment_lds(P, B, smem);
}
// ---- wide-mode segmentation: k_sw_* over tiles of SW_TILE cells, grid (tiles, scans) ----------
// labelComponents' result (imageProjection.cpp:412-496, :354-356) as in k_segment_lds: components
// of the edge relation by union-find (root = smallest member = the BFS seed), then each feasible
// root ranked in raster order.
//   k_sw_local   union of the edges inside 2-D tiles in LDS (parent := tile-local root)
//   k_sw_bound   union of the edges crossing tile borders (and the wrap), on the global parent[]
//   k_sw_roots   full path compression; size and non-seed row mask of every root
//   k_sw_count   per tile: feasible roots, segmented cells, outliers; each root's rank within its tile
//   k_sw_emit    label image (a root's label: 1 + its raster rank among the scan's feasible roots, or
//                999999) and the raster-order compaction (:358-396) at tile offsets
//   k_sw_finish  one workgroup a scan: 2-D scan compaction, adjustDistortion, counts
#define SW_NT 256
#define SW_TILE (SW_NT * 4)

LG_DEVICE int sw_load(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// uf_find / uf_unite on parent[] shared by the workgroups of a scan: reads through L2 (another
// CU's hook may be newer than this CU's L1), hooks by device-scope atomicMin.
LG_DEVICE int sw_find(int* parent, int x) {
  int p = sw_load(parent + x);
  while (p != x) {
    x = p;
    p = sw_load(parent + x);
  }
  return x;
}
LG_DEVICE void sw_unite(int* parent, int a, int b) {
  bool done;
  do {
    a = sw_find(parent, a);
    b = sw_find(parent, b);
    if (a < b) {
      const int old = atomicMin(&parent[b], a);
      done = (old == b);
      b = old;
    } else if (b < a) {
      const int old = atomicMin(&parent[a], b);
      done = (old == a);
      a = old;
    } else {
      done = true;
    }
  } while (!done);
}

// k_sw_local: 2-D tiles of SW_TR x SW_TC cells, grid (column tiles, row tiles, scans).  A cell takes
// part when _label_mat is 0 there (:293-300: not ground, has a return).  The edges inside a tile are
// united in LDS (local indices; the smallest local index is the smallest global one, rows dominating
// both orders); every cell's parent becomes its tile-local root (-1 for cells that take no part), and
// each tile-local root's component size / row mask start at 0 (every final root is a tile-local root).
#define SW_TR 8
#define SW_TC 128
__global__ __launch_bounds__(SW_NT) void k_sw_local(LgParams P, LgBufs B) {
  __shared__ int lp[SW_TR * SW_TC];
  __shared__ float lrg[SW_TR * SW_TC];
  const int s = P.s0 + blockIdx.z, V = P.V, H = P.H, VH = P.VH;
  const int i0 = blockIdx.y * SW_TR, j0 = blockIdx.x * SW_TC;
  int* parent = B.cc_parent + (size_t)s * VH;
  const float* range = B.range + (size_t)s * VH;
  const int8_t* ground = B.ground + (size_t)s * VH;
  bool ev[4];
  float rv[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int t = u * SW_NT + threadIdx.x, i = i0 + t / SW_TC, j = j0 + t % SW_TC;
    const int c = min(i, V - 1) * H + min(j, H - 1);
    const int g = ground[c];
    rv[u] = range[c];
    ev[u] = i < V && j < H && g != 1 && rv[u] != FLT_MAX;
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int t = u * SW_NT + threadIdx.x;
    lp[t] = ev[u] ? t : -1;
    lrg[t] = rv[u];
  }
  __syncthreads();
  const bool wrap_local = H <= SW_TC;  // one column tile: the horizontal wrap edge is inside it
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int t = u * SW_NT + threadIdx.x, lr = t / SW_TC, lc = t % SW_TC;
    const int i = i0 + lr, j = j0 + lc;
    if (lp[t] < 0) continue;
    const float r = lrg[t];
    int tr = -1;
    if (lc + 1 < SW_TC && j + 1 < H) tr = t + 1;
    else if (wrap_local && j == H - 1) tr = lr * SW_TC;  // (i, H-1) -> (i, 0)
    if (tr >= 0 && lp[tr] >= 0 && seg_edge(P, r, lrg[tr], true)) uf_unite(lp, t, tr);
    const int td = t + SW_TC;
    if (lr + 1 < SW_TR && i + 1 < V && lp[td] >= 0 && seg_edge(P, r, lrg[td], false))
      uf_unite(lp, t, td);
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int t = u * SW_NT + threadIdx.x, i = i0 + t / SW_TC, j = j0 + t % SW_TC;
    if (i < V && j < H) {
      const int c = i * H + j;
      const int rt = ev[u] ? uf_find(lp, t) : -1;
      parent[c] = rt >= 0 ? (i0 + rt / SW_TC) * H + j0 + rt % SW_TC : -1;
      if (rt == t) {  // only roots ever have their size / row mask read (k_sw_roots / k_sw_count)
        B.cc_cnt[(size_t)s * VH + c] = 0;
        B.cc_mask[(size_t)s * VH + c] = 0ull;
      }
    }
  }
}

// k_sw_bound: the edges that cross a tile's right edge (the horizontal wrap for the last column
// tile) or bottom edge, united on the scan's global parent[] (one thread an edge).
__global__ __launch_bounds__(SW_NT) void k_sw_bound(LgParams P, LgBufs B) {
  const int s = P.s0 + blockIdx.z, V = P.V, H = P.H, VH = P.VH;
  const int i0 = blockIdx.y * SW_TR, j0 = blockIdx.x * SW_TC;
  int* parent = B.cc_parent + (size_t)s * VH;
  const float* range = B.range + (size_t)s * VH;
  const int t = threadIdx.x;
  int c = -1, cn = -1;
  bool horiz = false;
  if (t < SW_TR) {  // right edge of row i0 + t
    const int i = i0 + t, j = min(j0 + SW_TC, H) - 1;
    if (i < V && !(H <= SW_TC)) {
      c = i * H + j;
      cn = (j + 1 < H) ? c + 1 : i * H;
      horiz = true;
    }
  } else if (t < SW_TR + SW_TC) {  // bottom edge of column j0 + t - SW_TR
    const int j = j0 + t - SW_TR, i = i0 + SW_TR - 1;
    if (j < H && i + 1 < V) {
      c = i * H + j;
      cn = c + H;
    }
  }
  if (c < 0) return;
  if (parent[c] < 0 || parent[cn] < 0) return;
  if (seg_edge(P, range[c], range[cn], horiz))
    sw_unite(parent, c, cn);
}

__global__ __launch_bounds__(SW_NT) void k_sw_roots(LgParams P, LgBufs B) {
  const int s = P.s0 + blockIdx.y, H = P.H, VH = P.VH;
  int* parent = B.cc_parent + (size_t)s * VH;
  int* ccnt = B.cc_cnt + (size_t)s * VH;
  unsigned long long* cmsk = B.cc_mask + (size_t)s * VH;
  const int lane = lane_id();
#pragma unroll 1
  for (int u = 0; u < 4; ++u) {
    const int c = blockIdx.x * SW_TILE + u * SW_NT + threadIdx.x;
    int r = -1;
    if (c < VH && parent[c] >= 0) {
      r = uf_find(parent, c);  // no hooks any more: plain (L1-cached) reads see valid ancestors
      parent[c] = r;
    }
    // one atomic per distinct root of the wave (neighbouring cells mostly share a component).  The
    // wave's 64 consecutive cells lie in at most two rows (H >= 64): the non-seed row mask of a root
    // is two ballots.
    unsigned long long todo = __ballot(r >= 0);
    const int rowA = __shfl(c, 0) / H;  // (c of lane 0 is the wave's first cell)
    const bool inA = c / H == rowA;
    while (todo) {
      const int r0 = __shfl(r, __ffsll((long long)todo) - 1);
      const unsigned long long m = __ballot(r == r0);
      unsigned long long rows;
      if (H >= 64) {
        const unsigned long long ns = __ballot(r == r0 && c != r0);
        const unsigned long long na = ns & __ballot(inA);
        rows = (na ? (1ull << rowA) : 0ull) | ((ns & ~na) ? (1ull << (rowA + 1)) : 0ull);
      } else {
        rows = (r == r0 && c != r0) ? (1ull << (c / H)) : 0ull;
        for (int o = 32; o > 0; o >>= 1) rows |= shfl64(rows, lane ^ o);
      }
      if (lane == __ffsll((long long)m) - 1) {
        atomicAdd(&ccnt[r0], __popcll(m));
        if (rows) atomicOr(&cmsk[r0], rows);
      }
      todo &= ~m;
    }
  }
}

LG_DEVICE bool sw_feasible(const LgParams& P, int n, unsigned long long rows) {  // :469-486
  return n >= 30 || (n >= P.seg_valid_pt && __popcll(rows) >= P.seg_valid_line);
}

// cloudSegmentation's classification of cell c (:358-396) from its label kind.
LG_DEVICE void sw_classify(const LgParams& P, int c, int lab, int g, bool& pseg, bool& pout) {
  const int i = c / P.H, j = c - i * P.H;
  pseg = pout = false;
  if (lab > 0 || g == 1) {
    if (lab == 999999) pout = (i > P.G && j % 5 == 0);
    else if (!(g == 1 && (j % 5 != 0 && j > 5 && j < P.H - 5))) pseg = true;
  }
}

// Also ranks the tile's feasible roots in raster order and leaves each root's rank in its label word,
// label[r] = -(2 + rank within the tile), 999999 for an infeasible root, so k_sw_emit labels every cell from
// its root's tile offset (no separate ranking launch).  Only a root's own tile writes its label word here;
// other tiles read the root's size / rows, which stay untouched.
#define SW_MAX_TILES ((64 * 2048) / SW_TILE)  // lego_params_validate: V <= 64, H <= 2048
__global__ __launch_bounds__(SW_NT) void k_sw_count(LgParams P, LgBufs B) {
  constexpr int NW = SW_NT / 64;
  __shared__ int red[3 * NW];
  __shared__ int wcnt[4 * NW];
  const int s = P.s0 + blockIdx.y, VH = P.VH;
  const int* parent = B.cc_parent + (size_t)s * VH;
  const int* ccnt = B.cc_cnt + (size_t)s * VH;
  const unsigned long long* cmsk = B.cc_mask + (size_t)s * VH;
  const int8_t* ground = B.ground + (size_t)s * VH;
  int32_t* label = B.label + (size_t)s * VH;
  int nroot = 0, nseg = 0, nout = 0;
  bool rt[4], rf[4];
  unsigned long long mf[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int c = blockIdx.x * SW_TILE + u * SW_NT + threadIdx.x;
    rt[u] = rf[u] = false;
    if (c < VH) {
      const int r = parent[c];
      int lab = -1;
      if (r >= 0) {
        const bool feas = sw_feasible(P, ccnt[r], cmsk[r]);
        lab = feas ? 1 : 999999;
        rt[u] = r == c;
        rf[u] = rt[u] && feas;
        nroot += rf[u] ? 1 : 0;
      }
      bool pseg, pout;
      sw_classify(P, c, lab, ground[c], pseg, pout);
      nseg += pseg;
      nout += pout;
    }
    mf[u] = __ballot(rf[u]);
  }
  {  // raster-order ranks of the feasible roots, local to the tile
    if (lane_id() == 0) {
#pragma unroll
      for (int u = 0; u < 4; ++u) wcnt[u * NW + wave_id()] = __popcll(mf[u]);
    }
    __syncthreads();
    int k = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      int before = 0, tot = 0;
      for (int w = 0; w < NW; ++w) {
        const int v = wcnt[u * NW + w];
        before += w < wave_id() ? v : 0;
        tot += v;
      }
      if (rt[u]) label[blockIdx.x * SW_TILE + u * SW_NT + threadIdx.x] = rf[u] ? -(2 + k + before + popc_below(mf[u])) : 999999;
      k += tot;
    }
  }
  nroot = wave_sum(nroot);
  nseg = wave_sum(nseg);
  nout = wave_sum(nout);
  if (lane_id() == 0) { red[wave_id()] = nroot; red[4 + wave_id()] = nseg; red[8 + wave_id()] = nout; }
  __syncthreads();
  if (threadIdx.x == 0) {
    int4 t = make_int4(0, 0, 0, 0);
    for (int w = 0; w < SW_NT / 64; ++w) { t.x += red[w]; t.y += red[4 + w]; t.z += red[8 + w]; }
    B.seg_tiles[(size_t)s * gridDim.x + blockIdx.x] = t;
  }
}

// Exclusive prefix of the tile counts before this tile (wave 0), in shared memory.
LG_DEVICE int4 sw_tile_base(const LgBufs& B, int s, int4* sh) {
  if (wave_id() == 0) {
    const int4* tc = B.seg_tiles + (size_t)s * gridDim.x;
    int4 a = make_int4(0, 0, 0, 0);
    for (int t = lane_id(); t < (int)blockIdx.x; t += 64) {
      const int4 v = tc[t];
      a.x += v.x; a.y += v.y; a.z += v.z;
    }
    a.x = wave_sum(a.x); a.y = wave_sum(a.y); a.z = wave_sum(a.z);
    if (lane_id() == 0) *sh = a;
  }
  __syncthreads();
  return *sh;
}


__global__ __launch_bounds__(SW_NT) void k_sw_emit(LgParams P, LgBufs B) {
  __shared__ int4 base;
  __shared__ int tpre[SW_MAX_TILES];  // exclusive prefix of the feasible roots over the scan's tiles
  const int s = P.s0 + blockIdx.y, V = P.V, H = P.H, VH = P.VH;
  const int* parent = B.cc_parent + (size_t)s * VH;
  const int8_t* ground = B.ground + (size_t)s * VH;
  const float* range = B.range + (size_t)s * VH;
  const float4* cloud = B.cloud + (size_t)s * VH;
  int32_t* label = B.label + (size_t)s * VH;
  float4* seg_pts = B.seg_pts + (size_t)s * VH;
  float* seg_range = B.seg_range + (size_t)s * VH;
  uint32_t* seg_col = B.seg_col + (size_t)s * VH;
  uint8_t* seg_ground = B.seg_ground + (size_t)s * VH;
  float4* outlier = B.outlier + (size_t)s * VH;
  float4* outlier_fa = B.outlier_fa + (size_t)s * VH;
  int32_t* ring_start = B.ring_start + (size_t)s * V;
  int32_t* ring_end = B.ring_end + (size_t)s * V;
  const bool swap_axes = B.fe_state[2 * s + 1] > 0;  // not the initialisation scan (:1414-1416)
  {  // the scan's tile offsets of the feasible roots (wave 0: a lane per (tiles / 64) tiles, then a wave scan)
    if (wave_id() == 0) {
      const int4* tc = B.seg_tiles + (size_t)s * gridDim.x;
      const int nt = (int)gridDim.x, per = (nt + 63) / 64, t0 = lane_id() * per;
      int own = 0;
      for (int t = t0; t < min(t0 + per, nt); ++t) own += tc[t].x;
      int incl = own;  // inclusive wave scan of the lanes' sums
      for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o);
        if (lane_id() >= o) incl += v;
      }
      int a = incl - own;
      for (int t = t0; t < min(t0 + per, nt); ++t) {
        tpre[t] = a;
        a += tc[t].x;
      }
    }
  }
  const int4 b0 = sw_tile_base(B, s, &base);  // (its barrier also publishes tpre)
  // The tile's 4 x SW_NT cells: every load of the four rounds in flight together, then one barrier
  // for the raster-order offsets of both compactions (wave counts of each round in LDS).
  __shared__ int wcnt[2 * 4 * (SW_NT / 64)];
  int c[4], r[4], g[4], lab[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    c[u] = blockIdx.x * SW_TILE + u * SW_NT + threadIdx.x;
    r[u] = c[u] < VH ? parent[c[u]] : -1;
    g[u] = c[u] < VH ? ground[c[u]] : 0;
  }
  {
    // the root's label word: -(2 + rank in its tile) from k_sw_count, or already the final label (its own tile's
    // k_sw_emit may have stored it), or 999999; the first decodes to 1 + the root's raster rank in the scan
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (r[u] < 0) {
        lab[u] = -1;
      } else {
        const int v = label[r[u]];
        lab[u] = v <= -2 ? tpre[r[u] / SW_TILE] + (-v - 2) + 1 : v;
      }
    }
  }
  bool pseg[4], pout[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    pseg[u] = pout[u] = false;
    if (c[u] < VH) {
      label[c[u]] = lab[u];
      sw_classify(P, c[u], lab[u], g[u], pseg[u], pout[u]);
    }
  }
  unsigned long long ms[4], mo[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    ms[u] = __ballot(pseg[u]);
    mo[u] = __ballot(pout[u]);
  }
  constexpr int NW = SW_NT / 64;
  if (lane_id() == 0) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      wcnt[u * NW + wave_id()] = __popcll(ms[u]);
      wcnt[4 * NW + u * NW + wave_id()] = __popcll(mo[u]);
    }
  }
  __syncthreads();
  int kseg = b0.y, kout = b0.z;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    int bs = 0, ts = 0, bo = 0, to = 0;
    for (int w = 0; w < NW; ++w) {
      const int vs = wcnt[u * NW + w], vo = wcnt[4 * NW + u * NW + w];
      bs += w < wave_id() ? vs : 0;
      bo += w < wave_id() ? vo : 0;
      ts += vs;
      to += vo;
    }
    const int oseg = kseg + bs + popc_below(ms[u]), oout = kout + bo + popc_below(mo[u]);
    if (c[u] < VH) {
      const int i = c[u] / H, j = c[u] - i * H;
      if (j == 0) {  // oseg = segmented points before this ring
        ring_start[i] = oseg - 1 + 5;
        if (i > 0) ring_end[i - 1] = oseg - 1 - 5;
      }
      if (pseg[u] || pout[u]) {
        const float4 p = cloud[c[u]];
        if (pseg[u]) {
          seg_pts[oseg] = p;
          seg_range[oseg] = range[c[u]];
          seg_col[oseg] = (uint32_t)j;
          seg_ground[oseg] = (uint8_t)(g[u] == 1);
        }
        if (pout[u]) {
          outlier[oout] = p;
          outlier_fa[oout] = swap_axes ? make_float4(p.y, p.z, p.x, p.w) : p;  // adjustOutlierCloud (fa.cpp:1273-1283)
        }
      }
    }
    kseg += ts;
    kout += to;
  }
}

// kNT threads a scan: 1,024 fills a CU's register file (128 VGPRs x 16 waves), 256 (four waves at <= 128 VGPRs)
// shares a CU with k_lm's and k_voxel's waves.
template <int kNT>
__global__ __launch_bounds__(kNT) __attribute__((amdgpu_waves_per_eu(4))) void k_sw_finish(LgParams P, LgBufs B, int tiles) {
  __shared__ int scratch[64];
  const int s = P.s0 + blockIdx.x, tid = threadIdx.x, V = P.V, H = P.H, VH = P.VH;
  __shared__ int tot[2];
  if (tid < 64) {
    const int4* tc = B.seg_tiles + (size_t)s * tiles;
    int a = 0, b = 0;
    for (int t = tid; t < tiles; t += 64) { a += tc[t].y; b += tc[t].z; }
    a = wave_sum(a);
    b = wave_sum(b);
    if (tid == 0) { tot[0] = a; tot[1] = b; }
  }
  __syncthreads();
  const int nseg = tot[0], nout = tot[1];
  if (tid == 0) B.ring_end[(size_t)s * V + V - 1] = nseg - 1 - 5;
  const int32_t* cand = B.scan_cand + (size_t)s * H;
  const float4* cloud = B.cloud + (size_t)s * VH;
  float4* scan = B.scan_msg + (size_t)s * H;
  const int nscan = wave_raster_compact(H, scratch, [&](int j, bool& p, bool&) { p = cand[j] >= 0; },
                                        [&](int j, bool p, bool, int k, int) { if (p) scan[k] = cloud[cand[j]]; }).x;
  distort_segmented(P, B, s, nseg, scratch);
  if (tid == 0) {
    int32_t* cnt = B.counts + (size_t)s * CNT_N;
    cnt[CNT_M] = nseg;
    cnt[CNT_OUTLIER] = nout;
    cnt[CNT_SCAN] = nscan;
  }
}

// ============================================================================================
// k_fa_prep: adjustDistortion + calculateSmoothness + markOccludedPoints + adjustOutlierCloud
// ============================================================================================
// calculateSmoothness + markOccludedPoints on LDS tiles of FP_TILE positions (+ halo) whose range /
// column loads are issued together.  markOccludedPoints'
// scattered OR-writes (:237-259) are evaluated in gather form, picked[k] = OR of the marks that land
// on k, which equals the reference's "zero [5, M-5) then OR the marks" for every k (positions
// outside [5, M-5) keep their stale value OR the marks, as there).  adjustDistortion and
// adjustOutlierCloud run in k_segment's epilogue, on the cloud it has just compacted; kDistort
// runs them here instead, for a ProjectionOut uploaded from the host (lego_feature_association_from).
// kNT threads a workgroup, FP_TILE = kNT * FP_U positions a tile.  The device-resident path runs
// k_fa_prep4 below (one tile per workgroup, four positions a lane); this template serves kDistort
// (whole-scan block minimum, looping over the tiles of its scan in one workgroup).
#define FP_HALO 8
template <bool kDistort, int kNT>
__global__ __launch_bounds__(kNT) void k_fa_prep(LgParams P, LgBufs B) {
  constexpr int FP_TILE = kNT * FP_U;
  __shared__ int scratch[64];
  __shared__ float sr[FP_TILE + 2 * FP_HALO];     // segmentedCloudRange[t0 - FP_HALO + x]
  __shared__ uint32_t sc[FP_TILE + 2 * FP_HALO];  // segmentedCloudColInd
  __shared__ uint8_t sf[FP_TILE + 2 * FP_HALO];   // marks of i: bit0 A (i-5..i), bit1 B (i+1..i+6), bit2 C (i)
  const int s = P.s0 + blockIdx.x, tid = threadIdx.x, nt = kNT;
  const int VH = P.VH;
  const int32_t* cnt = B.counts + (size_t)s * CNT_N;
  const int M = cnt[CNT_M];
  const float* __restrict__ r = B.seg_range + (size_t)s * VH;
  const uint32_t* __restrict__ col = B.seg_col + (size_t)s * VH;
  float* __restrict__ curv = B.curv + (size_t)s * VH;
  uint8_t* __restrict__ picked = B.picked + (size_t)s * VH;
  int8_t* __restrict__ flabel = B.flabel + (size_t)s * VH;
  int2* __restrict__ smooth = B.smooth + (size_t)s * VH;
  // k_extract's first pass may move the stale slot 4 while other rings check where it points
  if (tid == 0 && blockIdx.y == 0) B.fp_sync[2 * s] = smooth[4].y;
  if constexpr (kDistort) {
    distort_segmented(P, B, s, M, scratch);
    const int nout = cnt[CNT_OUTLIER];
    const float4* __restrict__ outl = B.outlier + (size_t)s * VH;
    float4* __restrict__ outa = B.outlier_fa + (size_t)s * VH;
    const bool swap_axes = B.fe_state[2 * s + 1] > 0;  // not the initialisation scan (:1414-1416)  // not on the initialisation scan (:1414-1416)
    for (int k = tid; k < nout; k += nt) {
      const float4 p = outl[k];
      outa[k] = swap_axes ? make_float4(p.y, p.z, p.x, p.w) : p;
    }
  }
  const int nTiles = (M + FP_TILE - 1) / FP_TILE;
  const int tile_lo = kDistort ? 0 : (int)blockIdx.y, tile_hi = kDistort ? nTiles : min((int)blockIdx.y + 1, nTiles);
  for (int tile = tile_lo; tile < tile_hi; ++tile) {
    const int t0 = tile * FP_TILE;
    PROF_T(t_f1);
    {  // range / column of positions [t0 - FP_HALO, t0 + FP_TILE + FP_HALO) into LDS, one batch
      float rv[FP_U];
      uint32_t cv[FP_U];
#pragma unroll
      for (int u = 0; u < FP_U; ++u) {
        const int q = min(t0 + u * nt + tid, M - 1);
        rv[u] = r[q];
        cv[u] = col[q];
      }
      float rh = 0.f;
      uint32_t ch = 0u;
      const int xh = tid < FP_HALO ? tid : FP_TILE + tid;  // halo slot of this lane (tid < 2 * FP_HALO)
      if (tid < 2 * FP_HALO) {
        const int q = min(max(t0 - FP_HALO + xh, 0), M - 1);
        rh = r[q];
        ch = col[q];
      }
#pragma unroll
      for (int u = 0; u < FP_U; ++u) {
        sr[FP_HALO + u * nt + tid] = rv[u];
        sc[FP_HALO + u * nt + tid] = cv[u];
      }
      if (tid < 2 * FP_HALO) { sr[xh] = rh; sc[xh] = ch; }
    }
    __syncthreads();
    PROF_ADD(33, t_f1);
    PROF_T(t_f2);
    // markOccludedPoints' per-i conditions for i in [t0 - 6, t0 + FP_TILE + 6), i in [5, M - 6)
    for (int x = 2 + tid; x < FP_TILE + 2 * FP_HALO - 2; x += nt) {
      const int i = t0 - FP_HALO + x;
      uint8_t f = 0;
      if (i >= 5 && i < M - 6) {
        const float depth1 = sr[x], depth2 = sr[x + 1];
        const int columnDiff = abs((int)(sc[x + 1] - sc[x]));
        if (columnDiff < 10) {
          if ((double)(depth1 - depth2) > 0.3) f |= 1;
          else if ((double)(depth2 - depth1) > 0.3) f |= 2;
        }
        const float diff1 = fabsf(sr[x - 1] - depth1), diff2 = fabsf(sr[x + 1] - depth1);
        if ((double)diff1 > 0.02 * (double)depth1 && (double)diff2 > 0.02 * (double)depth1) f |= 4;
      }
      sf[x] = f;
    }
    __syncthreads();
    PROF_ADD(34, t_f2);
    PROF_T(t_f3);
    // calculateSmoothness (:200-223) + the marks landing on each k
    for (int x = FP_HALO + tid; x < FP_HALO + FP_TILE; x += nt) {
      const int k = t0 - FP_HALO + x;
      if (k > M) break;
      bool mk = (sf[x] & 4) != 0;
#pragma unroll
      for (int d = 0; d <= 5; ++d) mk |= (sf[x + d] & 1) != 0;   // A(k + d) marks k
#pragma unroll
      for (int d = 1; d <= 6; ++d) mk |= (sf[x - d] & 2) != 0;   // B(k - d) marks k
      if (k >= 5 && k < M - 5) {
        const float d = sr[x - 5] + sr[x - 4] + sr[x - 3] + sr[x - 2] + sr[x - 1] - sr[x] * 10 + sr[x + 1] + sr[x + 2] +
                        sr[x + 3] + sr[x + 4] + sr[x + 5];
        const float cv = d * d;
        curv[k] = cv;
        picked[k] = mk ? 1 : 0;
        flabel[k] = 0;
        smooth[k] = make_int2(__float_as_int(cv), k);
      } else if (mk) {
        picked[k] = 1;
      }
    }
    __syncthreads();
    PROF_ADD(35, t_f3);
  }
}

// The device-resident k_fa_prep with four consecutive positions a lane: 16-byte loads of range /
// column into LDS, the occlusion marks of four positions from one window, the smoothness of four
// positions from five 16-byte LDS reads, and 16-byte (curvature, sort keys) / 4-byte (picked, label)
// stores where all four positions lie in [5, M - 5).  Same arithmetic, same order as k_fa_prep.
// Positions at or beyond M load as 0 (buffer range): no output reads them (marks need i < M - 6,
// the smoothness k + 5 < M).
#define FP4_NT 256
#ifndef FP4_G
#define FP4_G 2  // groups of four positions a lane
#endif
#define FP4_TILE (FP4_NT * 4 * FP4_G)
__global__ __launch_bounds__(FP4_NT) void k_fa_prep4(LgParams P, LgBufs B) {
  __shared__ __attribute__((aligned(16))) float sr[FP4_TILE + 2 * FP_HALO];
  __shared__ __attribute__((aligned(16))) uint32_t sc[FP4_TILE + 2 * FP_HALO];
  __shared__ __attribute__((aligned(16))) uint8_t sf[FP4_TILE + 2 * FP_HALO];
  const int s = P.s0 + blockIdx.x, tid = threadIdx.x;
  const int VH = P.VH;
  const int32_t* cnt = B.counts + (size_t)s * CNT_N;
  const int M = cnt[CNT_M];
  const float* __restrict__ r = B.seg_range + (size_t)s * VH;
  const uint32_t* __restrict__ col = B.seg_col + (size_t)s * VH;
  float* __restrict__ curv = B.curv + (size_t)s * VH;
  uint8_t* __restrict__ picked = B.picked + (size_t)s * VH;
  int8_t* __restrict__ flabel = B.flabel + (size_t)s * VH;
  int2* __restrict__ smooth = B.smooth + (size_t)s * VH;
  // k_extract's first pass may move the stale slot 4 while other rings check where it points
  if (tid == 0 && blockIdx.y == 0) B.fp_sync[2 * s] = smooth[4].y;
  const int t0 = blockIdx.y * FP4_TILE;
  if (t0 >= M) return;
  {  // range / column of [t0 - FP_HALO, t0 + FP4_TILE + FP_HALO) into LDS
    const __amdgpu_buffer_rsrc_t rr = buffer_rsrc(r, (uint32_t)M * 4u), rc = buffer_rsrc(col, (uint32_t)M * 4u);
    float4 rv[FP4_G];
    float4 cv[FP4_G];
#pragma unroll
    for (int g = 0; g < FP4_G; ++g) {
      const uint32_t off = (uint32_t)(t0 + 4 * (tid + g * FP4_NT)) * 4u;
      rv[g] = buffer_load_f4(rr, off);
      cv[g] = buffer_load_f4(rc, off);
    }
    float rh = 0.f;
    uint32_t ch = 0u;
    const int xh = tid < FP_HALO ? tid : FP4_TILE + tid;  // halo slot of this lane (tid < 2 * FP_HALO)
    if (tid < 2 * FP_HALO) {
      const int q = min(max(t0 - FP_HALO + xh, 0), M - 1);
      rh = r[q];
      ch = col[q];
    }
#pragma unroll
    for (int g = 0; g < FP4_G; ++g) {
      const int x = FP_HALO + 4 * (tid + g * FP4_NT);
      *(float4*)&sr[x] = rv[g];
      *(float4*)&sc[x] = cv[g];
    }
    if (tid < 2 * FP_HALO) { sr[xh] = rh; sc[xh] = ch; }
  }
  __syncthreads();
  // markOccludedPoints' per-i conditions (as k_fa_prep) for i in [t0 - 6, t0 + FP4_TILE + 6)
  auto mark = [&](int x) -> uint32_t {
    const int i = t0 - FP_HALO + x;
    uint32_t f = 0;
    if (i >= 5 && i < M - 6) {
      const float depth1 = sr[x], depth2 = sr[x + 1];
      const int columnDiff = abs((int)(sc[x + 1] - sc[x]));
      if (columnDiff < 10) {
        if ((double)(depth1 - depth2) > 0.3) f |= 1;
        else if ((double)(depth2 - depth1) > 0.3) f |= 2;
      }
      const float diff1 = fabsf(sr[x - 1] - depth1), diff2 = fabsf(sr[x + 1] - depth1);
      if ((double)diff1 > 0.02 * (double)depth1 && (double)diff2 > 0.02 * (double)depth1) f |= 4;
    }
    return f;
  };
#pragma unroll
  for (int g = 0; g < FP4_G; ++g) {
    const int x = FP_HALO + 4 * (tid + g * FP4_NT);
    const uint32_t w = mark(x) | (mark(x + 1) << 8) | (mark(x + 2) << 16) | (mark(x + 3) << 24);
    *(uint32_t*)&sf[x] = w;
  }
  if (tid < 12) {  // the halo marks: x in [2, FP_HALO) and [FP_HALO + FP4_TILE, FP_HALO + FP4_TILE + 6)
    const int x = tid < 6 ? 2 + tid : FP_HALO + FP4_TILE + (tid - 6);
    sf[x] = (uint8_t)mark(x);
  }
  __syncthreads();
  // calculateSmoothness (:200-223) + the marks landing on each k, four positions a lane
#pragma unroll
  for (int g = 0; g < FP4_G; ++g) {
    const int x = FP_HALO + 4 * (tid + g * FP4_NT);
    const int k0 = t0 + 4 * (tid + g * FP4_NT);
    if (k0 > M) break;
    float w[20];  // sr[x - 8, x + 12)
    uint8_t m[20];  // sf[x - 8, x + 12)
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      const float4 v = *(const float4*)&sr[x - 8 + 4 * q];
      w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
      const uint32_t f = *(const uint32_t*)&sf[x - 8 + 4 * q];
      m[4 * q] = f & 255; m[4 * q + 1] = (f >> 8) & 255; m[4 * q + 2] = (f >> 16) & 255; m[4 * q + 3] = f >> 24;
    }
    float cvs[4];
    bool mks[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = 8 + e;  // w[c] = sr[x + e]
      bool mk = (m[c] & 4) != 0;
#pragma unroll
      for (int d = 0; d <= 5; ++d) mk |= (m[c + d] & 1) != 0;   // A(k + d) marks k
#pragma unroll
      for (int d = 1; d <= 6; ++d) mk |= (m[c - d] & 2) != 0;   // B(k - d) marks k
      mks[e] = mk;
      const float dd = w[c - 5] + w[c - 4] + w[c - 3] + w[c - 2] + w[c - 1] - w[c] * 10 + w[c + 1] + w[c + 2] +
                       w[c + 3] + w[c + 4] + w[c + 5];
      cvs[e] = dd * dd;
    }
    if (k0 >= 5 && k0 + 3 < M - 5) {  // all four interior: vector stores
      *(float4*)&curv[k0] = make_float4(cvs[0], cvs[1], cvs[2], cvs[3]);
      *(uint32_t*)&picked[k0] = (uint32_t)mks[0] | ((uint32_t)mks[1] << 8) | ((uint32_t)mks[2] << 16) |
                                ((uint32_t)mks[3] << 24);
      *(uint32_t*)&flabel[k0] = 0u;
      *(int4*)&smooth[k0] = make_int4(__float_as_int(cvs[0]), k0, __float_as_int(cvs[1]), k0 + 1);
      *(int4*)&smooth[k0 + 2] = make_int4(__float_as_int(cvs[2]), k0 + 2, __float_as_int(cvs[3]), k0 + 3);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = k0 + e;
        if (k > M) break;
        if (k >= 5 && k < M - 5) {
          curv[k] = cvs[e];
          picked[k] = mks[e] ? 1 : 0;
          flabel[k] = 0;
          smooth[k] = make_int2(__float_as_int(cvs[e]), k);
        } else if (mks[e]) {
          picked[k] = 1;
        }
      }
    }
  }
}

// ============================================================================================
// k_extract: extractFeatures, one wave per ring
// ============================================================================================
#define SEG_MAX 512
#define RING_MAX 2048

// LDS of one wave.  Measured on MI355X (tools/lds_probe.py): 11 one-wave workgroups share a CU at
// 13,824 B each, not at 14,336; 12 not at 13,312 B.
struct ExtractLds {  // k_voxel: 12.1 KB per wave (LDS allows 12 a CU)
  unsigned pad[16];             // final_window reads (and ignores) up to 15 words below vkey[0]
  union {
    unsigned vkey[RING_MAX];    // voxel keys
  } u;
  uint16_t vval[RING_MAX];      // lessFlat positions of the ring (relative to the ring start), sorted with vkey
                                // (also read, and ignored, by final_window past vkey[n - 1])
};

struct SortTestLds {  // the sort test hooks (lego_test_sort): every path of wave_std_sort
  unsigned pad[16];
  union {
    struct { float skey[SEG_MAX]; int sval[SEG_MAX]; } seg;  // segment sort
    unsigned vkey[RING_MAX];
  } u;
  uint16_t vval[RING_MAX];
  unsigned blk[RING_MAX / 32];  // final-block start bits (the per-block insertion sorts)
};

struct SegLds {  // k_sortseg: 5.4 KB per wave
  union {
    struct { float skey[SEG_MAX]; int sval[SEG_MAX]; } seg;  // segment sort
    uint16_t col[SEG_MAX + 16];                             // colInd around the segment (info words)
  } u;
  unsigned blk[RING_MAX / 32];
};

template <typename T>
LG_DEVICE T perm_push(int dst_lane, T v) {  // ds_permute_b32: v to lane dst_lane (a permutation)
  return __builtin_bit_cast(T, __builtin_amdgcn_ds_permute(dst_lane << 2, __builtin_bit_cast(int, v)));
}
template <typename T>
LG_DEVICE T shfl_any(T v, int src) {
  return __builtin_bit_cast(T, __shfl(__builtin_bit_cast(int, v), src));
}
// __unguarded_partition_pivot on a range of 17..64 elements held one per lane; returns the cut.
template <typename K, typename V>
LG_DEVICE int wave_partition_small(const SortView<K, V>& a, int first, int last) {
  const int lane = lane_id();
  const int m = last - first;
  const bool in = lane < m;
  K k = in ? a.key[first + lane] : K(0);
  int v = in ? (int)a.val[first + lane] : 0;
  // __move_median_to_first(first, first+1, mid, last-1)
  const int im = m / 2, il = m - 1;
  const K kx = rdlane(k, 1), ky = rdlane(k, im), kz = rdlane(k, il);  // (uniform lanes: no LDS crossbar)
  int sel;
  if (kx < ky) {
    if (ky < kz) sel = im;
    else if (kx < kz) sel = il;
    else sel = 1;
  } else if (kx < kz) sel = 1;
  else if (ky < kz) sel = il;
  else sel = im;
  {
    const K k0 = rdlane(k, 0), ks = rdlane(k, sel);
    const int v0 = __builtin_amdgcn_readlane(v, 0), vs = __builtin_amdgcn_readlane(v, sel);
    if (lane == 0) { k = ks; v = vs; }
    else if (lane == sel) { k = k0; v = v0; }
  }
  const K pv = rdlane(k, 0);
  const bool lf = in && lane >= 1 && !(k < pv);
  const bool rf = in && lane >= 1 && !(pv < k);
  const unsigned long long bl = __ballot(lf), br = __ballot(rf);
  const int nL = __popcll(bl), nR = __popcll(br);
  const int lrank = popc_below(bl);                                   // k-th left stop, from first+1 up
  const int rrank = __popcll(br & ~((2ull << lane) - 1ull));          // k-th right stop, from last-1 down
  // lane k of Ls / Rs: the k-th left / right stop (forward permutes: the stops to their ranks, the
  // other lanes behind them)
  const int Ls = perm_push(lf ? lrank : nL + (lane - lrank), lane);
  const int nrb = __popcll(br & ((1ull << lane) - 1ull));             // right stops below this lane
  const int Rs = perm_push(rf ? rrank : nR + (lane - nrb), lane);
  int partner = -1;
  bool left_swap = false;  // a pivot-equal lane is both kinds of stop: count only its left role
  const int qr = __shfl(Rs, lf ? min(lrank, 63) : 0), ql = __shfl(Ls, rf ? min(rrank, 63) : 0);
  if (lf && lrank < nR) {
    if (lane < qr) { partner = qr; left_swap = true; }
  }
  if (rf && rrank < nL) {
    if (ql < lane) partner = ql;
  }
  const K kp = __shfl(k, partner < 0 ? lane : partner);
  const int vp = __shfl(v, partner < 0 ? lane : partner);
  const unsigned long long sw = __ballot(left_swap);
  const int nsw = __popcll(sw);
  if (partner >= 0) { k = kp; v = vp; }
  // cut = min(L[nsw], R[nsw-1]) (R[-1] = last)
  const unsigned long long lk = __ballot(lf && lrank == nsw);
  const unsigned long long rk = __ballot(rf && rrank == nsw - 1);
  const int cl = lk ? __ffsll((long long)lk) - 1 : m;
  const int cr = (nsw > 0 && rk) ? __ffsll((long long)rk) - 1 : m;
  if (in) { a.key[first + lane] = k; a.val[first + lane] = (V)v; }
  __syncthreads();
  return first + min(cl, cr);
}

// __unguarded_partition_pivot on [first, last) with the pivot already at first, > 64 elements.
// Hoare's loop pairs the k-th left stop L_k (!(key < pivot), scanning up from first+1) with the
// k-th right stop R_k (!(pivot < key), scanning down from last-1), swaps while L_k < R_k, and
// returns min(L_K, R_{K-1}) for the first crossing pair K (R_{-1} = last).  Here both scans advance
// 64 positions at a time and the stops found are queued one per lane; a pair is only formed when
// both of its stops are known.  Positions swapped by pair j (L_j, R_j) lie outside the span
// (L_k, R_k) of every later valid pair k, so stops read in a chunk before or after such a swap are
// the same up to the crossing, and the min() covers a left scan that has run into swapped
// territory.  Every position is read at most once.
// The stops are held in registers (one wave): each scanned chunk's keys and values are read once, its
// stops are packed into the queue lanes by a forward permute (stop of rank r to
// lane r, the other lanes behind them), and a swap writes the two held elements without reading
// them again.  A held element is exact when it is swapped: a valid pair (L_j < R_j) never meets a
// position an earlier pair swapped (L increases, R decreases), and only valid pairs swap.  LDS
// operations of one wave complete in order, so a later chunk read sees earlier swaps.
template <typename K, typename V>
LG_DEVICE int wave_partition_stream_reg(const SortView<K, V>& a, int first, int last) {
  // the queues: lanes [hL, hL + nqL) hold the pending left stops (position, key, value) in scan order,
  // lanes [hR, hR + nqR) the right stops; pair i = (left lane hL + i, right lane hR + i).  With 16-bit
  // values a stop's position and value travel as one word (positions < 2^16: n <= 2048 here).
  constexpr bool kPack = sizeof(V) == 2;
  const int lane = lane_id();
  const K pv = a.key[first];
  int lo = first + 1, hi = last - 1;
  int qL = 0, qR = 0, nqL = 0, nqR = 0, hL = 0, hR = 0;
  K kL = K(0), kR = K(0);
  int vL = 0, vR = 0;
  int lastR = last;
  auto pos_of = [](int q) { return kPack ? (q >> 16) : q; };
  while (true) {
    if (nqL == 0) {
      if (lo >= last) return min(last, lastR);  // unreachable for a median-of-3 pivot
      // Skip, four chunks at a time, the chunks without a left stop (keys only: a run of keys below the
      // pivot queues nothing).  A degenerate partition (a pivot near one end of the range, the VoxelGrid's
      // heavy rings) otherwise streams its long side chunk by chunk through the queue permutes.
      while (lo + 256 <= last) {
        bool any[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) any[u] = !(a.key[lo + 64 * u + lane] < pv);
        const unsigned long long b0 = __builtin_amdgcn_ballot_w64(any[0]), b1 = __builtin_amdgcn_ballot_w64(any[1]);
        const unsigned long long b2 = __builtin_amdgcn_ballot_w64(any[2]), b3 = __builtin_amdgcn_ballot_w64(any[3]);
        if (b0) break;
        if (b1) { lo += 64; break; }
        if (b2) { lo += 128; break; }
        if (b3) { lo += 192; break; }
        lo += 256;
      }
      const int pL = lo + lane;
      const bool in = pL < last;
      const K k = a.key[in ? pL : first];
      const int v = (int)a.val[in ? pL : first];
      const bool st = in && !(k < pv);
      const unsigned long long m = __ballot(st);
      const int ns = __popcll(m), below = popc_below(m);
      const int dst = st ? below : ns + (lane - below);
      qL = perm_push(dst, kPack ? (pL << 16) | v : pL);
      kL = perm_push(dst, k);
      if (!kPack) vL = perm_push(dst, v);
      nqL = ns;
      hL = 0;
      lo += 64;
    }
    if (nqR == 0) {
      while (hi - 255 >= first) {  // the same for the right scan: chunks without a right stop
        bool any[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) any[u] = !(pv < a.key[hi - 64 * u - lane]);
        const unsigned long long b0 = __builtin_amdgcn_ballot_w64(any[0]), b1 = __builtin_amdgcn_ballot_w64(any[1]);
        const unsigned long long b2 = __builtin_amdgcn_ballot_w64(any[2]), b3 = __builtin_amdgcn_ballot_w64(any[3]);
        if (b0) break;
        if (b1) { hi -= 64; break; }
        if (b2) { hi -= 128; break; }
        if (b3) { hi -= 192; break; }
        hi -= 256;
      }
      const int pR = hi - lane;
      const bool in = pR >= first;
      const K k = a.key[in ? pR : first];
      const int v = (int)a.val[in ? pR : first];
      const bool st = in && !(pv < k);
      const unsigned long long m = __ballot(st);
      const int ns = __popcll(m), below = popc_below(m);
      const int dst = st ? below : ns + (lane - below);
      qR = perm_push(dst, kPack ? (pR << 16) | v : pR);
      kR = perm_push(dst, k);
      if (!kPack) vR = perm_push(dst, v);
      nqR = ns;
      hR = 0;
      hi -= 64;
    }
    const int np = min(nqL, nqR);
    if (np == 0) continue;  // a scanned chunk without stops
    const int i = lane - hL;
    const int src = min(max(hR + i, 0), 63);
    const int rqw = __shfl(qR, src);
    const K rk = shfl_any(kR, src);
    const int rv = kPack ? (rqw & 0xffff) : __shfl(vR, src);
    const int lq = pos_of(qL), rq = pos_of(rqw);
    const bool valid = i >= 0 && i < np && lq < rq;
    const int nv = __popcll(__ballot(valid));  // valid pairs form a prefix (L increasing, R decreasing)
    if (valid) {
      a.key[lq] = rk; a.val[lq] = (V)rv;
      a.key[rq] = kL; a.val[rq] = (V)(kPack ? (qL & 0xffff) : vL);
    }
    if (nv < np) {
      const int Lk = __builtin_amdgcn_readlane(lq, hL + nv);
      const int Rk1 = nv > 0 ? __builtin_amdgcn_readlane(rq, hL + nv - 1) : lastR;
      return min(Lk, Rk1);
    }
    lastR = __builtin_amdgcn_readlane(rq, hL + np - 1);
    hL += np;
    hR += np;
    nqL -= np;
    nqR -= np;
  }
}

template <int R, typename K, typename V>
LG_DEVICE void final_bitonic(K* key, V* val, int n);

// __final_insertion_sort of the post-partition array [0, n) (integral keys, n <= 64 R): the stable
// order by key, and no element crosses a partition cut.  Every final range is either at most 16 long
// or heap-sorted, and the ranges are ordered (each key of a range <= each key of the next), so a
// position p moves by exactly #{q in (p, p + 15] : key_q < key_p} - #{q in [p - 15, p) : key_q > key_p}:
// neighbours in other ranges never count, and a heap-sorted range does not move.  Row-major positions
// (p = 64 r + lane: every read of a shifted window is conflict-free in LDS), 30 comparisons a
// position, then one scatter; replaces a register bitonic sort of all n (key, position) pairs.
// key[-15 .. n + 14] must be readable LDS (ExtractLds: pad before vkey, vval after it).
template <int R, typename K, typename V>
LG_DEVICE void final_window(K* key, V* val, int n) {
  static_assert(std::is_integral<K>::value, "final_window: integral keys");
  const int lane = lane_id();
  K kr[R];
  unsigned vn[R];  // value | new position << 16
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int p = 64 * r + lane;
    const K* kp = key + min(p, n - 1);  // (one base address: the window's reads take immediate offsets)
    const K k = kp[0];
    int mv = 0;
#pragma unroll
    for (int d = 1; d <= 15; ++d) {
      const K ka = kp[d], kb = kp[-d];
      mv += (p + d < n && ka < k) ? 1 : 0;
      mv -= (p - d >= 0 && k < kb) ? 1 : 0;
    }
    kr[r] = k;
    vn[r] = (unsigned)val[min(p, n - 1)] | ((unsigned)(p + mv) << 16);
    asm volatile("" : "+v"(vn[r]), "+v"(kr[r]));  // materialised here: the row's reads die with it
    __builtin_amdgcn_sched_barrier(0);  // one row's 31 reads in flight at a time (registers)
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (64 * r + lane < n) {
      const int np = (int)(vn[r] >> 16);
      key[np] = kr[r];
      val[np] = (V)(vn[r] & 0xffffu);
    }
  }
  __syncthreads();
}

// final_reg: __final_insertion_sort is computed as a register sort by (key, position): it is stable
// and never moves an element across a partition cut, so its result is the post-partition array
// stably sorted by key.  Needs key bit order == key order: unsigned keys, or float keys none
// negative or NaN (the caller checks); n <= 2048 (unsigned) / 512 (float).
// blk: the per-block insertion sorts' final-block bits (unused, may be null, when the register final pass
// serves the call: final_reg with integral keys, or with n <= 512)
template <typename K, typename V>
LG_DEVICE void wave_std_sort(K* key, V* val, int n, unsigned* blk, bool final_reg = false) {
  const int lane = lane_id();
  if (n <= 1) return;
  const int nwords = (n + 31) >> 5;
  // the register final pass serves unsigned keys of any n <= 2048 and float keys of n <= 512; every
  // other call falls through to the per-block insertion sorts below, which read blk
  const bool reg_final = final_reg && (std::is_integral<K>::value || n <= 512);
  if (!reg_final)
    for (int w = lane; w < nwords; w += 64) blk[w] = 0u;
  __syncthreads();
  SortView<K, V> a{key, val};
  PROF_T(t_part0);
  // The range stack in registers: frame i in lane i (written and read by lane index on the scalar
  // unit, no LDS round trip), one word a frame (first, last, depth): first and last <= 2048 (12 bits
  // each), depth <= 22.
  auto sort_frame = [](int f, int l, int d) { return f | (l << 12) | (d << 24); };
  int frames = lane == 0 ? sort_frame(0, n, 2 * floor_log2(n)) : 0;
  int sp = 1;
  while (sp > 0) {
    --sp;
    const int fr = __builtin_amdgcn_readlane(frames, sp);
    int first = fr & 0xfff, last = (fr >> 12) & 0xfff, depth = fr >> 24;
    while (last - first > 16) {
      if (depth == 0) {
        PROF_T(t_hs0);
        heap_sort_wave(a, first, last);
        PROF_ADD(7, t_hs0);
#ifdef LG_PROFILE
        if (lane == 0) atomicAdd(&PROF_SLOT(24), 1ull);
#endif
        break;
      }
      --depth;
      int cut;
      if (last - first <= 64) {  // one chunk: partition in registers
        cut = wave_partition_small(a, first, last);
      } else {
        if (lane == 0) move_median_to_first(a, first, first + 1, first + (last - first) / 2, last - 1);
        __syncthreads();
        cut = wave_partition_stream_reg(a, first, last);  // (every caller: one wave a workgroup)
        __syncthreads();
      }
      frames = lane == sp ? sort_frame(cut, last, depth) : frames;  // (sp <= 2 * 11 + 1)
      ++sp;
      last = cut;
    }
    if (!reg_final && lane == 0) blk[first >> 5] |= 1u << (first & 31);  // a final block starts here
  }
  __syncthreads();
  PROF_ADD(6, t_part0);
  PROF_T(t_fin0);
  if constexpr (std::is_integral<K>::value && sizeof(V) == 2) {
    if (final_reg) {
      if (n <= 64) final_window<1>(key, val, n);
      else if (n <= 128) final_window<2>(key, val, n);
      else if (n <= 256) final_window<4>(key, val, n);
      else if (n <= 512) final_window<8>(key, val, n);
      else if (n <= 1024) final_window<16>(key, val, n);
      else final_window<32>(key, val, n);
      PROF_ADD(11, t_fin0);
      return;
    }
  }
  if (reg_final) {
    if (n <= 64) final_bitonic<1>(key, val, n);
    else if (n <= 128) final_bitonic<2>(key, val, n);
    else if (n <= 256) final_bitonic<4>(key, val, n);
    else if (n <= 512) final_bitonic<8>(key, val, n);
    else if constexpr (std::is_integral<K>::value) {
      if (n <= 1024) final_bitonic<16>(key, val, n);
      else final_bitonic<32>(key, val, n);
    }
    PROF_ADD(11, t_fin0);
    return;
  }
  // __final_insertion_sort as independent per-block insertion sorts: lane h sorts the blocks that
  // start in positions [16h, 16h + 16).
  const int nhalf = (n + 15) >> 4;
  for (int h = lane; h < nhalf; h += 64) {
    unsigned bits = (blk[h >> 1] >> ((h & 1) * 16)) & 0xffffu;
    while (bits) {
      const int p = 16 * h + __ffs(bits) - 1;
      bits &= bits - 1u;
      int e = n;
      if (bits) {
        e = 16 * h + __ffs(bits) - 1;
      } else {
        const unsigned rest = blk[h >> 1] & ~((2u << ((h & 1) * 16 + 15)) - 1u);  // later bits of this word
        if ((h & 1) == 0 && rest) {
          e = 32 * (h >> 1) + __ffs(rest) - 1;
        } else {
          for (int ww = (h >> 1) + 1; ww < nwords; ++ww) {
            const unsigned nb = blk[ww];
            if (nb) { e = 32 * ww + __ffs(nb) - 1; break; }
          }
        }
      }
      for (int i = p + 1; i < e; ++i) {
        K vk = key[i];
        V vv = val[i];
        int j = i;
        while (j > p && vk < key[j - 1]) {
          key[j] = key[j - 1];
          val[j] = val[j - 1];
          --j;
        }
        key[j] = vk;
        val[j] = vv;
      }
    }
  }
  __syncthreads();
  PROF_ADD(11, t_fin0);
}

struct ScanView {
  int M, VH;
  const float* curv;
  uint8_t* picked;
  int8_t* flabel;
  const uint32_t* col;
  const uint8_t* gflag;
  const float4* fa;
  LG_DEVICE uint32_t col_at(int k) const { return k < M ? col[k] : 0u; }         // tail is 0 (:138)
  LG_DEVICE bool ground_at(int k) const { return k < M ? gflag[k] != 0 : false; }  // tail false (:137)
};

// The +-5 neighbour suppression with one wave: lanes 0..4 take l = 1..5, lanes 8..12 take
// l = -1..-5; each direction stops at its first column jump > 10 (the reference's `break`) and skips
// out-of-range l (`continue`), exactly as the sequential loops (all writes set picked to 1).
LG_DEVICE void suppress_wave(const ScanView& v, int ind) {
  const int lane = lane_id();
  const int l = (lane < 5) ? lane + 1 : (lane >= 8 && lane < 13) ? -(lane - 7) : 0;
  bool valid = false, brk = false;
  if (l > 0) {
    valid = (unsigned)(ind + l) < (unsigned)v.VH;
    if (valid) brk = abs((int)(v.col_at(ind + l) - v.col_at(ind + l - 1))) > 10;
  } else if (l < 0) {
    valid = ind + l >= 0;
    if (valid) brk = abs((int)(v.col_at(ind + l) - v.col_at(ind + l + 1))) > 10;
  }
  const unsigned long long bm = __ballot(brk);
  const unsigned fwd = (unsigned)(bm & 0x1full), bwd = (unsigned)((bm >> 8) & 0x1full);
  const int ff = fwd ? __ffs(fwd) - 1 : 5, fb = bwd ? __ffs(bwd) - 1 : 5;  // index of the breaking l
  if (l > 0 && valid && (l - 1) < ff) v.picked[ind + l] = 1;
  if (l < 0 && valid && (-l - 1) < fb) v.picked[ind + l] = 1;
  if (lane == 0) v.picked[ind] = 1;
}

// The extent of suppress_neighbours(ind): it sets picked[ind - fb .. ind + ff] (both <= 5).  Depends
// only on colInd, so a candidate can compute it before it is picked.
LG_DEVICE void supp_extent(const ScanView& v, int ind, int& ff, int& fb) {
  uint32_t c[11];
#pragma unroll
  for (int j = 0; j < 11; ++j) {
    const int k = ind - 5 + j;
    c[j] = (k >= 0 && k < v.M) ? v.col[k] : 0u;  // col_at
  }
  ff = 0;
#pragma unroll
  for (int l = 1; l <= 5; ++l) {
    if (ff != l - 1) break;
    if ((unsigned)(ind + l) >= (unsigned)v.VH) break;  // `continue` for this and every later l
    if (abs((int)(c[5 + l] - c[4 + l])) > 10) break;
    ff = l;
  }
  fb = 0;
#pragma unroll
  for (int l = 1; l <= 5; ++l) {
    if (fb != l - 1) break;
    if (ind - l < 0) break;
    if (abs((int)(c[5 - l] - c[6 - l])) > 10) break;
    fb = l;
  }
}

LG_DEVICE void suppress_neighbours(const ScanView& v, int ind) {  // :306-326
  v.picked[ind] = 1;
  for (int l = 1; l <= 5; l++) {
    if ((unsigned)(ind + l) >= (unsigned)v.VH) continue;
    int columnDiff = abs((int)(v.col_at(ind + l) - v.col_at(ind + l - 1)));
    if (columnDiff > 10) break;
    v.picked[ind + l] = 1;
  }
  for (int l = -1; l >= -5; l--) {
    if (ind + l < 0) continue;
    int columnDiff = abs((int)(v.col_at(ind + l) - v.col_at(ind + l + 1)));
    if (columnDiff > 10) break;
    v.picked[ind + l] = 1;
  }
}

// Ascending bitonic sort of R u64 values per lane (element lane*R + r), all in registers: strides
// j >= R exchange with lane ^ (j / R), smaller strides swap registers.  The k and cross-lane j
// loops stay rolled (code size); the in-register strides are unrolled with a uniform guard.
template <int R>
LG_DEVICE void reg_bitonic_u64(unsigned long long (&a)[R]) {
  const int lane = lane_id();
#pragma unroll 1
  for (int k = 2; k <= 64 * R; k <<= 1) {
#pragma unroll 1
    for (int j = k >> 1; j >= R; j >>= 1) {
      const int m = j / R;
      // k >= 2R here, so bit k of lane*R + r does not depend on r
      const bool take_min = ((lane & m) == 0) == (((lane * R) & k) == 0);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const unsigned long long x = a[r];
        const unsigned long long y = ((unsigned long long)(unsigned)__shfl_xor((int)(x >> 32), m) << 32) |
                                     (unsigned)__shfl_xor((int)(unsigned)x, m);
        a[r] = ((x < y) == take_min) ? x : y;
      }
    }
#pragma unroll
    for (int j = R / 2; j >= 1; j >>= 1) {
      if (j > (k >> 1)) continue;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (r & j) continue;
        const bool asc = (((lane * R + r) & k) == 0);
        const unsigned long long x = a[r], y = a[r | j];
        const bool sw = (x > y) == asc;
        a[r] = sw ? y : x;
        a[r | j] = sw ? x : y;
      }
    }
  }
}

LG_DEVICE unsigned key_bits(float k) { return (unsigned)__float_as_int(k); }
LG_DEVICE unsigned key_bits(unsigned k) { return k; }
LG_DEVICE void key_from_bits(float& k, unsigned b) { k = __int_as_float((int)b); }
LG_DEVICE void key_from_bits(unsigned& k, unsigned b) { k = b; }

// The post-partition array [0, n) sorted by (key bits, position), values gathered by position.
template <int R, typename K, typename V>
LG_DEVICE void final_bitonic(K* key, V* val, int n) {
  const int lane = lane_id();
  unsigned long long a[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int e = lane * R + r;
    a[r] = e < n ? (((unsigned long long)key_bits(key[e]) << 32) | (unsigned)e) : ~0ull;
  }
  reg_bitonic_u64<R>(a);
  V vg[R];
#pragma unroll
  for (int r = 0; r < R; ++r) vg[r] = (lane * R + r < n) ? val[(unsigned)a[r]] : V(0);
  __syncthreads();
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int e = lane * R + r;
    if (e < n) {
      key_from_bits(key[e], (unsigned)(a[r] >> 32));
      val[e] = vg[r];
    }
  }
  __syncthreads();
}

// (curvature bits << 32 | ring index) in registers; returns false (and leaves LDS untouched) when a
// key tie, a NaN or a sign bit makes the order depend on the sort algorithm (*anomaly: NaN / sign) --
// unless tie_ok(a) accepts the (key, index) order for the ties found (harmless ties, below).
struct NoTieOk {
  template <int R>
  LG_DEVICE bool operator()(const unsigned long long (&)[R], int) const { return false; }
};
template <int R, class TieOk = NoTieOk>
LG_DEVICE bool seg_sort_distinct(float* key, int* val, int n, bool* anomaly, const TieOk& tie_ok = TieOk()) {
  const int lane = lane_id();
  unsigned long long a[R];
  bool bad = false;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int e = lane * R + r;
    if (e < n) {
      const unsigned kb = (unsigned)__float_as_int(key[e]);
      bad |= kb > 0x7f800000u;  // NaN, or negative (incl. -0.0)
      a[r] = ((unsigned long long)kb << 32) | (unsigned)val[e];
    } else {
      a[r] = ~0ull;
    }
  }
  *anomaly = __ballot(bad) != 0ull;
  reg_bitonic_u64<R>(a);
  const unsigned nxt = (unsigned)__shfl_down((int)(a[0] >> 32), 1);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int e = lane * R + r;
    const unsigned kn = (r + 1 < R) ? (unsigned)(a[r + 1 < R ? r + 1 : r] >> 32) : nxt;
    if (e + 1 < n && (unsigned)(a[r] >> 32) == kn) bad = true;
  }
  if (__ballot(bad) != 0ull && (*anomaly || !tie_ok(a, n))) return false;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int e = lane * R + r;
    if (e < n) {
      key[e] = __int_as_float((int)(a[r] >> 32));
      val[e] = (int)(unsigned)a[r];
    }
  }
  __syncthreads();
  return true;
}

// Harmless ties of extractFeatures' segment sort (:285-286).  std::sort's order among equal curvature
// values reaches the outputs only through (a) the greedy passes, which walk the sorted entries and act
// on the eligible ones -- sharp: not picked, curvature > edge threshold, not ground; flat: not picked,
// curvature < surf threshold, ground (:289-349) -- and (b) the stale slot 4, which keeps the entry sorted
// into it for the next scan (ring 0's first segment).  When no run of equal values holds two entries
// eligible for the same pass (eligibility now includes every later one: picks only ever set picked[]),
// each pass meets its eligible entries in one order whatever the tie order, and when the entry sorted
// into slot 4 has a value of its own, every output equals the reference's; the sort by (value, index)
// is then as good as the introsort emulation.
LG_DEVICE unsigned long long shfl_up_u64(unsigned long long v, int o) {
  return ((unsigned long long)(unsigned)__shfl_up((int)(v >> 32), o) << 32) | (unsigned)__shfl_up((int)(unsigned)v, o);
}
struct SegTieOk {
  const float* curv;
  const uint8_t* picked;
  const uint8_t* gflag;
  int M, sp;
  float edge_thr, surf_thr;
  template <int R>
  LG_DEVICE bool operator()(const unsigned long long (&a)[R], int n) const {
    const int lane = lane_id();
    unsigned esm = 0u, efm = 0u;  // per position: sharp / flat eligible
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int e = lane * R + r;
      if (e < n) {
        const int ind = (int)(unsigned)a[r];
        const float c = curv[ind];
        const bool pk = picked[ind] != 0;
        const bool g = ind < M ? gflag[ind] != 0 : false;
        esm |= (unsigned)(!pk && c > edge_thr && !g) << r;
        efm |= (unsigned)(!pk && c < surf_thr && g) << r;
      }
    }
    // the previous eligible entry's value for every eligible entry: within the lane in order, across
    // lanes the last eligible value of the lanes below (a "last set" scan)
    bool clash = false;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const unsigned m = pass ? efm : esm;
      unsigned long long last = ~0ull;  // (has << 32 | value bits); ~0: none
#pragma unroll
      for (int r = 0; r < R; ++r)
        if ((m >> r) & 1u) last = a[r] >> 32;
      // inclusive "last eligible value" scan over the lanes (a higher lane's own value wins), then
      // shifted up by one lane: the last eligible value of the lanes below
      unsigned long long y = last;
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long t = shfl_up_u64(y, o);
        if (lane >= o && y == ~0ull) y = t;
      }
      const unsigned long long yb = shfl_up_u64(y, 1);  // (every lane shuffles: lane 0 is a source)
      const unsigned long long below = lane > 0 ? yb : ~0ull;
      unsigned long long prev = below;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if ((m >> r) & 1u) {
          const unsigned long long kv = a[r] >> 32;
          if (prev == kv) clash = true;
          prev = kv;
        }
      }
    }
    // slot 4: the entry sorted to position 4 - sp must be alone with its value
    const int p4 = 4 - sp;
    if (p4 >= 0 && p4 < n) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int e = lane * R + r;
        if (e == p4) {
          const unsigned k = (unsigned)(a[r] >> 32);
          const unsigned kp = r > 0 ? (unsigned)(a[r > 0 ? r - 1 : 0] >> 32) : ~0u;
          const unsigned kn = r + 1 < R ? (unsigned)(a[r + 1 < R ? r + 1 : r] >> 32) : ~0u;
          if ((e > 0 && r > 0 && kp == k) || (e + 1 < n && r + 1 < R && kn == k)) clash = true;
        }
      }
      // neighbours across a lane boundary
      const unsigned klast = (unsigned)(a[R - 1] >> 32), kfirst = (unsigned)(a[0] >> 32);
      const unsigned from_below = (unsigned)__shfl_up((int)klast, 1), from_above = (unsigned)__shfl_down((int)kfirst, 1);
      if (p4 == lane * R && p4 > 0 && lane > 0 && from_below == kfirst) clash = true;
      if (p4 == lane * R + R - 1 && p4 + 1 < n && lane < 63 && from_above == klast) clash = true;
    }
    return __ballot(clash) == 0ull;
  }
};

// Sort [0, n) of (key, val): all-distinct keys -> register bitonic sort (any correct sort gives the
// same permutation); ties that tie_ok accepts -> the same sort (by key, then val); other ties -> exact
// libstdc++ introsort emulation.
template <class Lds, class TieOk = NoTieOk>
LG_DEVICE void sort_segment(Lds& L, int n, const TieOk& tie_ok = TieOk()) {
  float* key = L.u.seg.skey;
  int* val = L.u.seg.sval;
  bool ok, anomaly = true;
  if (n <= 64) ok = seg_sort_distinct<1>(key, val, n, &anomaly, tie_ok);
  else if (n <= 128) ok = seg_sort_distinct<2>(key, val, n, &anomaly, tie_ok);
  else if (n <= 256) ok = seg_sort_distinct<4>(key, val, n, &anomaly, tie_ok);
  else ok = seg_sort_distinct<8>(key, val, n, &anomaly, tie_ok);
  if (!ok) {
#ifdef LG_PROFILE
    if (lane_id() == 0) atomicAdd(&PROF_SLOT(14), 1ull);
#endif
    wave_std_sort<float, int>(key, val, n, L.blk, !anomaly && n <= SEG_MAX);
  }
}

struct RingOut {
  float4* sharp; int32_t* sharp_ind;
  float4* lsharp; int32_t* lsharp_ind;
  float4* flat; int32_t* flat_ind;
  float4* lflat;
  int nS, nLS, nF, nLF;
  int status;
};

LG_DEVICE float4 seg_point(const ScanView& v, int ind, int& status) {  // segmentedCloud->points[ind]
  if (ind >= 0 && ind < v.M) return v.fa[ind];
  status |= LEGO_ST_STALE_IND_OOB;
  return make_float4(0.f, 0.f, 0.f, 0.f);
}

LG_DEVICE unsigned* vx_key(ExtractLds& L) { return L.u.vkey; }
LG_DEVICE uint16_t* vx_val(ExtractLds& L) { return L.vval; }
template <int R>
LG_DEVICE unsigned* vx_key(VoxLvlLds<R>& L) { return L.u.nat.key; }
template <int R>
LG_DEVICE uint16_t* vx_val(VoxLvlLds<R>& L) { return L.u.nat.val; }

// PCL VoxelGrid<PointXYZI> (leaf 0.2) over the ring's lessFlat points (positions in L.vval[0..n)).
// Ascending sort of n <= RING_MAX (key, val) pairs by (key, val), one wave, (key << 32 | val) in
// registers.  vals are distinct ring positions appended in point order, so this is the order
// std::stable_sort gives by key alone (lego_params.voxel_tie_order == 1).
template <int R>
LG_DEVICE void voxel_sort_reg(unsigned* key, uint16_t* val, int n) {
  const int lane = lane_id();
  unsigned long long a[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int e = lane * R + r;
    a[r] = e < n ? (((unsigned long long)key[e] << 32) | val[e]) : ~0ull;
  }
  reg_bitonic_u64<R>(a);
  __syncthreads();
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int e = lane * R + r;
    if (e < n) {
      key[e] = (unsigned)(a[r] >> 32);
      val[e] = (uint16_t)a[r];
    }
  }
  __syncthreads();
}

// kMode 2: rings of more than 1024 points (R = 32, 64 VGPRs of keys) only; mode 1 keeps R <= 16;
// mode 3 takes any ring.
template <int kMode>
LG_DEVICE void voxel_sort_stable(unsigned* key, uint16_t* val, int n) {
  if constexpr (kMode == 3) {
    if (n > 1024) voxel_sort_reg<32>(key, val, n);
    else voxel_sort_stable<1>(key, val, n);
  } else if constexpr (kMode == 2) {
    voxel_sort_reg<32>(key, val, n);
  } else {
    if (n <= 64) voxel_sort_reg<1>(key, val, n);
    else if (n <= 128) voxel_sort_reg<2>(key, val, n);
    else if (n <= 256) voxel_sort_reg<4>(key, val, n);
    else if (n <= 512) voxel_sort_reg<8>(key, val, n);
    else voxel_sort_reg<16>(key, val, n);
  }
}

// kMode 0: voxel_tie_order 0 (libstdc++ introsort permutation); 1 / 2: stable order, rings of at most /
// more than 1024 points; 3: either order, any ring (one kernel for the whole step).
// The ring's points are read in batches of VX_U a lane with every load of a batch issued before any is
// used (a loop of single loads pays one memory latency per point); L.vval is the identity on entry.
#define VX_U 8
template <int kMode, class Lds>
LG_DEVICE void voxel_ring(const LgParams& P, const ScanView& v, Lds& L, int n, int base_pos, RingOut& o) {
  unsigned* vkey = vx_key(L);
  uint16_t* vval = vx_val(L);
  const float4* fa = v.fa + base_pos;  // vval holds positions relative to the ring start
  const int lane = lane_id();
  o.nLF = 0;
  if (n == 0) return;
  const float leaf = 0.2f;
  const float inv = 1.0f / leaf;
  float mnx = FLT_MAX, mny = FLT_MAX, mnz = FLT_MAX, mxx = -FLT_MAX, mxy = -FLT_MAX, mxz = -FLT_MAX;
  for (int t0 = lane; t0 < n; t0 += 64 * VX_U) {  // getMinMax3D (clamped repeats do not change a min / max)
    float4 pk[VX_U];
#pragma unroll
    for (int u = 0; u < VX_U; ++u) pk[u] = fa[min(t0 + 64 * u, n - 1)];
#pragma unroll
    for (int u = 0; u < VX_U; ++u) {
      const float4 p = pk[u];
      mnx = (p.x < mnx) ? p.x : mnx; mny = (p.y < mny) ? p.y : mny; mnz = (p.z < mnz) ? p.z : mnz;
      mxx = (p.x > mxx) ? p.x : mxx; mxy = (p.y > mxy) ? p.y : mxy; mxz = (p.z > mxz) ? p.z : mxz;
    }
  }
  mnx = wave_min(mnx); mny = wave_min(mny); mnz = wave_min(mnz);
  mxx = wave_max(mxx); mxy = wave_max(mxy); mxz = wave_max(mxz);
  const long long dx = (long long)((mxx - mnx) * inv) + 1;
  const long long dy = (long long)((mxy - mny) * inv) + 1;
  const long long dz = (long long)((mxz - mnz) * inv) + 1;
  if (dx * dy * dz > 2147483647ll) {  // PCL: "Integer indices would overflow" -> output = input
    for (int t = lane; t < n; t += 64) o.lflat[t] = fa[vval[t]];
    o.nLF = n;
    o.status |= LEGO_ST_VOXEL_OVERFLOW;
    return;
  }
  const int minbx = (int)floorf(mnx * inv), minby = (int)floorf(mny * inv), minbz = (int)floorf(mnz * inv);
  const int maxbx = (int)floorf(mxx * inv), maxby = (int)floorf(mxy * inv);
  const int divx = maxbx - minbx + 1, divy = maxby - minby + 1;
  const int mul1 = divx, mul2 = divx * divy;
  for (int t0 = lane; t0 < n; t0 += 64 * VX_U) {
    float4 pk[VX_U];
#pragma unroll
    for (int u = 0; u < VX_U; ++u) pk[u] = fa[min(t0 + 64 * u, n - 1)];
#pragma unroll
    for (int u = 0; u < VX_U; ++u) {
      const int t = t0 + 64 * u;
      const float4 p = pk[u];
      const int i0 = (int)(floorf(p.x * inv) - (float)minbx);
      const int i1 = (int)(floorf(p.y * inv) - (float)minby);
      const int i2 = (int)(floorf(p.z * inv) - (float)minbz);
      if (t < n) vkey[t] = (unsigned)(i0 + i1 * mul1 + i2 * mul2);
    }
  }
  __syncthreads();
  PROF_T(t_vs0);
  if constexpr (kMode == 0) {
    wave_std_sort<unsigned, uint16_t>(vkey, vval, n, nullptr, true);
  } else if constexpr (kMode == 3) {
    if (P.voxel_stable) voxel_sort_stable<3>(vkey, vval, n);
    else wave_std_sort<unsigned, uint16_t>(vkey, vval, n, nullptr, true);
  } else {
    voxel_sort_stable<kMode>(vkey, vval, n);
  }
  PROF_ADD(5, t_vs0);
  int running = 0;
  for (int base = 0; base < n; base += 64) {
    const int t = base + lane;
    const bool start = t < n && (t == 0 || vkey[t] != vkey[t - 1]);
    const unsigned long long m = __ballot(start);
    if (start) {  // CentroidPoint: float sums in sorted order; the run's loads VX_U at a time in flight
      const unsigned k = vkey[t];
      int e = t + 1;
      while (e < n && vkey[e] == k) ++e;
      float sx = 0.f, sy = 0.f, sz = 0.f, si = 0.f;
      for (int g = t; g < e; g += VX_U) {
        float4 pk[VX_U];
#pragma unroll
        for (int u = 0; u < VX_U; ++u) pk[u] = fa[vval[min(g + u, e - 1)]];
#pragma unroll
        for (int u = 0; u < VX_U; ++u)
          if (g + u < e) { sx += pk[u].x; sy += pk[u].y; sz += pk[u].z; si += pk[u].w; }
      }
      const float cntf = (float)(e - t);
      o.lflat[running + popc_below(m)] = make_float4(sx / cntf, sy / cntf, sz / cntf, si / cntf);
    }
    running += __popcll(m);
  }
  o.nLF = running;
}

// Per-position greedy state of one ring's window [st - 5, en + 6), staged in LDS by its ring-wave:
// the static eligibility of each pass, the suppression extent (supp_extent: depends only on colInd)
// and picked[], kept in step with the global writes.  Rings never reach into each other's windows
// (a pick's +-5 stays inside [st - 5, en + 5], which lies strictly between the neighbouring rings'
// windows); the one exception, the stale slot 4's index, is read from global memory (info_global)
// and rings whose window it meets stage only after the first pass has run (k_extract).
#define EXT_STAGE 2064  // window <= H + 1 positions (H <= 2048)
#define IF_PK 0x100     // picked
#define IF_SH 0x40      // sharp-eligible: curvature > edge threshold, not ground
#define IF_FL 0x80      // flat-eligible: curvature < surf threshold, ground
struct ExtLds {  // k_extract: 8.9 KB per wave
  uint16_t sv[EXT_STAGE];    // the ring's sorted entries (k_sortseg), as indices relative to st
  uint16_t info[EXT_STAGE];  // ff | fb << 3 | IF_SH | IF_FL | IF_PK
  int pk_s[16], pk_ls[128], pk_f[32];  // this ring's picks, in pick order
};

LG_DEVICE int info_global(const LgParams& P, const ScanView& v, int ind) {
  int ff, fb;
  supp_extent(v, ind, ff, fb);
  const float c = v.curv[ind];
  const bool g = v.ground_at(ind);
  return ff | (fb << 3) | (c > P.edge_thr && !g ? IF_SH : 0) | (c < P.surf_thr && g ? IF_FL : 0) |
         (v.picked[ind] != 0 ? IF_PK : 0);
}

// Info words of positions [k0, k0 + cnt) (one segment [sp, ep]) into xinfo; colbuf: LDS of at least
// cnt + 10 entries for the colInd window (col_at with supp_extent's bounds).
LG_DEVICE void build_info(const LgParams& P, const ScanView& v, int k0, int cnt, uint16_t* xinfo, uint16_t* colbuf) {
  const int lane = lane_id();
  const int c0 = k0 - 5;
  for (int t0 = lane; t0 < cnt + 10; t0 += 64 * 4) {
    uint32_t cv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) cv[u] = v.col[min(max(c0 + t0 + 64 * u, 0), max(v.M - 1, 0))];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int t = t0 + 64 * u, k = c0 + t;
      if (t < cnt + 10) colbuf[t] = (uint16_t)((k >= 0 && k < v.M) ? cv[u] : 0u);
    }
  }
  __syncthreads();
  for (int t0 = lane; t0 < cnt; t0 += 64 * 4) {
    float cv[4];
    uint8_t pk[4], gf[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = min(k0 + t0 + 64 * u, k0 + cnt - 1);
      cv[u] = v.curv[k];
      pk[u] = v.picked[k];
      gf[u] = k < v.M ? v.gflag[k] : 0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int t = t0 + 64 * u;
      if (t >= cnt) break;
      const int ind = k0 + t;
      const int x = t + 5;  // ind's slot in colbuf
      int ff = 0;
#pragma unroll
      for (int l = 1; l <= 5; ++l) {
        if (ff != l - 1) break;
        if ((unsigned)(ind + l) >= (unsigned)v.VH) break;
        if (abs((int)colbuf[x + l] - (int)colbuf[x + l - 1]) > 10) break;
        ff = l;
      }
      int fb = 0;
#pragma unroll
      for (int l = 1; l <= 5; ++l) {
        if (fb != l - 1) break;
        if (ind - l < 0) break;
        if (abs((int)colbuf[x - l] - (int)colbuf[x - l + 1]) > 10) break;
        fb = l;
      }
      const bool g = gf[u] != 0;
      xinfo[ind] = (uint16_t)(ff | (fb << 3) | (cv[u] > P.edge_thr && !g ? IF_SH : 0) |
                              (cv[u] < P.surf_thr && g ? IF_FL : 0) | (pk[u] != 0 ? IF_PK : 0));
    }
  }
}

LG_DEVICE void extract_ring(const LgParams& P, const ScanView& v, int2* smooth, int st, int en, const uint16_t* xinfo,
                            int stale, ExtLds& L, RingOut& o) {
  const int lane = lane_id();
  if (en <= st) return;  // no segment with sp < ep
  // the window is the ring's candidate range [st, en]: its info words (k_sortseg) into LDS
  const int lo = st, nwin = en - st + 1;
  PROF_T(t_st0);
  for (int t0 = lane; t0 < nwin; t0 += 64 * 8) {  // with the sorted entries of every segment (k_sortseg)
    uint16_t w8[8];
    int e8[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = lo + min(t0 + 64 * u, nwin - 1);
      w8[u] = xinfo[k];
      e8[u] = smooth[k].y;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (t0 + 64 * u < nwin) {
        L.info[t0 + 64 * u] = w8[u];
        L.sv[t0 + 64 * u] = (uint16_t)((unsigned)(e8[u] - lo) < (unsigned)nwin ? e8[u] - lo : 0xffff);
      }
  }
  // the first pass's stale-slot pick may have marked picked[] around its index after k_sortseg built
  // the words (a ring whose window meets that zone waited for it): refresh those bits
  if (stale >= 0 && lane < 11) {
    const int k = stale - 5 + lane;
    if (k >= lo && k < lo + nwin && k < v.VH && v.picked[k]) L.info[k - lo] |= IF_PK;
  }
  __syncthreads();
  PROF_ADD(12, t_st0);
  // info word of a candidate position (global for the stale index outside the window)
  auto info_of = [&](int ind) -> int {
    const int rel = ind - lo;
    return (unsigned)rel < (unsigned)nwin ? (int)L.info[rel] : info_global(P, v, ind);
  };
  // a pick's suppression: picked[] in global memory (persistent state) and in the window
  auto suppress = [&](int aind, int aff, int afb) {
    if (lane <= aff + afb) {
      const int k = aind - afb + lane;
      v.picked[k] = 1;
      if ((unsigned)(k - lo) < (unsigned)nwin) L.info[k - lo] |= IF_PK;
    }
  };
  int nS = 0, nLS = 0, nF = 0;
  for (int j = 0; j < 6; j++) {
    const int sp = (st * (6 - j) + en * j) / 6;
    const int ep = (st * (5 - j) + en * (j + 1)) / 6 - 1;
    if (sp >= ep) continue;
    const int n = ep - sp;  // sorted range [sp, ep) (k_sortseg); ep itself is visited unsorted
    // the entry at position sp + t: its index relative to st from LDS, or (0xffff: the stale slot's
    // index outside the window) from the smoothness array itself
    auto entry = [&](int t) -> int {
      const int r = L.sv[sp - lo + t];
      return r != 0xffff ? lo + r : smooth[sp + t].y;
    };
    PROF_T(t_sharp0);
    // sharp: k = ep .. sp (descending curvature), first 2 eligible -> sharp, up to 20 -> less sharp.
    // A chunk of 64 candidates reads its info words once; a pick then kills the chunk's lanes inside
    // its suppression extent in registers (the same writes go to the window for later chunks).
    int largest = 0;
    bool stop = false;
    for (int base = n; base >= 0 && !stop; base -= 64) {
      const int t = base - lane;
      const bool valid = t >= 0;
      const int ind = valid ? entry(t) : 0;
      const int w = valid ? info_of(ind) : 0;
      bool cand = valid && !(w & IF_PK) && (w & IF_SH);
      if (__ballot(cand) == 0ull) continue;
      const int ff = w & 7, fb = (w >> 3) & 7;
      while (true) {
        const unsigned long long m = __ballot(cand);
        if (m == 0ull) break;
        const int f = __ffsll((long long)m) - 1;
        const int aind = __shfl(ind, f), aff = __shfl(ff, f), afb = __shfl(fb, f);
        largest++;
        if (largest > 20) { stop = true; break; }
        if (lane == 0) {
          if (largest <= 2) {
            v.flabel[aind] = 2;
            L.pk_s[nS] = aind;
          } else {
            v.flabel[aind] = 1;
          }
          L.pk_ls[nLS] = aind;
        }
        suppress(aind, aff, afb);
        if (largest <= 2) nS++;
        nLS++;
        cand = cand && lane > f && !(ind >= aind - afb && ind <= aind + aff);
      }
      __syncthreads();  // picked[] writes land before the next chunk reads them
    }
    PROF_ADD(1, t_sharp0);
    PROF_T(t_flat0);
    // flat: k = sp .. ep, ground points with curvature < surf threshold, at most 4
    int smallest = 0;
    stop = false;
    for (int base = 0; base <= n && !stop; base += 64) {
      const int t = base + lane;
      const bool valid = t <= n;
      const int ind = valid ? entry(t) : 0;
      const int w = valid ? info_of(ind) : 0;
      bool cand = valid && !(w & IF_PK) && (w & IF_FL);
      if (__ballot(cand) == 0ull) continue;
      const int ff = w & 7, fb = (w >> 3) & 7;
      while (true) {
        const unsigned long long m = __ballot(cand);
        if (m == 0ull) break;
        const int f = __ffsll((long long)m) - 1;
        const int aind = __shfl(ind, f), aff = __shfl(ff, f), afb = __shfl(fb, f);
        smallest++;
        if (lane == 0) {
          v.flabel[aind] = -1;
          L.pk_f[nF] = aind;
        }
        nF++;
        if (smallest >= 4) { stop = true; break; }  // the 4th breaks before its suppression
        suppress(aind, aff, afb);
        cand = cand && lane > f && !(ind >= aind - afb && ind <= aind + aff);
      }
      __syncthreads();
    }
    __syncthreads();
    PROF_ADD(2, t_flat0);
  }
  // the picked points, all loads in flight together
  int st_bits = 0;
  for (int t = lane; t < nLS; t += 64) {
    const int ind = L.pk_ls[t];
    o.lsharp[t] = seg_point(v, ind, st_bits);
    o.lsharp_ind[t] = ind;
  }
  for (int t = lane; t < nS; t += 64) {
    const int ind = L.pk_s[t];
    o.sharp[t] = seg_point(v, ind, st_bits);
    o.sharp_ind[t] = ind;
  }
  for (int t = lane; t < nF; t += 64) {
    const int ind = L.pk_f[t];
    o.flat[t] = seg_point(v, ind, st_bits);
    o.flat_ind[t] = ind;
  }
  o.status |= wave_or(st_bits);
  o.nS = nS; o.nLS = nLS; o.nF = nF;
  __syncthreads();
}

// lessFlat list of one ring: positions k in [sp, ep] of each segment whose label <= 0 (position
// order, not sorted order: :370-374).  Labels of a segment's positions are final once k_extract
// has processed that segment (later picks label their own segment; the stale slot-4 pick lands
// before its ring runs), so the list is rebuilt here from cloudLabel after k_extract.
LG_DEVICE int lessflat_list(const ScanView& v, int st, int en, uint16_t* list) {
  const int lane = lane_id();
  int nlist = 0;
  for (int j = 0; j < 6; j++) {
    const int sp = (st * (6 - j) + en * j) / 6;
    const int ep = (st * (5 - j) + en * (j + 1)) / 6 - 1;
    if (sp >= ep) continue;
    for (int k0 = sp; k0 <= ep; k0 += 64) {
      const int k = k0 + lane;
      const bool pr = k <= ep && v.flabel[k] <= 0;
      const unsigned long long m = __ballot(pr);
      if (pr) list[nlist + popc_below(m)] = (uint16_t)(k - st);
      nlist += __popcll(m);
    }
  }
  __syncthreads();
  return nlist;
}

// ============================================================================================
// k_voxel: surfPointsLessFlatScan -> VoxelGrid (leaf 0.2) per ring, one wave per ring.  A kernel
// of its own so the register-resident voxel sort's VGPRs do not cut k_extract's occupancy.
// ============================================================================================
// kMode as voxel_ring: 0 for voxel_tie_order 0 by the stack emulation; 1 and 2 split the stable order's
// rings by size; 3 either order.
template <int kM, class Lds>
LG_DEVICE void voxel_wave(const LgParams& P, const ScanView& v, Lds& L, int n, RingOut& o) {
  for (int t = lane_id(); t < n; t += 64) vx_val(L)[t] = (uint16_t)t;
  __syncthreads();
  voxel_ring<kM>(P, v, L, n, 0, o);
}
template <int kMode>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1)))
void k_voxel(LgParams P, LgBufs B) {
  __shared__ ExtractLds L;
  const int V = P.V;
  const int b = blockIdx.x, sl = b / V, s = P.s0 + sl;
  const int ring = (b % V + sl / max(P.ncu / V, 1)) % V;  // ring rotation as in k_extract
  const size_t rb = (size_t)s * V + ring;
  const size_t sb = (size_t)P.par * P.S * V + rb;  // staging half P.par
  ScanView v;
  v.fa = B.lf_stage + sb * P.H;  // the ring's lessFlat points, in surfPointsLessFlatScan order
  const int n = B.lf_count[sb];
  if (kMode != 3 && (P.voxel_stable ? (n > 1024 ? 2 : 1) : 0) != kMode) return;
  RingOut o;
  o.lflat = B.r_lflat + sb * P.H;  // output half P.par too (k_publish of this scan reads it)
  o.nLF = 0;
  o.status = 0;
#ifdef LG_PROFILE
  const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz, one clock for all XCDs
#endif
  PROF_T(t_vox0);
  voxel_wave<kMode>(P, v, L, n, o);
  PROF_ADD(4, t_vox0);
#ifdef LG_PROFILE
  if (lane_id() == 0 && b < 65536) {
    unsigned long long* lg = g_ring_log + (size_t)b * 4;
    lg[0] = rt0;
    lg[1] = __builtin_amdgcn_s_memrealtime();
    lg[2] = (unsigned long long)(unsigned)n | ((unsigned long long)(unsigned)rb << 32);
    lg[3] = (unsigned long long)P.par;
  }
#endif
  if (lane_id() == 0) {
    B.r_vcount[sb] = o.nLF;
    B.r_vstatus[sb] = o.status;
  }
}

// ============================================================================================
// k_sortseg: extractFeatures' std::sort of every segment (:285-286), one wave per (ring, segment).
// The six sorted ranges [sp, ep) of a ring are disjoint and the greedy passes only read them, so
// all segments of a scan sort up front (the stale slot 4 is sorted with ring 0's first segment, as
// there) and k_extract's ring-waves keep only the sequential greedy passes.
// ============================================================================================
__global__ __launch_bounds__(64) void k_sortseg(LgParams P, LgBufs B) {
  __shared__ SegLds L;
  const int V = P.V;
  const int b = blockIdx.x, sl = b / (V * 6), r = (b / 6) % V, j = b % 6;
  const int s = P.s0 + sl;
  const int st = B.ring_start[(size_t)s * V + r], en = B.ring_end[(size_t)s * V + r];
  const int sp = (st * (6 - j) + en * j) / 6;
  const int ep = (st * (5 - j) + en * (j + 1)) / 6 - 1;
  if (sp > ep) return;
  const int n = ep - sp;
  int2* smooth = B.smooth + (size_t)s * P.VH + sp;
  if (n > 0) {  // sorted range [sp, ep) (a one-position segment is never sorted, only visited)
    for (int t = lane_id(); t < n; t += 64) {
      const int2 e = smooth[t];
      L.u.seg.skey[t] = __int_as_float(e.x);
      L.u.seg.sval[t] = e.y;
    }
    __syncthreads();
    PROF_T(t_rs0);
    SegTieOk tie_ok;
    tie_ok.curv = B.curv + (size_t)s * P.VH;
    tie_ok.picked = B.picked + (size_t)s * P.VH;
    tie_ok.gflag = B.seg_ground + (size_t)s * P.VH;
    tie_ok.M = B.counts[(size_t)s * CNT_N + CNT_M];
    tie_ok.sp = sp;
    tie_ok.edge_thr = P.edge_thr;
    tie_ok.surf_thr = P.surf_thr;
    sort_segment(L, n, tie_ok);
    PROF_ADD(13, t_rs0);
    for (int t = lane_id(); t < n; t += 64) smooth[t] = make_int2(__float_as_int(L.u.seg.skey[t]), L.u.seg.sval[t]);
  }
  __syncthreads();  // u.seg is free for the colInd window
  // k_extract's info words for the segment's positions [sp, ep] (candidates are only ever there)
  ScanView v;
  v.M = B.counts[(size_t)s * CNT_N + CNT_M];
  v.VH = P.VH;
  v.curv = B.curv + (size_t)s * P.VH;
  v.picked = B.picked + (size_t)s * P.VH;
  v.col = B.seg_col + (size_t)s * P.VH;
  v.gflag = B.seg_ground + (size_t)s * P.VH;
  build_info(P, v, sp, n + 1, B.xinfo + (size_t)s * P.VH, L.u.col);
}

__global__ __launch_bounds__(64) void k_extract(LgParams P, LgBufs B) {
  __shared__ ExtLds L;
  const int V = P.V, VH = P.VH;
  // Blocks [0, n): the first pass of scan s0 + b.  Rings whose range starts at position 4 (the
  // leading rings) read the stale slot 4 of the persistent smoothness array, whose index may point
  // into any ring: they run first, in order, on one wave.  Blocks [n, n + n*V): one ring each.
  // Every other ring only reads/writes its own position range (+-5), so it runs at once unless
  // that range meets the stale index's +-5 zone; then it waits for its scan's first pass
  // (SURVEY.md Appendix B/C).  Workgroups are dispatched in index order, so a waiting ring only
  // ever waits on a first-pass wave that is already resident.
  const int nS = gridDim.x / (V + 1);
  const bool first_pass = (int)blockIdx.x < nS;
  const int b = first_pass ? (int)blockIdx.x : (int)blockIdx.x - nS;
  // Workgroups reach the CUs round-robin, so with ring = b % V a CU would only ever see one ring
  // index (the upper, non-ground rings are the heavy ones).  Rotating the ring by the stream block
  // (sl / (ncu / V)) gives every CU every ring index; the map stays a bijection per stream.
  const int sl = first_pass ? b : b / V;
  const int s = P.s0 + sl;
  const int rot = sl / max(P.ncu / V, 1);
  const int ring = first_pass ? 0 : (b % V + rot) % V;
  const int32_t* rs = B.ring_start + (size_t)s * V;
  const int32_t* re = B.ring_end + (size_t)s * V;
  int32_t* sync = B.fp_sync + 2 * (size_t)s;
  ScanView v;
  v.M = B.counts[(size_t)s * CNT_N + CNT_M];
  v.VH = VH;
  v.curv = B.curv + (size_t)s * VH;
  v.picked = B.picked + (size_t)s * VH;
  v.flabel = B.flabel + (size_t)s * VH;
  v.col = B.seg_col + (size_t)s * VH;
  v.gflag = B.seg_ground + (size_t)s * VH;
  v.fa = B.seg_fa + (size_t)s * VH;
  int2* smooth = B.smooth + (size_t)s * VH;
  int stale = -1;  // index the stale slot 4 holds (rings after the first pass only)
  if (!first_pass) {
    if (rs[ring] == 4) return;  // a leading ring: done by the first pass
    stale = sync[0];
    if (stale + 5 >= rs[ring] - 5 && stale - 5 <= re[ring] + 5) {
      while (__hip_atomic_load(sync + 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != P.epoch)
        __builtin_amdgcn_s_sleep(4);
#ifdef LG_PROFILE
      if (lane_id() == 0) atomicAdd(&PROF_SLOT(30), 1ull);
#endif
    }
  }
  const int r0 = first_pass ? 0 : ring, r1 = first_pass ? V : ring + 1;
  for (int r = r0; r < r1; ++r) {
    if (first_pass && rs[r] != 4) break;
    RingOut o;
    const size_t rb = (size_t)s * V + r;
    o.sharp = B.r_sharp + rb * P.cap_sharp; o.sharp_ind = B.r_sharp_ind + rb * P.cap_sharp;
    o.lsharp = B.r_lsharp + rb * P.cap_lsharp; o.lsharp_ind = B.r_lsharp_ind + rb * P.cap_lsharp;
    o.flat = B.r_flat + rb * P.cap_flat; o.flat_ind = B.r_flat_ind + rb * P.cap_flat;
    o.lflat = nullptr;  // the VoxelGrid output is k_voxel's
    o.nS = o.nLS = o.nF = o.nLF = 0;
    o.status = 0;
    PROF_T(t_ring0);
    extract_ring(P, v, smooth, rs[r], re[r], B.xinfo + (size_t)s * VH, stale, L, o);
#ifdef LG_PROFILE
    if (lane_id() == 0) {
      const unsigned long long dt = __builtin_amdgcn_s_memtime() - t_ring0;
      atomicAdd(&PROF_SLOT(64 + (first_pass ? 63 : r)), dt);
      atomicMax(&PROF_SLOT(128 + (first_pass ? 63 : r)), dt);
    }
#endif
    if (lane_id() == 0) {
      int32_t* rc = B.r_counts + rb * 4;
      rc[0] = o.nS; rc[1] = o.nLS; rc[2] = o.nF;  // rc[3] unused
      B.r_status[rb] = o.status;
    }
    __syncthreads();
  }
  if (first_pass) {
    __threadfence();
    if (lane_id() == 0) __hip_atomic_store(sync + 1, P.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ============================================================================================
// k_concat: ring-ordered concatenation (cornerPointsSharp etc. are appended ring by ring)
// ============================================================================================
// One wave a ring (grid S * V, 64-lane workgroups: a whole-scan workgroup waited for 16 free wave slots
// of one CU behind the VoxelGrid's waves); each ring's offsets are prefix sums over the ring counts.
__global__ __launch_bounds__(64) void k_concat(LgParams P, LgBufs B) {
  const int V = P.V;
  const int s = P.s0 + blockIdx.x / V, r = blockIdx.x % V, l = lane_id();
  int c0 = 0, c1 = 0, c2 = 0, stat = 0;
  if (l < V) {  // per-ring counts and status, one lane a ring
    const int32_t* rc = B.r_counts + ((size_t)s * V + l) * 4;
    c0 = rc[0]; c1 = rc[1]; c2 = rc[2];
    stat = B.r_status[(size_t)s * V + l];
  }
  const int o0 = wave_sum(l < r ? c0 : 0), o1 = wave_sum(l < r ? c1 : 0), o2 = wave_sum(l < r ? c2 : 0);
  const int n0 = __shfl(c0, r), n1 = __shfl(c1, r), n2 = __shfl(c2, r);
  if (r == 0) {
    const int a0 = wave_sum(c0), a1 = wave_sum(c1), a2 = wave_sum(c2), status = wave_or(stat);
    if (l == 0) {
      int32_t* cnt = B.counts + (size_t)s * CNT_N;
      cnt[CNT_SHARP] = a0; cnt[CNT_LSHARP] = a1; cnt[CNT_FLAT] = a2;
      cnt[CNT_STATUS] = status;
      int32_t* fc = B.fcnt + ((size_t)P.par * P.S + s) * 4;  // k_lm's copy, slot P.par
      fc[0] = a0; fc[1] = a1; fc[2] = a2; fc[3] = status;
      B.fe_state[2 * s + 1] += 1;  // read by the next scan's front end (adjustOutlierCloud)
    }
  }
  // feature clouds into slot P.par: k_lm of this scan may run after the next scans' k_concat
  const size_t hs = (size_t)P.par * P.S + s;
  {  // ring-ordered concatenation
    const size_t rb = (size_t)s * V + r;
    for (int t = l; t < n0; t += 64) {
      B.f_sharp[hs * V * P.cap_sharp + o0 + t] = B.r_sharp[rb * P.cap_sharp + t];
      B.f_sharp_ind[hs * V * P.cap_sharp + o0 + t] = B.r_sharp_ind[rb * P.cap_sharp + t];
    }
    for (int t = l; t < n1; t += 64) {
      B.f_lsharp[hs * V * P.cap_lsharp + o1 + t] = B.r_lsharp[rb * P.cap_lsharp + t];
      B.f_lsharp_ind[hs * V * P.cap_lsharp + o1 + t] = B.r_lsharp_ind[rb * P.cap_lsharp + t];
    }
    for (int t = l; t < n2; t += 64) {
      B.f_flat[hs * V * P.cap_flat + o2 + t] = B.r_flat[rb * P.cap_flat + t];
      B.f_flat_ind[hs * V * P.cap_flat + o2 + t] = B.r_flat_ind[rb * P.cap_flat + t];
    }
  }
  // surfPointsLessFlatScan of the ring (:370-374) into staging slot P.par: the
  // VoxelGrid (k_voxel) reads only this copy, so it may overlap the next scan's front end
  ScanView v;
  v.M = B.counts[(size_t)s * CNT_N + CNT_M];
  v.VH = P.VH;
  v.flabel = B.flabel + (size_t)s * P.VH;
  const float4* fa = B.seg_fa + (size_t)s * P.VH;
  const int lane = lane_id();
  // The six segments [sp, ep] of a ring tile [st, en'] without gaps (ep_j + 1 = sp_{j+1}); segments
  // with sp >= ep are skipped (their positions are not lessFlat candidates).  Eight chunks of 64
  // positions per batch: label loads issued together, point loads buffer-masked.
  const __amdgpu_buffer_rsrc_t rs_fa = buffer_rsrc(fa, (uint32_t)P.VH * 16u);
  {
    const size_t rb = (size_t)s * V + r;
    const size_t sb = (size_t)P.par * P.S * V + rb;
    float4* dst = B.lf_stage + sb * P.H;
    const int st = B.ring_start[rb], en = B.ring_end[rb];
    int nlist = 0;
    for (int j = 0; j < 6; j++) {
      const int sp = (st * (6 - j) + en * j) / 6;
      const int ep = (st * (5 - j) + en * (j + 1)) / 6 - 1;
      if (sp >= ep) continue;
      for (int k0 = sp; k0 <= ep; k0 += 64 * 8) {
        int8_t lab[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) lab[u] = v.flabel[min(k0 + 64 * u + lane, ep)];
        float4 pt[8];
        bool pr[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int k = k0 + 64 * u + lane;
          pr[u] = k <= ep && lab[u] <= 0;
          pt[u] = buffer_load_f4(rs_fa, pr[u] ? (uint32_t)k * 16u : 0xffffffffu);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const unsigned long long m = __ballot(pr[u]);
          if (pr[u]) dst[nlist + popc_below(m)] = pt[u];
          nlist += __popcll(m);
        }
      }
    }
    if (lane == 0) B.lf_count[sb] = nlist;
  }
}


// ============================================================================================
// k_lm: updateTransformation + integrateTransformation + publishOdometry + publishCloudsLast
// ============================================================================================
// k_lm<threads, queries>: 768 / 1536 in general, 512 / 384 for VLP-16-sized feature sets (lg_launch_lm)
#define GRID_MAX 8191  // grid cells (end offsets share LDS with the staged small cloud)
#define CGRID_MAX 2047  // grid cells over a staged small cloud

// TransformToStart / TransformToEnd (:388-471) in either libm model (Fp<kF1>, lego_libm.h): the
// unqualified sin / cos on float angles, the expression evaluated in T = float (fp_mode 0) or double
// (fp_mode 1) and rounded where the reference stores it to float.
template <bool kF1>
LG_DEVICE float4 transform_to_start(const float4 pi, const float* cur) {  // :388-418
  typedef Fp<kF1> F;
  typedef typename F::T T;
  float s = 10 * (pi.w - (float)(int)pi.w);
  float ry = s * cur[1];
  float rx = s * cur[0];
  float rz = s * cur[2];
  float tx = s * cur[3];
  float ty = s * cur[4];
  float tz = s * cur[5];
  const T crz = F::cs(rz), srz = F::sn(rz), crx = F::cs(rx), srx = F::sn(rx), cry = F::cs(ry), sry = F::sn(ry);
  float x1 = crz * (T)(pi.x - tx) + srz * (T)(pi.y - ty);
  float y1 = -srz * (T)(pi.x - tx) + crz * (T)(pi.y - ty);
  float z1 = (pi.z - tz);
  float x2 = x1;
  float y2 = crx * (T)y1 + srx * (T)z1;
  float z2 = -srx * (T)y1 + crx * (T)z1;
  return make_float4((float)(cry * (T)x2 - sry * (T)z2), y2, (float)(sry * (T)x2 + cry * (T)z2), pi.w);
}

// cos / sin of transformCur's rotation for TransformToEnd's second half (constant per scan)
template <bool kF1>
struct EndTrig {
  typename Fp<kF1>::T cx, sx, cy, sy, cz, sz;
};
template <bool kF1>
LG_DEVICE EndTrig<kF1> end_trig(const float* cur) {
  typedef Fp<kF1> F;
  return EndTrig<kF1>{F::cs(cur[0]), F::sn(cur[0]), F::cs(cur[1]), F::sn(cur[1]), F::cs(cur[2]), F::sn(cur[2])};
}
template <bool kF1>
LG_DEVICE float4 transform_to_end_t(const float4 pi, const float* cur, const EndTrig<kF1>& E) {  // :422-471
  typedef Fp<kF1> F;
  typedef typename F::T T;
  float s = 10 * (pi.w - (float)(int)pi.w);
  float rx = s * cur[0];
  float ry = s * cur[1];
  float rz = s * cur[2];
  float tx = s * cur[3];
  float ty = s * cur[4];
  float tz = s * cur[5];
  T c, sn;
  c = F::cs(rz); sn = F::sn(rz);
  float x1 = c * (T)(pi.x - tx) + sn * (T)(pi.y - ty);
  float y1 = -sn * (T)(pi.x - tx) + c * (T)(pi.y - ty);
  float z1 = (pi.z - tz);
  c = F::cs(rx); sn = F::sn(rx);
  float x2 = x1;
  float y2 = c * (T)y1 + sn * (T)z1;
  float z2 = -sn * (T)y1 + c * (T)z1;
  c = F::cs(ry); sn = F::sn(ry);
  float x3 = c * (T)x2 - sn * (T)z2;
  float y3 = y2;
  float z3 = sn * (T)x2 + c * (T)z2;
  tx = cur[3]; ty = cur[4]; tz = cur[5];
  float x4 = E.cy * (T)x3 + E.sy * (T)z3;
  float y4 = y3;
  float z4 = -E.sy * (T)x3 + E.cy * (T)z3;
  float x5 = x4;
  float y5 = E.cx * (T)y4 - E.sx * (T)z4;
  float z5 = E.sx * (T)y4 + E.cx * (T)z4;
  float x6 = E.cz * (T)x5 - E.sz * (T)y5 + (T)tx;
  float y6 = E.sz * (T)x5 + E.cz * (T)y5 + (T)ty;
  float z6 = z5 + tz;
  return make_float4(x6, y6, z6, (float)(int)pi.w);
}

// Eigen boundary model, identical to the oracle's: ColPivHouseholderQR<Matrix3f>::solve in float.
LG_DEVICE void qr_solve3(const float* A_in, const float* b_in, float* x) {
  // Fully unrolled with every array index a compile-time constant (pivot swaps and the rank-limited
  // loops become guarded static accesses), so the factorisation stays in registers.  The floating-
  // point operations and their order are unchanged.
  float A[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) A[i] = A_in[i];
  const float eps = FLT_EPSILON;
  float nu[3], nd[3], hc[3];
  int perm[3] = {0, 1, 2};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < 3; ++r) s += A[r * 3 + k] * A[r * 3 + k];
    nu[k] = nd[k] = sqrtf(s);
  }
  float maxn = fmaxf(nu[0], fmaxf(nu[1], nu[2]));
  float th_help = (maxn * eps) * (maxn * eps) / 3.0f;
  float ndt = sqrtf(eps);
  int nzp = 3;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    int bc = k;
    float bv = nu[k];
#pragma unroll
    for (int j = k + 1; j < 3; ++j)
      if (nu[j] > bv) { bc = j; bv = nu[j]; }
    float bsq = bv * bv;
    if (nzp == 3 && bsq < th_help * float(3 - k)) nzp = k;
#pragma unroll
    for (int j = k + 1; j < 3; ++j) {
      if (bc == j) {
#pragma unroll
        for (int r = 0; r < 3; ++r) { float t = A[r * 3 + k]; A[r * 3 + k] = A[r * 3 + j]; A[r * 3 + j] = t; }
        float t = nu[k]; nu[k] = nu[j]; nu[j] = t;
        t = nd[k]; nd[k] = nd[j]; nd[j] = t;
        int ti = perm[k]; perm[k] = perm[j]; perm[j] = ti;
      }
    }
    float tail = 0.f;
#pragma unroll
    for (int r = k + 1; r < 3; ++r) tail += A[r * 3 + k] * A[r * 3 + k];
    float c0 = A[k * 3 + k], tau, beta;
    if (tail <= FLT_MIN) {
      tau = 0.f; beta = c0;
#pragma unroll
      for (int r = k + 1; r < 3; ++r) A[r * 3 + k] = 0.f;
    } else {
      beta = sqrtf(c0 * c0 + tail);
      if (c0 >= 0.f) beta = -beta;
#pragma unroll
      for (int r = k + 1; r < 3; ++r) A[r * 3 + k] = A[r * 3 + k] / (c0 - beta);
      tau = (beta - c0) / beta;
    }
    hc[k] = tau;
    A[k * 3 + k] = beta;
    if (tau != 0.f) {
#pragma unroll
      for (int j = k + 1; j < 3; ++j) {
        float t = A[k * 3 + j];
#pragma unroll
        for (int r = k + 1; r < 3; ++r) t += A[r * 3 + k] * A[r * 3 + j];
        A[k * 3 + j] -= tau * t;
#pragma unroll
        for (int r = k + 1; r < 3; ++r) A[r * 3 + j] -= tau * A[r * 3 + k] * t;
      }
    }
#pragma unroll
    for (int j = k + 1; j < 3; ++j) {
      if (nu[j] != 0.f) {
        float t = fabsf(A[k * 3 + j]) / nu[j];
        t = (1.f + t) * (1.f - t);
        if (t < 0.f) t = 0.f;
        float q = nu[j] / nd[j];
        float t2 = t * q * q;
        if (t2 <= ndt) {
          float s = 0.f;
#pragma unroll
          for (int r = k + 1; r < 3; ++r) s += A[r * 3 + j] * A[r * 3 + j];
          nd[j] = sqrtf(s);
          nu[j] = nd[j];
        } else {
          nu[j] *= sqrtf(t);
        }
      }
    }
  }
  float c[3] = {b_in[0], b_in[1], b_in[2]};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (k >= nzp || hc[k] == 0.f) continue;
    float t = c[k];
#pragma unroll
    for (int r = k + 1; r < 3; ++r) t += A[r * 3 + k] * c[r];
    c[k] -= hc[k] * t;
#pragma unroll
    for (int r = k + 1; r < 3; ++r) c[r] -= hc[k] * A[r * 3 + k] * t;
  }
  float y[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 2; i >= 0; --i) {
    if (i >= nzp) continue;
    float t = c[i];
#pragma unroll
    for (int j = i + 1; j < 3; ++j)
      if (j < nzp) t -= A[i * 3 + j] * y[j];
    y[i] = t / A[i * 3 + i];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int m = 0; m < 3; ++m)
      if (perm[i] == m) x[m] = y[i];
  }
}

__device__ __attribute__((noinline)) double eig_max_sym3(const float* Af) {  // (cold: out of line)
  double a[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) a[i][j] = Af[i * 3 + j];
  for (int sweep = 0; sweep < 32; ++sweep) {
    double off = a[0][1] * a[0][1] + a[0][2] * a[0][2] + a[1][2] * a[1][2];
    if (off == 0.0) break;
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int q = p + 1; q < 3; ++q) {
        if (a[p][q] == 0.0) continue;
        double theta = (a[q][q] - a[p][p]) / (2.0 * a[p][q]);
        double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < 3; ++k) {
          double akp = a[k][p], akq = a[k][q];
          a[k][p] = c * akp - s * akq;
          a[k][q] = s * akp + c * akq;
        }
        for (int k = 0; k < 3; ++k) {
          double apk = a[p][k], aqk = a[q][k];
          a[p][k] = c * apk - s * aqk;
          a[q][k] = s * apk + c * aqk;
        }
      }
  }
  return fmax(a[0][0], fmax(a[1][1], a[2][2]));
}

// eig_max_sym3(A) < thr, decided without the Jacobi sweeps when the bounds settle it: for a
// symmetric A, max_i a_ii <= lambda_max <= max_i sum_j |a_ij| (Rayleigh quotient / Gershgorin).  The
// margin (1e-12 of the Frobenius norm) is far above the sweeps' rounding error, so the decision is
// the sweeps' decision; anything closer (or non-finite) runs them.
LG_DEVICE bool lambda_max_below(const float* Af, double thr) {
  double maxd = -1e300, gers = 0.0, fro = 0.0;
  for (int i = 0; i < 3; ++i) {
    double row = 0.0;
    for (int j = 0; j < 3; ++j) {
      const double v = Af[i * 3 + j];
      row += fabs(v);
      fro += v * v;
    }
    maxd = fmax(maxd, (double)Af[i * 4]);
    gers = fmax(gers, row);
  }
  const double tol = 1e-12 * sqrt(fro);
  if (isfinite(fro)) {
    if (maxd - tol > thr) return false;
    if (gers + tol < thr) return true;
  }
  return eig_max_sym3(Af) < thr;
}

#define LM_LAST_LDS 2048  // Last clouds up to this size (the corner cloud) are searched in LDS
#define LM_RMAX 72        // ring values -1 .. 70 (V <= 64)
template <int kMaxQ>
struct LmLdsT {  // kMaxQ: feature queries of one loop (V * max(cap_sharp, cap_flat))
  union {
    float4 lastc[LM_LAST_LDS];  // small Last cloud, staged
    int gcell[GRID_MAX + 1];    // larger cloud: uniform grid, end offset of every cell in grid_pts
  } u;
  float gmin[3], gcs;
  int gdim[3];
  int cgcell[CGRID_MAX + 1];  // grid cell table of a staged small cloud
  int grid_ring_ok;  // every grid record carries its ring ((int)w in [-1, 70])
  int grid_r;        // search radius in cells
  float4 sel[kMaxQ];
  float4 featl[kMaxQ];  // the loop's feature points (pointOri), staged once
  float4 plane[kMaxQ];  // surf: each correspondence's plane, once per search
  int ind1[kMaxQ], ind2[kMaxQ], ind3[kMaxQ];
  int first_ge[LM_RMAX + 4];  // first index with ring >= r (index r + 1), nl if none
  int last_le[LM_RMAX + 4];   // last index with ring <= r (index r + 1), -1 if none
  int nfall;                  // queries whose ring breaks need the sequential scan
  int fall[kMaxQ];
  int ntie;                   // queries of this search with an exact 1-NN distance tie
  int tieq[kMaxQ];
  int kd_built;               // nanoflann's tree of this loop's Last cloud is in B.kd_*
  int kd_n;                   // that cloud's size
  float kd_box[6];            // its root bbox
  lgkd::KdView kdv;           // the tree's scratch (B.kd_* of this stream) and cloud
  float fred[6][16];
  int iscan[16];
  float cur[6];
  int flag;      // 1 = keep iterating
  int iters;     // iterations run by the loop so far
  int status;
  int skip;
#ifdef LG_PROFILE
  unsigned long long plog[8];  // k_lm's per-scan phase log (profile build): build / search / iterations a loop
#endif
};

// candidate key compare: (dist, rank) lexicographic = sequential strict-< scan order
LG_DEVICE bool key_lt(float d1, int r1, float d2, int r2) { return d1 < d2 || (d1 == d2 && r1 < r2); }
LG_DEVICE void wave_argmin(float& d, int& r, int& idx) {
  for (int o = 32; o > 0; o >>= 1) {
    float d2 = __shfl_xor(d, o);
    int r2 = __shfl_xor(r, o), i2 = __shfl_xor(idx, o);
    if (key_lt(d2, r2, d, r)) { d = d2; r = r2; idx = i2; }
  }
}

// ---- kd-tree 1-NN (nanoflann_pcl.h:141-152) as an exact uniform-grid search --------------------
// The reference only uses the nearest neighbour when its squared distance is < 25
// (nearest_feature_search_distance^2, fa.cpp:516,654).  With cells >= 1.1 x that radius, every
// point closer than the radius lies in the query's 3x3x3 cell neighbourhood, so the grid returns
// the brute-force result -- the lowest index among exact distance ties (pinned against nanoflann by
// tests/test_oracle_cpu.py) -- whenever it is accepted, and "not accepted" otherwise.
template <class Lds>
LG_DEVICE int block_excl_scan_int(Lds& L, int v, int& total) {
  const int lane = lane_id(), w = wave_id();
  int x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) L.iscan[w] = x;
  __syncthreads();
  int off = 0, tot = 0;
  for (int k = 0; k < (int)(blockDim.x >> 6); ++k) {
    if (k < w) off += L.iscan[k];
    tot += L.iscan[k];
  }
  total = tot;
  __syncthreads();
  return off + x - v;
}

// ---- correspondence search over the Last cloud ------------------------------------------------
// The reference's searches only use points closer than nearest_feature_search_distance (5 m):
// the 1-NN is used only when d^2 < 25 (fa.cpp:516,654) and the 2nd / 3rd points of the ring-limited
// scans (:514-564, 652-713) start from the bound 25 with strict <.  So both searches are exact over
// the points inside a 5 m ball around the query, in the reference's own order keys:
//   1-NN: (d, lowest index) -- the brute-force answer, pinned against nanoflann (see grid_nn note);
//   scans: the forward scan visits j = closest+1 .. up to the first ring break (or the bound), the
//          backward scan closest-1 .. down to its break; (d, visit rank) lexicographic = the
//          sequential strict-< scans.  The break positions come from per-ring first / last indices.
// Small Last clouds (the corner cloud) are staged in LDS and scanned whole; larger ones (the surf
// cloud) are bucketed into an (x, y) column grid with cells of c = 5.01/3 m, so the 5 m ball is a
// handful of contiguous runs of columns.

// f(j, last[j]) over the whole Last cloud, block-wide, 8 loads in flight per lane; lanes of a wave
// hold consecutive j.
template <typename F>
LG_DEVICE void for_last_batched(const float4* __restrict__ last, int nl, F f) {
  for (int j0 = threadIdx.x; j0 < nl; j0 += (int)blockDim.x * 8) {
    float4 p[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) p[u] = last[min(j0 + u * (int)blockDim.x, nl - 1)];
#pragma unroll
    for (int u = 0; u < 8; ++u) f(j0 + u * (int)blockDim.x, p[u]);  // j may be >= nl: f checks
  }
}

LG_DEVICE int ring_of(float w) { return min(max((int)w + 1, 0), LM_RMAX - 1); }  // index of ring (int)w

// first_ge / last_le from the Last cloud's rings (block-wide); ring(j) = (int)last[j].w.  Only the
// positions where the ring value changes can be a ring's first / last index.
template <class Lds>
LG_DEVICE void ring_index(Lds& L, const float4* last, int nl) {
  const int tid = threadIdx.x;
  for (int r = tid; r < LM_RMAX + 4; r += (int)blockDim.x) { L.first_ge[r] = nl; L.last_le[r] = -1; }
  __syncthreads();
  for (int j0 = tid; j0 < nl; j0 += (int)blockDim.x * 4) {
    float w[4], wp[4], wn[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = j0 + u * (int)blockDim.x;
      w[u] = last[min(j, nl - 1)].w;
      wp[u] = last[min(max(j - 1, 0), nl - 1)].w;
      wn[u] = last[min(j + 1, nl - 1)].w;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = j0 + u * (int)blockDim.x;
      const int r = ring_of(w[u]);
      if (j < nl && (j == 0 || ring_of(wp[u]) != r)) atomicMin(&L.first_ge[r], j);
      if (j < nl && (j == nl - 1 || ring_of(wn[u]) != r)) atomicMax(&L.last_le[r], j);
    }
  }
  __syncthreads();
  if (tid == 0) {  // suffix min / prefix max
    for (int r = LM_RMAX - 2; r >= 0; --r) L.first_ge[r] = min(L.first_ge[r], L.first_ge[r + 1]);
    for (int r = 1; r < LM_RMAX; ++r) L.last_le[r] = max(L.last_le[r], L.last_le[r - 1]);
  }
  __syncthreads();
}

LG_DEVICE int grid_coord(float v, float mn, float cs, int dim) {
  float f = floorf((v - mn) / cs);
  f = fminf(fmaxf(f, -2.f), (float)dim + 1.f);
  return (int)f;
}

template <class Lds>
LG_DEVICE void build_grid(Lds& L, const float4* __restrict__ last, int nl, float4* gp, float cs0, int* gcell,
                           int maxcells) {
  const int tid = threadIdx.x;
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for_last_batched(last, nl, [&](int j, const float4 p) {
    if (j >= nl) return;
    mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
    mx[0] = fmaxf(mx[0], p.x); mx[1] = fmaxf(mx[1], p.y); mx[2] = fmaxf(mx[2], p.z);
  });
  for (int d = 0; d < 3; ++d) {
    const float a = wave_min(mn[d]), b = wave_max(mx[d]);
    if (lane_id() == 0) { L.fred[d][wave_id()] = a; L.fred[3 + d][wave_id()] = b; }
  }
  __syncthreads();
  if (tid == 0) {
    float lo[3], hi[3];
    for (int d = 0; d < 3; ++d) {
      lo[d] = L.fred[d][0]; hi[d] = L.fred[3 + d][0];
      for (int w = 1; w < (int)(blockDim.x >> 6); ++w) { lo[d] = fminf(lo[d], L.fred[d][w]); hi[d] = fmaxf(hi[d], L.fred[3 + d][w]); }
      if (nl == 0) { lo[d] = 0.f; hi[d] = 0.f; }
    }
    float cs = cs0;
    int dim[3];
    while (true) {
      long long tot = 1;
      for (int d = 0; d < 3; ++d) { dim[d] = (int)((hi[d] - lo[d]) / cs) + 1; tot *= dim[d]; }
      if (tot <= maxcells) break;
      cs *= 2.f;
    }
    for (int d = 0; d < 3; ++d) { L.gmin[d] = lo[d]; L.gdim[d] = dim[d]; }
    L.gcs = cs;
    L.grid_r = cs >= 3.f * cs0 ? 1 : cs >= 1.5f * cs0 ? 2 : 3;  // grid_r * cs >= 3 * cs0 = 5.01 m
    L.grid_ring_ok = 1;
  }
  __syncthreads();
  const int ncell = L.gdim[0] * L.gdim[1] * L.gdim[2];
  for (int c = tid; c <= ncell; c += (int)blockDim.x) gcell[c] = 0;
  __syncthreads();
  for_last_batched(last, nl, [&](int j, const float4 p) {
    if (j >= nl) return;
    const int cx = min(max(grid_coord(p.x, L.gmin[0], L.gcs, L.gdim[0]), 0), L.gdim[0] - 1);
    const int cy = min(max(grid_coord(p.y, L.gmin[1], L.gcs, L.gdim[1]), 0), L.gdim[1] - 1);
    const int cz = min(max(grid_coord(p.z, L.gmin[2], L.gcs, L.gdim[2]), 0), L.gdim[2] - 1);
    atomicAdd(&gcell[(cz * L.gdim[1] + cy) * L.gdim[0] + cx], 1);
  });
  __syncthreads();
  // exclusive scan of the counts -> cell start offsets (each thread a contiguous chunk)
  const int per = (ncell + (int)blockDim.x - 1) / (int)blockDim.x;
  const int c0 = min(tid * per, ncell), c1 = min(c0 + per, ncell);
  int local = 0;
  for (int c = c0; c < c1; ++c) local += gcell[c];
  int tot;
  int run = block_excl_scan_int(L, local, tot);
  for (int c = c0; c < c1; ++c) {
    const int n = gcell[c];
    gcell[c] = run;
    run += n;
  }
  __syncthreads();
  // scatter; afterwards gcell[c] = end of cell c = start of cell c+1
  for_last_batched(last, nl, [&](int j, const float4 p) {
    if (j >= nl) return;
    const int cx = min(max(grid_coord(p.x, L.gmin[0], L.gcs, L.gdim[0]), 0), L.gdim[0] - 1);
    const int cy = min(max(grid_coord(p.y, L.gmin[1], L.gcs, L.gdim[1]), 0), L.gdim[1] - 1);
    const int cz = min(max(grid_coord(p.z, L.gmin[2], L.gcs, L.gdim[2]), 0), L.gdim[2] - 1);
    const int slot = atomicAdd(&gcell[(cz * L.gdim[1] + cy) * L.gdim[0] + cx], 1);
    const int rp = (p.w > -2.f && p.w < (float)(LM_RMAX - 1)) ? (int)p.w + 1 : 0;  // (int)w in [-1, 70]
    if (!(p.w > -2.f && p.w < (float)(LM_RMAX - 1))) L.grid_ring_ok = 0;
    gp[slot] = make_float4(p.x, p.y, p.z, __int_as_float(j | (rp << 24)));
  });
  __syncthreads();
}

// Squared distance from q to grid cell (cx, cy, cz), the box shrunk by 1 mm against the rounding of
// the points' cell coordinates: no point of the cell is closer.
template <class Lds>
LG_DEVICE float cell_boxd2(const Lds& L, float4 q, int cx, int cy, int cz) {
  const float cs = L.gcs;
  const float qv[3] = {q.x, q.y, q.z};
  const int cv[3] = {cx, cy, cz};
  float d2 = 0.f;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const float lo = L.gmin[a] + (float)cv[a] * cs, hi = lo + cs;
    float e = fmaxf(fmaxf(lo - qv[a], qv[a] - hi), 0.f);
    e = fmaxf(e - 1e-3f, 0.f);
    d2 += e * e;
  }
  return d2;
}

// Visit the grid cells around q in shells of Chebyshev radius k = 0 .. L.grid_r (cells of size cs
// with grid_r * cs >= 5.01 m, so every point closer than the 5 m search radius is inside): a cell
// whose box lies farther than the lane's bound() is skipped, and shell k ends the search once
// (k - 1) * cs exceeds it, since none of those points can improve or tie the lane's best.  Bounds
// are per lane: a lane skips only its own share of a cell's points, each of which is farther than
// that lane's best and so farther than the group's final best.  tpq adjacent lanes share a query:
// lane `sub` takes every tpq-th point of a cell.  f(point) per candidate.
template <typename B, typename F, class Lds>
LG_DEVICE void grid_visit_pruned(const Lds& L, const int* gcell, const float4* __restrict__ gp, float4 q, int sub,
                                 int tpq, bool act,
                                 B bound, F f) {
  if (!act) return;
  const int R = L.grid_r;
  int qc[3];
  const float qv[3] = {q.x, q.y, q.z};
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const float t = floorf((qv[a] - L.gmin[a]) / L.gcs);
    qc[a] = (int)fminf(fmaxf(t, (float)(-R - 1)), (float)(L.gdim[a] + R));
  }
  for (int k = 0; k <= R; ++k) {
    if (k >= 2) {
      const float e = (float)(k - 1) * L.gcs - 1e-3f;
      if (e * e > bound()) break;
    }
    for (int dz = -k; dz <= k; ++dz)
      for (int dy = -k; dy <= k; ++dy)
        for (int dx = -k; dx <= k; ++dx) {
          if (max(abs(dx), max(abs(dy), abs(dz))) != k) continue;
          const int cx = qc[0] + dx, cy = qc[1] + dy, cz = qc[2] + dz;
          if (cx < 0 || cx >= L.gdim[0] || cy < 0 || cy >= L.gdim[1] || cz < 0 || cz >= L.gdim[2]) continue;
          if (k > 0 && cell_boxd2(L, q, cx, cy, cz) > bound()) continue;
          const int c = (cz * L.gdim[1] + cy) * L.gdim[0] + cx;
          const int b = c == 0 ? 0 : gcell[c - 1], e = gcell[c];
          int j = b + sub;
          for (; j + 3 * tpq < e; j += 4 * tpq) {
            float4 p4[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) p4[u] = gp[j + u * tpq];
#pragma unroll
            for (int u = 0; u < 4; ++u) f(p4[u]);
          }
          for (; j < e; j += tpq) f(gp[j]);
        }
  }
}

LG_DEVICE float group_min(float v, int tpq) {
  for (int o = tpq >> 1; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o));
  return v;
}

// 1-NN of q (index or -1 when none is closer than the radius) with the tie flag, tpq lanes a query.
// Inactive lanes (act = false) only join the shuffles.
template <class Lds>
LG_DEVICE int grid_nn(const Lds& L, const int* gcell, const float4* __restrict__ gp, float4 q, float r2, bool& tie,
                      int sub,
                      int tpq, bool act) {
  float bd = FLT_MAX;
  int bi = 0x7fffffff, bc = 0;
  grid_visit_pruned(L, gcell, gp, q, sub, tpq, act,
                    [&]() { return fminf(bd, r2); },
                    [&](const float4 p) {
                      const float dx = q.x - p.x, dy = q.y - p.y, dz = q.z - p.z;
                      const float d = dx * dx + dy * dy + dz * dz;  // nanoflann L2_Simple_Adaptor order
                      const int idx = __float_as_int(p.w) & 0xffffff;
                      if (d < bd) { bd = d; bi = idx; bc = 1; }
                      else if (d == bd) { bc++; bi = min(bi, idx); }
                    });
  for (int o = tpq >> 1; o > 0; o >>= 1) {
    const float d2 = __shfl_xor(bd, o);
    const int i2 = __shfl_xor(bi, o), c2 = __shfl_xor(bc, o);
    if (d2 < bd) { bd = d2; bi = i2; bc = c2; }
    else if (d2 == bd) { bi = min(bi, i2); bc += c2; }
  }
  tie = (bd < r2) && bc > 1;
  return (bd < r2) ? bi : -1;
}

// One wave: the reference's ring-limited linear scans for the 2nd (and 3rd) correspondence around
// the accepted nearest neighbour `closest` (fa.cpp:514-564, 652-713).  surf = plane (3 points),
// else line (2 points).
__device__ __attribute__((noinline)) void ring_scans(const LgParams& P, const float4* __restrict__ last, int nl, float4 sel, int fwd_bound,
                          bool surf, int closest, int& o2, int& o3, int& status) {
  const int lane = lane_id();
  o2 = -1; o3 = -1;
  const int ring0 = (int)last[closest].w;
  // rank -1: a candidate at exactly the initial bound is not taken (the reference's strict <)
  float b2d = P.nn_dist_sqr, b3d = P.nn_dist_sqr;
  int b2r = -1, b3r = -1, b2i = -1, b3i = -1;
  int bound = fwd_bound;  // reference bug: bounded by the current feature count (:522, :661)
  if (bound > nl) {
    if (closest + 1 < bound) status |= LEGO_ST_FWD_OOB;
    bound = nl;
  }
  auto consider = [&](int j, int rj, const float4 p, int rank, bool fwd) {
    const float d = (p.x - sel.x) * (p.x - sel.x) + (p.y - sel.y) * (p.y - sel.y) + (p.z - sel.z) * (p.z - sel.z);
    if (surf) {
      if (fwd ? rj <= ring0 : rj >= ring0) { if (key_lt(d, rank, b2d, b2r)) { b2d = d; b2r = rank; b2i = j; } }
      else { if (key_lt(d, rank, b3d, b3r)) { b3d = d; b3r = rank; b3i = j; } }
    } else if (fwd ? rj > ring0 : rj < ring0) {
      if (key_lt(d, rank, b2d, b2r)) { b2d = d; b2r = rank; b2i = j; }
    }
  };
  // forward j = closest+1 .. (bound), 4 chunks of 64 loaded at once; stop at the first ring break
  for (int base = closest + 1; base < bound; base += 256) {
    float4 p4[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = base + 64 * u + lane;
      p4[u] = (j < bound) ? last[j] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    bool stop = false;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (stop) break;
      const int j = base + 64 * u + lane;
      const bool valid = j < bound;
      const int rj = valid ? (int)p4[u].w : 0;
      const bool brk = valid && (double)rj > (double)ring0 + 2.5;
      const unsigned long long bm = __ballot(brk);
      const int fb = bm ? __ffsll((long long)bm) - 1 : 64;
      if (valid && lane < fb) consider(j, rj, p4[u], j - closest, true);
      if (bm || base + 64 * (u + 1) >= bound) stop = true;
    }
    if (stop) break;
  }
  // backward j = closest-1 .. 0
  for (int top = closest - 1; top >= 0; top -= 256) {
    float4 p4[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = top - 64 * u - lane;
      p4[u] = (j >= 0) ? last[j] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    bool stop = false;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (stop) break;
      const int j = top - 64 * u - lane;
      const bool valid = j >= 0;
      const int rj = valid ? (int)p4[u].w : 0;
      const bool brk = valid && (double)rj < (double)ring0 - 2.5;
      const unsigned long long bm = __ballot(brk);
      const int fb = bm ? __ffsll((long long)bm) - 1 : 64;
      if (valid && lane < fb) consider(j, rj, p4[u], (1 << 24) + (closest - j), false);
      if (bm || top - 64 * (u + 1) < 0) stop = true;
    }
    if (stop) break;
  }
  wave_argmin(b2d, b2r, b2i);
  o2 = b2i;
  if (surf) {
    wave_argmin(b3d, b3r, b3i);
    o3 = b3i;
  }
}

// AtA/AtB -> solve -> degeneracy -> update of cur (registers; every lane of the wave computes the
// same); returns keep-iterating
LG_DEVICE bool lm_solve_reg(float* cur, int& is_degenerate, int& status, const double* red, int iter, bool surf) {
  float AtA[9], AtB[3], x[3];
  AtA[0] = (float)red[0]; AtA[1] = (float)red[1]; AtA[2] = (float)red[2];
  AtA[3] = AtA[1]; AtA[4] = (float)red[3]; AtA[5] = (float)red[4];
  AtA[6] = AtA[2]; AtA[7] = AtA[5]; AtA[8] = (float)red[5];
  AtB[0] = (float)red[6]; AtB[1] = (float)red[7]; AtB[2] = (float)red[8];
  qr_solve3(AtA, AtB, x);
  if (iter == 0) {
    is_degenerate = lambda_max_below(AtA, 10.0);
  } else if (is_degenerate) {
    status |= LEGO_ST_DEGEN_UB;
  }
  if (is_degenerate) {
    status |= LEGO_ST_DEGENERATE;
    x[0] = x[1] = x[2] = 0.f;
  }
  const float RAD2DEG = (float)(180.0 / M_PI);
  float deltaR, deltaT;
  if (surf) {
    cur[0] += x[0]; cur[2] += x[1]; cur[4] += x[2];
  } else {
    cur[1] += x[0]; cur[3] += x[1]; cur[5] += x[2];
  }
  for (int i = 0; i < 6; i++)
    if (isnan(cur[i])) cur[i] = 0;
  if (surf) {
    double a = (double)(RAD2DEG * x[0]), b = (double)(RAD2DEG * x[1]);
    deltaR = (float)sqrt(a * a + b * b);
    double c = (double)(x[2] * 100);
    deltaT = (float)sqrt(c * c);
  } else {
    double a = (double)(RAD2DEG * x[0]);
    deltaR = (float)sqrt(a * a);
    double b = (double)(x[1] * 100), c = (double)(x[2] * 100);
    deltaT = (float)sqrt(b * b + c * c);
  }
  return !((double)deltaR < 0.1 && (double)deltaT < 0.1);
}

// sin / cos of transformCur's rotation, computed once per iteration (the reference computes them
// once per calculateTransformation* call, outside its row loop)
struct LmTrig {
  float srx, crx, sry, cry, srz, crz, tx, ty, tz;
};
template <bool kF1>
LG_DEVICE LmTrig lm_trig(const float* cur) {  // float srx = sin(transformCur[0]) (:797-802, :939-944)
  typedef Fp<kF1> F;
  LmTrig t;
  t.srx = (float)F::sn(cur[0]); t.crx = (float)F::cs(cur[0]); t.sry = (float)F::sn(cur[1]);
  t.cry = (float)F::cs(cur[1]); t.srz = (float)F::sn(cur[2]); t.crz = (float)F::cs(cur[2]);
  t.tx = cur[3]; t.ty = cur[4]; t.tz = cur[5];
  return t;
}

LG_DEVICE void accumulate_surf_row(const LmTrig& T, const float4 po, const float4 cf, double* acc) {
  // calculateTransformationSurf :797-857 (per-row Jacobian)
  const float srx = T.srx, crx = T.crx, sry = T.sry, cry = T.cry, srz = T.srz, crz = T.crz;
  const float tx = T.tx, ty = T.ty, tz = T.tz;
  float a1 = crx * sry * srz;
  float a2 = crx * crz * sry;
  float a3 = srx * sry;
  float a4 = tx * a1 - ty * a2 - tz * a3;
  float a5 = srx * srz;
  float a6 = crz * srx;
  float a7 = ty * a6 - tz * crx - tx * a5;
  float a8 = crx * cry * srz;
  float a9 = crx * cry * crz;
  float a10 = cry * srx;
  float a11 = tz * a10 + ty * a9 - tx * a8;
  float b1 = -crz * sry - cry * srx * srz;
  float b2 = cry * crz * srx - sry * srz;
  float b5 = cry * crz - srx * sry * srz;
  float b6 = cry * srz + crz * srx * sry;
  float c1 = -b6;
  float c2 = b5;
  float c3 = tx * b6 - ty * b5;
  float c4 = -crx * crz;
  float c5 = crx * srz;
  float c6 = ty * c5 + tx * -c4;
  float c7 = b2;
  float c8 = -b1;
  float c9 = tx * -b2 - ty * -b1;
  float arx = (-a1 * po.x + a2 * po.y + a3 * po.z + a4) * cf.x + (a5 * po.x - a6 * po.y + crx * po.z + a7) * cf.y +
              (a8 * po.x - a9 * po.y - a10 * po.z + a11) * cf.z;
  float arz = (c1 * po.x + c2 * po.y + c3) * cf.x + (c4 * po.x - c5 * po.y + c6) * cf.y + (c7 * po.x + c8 * po.y + c9) * cf.z;
  float aty = -b6 * cf.x + c4 * cf.y + b2 * cf.z;
  float bb = (float)(-0.05 * (double)cf.w);
  const float a[3] = {arx, arz, aty};
  acc[0] += (double)(a[0] * a[0]); acc[1] += (double)(a[0] * a[1]); acc[2] += (double)(a[0] * a[2]);
  acc[3] += (double)(a[1] * a[1]); acc[4] += (double)(a[1] * a[2]); acc[5] += (double)(a[2] * a[2]);
  acc[6] += (double)(a[0] * bb); acc[7] += (double)(a[1] * bb); acc[8] += (double)(a[2] * bb);
  acc[9] += 1.0;
}

LG_DEVICE void accumulate_corner_row(const LmTrig& T, const float4 po, const float4 cf, double* acc) {
  // calculateTransformationCorner :939-977
  const float srx = T.srx, crx = T.crx, sry = T.sry, cry = T.cry, srz = T.srz, crz = T.crz;
  const float tx = T.tx, ty = T.ty, tz = T.tz;
  float b1 = -crz * sry - cry * srx * srz;
  float b2 = cry * crz * srx - sry * srz;
  float b3 = crx * cry;
  float b4 = tx * -b1 + ty * -b2 + tz * b3;
  float b5 = cry * crz - srx * sry * srz;
  float b6 = cry * srz + crz * srx * sry;
  float b7 = crx * sry;
  float b8 = tz * b7 - ty * b6 - tx * b5;
  float c5 = crx * srz;
  float ary = (b1 * po.x + b2 * po.y - b3 * po.z + b4) * cf.x + (b5 * po.x + b6 * po.y - b7 * po.z + b8) * cf.z;
  float atx = -b5 * cf.x + c5 * cf.y + b1 * cf.z;
  float atz = b7 * cf.x - srx * cf.y - b3 * cf.z;
  float bb = (float)(-0.05 * (double)cf.w);
  const float a[3] = {ary, atx, atz};
  acc[0] += (double)(a[0] * a[0]); acc[1] += (double)(a[0] * a[1]); acc[2] += (double)(a[0] * a[2]);
  acc[3] += (double)(a[1] * a[1]); acc[4] += (double)(a[1] * a[2]); acc[5] += (double)(a[2] * a[2]);
  acc[6] += (double)(a[0] * bb); acc[7] += (double)(a[1] * bb); acc[8] += (double)(a[2] * bb);
  acc[9] += 1.0;
}

// coefficient of one correspondence (surf: plane :721-776, corner: line :571-635); returns accepted.
// The plane through the three Last points (:721-731) depends only on the correspondence, so it is
// computed once per search (surf_plane) and re-used by the iterations until the next search.
LG_DEVICE float4 surf_plane(const float4* last, int i1, int i2, int i3) {
  const float4 t1 = last[i1], t2 = last[i2], t3 = last[i3];
  float pa = (t2.y - t1.y) * (t3.z - t1.z) - (t3.y - t1.y) * (t2.z - t1.z);
  float pb = (t2.z - t1.z) * (t3.x - t1.x) - (t3.z - t1.z) * (t2.x - t1.x);
  float pc = (t2.x - t1.x) * (t3.y - t1.y) - (t3.x - t1.x) * (t2.y - t1.y);
  float pd = -(pa * t1.x + pb * t1.y + pc * t1.z);
  float ps = sqrtf(pa * pa + pb * pb + pc * pc);
  pa /= ps; pb /= ps; pc /= ps; pd /= ps;
  return make_float4(pa, pb, pc, pd);
}
template <bool kF1>
LG_DEVICE bool surf_coeff_pl(const float4 pl, float4 sel, int iter, float4& cf) {
  typedef Fp<kF1> F;
  typedef typename F::T T;
  const float pa = pl.x, pb = pl.y, pc = pl.z, pd = pl.w;
  float pd2 = pa * sel.x + pb * sel.y + pc * sel.z + pd;
  float s = 1;
  if (iter >= 5)  // :761: sqrt(sqrt(float sum)) in T
    s = (float)(1 - 1.8 * (double)fabsf(pd2) / (double)F::sq(F::sq((T)(sel.x * sel.x + sel.y * sel.y + sel.z * sel.z))));
  if ((double)s > 0.1 && pd2 != 0) {
    cf = make_float4(s * pa, s * pb, s * pc, s * pd2);
    return true;
  }
  return false;
}

LG_DEVICE bool corner_coeff(const float4* last, int i1, int i2, float4 sel, int iter, float4& cf) {
  if (!(i2 >= 0)) return false;
  const float4 tp1 = last[i1], tp2 = last[i2];
  float x0 = sel.x, y0 = sel.y, z0 = sel.z;
  float x1 = tp1.x, y1 = tp1.y, z1 = tp1.z;
  float x2 = tp2.x, y2 = tp2.y, z2 = tp2.z;
  float m11 = ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1));
  float m22 = ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1));
  float m33 = ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1));
  float a012 = sqrtf(m11 * m11 + m22 * m22 + m33 * m33);
  float l12 = sqrtf((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2));
  float la = ((y1 - y2) * m11 + (z1 - z2) * m22) / a012 / l12;
  float lb = -((x1 - x2) * m11 - (z1 - z2) * m33) / a012 / l12;
  float lc = -((x1 - x2) * m22 + (y1 - y2) * m33) / a012 / l12;
  float ld2 = a012 / l12;
  float s = 1;
  if (iter >= 5) s = (float)(1 - 1.8 * (double)fabsf(ld2));
  if ((double)s > 0.1 && ld2 != 0) {
    cf = make_float4(s * la, s * lb, s * lc, s * ld2);
    return true;
  }
  return false;
}

// The 2nd / 3rd correspondence of one query from candidate points, in the sequential scans' order
// keys (ring_scans): forward candidates closest < j < fe, backward be < j < closest.
struct ScanBest {
  float d2, d3;
  int r2, r3, i2, i3;
  LG_DEVICE void init(float bound) { d2 = d3 = bound; r2 = r3 = -1; i2 = i3 = -1; }
  LG_DEVICE void visit(float4 sel, float4 p, int j, int rj, int closest, int ring0, int fe, int be, bool surf) {
    bool fwd;
    if (j > closest && j < fe) fwd = true;
    else if (j < closest && j > be) fwd = false;
    else return;
    const int rank = fwd ? j - closest : (1 << 24) + (closest - j);
    const float d = (p.x - sel.x) * (p.x - sel.x) + (p.y - sel.y) * (p.y - sel.y) + (p.z - sel.z) * (p.z - sel.z);
    if (surf) {
      if (fwd ? rj <= ring0 : rj >= ring0) { if (key_lt(d, rank, d2, r2)) { d2 = d; r2 = rank; i2 = j; } }
      else { if (key_lt(d, rank, d3, r3)) { d3 = d; r3 = rank; i3 = j; } }
    } else if (fwd ? rj > ring0 : rj < ring0) {
      if (key_lt(d, rank, d2, r2)) { d2 = d; r2 = rank; i2 = j; }
    }
  }
  LG_DEVICE void merge(int tpq) {
    for (int o = tpq >> 1; o > 0; o >>= 1) {
      float d = __shfl_xor(d2, o);
      int r = __shfl_xor(r2, o), i = __shfl_xor(i2, o);
      if (key_lt(d, r, d2, r2)) { d2 = d; r2 = r; i2 = i; }
      d = __shfl_xor(d3, o); r = __shfl_xor(r3, o); i = __shfl_xor(i3, o);
      if (key_lt(d, r, d3, r3)) { d3 = d; r3 = r; i3 = i; }
    }
  }
  LG_DEVICE void take(const ScanBest& o) {
    if (key_lt(o.d2, o.r2, d2, r2)) { d2 = o.d2; r2 = o.r2; i2 = o.i2; }
    if (key_lt(o.d3, o.r3, d3, r3)) { d3 = o.d3; r3 = o.r3; i3 = o.i3; }
  }
};

// Scan ends around `closest`: fe = first j > closest with ring >= ring0 + 3 (the break, :522-524 /
// :661-663) or the bound; be = last j < closest with ring <= ring0 - 3, or -1.  False when the
// per-ring first / last indices cannot decide (a ring value out of order by 3 or more: never for
// the intensity-derived rings, kept exact by the sequential fallback).
template <class Lds>
LG_DEVICE bool scan_ends(const Lds& L, int closest, int ring0, int bound, int& fe, int& be) {
  const int tf = ring0 + 3 + 1, tb = ring0 - 3 + 1;
  bool ok = true;
  fe = bound;
  if (closest + 1 < bound && tf >= 0 && tf < LM_RMAX) {
    const int f = L.first_ge[tf];
    if (f > closest) fe = min(f, bound);
    else ok = false;
  } else if (closest + 1 < bound && tf < 0) {
    ok = false;
  }
  be = -1;
  if (closest > 0 && tb >= 0) {
    const int g = tb < LM_RMAX ? L.last_le[tb] : closest;
    if (g < closest) be = g;
    else ok = false;
  }
  return ok;
}

// Brute-force exact 1-NN over a Last cloud staged in LDS (small clouds: the corner cloud): the
// (d, lowest index) minimum and the tie count over all points equal the grid search's (and so
// nanoflann's) whenever the neighbour is accepted (d < r2).  tpq lanes per query, merged by xor
// shuffles as in grid_nn.
LG_DEVICE int lds_nn(const float4* last, int nl, float4 q, float r2, bool& tie, int sub, int tpq, bool act) {
  float bd = FLT_MAX;
  int bi = 0x7fffffff, bc = 0;
  if (act)
    for (int j = sub; j < nl; j += tpq) {
      const float4 p = last[j];
      const float dx = q.x - p.x, dy = q.y - p.y, dz = q.z - p.z;
      const float d = dx * dx + dy * dy + dz * dz;  // nanoflann L2_Simple_Adaptor order
      if (d < bd) { bd = d; bi = j; bc = 1; }
      else if (d == bd) { bc++; bi = min(bi, j); }
    }
  for (int o = tpq >> 1; o > 0; o >>= 1) {
    const float d2 = __shfl_xor(bd, o);
    const int i2 = __shfl_xor(bi, o), c2 = __shfl_xor(bc, o);
    if (d2 < bd) { bd = d2; bi = i2; bc = c2; }
    else if (d2 == bd) { bi = min(bi, i2); bc += c2; }
  }
  tie = (bd < r2) && bc > 1;
  return (bd < r2) ? bi : -1;
}

// ============================================================================================
// nanoflann's kd-tree, for the rare 1-NN with an exact distance tie (lego_kdtree.h)
// ============================================================================================
// Scratch per stream: B.kd_* (built once per LM loop, on demand).
using namespace lgkd;

// Re-resolve the tied queries L.tieq[0, L.ntie) with nanoflann's tree (built on first use in this LM
// loop).  Wave 0 only; the caller synchronises the workgroup around it.
// (out of line, each piece on its own: k_lm's register budget sets its co-residence with the front end)
__device__ __attribute__((noinline)) int kd_build_nl(const KdView* K, int n, float* box) { return kd_build(*K, n, box); }
__device__ __attribute__((noinline)) int kd_nn1_nl(const KdView* K, const float* box, float4 q, bool* ovf) {
  const int cap = (10 * K->vh) / (5 * 64);  // search frames per lane
  float d;
  int c;
  kd_knn<1>(*K, box, q, K->frames + (size_t)lane_id() * cap * 5, cap, &c, &d, *ovf);
  return c;
}
template <class Lds>
__device__ __attribute__((noinline)) void kd_resolve_ties(Lds& L) {
  if (!L.kd_built) {
    if (kd_build_nl(&L.kdv, L.kd_n, L.kd_box) < 0) {  // a build-stack overflow keeps the grid's lowest indices
      if (lane_id() == 0) atomicOr(&L.status, LEGO_ST_TIE_UNRESOLVED);
      return;
    }
    if (lane_id() == 0) L.kd_built = 1;
  }
  bool unres = false;
  for (int k0 = 0; k0 < L.ntie; k0 += 64) {
    const int k = k0 + lane_id();
    if (k < L.ntie) {
      const int q = L.tieq[k];
      bool ovf = false;
      const int c = kd_nn1_nl(&L.kdv, L.kd_box, L.sel[q], &ovf);
      if (!ovf) L.ind1[q] = c;  // (a stack overflow keeps the grid's lowest index)
      unres |= ovf;
    }
  }
  if (__ballot(unres) != 0ull && lane_id() == 0) atomicOr(&L.status, LEGO_ST_TIE_UNRESOLVED);
}

// one LM loop (surf or corner), <= 25 iterations.  The correspondence search (iterations 0, 5, 10,
// 15, 20) uses the whole workgroup; the other iterations only re-weight the same correspondences
// with the updated transform, so wave 0 runs each block of up to 5 iterations on its own
// (coefficients, a butterfly reduction that leaves the normal equations in every lane, the 3x3 solve
// in registers) and the workgroup meets once per block instead of three times per iteration.
template <bool kF1, class Lds>
LG_DEVICE void lm_loop(const LgParams& P, Lds& L, LgState& S, const float4* __restrict__ feat, int nq,
                       const float4* __restrict__ last_g, int nl, bool surf, float4* gp, int& iters) {
  const int tid = threadIdx.x;
  const int nw = (int)(blockDim.x >> 6);
  const bool small = nl <= LM_LAST_LDS;
  PROF_T(t_bg0);
  for (int q = tid; q < nq; q += (int)blockDim.x) L.featl[q] = feat[q];  // read back by the same thread first
  if (small) {
    for (int j = tid; j < nl; j += (int)blockDim.x) L.u.lastc[j] = last_g[j];
    __syncthreads();
  }
  // uniform grid for the 1-NN: the surf cloud's cell table takes the LDS of the staged small cloud;
  // a small (staged) cloud gets a coarser table of its own
  int* gcell = small ? L.cgcell : L.u.gcell;
  // A staged cloud of at most half the staging area keeps its grid-ordered copy in the other half, so its
  // 1-NN walks read LDS instead of global memory (the corner cloud: ~450 points, four or five searches a
  // loop); the grid itself is the same.
  const bool gl = small && nl <= LM_LAST_LDS / 2;
  float4* gpl = L.u.lastc + LM_LAST_LDS / 2;
  if (gl)
    build_grid(L, (const float4*)L.u.lastc, nl, gpl, (sqrtf(P.nn_dist_sqr) + 0.01f) / 3.f, gcell, CGRID_MAX);
  else
    build_grid(L, small ? (const float4*)L.u.lastc : last_g, nl, gp, (sqrtf(P.nn_dist_sqr) + 0.01f) / 3.f, gcell,
               small ? CGRID_MAX : GRID_MAX);
  const float4* last = small ? (const float4*)L.u.lastc : last_g;
  ring_index(L, last, nl);
  PROF_ADD(surf ? 16 : 48, t_bg0);
  PROF_LM(surf ? 0 : 1, t_bg0);
  if (tid == 0) { L.iters = 0; L.kd_built = 0; L.kdv.pts = last; L.kd_n = nl; }
  for (int iter = 0; iter < 25; iter += 5) {
    {  // search (all waves)
      float cur[6];
      for (int k = 0; k < 6; ++k) cur[k] = L.cur[k];
      PROF_T(t_sel0);
      for (int q = tid; q < nq; q += (int)blockDim.x) L.sel[q] = transform_to_start<kF1>(L.featl[q], cur);
      __syncthreads();
      PROF_ADD(8, t_sel0);
      PROF_T(t_srch0);
      PROF_T(t_nn0);
      int st = 0;
      // as many lanes per query as the block allows (8, 4, 2 or 1); with 512 threads (VLP-16) the
      // surf ~170 and corner ~115 queries get 2 and 4 lanes, with 768 threads both get 4
      const int tpq = nq * 8 <= (int)blockDim.x ? 8 : nq * 4 <= (int)blockDim.x ? 4 : nq * 2 <= (int)blockDim.x ? 2 : 1;
      if (tid == 0) { L.nfall = 0; L.ntie = 0; }
      for (int base = 0; base < nq * tpq; base += (int)blockDim.x) {
        const int t = base + tid, q = t / tpq, sub = t % tpq;
        const bool act = q < nq;
        bool tie = false;
        const float4 qs = act ? L.sel[q] : make_float4(0.f, 0.f, 0.f, 0.f);
        int c;
        if (gl) c = grid_nn(L, gcell, (const float4*)gpl, qs, P.nn_dist_sqr, tie, sub, tpq, act);
        else c = grid_nn(L, gcell, gp, qs, P.nn_dist_sqr, tie, sub, tpq, act);
        if (act && sub == 0) {
          L.ind1[q] = c;
          if (tie) {
            st |= LEGO_ST_NN_TIE;
            L.tieq[atomicAdd(&L.ntie, 1)] = q;
          }
        }
      }
      __syncthreads();
      if (L.ntie > 0) {  // exact ties: nanoflann's choice (its first visited point), from its tree
        if (wave_id() == 0) kd_resolve_ties(L);
        __syncthreads();
      }
      PROF_ADD(surf ? 37 : 46, t_nn0);
      PROF_T(t_rs0);
      // ring-limited 2nd / 3rd points (fa.cpp:514-564, 652-713).  Larger clouds: one wave per query
      // over the index ranges the per-ring first / last indices give, 8 loads in flight per lane.
      // (Visiting the 1-NN grid's cells instead, tpq lanes a query pruned by the lanes' bests, is exact
      // too but measured slower: 251k vs 271k scans/s, 239k with the staged clouds as well.)
      if (!small) for (int q = wave_id(); q < nq; q += nw) {
        const int c = L.ind1[q];
        int o2 = -1, o3 = -1;
        if (c >= 0) {
          const float4 qs = L.sel[q];
          const int ring0 = (int)last[c].w;
          int bound = nq;  // reference bug: bounded by the current feature count (:522, :661)
          if (bound > nl) {
            if (c + 1 < bound) st |= LEGO_ST_FWD_OOB;
            bound = nl;
          }
          int fe, be;
          if (scan_ends(L, c, ring0, bound, fe, be)) {
            ScanBest sb;
            sb.init(P.nn_dist_sqr);
            const int je = max(fe, c);
            int j = be + 1 + lane_id();
            for (; j + 7 * 64 < je; j += 8 * 64) {
              float4 p8[8];
#pragma unroll
              for (int u = 0; u < 8; ++u) p8[u] = last[j + 64 * u];
#pragma unroll
              for (int u = 0; u < 8; ++u) sb.visit(qs, p8[u], j + 64 * u, (int)p8[u].w, c, ring0, fe, be, surf);
            }
            for (; j < je; j += 64) {
              const float4 p = last[j];
              sb.visit(qs, p, j, (int)p.w, c, ring0, fe, be, surf);
            }
            sb.merge(64);
            o2 = sb.i2;
            o3 = surf ? sb.i3 : -1;
          } else {
            ring_scans(P, last, nl, qs, nq, surf, c, o2, o3, st);
          }
        }
        if (lane_id() == 0) { L.ind2[q] = o2; L.ind3[q] = o3; }
      }
      // smaller clouds: tpq lanes a query
      if (small) for (int base = 0; base < nq * tpq; base += (int)blockDim.x) {
        const int t = base + tid, q = t / tpq, sub = t % tpq;
        const bool act = q < nq;
        const float4 qs = act ? L.sel[q] : make_float4(0.f, 0.f, 0.f, 0.f);
        const int closest = act ? L.ind1[q] : -1;
        ScanBest sb;
        sb.init(P.nn_dist_sqr);
        bool run = closest >= 0;
        int fe = 0, be = 0, ring0 = 0;
        if (run) {
          ring0 = (int)last[closest].w;
          int bound = nq;  // reference bug: bounded by the current feature count (:522, :661)
          if (bound > nl) {
            if (closest + 1 < bound) st |= LEGO_ST_FWD_OOB;
            bound = nl;
          }
          if (!scan_ends(L, closest, ring0, bound, fe, be)) {
            run = false;
            if (sub == 0) L.fall[atomicAdd(&L.nfall, 1)] = q;
          }
        }
        if (run)
          for (int j = be + 1 + sub, je = max(fe, closest); j < je; j += tpq)
            sb.visit(qs, last[j], j, (int)last[j].w, closest, ring0, fe, be, surf);
        sb.merge(tpq);
        if (act && sub == 0 && (closest < 0 || run)) { L.ind2[q] = sb.i2; L.ind3[q] = surf ? sb.i3 : -1; }
      }
      __syncthreads();
      // sequential scans for the queries the per-ring indices could not decide (one wave each)
      for (int k = wave_id(); k < L.nfall; k += nw) {
        const int q = L.fall[k];
        int o2 = -1, o3 = -1;
        ring_scans(P, last, nl, L.sel[q], nq, surf, L.ind1[q], o2, o3, st);
        if (lane_id() == 0) { L.ind2[q] = o2; L.ind3[q] = o3; }
      }
      st = wave_or(st);
      if (lane_id() == 0 && st) atomicOr(&L.status, st);
      __syncthreads();
      if (surf) {
        for (int q = tid; q < nq; q += (int)blockDim.x)
          if (L.ind2[q] >= 0 && L.ind3[q] >= 0) L.plane[q] = surf_plane(last, L.ind1[q], L.ind2[q], L.ind3[q]);
        __syncthreads();
      }
      PROF_ADD(surf ? 38 : 47, t_rs0);
      PROF_ADD(9, t_srch0);
      PROF_LM(surf ? 2 : 3, t_srch0);
    }
    PROF_T(t_acc0);
    if (wave_id() == 0) {  // iterations iter .. iter + 4 on wave 0
      const int lane = lane_id();
      float cur[6];
      for (int k = 0; k < 6; ++k) cur[k] = L.cur[k];
      int deg = S.is_degenerate, status = 0, it = iter, run = L.iters;
      bool keep = true;
      for (; it < iter + 5 && it < 25; ++it) {
        PROF_T(t_i0);
        const LmTrig T = lm_trig<kF1>(cur);
        double acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int q = lane; q < nq; q += 64) {
          const float4 po = L.featl[q];
          const float4 sel = it == iter ? L.sel[q] : transform_to_start<kF1>(po, cur);
          float4 cf;
          const bool ok = surf ? (L.ind2[q] >= 0 && L.ind3[q] >= 0 && surf_coeff_pl<kF1>(L.plane[q], sel, it, cf))
                               : corner_coeff(last, L.ind1[q], L.ind2[q], sel, it, cf);
          if (ok) {
            if (surf) accumulate_surf_row(T, po, cf, acc);
            else accumulate_corner_row(T, po, cf, acc);
          }
        }
        PROF_ADD(surf ? 40 : 41, t_i0);
        PROF_T(t_i1);
#pragma unroll
        for (int k = 0; k < 10; ++k)
          for (int o = 32; o > 0; o >>= 1) acc[k] += __shfl_xor(acc[k], o);
        PROF_ADD(42, t_i1);
        PROF_T(t_i2);
        run = it + 1;
        if (acc[9] < 10.0) continue;  // too few correspondences: `continue`
        const bool go = lm_solve_reg(cur, deg, status, acc, it, surf);
        PROF_ADD(43, t_i2);
#ifdef LG_PROFILE
        if (lane_id() == 0) atomicAdd(&PROF_SLOT(surf ? 44 : 45), 1ull);
#endif
        if (!go) { keep = false; break; }
      }
      if (lane == 0) {
        for (int k = 0; k < 6; ++k) L.cur[k] = cur[k];
        S.is_degenerate = deg;
        if (status) L.status |= status;
        L.iters = run;
        L.flag = keep ? 1 : 0;
      }
    }
    __syncthreads();
    PROF_ADD(10, t_acc0);
    PROF_LM(surf ? 4 : 5, t_acc0);
    if (!L.flag) break;
  }
  iters = L.iters;
  __syncthreads();
}

// ============================================================================================
// k_publish: the lessFlat half of publishCloudsLast (:1329-1383): concatenate the rings' VoxelGrid
// outputs (surfPointsLessFlat) and TransformToEnd them into laserCloudSurfLast with the transform
// k_lm has just produced (untransformed on the initialisation scan, :1181-1209).  Runs after both
// k_lm and k_voxel of its scan, before the next scan's k_lm.
// ============================================================================================
// One wave a ring (grid S * V, 64-lane workgroups): a workgroup of a whole scan needed 16 wave slots of
// one CU at once and waited behind the VoxelGrid / segmentation waves for most of their duration (the
// trace showed 450-700 us a launch for < 20 us of work), with the next k_lm queued behind it.
template <bool kF1>
__global__ __launch_bounds__(64) void k_publish(LgParams P, LgBufs B) {
  const int V = P.V, VH = P.VH;
  const int s = P.s0 + blockIdx.x / V, r = blockIdx.x % V, lane = lane_id();
  const size_t hb = ((size_t)P.par * P.S + s) * V;  // k_voxel's output slot of this scan
  const int c = lane < V ? B.r_vcount[hb + lane] : 0;
  const int o = wave_sum(lane < r ? c : 0);  // the ring's offset: the lessFlat rings in ring order
  const int n_lflat = wave_sum(c);
  const int n = __shfl(c, r);
  const LgState& S0 = B.state[s];
  float c6[6];
  for (int k = 0; k < 6; ++k) c6[k] = S0.cur[k];
  const int copy = S0.pub_copy, nb = S0.last_buf;
  const EndTrig<kF1> E = end_trig<kF1>(c6);
  float4* sl = B.surf_last + (size_t)s * 2 * VH + (size_t)nb * VH;
  float4* fl = B.f_lflat + (size_t)s * VH;
  const float4* src = B.r_lflat + (hb + r) * P.H;
  for (int t0 = lane; t0 < n; t0 += 64 * 4) {
    float4 p4[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) p4[u] = src[min(t0 + 64 * u, n - 1)];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int t = t0 + 64 * u;
      if (t < n) {
        fl[o + t] = p4[u];
        sl[o + t] = copy ? p4[u] : transform_to_end_t<kF1>(p4[u], c6, E);
      }
    }
  }
  if (r == 0) {
    const int st = wave_or(lane < V ? B.r_vstatus[hb + lane] : 0);
    if (lane == 0) {
      LgState& S = B.state[s];
      S.n_surf_last = n_lflat;
      S.tree_stale = copy ? 0 : !(S.n_corner_last > 10 && n_lflat > 100);
      S.status |= st;
      B.counts[(size_t)s * CNT_N + CNT_LFLAT] = n_lflat;
    }
  }
}

// The stream's per-scan odometry record (lego_batch_set_trajectory): transformCur and transformSum after
// this association (publishOdometry, :1286-1298, runs every scan), at the stream's association count.
LG_DEVICE void lm_record(const LgParams& P, const LgBufs& B, int s, LgState& S) {
  if (B.traj && S.n_assoc < P.traj_cap) {
    float* r = B.traj + ((size_t)s * P.traj_cap + S.n_assoc) * 12;
    for (int k = 0; k < 6; ++k) {
      r[k] = S.cur[k];
      r[6 + k] = S.sum[k];
    }
  }
  S.n_assoc++;
}

// integrateTransformation (:1241-1270): transformSum from transformCur (AccumulateRotation :474-500)
template <bool kF1>
__device__ __attribute__((noinline)) void integrate_transformation(const float* cur, float* sum) {
  typedef Fp<kF1> F;
  typedef typename F::T T;
  float cx = sum[0], cy = sum[1], cz = sum[2], lx = -cur[0], ly = -cur[1], lz = -cur[2];
  // AccumulateRotation (:474-500)
  const T clx = F::cs(lx), slx = F::sn(lx), cly = F::cs(ly), sly = F::sn(ly), clz = F::cs(lz), slz = F::sn(lz);
  const T ccx = F::cs(cx), scx = F::sn(cx), ccy = F::cs(cy), scy = F::sn(cy), ccz = F::cs(cz), scz = F::sn(cz);
  float srx = clx * ccx * sly * scz - ccx * ccz * slx - clx * cly * scx;
  float ox = -F::as(srx);
  float srycrx = slx * (ccy * scz - ccz * scx * scy) + clx * sly * (ccy * ccz + scx * scy * scz) + clx * cly * ccx * scy;
  float crycrx = clx * cly * ccx * ccy - clx * sly * (ccz * scy - ccy * scx * scz) - slx * (scy * scz + ccy * ccz * scx);
  const T cox = F::cs(ox);
  float oy = F::at2((T)srycrx / cox, (T)crycrx / cox);
  float srzcrx = scx * (clz * sly - cly * slx * slz) + ccx * scz * (cly * clz + slx * sly * slz) + clx * ccx * ccz * slz;
  float crzcrx = clx * clz * ccx * ccz - ccx * scz * (cly * slz - clz * slx * sly) - scx * (sly * slz + cly * clz * slx);
  float oz = F::at2((T)srzcrx / cox, (T)crzcrx / cox);
  float rx = ox, ry = oy, rz = oz;
  const T crz_ = F::cs(rz), srz_ = F::sn(rz), crx_ = F::cs(rx), srx_ = F::sn(rx), cry_ = F::cs(ry), sry_ = F::sn(ry);
  float x1 = crz_ * (T)(cur[3]) - srz_ * (T)(cur[4]);
  float y1 = srz_ * (T)(cur[3]) + crz_ * (T)(cur[4]);
  float z1 = cur[5];
  float x2 = x1;
  float y2 = crx_ * (T)y1 - srx_ * (T)z1;
  float z2 = srx_ * (T)y1 + crx_ * (T)z1;
  float tx = (T)sum[3] - (cry_ * (T)x2 + sry_ * (T)z2);
  float ty = sum[4] - y2;
  float tz = (T)sum[5] - (-sry_ * (T)x2 + cry_ * (T)z2);
  sum[0] = rx; sum[1] = ry; sum[2] = rz; sum[3] = tx; sum[4] = ty; sum[5] = tz;
}

// kWpe: waves a SIMD the compiler budgets registers for.  With more than half a scan a CU in flight the VLP-16
// layout (512 threads, two waves a SIMD) runs at 4 (128 VGPRs; 49-66 spilled to scratch in round 5, 11-12
// since round 6's out-of-line cold paths): 2 x 128 of a SIMD's 512 registers leave room for two VoxelGrid
// waves (105 VGPRs) beside it instead of one (155 VGPRs a wave otherwise, 177 in round 5): +0.9 % C3 order 0
// in the pipeline (238.1k -> 240.3k scans/s, three A/B pairs on one box), +4.2 % order 1 (295.6k -> 307.9k,
// two pairs) although k_lm alone is 5 % slower (0.53 -> 0.56 ms).  With fewer scans (C5's 80 sequences:
// 157.4k -> 148.1k) the LM's own speed counts: kWpe 1 and, since round 6, 1,024 threads (lg_launch_lm).  (The
// compiler drops a request the block's own LDS makes unreachable: 5 for this layout, 4 for 768 threads.)
template <int kNT, int kMaxQ, bool kF1, int kWpe>
__global__ __launch_bounds__(kNT) __attribute__((amdgpu_waves_per_eu(kWpe)))
void k_lm(LgParams P, LgBufs B) {
  __shared__ LmLdsT<kMaxQ> L;
  __shared__ LgState S;
  const int s = P.s0 + blockIdx.x, tid = threadIdx.x;
  const int V = P.V, VH = P.VH;
  // the scan's features: half P.par (k_concat), which the next scan's front end does not touch
  const size_t hs = (size_t)P.par * P.S + s;
  const int32_t* fc = B.fcnt + hs * 4;
  const int n_sharp = fc[0], n_lsharp = fc[1], n_flat = fc[2];
  const float4* f_sharp = B.f_sharp + hs * V * P.cap_sharp;
  const float4* f_lsharp = B.f_lsharp + hs * V * P.cap_lsharp;
  const float4* f_flat = B.f_flat + hs * V * P.cap_flat;
#ifdef LG_PROFILE
  const unsigned long long rt_lm0 = __builtin_amdgcn_s_memrealtime();
  if (tid < 8) L.plog[tid] = 0ull;
#endif
  if (tid == 0) {
    S = B.state[s];
    L.status = fc[3];
    for (int k = 0; k < 6; ++k) L.cur[k] = S.cur[k];
  }
  __syncthreads();
  const size_t cl_stride = (size_t)V * P.cap_lsharp, sl_stride = (size_t)VH;
  float4* corner_base = B.corner_last + (size_t)s * 2 * cl_stride;
  float4* surf_base = B.surf_last + (size_t)s * 2 * sl_stride;
  if (!S.initialized) {  // checkSystemInitialization (:1181-1209): Last = current, untransformed
    float4* cl = corner_base + (size_t)S.last_buf * cl_stride;
    for (int k = tid; k < n_lsharp; k += (int)blockDim.x) cl[k] = f_lsharp[k];
    if (tid == 0) {  // the lessFlat cloud follows in k_publish (untransformed)
      S.initialized = 1;
      S.pub_copy = 1;
      S.n_corner_last = n_lsharp;
      S.tree_stale = 0;
      S.status = L.status | LEGO_ST_INIT;
      S.iters_surf = S.iters_corner = 0;
      lm_record(P, B, s, S);
      B.state[s] = S;
    }
    return;
  }
  const float4* clast = corner_base + (size_t)S.last_buf * cl_stride;
  const float4* slast = surf_base + (size_t)S.last_buf * sl_stride;
  int it_s = 0, it_c = 0;
  // updateTransformation (:1213-1235)
  if (S.n_corner_last < 10 || S.n_surf_last < 100) {
    if (tid == 0) L.status |= LEGO_ST_LM_SKIPPED;
  } else {
    if (tid == 0 && S.tree_stale) L.status |= LEGO_ST_STALE_TREE;
    float4* gp = B.grid_pts + (size_t)s * VH;
    if (tid == 0) {  // the tie path's tree scratch (read after the loops' barriers)
      L.kdv.pts = nullptr;
      L.kdv.node = B.kd_node + (size_t)s * 2 * VH;
      L.kdv.vind = B.kd_vind + (size_t)s * VH;
      L.kdv.tmp = B.kd_tmp + (size_t)s * 2 * VH;
      L.kdv.frames = B.kd_frames + (size_t)s * 10 * VH;
      L.kdv.vh = VH;
    }
    PROF_T(t_ls0);
    lm_loop<kF1>(P, L, S, f_flat, n_flat, slast, S.n_surf_last, true, gp, it_s);
    PROF_ADD(17, t_ls0);
    PROF_T(t_lc0);
    lm_loop<kF1>(P, L, S, f_sharp, n_sharp, clast, S.n_corner_last, false, gp, it_c);
    PROF_ADD(18, t_lc0);
  }
  __syncthreads();
  // integrateTransformation (:1241-1270) + publishOdometry (:1286-1298), thread 0 (out of line: one lane's
  // chain of libm calls, which inlined set the kernel's register peak)
  if (tid == 0) {
    integrate_transformation<kF1>(L.cur, S.sum);
    for (int k = 0; k < 6; ++k) S.cur[k] = L.cur[k];
    // publishOdometry's quaternion (:1287-1294, tf::createQuaternionMsgFromRollPitchYaw in double) is
    // computed from transformSum on the host when the odometry is read (lego_frontend.hip odom_quat, glibc's
    // sin / cos)
    S.pos[0] = S.sum[3]; S.pos[1] = S.sum[4]; S.pos[2] = S.sum[5];
    S.iters_surf = it_s;
    S.iters_corner = it_c;
  }
  __syncthreads();
  // publishCloudsLast (:1329-1383): TransformToEnd into the other half of the Last double buffer
  // (the lessSharp half here; the lessFlat half is k_publish's, after the VoxelGrid)
  {
    float cur[6];
    for (int k = 0; k < 6; ++k) cur[k] = L.cur[k];
    const int nb = S.last_buf ^ 1;
    float4* cl = corner_base + (size_t)nb * cl_stride;
    const EndTrig<kF1> E = end_trig<kF1>(cur);
    for (int k = tid; k < n_lsharp; k += (int)blockDim.x) cl[k] = transform_to_end_t<kF1>(f_lsharp[k], cur, E);
  }
  __syncthreads();
  if (tid == 0) {
    S.last_buf ^= 1;
    S.pub_copy = 0;
    S.n_corner_last = n_lsharp;
    S.cycle++;
    if (S.cycle == P.map_div) {
      S.cycle = 0;
      L.status |= LEGO_ST_EMITTED;
    }
    S.status = L.status;
    lm_record(P, B, s, S);
    B.state[s] = S;
#ifdef LG_PROFILE
    if (blockIdx.x < 4096) {
      unsigned long long* lg = g_lm_log + (size_t)blockIdx.x * 16;
      lg[0] = rt_lm0;
      lg[1] = __builtin_amdgcn_s_memrealtime();
      for (int k = 0; k < 6; ++k) lg[2 + k] = L.plog[k];
      lg[8] = (unsigned)S.iters_surf; lg[9] = (unsigned)S.iters_corner;
      lg[10] = (unsigned)n_flat; lg[11] = (unsigned)n_sharp;
      lg[12] = (unsigned)S.n_surf_last; lg[13] = (unsigned)n_lsharp;
    }
#endif
  }
}

// ============================================================================================
// launchers
// ============================================================================================
#define LG_CHECK_LAUNCH()                                  \
  do {                                                     \
    hipError_t e_ = hipGetLastError();                     \
    if (e_ != hipSuccess) return LEGO_EDEVICE;             \
  } while (0)

bool lg_lds_projection(const LgParams& P) {
  return (size_t)(P.VH + 64 + 16 * PQ_CAP) * 4 <= 160 * 1024;
}
bool lg_lds_segment(const LgParams& P) {  // k_segment_lds packing
  return P.V <= 16 && P.VH <= SEG_VH_MAX && P.seg_valid_line <= SEG_DMAX;
}

int lg_launch_project(const LgParams& P, const LgBufs& B, int S, const float4* pts, const int64_t* offs,
                      const int32_t* cnts, hipStream_t st) {
  if (P.wide == 1) {  // (mode 2: the one-workgroup projection, the wide segmentation)
#ifndef LG_PW_SLICE
    if (S >= 64)
      hipLaunchKernelGGL(k_pw_scatter<4>, dim3((P.max_points + 4 * PW_PTS - 1) / (4 * PW_PTS), S), dim3(PW_NT), 0, st,
                         P, B, pts, offs, cnts);
    else
      hipLaunchKernelGGL(k_pw_scatter<1>, dim3((P.max_points + PW_PTS - 1) / PW_PTS, S), dim3(PW_NT), 0, st, P, B,
                         pts, offs, cnts);
    LG_CHECK_LAUNCH();
    if (P.V <= 16)
      hipLaunchKernelGGL((k_pw_columns<1, 128>), dim3((P.H + 127) / 128, S), dim3(128), 0, st, P, B, pts, offs, cnts);
    else if (P.V <= 32)
      hipLaunchKernelGGL((k_pw_columns<2, 256>), dim3((P.H + 127) / 128, S), dim3(256), 0, st, P, B, pts, offs, cnts);
    else
      hipLaunchKernelGGL((k_pw_columns<4, 256>), dim3((P.H + 63) / 64, S), dim3(256), 0, st, P, B, pts, offs, cnts);
#else
#ifndef LG_PWS_KU
#define LG_PWS_KU 8
#endif
    constexpr int kU = LG_PWS_KU, PS = PWS_NT * kU;
    const dim3 gs((P.max_points + PS - 1) / PS, S);
#ifndef LG_PWS_CPL
#define LG_PWS_CPL 1
#endif
    // band columns held: VLP-16's 2,048-point slices span ~100-175 columns, HDL-64E's ~30-40
    if (P.V <= 16) {
      hipLaunchKernelGGL((k_pw_slice<kU, 16, 192>), gs, dim3(PWS_NT), 0, st, P, B, pts, offs, cnts);
      LG_CHECK_LAUNCH();
      hipLaunchKernelGGL((k_pw_fix<1, 128, LG_PWS_CPL>), dim3((P.H + 128 * LG_PWS_CPL - 1) / (128 * LG_PWS_CPL), S), dim3(128), 0, st, P, B, pts, offs, cnts);
    } else if (P.V <= 32) {
      hipLaunchKernelGGL((k_pw_slice<kU, 32, 96>), gs, dim3(PWS_NT), 0, st, P, B, pts, offs, cnts);
      LG_CHECK_LAUNCH();
      hipLaunchKernelGGL((k_pw_fix<2, 256, LG_PWS_CPL>), dim3((P.H + 128 * LG_PWS_CPL - 1) / (128 * LG_PWS_CPL), S), dim3(256), 0, st, P, B, pts, offs, cnts);
    } else {
      hipLaunchKernelGGL((k_pw_slice<kU, 64, 48>), gs, dim3(PWS_NT), 0, st, P, B, pts, offs, cnts);
      LG_CHECK_LAUNCH();
      hipLaunchKernelGGL((k_pw_fix<4, 256, LG_PWS_CPL>), dim3((P.H + 64 * LG_PWS_CPL - 1) / (64 * LG_PWS_CPL), S), dim3(256), 0, st, P, B, pts, offs, cnts);
    }
#endif
  } else {  // !wide implies the LDS images fit (lego_batch_set_wide)
    size_t sm = (size_t)(P.VH + 64 + 16 * PQ_CAP) * 4;
    hipLaunchKernelGGL(k_project, dim3(S), dim3(1024), sm, st, P, B, pts, offs, cnts);
  }
  LG_CHECK_LAUNCH();
  return LEGO_OK;
}

int lg_launch_segment(const LgParams& P, const LgBufs& B, int S, hipStream_t st) {
  if (P.wide) {  // modes 1 and 2: both projections leave the same range / cloud / ground images, 2-D scan
                 // candidates and orientation, which are all the k_sw_* kernels read
    const dim3 g((P.VH + SW_TILE - 1) / SW_TILE, S);
    const dim3 g2((P.H + SW_TC - 1) / SW_TC, (P.V + SW_TR - 1) / SW_TR, S);
    hipLaunchKernelGGL(k_sw_local, g2, dim3(SW_NT), 0, st, P, B);
    LG_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_sw_bound, g2, dim3(SW_NT), 0, st, P, B);
    LG_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_sw_roots, g, dim3(SW_NT), 0, st, P, B);
    LG_CHECK_LAUNCH();
    if (g.x > SW_MAX_TILES) return LEGO_EINVAL;  // (unreachable for validated parameters)
    hipLaunchKernelGGL(k_sw_count, g, dim3(SW_NT), 0, st, P, B);  // counts + the tile-local root ranks
    LG_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_sw_emit, g, dim3(SW_NT), 0, st, P, B);
    LG_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_sw_finish<1024>, dim3(S), dim3(1024), 0, st, P, B, (int)g.x);
  } else {
    size_t sm = (size_t)64 * 4 + (((size_t)P.VH * 2 + 3) & ~(size_t)3);
    hipLaunchKernelGGL(k_segment_lds, dim3(S), dim3(1024), sm, st, P, B);
  }
  LG_CHECK_LAUNCH();
  return LEGO_OK;
}

int lg_launch_fa_prep(const LgParams& P, const LgBufs& B, int S, hipStream_t st, bool distort) {
  if (distort) {
    hipLaunchKernelGGL((k_fa_prep<true, 1024>), dim3(S), dim3(1024), 0, st, P, B);
  } else {
    const int tiles = (P.VH + FP4_TILE - 1) / FP4_TILE;
    hipLaunchKernelGGL(k_fa_prep4, dim3(S, tiles), dim3(FP4_NT), 0, st, P, B);
  }
  LG_CHECK_LAUNCH();
  return LEGO_OK;
}

int lg_launch_extract(const LgParams& P, const LgBufs& B, int S, hipStream_t st) {
  hipLaunchKernelGGL(k_sortseg, dim3(S * P.V * 6), dim3(64), 0, st, P, B);
  LG_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_extract, dim3(S * (P.V + 1)), dim3(64), 0, st, P, B);
  LG_CHECK_LAUNCH();
  return LEGO_OK;
}

int lg_launch_voxel(const LgParams& P, const LgBufs& B, int S, hipStream_t st) {
  // At most one scan per CU (S <= ncu), one kernel for all rings: its register budget keeps its waves
  // off the SIMDs k_lm holds, which measured faster there.  With more scans than CUs the split
  // kernels (the common one at 83 VGPRs shares SIMDs with k_lm) measured faster: 245k vs 226k
  // scans/s at S = 512.
  // voxel_tie_order 0 takes the stack emulation: the level-synchronous sort (lvl_sort) has the lower
  // latency on one ring but more instructions, and in the pipeline, where the VoxelGrid shares the CUs
  // with k_lm and the next front end, it measured slower (C3: 143-151k / 164k vs 176-195k scans/s;
  // DESIGN §4).  It serves the map clouds (lego_s2m.hip).
  if (S <= P.ncu) {
    hipLaunchKernelGGL(k_voxel<3>, dim3(S * P.V), dim3(64), 0, st, P, B);
  } else if (P.voxel_stable) {
    hipLaunchKernelGGL(k_voxel<1>, dim3(S * P.V), dim3(64), 0, st, P, B);
    LG_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_voxel<2>, dim3(S * P.V), dim3(64), 0, st, P, B);
  } else {
    hipLaunchKernelGGL(k_voxel<0>, dim3(S * P.V), dim3(64), 0, st, P, B);
  }
  LG_CHECK_LAUNCH();
  return LEGO_OK;
}

int lg_launch_publish(const LgParams& P, const LgBufs& B, int S, hipStream_t st) {
  if (P.fp1)
    hipLaunchKernelGGL(k_publish<true>, dim3(S * P.V), dim3(64), 0, st, P, B);
  else
    hipLaunchKernelGGL(k_publish<false>, dim3(S * P.V), dim3(64), 0, st, P, B);
  LG_CHECK_LAUNCH();
  return LEGO_OK;
}

int lg_launch_concat(const LgParams& P, const LgBufs& B, int S, hipStream_t st) {
  hipLaunchKernelGGL(k_concat, dim3(S * P.V), dim3(64), 0, st, P, B);
  LG_CHECK_LAUNCH();
  return LEGO_OK;
}

int lg_launch_lm(const LgParams& P, const LgBufs& B, int S, hipStream_t st) {
  // VLP-16-sized feature sets (<= 384 queries a loop):
  //  * more than half a scan a CU in flight (C3's 256 streams): 512 threads compiled for four waves a SIMD
  //    (128 VGPRs, 68 KB of LDS), so two VoxelGrid waves share each of its SIMDs;
  //  * fewer (C5's shards, one scan in flight): each scan's LM latency sets the step, so 1,024 threads a
  //    scan — twice the waves for the per-query ring scans, searches and grid builds (round 6: +7-10 % at
  //    10-80 streams; 512 threads measured 0.581 vs 0.539 ms a step at 10 streams).
  // Larger sensors keep 768 threads and LDS for 1,536 queries.
  const bool vlp = P.V * std::max(P.cap_sharp, P.cap_flat) <= 384;
  const bool cap = 2 * S > P.ncu;
  if (vlp && cap && !P.fp1)
    hipLaunchKernelGGL((k_lm<512, 384, false, 4>), dim3(S), dim3(512), 0, st, P, B);
  else if (vlp && cap)
    hipLaunchKernelGGL((k_lm<512, 384, true, 4>), dim3(S), dim3(512), 0, st, P, B);
  else if (vlp && !P.fp1)
    hipLaunchKernelGGL((k_lm<1024, 384, false, 1>), dim3(S), dim3(1024), 0, st, P, B);
  else if (vlp)
    hipLaunchKernelGGL((k_lm<1024, 384, true, 1>), dim3(S), dim3(1024), 0, st, P, B);
  else if (!P.fp1)
    hipLaunchKernelGGL((k_lm<768, 1536, false, 1>), dim3(S), dim3(768), 0, st, P, B);
  else
    hipLaunchKernelGGL((k_lm<768, 1536, true, 1>), dim3(S), dim3(768), 0, st, P, B);
  LG_CHECK_LAUNCH();
  return LEGO_OK;
}

// ============================================================================================
// test hooks (declared in include/lego_frontend.h under "test hooks")
// ============================================================================================
__global__ void k_libm_test(const float* a, const float* b, float* out, int n, int which) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float r;
  if (which == 0) r = asinf_g(a[i]);
  else if (which == 1) r = atan2f_g(a[i], b[i]);
  else if (which == 2) r = atanf_g(a[i]);
  else if (which == 3) r = sqrtf(a[i]);
  else if (which == 4) r = a[i] / b[i];
  else if (which == 5) r = ground_pair(a[i], b[i] * b[i], 0.f, 0) ? 1.f : 0.f;              // fast + exact
  else if (which == 7) r = sinf_g(a[i]);
  else if (which == 8) r = cosf_g(a[i]);
  else if (which == 9) r = ground_pair(a[i], b[i] * b[i], 0.f, 1) ? 1.f : 0.f;              // fp_mode 1
  else if (which == 10) r = ground_pair_exact(a[i], b[i] * b[i], 0.f, 1) ? 1.f : 0.f;
  else r = ground_pair_exact(a[i], b[i] * b[i], 0.f, 0) ? 1.f : 0.f;                         // exact only
  out[i] = r;
}

int lg_derive_params(const lego_params& p, LgParams* out);  // lego_frontend.hip

__global__ void k_proj_test(LgParams P, const float4* pts, int n, int* fast, int* exact) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fast[i] = proj_cell_fast(P, pts[i]);
  exact[i] = proj_cell_exact(P, pts[i]);
}


// Projection cell of n points (x, y, z, w) by the fast path (-2 = undecided) and the exact path.
extern "C" int lego_test_project_cells(const lego_params* p, const float* h_xyzw, int32_t n, int32_t* h_fast,
                                       int32_t* h_exact) {
  if (!p || n <= 0 || !h_xyzw || !h_fast || !h_exact) return LEGO_EINVAL;
  LgParams P;
  int rc = lg_derive_params(*p, &P);
  if (rc) return rc;
  float4* d = nullptr;
  int *f = nullptr, *e = nullptr;
  if (hipMalloc((void**)&d, (size_t)n * 16) != hipSuccess) return LEGO_ENOMEM;
  if (hipMalloc((void**)&f, (size_t)n * 4) != hipSuccess) { hipFree(d); return LEGO_ENOMEM; }
  if (hipMalloc((void**)&e, (size_t)n * 4) != hipSuccess) { hipFree(d); hipFree(f); return LEGO_ENOMEM; }
  rc = LEGO_OK;
  if (hipMemcpy(d, h_xyzw, (size_t)n * 16, hipMemcpyHostToDevice) != hipSuccess) rc = LEGO_EDEVICE;
  if (rc == LEGO_OK) {
    hipLaunchKernelGGL(k_proj_test, dim3((n + 255) / 256), dim3(256), 0, 0, P, d, n, f, e);
    if (hipGetLastError() != hipSuccess || hipMemcpy(h_fast, f, (size_t)n * 4, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(h_exact, e, (size_t)n * 4, hipMemcpyDeviceToHost) != hipSuccess)
      rc = LEGO_EDEVICE;
  }
  hipFree(d); hipFree(f); hipFree(e);
  return rc;
}

extern "C" int lego_test_libm(const float* h_a, const float* h_b, float* h_out, int32_t n, int32_t which) {
  if (n <= 0 || !h_a || !h_b || !h_out) return LEGO_EINVAL;
  float *a = nullptr, *b = nullptr, *o = nullptr;
  const size_t bytes = (size_t)n * sizeof(float);
  if (hipMalloc((void**)&a, bytes) != hipSuccess) return LEGO_ENOMEM;
  if (hipMalloc((void**)&b, bytes) != hipSuccess) { hipFree(a); return LEGO_ENOMEM; }
  if (hipMalloc((void**)&o, bytes) != hipSuccess) { hipFree(a); hipFree(b); return LEGO_ENOMEM; }
  int rc = LEGO_OK;
  if (hipMemcpy(a, h_a, bytes, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(b, h_b, bytes, hipMemcpyHostToDevice) != hipSuccess) rc = LEGO_EDEVICE;
  if (rc == LEGO_OK) {
    hipLaunchKernelGGL(k_libm_test, dim3((n + 255) / 256), dim3(256), 0, 0, a, b, o, n, which);
    if (hipGetLastError() != hipSuccess || hipMemcpy(h_out, o, bytes, hipMemcpyDeviceToHost) != hipSuccess)
      rc = LEGO_EDEVICE;
  }
  hipFree(a); hipFree(b); hipFree(o);
  return rc;
}

template <int KN>
__global__ __launch_bounds__(64) void k_kd_test(KdView K, int n, const float4* q, int m, int* idx, float* dist) {
  __shared__ float box[6];
  const bool built = kd_build(K, n, box) >= 0;
  const int cap = (10 * K.vh) / (5 * 64);
  for (int k0 = 0; k0 < m; k0 += 64) {
    const int k = k0 + lane_id();
    if (k < m) {
      int ix[KN];
      float d[KN];
      bool ovf = !built;
      if (n > 0 && built) kd_knn<KN>(K, box, q[k], K.frames + (size_t)lane_id() * cap * 5, cap, ix, d, ovf);
      for (int j = 0; j < KN; ++j) {
        idx[(size_t)k * KN + j] = ovf ? -2 : (n > 0 ? ix[j] : -1);
        dist[(size_t)k * KN + j] = n > 0 && !ovf ? d[j] : FLT_MAX;
      }
    }
  }
}

// nanoflann's kNN (k = 1: the LM's exact-tie path; k = 5: MapOptimization's) on the device (kd_build +
// kd_knn) for m queries against a cloud of n points (x, y, z, w float32 each); idx[m][k] nearest first,
// -1 past the count found, -2 = stack overflow.
extern "C" int lego_test_kd_knn(const float* h_cloud, int32_t n, const float* h_q, int32_t m, int32_t k,
                                int32_t* h_idx, float* h_dist) {
  if (n < 0 || m < 0 || (k != 1 && k != 5) || (n && !h_cloud) || (m && (!h_q || !h_idx || !h_dist)) || n > (1 << 22))
    return LEGO_EINVAL;
  const int vh = std::max(n, 1024);
  float4 *c = nullptr, *q = nullptr;
  KdView K = {};
  int *idx = nullptr;
  float* dist = nullptr;
  int rc = LEGO_OK;
  if (hipMalloc((void**)&c, (size_t)vh * 16) != hipSuccess || hipMalloc((void**)&q, (size_t)std::max(m, 1) * 16) != hipSuccess ||
      hipMalloc((void**)&K.node, (size_t)2 * vh * sizeof(KdNode)) != hipSuccess ||
      hipMalloc((void**)&K.vind, (size_t)vh * 4) != hipSuccess || hipMalloc((void**)&K.tmp, (size_t)2 * vh * 4) != hipSuccess ||
      hipMalloc((void**)&K.frames, (size_t)10 * vh * 4) != hipSuccess ||
      hipMalloc((void**)&idx, (size_t)std::max(m, 1) * 4 * k) != hipSuccess ||
      hipMalloc((void**)&dist, (size_t)std::max(m, 1) * 4 * k) != hipSuccess)
    rc = LEGO_ENOMEM;
  K.pts = c;
  K.vh = vh;
  if (rc == LEGO_OK && ((n && hipMemcpy(c, h_cloud, (size_t)n * 16, hipMemcpyHostToDevice) != hipSuccess) ||
                        (m && hipMemcpy(q, h_q, (size_t)m * 16, hipMemcpyHostToDevice) != hipSuccess)))
    rc = LEGO_EDEVICE;
  if (rc == LEGO_OK) {
    if (k == 1) hipLaunchKernelGGL(k_kd_test<1>, dim3(1), dim3(64), 0, 0, K, n, q, m, idx, dist);
    else hipLaunchKernelGGL(k_kd_test<5>, dim3(1), dim3(64), 0, 0, K, n, q, m, idx, dist);
    if (hipGetLastError() != hipSuccess || (m && (hipMemcpy(h_idx, idx, (size_t)m * 4 * k, hipMemcpyDeviceToHost) != hipSuccess ||
                                                  hipMemcpy(h_dist, dist, (size_t)m * 4 * k, hipMemcpyDeviceToHost) != hipSuccess)))
      rc = LEGO_EDEVICE;
  }
  for (void* p : {(void*)c, (void*)q, (void*)K.node, (void*)K.vind, (void*)K.tmp, (void*)K.frames, (void*)idx, (void*)dist})
    if (p) hipFree(p);
  return rc;
}

__global__ void k_libm_d_test(const double* a, const double* b, double* out, int n, int which) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double r;
  if (which == 0) r = sin_d(a[i]);
  else if (which == 1) r = cos_d(a[i]);
  else if (which == 2) r = atan2_d(a[i], b[i]);
  else if (which == 3) r = asin_d(a[i]);
  else if (which == 4) r = sqrt(a[i]);
  else r = a[i] / b[i];
  out[i] = r;
}

extern "C" int lego_test_libm_d(const double* h_a, const double* h_b, double* h_out, int32_t n, int32_t which) {
  if (n <= 0 || !h_a || !h_b || !h_out) return LEGO_EINVAL;
  double *a = nullptr, *b = nullptr, *o = nullptr;
  const size_t bytes = (size_t)n * sizeof(double);
  if (hipMalloc((void**)&a, bytes) != hipSuccess) return LEGO_ENOMEM;
  if (hipMalloc((void**)&b, bytes) != hipSuccess) { hipFree(a); return LEGO_ENOMEM; }
  if (hipMalloc((void**)&o, bytes) != hipSuccess) { hipFree(a); hipFree(b); return LEGO_ENOMEM; }
  int rc = LEGO_OK;
  if (hipMemcpy(a, h_a, bytes, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(b, h_b, bytes, hipMemcpyHostToDevice) != hipSuccess) rc = LEGO_EDEVICE;
  if (rc == LEGO_OK) {
    hipLaunchKernelGGL(k_libm_d_test, dim3((n + 255) / 256), dim3(256), 0, 0, a, b, o, n, which);
    if (hipGetLastError() != hipSuccess || hipMemcpy(h_out, o, bytes, hipMemcpyDeviceToHost) != hipSuccess)
      rc = LEGO_EDEVICE;
  }
  hipFree(a); hipFree(b); hipFree(o);
  return rc;
}

template <int R>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(R == 32 ? 2 : 3)))
void k_sort_test_lvl(unsigned* keys, int* vals, int n) {  // as k_voxel<4 / 5>
  __shared__ VoxLvlLds<R> L;
  for (int i = lane_id(); i < n; i += 64) { L.u.nat.key[i] = keys[i]; L.u.nat.val[i] = (uint16_t)vals[i]; }
  __syncthreads();
  lvl_sort<R>(L.u.nat.key, L.u.nat.val, L.u.buf, n);
  for (int i = lane_id(); i < n; i += 64) { keys[i] = L.u.nat.key[i]; vals[i] = L.u.nat.val[i]; }
}

__global__ __launch_bounds__(64) void k_sort_test(unsigned* keys, int* vals, int n, int is_float) {
  __shared__ SortTestLds L;
  const int lane = lane_id();
  for (int i = lane; i < n; i += 64) { L.u.vkey[i] = keys[i]; L.vval[i] = (uint16_t)vals[i]; }
  __syncthreads();
  if (is_float == 2) {  // k_extract's segment sort (n <= SEG_MAX)
    for (int i = lane; i < n; i += 64) { L.u.seg.skey[i] = __int_as_float((int)keys[i]); L.u.seg.sval[i] = vals[i]; }
    __syncthreads();
    sort_segment(L, n);
    for (int i = lane; i < n; i += 64) { keys[i] = (unsigned)__float_as_int(L.u.seg.skey[i]); vals[i] = L.u.seg.sval[i]; }
    return;
  } else if (is_float) {
    wave_std_sort<float, uint16_t>((float*)L.u.vkey, L.vval, n, L.blk);
  } else {
    wave_std_sort<unsigned, uint16_t>(L.u.vkey, L.vval, n, nullptr, true);  // as k_voxel
  }
  for (int i = lane; i < n; i += 64) { keys[i] = L.u.vkey[i]; vals[i] = L.vval[i]; }
}

extern "C" int lego_test_sort(uint32_t* h_keys, int32_t* h_vals, int32_t n, int32_t is_float) {
  if (n < 0 || n > RING_MAX || !h_keys || !h_vals || is_float < 0 || is_float > 3) return LEGO_EINVAL;
  if (is_float == 2 && n > SEG_MAX) return LEGO_EINVAL;
  if (is_float == 3)
    for (int i = 0; i < n; ++i)
      if (h_keys[i] >= 0x7fffffffu || (uint32_t)h_vals[i] > 0xffffu) return LEGO_EINVAL;
  if (n == 0) return LEGO_OK;
  unsigned* k = nullptr;
  int* v = nullptr;
  if (hipMalloc((void**)&k, n * 4) != hipSuccess) return LEGO_ENOMEM;
  if (hipMalloc((void**)&v, n * 4) != hipSuccess) { hipFree(k); return LEGO_ENOMEM; }
  int rc = LEGO_OK;
  if (hipMemcpy(k, h_keys, n * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(v, h_vals, n * 4, hipMemcpyHostToDevice) != hipSuccess) rc = LEGO_EDEVICE;
  if (rc == LEGO_OK) {
    if (is_float == 3 && n > 1024) hipLaunchKernelGGL(k_sort_test_lvl<32>, dim3(1), dim3(64), 0, 0, k, v, n);
    else if (is_float == 3 && n > 512) hipLaunchKernelGGL(k_sort_test_lvl<16>, dim3(1), dim3(64), 0, 0, k, v, n);
    else if (is_float == 3) hipLaunchKernelGGL(k_sort_test_lvl<8>, dim3(1), dim3(64), 0, 0, k, v, n);
    else hipLaunchKernelGGL(k_sort_test, dim3(1), dim3(64), 0, 0, k, v, n, is_float);
    if (hipGetLastError() != hipSuccess || hipMemcpy(h_keys, k, n * 4, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(h_vals, v, n * 4, hipMemcpyDeviceToHost) != hipSuccess) rc = LEGO_EDEVICE;
  }
  hipFree(k); hipFree(v);
  return rc;
}

#ifdef LG_PROFILE
// kV 0: as k_voxel (partitions + final_window); 2: partitions + per-block insertion sorts; 3: final_window
// alone; 4: final_bitonic alone (3 and 4 on the unpartitioned keys: their cost only)
template <int kV>
__global__ __launch_bounds__(64) void k_sort_bench(const unsigned* keys, int n, unsigned* out) {
  __shared__ std::conditional_t<kV == 2, SortTestLds, ExtractLds> L;
  const int lane = lane_id();
  for (int i = lane; i < n; i += 64) { L.u.vkey[i] = keys[i]; L.vval[i] = (uint16_t)i; }
  __syncthreads();
  if constexpr (kV == 0 || kV == 2) {
    if constexpr (kV == 2) wave_std_sort<unsigned, uint16_t>(L.u.vkey, L.vval, n, L.blk, false);
    else wave_std_sort<unsigned, uint16_t>(L.u.vkey, L.vval, n, nullptr, true);
  } else if constexpr (kV == 3) {
    if (n > 1024) final_window<32>(L.u.vkey, L.vval, n);
    else final_window<16>(L.u.vkey, L.vval, n);
  } else {
    if (n > 1024) final_bitonic<32>(L.u.vkey, L.vval, n);
    else final_bitonic<16>(L.u.vkey, L.vval, n);
  }
  if (lane == 0) out[blockIdx.x] = L.vval[n / 2];
}
template <int R>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(R == 32 ? 2 : 3)))
void k_sort_bench_lvl(const unsigned* keys, int n, unsigned* out) {
  __shared__ VoxLvlLds<R> L;
  for (int i = lane_id(); i < n; i += 64) { L.u.nat.key[i] = keys[i]; L.u.nat.val[i] = (uint16_t)i; }
  __syncthreads();
  lvl_sort<R>(L.u.nat.key, L.u.nat.val, L.u.buf, n);
  if (lane_id() == 0) out[blockIdx.x] = L.u.nat.val[n / 2];
}
#endif

#ifdef LG_PROFILE
// Counter calibration (profile build only; MI355X_MICROARCH.md: FETCH_SIZE is calibrated only for
// 16-B-per-lane streaming reads): k_project's input read patterns over S scans of points, one 1024-thread workgroup a scan,
// nothing else read and one float a lane written.  mode 0: the scatter pass's 12-byte buffer loads;
// 1: 16-byte loads of the same points; 2: mode 0, then every point again as a 16-byte load (the
// column pass's re-gather, in point order).
__global__ __launch_bounds__(1024) void k_fetch_probe(int mode, const float4* __restrict__ pts,
                                                      const int64_t* __restrict__ offs,
                                                      const int32_t* __restrict__ cnts, float* out) {
  const int s = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  const float4* in = pts + offs[s];
  const int n = cnts[s];
  float acc = 0.f;
  constexpr int kU = 8;
  if (mode == 1) {
    for (int i0 = tid; i0 < n; i0 += nt * kU) {
      float4 pk[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) pk[u] = in[min(i0 + u * nt, n - 1)];
#pragma unroll
      for (int u = 0; u < kU; ++u) acc += pk[u].x + pk[u].y + pk[u].z;
    }
  } else {
    const __amdgpu_buffer_rsrc_t rin = buffer_rsrc(in, (uint32_t)n * 16u);
    for (int i0 = tid; i0 < n; i0 += nt * kU) {
      float3 pk[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) pk[u] = buffer_load_f3(rin, (uint32_t)(i0 + u * nt) * 16u);
#pragma unroll
      for (int u = 0; u < kU; ++u) acc += pk[u].x + pk[u].y + pk[u].z;
    }
    if (mode == 2) {
      __syncthreads();
      for (int i0 = tid; i0 < n; i0 += nt * kU) {
        float4 pk[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) pk[u] = in[min(i0 + u * nt, n - 1)];
#pragma unroll
        for (int u = 0; u < kU; ++u) acc += pk[u].w;
      }
    }
  }
  out[(size_t)s * nt + tid] = acc;
}

#endif

#ifdef LG_PROFILE  // the diagnostic entry points (include/lego_debug.h): profile build only
#include "../../include/lego_debug.h"
extern "C" int lego_debug_fetch_probe(int32_t mode, int32_t S, const void* pts, const int64_t* offs,
                                      const int32_t* cnts, float* out, void* stream) {
  if (mode < 0 || mode > 2 || S < 1 || !pts || !offs || !cnts || !out) return LEGO_EINVAL;
  hipLaunchKernelGGL(k_fetch_probe, dim3(S), dim3(1024), 0, (hipStream_t)stream, mode, (const float4*)pts, offs,
                     cnts, out);
  return hipGetLastError() == hipSuccess ? LEGO_OK : LEGO_EDEVICE;
}

// Diagnostics (profile build only): time `blocks` concurrent copies of one device sort.
// mode 0: the stack emulation (wave_std_sort), 1: the level-synchronous one (lvl_sort, R by size)
extern "C" int lego_debug_sort_bench(const uint32_t* h_keys, int32_t n, int32_t blocks, int32_t mode, float* ms) {
  unsigned *k = nullptr, *o = nullptr;
  if (n < 1 || n > RING_MAX || blocks < 1 || (mode == 1 && n > 2048)) return LEGO_EINVAL;
  hipMalloc((void**)&k, n * 4);
  hipMalloc((void**)&o, blocks * 4);
  hipMemcpy(k, h_keys, n * 4, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto launch = [&]() {
    if (mode == 0) hipLaunchKernelGGL(k_sort_bench<0>, dim3(blocks), dim3(64), 0, 0, k, n, o);
    else if (mode == 2) hipLaunchKernelGGL(k_sort_bench<2>, dim3(blocks), dim3(64), 0, 0, k, n, o);
    else if (mode == 3) hipLaunchKernelGGL(k_sort_bench<3>, dim3(blocks), dim3(64), 0, 0, k, n, o);
    else if (mode == 4) hipLaunchKernelGGL(k_sort_bench<4>, dim3(blocks), dim3(64), 0, 0, k, n, o);
    else if (n > 1024) hipLaunchKernelGGL(k_sort_bench_lvl<32>, dim3(blocks), dim3(64), 0, 0, k, n, o);
    else if (n > 512) hipLaunchKernelGGL(k_sort_bench_lvl<16>, dim3(blocks), dim3(64), 0, 0, k, n, o);
    else hipLaunchKernelGGL(k_sort_bench_lvl<8>, dim3(blocks), dim3(64), 0, 0, k, n, o);
  };
  launch();
  hipEventRecord(a, 0);
  launch();
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  hipEventElapsedTime(ms, a, b);
  hipEventDestroy(a);
  hipEventDestroy(b);
  hipFree(k);
  hipFree(o);
  return LEGO_OK;
}

// LDS allocation probe: one wave a block holding `bytes` of dynamic LDS, each sleeping ~20 us
__global__ __launch_bounds__(64) void k_lds_probe(int* out) {
  extern __shared__ int dyn[];
  dyn[threadIdx.x] = threadIdx.x;
  for (int i = 0; i < 400; ++i) __builtin_amdgcn_s_sleep(127);
  if (threadIdx.x == 0) out[blockIdx.x] = dyn[1];
}
// Diagnostics (profile build only): ms of `blocks` one-wave blocks of `bytes` LDS each (co-residency).
extern "C" int lego_debug_lds_probe(int32_t bytes, int32_t blocks, float* ms) {
  int* o = nullptr;
  hipMalloc((void**)&o, blocks * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(k_lds_probe, dim3(blocks), dim3(64), bytes, 0, o);
  hipEventRecord(a, 0);
  hipLaunchKernelGGL(k_lds_probe, dim3(blocks), dim3(64), bytes, 0, o);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  hipEventElapsedTime(ms, a, b);
  hipEventDestroy(a);
  hipEventDestroy(b);
  hipFree(o);
  return LEGO_OK;
}

extern "C" int lego_debug_lm_log(uint64_t* out, int32_t n_blocks) {  // k_lm's last launch
  if (!out || n_blocks < 0 || n_blocks > 4096) return LEGO_EINVAL;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lm_log), sizeof(uint64_t) * 16 * (size_t)n_blocks) == hipSuccess
             ? LEGO_OK : LEGO_EDEVICE;
}

extern "C" int lego_debug_ring_log(uint64_t* out, int32_t n_blocks) {  // k_voxel's last launch
  if (!out || n_blocks < 0 || n_blocks > 65536) return LEGO_EINVAL;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ring_log), sizeof(uint64_t) * 4 * (size_t)n_blocks) == hipSuccess
             ? LEGO_OK : LEGO_EDEVICE;
}

extern "C" int lego_debug_prof(uint64_t* out32, int32_t reset) {
  std::vector<uint64_t> h(256 * 64, 0);
  if (out32) {
    if (hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_prof), sizeof(uint64_t) * h.size()) != hipSuccess) return LEGO_EDEVICE;
    for (int i = 0; i < 256; ++i) {
      const bool is_max = (i >= 128 && i < 192) || i >= 192;
      uint64_t r = 0;
      for (int c = 0; c < 64; ++c) r = is_max ? std::max(r, h[(size_t)i * 64 + c]) : r + h[(size_t)i * 64 + c];
      out32[i] = r;
    }
  }
  if (reset) {
    std::fill(h.begin(), h.end(), 0);
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_prof), h.data(), sizeof(uint64_t) * h.size()) != hipSuccess) return LEGO_EDEVICE;
  }
  return LEGO_OK;
}
#endif  // LG_PROFILE

#ifdef LG_PWS_STATS
extern "C" int lego_debug_pws_stats(uint64_t* out8, int32_t reset) {
  if (out8 && hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_pws), 64) != hipSuccess) return LEGO_EDEVICE;
  if (reset) {
    uint64_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_pws), z, 64) != hipSuccess) return LEGO_EDEVICE;
  }
  return LEGO_OK;
}
#endif
