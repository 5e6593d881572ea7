// lego_device.h — device-side types and libm restatement for the gfx950 kernels.
//
// Numerics contract: every kernel is compiled with -ffp-contract=off
// (x86-64 reference has no FMA), float division/sqrt correctly rounded (HIP default), and the
// reference's float/double promotions written out explicitly.
//
// libm: the reference calls glibc's float asinf / atan2f (std::asin/std::atan2 on float, and the
// unqualified float overloads, fp_mode 0).  glibc 2.35's implementations of these are the fdlibm
// algorithms (flt-32/e_asinf.c, s_atanf.c, e_atan2f.c): restated below operation for operation.
// Verified bit-identical against the container's glibc on all 2^31 asinf inputs in [-1,1], every
// 3rd float for atanf and 3e8 random atan2f pairs (tests/test_libm.py keeps a sampled check).
// sinf/cosf (used only inside the LM, which is checked within tolerance) are evaluated in double
// and rounded once.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define LG_DEVICE __device__ __forceinline__

namespace lg {

LG_DEVICE uint32_t fbits(float f) { return __float_as_uint(f); }
LG_DEVICE float bitsf(uint32_t u) { return __uint_as_float(u); }

// ---- glibc/fdlibm atanf (sysdeps/ieee754/flt-32/s_atanf.c) ---------------------------------
LG_DEVICE float atanf_g(float x) {
  const float atanhi0 = 4.6364760399e-01f, atanhi1 = 7.8539812565e-01f, atanhi2 = 9.8279368877e-01f,
              atanhi3 = 1.5707962513e+00f;
  const float atanlo0 = 5.0121582440e-09f, atanlo1 = 3.7748947079e-08f, atanlo2 = 3.4473217170e-08f,
              atanlo3 = 7.5497894159e-08f;
  const float aT0 = 3.3333334327e-01f, aT1 = -2.0000000298e-01f, aT2 = 1.4285714924e-01f,
              aT3 = -1.1111110449e-01f, aT4 = 9.0908870101e-02f, aT5 = -7.6918758452e-02f,
              aT6 = 6.6610731184e-02f, aT7 = -5.8335702866e-02f, aT8 = 4.9768779427e-02f,
              aT9 = -3.6531571299e-02f, aT10 = 1.6285819933e-02f;
  int32_t hx = (int32_t)fbits(x);
  int32_t ix = hx & 0x7fffffff;
  int id;
  if (ix >= 0x4c000000) {
    if (ix > 0x7f800000) return x + x;
    return (hx > 0) ? atanhi3 + atanlo3 : -atanhi3 - atanlo3;
  }
  if (ix < 0x3ee00000) {
    if (ix < 0x31000000) return x;
    id = -1;
  } else {
    x = fabsf(x);
    if (ix < 0x3f980000) {
      if (ix < 0x3f300000) { id = 0; x = (2.0f * x - 1.0f) / (2.0f + x); }
      else { id = 1; x = (x - 1.0f) / (x + 1.0f); }
    } else {
      if (ix < 0x401c0000) { id = 2; x = (x - 1.5f) / (1.0f + 1.5f * x); }
      else { id = 3; x = -1.0f / x; }
    }
  }
  float z = x * x;
  float w = z * z;
  float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
  float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
  if (id < 0) return x - x * (s1 + s2);
  float hi = id == 0 ? atanhi0 : id == 1 ? atanhi1 : id == 2 ? atanhi2 : atanhi3;
  float lo = id == 0 ? atanlo0 : id == 1 ? atanlo1 : id == 2 ? atanlo2 : atanlo3;
  z = hi - ((x * (s1 + s2) - lo) - x);
  return (hx < 0) ? -z : z;
}

// ---- glibc/fdlibm atan2f (sysdeps/ieee754/flt-32/e_atan2f.c) -------------------------------
LG_DEVICE float atan2f_g(float y, float x) {
  const float pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f, pi = 3.1415927410e+00f,
              pi_lo = -8.7422776573e-08f, tiny = 1.0e-30f;
  int32_t hx = (int32_t)fbits(x), hy = (int32_t)fbits(y);
  int32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
  if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
  if (hx == 0x3f800000) return atanf_g(y);
  int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
  if (iy == 0) {
    switch (m) {
      case 0:
      case 1: return y;
      case 2: return pi + tiny;
      default: return -pi - tiny;
    }
  }
  if (ix == 0) return (hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
  if (ix == 0x7f800000) {
    if (iy == 0x7f800000) {
      switch (m) {
        case 0: return pi_o_4 + tiny;
        case 1: return -pi_o_4 - tiny;
        case 2: return 3.0f * pi_o_4 + tiny;
        default: return -3.0f * pi_o_4 - tiny;
      }
    } else {
      switch (m) {
        case 0: return 0.0f;
        case 1: return -0.0f;
        case 2: return pi + tiny;
        default: return -pi - tiny;
      }
    }
  }
  if (iy == 0x7f800000) return (hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
  int k = (iy - ix) >> 23;
  float z;
  if (k > 60) z = pi_o_2 + 0.5f * pi_lo;
  else if (hx < 0 && k < -60) z = 0.0f;
  else z = atanf_g(fabsf(y / x));
  switch (m) {
    case 0: return z;
    case 1: return -z;
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
  }
}

// ---- glibc asinf (sysdeps/ieee754/flt-32/e_asinf.c) ----------------------------------------
LG_DEVICE float asinf_g(float x) {
  const float pio2_hi = 1.57079637050628662109375f, pio2_lo = -4.37113900018624283e-8f,
              pio4_hi = 0.785398185253143310546875f, p0 = 1.666675248e-1f, p1 = 7.495297643e-2f,
              p2 = 4.547037598e-2f, p3 = 2.417951451e-2f, p4 = 4.216630880e-2f;
  int32_t hx = (int32_t)fbits(x);
  int32_t ix = hx & 0x7fffffff;
  float t, w, p, q, c, r, s;
  if (ix == 0x3f800000) return x * pio2_hi + x * pio2_lo;
  if (ix > 0x3f800000) return (x - x) / (x - x);
  if (ix < 0x3f000000) {
    if (ix < 0x32000000) return x;
    t = x * x;
    w = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
    return x + x * w;
  }
  w = 1.0f - fabsf(x);
  t = w * 0.5f;
  p = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
  s = sqrtf(t);
  if (ix >= 0x3F79999A) {
    t = pio2_hi - (2.0f * (s + s * p) - pio2_lo);
  } else {
    w = bitsf(fbits(s) & 0xfffff000u);
    c = (t - w * w) / (s + w);
    r = p;
    p = 2.0f * s * r - (pio2_lo - 2.0f * c);
    q = pio4_hi - 2.0f * w;
    t = pio4_hi - (p - q);
  }
  return (hx > 0) ? t : -t;
}

// sinf/cosf: double evaluation rounded once (glibc's own sinf/cosf differ on ~1e-3 of inputs;
// they are used only inside the LM, which is parity-checked within 1e-4).
LG_DEVICE float sinf_g(float x) { return (float)sin((double)x); }
LG_DEVICE float cosf_g(float x) { return (float)cos((double)x); }

LG_DEVICE bool isfinite_f(float x) { return (fbits(x) & 0x7f800000u) != 0x7f800000u; }

}  // namespace lg

// ---- shared POD types (host + device) ---------------------------------------------------------
struct LgParams {  // ImageProjection / FeatureAssociation ctor constants (host-derived)
  int V, H, G, VH;
  float ang_res_x, ang_res_y, ang_bottom, mount;
  float sinX, cosX, sinY, cosY, theta_thr;
  int seg_valid_pt, seg_valid_line;
  float scan_period, edge_thr, surf_thr, nn_dist_sqr;
  int map_div;
  int cap_sharp, cap_lsharp, cap_flat;  // per-ring caps: 12, 120, 24
};

struct LgState {  // FeatureAssociation members that persist across scans (featureAssociation.h)
  float cur[6];
  float sum[6];
  int initialized;       // systemInitedLM
  int is_degenerate;     // isDegenerate
  int cycle;             // _cycle_count
  int last_buf;          // which half of the Last double buffer holds *Last
  int n_corner_last, n_surf_last;
  int tree_stale;        // kd-trees were not rebuilt at the last publishCloudsLast
  int status;            // LEGO_ST_* of the last association
  int iters_surf, iters_corner;
  int proj_status;       // 0 or LEGO_EEMPTY for the last projection
  int pad;
  double quat[4];
  double pos[3];
};

// counts[] slots per stream
enum {
  CNT_M = 0, CNT_OUTLIER = 1, CNT_SCAN = 2, CNT_SHARP = 3, CNT_LSHARP = 4, CNT_FLAT = 5, CNT_LFLAT = 6,
  CNT_STATUS = 7, CNT_N = 8
};

struct LgBufs {  // device buffers, all indexed [stream][...]
  // ImageProjection
  float* range;          // [S][VH]
  float4* cloud;         // [S][VH]  _full_cloud
  int8_t* ground;        // [S][VH]
  int32_t* label;        // [S][VH]
  int32_t* winner;       // [S][VH]  (global-winner path only)
  int32_t* cc_parent;    // [S][VH]  (global union-find path only)
  int32_t* cc_cnt;       // [S][VH]
  unsigned long long* cc_mask;  // [S][VH]
  int32_t* scan_cand;    // [S][H]
  float* orient;         // [S][4]
  float4* seg_pts;       // [S][VH]
  float* seg_range;      // [S][VH]
  uint32_t* seg_col;     // [S][VH]
  uint8_t* seg_ground;   // [S][VH]
  int32_t* ring_start;   // [S][V]
  int32_t* ring_end;     // [S][V]
  float4* outlier;       // [S][VH]
  float4* scan_msg;      // [S][H]
  int32_t* counts;       // [S][CNT_N]
  // FeatureAssociation persistent work arrays
  float* curv;           // [S][VH]
  uint8_t* picked;       // [S][VH]
  int8_t* flabel;        // [S][VH]
  int2* smooth;          // [S][VH]  {float bits of value, ind}
  float4* seg_fa;        // [S][VH]  segmentedCloud after adjustDistortion
  float4* outlier_fa;    // [S][VH]  adjustOutlierCloud
  // per-ring staging
  float4* r_sharp; int32_t* r_sharp_ind;    // [S][V][cap_sharp]
  float4* r_lsharp; int32_t* r_lsharp_ind;  // [S][V][cap_lsharp]
  float4* r_flat; int32_t* r_flat_ind;      // [S][V][cap_flat]
  float4* r_lflat;                          // [S][V][H]
  int32_t* r_counts;                        // [S][V][4]
  int32_t* r_status;                        // [S][V]
  // concatenated features
  float4* f_sharp; int32_t* f_sharp_ind;    // [S][V*cap_sharp]
  float4* f_lsharp; int32_t* f_lsharp_ind;  // [S][V*cap_lsharp]
  float4* f_flat; int32_t* f_flat_ind;      // [S][V*cap_flat]
  float4* f_lflat;                          // [S][VH]
  // Last clouds, double-buffered
  float4* corner_last;   // [S][2][V*cap_lsharp]
  float4* surf_last;     // [S][2][VH]
  LgState* state;        // [S]
};
