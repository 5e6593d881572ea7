// lego_libm.h — glibc-faithful float libm for host and device (see lego_device.h for the contract).
//
// glibc 2.35's asinf / atanf / atan2f are the fdlibm algorithms (sysdeps/ieee754/flt-32/e_asinf.c,
// s_atanf.c, e_atan2f.c); restated here operation for operation so that the gfx950 kernels reproduce
// the reference's float std::asin / std::atan2 results bit for bit.  Compile without FMA contraction.
#pragma once
#include <math.h>
#include <stdint.h>

#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define LG_LIBM __host__ __device__ __forceinline__
#else
#define LG_LIBM inline
#endif

namespace lg {

LG_LIBM uint32_t fbits(float f) { return __builtin_bit_cast(uint32_t, f); }
LG_LIBM float bitsf(uint32_t u) { return __builtin_bit_cast(float, u); }

// ---- glibc/fdlibm atanf (sysdeps/ieee754/flt-32/s_atanf.c) ---------------------------------
LG_LIBM float atanf_g(float x) {
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
LG_LIBM float atan2f_g(float y, float x) {
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
LG_LIBM float asinf_g(float x) {
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

// ---- glibc 2.35 sinf / cosf (sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, sincosf.h, sincosf_data.c) --
// The x86-64 build the reference links runs the FMA ifunc variant (sysdeps/x86_64/fpu/multiarch/
// s_sinf-fma.c) on any AVX2/FMA host: the polynomial's a + b * c steps and the range reduction's
// x - n * pi/2 are fused there, so they are __builtin_fma here.  Bit-exact with the host's sinf / cosf
// for every float in [-120, 120] (checked exhaustively, tests/native/trig_check.cpp); beyond 120 rad
// (never an LM angle) glibc's large-argument reduction is not restated: float(sin(double x)) instead.
struct SinCosTab {
  double c0, c1, c2, c3, c4, s1, s2, s3;
};
LG_LIBM SinCosTab sincos_tab(bool second) {  // __sincosf_table[0] / [1]: [1] negates the cosine terms
  const double k = second ? -1.0 : 1.0;
  return SinCosTab{k * 0x1p0, k * -0x1.ffffffd0c621cp-2, k * 0x1.55553e1068f19p-5, k * -0x1.6c087e89a359dp-10,
                   k * 0x1.99343027bf8c3p-16, -0x1.555545995a603p-3, 0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13};
}
// sinf_poly: n even -> sin(x), odd -> cos(x) (table [1]: -cos(x))
LG_LIBM float sincos_poly(double x, double x2, const SinCosTab& p, int n) {
  if ((n & 1) == 0) {
    const double x3 = x * x2;
    const double s1 = __builtin_fma(x2, p.s3, p.s2);
    const double x7 = x3 * x2;
    const double s = __builtin_fma(x3, p.s1, x);
    return (float)__builtin_fma(x7, s1, s);
  }
  const double x4 = x2 * x2;
  const double c2 = __builtin_fma(x2, p.c4, p.c3);
  const double c1 = __builtin_fma(x2, p.c1, p.c0);
  const double x6 = x4 * x2;
  const double c = __builtin_fma(x4, p.c2, c1);
  return (float)__builtin_fma(x6, c2, c);
}
LG_LIBM uint32_t abstop12(float x) { return (fbits(x) >> 20) & 0x7ff; }
// reduce_fast: n = nearest multiple of pi/2 (fixed point, 2/pi * 2^24), x - n * pi/2
LG_LIBM double sincos_reduce(double x, int& n) {
  const double r = x * 0x1.45f306dc9c883p+23;
  n = ((int32_t)r + 0x800000) >> 24;
  return __builtin_fma(-(double)n, 0x1.921fb54442d18p0, x);
}
LG_LIBM float sinf_g(float y) {
  const double x = (double)y;
  if (abstop12(y) < abstop12(0x1.921fb6p-1f)) {
    if (abstop12(y) < abstop12(0x1p-12f)) return y;
    return sincos_poly(x, x * x, sincos_tab(false), 0);
  }
  if (abstop12(y) < abstop12(120.0f)) {
    int n;
    const double r = sincos_reduce(x, n);
    const double sg = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0;  // sign[] = {1, -1, -1, 1}
    return sincos_poly(r * sg, r * r, sincos_tab((n & 2) != 0), n);
  }
  return (float)sin(x);
}
LG_LIBM float cosf_g(float y) {
  const double x = (double)y;
  if (abstop12(y) < abstop12(0x1.921fb6p-1f)) {
    if (abstop12(y) < abstop12(0x1p-12f)) return 1.0f;
    return sincos_poly(x, x * x, sincos_tab(false), 1);
  }
  if (abstop12(y) < abstop12(120.0f)) {
    int n;
    const double r = sincos_reduce(x, n);
    const double sg = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0;
    return sincos_poly(r * sg, r * r, sincos_tab((n & 2) != 0), n ^ 1);
  }
  return (float)cos(x);
}

LG_LIBM bool isfinite_f(float x) { return (fbits(x) & 0x7f800000u) != 0x7f800000u; }

}  // namespace lg
