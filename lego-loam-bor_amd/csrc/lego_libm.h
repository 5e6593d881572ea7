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
// Out of line (one copy a translation unit): the large-argument fallbacks, never taken for an LM angle.
// Inlined, OCML's double sin / cos (Payne-Hanek reduction) set the register peak of every kernel that
// evaluates a float sin / cos (k_lm: 177 VGPRs).
#define LG_LIBM_COLD static __host__ __device__ __attribute__((noinline))
#else
#define LG_LIBM inline
#define LG_LIBM_COLD static inline
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
LG_LIBM_COLD float sinf_big(float y) { return (float)sin((double)y); }
LG_LIBM_COLD float cosf_big(float y) { return (float)cos((double)y); }
LG_LIBM_COLD double sin_big(double x) { return sin(x); }
LG_LIBM_COLD double cos_big(double x) { return cos(x); }
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
  return sinf_big(y);
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
  return cosf_big(y);
}

LG_LIBM bool isfinite_f(float x) { return (fbits(x) & 0x7f800000u) != 0x7f800000u; }

// ================================================================================================
// Double-precision sin / cos / atan / atan2 / asin for fp_mode 1: on the
// pre-GCC-6 toolchains the reference README names (ROS Indigo / Kinetic), unqualified sin(float)
// etc. resolve to ::sin(double), so those expressions are evaluated in double and rounded where the
// reference stores to float.  These are the fdlibm 5.3 double algorithms (k_sin.c, k_cos.c,
// e_rem_pio2.c's medium-size Cody-Waite reduction, s_sin.c, s_cos.c, s_atan.c, e_atan2.c, e_asin.c),
// each < 1 ulp.  glibc 2.35 evaluates these functions with the IBM Accurate Mathematical Library
// instead (nearly correctly rounded), so results can differ in the last bit of the double; after the
// rounding to float that the reference applies they agree except when the exact value lies within
// ~1 double ulp of a float rounding boundary.  tests/native/libm_d_check.cpp measures both rates
// against the host's glibc.
// ================================================================================================
LG_LIBM uint64_t dbits_of(double d) { return __builtin_bit_cast(uint64_t, d); }
LG_LIBM double dbits(uint64_t u) { return __builtin_bit_cast(double, u); }
LG_LIBM int32_t dhi(double d) { return (int32_t)(dbits_of(d) >> 32); }
LG_LIBM uint32_t dlo(double d) { return (uint32_t)dbits_of(d); }

// k_sin.c: sin(x + y) on |x| <= pi/4, y the tail of x (iy = 0: y is 0)
LG_LIBM double ksin_d(double x, double y, int iy) {
  const double S1 = dbits(0xBFC5555555555549ull), S2 = dbits(0x3F8111111110F8A6ull),
               S3 = dbits(0xBF2A01A019C161D5ull), S4 = dbits(0x3EC71DE357B1FE7Dull),
               S5 = dbits(0xBE5AE5E68A2B9CEBull), S6 = dbits(0x3DE5D93A5ACFD57Cull);
  const int32_t ix = dhi(x) & 0x7fffffff;
  if (ix < 0x3e400000) return x;  // |x| < 2^-27
  const double z = x * x;
  const double v = z * x;
  const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  if (iy == 0) return x + v * (S1 + z * r);
  return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}
// k_cos.c: cos(x + y) on |x| <= pi/4
LG_LIBM double kcos_d(double x, double y) {
  const double C1 = dbits(0x3FA555555555554Cull), C2 = dbits(0xBF56C16C16C15177ull),
               C3 = dbits(0x3EFA01A019CB1590ull), C4 = dbits(0xBE927E4F809C52ADull),
               C5 = dbits(0x3E21EE9EBDB4B1C4ull), C6 = dbits(0xBDA8FAE9BE8838D4ull);
  const int32_t ix = dhi(x) & 0x7fffffff;
  if (ix < 0x3e400000) return 1.0;  // |x| < 2^-27
  const double z = x * x;
  const double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
  if (ix < 0x3FD33333) return 1.0 - (0.5 * z - (z * r - x * y));  // |x| < 0.3
  const double qx = ix > 0x3fe90000 ? 0.28125 : dbits((uint64_t)(uint32_t)(ix - 0x00200000) << 32);  // x / 4
  const double hz = 0.5 * z - qx;
  const double a = 1.0 - qx;
  return a - (hz - (z * r - x * y));
}
// e_rem_pio2.c, medium size (|x| < 2^20 * pi/2): x = n * pi/2 + (y0 + y1), returns n
LG_LIBM int rem_pio2_d(double x, double& y0, double& y1) {
  const double invpio2 = dbits(0x3FE45F306DC9C883ull), pio2_1 = dbits(0x3FF921FB54400000ull),
               pio2_1t = dbits(0x3DD0B4611A626331ull), pio2_2 = dbits(0x3DD0B4611A600000ull),
               pio2_2t = dbits(0x3BA3198A2E037073ull), pio2_3 = dbits(0x3BA3198A2E000000ull),
               pio2_3t = dbits(0x397B839A252049C1ull);
  const int32_t hx = dhi(x), ix = hx & 0x7fffffff;
  const double t0 = fabs(x);
  const int n = (int)(t0 * invpio2 + 0.5);
  const double fn = (double)n;
  double r = t0 - fn * pio2_1;
  double w = fn * pio2_1t;  // 1st round good to 85 bits
  const int j = ix >> 20;
  y0 = r - w;
  int i = j - ((dhi(y0) >> 20) & 0x7ff);
  if (i > 16) {  // 2nd iteration, good to 118 bits
    double t = r;
    w = fn * pio2_2;
    r = t - w;
    w = fn * pio2_2t - ((t - r) - w);
    y0 = r - w;
    i = j - ((dhi(y0) >> 20) & 0x7ff);
    if (i > 49) {  // 3rd iteration, 151 bits
      t = r;
      w = fn * pio2_3;
      r = t - w;
      w = fn * pio2_3t - ((t - r) - w);
      y0 = r - w;
    }
  }
  y1 = (r - y0) - w;
  if (hx < 0) {
    y0 = -y0;
    y1 = -y1;
    return -n;
  }
  return n;
}
LG_LIBM double sin_d(double x) {  // s_sin.c
  const int32_t ix = dhi(x) & 0x7fffffff;
  if (ix <= 0x3fe921fb) return ksin_d(x, 0.0, 0);
  if (ix >= 0x7ff00000) return x - x;
  if (ix >= 0x413921fb) return sin_big(x);  // |x| >= 2^20 * pi/2: never an angle here
  double y0, y1;
  const int n = rem_pio2_d(x, y0, y1);
  switch (n & 3) {
    case 0: return ksin_d(y0, y1, 1);
    case 1: return kcos_d(y0, y1);
    case 2: return -ksin_d(y0, y1, 1);
    default: return -kcos_d(y0, y1);
  }
}
LG_LIBM double cos_d(double x) {  // s_cos.c
  const int32_t ix = dhi(x) & 0x7fffffff;
  if (ix <= 0x3fe921fb) return kcos_d(x, 0.0);
  if (ix >= 0x7ff00000) return x - x;
  if (ix >= 0x413921fb) return cos_big(x);
  double y0, y1;
  const int n = rem_pio2_d(x, y0, y1);
  switch (n & 3) {
    case 0: return kcos_d(y0, y1);
    case 1: return -ksin_d(y0, y1, 1);
    case 2: return -kcos_d(y0, y1);
    default: return ksin_d(y0, y1, 1);
  }
}
LG_LIBM double atan_d(double x) {  // s_atan.c
  const double atanhi0 = dbits(0x3FDDAC670561BB4Full), atanhi1 = dbits(0x3FE921FB54442D18ull),
               atanhi2 = dbits(0x3FEF730BD281F69Bull), atanhi3 = dbits(0x3FF921FB54442D18ull);
  const double atanlo0 = dbits(0x3C7A2B7F222F65E2ull), atanlo1 = dbits(0x3C81A62633145C07ull),
               atanlo2 = dbits(0x3C7007887AF0CBBDull), atanlo3 = dbits(0x3C91A62633145C07ull);
  const double aT0 = dbits(0x3FD555555555550Dull), aT1 = dbits(0xBFC999999998EBC4ull),
               aT2 = dbits(0x3FC24924920083FFull), aT3 = dbits(0xBFBC71C6FE231671ull),
               aT4 = dbits(0x3FB745CDC54C206Eull), aT5 = dbits(0xBFB3B0F2AF749A6Dull),
               aT6 = dbits(0x3FB10D66A0D03D51ull), aT7 = dbits(0xBFADDE2D52DEFD9Aull),
               aT8 = dbits(0x3FA97B4B24760DEBull), aT9 = dbits(0xBFA2B4442C6A6C2Full),
               aT10 = dbits(0x3F90AD3AE322DA11ull);
  const int32_t hx = dhi(x), ix = hx & 0x7fffffff;
  int id;
  if (ix >= 0x44100000) {  // |x| >= 2^66
    if (ix > 0x7ff00000 || (ix == 0x7ff00000 && dlo(x) != 0)) return x + x;  // NaN
    return hx > 0 ? atanhi3 + atanlo3 : -atanhi3 - atanlo3;
  }
  if (ix < 0x3fdc0000) {  // |x| < 0.4375
    if (ix < 0x3e200000) return x;  // |x| < 2^-29
    id = -1;
  } else {
    x = fabs(x);
    if (ix < 0x3ff30000) {  // |x| < 1.1875
      if (ix < 0x3fe60000) { id = 0; x = (2.0 * x - 1.0) / (2.0 + x); }  // 7/16 <= |x| < 11/16
      else { id = 1; x = (x - 1.0) / (x + 1.0); }                        // 11/16 <= |x| < 19/16
    } else {
      if (ix < 0x40038000) { id = 2; x = (x - 1.5) / (1.0 + 1.5 * x); }  // |x| < 2.4375
      else { id = 3; x = -1.0 / x; }
    }
  }
  const double z = x * x;
  const double w = z * z;
  const double s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
  const double s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
  if (id < 0) return x - x * (s1 + s2);
  const double hi = id == 0 ? atanhi0 : id == 1 ? atanhi1 : id == 2 ? atanhi2 : atanhi3;
  const double lo = id == 0 ? atanlo0 : id == 1 ? atanlo1 : id == 2 ? atanlo2 : atanlo3;
  const double zz = hi - ((x * (s1 + s2) - lo) - x);
  return hx < 0 ? -zz : zz;
}
LG_LIBM double atan2_d(double y, double x) {  // e_atan2.c
  const double tiny = 1.0e-300, pi_o_4 = dbits(0x3FE921FB54442D18ull), pi_o_2 = dbits(0x3FF921FB54442D18ull),
               pi = dbits(0x400921FB54442D18ull), pi_lo = dbits(0x3CA1A62633145C07ull);
  const int32_t hx = dhi(x), hy = dhi(y);
  const uint32_t lx = dlo(x), ly = dlo(y);
  const int32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
  if (((uint32_t)ix | ((lx | (0u - lx)) >> 31)) > 0x7ff00000u ||
      ((uint32_t)iy | ((ly | (0u - ly)) >> 31)) > 0x7ff00000u)
    return x + y;  // NaN
  if (hx == 0x3ff00000 && lx == 0) return atan_d(y);  // x = 1.0
  const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);  // 2 * sign(x) + sign(y)
  if ((iy | (int32_t)ly) == 0) {
    switch (m) {
      case 0:
      case 1: return y;
      case 2: return pi + tiny;
      default: return -pi - tiny;
    }
  }
  if ((ix | (int32_t)lx) == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
  if (ix == 0x7ff00000) {
    if (iy == 0x7ff00000) {
      switch (m) {
        case 0: return pi_o_4 + tiny;
        case 1: return -pi_o_4 - tiny;
        case 2: return 3.0 * pi_o_4 + tiny;
        default: return -3.0 * pi_o_4 - tiny;
      }
    }
    switch (m) {
      case 0: return 0.0;
      case 1: return -0.0;
      case 2: return pi + tiny;
      default: return -pi - tiny;
    }
  }
  if (iy == 0x7ff00000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
  const int k = (iy - ix) >> 20;
  double z;
  if (k > 60) z = pi_o_2 + 0.5 * pi_lo;  // |y / x| > 2^60
  else if (hx < 0 && k < -60) z = 0.0;   // |y| / x < -2^60
  else z = atan_d(fabs(y / x));
  switch (m) {
    case 0: return z;
    case 1: return -z;
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
  }
}
LG_LIBM double asin_d(double x) {  // e_asin.c
  const double pio2_hi = dbits(0x3FF921FB54442D18ull), pio2_lo = dbits(0x3C91A62633145C07ull),
               pio4_hi = dbits(0x3FE921FB54442D18ull);
  const double pS0 = dbits(0x3FC5555555555555ull), pS1 = dbits(0xBFD4D61203EB6F7Dull),
               pS2 = dbits(0x3FC9C1550E884455ull), pS3 = dbits(0xBFA48228B5688F3Bull),
               pS4 = dbits(0x3F49EFE07501B288ull), pS5 = dbits(0x3F023DE10DFDF709ull),
               qS1 = dbits(0xC0033A271C8A2D4Bull), qS2 = dbits(0x40002AE59C598AC8ull),
               qS3 = dbits(0xBFE6066C1B8D0159ull), qS4 = dbits(0x3FB3B8C5B12E9282ull);
  const int32_t hx = dhi(x), ix = hx & 0x7fffffff;
  if (ix >= 0x3ff00000) {  // |x| >= 1
    if (((ix - 0x3ff00000) | (int32_t)dlo(x)) == 0) return x * pio2_hi + x * pio2_lo;
    return (x - x) / (x - x);
  }
  if (ix < 0x3fe00000) {  // |x| < 0.5
    if (ix < 0x3e400000) return x;
    const double t = x * x;
    const double p = t * (pS0 + t * (pS1 + t * (pS2 + t * (pS3 + t * (pS4 + t * pS5)))));
    const double q = 1.0 + t * (qS1 + t * (qS2 + t * (qS3 + t * qS4)));
    const double w = p / q;
    return x + x * w;
  }
  double w = 1.0 - fabs(x);
  double t = w * 0.5;
  double p = t * (pS0 + t * (pS1 + t * (pS2 + t * (pS3 + t * (pS4 + t * pS5)))));
  double q = 1.0 + t * (qS1 + t * (qS2 + t * (qS3 + t * qS4)));
  const double s = sqrt(t);
  if (ix >= 0x3FEF3333) {  // |x| > 0.975
    w = p / q;
    t = pio2_hi - (2.0 * (s + s * w) - pio2_lo);
  } else {
    w = dbits(dbits_of(s) & 0xffffffff00000000ull);
    const double c = (t - w * w) / (s + w);
    const double r = p / q;
    p = 2.0 * s * r - (pio2_lo - 2.0 * c);
    q = pio4_hi - 2.0 * w;
    t = pio4_hi - (p - q);
  }
  return hx > 0 ? t : -t;
}

// The two libm overload models behind one interface (float arguments, as the reference passes):
// Fp<false> = fp_mode 0 (float overloads: glibc's float functions), Fp<true> = fp_mode 1 (::sin(double)
// etc.).  T is the type the reference's expression is evaluated in.
template <bool kF1>
struct Fp;
template <>
struct Fp<false> {
  typedef float T;
  static LG_LIBM float sn(float x) { return sinf_g(x); }
  static LG_LIBM float cs(float x) { return cosf_g(x); }
  static LG_LIBM float at2(float y, float x) { return atan2f_g(y, x); }
  static LG_LIBM float as(float x) { return asinf_g(x); }
  static LG_LIBM float sq(float x) { return sqrtf(x); }
};
template <>
struct Fp<true> {
  typedef double T;
  static LG_LIBM double sn(double x) { return sin_d(x); }
  static LG_LIBM double cs(double x) { return cos_d(x); }
  static LG_LIBM double at2(double y, double x) { return atan2_d(y, x); }
  static LG_LIBM double as(double x) { return asin_d(x); }
  static LG_LIBM double sq(double x) { return sqrt(x); }
};

}  // namespace lg
