// fp_mode 1 libm: lego_libm.h's double sin / cos / atan2 / asin (fdlibm, as the device runs them) against
// the host's glibc double functions, which the reference calls when unqualified sin(float) etc. resolve
// to ::sin(double).  Reports, per function, how often the double results differ
// (last-bit disagreements between two < 1 ulp implementations: informational) and how often they
// differ after the rounding to float the reference applies when it stores the result (the parity
// figure: must be 0 on the sample).
//
// usage: libm_d_check [samples]   exit status 1 if any float-rounded mismatch
#ifndef _GNU_SOURCE
#define _GNU_SOURCE  // sincos
#endif
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <initializer_list>

#include "lego_libm.h"

static uint64_t st = 0x9E3779B97F4A7C15ULL;
static uint64_t rnd() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; }
static double u01() { return (double)(rnd() >> 11) * (1.0 / 9007199254740992.0); }
static uint64_t bd(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
static uint32_t bf(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

struct Count {
  const char* name;
  long n = 0, dbl = 0, flt = 0;
  void add(double g, double m) {
    ++n;
    if (bd(g) != bd(m) && !(std::isnan(g) && std::isnan(m))) ++dbl;
    const float gf = (float)g, mf = (float)m;
    if (bf(gf) != bf(mf) && !(std::isnan(gf) && std::isnan(mf))) {
      if (flt < 5) printf("  %s float mismatch: glibc %.17g lego %.17g\n", name, g, m);
      ++flt;
    }
  }
};

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 20000000;
  Count s{"sin"}, c{"cos"}, a2{"atan2"}, as{"asin"}, ori{"ori"}, gr{"ground"}, tg{"tang"};
  const double sA = sin((double)(float)(M_PI * 2 / 1800)), cA = cos((double)(float)(M_PI * 2 / 1800));
  for (long i = 0; i < n; ++i) {
    // LM / TransformToStart angles: s * transformCur (small) and transformSum (any heading)
    const float x = (float)((u01() * 2 - 1) * (i & 1 ? 0.05 : 3.5));
    double gs, gc;  // the reference's sin / cos pairs are one glibc sincos call (GCC's cse_sincos)
    sincos((double)x, &gs, &gc);
    s.add(gs, lg::sin_d(x));
    c.add(gc, lg::cos_d(x));
    // adjustDistortion: -atan2(point.x, point.z) of lidar points (featureAssociation.cpp:172)
    const float py = (float)((u01() * 2 - 1) * 80), px = (float)((u01() * 2 - 1) * 80);
    ori.add(-atan2((double)py, (double)px), -lg::atan2_d(py, px));
    const float ry = (float)(int32_t)rnd(), rx = (float)(int32_t)rnd();
    a2.add(atan2((double)ry, (double)rx), lg::atan2_d(ry, rx));
    // AccumulateRotation: -asin(srx) (:479)
    const float sx = (float)((u01() * 2 - 1) * (i & 2 ? 1.0 : 0.1));
    as.add(asin((double)sx), lg::asin_d(sx));
    // groundRemoval (imageProjection.cpp:278): atan2(dZ, sqrt(float sum)) in double
    const float dz = (float)((u01() * 2 - 1) * 2), dx = (float)((u01() * 2 - 1) * 2), dy = (float)(u01() * 0.5);
    const float s2 = dx * dx + dy * dy + dz * dz;
    gr.add(atan2((double)dz, sqrt((double)s2)), lg::atan2_d(dz, sqrt((double)s2)));
    // labelComponents (:463): exact double arithmetic with host constants: identical by construction
    const float d1 = (float)(1 + u01() * 60), d2 = (float)(u01() * 60);
    tg.add((double)d2 * sA / ((double)d1 - (double)d2 * cA), (double)d2 * sA / ((double)d1 - (double)d2 * cA));
  }
  const double sp[] = {0.0, -0.0, 1.0, -1.0, 0.5, -0.5, INFINITY, -INFINITY, NAN, 1e-300, 2.0, M_PI, -M_PI / 2};
  for (double p : sp) {
    s.add(sin(p), lg::sin_d(p));
    c.add(cos(p), lg::cos_d(p));
    as.add(asin(p), lg::asin_d(p));
    for (double q : sp) a2.add(atan2(p, q), lg::atan2_d(p, q));
  }
  long bad = 0;
  for (const Count* k : {&s, &c, &a2, &as, &ori, &gr, &tg}) {
    printf("%-7s samples %ld  double-result differences %ld (%.2e)  float-rounded differences %ld\n", k->name, k->n,
           k->dbl, (double)k->dbl / (double)k->n, k->flt);
    bad += k->flt;
  }
  return bad != 0;
}
