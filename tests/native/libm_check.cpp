// Checks lego_libm.h (the device's glibc asinf/atanf/atan2f restatement, compiled here for the
// host with the same float operations) against the host's glibc, bit for bit.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "lego_libm.h"

static uint64_t st = 0x243F6A8885A308D3ULL;
static uint64_t rnd() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; }
static uint32_t b(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float f(uint32_t u) { float x; memcpy(&x, &u, 4); return x; }
static bool eq(float a, float c) { return b(a) == b(c) || (std::isnan(a) && std::isnan(c)); }

int main(int argc, char** argv) {
  long n = argc > 1 ? atol(argv[1]) : 20000000;
  long bad = 0;
  for (long i = 0; i < n; ++i) {
    float x = f((uint32_t)rnd() & 0xbf7fffffu);  // |x| < 1 region and beyond
    if (!eq(asinf(x), lg::asinf_g(x))) bad++;
    float y = f((uint32_t)rnd());
    float z = f((uint32_t)rnd());
    if (!eq(atan2f(y, z), lg::atan2f_g(y, z))) bad++;
    if (!eq(atanf(y), lg::atanf_g(y))) bad++;
    // lidar-like magnitudes
    float px = (float)((int64_t)(rnd() % 200000) - 100000) / 1000.0f;
    float py = (float)((int64_t)(rnd() % 200000) - 100000) / 1000.0f;
    if (!eq(atan2f(px, py), lg::atan2f_g(px, py))) bad++;
    float r = std::sqrt(px * px + py * py + 1.0f);
    if (!eq(asinf(px / r), lg::asinf_g(px / r))) bad++;
  }
  const float special[] = {0.f, -0.f, 1.f, -1.f, 0.5f, -0.5f, INFINITY, -INFINITY, NAN, 1e-30f, -1e-30f, 2.f};
  for (float s1 : special)
    for (float s2 : special) {
      if (!eq(atan2f(s1, s2), lg::atan2f_g(s1, s2))) bad++;
      if (!eq(asinf(s1), lg::asinf_g(s1))) bad++;
    }
  printf("libm checked %ld samples, mismatches %ld\n", n, bad);
  return bad != 0;
}
