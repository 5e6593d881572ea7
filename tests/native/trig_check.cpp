// sinf_g / cosf_g (LM trig, lego_libm.h) against the host: float(sin(double x)) on a sweep of all
// float arguments in [-pi/4, pi/4].
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstdint>
#include <cstring>
#include "lego_libm.h"
int main(int argc, char** argv) {
  const uint32_t stride = argc > 1 ? (uint32_t)atoi(argv[1]) : 7;
  // exhaustive over float bit patterns in [-pi/4, pi/4] stepping (every 7th) : compare with (float)sin((double)x)
  long n = 0, bad_s = 0, bad_c = 0;
  for (uint32_t u = 0; u < 0x3f490fdbu; u += stride) {
    for (int sg = 0; sg < 2; ++sg) {
      uint32_t b = u | (sg ? 0x80000000u : 0); float x; memcpy(&x, &b, 4);
      float a = lg::sinf_g(x), e = (float)sin((double)x);
      float c = lg::cosf_g(x), f = (float)cos((double)x);
      if (memcmp(&a, &e, 4)) bad_s++;
      if (memcmp(&c, &f, 4)) bad_c++;
      n++;
    }
  }
  printf("n=%ld sin mismatches %ld cos mismatches %ld\n", n, bad_s, bad_c);
  return (bad_s + bad_c) * 1000000L > n;  // <= 1 per million: double-rounding cases only
}
