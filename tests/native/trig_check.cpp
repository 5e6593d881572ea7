// sinf_g / cosf_g (lego_libm.h: glibc 2.35's sinf / cosf, FMA variant, restated for the device) against
// the host's glibc, bit for bit, on every stride-th float in [-120, 120] (stride 1: exhaustive).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "lego_libm.h"

int main(int argc, char** argv) {
  const uint32_t stride = argc > 1 ? (uint32_t)atoi(argv[1]) : 7;
  long n = 0, bad_s = 0, bad_c = 0;
  for (uint32_t u = 0; u < 0x42f00000u; u += stride) {  // 0x42f00000 = 120.0f
    for (int sg = 0; sg < 2; ++sg) {
      const uint32_t b = u | (sg ? 0x80000000u : 0);
      float x;
      memcpy(&x, &b, 4);
      const float a = lg::sinf_g(x), e = sinf(x);
      const float c = lg::cosf_g(x), f = cosf(x);
      if (memcmp(&a, &e, 4)) bad_s++;
      if (memcmp(&c, &f, 4)) bad_c++;
      n++;
    }
  }
  printf("n=%ld sin mismatches %ld cos mismatches %ld\n", n, bad_s, bad_c);
  return bad_s + bad_c != 0;
}
