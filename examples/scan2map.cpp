// scan2map.cpp — MapOptimization::scan2MapOptimization through the C++ mirror (ScanToMapOptimization).
//
//   scan2map <problem.bin> [device]
// problem.bin: 4 clouds (laserCloudCornerLastDS, laserCloudSurfTotalLastDS, laserCloudCornerFromMapDS,
// laserCloudSurfFromMapDS), each int32 n then n x (float x, y, z, intensity); then float
// transformTobeMapped[6].  Prints "transform t0 .. t5 degenerate d ran r iterations i correspondences c
// status s".
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "lego_loam_amd.hpp"

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s problem.bin [device]\n", argv[0]);
    return 2;
  }
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<lego_point> clouds[4];
  for (auto& c : clouds) {
    int32_t n = 0;
    if (std::fread(&n, 4, 1, f) != 1 || n < 0) return 2;
    c.resize(n);
    if (n && std::fread(c.data(), sizeof(lego_point), n, f) != (size_t)n) return 2;
  }
  float t[6];
  if (std::fread(t, 4, 6, f) != 6) return 2;
  std::fclose(f);
  try {
    lego_amd::ScanToMapOptimization mo(argc > 2 ? std::atoi(argv[2]) : 0);
    for (int k = 0; k < 6; ++k) mo.transformTobeMapped[k] = t[k];  // transformAssociateToMap's result
    const auto info = mo.scan2MapOptimization(clouds[0], clouds[1], clouds[2], clouds[3]);
    std::printf("transform");
    for (int k = 0; k < 6; ++k) std::printf(" %.9g", mo.transformTobeMapped[k]);
    std::printf(" degenerate %d ran %d iterations %d correspondences %d status %d\n", mo.isDegenerate ? 1 : 0,
                info.ran ? 1 : 0, info.iterations, info.correspondences, info.status);
  } catch (const lego_amd::Error& e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 1;
  }
  return 0;
}
