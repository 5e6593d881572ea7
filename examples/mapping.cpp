// mapping.cpp — MapOptimization's mapping loop (loop closure off) through the C++ mirror (Mapper, one pass
// per call).
//
//   mapping <cycles.bin> [device]
// cycles.bin: int32 cycle count, then per cycle 3 clouds (laserCloudCornerLast, laserCloudSurfLast,
// laserCloudOutlierLast), each int32 n then n x (float x, y, z, intensity), then the odometry message:
// double orientation x, y, z, w and position x, y, z (AssociationOut.laser_odometry).
// Prints one line per cycle, "aft t0 .. t5 ran r iterations i", then "keys n".
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "lego_loam_amd.hpp"

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s cycles.bin [device]\n", argv[0]);
    return 2;
  }
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  int32_t cycles = 0;
  if (std::fread(&cycles, 4, 1, f) != 1 || cycles < 0) return 2;
  try {
    lego_amd::Mapper mo(argc > 2 ? std::atoi(argv[2]) : 0, 150000, 8000000);
    for (int32_t c = 0; c < cycles; ++c) {
      std::vector<lego_point> clouds[3];
      for (auto& v : clouds) {
        int32_t n = 0;
        if (std::fread(&n, 4, 1, f) != 1 || n < 0) return 2;
        v.resize(n);
        if (n && std::fread(v.data(), sizeof(lego_point), n, f) != (size_t)n) return 2;
      }
      lego_amd::Odometry odom;
      if (std::fread(odom.orientation, 8, 4, f) != 4 || std::fread(odom.position, 8, 3, f) != 3) return 2;
      const auto info = mo.run(clouds[0], clouds[1], clouds[2], odom);
      std::printf("aft");
      for (int k = 0; k < 6; ++k) std::printf(" %.9g", mo.transformAftMapped[k]);
      std::printf(" ran %d iterations %d\n", info.ran ? 1 : 0, info.iterations);
    }
    std::printf("keys %zu\n", mo.keyPoses().size());
  } catch (const lego_amd::Error& e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 1;
  }
  std::fclose(f);
  return 0;
}
