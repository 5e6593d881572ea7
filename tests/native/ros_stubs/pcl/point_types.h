// test stub: pcl::PointXYZI (PCL 1.8: x, y, z in a 16-byte-aligned union with data[4], intensity)
#pragma once
namespace pcl {
struct alignas(16) PointXYZI {
  union {
    float data[4];
    struct { float x, y, z; };
  };
  union {
    struct { float intensity; };
    float data_c[4];
  };
};
}  // namespace pcl
