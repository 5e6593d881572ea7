// CPU checks of include/lego_loam_amd.hpp's message helpers (the pieces ros/lego_nodes.cpp uses between a
// ROS message and the C-ABI): xyz_offsets, packed_rows, fill_cloud_info, projection_in and
// FeatureAssociationCycle's publication decisions.  Prints "ok" and exits 0, or names the first failure.
#include <cstdio>
#include <string>
#include <vector>

#include "lego_loam_amd.hpp"

using namespace lego_amd;

#define CHECK(c)                                                     \
  do {                                                               \
    if (!(c)) {                                                      \
      std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);        \
      return 1;                                                      \
    }                                                                \
  } while (0)

struct Field {  // sensor_msgs::PointField's members
  std::string name;
  uint32_t offset;
  uint8_t datatype;
  uint32_t count;
};

int main() {
  // x / y / z offsets: float32 fields by name, others ignored; missing fields and big-endian rejected
  {
    std::vector<Field> f = {{"x", 0, 7, 1}, {"y", 4, 7, 1}, {"z", 8, 7, 1}, {"intensity", 16, 7, 1}, {"ring", 20, 4, 1}};
    int ox, oy, oz;
    CHECK(xyz_offsets(f, false, ox, oy, oz) && ox == 0 && oy == 4 && oz == 8);
    CHECK(!xyz_offsets(f, true, ox, oy, oz));
    std::vector<Field> g = {{"z", 12, 7, 1}, {"x", 4, 7, 1}, {"y", 8, 7, 1}};
    CHECK(xyz_offsets(g, false, ox, oy, oz) && ox == 4 && oy == 8 && oz == 12);
    std::vector<Field> h = {{"x", 0, 7, 1}, {"y", 4, 8, 1}, {"z", 8, 7, 1}};  // y as float64
    CHECK(!xyz_offsets(h, false, ox, oy, oz));
    std::vector<Field> k = {{"x", 0, 7, 3}, {"y", 4, 7, 1}, {"z", 8, 7, 1}};  // x with count 3
    CHECK(!xyz_offsets(k, false, ox, oy, oz));
  }
  // padded rows packed; unpadded or single-row payloads passed through
  {
    const uint32_t w = 3, hgt = 2, ps = 4, rs = 16;
    std::vector<uint8_t> d(rs * hgt, 0xee), buf;
    for (uint32_t r = 0; r < hgt; ++r)
      for (uint32_t i = 0; i < w * ps; ++i) d[r * rs + i] = (uint8_t)(r * 100 + i);
    const uint8_t* p = packed_rows(d.data(), w, hgt, ps, rs, buf);
    CHECK(p == buf.data() && buf.size() == w * ps * hgt);
    for (uint32_t r = 0; r < hgt; ++r)
      for (uint32_t i = 0; i < w * ps; ++i) CHECK(p[r * w * ps + i] == (uint8_t)(r * 100 + i));
    CHECK(packed_rows(d.data(), w, hgt, ps, w * ps, buf) == d.data());
    CHECK(packed_rows(d.data(), w, 1, ps, rs, buf) == d.data());
  }
  // cloud_info from the C-ABI view: trimmed and V*H with a zero tail; projection_in inverts it
  {
    const int V = 2, VH = 8, M = 3;
    int32_t sr[V] = {4, 5}, er[V] = {7, 9};
    uint8_t gf[M] = {1, 0, 1};
    uint32_t col[M] = {10, 11, 12};
    float rng[M] = {1.5f, 2.5f, 3.5f};
    lego_point seg[M] = {{1, 2, 3, 4}, {5, 6, 7, 8}, {9, 10, 11, 12}};
    lego_projection_out o;
    std::memset(&o, 0, sizeof(o));
    o.n_segmented = M;
    o.segmented_cloud = seg;
    o.start_ring_index = sr;
    o.end_ring_index = er;
    o.start_orientation = -1.f;
    o.end_orientation = 5.f;
    o.orientation_diff = 6.f;
    o.segmented_cloud_ground_flag = gf;
    o.segmented_cloud_col_ind = col;
    o.segmented_cloud_range = rng;
    CloudInfo a, b;
    fill_cloud_info(o, V, VH, false, a);
    fill_cloud_info(o, V, VH, true, b);
    CHECK(a.segmentedCloudRange.size() == (size_t)M && b.segmentedCloudRange.size() == (size_t)VH);
    CHECK(b.segmentedCloudColInd[M - 1] == 12 && b.segmentedCloudColInd[M] == 0 && b.segmentedCloudGroundFlag[VH - 1] == 0);
    CHECK(a.startRingIndex.size() == (size_t)V && a.endRingIndex[1] == 9 && a.orientationDiff == 6.f);
    lego_projection_out in;
    CHECK(projection_in(seg, M, nullptr, 0, nullptr, 0, b, V, in));
    CHECK(in.n_segmented == M && in.segmented_cloud_col_ind[2] == 12 && in.segmented_cloud_ground_flag[0] == 1 &&
          in.start_ring_index[1] == 5 && in.end_orientation == 5.f && !in.label_mat);
    CloudInfo bad = a;
    bad.segmentedCloudRange.pop_back();
    CHECK(!projection_in(seg, M, nullptr, 0, nullptr, 0, bad, V, in));
    bad = a;
    bad.endRingIndex.pop_back();
    CHECK(!projection_in(seg, M, nullptr, 0, nullptr, 0, bad, V, in));
  }
  // publication decisions: nothing but the features on the initialisation scan, odometry every cycle,
  // publishCloudsLast every second cycle (frameCount from skipFrameNum = 1), the hand-off on EMITTED
  {
    FeatureAssociationCycle c;
    FeatureAssociationCycle::Decision d = c.next(LEGO_ST_INIT);
    CHECK(d.init && !d.odometry && !d.clouds_last && !d.emit);
    const bool last[6] = {true, false, true, false, true, false};
    for (int k = 0; k < 6; ++k) {
      d = c.next(k == 4 ? LEGO_ST_EMITTED : 0);
      CHECK(!d.init && d.odometry && d.clouds_last == last[k] && d.emit == (k == 4));
    }
    d = c.next(LEGO_ST_INIT | LEGO_ST_EMITTED);  // no hand-off without odometry
    CHECK(d.init && !d.emit && !d.clouds_last);
  }
  std::printf("ok\n");
  return 0;
}
