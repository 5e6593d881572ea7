// bag_tool.cpp — package sweeps as a ROS bag and inspect bags (include/lego_rosbag.hpp).
//
//   bag_tool write <scans.bin> <out.bag> [topic]   scans.bin as replay_pipeline reads it; one
//                                                  PointCloud2 per scan, stamps 0.1 s apart
//   bag_tool info  <in.bag> [topic]                per topic: type and message count; for the
//                                                  PointCloud2 topic: points of every message
//   bag_tool dump  <in.bag> <out.bin> [topic]      decode every PointCloud2 back to scans.bin (x, y, z
//                                                  at the message's field offsets, intensity 0)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "lego_rosbag.hpp"

using namespace lego_amd;

static std::vector<std::vector<float>> read_scans(const char* path) {
  std::vector<std::vector<float>> scans;
  FILE* f = std::fopen(path, "rb");
  if (!f) throw BagError(std::string("cannot open ") + path);
  int32_t ns = 0;
  if (std::fread(&ns, 4, 1, f) != 1) throw BagError("bad scans file");
  scans.resize(ns);
  for (auto& s : scans) {
    int32_t n = 0;
    if (std::fread(&n, 4, 1, f) != 1) throw BagError("bad scans file");
    s.resize((size_t)n * 4);
    if (n && std::fread(s.data(), 16, n, f) != (size_t)n) throw BagError("bad scans file");
  }
  std::fclose(f);
  return scans;
}

int main(int argc, char** argv) {
  try {
    if (argc >= 4 && !std::strcmp(argv[1], "write")) {
      const auto scans = read_scans(argv[2]);
      BagWriter w(argv[3], argc > 4 ? argv[4] : "/velodyne_points");
      for (size_t i = 0; i < scans.size(); ++i) w.write(1000.0 + 0.1 * i, scans[i].data(), (int32_t)(scans[i].size() / 4));
      w.close();
      std::printf("wrote %zu messages\n", scans.size());
      return 0;
    }
    if (argc >= 3 && !std::strcmp(argv[1], "info")) {
      BagReader bag(argv[2]);
      std::map<std::string, std::pair<std::string, int>> count;
      std::vector<int> pts;
      const std::string want = argc > 3 ? argv[3] : "/velodyne_points";
      bag.for_each("", [&](const BagMessage& m) {
        auto& c = count[m.topic];
        c.first = m.type;
        c.second++;
        if (m.topic == want && m.type == "sensor_msgs/PointCloud2") pts.push_back(decode_pointcloud2(m).width);
      });
      for (const auto& c : count) std::printf("topic %s type %s messages %d\n", c.first.c_str(), c.second.first.c_str(), c.second.second);
      std::printf("points");
      for (int n : pts) std::printf(" %d", n);
      std::printf("\n");
      return 0;
    }
    if (argc >= 4 && !std::strcmp(argv[1], "dump")) {
      BagReader bag(argv[2]);
      std::vector<std::vector<float>> scans;
      bag.for_each(argc > 4 ? argv[4] : "/velodyne_points", [&](const BagMessage& m) {
        if (m.type != "sensor_msgs/PointCloud2") return;
        const PointCloud2View v = decode_pointcloud2(m);
        std::vector<float> s((size_t)v.width * 4, 0.f);
        const uint8_t* d = (const uint8_t*)v.data;
        for (int i = 0; i < v.width; ++i) {
          std::memcpy(&s[4 * i + 0], d + (size_t)i * v.point_step + v.off_x, 4);
          std::memcpy(&s[4 * i + 1], d + (size_t)i * v.point_step + v.off_y, 4);
          std::memcpy(&s[4 * i + 2], d + (size_t)i * v.point_step + v.off_z, 4);
        }
        scans.push_back(std::move(s));
      });
      FILE* f = std::fopen(argv[3], "wb");
      if (!f) return 2;
      const int32_t ns = (int32_t)scans.size();
      std::fwrite(&ns, 4, 1, f);
      for (const auto& s : scans) {
        const int32_t n = (int32_t)(s.size() / 4);
        std::fwrite(&n, 4, 1, f);
        std::fwrite(s.data(), 16, n, f);
      }
      std::fclose(f);
      return 0;
    }
  } catch (const BagError& e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 1;
  }
  std::fprintf(stderr, "usage: bag_tool write scans.bin out.bag [topic] | info in.bag [topic] | dump in.bag out.bin [topic]\n");
  return 2;
}
