// replay_pipeline.cpp — the reference's main.cpp topology (LeGO-LOAM/src/main.cpp:37-47,72-95)
// without ROS: ImageProjection on the caller thread, FeatureAssociation on its own thread, joined by
// a blocking Channel<ProjectionOut>; AssociationOut goes to a non-blocking channel (live mode).
//
//   replay_pipeline <scans.bin | file.bag> [device] [topic] [--mapping]
// --mapping: MapOptimization on its own thread behind a blocking Channel<AssociationOut> (main.cpp's
// rosbag mode, use_rosbag = true) and a second line "mapping cycles <n> keys <k> aft x y z qx qy qz qw".
// scans.bin: int32 nscans, then per scan: int32 n, n x (float x, y, z, intensity).
// file.bag: a ROS bag v2.0; every sensor_msgs/PointCloud2 on `topic` (default /velodyne_points,
// the reference's pointCloudTopic, utility.h:28) is decoded zero-copy (lego_rosbag.hpp) and replayed
// in file order, as main.cpp:62-76 does with rosbag::View.
// Prints one line per run: "cycles <n> status <bits> position x y z orientation x y z w last <publishCloudsLast
// publications> emitted <AssociationOut hand-offs>".
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

#include "lego_loam_amd.hpp"
#include "lego_rosbag.hpp"

int main(int argc, char** argv) {
  bool mapping = false;
  for (int i = 1; i < argc; ++i)
    if (std::string(argv[i]) == "--mapping") {
      mapping = true;
      for (int j = i; j + 1 < argc; ++j) argv[j] = argv[j + 1];
      --argc;
      break;
    }
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s scans.bin|file.bag [device] [topic]\n", argv[0]);
    return 2;
  }
  const int device = argc > 2 ? std::atoi(argv[2]) : 0;
  const std::string path = argv[1], topic = argc > 3 ? argv[3] : "/velodyne_points";
  const bool is_bag = path.size() > 4 && path.compare(path.size() - 4, 4, ".bag") == 0;
  std::vector<std::vector<float>> scans;
  if (!is_bag) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return 2;
    int32_t nscans = 0;
    if (std::fread(&nscans, 4, 1, f) != 1) return 2;
    scans.resize(nscans);
    for (int i = 0; i < nscans; ++i) {
      int32_t n = 0;
      if (std::fread(&n, 4, 1, f) != 1) return 2;
      scans[i].resize((size_t)n * 4);
      if (n && std::fread(scans[i].data(), 16, n, f) != (size_t)n) return 2;
    }
    std::fclose(f);
  }

  using namespace lego_amd;
  lego_params params = vlp16_params();
  Channel<ProjectionOut> projection_out_channel(true);
  Channel<AssociationOut> association_out_channel(mapping);  // main.cpp:38: blocking in rosbag mode
  Odometry odom;
  int status = 0, cycles = 0, map_cycles = 0, keys = 0, n_last = 0, n_emit = 0;
  Odometry aft;
  try {
    ImageProjection IP(params, projection_out_channel, device);
    std::unique_ptr<MapOptimization> MO;
    if (mapping) MO.reset(new MapOptimization(association_out_channel, device, 200000, 20000000));
    FeatureAssociation FA(params, projection_out_channel, association_out_channel, device);
    int nscans = 0;
    if (is_bag) {  // rosbag replay loop (main.cpp:62-76)
      BagReader bag(path);
      bag.for_each(topic, [&](const BagMessage& m) {
        if (m.type != "sensor_msgs/PointCloud2") return;
        IP.cloudHandler(decode_pointcloud2(m));
        ++nscans;
      });
    } else {
      nscans = (int)scans.size();
      for (int i = 0; i < nscans; ++i) {
        PointCloud2View msg;
        msg.stamp = 0.1 * i;
        msg.data = scans[i].data();
        msg.width = (int32_t)(scans[i].size() / 4);
        IP.cloudHandler(msg);
      }
    }
    // hand the worker a sentinel after the last scan and wait for it (the dtor does the same)
    while (FA.cycles() < nscans && FA.error().empty()) std::this_thread::sleep_for(std::chrono::milliseconds(1));
    if (!FA.error().empty()) {
      std::fprintf(stderr, "%s\n", FA.error().c_str());
      return 1;
    }
    odom = FA.last_odometry();
    status = FA.last_status();
    cycles = FA.cycles();
    n_last = FA.clouds_last_published();
    n_emit = FA.emitted();
    if (MO) {
      MO->finish();  // every AssociationOut FA sent has been through the mapping loop
      if (!MO->error().empty()) {
        std::fprintf(stderr, "%s\n", MO->error().c_str());
        return 1;
      }
      map_cycles = MO->cycles();
      keys = (int)MO->keyPoses().size();
      aft = MO->aft_mapped();
    }
  } catch (const Error& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    return 1;
  } catch (const BagError& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    return 2;
  }
  std::printf("cycles %d status %d position %.9g %.9g %.9g orientation %.9g %.9g %.9g %.9g last %d emitted %d\n",
              cycles, status, odom.position[0], odom.position[1], odom.position[2], odom.orientation[0],
              odom.orientation[1], odom.orientation[2], odom.orientation[3], n_last, n_emit);
  if (mapping)
    std::printf("mapping cycles %d keys %d aft %.9g %.9g %.9g %.9g %.9g %.9g %.9g\n", map_cycles, keys, aft.position[0],
                aft.position[1], aft.position[2], aft.orientation[0], aft.orientation[1], aft.orientation[2],
                aft.orientation[3]);
  return 0;
}
