// lego_loam_amd.hpp — C++ mirror of LeGO-LOAM-BOR's per-scan surfaces over the C-ABI.
//
// Same names, argument meaning and threading as the reference, minus ROS/PCL:
//   Channel<T>                  LeGO-LOAM/include/lego_loam/channel.h:11-56 (1 writer / 1 reader,
//                               blocking or non-blocking send)
//   ProjectionOut, AssociationOut  utility.h:64-80 (PCL clouds -> std::vector<lego_point>,
//                               cloud_msgs::cloud_info -> CloudInfo, nav_msgs::Odometry -> Odometry)
//   ImageProjection             imageProjection.h:9-16: ctor(params, output channel),
//                               cloudHandler(PointCloud2 view) -> sends one ProjectionOut
//   FeatureAssociation          featureAssociation.h:11-19: ctor(params, input channel, output
//                               channel) spawns the worker thread; dtor sends an empty item and joins
//                               (featureAssociation.cpp:87-94); every mapping_frequency_divider-th
//                               odometry cycle sends an AssociationOut (:1431-1448)
//   ScanToMapOptimization       mapOptimization.h / mapOptmization.cpp:1315-1332: scan2MapOptimization
//                               with the members it owns (transformTobeMapped, isDegenerate), over
//                               lego_s2m.h; the rest of MapOptimization (key frames, GTSAM, loop
//                               closure) stays with the caller
// Each stage owns its own GPU context (lego_ctx); all compute runs in the HIP kernels of
// liblego_frontend.so.  Header-only; link with -llego_frontend.  Errors throw lego_amd::Error
// (the C-ABI itself never throws).
#pragma once

#include <array>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "lego_frontend.h"
#include "lego_s2m.h"

namespace lego_amd {

struct Error : std::runtime_error {
  int code;
  Error(const std::string& what, int rc) : std::runtime_error(what + " (rc=" + std::to_string(rc) + ")"), code(rc) {}
};

inline void check(int rc, const char* what) {
  if (rc != LEGO_OK) throw Error(what, rc);
}

// channel.h:11-56, same contract
template <class T>
class Channel {
  T _item;
  bool _empty = true;
  bool _blocking_send;
  std::mutex _m;
  std::condition_variable _cv;

 public:
  explicit Channel(bool blocking_send) : _blocking_send(blocking_send) {}
  void send(T&& item) {
    std::unique_lock<std::mutex> lock(_m);
    if (_blocking_send) _cv.wait(lock, [&]() { return _empty; });
    _item = std::move(item);
    _empty = false;
    _cv.notify_all();
  }
  void receive(T& item) {
    std::unique_lock<std::mutex> lock(_m);
    _cv.wait(lock, [&]() { return !_empty; });
    item = std::move(_item);
    _empty = true;
    _cv.notify_all();
  }
};

typedef std::vector<lego_point> Cloud;  // pcl::PointCloud<PointXYZI>

// cloud_msgs/msg/cloud_info.msg
struct CloudInfo {
  double stamp = 0.0;
  std::vector<int32_t> startRingIndex, endRingIndex;
  float startOrientation = 0.f, endOrientation = 0.f, orientationDiff = 0.f;
  std::vector<uint8_t> segmentedCloudGroundFlag;
  std::vector<uint32_t> segmentedCloudColInd;
  std::vector<float> segmentedCloudRange;
};

// utility.h:64-70
struct ProjectionOut {
  bool valid = false;  // the destructor's empty item (featureAssociation.cpp:92) has valid == false
  Cloud segmented_cloud;
  Cloud outlier_cloud;
  CloudInfo seg_msg;
  Cloud scan_msg;
};

// nav_msgs::Odometry on /laser_odom_to_init (featureAssociation.cpp:1286-1298)
struct Odometry {
  double stamp = 0.0;
  double orientation[4] = {0, 0, 0, 1};  // x, y, z, w
  double position[3] = {0, 0, 0};
};

// utility.h:73-80
struct AssociationOut {
  bool valid = false;
  Cloud cloud_outlier_last, cloud_corner_last, cloud_surf_last;
  Odometry laser_odometry;
  Cloud scan_msg;
};

// sensor_msgs::PointCloud2, viewed zero-copy: x,y,z float32 at byte offsets within point_step
struct PointCloud2View {
  double stamp = 0.0;
  const void* data = nullptr;
  int32_t width = 0;  // number of points (height 1)
  int32_t point_step = 16;
  int32_t off_x = 0, off_y = 4, off_z = 8;
};

inline lego_params vlp16_params() {
  lego_params p;
  lego_params_vlp16(&p);
  return p;
}

class ImageProjection {
 public:
  ImageProjection(const lego_params& params, Channel<ProjectionOut>& output_channel, int device = 0)
      : _output_channel(output_channel), _V(params.num_vertical_scans) {
    check(lego_ctx_create(&params, device, &_ctx), "lego_ctx_create (ImageProjection)");
  }
  ~ImageProjection() { lego_ctx_destroy(_ctx); }
  ImageProjection(const ImageProjection&) = delete;
  ImageProjection& operator=(const ImageProjection&) = delete;

  // imageProjection.cpp:153-174 + publishClouds' hand-off (:538-547)
  void cloudHandler(const PointCloud2View& msg) {
    lego_projection_out o;
    check(lego_cloud_handler(_ctx, msg.data, msg.width, msg.point_step, msg.off_x, msg.off_y, msg.off_z, &o),
          "lego_cloud_handler");
    ProjectionOut out;
    out.valid = true;
    out.segmented_cloud.assign(o.segmented_cloud, o.segmented_cloud + o.n_segmented);
    out.outlier_cloud.assign(o.outlier_cloud, o.outlier_cloud + o.n_outlier);
    out.scan_msg.assign(o.scan_msg, o.scan_msg + o.n_scan);
    CloudInfo& ci = out.seg_msg;
    ci.stamp = msg.stamp;
    ci.startRingIndex.assign(o.start_ring_index, o.start_ring_index + _V);
    ci.endRingIndex.assign(o.end_ring_index, o.end_ring_index + _V);
    ci.startOrientation = o.start_orientation;
    ci.endOrientation = o.end_orientation;
    ci.orientationDiff = o.orientation_diff;
    ci.segmentedCloudGroundFlag.assign(o.segmented_cloud_ground_flag, o.segmented_cloud_ground_flag + o.n_segmented);
    ci.segmentedCloudColInd.assign(o.segmented_cloud_col_ind, o.segmented_cloud_col_ind + o.n_segmented);
    ci.segmentedCloudRange.assign(o.segmented_cloud_range, o.segmented_cloud_range + o.n_segmented);
    _output_channel.send(std::move(out));
  }

 private:
  lego_ctx* _ctx = nullptr;
  Channel<ProjectionOut>& _output_channel;
  int _V;
};

class FeatureAssociation {
 public:
  FeatureAssociation(const lego_params& params, Channel<ProjectionOut>& input_channel,
                     Channel<AssociationOut>& output_channel, int device = 0)
      : _input_channel(input_channel), _output_channel(output_channel) {
    check(lego_ctx_create(&params, device, &_ctx), "lego_ctx_create (FeatureAssociation)");
    _run_thread = std::thread(&FeatureAssociation::runFeatureAssociation, this);
  }
  ~FeatureAssociation() {  // featureAssociation.cpp:90-94
    _input_channel.send(ProjectionOut());
    _run_thread.join();
    lego_ctx_destroy(_ctx);
  }
  FeatureAssociation(const FeatureAssociation&) = delete;
  FeatureAssociation& operator=(const FeatureAssociation&) = delete;

  // latest odometry and status bits (publishOdometry's /laser_odom_to_init message)
  Odometry last_odometry() {
    std::lock_guard<std::mutex> g(_m);
    return _odom;
  }
  int last_status() {
    std::lock_guard<std::mutex> g(_m);
    return _status;
  }
  int cycles() {
    std::lock_guard<std::mutex> g(_m);
    return _n;
  }
  std::string error() {
    std::lock_guard<std::mutex> g(_m);
    return _error;
  }

 private:
  void runFeatureAssociation() {  // featureAssociation.cpp:1386-1450
    while (true) {
      ProjectionOut projection;
      _input_channel.receive(projection);
      if (!projection.valid) break;
      lego_projection_out in;
      const CloudInfo& ci = projection.seg_msg;
      in.n_segmented = (int32_t)projection.segmented_cloud.size();
      in.n_outlier = (int32_t)projection.outlier_cloud.size();
      in.n_scan = (int32_t)projection.scan_msg.size();
      in.segmented_cloud = projection.segmented_cloud.data();
      in.outlier_cloud = projection.outlier_cloud.data();
      in.scan_msg = projection.scan_msg.data();
      in.start_ring_index = ci.startRingIndex.data();
      in.end_ring_index = ci.endRingIndex.data();
      in.start_orientation = ci.startOrientation;
      in.end_orientation = ci.endOrientation;
      in.orientation_diff = ci.orientationDiff;
      in.segmented_cloud_ground_flag = ci.segmentedCloudGroundFlag.data();
      in.segmented_cloud_col_ind = ci.segmentedCloudColInd.data();
      in.segmented_cloud_range = ci.segmentedCloudRange.data();
      in.label_mat = nullptr;
      in.ground_mat = nullptr;
      in.range_mat = nullptr;
      lego_association_out o;
      const int rc = lego_feature_association_from(_ctx, &in, &o);
      std::lock_guard<std::mutex> g(_m);
      if (rc != LEGO_OK) {
        _error = "lego_feature_association_from rc=" + std::to_string(rc);
        continue;
      }
      _status = o.status;
      ++_n;
      if (o.status & LEGO_ST_INIT) continue;  // checkSystemInitialization: no odometry (:1414-1417)
      _odom.stamp = ci.stamp;
      for (int k = 0; k < 4; ++k) _odom.orientation[k] = o.odom_orientation[k];
      for (int k = 0; k < 3; ++k) _odom.position[k] = o.odom_position[k];
      if (o.status & LEGO_ST_EMITTED) {
        AssociationOut out;
        out.valid = true;
        out.cloud_corner_last.assign(o.cloud_corner_last, o.cloud_corner_last + o.n_corner_last);
        out.cloud_surf_last.assign(o.cloud_surf_last, o.cloud_surf_last + o.n_surf_last);
        out.cloud_outlier_last.assign(o.cloud_outlier_last, o.cloud_outlier_last + o.n_outlier_last);
        out.laser_odometry = _odom;
        out.scan_msg = projection.scan_msg;
        _output_channel.send(std::move(out));
      }
    }
  }

  lego_ctx* _ctx = nullptr;
  Channel<ProjectionOut>& _input_channel;
  Channel<AssociationOut>& _output_channel;
  std::thread _run_thread;
  std::mutex _m;
  Odometry _odom;
  int _status = 0;
  int _n = 0;
  std::string _error;
};

// MapOptimization's scan-to-map LM.  transformTobeMapped / isDegenerate are the reference's members
// (mapOptimization.h:208-210, 226): set transformTobeMapped (transformAssociateToMap) before the call,
// read it after; isDegenerate carries over between calls as the member does.
class ScanToMapOptimization {
 public:
  explicit ScanToMapOptimization(int device = 0, int max_map_points = 200000) {
    check(lego_s2m_create(device, 1, max_map_points, &_m), "lego_s2m_create");
  }
  ~ScanToMapOptimization() { lego_s2m_destroy(_m); }
  ScanToMapOptimization(const ScanToMapOptimization&) = delete;
  ScanToMapOptimization& operator=(const ScanToMapOptimization&) = delete;

  float transformTobeMapped[6] = {0, 0, 0, 0, 0, 0};
  bool isDegenerate = false;

  struct Info {
    bool ran;        // the :1316 gate passed (false: transform untouched, transformUpdate not due)
    int iterations;  // LMOptimization calls (<= 10)
    int correspondences;
    int status;      // LEGO_S2M_ST_*
  };
  // scan2MapOptimization (:1315-1332) on laserCloudCornerLastDS, laserCloudSurfTotalLastDS and the
  // surrounding map's laserCloudCornerFromMapDS / laserCloudSurfFromMapDS
  Info scan2MapOptimization(const std::vector<lego_point>& cornerLastDS, const std::vector<lego_point>& surfTotalLastDS,
                            const std::vector<lego_point>& cornerFromMapDS,
                            const std::vector<lego_point>& surfFromMapDS) {
    int32_t dg = isDegenerate ? 1 : 0, info[4];
    check(lego_s2m_run_host(_m, cornerLastDS.data(), (int32_t)cornerLastDS.size(), surfTotalLastDS.data(),
                            (int32_t)surfTotalLastDS.size(), cornerFromMapDS.data(), (int32_t)cornerFromMapDS.size(),
                            surfFromMapDS.data(), (int32_t)surfFromMapDS.size(), transformTobeMapped, &dg, info),
          "lego_s2m_run_host");
    if (info[0] < 0) throw Error("scan2MapOptimization: a map cloud exceeds max_map_points", LEGO_EINVAL);
    isDegenerate = dg != 0;
    return Info{info[0] == 1, info[1], info[2], info[3]};
  }

 private:
  lego_s2m* _m = nullptr;
};

// One pass of MapOptimization's mapping loop, loop closure off (mapOptmization.cpp:1521-1570), per call:
// OdometryToTransform, transformAssociateToMap, extractSurroundingKeyFrames, downsampleCurrentScan,
// scan2MapOptimization, saveKeyFramesAndFactor, with the key frames' clouds kept on the GPU.
// transformAftMapped is the reference's member after the pass.
class Mapper {
 public:
  explicit Mapper(int device = 0, int max_map_points = 200000, int64_t max_key_points = 50000000) {
    check(lego_mapper_create(device, max_map_points, max_key_points, &_m), "lego_mapper_create");
  }
  ~Mapper() { lego_mapper_destroy(_m); }
  Mapper(const Mapper&) = delete;
  Mapper& operator=(const Mapper&) = delete;

  float transformAftMapped[6] = {0, 0, 0, 0, 0, 0};

  ScanToMapOptimization::Info run(const Cloud& cornerLast, const Cloud& surfLast, const Cloud& outlierLast,
                                  const Odometry& laserOdometry) {
    float transformSum[6];
    check(lego_map_odometry_to_transform(laserOdometry.orientation, laserOdometry.position, transformSum),
          "lego_map_odometry_to_transform");  // OdometryToTransform (:1540)
    int32_t info[4];
    check(lego_mapper_step(_m, cornerLast.data(), (int32_t)cornerLast.size(), surfLast.data(), (int32_t)surfLast.size(),
                           outlierLast.data(), (int32_t)outlierLast.size(), transformSum, transformAftMapped, info),
          "lego_mapper_step");
    return ScanToMapOptimization::Info{info[0] == 1, info[1], info[2], info[3]};
  }
  // cloudKeyPoses6D: (roll, pitch, yaw, x, y, z) per key frame
  std::vector<std::array<float, 6>> keyPoses() const {
    int32_t n = 0;
    check(lego_mapper_key_poses(_m, nullptr, 0, &n), "lego_mapper_key_poses");
    std::vector<std::array<float, 6>> out(n);
    if (n) check(lego_mapper_key_poses(_m, out[0].data(), n, &n), "lego_mapper_key_poses");
    return out;
  }

 private:
  lego_mapper* _m = nullptr;
};

// publishTF's /aft_mapped_to_init pose (mapOptmization.cpp:510-522): tf::createQuaternionMsgFromRollPitchYaw
// in double, as FeatureAssociation::publishOdometry
inline Odometry aft_mapped_odometry(const float t[6], double stamp) {
  const double roll = t[2], pitch = -(double)t[0], yaw = -(double)t[1];
  const double hy = yaw * 0.5, hp = pitch * 0.5, hr = roll * 0.5;
  const double cy = std::cos(hy), sy = std::sin(hy), cp = std::cos(hp), sp = std::sin(hp), cr = std::cos(hr),
               sr = std::sin(hr);
  const double qx = sr * cp * cy - cr * sp * sy, qy = cr * sp * cy + sr * cp * sy;
  const double qz = cr * cp * sy - sr * sp * cy, qw = cr * cp * cy + sr * sp * sy;
  Odometry o;
  o.stamp = stamp;
  o.orientation[0] = -qy;
  o.orientation[1] = -qz;
  o.orientation[2] = qx;
  o.orientation[3] = qw;
  for (int k = 0; k < 3; ++k) o.position[k] = t[3 + k];
  return o;
}

// mapOptimization.h's surface: the constructor starts the mapping thread on input_channel (the
// AssociationOut channel FeatureAssociation feeds, main.cpp:38-45); the destructor sends the empty item
// and joins (:126-129).  Loop closure and the global-map publisher are not built (loop closure off).
class MapOptimization {
 public:
  MapOptimization(Channel<AssociationOut>& input_channel, int device = 0, int max_map_points = 200000,
                  int64_t max_key_points = 50000000)
      : _mapper(device, max_map_points, max_key_points), _input_channel(input_channel) {
    _run_thread = std::thread(&MapOptimization::run, this);
  }
  ~MapOptimization() { finish(); }
  // the destructor's hand-off: the empty item after everything already sent, then join (idempotent)
  void finish() {
    if (!_run_thread.joinable()) return;
    _input_channel.send(AssociationOut());
    _run_thread.join();
  }
  MapOptimization(const MapOptimization&) = delete;
  MapOptimization& operator=(const MapOptimization&) = delete;

  Odometry aft_mapped() {  // the last /aft_mapped_to_init
    std::lock_guard<std::mutex> g(_mtx);
    return _aft;
  }
  int cycles() {
    std::lock_guard<std::mutex> g(_mtx);
    return _n;
  }
  std::string error() {
    std::lock_guard<std::mutex> g(_mtx);
    return _error;
  }
  std::vector<std::array<float, 6>> keyPoses() {
    std::lock_guard<std::mutex> g(_mtx);
    return _mapper.keyPoses();
  }

 private:
  void run() {  // :1521-1570
    while (true) {
      AssociationOut association;
      _input_channel.receive(association);
      if (!association.valid) break;
      std::lock_guard<std::mutex> g(_mtx);
      try {
        _mapper.run(association.cloud_corner_last, association.cloud_surf_last, association.cloud_outlier_last,
                    association.laser_odometry);
        _aft = aft_mapped_odometry(_mapper.transformAftMapped, association.laser_odometry.stamp);  // publishTF
      } catch (const Error& e) {
        _error = e.what();
      }
      ++_n;
    }
  }

  Mapper _mapper;
  Channel<AssociationOut>& _input_channel;
  std::thread _run_thread;
  std::mutex _mtx;
  Odometry _aft;
  int _n = 0;
  std::string _error;
};

}  // namespace lego_amd
