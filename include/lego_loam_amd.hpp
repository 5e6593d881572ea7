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
#include <cstring>
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

// ---- Pieces shared by the classes below and the ROS node (ros/lego_nodes.cpp) ----------------------
// Everything between a ROS message and the C-ABI that is not a field-by-field copy lives here, so the
// ROS translation unit keeps only message conversion and publishing (tests/native/mirror_check.cpp,
// tests/test_cpp_mirror.py).

constexpr int kPointFieldFloat32 = 7;  // sensor_msgs::PointField::FLOAT32

// fromROSMsg's x / y / z (imageProjection.cpp:159): the byte offsets of the float32 fields named x, y
// and z in any container of fields with name / offset / datatype / count (sensor_msgs::PointField).
// False when one is missing or the payload is big-endian.
template <class Fields>
bool xyz_offsets(const Fields& fields, bool big_endian, int& ox, int& oy, int& oz) {
  ox = oy = oz = -1;
  for (const auto& f : fields) {
    if ((int)f.datatype != kPointFieldFloat32 || f.count != 1) continue;
    if (f.name == "x") ox = (int)f.offset;
    else if (f.name == "y") oy = (int)f.offset;
    else if (f.name == "z") oz = (int)f.offset;
  }
  return ox >= 0 && oy >= 0 && oz >= 0 && !big_endian;
}

// A PointCloud2 payload as lego_cloud_handler takes it (width * height points of point_step bytes,
// back to back): rows with padding (row_step > width * point_step) are packed into buf.
inline const uint8_t* packed_rows(const uint8_t* data, uint32_t width, uint32_t height, uint32_t point_step,
                                  uint32_t row_step, std::vector<uint8_t>& buf) {
  const size_t row = (size_t)width * point_step;
  if (height <= 1 || row_step == row) return data;
  buf.resize(row * height);
  for (uint32_t r = 0; r < height; ++r) std::memcpy(&buf[row * r], data + (size_t)row_step * r, row);
  return buf.data();
}

// publishClouds' cloud_info (imageProjection.cpp:498-536) from the C-ABI's view into any type with the
// cloud_info fields (cloud_msgs::cloud_info or CloudInfo): the per-point arrays either trimmed to the
// segmented cloud or, as the reference's resetParameters leaves them (:137-139), V * H entries with a
// zero tail.
template <class Info>
void fill_cloud_info(const lego_projection_out& o, int V, int VH, bool full, Info& s) {
  s.startRingIndex.assign(o.start_ring_index, o.start_ring_index + V);
  s.endRingIndex.assign(o.end_ring_index, o.end_ring_index + V);
  s.startOrientation = o.start_orientation;
  s.endOrientation = o.end_orientation;
  s.orientationDiff = o.orientation_diff;
  const int n = full ? VH : o.n_segmented;
  s.segmentedCloudGroundFlag.assign(n, 0);
  s.segmentedCloudColInd.assign(n, 0);
  s.segmentedCloudRange.assign(n, 0);
  for (int i = 0; i < o.n_segmented && i < n; ++i) {
    s.segmentedCloudGroundFlag[i] = o.segmented_cloud_ground_flag[i] != 0;
    s.segmentedCloudColInd[i] = o.segmented_cloud_col_ind[i];
    s.segmentedCloudRange[i] = o.segmented_cloud_range[i];
  }
}

// runFeatureAssociation's input (featureAssociation.cpp:1394-1407): a ProjectionOut's clouds and
// cloud_info as the C-ABI's view (lego_feature_association_from).  False for a malformed cloud_info
// (arrays shorter than the segmented cloud, ring indices shorter than V): the scan is dropped.
template <class Info>
bool projection_in(const lego_point* seg, int M, const lego_point* outl, int n_outlier, const lego_point* scan,
                   int n_scan, const Info& si, int V, lego_projection_out& in) {
  if ((int)si.segmentedCloudGroundFlag.size() < M || (int)si.segmentedCloudColInd.size() < M ||
      (int)si.segmentedCloudRange.size() < M || (int)si.startRingIndex.size() < V || (int)si.endRingIndex.size() < V)
    return false;
  in.n_segmented = M;
  in.n_outlier = n_outlier;
  in.n_scan = n_scan;
  in.segmented_cloud = seg;
  in.outlier_cloud = outl;
  in.scan_msg = scan;
  in.start_ring_index = si.startRingIndex.data();
  in.end_ring_index = si.endRingIndex.data();
  in.start_orientation = si.startOrientation;
  in.end_orientation = si.endOrientation;
  in.orientation_diff = si.orientationDiff;
  in.segmented_cloud_ground_flag = reinterpret_cast<const uint8_t*>(si.segmentedCloudGroundFlag.data());
  in.segmented_cloud_col_ind = si.segmentedCloudColInd.data();
  in.segmented_cloud_range = si.segmentedCloudRange.data();
  in.label_mat = nullptr;
  in.ground_mat = nullptr;
  in.range_mat = nullptr;
  return true;
}

// What one runFeatureAssociation cycle (featureAssociation.cpp:1408-1450) publishes after the GPU
// association, from its status bits: the feature clouds always (:1410), nothing else on the
// initialisation scan (checkSystemInitialization, :1413-1416), otherwise the odometry (:1422),
// publishCloudsLast's clouds every skipFrameNum + 1-th time (:1362-1382, frameCount starting at
// skipFrameNum = 1) and the AssociationOut on mapping cycles (:1431-1448, LEGO_ST_EMITTED).
class FeatureAssociationCycle {
 public:
  struct Decision {
    bool init, odometry, clouds_last, emit;
  };
  Decision next(int status) {
    Decision d;
    d.init = (status & LEGO_ST_INIT) != 0;
    d.odometry = !d.init;
    d.clouds_last = false;
    if (!d.init && ++_frame_count >= kSkipFrameNum + 1) {
      _frame_count = 0;
      d.clouds_last = true;
    }
    d.emit = !d.init && (status & LEGO_ST_EMITTED) != 0;
    return d;
  }

 private:
  static constexpr int kSkipFrameNum = 1;  // featureAssociation.cpp:132
  int _frame_count = kSkipFrameNum;
};

// runFeatureAssociation's loop (featureAssociation.cpp:1386-1450) over a Channel of ProjectionOut-like
// items, for the C++ mirror and the ROS node alike.  The sink converts and publishes:
//   bool end(const In&)                                  the destructor's empty item ends the loop
//   bool view(const In&, lego_projection_out&)           the C-ABI view (projection_in); false: drop
//   void dropped(const char* why, int rc)
//   void features(const In&, const lego_association_out&)     publishClouds (:1410)
//   void odometry(const In&, const lego_association_out&)     publishOdometry (:1422)
//   void clouds_last(const In&, const lego_association_out&)  publishCloudsLast's publication (:1424)
//   void emit(const In&, const lego_association_out&)         the AssociationOut hand-off (:1448)
template <class In, class Chan, class Sink>
void run_feature_association(lego_ctx* ctx, Chan& input, Sink& sink) {
  FeatureAssociationCycle cycle;
  while (true) {
    In projection;
    input.receive(projection);
    if (sink.end(projection)) break;
    lego_projection_out in;
    if (!sink.view(projection, in)) {
      sink.dropped("malformed cloud_info", LEGO_EINVAL);
      continue;
    }
    lego_association_out o;
    const int rc = lego_feature_association_from(ctx, &in, &o);
    if (rc != LEGO_OK) {
      sink.dropped("lego_feature_association_from", rc);
      continue;
    }
    const FeatureAssociationCycle::Decision d = cycle.next(o.status);
    sink.features(projection, o);
    if (d.init) continue;
    sink.odometry(projection, o);
    if (d.clouds_last) sink.clouds_last(projection, o);
    if (d.emit) sink.emit(projection, o);
  }
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
    out.seg_msg.stamp = msg.stamp;
    fill_cloud_info(o, _V, 0, false, out.seg_msg);
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
      : _input_channel(input_channel), _output_channel(output_channel), _V(params.num_vertical_scans) {
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
  // publishCloudsLast publications and AssociationOut hand-offs so far
  int clouds_last_published() {
    std::lock_guard<std::mutex> g(_m);
    return _n_last;
  }
  int emitted() {
    std::lock_guard<std::mutex> g(_m);
    return _n_emit;
  }
  std::string error() {
    std::lock_guard<std::mutex> g(_m);
    return _error;
  }

 private:
  struct Sink {  // this mirror's conversions: the clouds are std::vector<lego_point> already
    FeatureAssociation& fa;
    bool end(const ProjectionOut& p) { return !p.valid; }
    bool view(const ProjectionOut& p, lego_projection_out& in) {
      return projection_in(p.segmented_cloud.data(), (int)p.segmented_cloud.size(), p.outlier_cloud.data(),
                           (int)p.outlier_cloud.size(), p.scan_msg.data(), (int)p.scan_msg.size(), p.seg_msg, fa._V, in);
    }
    void dropped(const char* why, int rc) {
      std::lock_guard<std::mutex> g(fa._m);
      fa._error = std::string(why) + " rc=" + std::to_string(rc);
    }
    void features(const ProjectionOut&, const lego_association_out& o) {
      std::lock_guard<std::mutex> g(fa._m);
      fa._status = o.status;
      ++fa._n;
    }
    void odometry(const ProjectionOut& p, const lego_association_out& o) {
      std::lock_guard<std::mutex> g(fa._m);
      fa._odom.stamp = p.seg_msg.stamp;
      for (int k = 0; k < 4; ++k) fa._odom.orientation[k] = o.odom_orientation[k];
      for (int k = 0; k < 3; ++k) fa._odom.position[k] = o.odom_position[k];
    }
    void clouds_last(const ProjectionOut&, const lego_association_out&) {
      std::lock_guard<std::mutex> g(fa._m);
      ++fa._n_last;
    }
    void emit(const ProjectionOut& p, const lego_association_out& o) {
      AssociationOut out;
      out.valid = true;
      out.cloud_corner_last.assign(o.cloud_corner_last, o.cloud_corner_last + o.n_corner_last);
      out.cloud_surf_last.assign(o.cloud_surf_last, o.cloud_surf_last + o.n_surf_last);
      out.cloud_outlier_last.assign(o.cloud_outlier_last, o.cloud_outlier_last + o.n_outlier_last);
      {
        std::lock_guard<std::mutex> g(fa._m);
        out.laser_odometry = fa._odom;
        ++fa._n_emit;
      }
      out.scan_msg = p.scan_msg;
      fa._output_channel.send(std::move(out));
    }
  };
  void runFeatureAssociation() {  // featureAssociation.cpp:1386-1450
    Sink sink{*this};
    run_feature_association<ProjectionOut>(_ctx, _input_channel, sink);
  }

  lego_ctx* _ctx = nullptr;
  Channel<ProjectionOut>& _input_channel;
  Channel<AssociationOut>& _output_channel;
  int _V;
  std::thread _run_thread;
  std::mutex _m;
  Odometry _odom;
  int _status = 0;
  int _n = 0, _n_last = 0, _n_emit = 0;
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
