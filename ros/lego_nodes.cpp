// lego_nodes.cpp — ImageProjection / FeatureAssociation over the MI355X C-ABI (see lego_nodes.h).
//
// A thin ROS layer over include/lego_loam_amd.hpp: every decision between a message and the C-ABI is
// the GPU-tested mirror's (tests/test_cpp_mirror.py, tests/native/mirror_check.cpp):
//   * ImageProjection::cloudHandler (imageProjection.cpp:153-174): xyz_offsets + packed_rows hand the
//     PointCloud2 payload to lego_cloud_handler (fromROSMsg + removeNaN + projection + ground removal +
//     segmentation on the GPU); fill_cloud_info builds the cloud_info of the ProjectionOut (utility.h:64-70)
//     sent on the channel, as publishClouds does (:498-548);
//   * FeatureAssociation::runFeatureAssociation (featureAssociation.cpp:1386-1450) is the mirror's
//     run_feature_association loop (projection_in, lego_feature_association_from, FeatureAssociationCycle's
//     publication decisions) with a sink that converts PCL <-> lego_point and publishes.
// What remains here is message conversion and publishing.
#include "lego_nodes.h"

#include <cstring>
#include <stdexcept>
#include <string>

#include "lego_loam_amd.hpp"

namespace {

pcl::PointCloud<PointType>::Ptr to_pcl(const lego_point* p, int n) {
  pcl::PointCloud<PointType>::Ptr c(new pcl::PointCloud<PointType>());
  c->points.resize(n > 0 ? n : 0);
  for (int i = 0; i < n; ++i) {  // pcl::PointXYZI is padded: per field
    PointType& q = c->points[i];
    q.x = p[i].x;
    q.y = p[i].y;
    q.z = p[i].z;
    q.intensity = p[i].intensity;
  }
  c->width = c->points.size();
  c->height = 1;
  return c;
}

void from_pcl(const pcl::PointCloud<PointType>::Ptr& c, std::vector<lego_point>& v) {
  v.resize(c ? c->points.size() : 0);
  for (size_t i = 0; i < v.size(); ++i) {
    const PointType& q = c->points[i];
    v[i] = lego_point{q.x, q.y, q.z, q.intensity};
  }
}

void publish_cloud(ros::Publisher& pub, const pcl::PointCloud<PointType>::Ptr& cloud, const ros::Time& stamp,
                   const char* frame) {
  if (pub.getNumSubscribers() == 0) return;
  sensor_msgs::PointCloud2 msg;
  pcl::toROSMsg(*cloud, msg);
  msg.header.stamp = stamp;
  msg.header.frame_id = frame;
  pub.publish(msg);
}

}  // namespace

lego_params lego_params_from_ros(ros::NodeHandle& nh) {
  lego_params p;
  lego_params_vlp16(&p);
  int i;
  float f;
  if (nh.getParam("/lego_loam/laser/num_vertical_scans", i)) p.num_vertical_scans = i;
  if (nh.getParam("/lego_loam/laser/num_horizontal_scans", i)) p.num_horizontal_scans = i;
  if (nh.getParam("/lego_loam/laser/ground_scan_index", i)) p.ground_scan_index = i;
  if (nh.getParam("/lego_loam/laser/vertical_angle_bottom", f)) p.vertical_angle_bottom = f;
  if (nh.getParam("/lego_loam/laser/vertical_angle_top", f)) p.vertical_angle_top = f;
  if (nh.getParam("/lego_loam/laser/sensor_mount_angle", f)) p.sensor_mount_angle = f;
  if (nh.getParam("/lego_loam/laser/scan_period", f)) p.scan_period = f;
  if (nh.getParam("/lego_loam/imageProjection/segment_valid_point_num", i)) p.segment_valid_point_num = i;
  if (nh.getParam("/lego_loam/imageProjection/segment_valid_line_num", i)) p.segment_valid_line_num = i;
  if (nh.getParam("/lego_loam/imageProjection/segment_theta", f)) p.segment_theta = f;
  if (nh.getParam("/lego_loam/featureAssociation/edge_threshold", f)) p.edge_threshold = f;
  if (nh.getParam("/lego_loam/featureAssociation/surf_threshold", f)) p.surf_threshold = f;
  if (nh.getParam("/lego_loam/featureAssociation/nearest_feature_search_distance", f))
    p.nearest_feature_search_distance = f;
  if (nh.getParam("/lego_loam/mapping/mapping_frequency_divider", i)) p.mapping_frequency_divider = i;
  if (nh.getParam("fp_mode", i)) p.fp_mode = i;                  // private (~) parameters of this build
  if (nh.getParam("voxel_tie_order", i)) p.voxel_tie_order = i;
  return p;
}

// ---- ImageProjection --------------------------------------------------------------------------------
ImageProjection::ImageProjection(ros::NodeHandle& nh, Channel<ProjectionOut>& output_channel)
    : _nh(nh), _output_channel(output_channel) {
  _sub_laser_cloud = nh.subscribe<sensor_msgs::PointCloud2>("/lidar_points", 1, &ImageProjection::cloudHandler, this);
  _pub_segmented_cloud = nh.advertise<sensor_msgs::PointCloud2>("/segmented_cloud", 1);
  _pub_segmented_cloud_info = nh.advertise<cloud_msgs::cloud_info>("/segmented_cloud_info", 1);
  _pub_outlier_cloud = nh.advertise<sensor_msgs::PointCloud2>("/outlier_cloud", 1);
  _pub_laser = nh.advertise<sensor_msgs::PointCloud2>("/scan", 1);
  _params = lego_params_from_ros(nh);
  const int rc = lego_ctx_create(&_params, 0, &_gpu);
  if (rc != LEGO_OK) {
    ROS_FATAL("lego_ctx_create failed (rc=%d): no usable MI355X device or bad parameters", rc);
    throw std::runtime_error("ImageProjection: lego_ctx_create failed");
  }
}

ImageProjection::~ImageProjection() { lego_ctx_destroy(_gpu); }

void ImageProjection::cloudHandler(const sensor_msgs::PointCloud2ConstPtr& msg) {
  int ox, oy, oz;  // the float32 x, y, z fields (fromROSMsg, :159)
  if (!lego_amd::xyz_offsets(msg->fields, msg->is_bigendian, ox, oy, oz)) {
    ROS_ERROR_THROTTLE(1.0, "lidar PointCloud2 without little-endian float32 x, y, z fields");
    return;
  }
  const uint8_t* data =
      lego_amd::packed_rows(msg->data.data(), msg->width, msg->height, msg->point_step, msg->row_step, _packed);
  lego_projection_out o;
  const int rc = lego_cloud_handler(_gpu, data, (int)(msg->width * msg->height), (int)msg->point_step, ox, oy, oz, &o);
  if (rc != LEGO_OK) {  // an empty or all-NaN cloud (UB in the reference's findStartEndAngle)
    ROS_WARN_THROTTLE(1.0, "lego_cloud_handler rc=%d: scan dropped", rc);
    return;
  }
  ProjectionOut out;
  publishClouds(o, msg->header, out);
  _output_channel.send(std::move(out));  // imageProjection.cpp:547
}

void ImageProjection::publishClouds(const lego_projection_out& o, const std_msgs::Header& header, ProjectionOut& out) {
  const int V = _params.num_vertical_scans, VH = V * _params.num_horizontal_scans;
  out.segmented_cloud = to_pcl(o.segmented_cloud, o.n_segmented);
  out.outlier_cloud = to_pcl(o.outlier_cloud, o.n_outlier);
  out.scan_msg = to_pcl(o.scan_msg, o.n_scan);
  out.seg_msg.header = header;
  lego_amd::fill_cloud_info(o, V, VH, true, out.seg_msg);  // V*H entries with a zero tail (:137-139)
  publish_cloud(_pub_outlier_cloud, out.outlier_cloud, header.stamp, "base_link");
  publish_cloud(_pub_segmented_cloud, out.segmented_cloud, header.stamp, "base_link");
  publish_cloud(_pub_laser, out.scan_msg, header.stamp, "base_link");
  if (_pub_segmented_cloud_info.getNumSubscribers() != 0) _pub_segmented_cloud_info.publish(out.seg_msg);
}

// ---- FeatureAssociation -----------------------------------------------------------------------------
FeatureAssociation::FeatureAssociation(ros::NodeHandle& node, Channel<ProjectionOut>& input_channel,
                                       Channel<AssociationOut>& output_channel)
    : nh(node), _input_channel(input_channel), _output_channel(output_channel) {
  pubCornerPointsSharp = nh.advertise<sensor_msgs::PointCloud2>("/laser_cloud_sharp", 1);
  pubCornerPointsLessSharp = nh.advertise<sensor_msgs::PointCloud2>("/laser_cloud_less_sharp", 1);
  pubSurfPointsFlat = nh.advertise<sensor_msgs::PointCloud2>("/laser_cloud_flat", 1);
  pubSurfPointsLessFlat = nh.advertise<sensor_msgs::PointCloud2>("/laser_cloud_less_flat", 1);
  _pub_cloud_corner_last = nh.advertise<sensor_msgs::PointCloud2>("/laser_cloud_corner_last", 2);
  _pub_cloud_surf_last = nh.advertise<sensor_msgs::PointCloud2>("/laser_cloud_surf_last", 2);
  _pub_outlier_cloudLast = nh.advertise<sensor_msgs::PointCloud2>("/outlier_cloud_last", 2);
  pubLaserOdometry = nh.advertise<nav_msgs::Odometry>("/laser_odom_to_init", 5);
  laserOdometry.header.frame_id = "/camera_init";  // initializationValue (:148-152)
  laserOdometry.child_frame_id = "/laser_odom";
  laserOdometryTrans.frame_id_ = "/camera_init";
  laserOdometryTrans.child_frame_id_ = "/laser_odom";
  _params = lego_params_from_ros(nh);
  const int rc = lego_ctx_create(&_params, 0, &_gpu);
  if (rc != LEGO_OK) {
    ROS_FATAL("lego_ctx_create failed (rc=%d): no usable MI355X device or bad parameters", rc);
    throw std::runtime_error("FeatureAssociation: lego_ctx_create failed");
  }
  _run_thread = std::thread(&FeatureAssociation::runFeatureAssociation, this);
}

FeatureAssociation::~FeatureAssociation() {
  _input_channel.send({});  // the empty ProjectionOut ends the loop (featureAssociation.cpp:89-93)
  _run_thread.join();
  lego_ctx_destroy(_gpu);
}

// run_feature_association's sink: PCL <-> lego_point conversion and the publishers
struct FeatureAssociation::Sink {
  FeatureAssociation& fa;
  std::vector<lego_point> seg, outl;
  bool end(const ProjectionOut& p) { return !ros::ok() || !p.segmented_cloud; }  // the dtor's empty item
  bool view(const ProjectionOut& p, lego_projection_out& in) {
    fa.cloudHeader = p.seg_msg.header;
    from_pcl(p.segmented_cloud, seg);
    from_pcl(p.outlier_cloud, outl);
    return lego_amd::projection_in(seg.data(), (int)seg.size(), outl.data(), (int)outl.size(), nullptr, 0, p.seg_msg,
                                   fa._params.num_vertical_scans, in);
  }
  void dropped(const char* why, int rc) { ROS_ERROR("%s (rc=%d): scan dropped", why, rc); }
  void features(const ProjectionOut&, const lego_association_out& o) { fa.publishClouds(o); }      // :1410
  void odometry(const ProjectionOut&, const lego_association_out& o) { fa.publishOdometry(o); }    // :1422
  void clouds_last(const ProjectionOut&, const lego_association_out& o) { fa.publishCloudsLast(o); }  // :1424
  void emit(const ProjectionOut& p, const lego_association_out& o) {  // :1431-1448
    AssociationOut out;
    out.cloud_corner_last = to_pcl(o.cloud_corner_last, o.n_corner_last);
    out.cloud_surf_last = to_pcl(o.cloud_surf_last, o.n_surf_last);
    out.cloud_outlier_last = to_pcl(o.cloud_outlier_last, o.n_outlier_last);
    out.laser_odometry = fa.laserOdometry;
    out.scan_msg = p.scan_msg ? p.scan_msg : pcl::PointCloud<PointType>::Ptr(new pcl::PointCloud<PointType>());
    fa._output_channel.send(std::move(out));
  }
};

void FeatureAssociation::runFeatureAssociation() {
  Sink sink{*this, {}, {}};
  lego_amd::run_feature_association<ProjectionOut>(_gpu, _input_channel, sink);
}

void FeatureAssociation::publishOdometry(const lego_association_out& o) {  // :1286-1306
  laserOdometry.header.stamp = cloudHeader.stamp;
  laserOdometry.pose.pose.orientation.x = o.odom_orientation[0];  // (-geoQuat.y, -geoQuat.z, geoQuat.x, geoQuat.w)
  laserOdometry.pose.pose.orientation.y = o.odom_orientation[1];
  laserOdometry.pose.pose.orientation.z = o.odom_orientation[2];
  laserOdometry.pose.pose.orientation.w = o.odom_orientation[3];
  laserOdometry.pose.pose.position.x = o.odom_position[0];
  laserOdometry.pose.pose.position.y = o.odom_position[1];
  laserOdometry.pose.pose.position.z = o.odom_position[2];
  pubLaserOdometry.publish(laserOdometry);
  laserOdometryTrans.stamp_ = cloudHeader.stamp;
  laserOdometryTrans.setRotation(
      tf::Quaternion(o.odom_orientation[0], o.odom_orientation[1], o.odom_orientation[2], o.odom_orientation[3]));
  laserOdometryTrans.setOrigin(tf::Vector3(o.odom_position[0], o.odom_position[1], o.odom_position[2]));
  tfBroadcaster.sendTransform(laserOdometryTrans);
}

void FeatureAssociation::publishClouds(const lego_association_out& o) {  // publishCloud (:1309-1326)
  const ros::Time t = cloudHeader.stamp;
  if (pubCornerPointsSharp.getNumSubscribers())
    publish_cloud(pubCornerPointsSharp, to_pcl(o.corner_points_sharp, o.n_sharp), t, "/camera");
  if (pubCornerPointsLessSharp.getNumSubscribers())
    publish_cloud(pubCornerPointsLessSharp, to_pcl(o.corner_points_less_sharp, o.n_less_sharp), t, "/camera");
  if (pubSurfPointsFlat.getNumSubscribers())
    publish_cloud(pubSurfPointsFlat, to_pcl(o.surf_points_flat, o.n_flat), t, "/camera");
  if (pubSurfPointsLessFlat.getNumSubscribers())
    publish_cloud(pubSurfPointsLessFlat, to_pcl(o.surf_points_less_flat, o.n_less_flat), t, "/camera");
}

void FeatureAssociation::publishCloudsLast(const lego_association_out& o) {
  // :1362-1382's publications; FeatureAssociationCycle decides the every-second-frame gate
  const ros::Time t = cloudHeader.stamp;
  if (_pub_outlier_cloudLast.getNumSubscribers())
    publish_cloud(_pub_outlier_cloudLast, to_pcl(o.cloud_outlier_last, o.n_outlier_last), t, "/camera");
  if (_pub_cloud_corner_last.getNumSubscribers())
    publish_cloud(_pub_cloud_corner_last, to_pcl(o.cloud_corner_last, o.n_corner_last), t, "/camera");
  if (_pub_cloud_surf_last.getNumSubscribers())
    publish_cloud(_pub_cloud_surf_last, to_pcl(o.cloud_surf_last, o.n_surf_last), t, "/camera");
}
