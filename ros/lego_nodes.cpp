// lego_nodes.cpp — ImageProjection / FeatureAssociation over the MI355X C-ABI (see lego_nodes.h).
//
// ImageProjection::cloudHandler (imageProjection.cpp:153-174) hands the PointCloud2 payload to
// lego_cloud_handler (fromROSMsg + removeNaN + projection + ground removal + segmentation on the GPU) and
// sends the reference's ProjectionOut (utility.h:64-70) on the channel, as publishClouds does (:498-548).
// FeatureAssociation::runFeatureAssociation (featureAssociation.cpp:1386-1450) receives it and runs one
// lego_feature_association_from (adjustDistortion ... publishCloudsLast on the GPU), then publishes the
// odometry (:1286-1306) and the clouds, and sends AssociationOut every mapping_frequency_divider cycles.
#include "lego_nodes.h"

#include <cstring>
#include <stdexcept>
#include <string>

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
  int ox = -1, oy = -1, oz = -1;  // the float32 x, y, z fields (fromROSMsg, :159)
  for (const auto& fld : msg->fields) {
    if (fld.datatype != sensor_msgs::PointField::FLOAT32 || fld.count != 1) continue;
    if (fld.name == "x") ox = fld.offset;
    else if (fld.name == "y") oy = fld.offset;
    else if (fld.name == "z") oz = fld.offset;
  }
  if (ox < 0 || oy < 0 || oz < 0 || msg->is_bigendian) {
    ROS_ERROR_THROTTLE(1.0, "lidar PointCloud2 without little-endian float32 x, y, z fields");
    return;
  }
  const int n = (int)(msg->width * msg->height);
  const uint8_t* data = msg->data.data();
  if (msg->height > 1 && msg->row_step != msg->width * msg->point_step) {  // padded rows: pack them
    _packed.resize((size_t)n * msg->point_step);
    for (uint32_t r = 0; r < msg->height; ++r)
      std::memcpy(&_packed[(size_t)r * msg->width * msg->point_step], data + (size_t)r * msg->row_step,
                  (size_t)msg->width * msg->point_step);
    data = _packed.data();
  }
  lego_projection_out o;
  const int rc = lego_cloud_handler(_gpu, data, n, (int)msg->point_step, ox, oy, oz, &o);
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
  cloud_msgs::cloud_info& s = out.seg_msg;
  s.header = header;
  s.startRingIndex.assign(o.start_ring_index, o.start_ring_index + V);
  s.endRingIndex.assign(o.end_ring_index, o.end_ring_index + V);
  s.startOrientation = o.start_orientation;
  s.endOrientation = o.end_orientation;
  s.orientationDiff = o.orientation_diff;
  // sized V*H with a zero tail, as resetParameters leaves them (imageProjection.cpp:137-139)
  s.segmentedCloudGroundFlag.assign(VH, false);
  s.segmentedCloudColInd.assign(VH, 0);
  s.segmentedCloudRange.assign(VH, 0);
  for (int i = 0; i < o.n_segmented; ++i) {
    s.segmentedCloudGroundFlag[i] = o.segmented_cloud_ground_flag[i] != 0;
    s.segmentedCloudColInd[i] = o.segmented_cloud_col_ind[i];
    s.segmentedCloudRange[i] = o.segmented_cloud_range[i];
  }
  publish_cloud(_pub_outlier_cloud, out.outlier_cloud, header.stamp, "base_link");
  publish_cloud(_pub_segmented_cloud, out.segmented_cloud, header.stamp, "base_link");
  publish_cloud(_pub_laser, out.scan_msg, header.stamp, "base_link");
  if (_pub_segmented_cloud_info.getNumSubscribers() != 0) _pub_segmented_cloud_info.publish(s);
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

void FeatureAssociation::runFeatureAssociation() {
  std::vector<lego_point> seg, outl;
  std::vector<uint8_t> gflag;
  while (ros::ok()) {
    ProjectionOut projection;
    _input_channel.receive(projection);
    if (!ros::ok() || !projection.segmented_cloud) break;
    const cloud_msgs::cloud_info& si = projection.seg_msg;
    cloudHeader = si.header;
    from_pcl(projection.segmented_cloud, seg);
    from_pcl(projection.outlier_cloud, outl);
    const int M = (int)seg.size();
    if ((int)si.segmentedCloudGroundFlag.size() < M || (int)si.segmentedCloudColInd.size() < M ||
        (int)si.segmentedCloudRange.size() < M || (int)si.startRingIndex.size() < _params.num_vertical_scans ||
        (int)si.endRingIndex.size() < _params.num_vertical_scans) {
      ROS_ERROR("malformed cloud_info: scan dropped");
      continue;
    }
    gflag.assign(si.segmentedCloudGroundFlag.begin(), si.segmentedCloudGroundFlag.begin() + M);
    lego_projection_out in;
    std::memset(&in, 0, sizeof(in));
    in.n_segmented = M;
    in.n_outlier = (int)outl.size();
    in.segmented_cloud = seg.data();
    in.outlier_cloud = outl.data();
    in.start_ring_index = si.startRingIndex.data();
    in.end_ring_index = si.endRingIndex.data();
    in.start_orientation = si.startOrientation;
    in.end_orientation = si.endOrientation;
    in.orientation_diff = si.orientationDiff;
    in.segmented_cloud_ground_flag = gflag.data();
    in.segmented_cloud_col_ind = si.segmentedCloudColInd.data();
    in.segmented_cloud_range = si.segmentedCloudRange.data();
    lego_association_out o;
    const int rc = lego_feature_association_from(_gpu, &in, &o);
    if (rc != LEGO_OK) {
      ROS_ERROR("lego_feature_association_from rc=%d: scan dropped", rc);
      continue;
    }
    publishClouds(o);                     // :1410 (visualization)
    if (o.status & LEGO_ST_INIT) continue;  // checkSystemInitialization (:1413-1416)
    publishOdometry(o);                   // :1422
    publishCloudsLast(o);                 // :1424
    if (o.status & LEGO_ST_EMITTED) {     // _cycle_count == _mapping_frequency_div (:1431-1448)
      AssociationOut out;
      out.cloud_corner_last = to_pcl(o.cloud_corner_last, o.n_corner_last);
      out.cloud_surf_last = to_pcl(o.cloud_surf_last, o.n_surf_last);
      out.cloud_outlier_last = to_pcl(o.cloud_outlier_last, o.n_outlier_last);
      out.laser_odometry = laserOdometry;
      out.scan_msg = projection.scan_msg ? projection.scan_msg : pcl::PointCloud<PointType>::Ptr(new pcl::PointCloud<PointType>());
      _output_channel.send(std::move(out));
    }
  }
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

void FeatureAssociation::publishCloudsLast(const lego_association_out& o) {  // :1362-1382 (every 2nd frame)
  frameCount++;
  if (frameCount < 2) return;  // frameCount >= skipFrameNum + 1
  frameCount = 0;
  const ros::Time t = cloudHeader.stamp;
  if (_pub_outlier_cloudLast.getNumSubscribers())
    publish_cloud(_pub_outlier_cloudLast, to_pcl(o.cloud_outlier_last, o.n_outlier_last), t, "/camera");
  if (_pub_cloud_corner_last.getNumSubscribers())
    publish_cloud(_pub_cloud_corner_last, to_pcl(o.cloud_corner_last, o.n_corner_last), t, "/camera");
  if (_pub_cloud_surf_last.getNumSubscribers())
    publish_cloud(_pub_cloud_surf_last, to_pcl(o.cloud_surf_last, o.n_surf_last), t, "/camera");
}
