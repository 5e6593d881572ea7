// lego_nodes.h — drop-in replacements for LeGO-LOAM-BOR's ImageProjection and FeatureAssociation ROS
// classes (LeGO-LOAM/src/imageProjection.h:9-16, featureAssociation.h:11-19), running the per-scan path
// on the MI355X through the C-ABI of include/lego_frontend.h.
//
// Same constructors, same public methods, same topics and the same Channel<ProjectionOut> /
// Channel<AssociationOut> hand-offs as the reference, so LeGO-LOAM/src/main.cpp:37-47 compiles unchanged:
//
//   Channel<ProjectionOut> projection_out_channel(true);
//   Channel<AssociationOut> association_out_channel(use_rosbag);
//   ImageProjection IP(nh, projection_out_channel);
//   FeatureAssociation FA(nh, projection_out_channel, association_out_channel);
//
// Build (where ROS Kinetic/Melodic, PCL and the reference's catkin package exist): replace
// src/imageProjection.cpp and src/featureAssociation.cpp in LeGO-LOAM/CMakeLists.txt's lego_loam target
// by ros/lego_nodes.cpp, add include/ and ros/ to its include directories and link
// lego-loam-bor_amd/lego_amd/liblego_frontend.so.  ROS is not installed here: the
// unit is syntax-checked against test-only declaration stubs of the ROS / PCL / tf symbols it uses
// (tests/test_ros_unit_cpu.py, tests/native/ros_stubs/).
#ifndef LEGO_AMD_ROS_NODES_H
#define LEGO_AMD_ROS_NODES_H

#include <thread>
#include <vector>

#include "lego_frontend.h"
#include "lego_loam/channel.h"
#include "lego_loam/utility.h"

// The reference's getParam reads (imageProjection.cpp:57-84, featureAssociation.cpp:69-81; the keys of
// config/loam_config.yaml:4-25) over lego_params_vlp16's defaults; fp_mode / voxel_tie_order from the
// private parameters ~fp_mode / ~voxel_tie_order when set (defaults 0).
lego_params lego_params_from_ros(ros::NodeHandle& nh);

class ImageProjection {
 public:
  ImageProjection(ros::NodeHandle& nh, Channel<ProjectionOut>& output_channel);
  ~ImageProjection();

  void cloudHandler(const sensor_msgs::PointCloud2ConstPtr& laserCloudMsg);

 private:
  void publishClouds(const lego_projection_out& o, const std_msgs::Header& header, ProjectionOut& out);

  ros::NodeHandle& _nh;
  Channel<ProjectionOut>& _output_channel;
  lego_params _params;
  lego_ctx* _gpu = nullptr;
  std::vector<uint8_t> _packed;  // PointCloud2 rows with padding, packed

  ros::Subscriber _sub_laser_cloud;
  ros::Publisher _pub_segmented_cloud;
  ros::Publisher _pub_segmented_cloud_info;
  ros::Publisher _pub_outlier_cloud;
  ros::Publisher _pub_laser;
};

class FeatureAssociation {
 public:
  FeatureAssociation(ros::NodeHandle& node, Channel<ProjectionOut>& input_channel,
                     Channel<AssociationOut>& output_channel);
  ~FeatureAssociation();

  void runFeatureAssociation();

 private:
  struct Sink;  // lego_amd::run_feature_association's conversions and publishers (lego_nodes.cpp)
  void publishOdometry(const lego_association_out& o);
  void publishClouds(const lego_association_out& o);
  void publishCloudsLast(const lego_association_out& o);

  ros::NodeHandle& nh;
  Channel<ProjectionOut>& _input_channel;
  Channel<AssociationOut>& _output_channel;
  lego_params _params;
  lego_ctx* _gpu = nullptr;  // its own context: this thread associates the ProjectionOut it receives
  std::thread _run_thread;

  std_msgs::Header cloudHeader;
  nav_msgs::Odometry laserOdometry;
  tf::StampedTransform laserOdometryTrans;
  tf::TransformBroadcaster tfBroadcaster;

  ros::Publisher pubCornerPointsSharp;
  ros::Publisher pubCornerPointsLessSharp;
  ros::Publisher pubSurfPointsFlat;
  ros::Publisher pubSurfPointsLessFlat;
  ros::Publisher _pub_cloud_corner_last;
  ros::Publisher _pub_cloud_surf_last;
  ros::Publisher _pub_outlier_cloudLast;
  ros::Publisher pubLaserOdometry;
};

#endif  // LEGO_AMD_ROS_NODES_H
