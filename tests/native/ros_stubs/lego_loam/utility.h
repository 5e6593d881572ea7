// test stub: the reference package's utility.h types the ROS unit uses (LeGO-LOAM/include/lego_loam/
// utility.h:55-80: PointType, ProjectionOut, AssociationOut) and the headers it brings in
#pragma once
#include <thread>
#include <vector>
#include "cloud_msgs/cloud_info.h"
#include "nav_msgs/Odometry.h"
#include "pcl/point_cloud.h"
#include "pcl/point_types.h"
#include "pcl_conversions/pcl_conversions.h"
#include "ros/ros.h"
#include "sensor_msgs/PointCloud2.h"
#include "tf/transform_broadcaster.h"
#include "tf/transform_datatypes.h"
typedef pcl::PointXYZI PointType;
struct ProjectionOut {
  pcl::PointCloud<PointType>::Ptr segmented_cloud;
  pcl::PointCloud<PointType>::Ptr outlier_cloud;
  cloud_msgs::cloud_info seg_msg;
  pcl::PointCloud<PointType>::Ptr scan_msg;
};
struct AssociationOut {
  pcl::PointCloud<PointType>::Ptr cloud_outlier_last;
  pcl::PointCloud<PointType>::Ptr cloud_corner_last;
  pcl::PointCloud<PointType>::Ptr cloud_surf_last;
  nav_msgs::Odometry laser_odometry;
  pcl::PointCloud<PointType>::Ptr scan_msg;
};
