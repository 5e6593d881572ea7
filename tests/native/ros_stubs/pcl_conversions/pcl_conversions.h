// test stub: pcl_conversions' toROSMsg / fromROSMsg (pcl::PointCloud<T> <-> sensor_msgs::PointCloud2)
#pragma once
#include "pcl/point_cloud.h"
#include "sensor_msgs/PointCloud2.h"
namespace pcl {
template <typename T>
void toROSMsg(const pcl::PointCloud<T>& pcl_cloud, sensor_msgs::PointCloud2& cloud);
template <typename T>
void fromROSMsg(const sensor_msgs::PointCloud2& cloud, pcl::PointCloud<T>& pcl_cloud);
}  // namespace pcl
