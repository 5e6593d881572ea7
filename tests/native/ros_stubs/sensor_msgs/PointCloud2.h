// test stub: sensor_msgs/PointCloud2 (genmsg C++; bool fields map to uint8_t)
#pragma once
#include <cstdint>
#include <vector>
#include "boost/shared_ptr.hpp"
#include "sensor_msgs/PointField.h"
#include "std_msgs/Header.h"
namespace sensor_msgs {
struct PointCloud2 {
  std_msgs::Header header;
  uint32_t height = 0, width = 0;
  std::vector<PointField> fields;
  uint8_t is_bigendian = 0;
  uint32_t point_step = 0, row_step = 0;
  std::vector<uint8_t> data;
  uint8_t is_dense = 0;
};
typedef boost::shared_ptr<PointCloud2> PointCloud2Ptr;
typedef boost::shared_ptr<PointCloud2 const> PointCloud2ConstPtr;
}  // namespace sensor_msgs
