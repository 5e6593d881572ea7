// test stub: nav_msgs/Odometry (genmsg C++)
#pragma once
#include <string>
#include "geometry_msgs/Pose.h"
#include "std_msgs/Header.h"
namespace nav_msgs {
struct Odometry {
  std_msgs::Header header;
  std::string child_frame_id;
  geometry_msgs::PoseWithCovariance pose;
  geometry_msgs::TwistWithCovariance twist;
};
}  // namespace nav_msgs
