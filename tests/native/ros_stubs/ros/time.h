// test stub: ros::Time (roscpp_core rostime)
#pragma once
#include <cstdint>
namespace ros {
class Time {
 public:
  uint32_t sec = 0, nsec = 0;
  Time() = default;
  double toSec() const;
};
}  // namespace ros
