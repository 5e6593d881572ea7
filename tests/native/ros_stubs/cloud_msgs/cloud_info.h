// test stub: the reference's cloud_msgs/cloud_info (cloud_msgs/msg/cloud_info.msg) as genmsg generates it
// for C++: int32[] -> std::vector<int32_t>, float32 -> float, bool[] -> std::vector<uint8_t>,
// uint32[] -> std::vector<uint32_t>, float32[] -> std::vector<float>
#pragma once
#include <cstdint>
#include <vector>
#include "std_msgs/Header.h"
namespace cloud_msgs {
struct cloud_info {
  std_msgs::Header header;
  std::vector<int32_t> startRingIndex;
  std::vector<int32_t> endRingIndex;
  float startOrientation = 0.f;
  float endOrientation = 0.f;
  float orientationDiff = 0.f;
  std::vector<uint8_t> segmentedCloudGroundFlag;
  std::vector<uint32_t> segmentedCloudColInd;
  std::vector<float> segmentedCloudRange;
};
}  // namespace cloud_msgs
