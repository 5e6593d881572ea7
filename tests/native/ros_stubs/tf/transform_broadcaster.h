// test stub: tf::TransformBroadcaster
#pragma once
#include "tf/transform_datatypes.h"
namespace tf {
class TransformBroadcaster {
 public:
  void sendTransform(const StampedTransform& transform);
};
}  // namespace tf
