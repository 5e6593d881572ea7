// test stub: tf Quaternion / Vector3 / Transform / StampedTransform (tfScalar = double)
#pragma once
#include <string>
#include "ros/time.h"
namespace tf {
typedef double tfScalar;
class Quaternion {
 public:
  Quaternion(const tfScalar& x, const tfScalar& y, const tfScalar& z, const tfScalar& w);
};
class Vector3 {
 public:
  Vector3(const tfScalar& x, const tfScalar& y, const tfScalar& z);
};
class Transform {
 public:
  void setOrigin(const Vector3& origin);
  void setRotation(const Quaternion& q);
};
class StampedTransform : public Transform {
 public:
  ros::Time stamp_;
  std::string frame_id_;
  std::string child_frame_id_;
};
}  // namespace tf
