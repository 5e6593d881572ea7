// test stub: pcl::PointCloud<T> (PCL 1.8: points vector, width, height, is_dense; boost::shared_ptr Ptr)
#pragma once
#include <cstdint>
#include <vector>
#include "boost/shared_ptr.hpp"
namespace pcl {
template <typename PointT>
class PointCloud {
 public:
  std::vector<PointT> points;
  uint32_t width = 0, height = 0;
  bool is_dense = true;
  typedef boost::shared_ptr<PointCloud<PointT> > Ptr;
  typedef boost::shared_ptr<const PointCloud<PointT> > ConstPtr;
  size_t size() const { return points.size(); }
};
}  // namespace pcl
