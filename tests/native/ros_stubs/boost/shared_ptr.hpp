// test stub: boost::shared_ptr (ROS / PCL 1.8 smart pointer); std::shared_ptr has the interface used
#pragma once
#include <memory>
namespace boost {
template <class T>
using shared_ptr = std::shared_ptr<T>;
}
