// test stub: the roscpp declarations the ROS unit uses (ros/node_handle.h, publisher.h, subscriber.h,
// console.h, init.h), with roscpp's signatures
#pragma once
#include <cstdint>
#include <string>
#include "boost/shared_ptr.hpp"
#include "ros/time.h"
namespace ros {
class TransportHints {};
class Publisher {
 public:
  template <typename M>
  void publish(const M& message) const;
  uint32_t getNumSubscribers() const;
};
class Subscriber {};
class NodeHandle {
 public:
  bool getParam(const std::string& key, std::string& s) const;
  bool getParam(const std::string& key, double& d) const;
  bool getParam(const std::string& key, float& f) const;
  bool getParam(const std::string& key, int& i) const;
  bool getParam(const std::string& key, bool& b) const;
  template <class M>
  Publisher advertise(const std::string& topic, uint32_t queue_size, bool latch = false);
  template <class M, class T>
  Subscriber subscribe(const std::string& topic, uint32_t queue_size,
                       void (T::*fp)(const boost::shared_ptr<M const>&), T* obj,
                       const TransportHints& transport_hints = TransportHints());
};
bool ok();
namespace console {
void print(const char* level, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
}
}  // namespace ros
#define ROS_FATAL(...) ::ros::console::print("FATAL", __VA_ARGS__)
#define ROS_ERROR(...) ::ros::console::print("ERROR", __VA_ARGS__)
#define ROS_WARN(...) ::ros::console::print("WARN", __VA_ARGS__)
#define ROS_INFO(...) ::ros::console::print("INFO", __VA_ARGS__)
#define ROS_ERROR_THROTTLE(rate, ...) ((void)(double)(rate), ::ros::console::print("ERROR", __VA_ARGS__))
#define ROS_WARN_THROTTLE(rate, ...) ((void)(double)(rate), ::ros::console::print("WARN", __VA_ARGS__))
