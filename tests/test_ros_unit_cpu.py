"""The ROS drop-in translation unit (ros/lego_nodes.cpp) compiles.

ROS 1, PCL, tf and pcl_conversions are not installed here, so the unit is syntax-checked against the
test-only declaration stubs in tests/native/ros_stubs/ (roscpp's NodeHandle::subscribe / advertise /
getParam, Publisher::publish / getNumSubscribers, the ROS_* console macros, the genmsg C++ layouts of
std_msgs/Header, sensor_msgs/PointCloud2 + PointField, nav_msgs/Odometry and the reference's
cloud_msgs/cloud_info, pcl::PointCloud<PointXYZI>, pcl::toROSMsg, tf's Quaternion / Vector3 /
StampedTransform / TransformBroadcaster, and the reference package's Channel<T>, ProjectionOut and
AssociationOut, LeGO-LOAM/include/lego_loam/utility.h:55-80, channel.h:11-56).  Negative controls show
the stubs reject what the real headers reject.
"""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUBS = os.path.join(REPO, "tests", "native", "ros_stubs")
FLAGS = ["g++", "-std=c++14", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-I" + STUBS,
         "-I" + os.path.join(REPO, "include"), "-I" + os.path.join(REPO, "ros")]


def _compile(src):
    return subprocess.run(FLAGS + ["-x", "c++", "-"], input=src, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                          universal_newlines=True, timeout=120)


def test_ros_nodes_unit_compiles():
    r = subprocess.run(FLAGS + [os.path.join(REPO, "ros", "lego_nodes.cpp")], stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, universal_newlines=True, timeout=120)
    assert r.returncode == 0, r.stdout[-4000:]


def test_main_cpp_topology_compiles():
    """LeGO-LOAM/src/main.cpp:37-47's construction of the two nodes on their channels."""
    r = _compile('''#include "lego_nodes.h"
void f(ros::NodeHandle& nh, bool use_rosbag) {
  Channel<ProjectionOut> projection_out_channel(true);
  Channel<AssociationOut> association_out_channel(use_rosbag);
  ImageProjection IP(nh, projection_out_channel);
  FeatureAssociation FA(nh, projection_out_channel, association_out_channel);
}
''')
    assert r.returncode == 0, r.stdout[-4000:]


@pytest.mark.parametrize("snippet", [
    # a subscriber callback taking the message by value: roscpp's subscribe wants const shared_ptr<M const>&
    '''struct N { void cb(sensor_msgs::PointCloud2 m); };
void f(ros::NodeHandle& nh, N* n) { nh.subscribe<sensor_msgs::PointCloud2>("/x", 1, &N::cb, n); }''',
    # cloud_info's bool[] is std::vector<uint8_t> in C++, not std::vector<bool>
    '''void f(cloud_msgs::cloud_info& c) { std::vector<bool>& g = c.segmentedCloudGroundFlag; (void)g; }''',
    # tf::Quaternion from three components (the RPY constructor is deprecated / absent)
    '''void f() { tf::Quaternion q(0.0, 0.0, 0.0); (void)q; }''',
    # a Header's stamp is ros::Time, not a double
    '''void f(std_msgs::Header& h) { double t = h.stamp; (void)t; }''',
])
def test_stubs_reject_wrong_signatures(snippet):
    r = _compile('#include "lego_loam/utility.h"\n#include "lego_loam/channel.h"\n' + snippet + "\n")
    assert r.returncode != 0, snippet
