// Transforms — ROS/tf2-free mirror of include/f110-mpc/transforms.h:7-15 for planar poses.
#pragma once
#include <utility>

// geometry_msgs::Pose of a planar car: position (x, y), orientation quaternion (0, 0, qz, qw).
struct Pose {
  double x = 0.0, y = 0.0, qz = 0.0, qw = 1.0;
};

class Transforms {
 public:
  // transforms.cpp:3-20: rotate (x, y) by the pose's tf2 basis (double), add the (float) position
  static std::pair<float, float> CarPointToWorldPoint(float x, float y, const Pose& pose);
  // transforms.cpp:44-47
  static float GetCarOrientation(const Pose& pose);
  // transforms.cpp:49-53
  static float CalcDist(std::pair<float, float> p1, std::pair<float, float> p2);
};
