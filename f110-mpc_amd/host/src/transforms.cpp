// Transforms — host restatement of src/transforms.cpp (tf2 Matrix3x3::setRotation of the planar
// quaternion, double rotation, float results).
#include "f110mpc/transforms.h"

#include <cmath>

std::pair<float, float> Transforms::CarPointToWorldPoint(float x, float y, const Pose& pose) {
  const double d = pose.qz * pose.qz + pose.qw * pose.qw;  // tf2 Quaternion::length2
  const double s = 2.0 / d, zs = pose.qz * s, wz = pose.qw * zs, zz = pose.qz * zs;
  const double vx = x, vy = y;
  const double wx = (1.0 - zz) * vx + (-wz) * vy, wy = wz * vx + (1.0 - zz) * vy;
  const float cx = static_cast<float>(pose.x), cy = static_cast<float>(pose.y);  // :16-17
  return {static_cast<float>(wx + cx), static_cast<float>(wy + cy)};
}

float Transforms::GetCarOrientation(const Pose& pose) {
  return static_cast<float>(std::atan2(2 * pose.qw * pose.qz, 1 - 2 * pose.qz * pose.qz));
}

float Transforms::CalcDist(std::pair<float, float> p1, std::pair<float, float> p2) {
  return static_cast<float>(std::sqrt(std::pow(p1.first - p2.first, 2) + std::pow(p1.second - p2.second, 2)));
}
