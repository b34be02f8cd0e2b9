// Minimal sensor_msgs/LaserScan stand-in (only the fields FindHalfSpaces reads).
#pragma once
#include <vector>

struct LaserScan {
  float angle_min = 0.f;
  float angle_max = 0.f;
  float angle_increment = 0.f;
  std::vector<float> ranges;
};
