// State (x, y, ori) — ROS/Eigen-free mirror of include/f110-mpc/state.h:10-45.
#pragma once
#include <array>
#include <utility>

class State {
 public:
  State() : x_(0), y_(0), ori_(0), size_(3) {}
  State(double x, double y, double ori) : x_(x), y_(y), ori_(ori), size_(3) {}
  virtual ~State() = default;

  std::array<double, 3> StateToVector() const { return {x_, y_, ori_}; }  // state.cpp:19-25
  void set_x(double x) { x_ = x; }
  void set_y(double y) { y_ = y; }
  void set_ori(double ori) { ori_ = ori; }
  std::pair<float, float> GetPair() const { return {static_cast<float>(x_), static_cast<float>(y_)}; }
  double x() const { return x_; }
  double y() const { return y_; }
  double ori() const { return ori_; }
  int size() const { return size_; }

 private:
  double x_, y_, ori_;
  int size_;
};
