// Input (v, steer_ang) — mirror of include/f110-mpc/input.h:11-34.
#pragma once
#include <array>

class Input {
 public:
  Input() : v_(0), steer_ang_(0), size_(2) {}
  Input(double v, double steer_ang) : v_(v), steer_ang_(steer_ang), size_(2) {}
  virtual ~Input() = default;

  std::array<double, 2> InputToVector() const { return {v_, steer_ang_}; }  // input.cpp:15-21
  void set_v(double v) { v_ = v; }
  void set_steer_ang(double s) { steer_ang_ = s; }
  double v() const { return v_; }
  double steer_ang() const { return steer_ang_; }

 private:
  double v_, steer_ang_;
  int size_;
};
