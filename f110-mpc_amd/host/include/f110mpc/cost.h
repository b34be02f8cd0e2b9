// Cost: dense Q (3x3) and R (2x2) built from diagonals — mirror of include/f110-mpc/cost.h:8-20
// (mpc.cpp:20-24 builds them from q0..q2, r0, r1).
#pragma once
#include <array>

class Cost {
 public:
  using Mat3 = std::array<std::array<double, 3>, 3>;
  using Mat2 = std::array<std::array<double, 2>, 2>;
  Cost() : q_{}, r_{} {}
  Cost(const Mat3& q, const Mat2& r) : q_(q), r_(r) {}
  static Cost FromDiagonals(double q0, double q1, double q2, double r0, double r1) {
    Mat3 q{};
    Mat2 r{};
    q[0][0] = q0; q[1][1] = q1; q[2][2] = q2;
    r[0][0] = r0; r[1][1] = r1;
    return Cost(q, r);
  }
  virtual ~Cost() = default;
  Mat3 q() const { return q_; }
  Mat2 r() const { return r_; }

 private:
  Mat3 q_;
  Mat2 r_;
};
