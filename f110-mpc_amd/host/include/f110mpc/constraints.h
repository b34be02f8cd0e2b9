// Constraints — mirror of include/f110-mpc/constraints.h:17-66 (src/constraints.cpp).
#pragma once
#include <array>
#include <utility>

#include "f110mpc/laser_scan.h"
#include "f110mpc/params.h"
#include "f110mpc/state.h"

class Constraints {
 public:
  using Vec = std::array<double, 3>;
  using Vec2 = std::array<double, 2>;
  explicit Constraints(const Params& p);  // constraints.cpp:4-42
  virtual ~Constraints() = default;

  void set_x_max(const Vec& v) { x_max_ = v; }
  void set_u_max(const Vec2& v) { u_max_ = v; }
  void set_x_min(const Vec& v) { x_min_ = v; }
  void set_u_min(const Vec2& v) { u_min_ = v; }
  void set_state(State& s) { state_ = s; }
  void SetXLims(State s);  // constraints.cpp:108-114

  Vec x_max() const { return x_max_; }
  Vec2 u_max() const { return u_max_; }
  Vec x_min() const { return x_min_; }
  Vec2 u_min() const { return u_min_; }
  Vec l1() const { return l1_; }  // (a, b, c + 0.5)
  Vec l2() const { return l2_; }
  bool has_half_spaces() const { return has_hs_; }

  // constraints.cpp:116-265 via f110qp_find_half_spaces (the marker publish is not
  // reproduced). Returns false when the scan holds no gap (the reference reads ranges[-1]).
  bool FindHalfSpaces(State& state, const LaserScan& scan);

 private:
  Vec x_max_, x_min_, l1_{}, l2_{};
  Vec2 u_max_, u_min_;
  State state_;
  float d_, ftg_thresh_, divider_, buffer_;
  bool has_hs_ = false;
};
