// Constraints — reference src/constraints.cpp:4-265 without ROS (no marker publisher).
#include "f110mpc/constraints.h"

#include "f110qp.h"

static constexpr double kInfty = 1e30;  // OsqpEigen::INFTY (constraints.cpp:15,17)

Constraints::Constraints(const Params& p)
    : x_max_{kInfty, kInfty, kInfty},
      x_min_{-kInfty, -kInfty, -kInfty},
      u_max_{p.umax, 0.43f},   // constraints.cpp:19
      u_min_{p.umin, -0.43f},  // constraints.cpp:21
      d_(p.state_lims),
      ftg_thresh_(p.follow_gap_thresh),
      divider_(p.fov_divider),
      buffer_(p.buffer) {}

void Constraints::SetXLims(State state) {
  x_max_[0] = state.x() + d_;
  x_max_[1] = state.y() + d_;
  x_min_[0] = state.x() - d_;
  x_min_[1] = state.y() - d_;
}

bool Constraints::FindHalfSpaces(State& state, const LaserScan& scan) {
  const double st[3] = {state.x(), state.y(), state.ori()};
  double l1[3], l2[3];
  if (scan.ranges.empty()) return false;
  const int rc = f110qp_find_half_spaces(st, scan.ranges.data(), static_cast<int>(scan.ranges.size()),
                                         scan.angle_min, scan.angle_increment, scan.angle_max,
                                         ftg_thresh_, divider_, buffer_, l1, l2);
  if (rc != F110QP_OK) return false;
  for (int i = 0; i < 3; i++) {
    l1_[i] = l1[i];
    l2_[i] = l2[i];
  }
  has_hs_ = true;
  return true;
}
