// Trajectory / Traj_Plan over the f110qp C ABI (reference src/trajectory.cpp,
// src/trajectory_planner.cpp).
#include "f110mpc/trajectory.h"

#include <cfloat>
#include <cmath>
#include <fstream>
#include <sstream>

#include "f110qp.h"

bool Trajectory::ReadCSV(const std::string& path) {
  std::ifstream f(path);
  if (!f.is_open()) return false;  // :50-53
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string text = ss.str();
  std::vector<double> wp(3 * (text.size() / 2 + 1));
  int n = 0;
  if (f110qp_parse_waypoints(text.c_str(), wp.data(), static_cast<int>(wp.size() / 3), &n) != F110QP_OK)
    return false;
  waypoints_.clear();
  for (int i = 0; i < n; i++) waypoints_.emplace_back(wp[3 * i], wp[3 * i + 1], wp[3 * i + 2]);
  return true;
}

int Trajectory::get_best_global_idx(const Pose& pose) const {
  // world -> car: the inverse tf2 transform (basis^T, -basis^T p), then the float pair
  const double d = pose.qz * pose.qz + pose.qw * pose.qw;
  const double s = 2.0 / d, zs = pose.qz * s, wz = pose.qw * zs, zz = pose.qz * zs;
  const double r00 = 1.0 - zz, r01 = -wz, r10 = wz, r11 = 1.0 - zz;
  const double tx = r00 * (-pose.x) + r10 * (-pose.y), ty = r01 * (-pose.x) + r11 * (-pose.y);
  float min_d = FLT_MAX;  // :88
  int closest = -1;
  for (size_t i = 0; i < waypoints_.size(); i++) {
    const double px = static_cast<float>(waypoints_[i].x()), py = static_cast<float>(waypoints_[i].y());
    const float cx = static_cast<float>(r00 * px + r10 * py + tx);
    const float cy = static_cast<float>(r01 * px + r11 * py + ty);
    if (cx < 0) continue;  // :100
    const double dist = std::sqrt(static_cast<double>(cx) * cx + static_cast<double>(cy) * cy);
    const double diff = std::fabs(dist - static_cast<double>(lookahead));
    if (diff < min_d) {  // :103-107 (the running minimum is a float)
      min_d = static_cast<float>(diff);
      closest = static_cast<int>(i);
    }
  }
  return closest;
}

Traj_Plan::Traj_Plan(const Params& p)
    : speed_max(p.umax), steer_max(p.steer_max), dt(p.dt_double), steer_discrete(p.steer_discrete),
      traj_discrete(p.traj_discrete) {}

std::vector<std::vector<State>> Traj_Plan::generate_traj_table() {
  f110qp_plan_config c;
  f110qp_default_plan_config(&c);
  c.speed_max = speed_max;
  c.steer_max = steer_max;
  c.dt = dt;
  c.steer_discrete = steer_discrete;
  c.traj_discrete = traj_discrete;
  const int T = steer_discrete + 1, P = traj_discrete;
  table_.assign(static_cast<size_t>(T) * P * 3, 0.0);
  std::vector<std::vector<State>> out;
  if (f110qp_traj_table(&c, table_.data()) != T) return out;
  for (int i = 0; i < T; i++) {
    std::vector<State> tr;
    for (int j = 0; j < P; j++) {
      const double* q = &table_[(static_cast<size_t>(i) * P + j) * 3];
      tr.emplace_back(q[0], q[1], q[2]);
    }
    out.push_back(tr);
  }
  return out;
}
