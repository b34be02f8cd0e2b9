// Trajectory / Traj_Plan — ROS-free mirrors of include/f110-mpc/trajectory.h:9-41 and
// include/f110-mpc/trajectory_planner.h:9-35 over the f110qp C ABI.
#pragma once
#include <string>
#include <vector>

#include "f110mpc/params.h"
#include "f110mpc/state.h"
#include "f110mpc/transforms.h"

class Trajectory {
 public:
  explicit Trajectory(const Params& p) : lookahead(static_cast<float>(p.lookahead)) {}
  // trajectory.cpp:18-55 (f110qp_parse_waypoints on the file's text)
  bool ReadCSV(const std::string& path);
  // trajectory.cpp:81-126 on the host (the device planner does the same per scenario)
  int get_best_global_idx(const Pose& pose) const;
  std::vector<State> waypoints_;

 private:
  float lookahead;
};

class Traj_Plan {
 public:
  explicit Traj_Plan(const Params& p);
  // trajectory_planner.cpp:26-72 (f110qp_traj_table)
  std::vector<std::vector<State>> generate_traj_table();
  const std::vector<double>& flat_table() const { return table_; }  // [T][P][3] doubles

 private:
  double speed_max, steer_max, dt;
  int steer_discrete, traj_discrete;
  std::vector<double> table_;
};
