// ROS-free parameter set with the reference's params.yaml keys and defaults
// (params.yaml:1-59, read by getParam in mpc.cpp:5-16, constraints.cpp:7-12,
// trajectory_planner.cpp:5-10).
#pragma once
#include <string>

struct Params {
  double q0 = 10.0, q1 = 10.0, q2 = 0.0;  // :1-3
  double r0 = 0.10, r1 = 5.0;             // :5-6
  int horizon = 30;                       // :12
  float dt = 0.01f;                       // :13 (MPC::dt_ is a float)
  double dt_double = 0.01;                // :13 as Traj_Plan reads it (a double member)
  double des_vel = 4.5, des_steer = 0.0;  // :42-43
  float umax = 4.5f, umin = 3.0f;         // :46-47 (Constraints members are float)
  float follow_gap_thresh = 3.f;          // :49
  float state_lims = 1.f;                 // :50
  float fov_divider = 1.5f;               // :51
  float buffer = 3.f;                     // :52
  int speed_discrete = 40, steer_discrete = 30;  // :54-55
  double steer_max = 0.4;                 // :56
  int traj_discrete = 50;                 // :57
  double lookahead = 2.5;                 // :59
  int occ_size = 10;                      // :16 (OccGrid::size_ int)
  float occ_discrete = 0.1f;              // :17 (float)
  float occ_dilation = 0.15f;             // :18 (float)
  bool gap_constraints = false;           // build option: enforce the gap rows (C3 semantic)
};

// Parse "key: value" lines (comments after '#'); unknown keys are ignored. Returns false if
// the file cannot be opened.
bool LoadParams(const std::string& path, Params* out);
