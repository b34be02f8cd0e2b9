// project — ROS-free mirror of include/f110-mpc/project.h:24-80: the node's callbacks as plain
// methods. The planning branch of OdomCallback (occupancy grid, collision check of the
// candidate table, lookahead waypoint, end-point selection; src/project.cpp:73-152) runs on the
// GPU through f110qp_plan_batch, the MPC branch (:155-198) through MPC::Update.
//
// Deviation (documented): the reference fills its occupancy grid in ScanCallback with the pose
// current at scan time (:44-51); here the grid is built at planning time from the latest scan at
// the planning pose (the two coincide for synchronised odometry and scans).
#pragma once
#include <atomic>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "f110mpc/input.h"
#include "f110mpc/input_handoff.h"
#include "f110mpc/laser_scan.h"
#include "f110mpc/mpc.h"
#include "f110mpc/params.h"
#include "f110mpc/state.h"
#include "f110mpc/trajectory.h"
#include "f110mpc/transforms.h"

class Project {
 public:
  // project.cpp:9-39 (the global path comes from Trajectory::ReadCSV or is given directly)
  Project(const Params& p, const std::vector<State>& global_path);
  ~Project();
  Project(const Project&) = delete;
  Project& operator=(const Project&) = delete;
  void ScanCallback(const LaserScan& scan);  // project.cpp:41-56
  void OdomCallback(const Pose& pose);       // project.cpp:59-205
  Input GetNextInput();                      // project.cpp:207-215
  // One iteration of DriveLoop (project.cpp:217-236) without the thread and the sleep: the
  // input to publish; false until a pose and a scan have arrived.
  bool DriveStep(Input* out);
  // DriveLoop (project.cpp:217-236) on its own thread, as the constructor of the reference starts
  // it (:31-32): every period_ms (default 2 * dt * 1000 = 20 ms, :233-235) publish() receives
  // GetNextInput() and the index advances. The hand-over with OdomCallback goes through
  // InputHandoff (one mutex), not the reference's unsynchronised members. Until a pose and a
  // scan have arrived the loop waits 1 ms per check (the reference spins). StopDriveLoop joins.
  void StartDriveLoop(std::function<void(const Input&)> publish, int period_ms = -1);
  void StopDriveLoop();

  // observers for tests / callers
  bool planned_last_tick() const { return planned_; }
  int last_plan_status() const { return plan_status_; }
  int best_traj_idx() const { return best_traj_; }
  int best_global_idx() const { return best_global_; }
  const std::vector<State>& mini_path() const { return miniPath_; }
  std::vector<Input> current_inputs() const { return inputs_.Snapshot(); }
  unsigned inputs_idx() const { return inputs_.index(); }
  const MPC& mpc() const { return mpc_; }

 private:
  Params params_;
  MPC mpc_;
  Traj_Plan traj_plan_;
  std::vector<State> global_path_;
  std::vector<double> table_, wp_;
  LaserScan scan_;
  bool have_scan_ = false;
  std::atomic<bool> first_pose_estimate_{false}, first_scan_estimate_{false};  // read by DriveLoop
  bool get_mini_path_ = false;
  Pose current_pose_;
  std::vector<State> miniPath_;
  InputHandoff inputs_;  // current_inputs_ + inputs_idx_ of the reference, behind one mutex
  std::thread drive_thread_;
  std::atomic<bool> drive_run_{false};
  bool planned_ = false;
  int plan_status_ = -1, best_traj_ = -1, best_global_ = -1;
};
