// project — the reference node's control logic (src/project.cpp) without ROS.
#include "f110mpc/project.h"

#include <chrono>
#include <cstdio>

#include "f110qp.h"

Project::Project(const Params& p, const std::vector<State>& global_path)
    : params_(p), mpc_(p), traj_plan_(p), global_path_(global_path) {
  traj_plan_.generate_traj_table();  // project.cpp:37
  table_ = traj_plan_.flat_table();
  for (const State& s : global_path_) {
    wp_.push_back(s.x());
    wp_.push_back(s.y());
  }
}

Project::~Project() { StopDriveLoop(); }

void Project::ScanCallback(const LaserScan& scan) {
  if (!first_pose_estimate_) return;  // :43
  if (!first_scan_estimate_) {
    first_scan_estimate_ = true;
    mpc_.UpdateScan(scan);  // :48
  }
  scan_ = scan;
  have_scan_ = true;
}

void Project::OdomCallback(const Pose& pose) {
  current_pose_ = pose;  // :65
  first_pose_estimate_ = true;
  planned_ = false;
  if (!get_mini_path_) {
    if (!have_scan_) return;  // no grid yet
    f110qp_plan_config c;
    f110qp_default_plan_config(&c);
    c.size = params_.occ_size;
    c.discrete = params_.occ_discrete;
    c.dilation = params_.occ_dilation;
    c.lookahead = static_cast<float>(params_.lookahead);
    c.speed_max = params_.umax;
    c.steer_max = params_.steer_max;
    c.steer_discrete = params_.steer_discrete;
    c.traj_discrete = params_.traj_discrete;
    c.dt = params_.dt_double;
    const int P = c.traj_discrete;
    const double ps[4] = {pose.x, pose.y, pose.qz, pose.qw};
    std::vector<float> xr(3 * P);
    float x0[3];
    int bg = -1, bt = -1, st = -1;
    const int rc = f110qp_plan_batch(&c, 1, ps, scan_.ranges.data(), static_cast<int>(scan_.ranges.size()),
                                     scan_.angle_min, scan_.angle_increment, scan_.angle_max, table_.data(),
                                     wp_.data(), static_cast<int>(wp_.size() / 2), nullptr, nullptr, &bg, &bt,
                                     xr.data(), x0, &st);
    planned_ = true;
    plan_status_ = rc == F110QP_OK ? st : -1;
    best_global_ = bg;
    best_traj_ = bt;
    if (rc != F110QP_OK || st != 0) {
      std::fprintf(stderr, "NO VALID TRAJS\n");  // :117-121
      return;
    }
    miniPath_.clear();
    for (int j = 0; j < P; j++) miniPath_.emplace_back(xr[3 * j], xr[3 * j + 1], 0.0);  // :149-152
    get_mini_path_ = true;  // :158
    return;
  }
  // MPC branch (:160-198)
  const float current_angle = Transforms::GetCarOrientation(pose);
  const State current_state(pose.x, pose.y, current_angle);
  if (!first_scan_estimate_) return;
  Input input = GetNextInput();
  input.set_v(4.5);  // :170
  const std::pair<float, float> end_point(static_cast<float>(miniPath_.back().x()),
                                          static_cast<float>(miniPath_.back().y()));
  const std::pair<float, float> car_point(static_cast<float>(pose.x), static_cast<float>(pose.y));
  if (Transforms::CalcDist(car_point, end_point) < 1.98) {  // :180-188
    get_mini_path_ = false;
    miniPath_.clear();
  }
  // with an emptied miniPath the reference reads past its end (CreateGradientVector); here
  // MPC::Update refuses a path shorter than the horizon and keeps its previous solution
  mpc_.Update(current_state, input, miniPath_);  // :190
  inputs_.Publish(mpc_.solved_trajectory());     // :192-193, atomically with inputs_idx_ = 0
}

Input Project::GetNextInput() {
  bool ran_out = false;
  const Input in = inputs_.Peek(&ran_out);
  if (ran_out) std::fprintf(stderr, "ran out of QP soln\n");  // :210-213
  return in;
}

bool Project::DriveStep(Input* out) {
  if (!(first_pose_estimate_ && first_scan_estimate_)) return false;  // :221
  *out = inputs_.Take();  // GetNextInput() + inputs_idx_++ (:224-233) in one critical section
  return true;
}

void Project::StartDriveLoop(std::function<void(const Input&)> publish, int period_ms) {
  StopDriveLoop();
  if (period_ms < 0) period_ms = static_cast<int>(2 * params_.dt * 1000);  // :233 int dt_ms
  drive_run_ = true;
  drive_thread_ = std::thread([this, publish, period_ms] {
    while (drive_run_) {
      Input in;
      if (DriveStep(&in)) {
        publish(in);  // drive_pub_.publish(drive_msg) (:226-231)
        std::this_thread::sleep_for(std::chrono::milliseconds(period_ms));
      } else {
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
      }
    }
  });
}

void Project::StopDriveLoop() {
  drive_run_ = false;
  if (drive_thread_.joinable()) drive_thread_.join();
}
