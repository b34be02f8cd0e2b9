// MPC — ROS-free mirror of include/f110-mpc/mpc.h:18-95 on top of the f110qp C ABI.
// The OsqpEigen::Solver member (mpc.h:63) is replaced by an f110qp context; Update() runs the
// whole tick (linearise, condense, solve, extract) on the GPU.
#pragma once
#include <string>
#include <vector>

#include "f110mpc/constraints.h"
#include "f110mpc/cost.h"
#include "f110mpc/input.h"
#include "f110mpc/laser_scan.h"
#include "f110mpc/model.h"
#include "f110mpc/params.h"
#include "f110mpc/state.h"

struct f110qp_ctx;

class MPC {
 public:
  explicit MPC(const Params& p);  // mpc.cpp:3-47
  virtual ~MPC();
  MPC(const MPC&) = delete;
  MPC& operator=(const MPC&) = delete;

  // One tick (mpc.cpp:69-143). desired_state_trajectory needs >= horizon() states (the
  // reference reads the first N; CreateGradientVector, mpc.cpp:223-228). On failure the
  // previous solution is kept, as on solver_.solve() == false (mpc.cpp:133-136).
  void Update(State current_state, Input input, std::vector<State>& desired_state_trajectory);

  // Batched tick over candidates (the f110qp extension): one QP per candidate path, all
  // linearised at (current_state, input). Returns per-candidate status (1 = solved) and
  // writes the candidates' (u, x) in the f110qp layouts.
  std::vector<int> UpdateBatch(State current_state, Input input,
                               const std::vector<std::vector<State>>& candidates,
                               std::vector<float>* u_out, std::vector<float>* x_out);

  void UpdateScan(const LaserScan& scan);  // mpc.cpp:64-67
  Constraints constraints() const { return constraints_; }  // declared, never defined upstream
  float dt() const { return dt_; }
  int horizon() const { return horizon_; }
  std::vector<Input> solved_trajectory() const { return solved_trajectory_; }
  // OSQP-layout solution z = [x_0..x_N | u_0..u_{N-1}] (QPsolution_, read by Visualize).
  const std::vector<double>& solution() const { return QPsolution_; }
  int last_status() const { return last_status_; }
  bool solver_ok() const { return ctx_ != nullptr; }
  std::string last_error() const;

 private:
  void UpdateSolvedTrajectory();  // mpc.cpp:145-159

  int horizon_, input_size_ = 2, state_size_ = 3;
  int num_states_, num_inputs_, num_variables_, num_constraints_;
  float dt_;
  Cost cost_;
  Constraints constraints_;
  Model model_;
  State current_state_;
  Input desired_input_;
  std::vector<State> desired_state_trajectory_;
  LaserScan scan_;
  bool have_scan_ = false;
  bool gap_constraints_;
  std::vector<double> QPsolution_;
  std::vector<Input> solved_trajectory_;
  f110qp_ctx* ctx_ = nullptr;
  int last_status_ = 0;
};
