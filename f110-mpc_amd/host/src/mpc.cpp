// MPC — reference src/mpc.cpp on the f110qp C ABI (no ROS, no Eigen, no OSQP).
#include "f110mpc/mpc.h"

#include <cmath>
#include <cstdio>
#include <algorithm>
#include <limits>

#include "f110qp.h"

MPC::MPC(const Params& p)
    : horizon_(p.horizon),
      dt_(p.dt),
      cost_(Cost::FromDiagonals(p.q0, p.q1, p.q2, p.r0, p.r1)),  // mpc.cpp:20-24
      constraints_(p),
      desired_input_(p.des_vel, p.des_steer),                     // mpc.cpp:18-19
      gap_constraints_(p.gap_constraints) {
  num_inputs_ = input_size_ * horizon_;                            // mpc.cpp:26-29
  num_states_ = state_size_ * (horizon_ + 1);
  num_variables_ = num_states_ + num_inputs_;
  num_constraints_ = num_states_ + 2 * (horizon_ + 1) + num_inputs_;
  QPsolution_.assign(num_variables_, 0.0);                          // mpc.cpp:42
  f110qp_config cfg;
  f110qp_default_config(&cfg, horizon_);
  cfg.dt = dt_;
  cfg.q[0] = p.q0; cfg.q[1] = p.q1; cfg.q[2] = p.q2;
  cfg.r[0] = p.r0; cfg.r[1] = p.r1;
  cfg.u_des[0] = p.des_vel; cfg.u_des[1] = p.des_steer;
  const auto umin = constraints_.u_min(), umax = constraints_.u_max();
  cfg.u_min[0] = static_cast<float>(umin[0]); cfg.u_min[1] = static_cast<float>(umin[1]);
  cfg.u_max[0] = static_cast<float>(umax[0]); cfg.u_max[1] = static_cast<float>(umax[1]);
  cfg.gap_mode = gap_constraints_ ? F110QP_GAP_ACTIVE : F110QP_GAP_INACTIVE;
  if (f110qp_create(&ctx_, &cfg) != F110QP_OK) {
    std::fprintf(stderr, "mpc: solver setup failed: %s\n", f110qp_last_error());  // mpc.cpp:122-124
    ctx_ = nullptr;
  }
}

MPC::~MPC() { f110qp_destroy(ctx_); }

std::string MPC::last_error() const { return f110qp_last_error(); }

void MPC::UpdateScan(const LaserScan& scan) {
  scan_ = scan;
  have_scan_ = true;
}

void MPC::Update(State current_state, Input input, std::vector<State>& desired) {
  current_state_ = current_state;
  desired_state_trajectory_ = desired;
  model_.Linearize(current_state_, input, dt_);  // mpc.cpp:73 (host copy for A()/B()/C())
  constraints_.set_state(current_state_);
  bool hs_ok = false;
  if (have_scan_) hs_ok = constraints_.FindHalfSpaces(current_state_, scan_);  // mpc.cpp:75
  last_status_ = 0;
  if (!ctx_ || static_cast<int>(desired.size()) < horizon_) {
    std::fprintf(stderr, "solve failed\n");
    return;
  }
  const int N = horizon_;
  float x0[3] = {static_cast<float>(current_state.x()), static_cast<float>(current_state.y()),
                 static_cast<float>(current_state.ori())};
  float ul[2] = {static_cast<float>(input.v()), static_cast<float>(input.steer_ang())};
  std::vector<float> xr(3 * N), u(2 * N), x(3 * (N + 1));
  for (int i = 0; i < N; i++) {
    xr[3 * i + 0] = static_cast<float>(desired[i].x());
    xr[3 * i + 1] = static_cast<float>(desired[i].y());
    xr[3 * i + 2] = static_cast<float>(desired[i].ori());
  }
  float hs[6];
  const float* hsp = nullptr;
  if (gap_constraints_) {
    if (!hs_ok) {  // gap rows requested but no half spaces: the reference would read garbage
      std::fprintf(stderr, "solve failed: no half spaces\n");
      return;
    }
    const auto l1 = constraints_.l1(), l2 = constraints_.l2();
    for (int i = 0; i < 3; i++) {
      hs[i] = static_cast<float>(l1[i]);
      hs[3 + i] = static_cast<float>(l2[i]);
    }
    hsp = hs;
  }
  int status = 0;
  if (f110qp_solve_batch(ctx_, 1, x0, ul, xr.data(), hsp, u.data(), x.data(), &status, nullptr) !=
      F110QP_OK) {
    std::fprintf(stderr, "solve failed: %s\n", f110qp_last_error());
    return;
  }
  last_status_ = status;
  if (status != F110QP_SOLVED) {
    std::fprintf(stderr, "solve failed\n");  // mpc.cpp:133-136: keep the old QPsolution_
    return;
  }
  for (int k = 0; k < num_states_; k++) QPsolution_[k] = x[k];
  for (int k = 0; k < num_inputs_; k++) QPsolution_[num_states_ + k] = u[k];
  UpdateSolvedTrajectory();
}

std::vector<int> MPC::UpdateBatch(State current_state, Input input,
                                  const std::vector<std::vector<State>>& candidates,
                                  std::vector<float>* u_out, std::vector<float>* x_out) {
  const int B = static_cast<int>(candidates.size());
  const int N = horizon_;
  std::vector<int> status(B, 0);
  if (!ctx_ || B == 0) return status;
  std::vector<float> x0(3 * B), ul(2 * B), xr(static_cast<size_t>(3) * N * B);
  for (int b = 0; b < B; b++) {
    x0[3 * b + 0] = static_cast<float>(current_state.x());
    x0[3 * b + 1] = static_cast<float>(current_state.y());
    x0[3 * b + 2] = static_cast<float>(current_state.ori());
    ul[2 * b + 0] = static_cast<float>(input.v());
    ul[2 * b + 1] = static_cast<float>(input.steer_ang());
    const auto& c = candidates[b];
    for (int i = 0; i < N; i++) {
      const State& s = c[i < static_cast<int>(c.size()) ? i : c.size() - 1];
      xr[(static_cast<size_t>(b) * N + i) * 3 + 0] = static_cast<float>(s.x());
      xr[(static_cast<size_t>(b) * N + i) * 3 + 1] = static_cast<float>(s.y());
      xr[(static_cast<size_t>(b) * N + i) * 3 + 2] = static_cast<float>(s.ori());
    }
  }
  std::vector<float> hsv;
  if (gap_constraints_) {
    if (!have_scan_ || !constraints_.FindHalfSpaces(current_state, scan_)) return status;
    const auto l1 = constraints_.l1(), l2 = constraints_.l2();
    hsv.resize(6 * B);
    for (int b = 0; b < B; b++)
      for (int i = 0; i < 3; i++) {
        hsv[6 * b + i] = static_cast<float>(l1[i]);
        hsv[6 * b + 3 + i] = static_cast<float>(l2[i]);
      }
  }
  u_out->assign(static_cast<size_t>(2) * N * B, 0.f);
  x_out->assign(static_cast<size_t>(3) * (N + 1) * B, 0.f);
  if (f110qp_solve_batch(ctx_, B, x0.data(), ul.data(), xr.data(), hsv.empty() ? nullptr : hsv.data(),
                         u_out->data(), x_out->data(), status.data(), nullptr) != F110QP_OK)
    std::fill(status.begin(), status.end(), 0);
  return status;
}

void MPC::UpdateSolvedTrajectory() {  // mpc.cpp:145-159
  solved_trajectory_.clear();
  for (int i = num_states_; i < static_cast<int>(QPsolution_.size()) - 1; i += 2) {
    const double v = QPsolution_[i], angle = QPsolution_[i + 1];
    if (std::isnan(v) || std::isnan(angle)) return;
    solved_trajectory_.push_back(Input(v, angle));
  }
}
