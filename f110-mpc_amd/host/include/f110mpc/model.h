// Model — mirror of include/f110-mpc/model.h:14-33 (src/model.cpp).
// The batched solve linearises on the device (csrc/f110qp_kernels.hip); this host class keeps
// the reference's API for callers that inspect A, B, C or roll out candidate paths.
#pragma once
#include <array>

#include "f110mpc/input.h"
#include "f110mpc/state.h"

class Model {
 public:
  using Mat3 = std::array<std::array<double, 3>, 3>;
  using Mat32 = std::array<std::array<double, 2>, 3>;
  using Vec3 = std::array<double, 3>;
  Model() : A_{}, B_{}, C_{} {}
  virtual ~Model() = default;
  Mat3 A() const { return A_; }
  Mat32 B() const { return B_; }
  Vec3 C() const { return C_; }
  // Forward-Euler Jacobians of the kinematic bicycle (model.cpp:30-59, L = 0.3302f).
  void Linearize(State& S, Input& I, double dt);
  // One nonlinear Euler step (model.cpp:61-75, CAR_LENGTH = 0.35).
  void simulate_dynamics(State& state, Input& input, double dt, State& new_state);

 private:
  Mat3 A_;
  Mat32 B_;
  Vec3 C_;
};
