// Model::Linearize / simulate_dynamics — reference src/model.cpp:30-75.
#include "f110mpc/model.h"

#include <cmath>

void Model::Linearize(State& S, Input& I, double dt) {
  const float L = 0.3302f;  // model.cpp:32
  A_ = Mat3{};
  B_ = Mat32{};
  C_ = Vec3{};
  A_[0][2] = -1 * I.v() * std::sin(S.ori()) * dt;  // :42
  A_[1][2] = I.v() * std::cos(S.ori()) * dt;       // :43
  A_[0][0] = 1; A_[1][1] = 1; A_[2][2] = 1;       // :44-46
  const double sec2 = std::pow(std::cos(I.steer_ang()), -2);
  B_[0][0] = std::cos(S.ori()) * dt;                // :48
  B_[1][0] = std::sin(S.ori()) * dt;                // :49
  B_[2][0] = std::tan(I.steer_ang()) * dt / L;      // :50
  B_[2][1] = I.v() * sec2 * dt / L;                 // :51
  C_[0] = I.v() * S.ori() * std::sin(S.ori()) * dt;             // :53
  C_[1] = -1 * I.v() * S.ori() * std::cos(S.ori()) * dt;        // :54
  C_[2] = -1 * I.steer_ang() * I.v() * sec2 * dt / L;           // :55
}

void Model::simulate_dynamics(State& state, Input& input, double dt, State& new_state) {
  const double CAR_LENGTH = 0.35;  // model.cpp:2
  const double d0 = input.v() * std::cos(state.ori());
  const double d1 = input.v() * std::sin(state.ori());
  const double d2 = std::tan(input.steer_ang()) * input.v() / CAR_LENGTH;
  new_state.set_x(state.x() + d0 * dt);
  new_state.set_y(state.y() + d1 * dt);
  new_state.set_ori(state.ori() + d2 * dt);
}
