// LoadParams — the ROS param server's role for params.yaml (launch/project.launch:4).
#include <cstdlib>
#include <fstream>
#include <string>

#include "f110mpc/params.h"

static std::string trim(const std::string& s) {
  const auto b = s.find_first_not_of(" \t\r\"'");
  const auto e = s.find_last_not_of(" \t\r\"'");
  return b == std::string::npos ? std::string() : s.substr(b, e - b + 1);
}

bool LoadParams(const std::string& path, Params* p) {
  std::ifstream f(path);
  if (!f) return false;
  std::string line;
  while (std::getline(f, line)) {
    const auto hash = line.find('#');
    if (hash != std::string::npos) line = line.substr(0, hash);
    const auto colon = line.find(':');
    if (colon == std::string::npos) continue;
    const std::string k = trim(line.substr(0, colon)), v = trim(line.substr(colon + 1));
    if (k.empty() || v.empty()) continue;
    const double d = std::atof(v.c_str());
    if (k == "q0") p->q0 = d;
    else if (k == "q1") p->q1 = d;
    else if (k == "q2") p->q2 = d;
    else if (k == "r0") p->r0 = d;
    else if (k == "r1") p->r1 = d;
    else if (k == "horizon") p->horizon = static_cast<int>(d);
    else if (k == "dt") { p->dt = static_cast<float>(d); p->dt_double = d; }
    else if (k == "occ_size") p->occ_size = static_cast<int>(d);
    else if (k == "occ_discrete") p->occ_discrete = static_cast<float>(d);
    else if (k == "occ_dilation") p->occ_dilation = static_cast<float>(d);
    else if (k == "des_vel") p->des_vel = d;
    else if (k == "des_steer") p->des_steer = d;
    else if (k == "umax") p->umax = static_cast<float>(d);
    else if (k == "umin") p->umin = static_cast<float>(d);
    else if (k == "follow_gap_thresh") p->follow_gap_thresh = static_cast<float>(d);
    else if (k == "state_lims") p->state_lims = static_cast<float>(d);
    else if (k == "fov_divider") p->fov_divider = static_cast<float>(d);
    else if (k == "buffer") p->buffer = static_cast<float>(d);
    else if (k == "speed_discrete") p->speed_discrete = static_cast<int>(d);
    else if (k == "steer_discrete") p->steer_discrete = static_cast<int>(d);
    else if (k == "steer_max") p->steer_max = d;
    else if (k == "traj_discrete") p->traj_discrete = static_cast<int>(d);
    else if (k == "lookahead") p->lookahead = d;
    else if (k == "gap_constraints") p->gap_constraints = (v == "true" || d != 0.0);
  }
  return true;
}
