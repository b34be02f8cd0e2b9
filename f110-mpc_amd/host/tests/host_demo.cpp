// host_demo — drives the ROS-free C++ class surface (MPC / Constraints / Model / Cost / State /
// Input / LoadParams) for the pytest suite.
//   host_demo cpu <params.yaml>                         host-only checks, JSON on stdout
//   host_demo tick <params.yaml> <in.bin> <out.bin>     MPC::Update over T ticks (GPU)
//   host_demo batch <params.yaml> <in.bin> <out.bin>    MPC::UpdateBatch over B candidates (GPU)
//   host_demo project <params.yaml> <in.bin> <out.bin>  the project node's callbacks over T ticks
//     in.bin (float64): T, R, W, angle_min, angle_inc, angle_max, waypoints[W][2], then per tick
//     pose[4] (x, y, qz, qw) and ranges[R]; each tick = OdomCallback, ScanCallback, DriveStep.
//     out.bin (float64) per tick: planned, plan_status, best_traj, best_global, mpc_status,
//     drive v, drive steer, miniPath size, then the first 2N entries of MPC's u (NaN if none).
// in.bin (float32): T, N, then per tick x0[3], u_lin[2], x_ref[N*3]; gap mode adds
// scan geometry (3) + R ranges per tick after an R header.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <chrono>
#include <mutex>
#include <thread>
#include <vector>

#include "f110mpc/mpc.h"
#include "f110mpc/project.h"

static std::vector<float> read_all(const char* path) {
  std::ifstream f(path, std::ios::binary);
  f.seekg(0, std::ios::end);
  const size_t n = static_cast<size_t>(f.tellg()) / 4;
  f.seekg(0);
  std::vector<float> v(n);
  f.read(reinterpret_cast<char*>(v.data()), n * 4);
  return v;
}

static int cpu(const char* params_path) {
  Params p;
  if (!LoadParams(params_path, &p)) return 2;
  std::printf("{\"params\": {\"q\": [%.17g, %.17g, %.17g], \"r\": [%.17g, %.17g], \"horizon\": %d, "
              "\"dt\": %.17g, \"des_vel\": %.17g, \"umax\": %.17g, \"umin\": %.17g, \"buffer\": %.17g, "
              "\"fov_divider\": %.9g, \"follow_gap_thresh\": %.9g},\n",
              p.q0, p.q1, p.q2, p.r0, p.r1, p.horizon, (double)p.dt, p.des_vel, (double)p.umax, (double)p.umin, (double)p.buffer,
              (double)p.fov_divider, (double)p.follow_gap_thresh);
  Model m;
  State s(1.0, 2.0, 0.5);
  Input in(4.5, 0.2);
  m.Linearize(s, in, p.dt);
  const auto A = m.A();
  const auto B = m.B();
  const auto C = m.C();
  std::printf("\"linearize\": {\"A02\": %.17g, \"A12\": %.17g, \"B00\": %.17g, \"B10\": %.17g, "
              "\"B20\": %.17g, \"B21\": %.17g, \"C\": [%.17g, %.17g, %.17g]},\n",
              A[0][2], A[1][2], B[0][0], B[1][0], B[2][0], B[2][1], C[0], C[1], C[2]);
  State ns;
  m.simulate_dynamics(s, in, 0.01, ns);
  std::printf("\"simulate\": [%.17g, %.17g, %.17g],\n", ns.x(), ns.y(), ns.ori());
  Constraints c(p);
  std::printf("\"u_min\": [%.17g, %.17g], \"u_max\": [%.17g, %.17g],\n", c.u_min()[0], c.u_min()[1],
              c.u_max()[0], c.u_max()[1]);
  LaserScan scan;
  scan.angle_min = static_cast<float>(-M_PI);
  scan.angle_increment = static_cast<float>(2 * M_PI / 1080);
  scan.angle_max = scan.angle_min + scan.angle_increment * 1079;
  scan.ranges.assign(1080, 1.5f);
  for (int i = 480; i < 560; i++) scan.ranges[i] = 6.0f;
  State car(3.0, -4.0, 0.3);
  const bool ok = c.FindHalfSpaces(car, scan);
  std::printf("\"half_spaces\": {\"ok\": %s, \"l1\": [%.17g, %.17g, %.17g], \"l2\": [%.17g, %.17g, %.17g]},\n",
              ok ? "true" : "false", c.l1()[0], c.l1()[1], c.l1()[2], c.l2()[0], c.l2()[1], c.l2()[2]);
  Cost cost = Cost::FromDiagonals(p.q0, p.q1, p.q2, p.r0, p.r1);
  std::printf("\"cost_diag\": [%.17g, %.17g, %.17g, %.17g, %.17g]}\n", cost.q()[0][0], cost.q()[1][1],
              cost.q()[2][2], cost.r()[0][0], cost.r()[1][1]);
  return 0;
}

static int tick(const char* params_path, const char* in, const char* out, bool batch) {
  Params p;
  if (!LoadParams(params_path, &p)) return 2;
  const std::vector<float> d = read_all(in);
  const int T = static_cast<int>(d[0]), N = static_cast<int>(d[1]);
  p.horizon = N;
  MPC mpc(p);
  if (!mpc.solver_ok()) {
    std::fprintf(stderr, "%s\n", mpc.last_error().c_str());
    return 3;
  }
  std::vector<float> res;
  size_t o = 2;
  if (!batch) {
    for (int t = 0; t < T; t++) {
      State x0(d[o], d[o + 1], d[o + 2]);
      Input ul(d[o + 3], d[o + 4]);
      o += 5;
      std::vector<State> xr;
      for (int i = 0; i < N; i++, o += 3) xr.emplace_back(d[o], d[o + 1], d[o + 2]);
      mpc.Update(x0, ul, xr);
      res.push_back(static_cast<float>(mpc.last_status()));
      for (double z : mpc.solution()) res.push_back(static_cast<float>(z));
      res.push_back(static_cast<float>(mpc.solved_trajectory().size()));
    }
  } else {
    State x0(d[o], d[o + 1], d[o + 2]);
    Input ul(d[o + 3], d[o + 4]);
    o += 5;
    std::vector<std::vector<State>> cands(T);
    for (int t = 0; t < T; t++)
      for (int i = 0; i < N; i++, o += 3) cands[t].emplace_back(d[o], d[o + 1], d[o + 2]);
    std::vector<float> u, x;
    const std::vector<int> st = mpc.UpdateBatch(x0, ul, cands, &u, &x);
    for (int s : st) res.push_back(static_cast<float>(s));
    res.insert(res.end(), u.begin(), u.end());
    res.insert(res.end(), x.begin(), x.end());
  }
  std::ofstream f(out, std::ios::binary);
  f.write(reinterpret_cast<const char*>(res.data()), res.size() * 4);
  return 0;
}

static int project(const char* params_path, const char* in, const char* out) {
  Params p;
  if (!LoadParams(params_path, &p)) return 2;
  std::ifstream f(in, std::ios::binary);
  f.seekg(0, std::ios::end);
  const size_t n = static_cast<size_t>(f.tellg()) / 8;
  f.seekg(0);
  std::vector<double> v(n);
  f.read(reinterpret_cast<char*>(v.data()), n * 8);
  const int T = static_cast<int>(v[0]), R = static_cast<int>(v[1]), W = static_cast<int>(v[2]);
  LaserScan scan;
  scan.angle_min = static_cast<float>(v[3]);
  scan.angle_increment = static_cast<float>(v[4]);
  scan.angle_max = static_cast<float>(v[5]);
  size_t o = 6;
  std::vector<State> path;
  for (int i = 0; i < W; i++, o += 2) path.emplace_back(v[o], v[o + 1], 0.0);
  Project prj(p, path);
  const int N = p.horizon;
  std::vector<double> res;
  for (int t = 0; t < T; t++) {
    Pose pose;
    pose.x = v[o]; pose.y = v[o + 1]; pose.qz = v[o + 2]; pose.qw = v[o + 3];
    o += 4;
    scan.ranges.assign(R, 0.f);
    for (int r = 0; r < R; r++) scan.ranges[r] = static_cast<float>(v[o + r]);
    o += R;
    prj.OdomCallback(pose);   // odometry first: the first scan is only taken after a pose (:43)
    prj.ScanCallback(scan);
    Input drive(0, 0);
    const bool drove = prj.DriveStep(&drive);
    res.push_back(prj.planned_last_tick());
    res.push_back(prj.last_plan_status());
    res.push_back(prj.best_traj_idx());
    res.push_back(prj.best_global_idx());
    res.push_back(prj.mpc().last_status());
    res.push_back(drove ? drive.v() : NAN);
    res.push_back(drove ? drive.steer_ang() : NAN);
    res.push_back(static_cast<double>(prj.mini_path().size()));
    const auto& z = prj.mpc().solution();
    const int ns = 3 * (N + 1);
    for (int k = 0; k < 2 * N; k++) res.push_back(prj.mpc().last_status() == 1 ? z[ns + k] : NAN);
  }
  std::ofstream fo(out, std::ios::binary);
  fo.write(reinterpret_cast<const char*>(res.data()), res.size() * 8);
  return 0;
}

// The scripted drive with the DriveLoop thread running (Project::StartDriveLoop, 1 ms period)
// while the callbacks run on this thread: every published input must be an element of one of the
// solutions MPC::Update produced (or the Input(0.5, 0) fallback). Prints a JSON summary.
static int project_threaded(const char* params_path, const char* in) {
  Params p;
  if (!LoadParams(params_path, &p)) return 2;
  std::ifstream f(in, std::ios::binary);
  f.seekg(0, std::ios::end);
  const size_t n = static_cast<size_t>(f.tellg()) / 8;
  f.seekg(0);
  std::vector<double> v(n);
  f.read(reinterpret_cast<char*>(v.data()), n * 8);
  const int T = static_cast<int>(v[0]), R = static_cast<int>(v[1]), W = static_cast<int>(v[2]);
  LaserScan scan;
  scan.angle_min = static_cast<float>(v[3]);
  scan.angle_increment = static_cast<float>(v[4]);
  scan.angle_max = static_cast<float>(v[5]);
  size_t o = 6;
  std::vector<State> path;
  for (int i = 0; i < W; i++, o += 2) path.emplace_back(v[o], v[o + 1], 0.0);
  Project prj(p, path);
  std::mutex mu;
  std::vector<Input> published;
  prj.StartDriveLoop([&](const Input& in) {
    std::lock_guard<std::mutex> lk(mu);
    published.push_back(in);
  }, 1);
  std::vector<std::vector<Input>> solutions;
  for (int t = 0; t < T; t++) {
    Pose pose;
    pose.x = v[o]; pose.y = v[o + 1]; pose.qz = v[o + 2]; pose.qw = v[o + 3];
    o += 4;
    scan.ranges.assign(R, 0.f);
    for (int r = 0; r < R; r++) scan.ranges[r] = static_cast<float>(v[o + r]);
    o += R;
    prj.OdomCallback(pose);
    prj.ScanCallback(scan);
    solutions.push_back(prj.current_inputs());
    std::this_thread::sleep_for(std::chrono::milliseconds(2));
  }
  prj.StopDriveLoop();
  long ok = 0, fallback = 0, bad = 0;
  for (const Input& in : published) {
    bool found = in.v() == 0.5 && in.steer_ang() == 0.0;
    fallback += found;
    for (size_t s = 0; s < solutions.size() && !found; s++)
      for (const Input& u : solutions[s])
        if (u.v() == in.v() && u.steer_ang() == in.steer_ang()) { found = true; break; }
    ok += found;
    bad += !found;
  }
  int changes = 0;
  for (size_t s = 1; s < solutions.size(); s++) {
    bool same = solutions[s].size() == solutions[s - 1].size();
    for (size_t k = 0; same && k < solutions[s].size(); k++)
      same = solutions[s][k].v() == solutions[s - 1][k].v() && solutions[s][k].steer_ang() == solutions[s - 1][k].steer_ang();
    changes += !same;
  }
  std::printf("{\"published\": %zu, \"from_solutions\": %ld, \"fallback\": %ld, \"unknown\": %ld, \"new_solutions\": %d}\n",
              published.size(), ok - fallback, fallback, bad, changes);
  return bad == 0 ? 0 : 3;
}

int main(int argc, char** argv) {
  if (argc >= 4 && !std::strcmp(argv[1], "project_threaded")) return project_threaded(argv[2], argv[3]);
  if (argc >= 5 && !std::strcmp(argv[1], "project")) return project(argv[2], argv[3], argv[4]);
  if (argc >= 3 && !std::strcmp(argv[1], "cpu")) return cpu(argv[2]);
  if (argc >= 5 && !std::strcmp(argv[1], "tick")) return tick(argv[2], argv[3], argv[4], false);
  if (argc >= 5 && !std::strcmp(argv[1], "batch")) return tick(argv[2], argv[3], argv[4], true);
  std::fprintf(stderr, "usage: host_demo cpu|tick|batch ...\n");
  return 1;
}
