/*
 * plan_oracle.c — CPU restatement of the reference's planning stage in front of MPC::Update
 * (TEST INFRASTRUCTURE ONLY, see f110_oracle.h): the candidate table, the occupancy grid, the
 * collision check, the lookahead waypoint and the end-point selection of
 * project::OdomCallback (src/project.cpp:64-152).
 *
 * Float/double semantics follow the reference's member and message types:
 *   OccGrid: size_ int, discrete_ / dilation_ float, occ_offset_ pair<float,float>
 *            (include/f110-mpc/occupancy_grid.h:29-35); LaserScan ranges/angles float32;
 *   Transforms::CarPointToWorldPoint(float x, float y, Pose&) -> pair<float,float>
 *            (src/transforms.cpp:3-20), tf2 rotation in double;
 *   Trajectory::lookahead float (include/f110-mpc/trajectory.h:38), minDistance float
 *            (src/trajectory.cpp:88);
 *   Traj_Plan table in double (State), speed_max / steer_max / dt double
 *            (include/f110-mpc/trajectory_planner.h:27-33).
 * cos/sin/atan2 of float arguments are taken in double (the ::cos(double) overload a ROS/Eigen
 * translation unit resolves to). The pose's quaternion is planar (qx = qy = 0, odometry of a
 * car); the tf2 basis is computed once from it (tf2 round-trips the quaternion through
 * toMsg/fromMsg, which can move the double basis by ~1 ulp; that never survives the float
 * rounding of the results).
 */
#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "f110_oracle.h"

void f110o_default_plan_params(f110o_plan_params* p) {
  memset(p, 0, sizeof(*p));
  p->size = 10;              /* occ_size, params.yaml:16 */
  p->discrete = 0.1f;        /* occ_discrete, params.yaml:17 */
  p->dilation = 0.15f;       /* occ_dilation, params.yaml:18 */
  p->lookahead = 2.5f;       /* lookahead, params.yaml:63 */
  p->speed_max = 4.5;        /* umax (Traj_Plan reads "umax"), params.yaml:46 */
  p->steer_max = 0.4;        /* steer_max, params.yaml:60 */
  p->steer_discrete = 30;    /* steer_discrete, params.yaml:59 */
  p->traj_discrete = 50;     /* traj_discrete, params.yaml:61 */
  p->dt = 0.01;              /* dt, params.yaml:13 */
}

int f110o_grid_blocks(const f110o_plan_params* p) {
  return (int)((float)p->size / p->discrete); /* occupancy_grid.cpp:9 grid_blocks_ = size_/discrete_ */
}

/* Traj_Plan::generate_traj_table (trajectory_planner.cpp:26-72): T = steer_discrete + 1
 * constant-steer rollouts of traj_discrete states from the origin, table[T][P][3]. */
int f110o_traj_table(const f110o_plan_params* p, double* table) {
  const double ds = 2 * +p->steer_max / p->steer_discrete; /* :31 */
  const int T = p->steer_discrete + 1, P = p->traj_discrete;
  for (int i = 0; i < T; i++) {
    const double steer = -p->steer_max + i * ds; /* :43 */
    const double u[2] = {p->speed_max, steer};
    double s[3] = {0.0, 0.0, 0.0}, ns[3];
    double* row = table + (size_t)i * P * 3;
    int n = 0;
    for (int k = 0; k < P - 1; k++) { /* :52-58 */
      if (k == 0) { row[3 * n] = s[0]; row[3 * n + 1] = s[1]; row[3 * n + 2] = s[2]; n++; }
      f110o_simulate_dynamics(s, u, p->dt, ns);
      row[3 * n] = ns[0]; row[3 * n + 1] = ns[1]; row[3 * n + 2] = ns[2]; n++;
      s[0] = ns[0]; s[1] = ns[1]; s[2] = ns[2];
    }
  }
  return T;
}

/* tf2 basis of the planar quaternion (0, 0, qz, qw): Matrix3x3::setRotation */
static void basis(double qz, double qw, double R[4]) {
  const double d = 0.0 * 0.0 + 0.0 * 0.0 + qz * qz + qw * qw;
  const double s = 2.0 / d;
  const double zs = qz * s, wz = qw * zs, zz = qz * zs;
  R[0] = 1.0 - (0.0 + zz); R[1] = 0.0 - wz; /* row 0: 1-(yy+zz), xy-wz */
  R[2] = 0.0 + wz; R[3] = 1.0 - (0.0 + zz); /* row 1: xy+wz, 1-(xx+zz) */
}

/* Transforms::CarPointToWorldPoint (transforms.cpp:3-20) */
static void car_to_world(const double R[4], const double pose[4], float x, float y, float* wx,
                         float* wy) {
  const double vx = (double)x, vy = (double)y;
  const double rx = R[0] * vx + R[1] * vy + 0.0 * 0.0; /* basis row . (x, y, 0) */
  const double ry = R[2] * vx + R[3] * vy + 0.0 * 0.0;
  const float cx = (float)pose[0], cy = (float)pose[1]; /* :16-17 */
  *wx = (float)(rx + cx);
  *wy = (float)(ry + cy);
}

/* Transforms::GetCarOrientation (transforms.cpp:44-47) / occupancy_grid.cpp:60 */
float f110o_car_orientation(const double pose[4]) {
  return (float)atan2(2 * pose[3] * pose[2], 1 - 2 * pose[2] * pose[2]);
}

/* float -> int as x86 cvttss2si converts (a plain cast is UB in C for NaN / out of range) */
static int cvtt(float v) {
  if (!(v >= -2147483648.0f && v < 2147483648.0f)) return (int)0x80000000u;
  return (int)v;
}

/* OccGrid::WorldToOccupancy (occupancy_grid.cpp:27-33) -> (col, row) */
static void world_to_occ(const f110o_plan_params* p, int G, const float off[2], float x, float y,
                         int* col, int* row) {
  *col = cvtt((x - off[0]) / p->discrete + G / 2);
  *row = cvtt((y - off[1]) / p->discrete + G / 2);
}

/* The dilation offsets of FillOccGrid's float loops (occupancy_grid.cpp:77-78). */
int f110o_dilation_offsets(const f110o_plan_params* p, float* offs, int max_n) {
  int n = 0;
  for (float o = -p->dilation; o <= p->dilation; o += p->discrete) {
    if (n < max_n) offs[n] = o;
    n++;
  }
  return n;
}

/* OccGrid::FillOccGrid (occupancy_grid.cpp:55-88). grid[G][G] row-major (row = y cell). */
void f110o_fill_occ_grid(const f110o_plan_params* p, const double pose[4], const float* ranges,
                         int nr, float angle_min, float angle_inc, float angle_max,
                         unsigned char* grid, float off[2]) {
  const int G = f110o_grid_blocks(p);
  memset(grid, 0, (size_t)G * G); /* :57 */
  const float current_angle = f110o_car_orientation(pose); /* :60 */
  off[0] = (float)(pose[0] + 0.275 * cos((double)current_angle)); /* :63-64 */
  off[1] = (float)(pose[1] + 0.275 * sin((double)current_angle));
  int num_scans = (int)((angle_max - angle_min) / angle_inc + 1); /* :66 */
  if (num_scans > nr) num_scans = nr;
  float offs[64];
  const int no = f110o_dilation_offsets(p, offs, 64);
  for (int ii = 0; ii < num_scans; ii++) {
    const float angle = angle_min + ii * angle_inc + current_angle; /* :71 */
    float cx = (float)(ranges[ii] * cos((double)angle));            /* PolarToCartesian :47-52 */
    float cy = (float)(ranges[ii] * sin((double)angle));
    cx += off[0]; /* :73-74 */
    cy += off[1];
    for (int a = 0; a < no && a < 64; a++)
      for (int c = 0; c < no && c < 64; c++) {
        int col, row;
        world_to_occ(p, G, off, cx + offs[a], cy + offs[c], &col, &row); /* :81 */
        if (col >= 0 && col < G && row >= 0 && row < G) grid[(size_t)row * G + col] = 1; /* :82-85 */
      }
  }
}

/* project::OdomCallback's planning branch (project.cpp:73-152) for one pose/grid. */
int f110o_plan(const f110o_plan_params* p, const double pose[4], const unsigned char* grid,
               const float off[2], const double* table, const double* waypoints, int W,
               unsigned char* valid, int* best_global, int* best_traj, float* x_ref,
               float x0[3]) {
  const int G = f110o_grid_blocks(p);
  const int T = p->steer_discrete + 1, P = p->traj_discrete;
  double R[4];
  basis(pose[2], pose[3], R);
  /* collision check of every candidate (:76-113) */
  double* ends = (double*)malloc((size_t)T * 2 * sizeof(double));
  int* vidx = (int*)malloc((size_t)T * sizeof(int));
  int nv = 0;
  for (int i = 0; i < T; i++) {
    int free_points = 0;
    for (int j = 0; j < P; j++) {
      const double* pt = table + ((size_t)i * P + j) * 3;
      float wx, wy;
      car_to_world(R, pose, (float)pt[0], (float)pt[1], &wx, &wy); /* :88 */
      int col, row;
      world_to_occ(p, G, off, wx, wy, &col, &row);                 /* :89 */
      if (row >= 0 && row < G && col >= 0 && col < G) {            /* :91 InGrid(row, col) */
        if (!grid[(size_t)row * G + col]) free_points++;           /* :94 IsOccupied(row, col) */
      }
    }
    valid[i] = (unsigned char)(free_points == P); /* :105 */
    if (valid[i]) {
      const double* e = table + ((size_t)i * P + P - 1) * 3;
      float wx, wy;
      car_to_world(R, pose, (float)e[0], (float)e[1], &wx, &wy); /* :110 */
      ends[2 * nv] = wx; ends[2 * nv + 1] = wy;
      vidx[nv++] = i;
    }
  }
  x0[0] = (float)pose[0];  /* State(current_pose_.position.x, ...) (:162) */
  x0[1] = (float)pose[1];
  x0[2] = f110o_car_orientation(pose);
  *best_global = -1;
  *best_traj = -1;
  if (nv == 0) { free(ends); free(vidx); return 1; } /* :117-121 "NO VALID TRAJS" */
  /* Trajectory::get_best_global_idx (trajectory.cpp:81-126): world -> car frame by the inverse
   * transform (basis^T, basis^T * -origin), nearest to the lookahead among points ahead */
  const double tx = R[0] * (-pose[0]) + R[2] * (-pose[1]) + 0.0 * (-0.0);
  const double ty = R[1] * (-pose[0]) + R[3] * (-pose[1]) + 0.0 * (-0.0);
  float min_d = FLT_MAX;
  int closest = -1;
  for (int i = 0; i < W; i++) {
    const double px = (double)(float)waypoints[2 * i], py = (double)(float)waypoints[2 * i + 1];
    const double rx = R[0] * px + R[2] * py + 0.0 * 0.0; /* transposed basis row . (x, y, 0) */
    const double ry = R[1] * px + R[3] * py + 0.0 * 0.0;
    const float cx = (float)(rx + tx), cy = (float)(ry + ty); /* TransformPoint (transforms.cpp:31-42) */
    if (cx < 0) continue;                                       /* :100 */
    const double dist = sqrt((double)cx * (double)cx + (double)cy * (double)cy); /* :101 pow(.., 0.5) */
    const double diff = fabs(dist - (double)p->lookahead);                      /* :102 */
    if (diff < (double)min_d) { min_d = (float)diff; closest = i; }            /* :103-107 */
  }
  if (closest < 0) { free(ends); free(vidx); return 2; } /* waypoints_.at(-1) throws in the reference */
  *best_global = closest;
  /* DWA cost (:127-141): valid end point nearest to the global point */
  const double gx = (double)(float)waypoints[2 * closest], gy = (double)(float)waypoints[2 * closest + 1];
  double min_dist = DBL_MAX;
  int bt = 0;
  for (int it = 0; it < nv; it++) {
    const double dx = ends[2 * it] - gx, dy = ends[2 * it + 1] - gy;
    const double dist = sqrt(dx * dx + dy * dy);
    if (dist < min_dist) { min_dist = dist; bt = it; }
  }
  const int best = vidx[bt]; /* :145 */
  *best_traj = best;
  /* miniPath_ (:149-153): the chosen candidate in the map frame, ori = 0 */
  for (int j = 0; j < P; j++) {
    const double* pt = table + ((size_t)best * P + j) * 3;
    float wx, wy;
    car_to_world(R, pose, (float)pt[0], (float)pt[1], &wx, &wy);
    x_ref[3 * j] = wx; x_ref[3 * j + 1] = wy; x_ref[3 * j + 2] = 0.0f;
  }
  free(ends);
  free(vidx);
  return 0;
}

/* Trajectory::ReadCSV (trajectory.cpp:18-55) on text already in memory: x = stof(field 1),
 * y = stof(rest of the line), ori = atan2 of the step from the previous point, where the
 * previous index of point 0 is (0u - 1) % n (the unsigned wrap the reference computes). */
int f110o_parse_waypoints(const char* text, double* wp, int max_n) {
  float* tmp = (float*)malloc((size_t)max_n * 2 * sizeof(float));
  int n = 0;
  const char* s = text;
  while (*s && n < max_n) {
    char* end;
    const float x = strtof(s, &end);
    if (end == s) break;
    s = end;
    while (*s && *s != ',' && *s != '\n') s++;
    if (*s != ',') break;
    s++;
    const float y = strtof(s, &end);
    if (end == s) break;
    tmp[2 * n] = x; tmp[2 * n + 1] = y;
    n++;
    s = end;
    while (*s && *s != '\n') s++;
    if (*s == '\n') s++;
  }
  for (unsigned int i = 0; i < (unsigned int)n; i++) {
    const unsigned int prev = (i - 1) % (unsigned int)n; /* trajectory.cpp:42-43 */
    const float px = tmp[2 * prev], py = tmp[2 * prev + 1];
    const float x = tmp[2 * i], y = tmp[2 * i + 1];
    wp[3 * i] = x; wp[3 * i + 1] = y;
    wp[3 * i + 2] = (float)atan2(y - py, x - px); /* float ori = atan2(...) (:46) */
  }
  free(tmp);
  return n;
}
