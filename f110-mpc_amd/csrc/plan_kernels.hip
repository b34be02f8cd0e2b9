// plan_kernels.hip — the planning stage in front of MPC::Update on gfx950, batched over
// scenarios (one pose + one LaserScan each): the reference's project::OdomCallback planning
// branch (src/project.cpp:73-152) with its inputs
//   OccGrid::FillOccGrid            src/occupancy_grid.cpp:55-88
//   collision check of the table    src/project.cpp:76-113 (table: trajectory_planner.cpp:26-72)
//   Trajectory::get_best_global_idx src/trajectory.cpp:81-126
//   end-point (DWA) selection       src/project.cpp:122-141
//   miniPath_ in the map frame      src/project.cpp:145-152
// and its output is exactly the x_ref / x0 the QP batch (f110qp_solve_batch_dev) consumes.
//
// One 256-thread workgroup per scenario; the occupancy grid (G x G bytes, 10 KB at the default
// 10 m / 0.1 m) lives in LDS and never touches HBM (grid_out is an optional debug copy).
// Integer/index work must be bit-identical to the reference, so every float/double expression
// keeps the reference's types and operation order, with FP contraction off (no FMA fusion) and
// float->int conversions that reproduce x86's cvtt (NaN / out of range -> INT_MIN).
// The reference's sequential "running minimum stored in a float" waypoint search is replaced by
// an equivalent parallel form (see best_waypoint below).
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include "f110qp_kernels.h"

namespace f110qp {

namespace {

#pragma clang fp contract(off)

__device__ __forceinline__ int cvtt(float v) {  // x86 cvttss2si semantics
  if (!(v >= -2147483648.0f && v < 2147483648.0f)) return (int)0x80000000;
  return (int)v;
}

// tf2 basis of the planar quaternion (0, 0, qz, qw) (Matrix3x3::setRotation)
struct Basis {
  double r00, r01, r10, r11;
};
__device__ __forceinline__ Basis basis(double qz, double qw) {
  const double d = 0.0 * 0.0 + 0.0 * 0.0 + qz * qz + qw * qw;
  const double s = 2.0 / d;
  const double zs = qz * s, wz = qw * zs, zz = qz * zs;
  Basis R;
  R.r00 = 1.0 - (0.0 + zz); R.r01 = 0.0 - wz;
  R.r10 = 0.0 + wz; R.r11 = 1.0 - (0.0 + zz);
  return R;
}

// Transforms::CarPointToWorldPoint (transforms.cpp:3-20)
__device__ __forceinline__ void car_to_world(const Basis& R, double px, double py, float x,
                                             float y, float& wx, float& wy) {
  const double vx = (double)x, vy = (double)y;
  const double rx = R.r00 * vx + R.r01 * vy + 0.0 * 0.0;
  const double ry = R.r10 * vx + R.r11 * vy + 0.0 * 0.0;
  const float cx = (float)px, cy = (float)py;
  wx = (float)(rx + (double)cx);
  wy = (float)(ry + (double)cy);
}

// OccGrid::WorldToOccupancy (occupancy_grid.cpp:27-33)
__device__ __forceinline__ void world_to_occ(float disc, int G, float o0, float o1, float x,
                                             float y, int& col, int& row) {
  col = cvtt((x - o0) / disc + (float)(G / 2));
  row = cvtt((y - o1) / disc + (float)(G / 2));
}

}  // namespace

__global__ __launch_bounds__(256) void plan_kernel(const PlanKParams K, const int B,
                                                   const double* __restrict__ pose,
                                                   const float* __restrict__ ranges, const int nr,
                                                   const float angle_min, const float angle_inc,
                                                   const float angle_max,
                                                   const double* __restrict__ table,
                                                   const double* __restrict__ wp, const int W,
                                                   unsigned char* __restrict__ grid_out,
                                                   unsigned char* __restrict__ valid_out,
                                                   int* __restrict__ best_global,
                                                   int* __restrict__ best_traj,
                                                   float* __restrict__ xref_out,
                                                   float* __restrict__ x0_out,
                                                   int* __restrict__ status_out) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) unsigned char plds[];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int G = K.G, T = K.T, P = K.P;
  const int gwords = (G * G + 3) / 4;
  unsigned long long* red64 = reinterpret_cast<unsigned long long*>(plds);  // DWA min (8 B)
  unsigned* red = reinterpret_cast<unsigned*>(plds + 8);                   // 4 reductions
  int* vflag = reinterpret_cast<int*>(plds + 24);                          // [T]
  unsigned char* grid = plds + 24 + 4 * T;                                 // [G][G]

  const double px = pose[4 * b + 0], py = pose[4 * b + 1];
  const double qz = pose[4 * b + 2], qw = pose[4 * b + 3];
  // GetCarOrientation (transforms.cpp:44-47) = FillOccGrid's current_angle (:60)
  const float cur = (float)atan2(2 * qw * qz, 1 - 2 * qz * qz);
  const float o0 = (float)(px + 0.275 * cos((double)cur));  // occ_offset_ (:63-64)
  const float o1 = (float)(py + 0.275 * sin((double)cur));
  const Basis R = basis(qz, qw);

  // ---- FillOccGrid (:55-88) --------------------------------------------------------------
  for (int w = tid; w < gwords; w += 256) reinterpret_cast<unsigned*>(grid)[w] = 0u;
  for (int i = tid; i < T; i += 256) vflag[i] = 1;
  if (tid == 0) {
    red[0] = 0x7f7fffffu;  // FLT_MAX bits: float min of the waypoint distances
    red[1] = 0x7fffffffu;  // first index reaching it
    red[2] = 0u;           // 1 + last later index strictly below it
    red64[0] = 0x7fefffffffffffffull;  // DBL_MAX bits: DWA min distance
  }
  __syncthreads();
  int num_scans = (int)((angle_max - angle_min) / angle_inc + 1);  // :66
  if (num_scans > nr) num_scans = nr;
  const float* rr = ranges + (size_t)b * nr;
  for (int ii = tid; ii < num_scans; ii += 256) {
    const float angle = angle_min + ii * angle_inc + cur;                 // :71
    float cx = (float)((double)rr[ii] * cos((double)angle));             // PolarToCartesian
    float cy = (float)((double)rr[ii] * sin((double)angle));
    cx += o0;
    cy += o1;
    for (float xo = -K.dilation; xo <= K.dilation; xo += K.discrete)     // :77-78
      for (float yo = -K.dilation; yo <= K.dilation; yo += K.discrete) {
        int col, row;
        world_to_occ(K.discrete, G, o0, o1, cx + xo, cy + yo, col, row);
        if (col >= 0 && col < G && row >= 0 && row < G) grid[row * G + col] = 1;
      }
  }
  __syncthreads();

  // ---- collision check of the candidate table (:76-113) -----------------------------------
  for (int k = tid; k < T * P; k += 256) {
    const int i = k / P;
    const double* pt = table + (size_t)k * 3;
    float wx, wy;
    car_to_world(R, px, py, (float)pt[0], (float)pt[1], wx, wy);
    int col, row;
    world_to_occ(K.discrete, G, o0, o1, wx, wy, col, row);
    const bool in = row >= 0 && row < G && col >= 0 && col < G;          // :91
    if (!in || grid[row * G + col]) vflag[i] = 0;                        // :94-105
  }
  __syncthreads();

  // ---- best waypoint (trajectory.cpp:81-126) -----------------------------------------------
  // The reference keeps the running minimum in a float: index i is taken when
  // d_i < float(min so far). Equivalently: F = min_i float(d_i); i0 = first index with
  // float(d_i) = F (it is always taken, and the minimum stays F afterwards); the result is the
  // last j > i0 with d_j < F (double comparison), or i0.
  const double tx = R.r00 * (-px) + R.r10 * (-py) + 0.0 * (-0.0);  // inverse: basis^T, -basis^T p
  const double ty = R.r01 * (-px) + R.r11 * (-py) + 0.0 * (-0.0);
  for (int i = tid; i < W; i += 256) {
    const double wx = (double)(float)wp[2 * i], wy = (double)(float)wp[2 * i + 1];
    const double rx = R.r00 * wx + R.r10 * wy + 0.0 * 0.0;
    const double ry = R.r01 * wx + R.r11 * wy + 0.0 * 0.0;
    const float cx = (float)(rx + tx), cy = (float)(ry + ty);            // TransformPoint
    if (cx < 0) continue;                                                 // :100
    const double dist = sqrt((double)cx * (double)cx + (double)cy * (double)cy);
    const double diff = fabs(dist - (double)K.lookahead);
    atomicMin(&red[0], __float_as_uint((float)diff));                     // diff >= 0
  }
  __syncthreads();
  const float F = __uint_as_float(red[0]);
  for (int i = tid; i < W; i += 256) {
    const double wx = (double)(float)wp[2 * i], wy = (double)(float)wp[2 * i + 1];
    const double rx = R.r00 * wx + R.r10 * wy + 0.0 * 0.0;
    const double ry = R.r01 * wx + R.r11 * wy + 0.0 * 0.0;
    const float cx = (float)(rx + tx), cy = (float)(ry + ty);
    if (cx < 0) continue;
    const double dist = sqrt((double)cx * (double)cx + (double)cy * (double)cy);
    const double diff = fabs(dist - (double)K.lookahead);
    if ((float)diff == F) atomicMin(&red[1], (unsigned)i);
  }
  __syncthreads();
  const int i0 = (int)red[1];
  for (int i = tid; i < W; i += 256) {
    if (i <= i0) continue;
    const double wx = (double)(float)wp[2 * i], wy = (double)(float)wp[2 * i + 1];
    const double rx = R.r00 * wx + R.r10 * wy + 0.0 * 0.0;
    const double ry = R.r01 * wx + R.r11 * wy + 0.0 * 0.0;
    const float cx = (float)(rx + tx), cy = (float)(ry + ty);
    if (cx < 0) continue;
    const double dist = sqrt((double)cx * (double)cx + (double)cy * (double)cy);
    const double diff = fabs(dist - (double)K.lookahead);
    if (diff < (double)F) atomicMax(&red[2], (unsigned)(i + 1));
  }
  __syncthreads();
  const int closest = (red[1] == 0x7fffffffu) ? -1 : (red[2] ? (int)red[2] - 1 : i0);

  // ---- end-point selection among the valid candidates (:122-145) ---------------------------
  int nvalid = 0;
  for (int i = 0; i < T; i++) nvalid += vflag[i];
  int best = -1;
  if (nvalid > 0 && closest >= 0) {
    const double gx = (double)(float)wp[2 * closest], gy = (double)(float)wp[2 * closest + 1];
    for (int i = tid; i < T; i += 256) {
      if (!vflag[i]) continue;
      const double* e = table + ((size_t)i * P + P - 1) * 3;
      float ex, ey;
      car_to_world(R, px, py, (float)e[0], (float)e[1], ex, ey);
      const double dx = (double)ex - gx, dy = (double)ey - gy;
      const double dist = sqrt(dx * dx + dy * dy);
      atomicMin(&red64[0], (unsigned long long)__double_as_longlong(dist));
    }
    __syncthreads();
    const double dmin = __longlong_as_double((long long)red64[0]);
    if (tid == 0) red[3] = 0x7fffffffu;
    __syncthreads();
    for (int i = tid; i < T; i += 256) {
      if (!vflag[i]) continue;
      const double* e = table + ((size_t)i * P + P - 1) * 3;
      float ex, ey;
      car_to_world(R, px, py, (float)e[0], (float)e[1], ex, ey);
      const double dx = (double)ex - gx, dy = (double)ey - gy;
      if (sqrt(dx * dx + dy * dy) == dmin) atomicMin(&red[3], (unsigned)i);
    }
    __syncthreads();
    best = (int)red[3];
  }

  // ---- outputs: miniPath_ in the map frame (:145-152), x0, status ----------------------------
  const int status = nvalid == 0 ? 1 : (closest < 0 ? 2 : 0);
  if (tid == 0) {
    status_out[b] = status;
    best_global[b] = nvalid == 0 ? -1 : closest;
    best_traj[b] = best;
    x0_out[3 * b + 0] = (float)px;  // State(position.x, position.y, GetCarOrientation) (:162)
    x0_out[3 * b + 1] = (float)py;
    x0_out[3 * b + 2] = cur;
  }
  float* xo = xref_out + (size_t)b * P * 3;
  for (int j = tid; j < P; j += 256) {
    float wx = __int_as_float(0x7fc00000), wy = wx, wo = wx;  // NaN when no candidate is taken
    if (best >= 0) {
      const double* pt = table + ((size_t)best * P + j) * 3;
      car_to_world(R, px, py, (float)pt[0], (float)pt[1], wx, wy);
      wo = 0.0f;
    }
    xo[3 * j] = wx; xo[3 * j + 1] = wy; xo[3 * j + 2] = wo;
  }
  if (valid_out)
    for (int i = tid; i < T; i += 256) valid_out[(size_t)b * T + i] = (unsigned char)vflag[i];
  if (grid_out) {
    unsigned char* go = grid_out + (size_t)b * G * G;
    for (int k = tid; k < G * G; k += 256) go[k] = grid[k];
  }
}

hipError_t launch_plan(const PlanKParams& K, int B, const double* pose, const float* ranges,
                       int nr, float angle_min, float angle_inc, float angle_max,
                       const double* table, const double* wp, int W, unsigned char* grid_out,
                       unsigned char* valid_out, int* best_global, int* best_traj, float* x_ref,
                       float* x0, int* status, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  const size_t lds = 24 + 4 * (size_t)K.T + 4 * (size_t)((K.G * K.G + 3) / 4);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&plan_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(plan_kernel, dim3(B), dim3(256), lds, s, K, B, pose, ranges, nr, angle_min,
                     angle_inc, angle_max, table, wp, W, grid_out, valid_out, best_global,
                     best_traj, x_ref, x0, status);
  return hipGetLastError();
}

}  // namespace f110qp
