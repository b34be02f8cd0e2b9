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

// Trajectory::get_best_global_idx's distance test for waypoint i (trajectory.cpp:92-108): the
// waypoint in the car frame (TransformPoint), -1 when it is behind the car (:100), else
// |dist - lookahead|.
__device__ __forceinline__ double waypoint_diff(const Basis& R, double tx, double ty,
                                                const double* __restrict__ wp, int i,
                                                float lookahead) {
  const double wx = (double)(float)wp[2 * i], wy = (double)(float)wp[2 * i + 1];
  const double rx = R.r00 * wx + R.r10 * wy + 0.0 * 0.0;
  const double ry = R.r01 * wx + R.r11 * wy + 0.0 * 0.0;
  const float cx = (float)(rx + tx), cy = (float)(ry + ty);
  if (cx < 0) return -1.0;
  const double dist = sqrt((double)cx * (double)cx + (double)cy * (double)cy);
  return fabs(dist - (double)lookahead);
}

// (bits(FLT_MAX), ~0): the float-minimum's initial value (trajectory.cpp:88) with no index
constexpr unsigned long long kWpNone = (0x7f7fffffull << 32) | 0xffffffffull;

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    const unsigned long long o = __shfl_xor(v, m, 64);
    v = o < v ? o : v;
  }
  return v;
}

__device__ __forceinline__ int wave_max_i32(int v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = max(v, __shfl_xor(v, m, 64));
  return v;
}

}  // namespace

// Diagnostic build only (-DF110QP_STAMPS): per-workgroup cycles at each phase boundary (thread 0),
// read back with f110qp_read_plan_stamps(). The shipped library never executes a stamp.
#ifdef F110QP_STAMPS
constexpr int kPlanStampSlots = 8;
__device__ unsigned long long g_pstamps[4096 * kPlanStampSlots];
#define PSTAMP(k) \
  if (tid == 0 && b < 4096) g_pstamps[(size_t)b * kPlanStampSlots + (k)] = __builtin_amdgcn_s_memtime() - t_start
#else
#define PSTAMP(k)
#endif

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
#ifdef F110QP_STAMPS
  const unsigned long long t_start = __builtin_amdgcn_s_memtime();
#endif
  const int G = K.G, T = K.T, P = K.P;
  const int gwords = (G * G + 3) / 4;
  unsigned long long* red64 = reinterpret_cast<unsigned long long*>(plds);  // DWA min, wp key
  unsigned* red = reinterpret_cast<unsigned*>(plds + 16);                  // 4 reductions
  int* vflag = reinterpret_cast<int*>(plds + 32);                          // [T]
  unsigned char* grid = plds + 32 + 4 * T;                                 // [G][G]

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
    red[2] = 0u;           // 1 + last waypoint index strictly below the float minimum
    red64[0] = 0x7fefffffffffffffull;  // DBL_MAX bits: DWA min distance
    red64[1] = kWpNone;    // (float minimum, first index reaching it)
  }
  __syncthreads();
  PSTAMP(0);
  int num_scans = (int)((angle_max - angle_min) / angle_inc + 1);  // :66
  if (num_scans > nr) num_scans = nr;
  const float* rr = ranges + (size_t)b * nr;
  // The dilation loops (:77-78) visit the same float offsets for every beam, and the column of
  // WorldToOccupancy depends only on x, the row only on y: run the offset loop once, then per
  // beam convert nd columns and nd rows (2 nd divisions instead of 2 nd^2) and mark their nd^2
  // products. kDil offsets per axis cover dilation / discrete < 4 (the default has nd = 4).
  constexpr int kDil = 8;
  float offs[kDil];
  int nd = 0;
  bool more = true;
  {
    float o = -K.dilation;
#pragma unroll
    for (int k = 0; k < kDil; k++) {
      more = more && (o <= K.dilation);
      if (more) nd = k + 1;
      offs[k] = o;
      o += K.discrete;
    }
    more = more && (o <= K.dilation);  // the loop would run past kDil offsets
  }
  const float halfG = (float)(G / 2), fG = (float)G;
  for (int ii = tid; ii < num_scans; ii += 256) {
    const float angle = angle_min + ii * angle_inc + cur;                 // :71
    double sa, ca;
    sincos((double)angle, &sa, &ca);
    const double rng = (double)rr[ii];
    float cx = (float)(rng * ca);                                          // PolarToCartesian
    float cy = (float)(rng * sa);
    cx += o0;
    cy += o1;
    if (!more) {
      // cvtt(v) lands in [0, G) exactly when -1 < v < G (NaN fails both compares)
      int col[kDil], row[kDil];
      bool cok[kDil], rok[kDil];
#pragma unroll
      for (int k = 0; k < kDil; k++) {
        const float vx = (cx + offs[k] - o0) / K.discrete + halfG;
        const float vy = (cy + offs[k] - o1) / K.discrete + halfG;
        cok[k] = k < nd && vx > -1.0f && vx < fG;
        rok[k] = k < nd && vy > -1.0f && vy < fG;
        col[k] = cok[k] ? (int)vx : 0;
        row[k] = rok[k] ? (int)vy * G : 0;
      }
#pragma unroll
      for (int i = 0; i < kDil; i++)
#pragma unroll
        for (int j = 0; j < kDil; j++)
          if (cok[i] && rok[j]) grid[row[j] + col[i]] = 1;
    } else {
      for (float xo = -K.dilation; xo <= K.dilation; xo += K.discrete)   // :77-78
        for (float yo = -K.dilation; yo <= K.dilation; yo += K.discrete) {
          int c, r;
          world_to_occ(K.discrete, G, o0, o1, cx + xo, cy + yo, c, r);
          if (c >= 0 && c < G && r >= 0 && r < G) grid[r * G + c] = 1;
        }
    }
  }
  __syncthreads();
  PSTAMP(1);

  // ---- collision check of the candidate table (:76-113) -----------------------------------
  // candidate of point k = k / P: (k + 0.5) * (1/P) is at least 0.5/P from an integer and its
  // float error stays below 2^-5/P for k < T * P <= 2^18, so the truncation is exact
  const float invP = 1.0f / (float)P;
  for (int k = tid; k < T * P; k += 256) {
    const int i = (int)(((float)k + 0.5f) * invP);
    if (!vflag[i]) continue;  // an earlier point already hit
    const double* pt = table + (size_t)k * 3;
    float wx, wy;
    car_to_world(R, px, py, (float)pt[0], (float)pt[1], wx, wy);
    int col, row;
    world_to_occ(K.discrete, G, o0, o1, wx, wy, col, row);
    const bool in = row >= 0 && row < G && col >= 0 && col < G;          // :91
    if (!in || grid[row * G + col]) vflag[i] = 0;                        // :94-105
  }
  __syncthreads();
  // nvalid > 0 is all the selection needs (:118-121)
  bool anyv = false;
  for (int i = tid; i < T; i += 256) anyv |= vflag[i] != 0;
  const bool any_valid = __syncthreads_or(anyv);
  PSTAMP(2);

  // ---- best waypoint (trajectory.cpp:81-126) -----------------------------------------------
  // The reference keeps the running minimum in a float: index i is taken when
  // d_i < float(min so far). Equivalently: F = min_i float(d_i) over the waypoints ahead,
  // i0 = the first index with float(d_i) = F (it is always taken, and the minimum stays F
  // afterwards); the result is the last j with d_j < F (double comparison; such a j has
  // float(d_j) = F, so j >= i0), or i0. Pass 1 reduces the key (bits(float d_i), i) to its
  // minimum, which is (F, i0) at once; pass 2 reduces the last j. Each thread folds its own
  // waypoints, the wave folds its lanes, and one LDS atomic per wave publishes the result.
  const double tx = R.r00 * (-px) + R.r10 * (-py) + 0.0 * (-0.0);  // inverse: basis^T, -basis^T p
  const double ty = R.r01 * (-px) + R.r11 * (-py) + 0.0 * (-0.0);
  unsigned long long key = kWpNone;
  for (int i = tid; i < W; i += 256) {
    const double diff = waypoint_diff(R, tx, ty, wp, i, K.lookahead);
    if (diff < 0.0) continue;                                             // behind the car (:100)
    const float fd = (float)diff;
    const unsigned long long k = ((unsigned long long)__float_as_uint(fd) << 32) | (unsigned)i;
    key = k < key ? k : key;  // inf / NaN bits sort above kWpNone's FLT_MAX and never win
  }
  key = wave_min_u64(key);
  if ((tid & 63) == 0 && key < kWpNone) atomicMin(&red64[1], key);
  __syncthreads();
  PSTAMP(3);
  const unsigned long long kmin = red64[1];
  int closest = -1;
  if (kmin < kWpNone) {  // uniform
    const int i0 = (int)(unsigned)kmin;
    const float F = __uint_as_float((unsigned)(kmin >> 32));
    int jl = -1;
    for (int i = tid; i < W; i += 256) {
      const double diff = waypoint_diff(R, tx, ty, wp, i, K.lookahead);
      if (diff >= 0.0 && diff < (double)F) jl = i;
    }
    jl = wave_max_i32(jl);
    if ((tid & 63) == 0 && jl >= 0) atomicMax(&red[2], (unsigned)(jl + 1));
    __syncthreads();
    closest = max(i0, (int)red[2] - 1);
  }
  PSTAMP(4);

  // ---- end-point selection among the valid candidates (:122-145) ---------------------------
  int best = -1;
  if (any_valid && closest >= 0) {
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
    best = red[3] == 0x7fffffffu ? -1 : (int)red[3];  // no finite distance: nothing to index
  }

  PSTAMP(5);
  // ---- outputs: miniPath_ in the map frame (:145-152), x0, status ----------------------------
  const int status = !any_valid ? 1 : (closest < 0 ? 2 : 0);
  if (tid == 0) {
    status_out[b] = status;
    best_global[b] = !any_valid ? -1 : closest;
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
  PSTAMP(6);
}

hipError_t launch_plan(const PlanKParams& K, int B, const double* pose, const float* ranges,
                       int nr, float angle_min, float angle_inc, float angle_max,
                       const double* table, const double* wp, int W, unsigned char* grid_out,
                       unsigned char* valid_out, int* best_global, int* best_traj, float* x_ref,
                       float* x0, int* status, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  const size_t lds = 32 + 4 * (size_t)K.T + 4 * (size_t)((K.G * K.G + 3) / 4);
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

#ifdef F110QP_STAMPS
extern "C" int f110qp_read_plan_stamps(unsigned long long* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(f110qp::g_pstamps),
                                  (size_t)n * f110qp::kPlanStampSlots * sizeof(unsigned long long));
}
#endif
