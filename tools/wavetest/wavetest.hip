#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
namespace t {
__device__ __forceinline__ void wsync() { __syncthreads(); }

// DPP controls (gfx9 family encodings)
constexpr int DPP_ROW_SHR1 = 0x111, DPP_ROW_SHR2 = 0x112, DPP_ROW_SHR4 = 0x114, DPP_ROW_SHR8 = 0x118;
constexpr int DPP_ROW_BCAST15 = 0x142, DPP_ROW_BCAST31 = 0x143;
constexpr int DPP_QUAD_XOR1 = 0xB1;  // quad_perm [1,0,3,2]
constexpr int DPP_QUAD_XOR2 = 0x4E;  // quad_perm [2,3,0,1]
constexpr int DPP_QUAD_ODD = 0xF5;   // quad_perm [1,1,3,3]: every lane gets lane|1
constexpr int DPP_ROW_HALF_MIRROR = 0x141, DPP_ROW_MIRROR = 0x140;

template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ int dpp_i(int v) {  // lanes without a source read 0
  return __builtin_amdgcn_update_dpp(0, v, CTRL, ROWMASK, 0xf, false);
}
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(dpp_i<CTRL, ROWMASK>(__float_as_int(v)));
}
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ double dpp_d(double v) {
  int2 p = *reinterpret_cast<int2*>(&v);
  p.x = dpp_i<CTRL, ROWMASK>(p.x);
  p.y = dpp_i<CTRL, ROWMASK>(p.y);
  return *reinterpret_cast<double*>(&p);
}
// full-permutation DPPs (every lane has a source)
template <int CTRL>
__device__ __forceinline__ float perm_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, false));
}
template <int CTRL>
__device__ __forceinline__ int perm_i(int v) {
  return __builtin_amdgcn_mov_dpp(v, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ double perm_d(double v) {
  int2 p = *reinterpret_cast<int2*>(&v);
  p.x = __builtin_amdgcn_mov_dpp(p.x, CTRL, 0xf, 0xf, false);
  p.y = __builtin_amdgcn_mov_dpp(p.y, CTRL, 0xf, 0xf, false);
  return *reinterpret_cast<double*>(&p);
}

__device__ __forceinline__ float readlane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ int readlane_i(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ double readlane_d(double v, int l) {
  int2 p = *reinterpret_cast<int2*>(&v);
  p.x = __builtin_amdgcn_readlane(p.x, l);
  p.y = __builtin_amdgcn_readlane(p.y, l);
  return *reinterpret_cast<double*>(&p);
}

// inclusive prefix sum over the 64 lanes (row shifts, then row broadcasts 15 and 31)
__device__ __forceinline__ float scan_incl(float x, int) {
  x += dpp_f<DPP_ROW_SHR1>(x);
  x += dpp_f<DPP_ROW_SHR2>(x);
  x += dpp_f<DPP_ROW_SHR4>(x);
  x += dpp_f<DPP_ROW_SHR8>(x);
  x += dpp_f<DPP_ROW_BCAST15, 0xa>(x);
  x += dpp_f<DPP_ROW_BCAST31, 0xc>(x);
  return x;
}
__device__ __forceinline__ double scan_incl(double x, int) {
  x += dpp_d<DPP_ROW_SHR1>(x);
  x += dpp_d<DPP_ROW_SHR2>(x);
  x += dpp_d<DPP_ROW_SHR4>(x);
  x += dpp_d<DPP_ROW_SHR8>(x);
  x += dpp_d<DPP_ROW_BCAST15, 0xa>(x);
  x += dpp_d<DPP_ROW_BCAST31, 0xc>(x);
  return x;
}
// inclusive suffix sum: total - inclusive prefix + own
template <typename T>
__device__ __forceinline__ T scan_suffix_incl(T x, int lane) {
  const T p = scan_incl(x, lane);
  T tot;
  if constexpr (sizeof(T) == 8) tot = readlane_d(p, 63);
  else tot = readlane_f(p, 63);
  return tot - p + x;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
  const T p = scan_incl(v, 0);
  if constexpr (sizeof(T) == 8) return readlane_d(p, 63);
  else return readlane_f(p, 63);
}

// value of lane|1 (the steering lane of the stage pair)
__device__ __forceinline__ float odd_lane(float v) { return perm_f<DPP_QUAD_ODD>(v); }
__device__ __forceinline__ double odd_lane(double v) { return perm_d<DPP_QUAD_ODD>(v); }

// argmin of (val, idx) over the wave, result uniform; ties -> smaller idx
__device__ __forceinline__ void amin_step(float& v, int& i, float ov, int oi) {
  const bool take = (ov < v) || (ov == v && oi < i);
  v = take ? ov : v;
  i = take ? oi : i;
}
__device__ __forceinline__ void wave_argmin(float& val, int& idx) {
  amin_step(val, idx, perm_f<DPP_QUAD_XOR1>(val), perm_i<DPP_QUAD_XOR1>(idx));
  amin_step(val, idx, perm_f<DPP_QUAD_XOR2>(val), perm_i<DPP_QUAD_XOR2>(idx));
  amin_step(val, idx, perm_f<DPP_ROW_HALF_MIRROR>(val), perm_i<DPP_ROW_HALF_MIRROR>(idx));
  amin_step(val, idx, perm_f<DPP_ROW_MIRROR>(val), perm_i<DPP_ROW_MIRROR>(idx));
  float v0 = readlane_f(val, 0);
  int i0 = readlane_i(idx, 0);
  amin_step(v0, i0, readlane_f(val, 16), readlane_i(idx, 16));
  amin_step(v0, i0, readlane_f(val, 32), readlane_i(idx, 32));
  amin_step(v0, i0, readlane_f(val, 48), readlane_i(idx, 48));
  val = v0;
  idx = i0;
}


__global__ void k(float* out, double* outd, int* oi) {
  int lane = threadIdx.x;
  float x = (float)(lane + 1);
  out[0 * 64 + lane] = scan_incl(x, lane);
  out[1 * 64 + lane] = scan_suffix_incl(x, lane);
  out[2 * 64 + lane] = wave_sum(x);
  out[3 * 64 + lane] = odd_lane(x);
  double xd = (double)(lane + 1);
  outd[0 * 64 + lane] = scan_incl(xd, lane);
  outd[1 * 64 + lane] = scan_suffix_incl(xd, lane);
  outd[2 * 64 + lane] = odd_lane(xd);
  float v = (float)((lane * 37) % 64) - 20.f; int i = lane;
  if (lane == 45) v = -100.f;
  wave_argmin(v, i);
  out[4 * 64 + lane] = v; oi[lane] = i;
  out[5 * 64 + lane] = perm_f<DPP_QUAD_XOR1>(x);
  out[6 * 64 + lane] = perm_f<DPP_ROW_MIRROR>(x);
  out[7 * 64 + lane] = dpp_f<DPP_ROW_BCAST15, 0xa>(x);
  out[8 * 64 + lane] = dpp_f<DPP_ROW_SHR1>(x);
}
}
int main() {
  float* o; double* od; int* oi;
  hipMalloc(&o, 9 * 64 * 4); hipMalloc(&od, 3 * 64 * 8); hipMalloc(&oi, 64 * 4);
  hipLaunchKernelGGL(t::k, dim3(1), dim3(64), 0, 0, o, od, oi);
  float h[9 * 64]; double hd[3 * 64]; int hi[64];
  hipMemcpy(h, o, sizeof(h), hipMemcpyDeviceToHost); hipMemcpy(hd, od, sizeof(hd), hipMemcpyDeviceToHost);
  hipMemcpy(hi, oi, sizeof(hi), hipMemcpyDeviceToHost);
  const char* names[] = {"scan", "suffix", "sum", "odd", "argmin_v", "xor1", "mirror", "bcast15", "shr1"};
  for (int r = 0; r < 9; r++) { printf("%-8s", names[r]); for (int l = 0; l < 64; l++) printf(" %g", h[r * 64 + l]); printf("\n"); }
  const char* dn[] = {"dscan", "dsuffix", "dodd"};
  for (int r = 0; r < 3; r++) { printf("%-8s", dn[r]); for (int l = 0; l < 64; l++) printf(" %g", hd[r * 64 + l]); printf("\n"); }
  printf("argmin_i"); for (int l = 0; l < 64; l++) printf(" %d", hi[l]); printf("\n");
  return 0;
}
