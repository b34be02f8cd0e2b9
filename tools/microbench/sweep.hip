// sweep.hip — gfx950 micro-benchmark for the wave kernel's explicit inverse (Goodnight symmetric
// sweep of the condensed Hessian, rows in registers, one 64-lane wave per QP). Compares the
// pivot broadcast by v_readlane (SGPR operands) against a broadcast through LDS (one ds_write of
// the pivot column, ds_read_b128 of the whole column by every lane), one and two pivots per
// step. One wave per workgroup, 1,024 workgroups (one wave per SIMD, the C2 regime).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 sweep.hip -o sweep
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#ifndef NUM
#define NUM 40
#endif
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float readlane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// ---- A: readlane broadcast of the pivot row (the shipped kernel) ----
template <int P>
__device__ __forceinline__ void step_rl(float (&h)[NUM], int lane) {
  float rk[NUM];
#pragma unroll
  for (int j = 0; j < NUM; j++) rk[j] = readlane_f(h[j], P);
  const float inv = __builtin_amdgcn_rcpf(rk[P]);
  const bool piv = lane == P;
  const float hp = h[P];
  const float f = piv ? (1.f - inv) : hp * inv;
  const f32x2 nf = {-f, -f};
#pragma unroll
  for (int j = 0; j < NUM; j += 2) {
    const f32x2 rr = {rk[j], rk[j + 1]};
    f32x2 x = {h[j], h[j + 1]};
    x = __builtin_elementwise_fma(nf, rr, x);
    h[j] = x.x; h[j + 1] = x.y;
  }
  h[P] = piv ? -inv : hp * inv;
}
template <int P>
__device__ __forceinline__ void step_rls(float (&h)[NUM], int lane) {  // scalar v_fma_f32
  float rk[NUM];
#pragma unroll
  for (int j = 0; j < NUM; j++) rk[j] = readlane_f(h[j], P);
  const float inv = __builtin_amdgcn_rcpf(rk[P]);
  const bool piv = lane == P;
  const float hp = h[P];
  const float f = piv ? (1.f - inv) : hp * inv;
#pragma unroll
  for (int j = 0; j < NUM; j++) h[j] = fmaf(-f, rk[j], h[j]);
  h[P] = piv ? -inv : hp * inv;
}
template <int P> struct SweepRLS {
  static __device__ __forceinline__ void run(float (&h)[NUM], int lane) { step_rls<P>(h, lane); SweepRLS<P + 1>::run(h, lane); }
};
template <> struct SweepRLS<NUM> { static __device__ __forceinline__ void run(float (&)[NUM], int) {} };
// FMA work only (pivot values from registers of this lane, no broadcast): the VALU floor
template <int P>
__device__ __forceinline__ void step_fma(float (&h)[NUM], int lane) {
  const float inv = __builtin_amdgcn_rcpf(h[P]);
  const float f = h[(P + 1) % NUM] * inv;
  const f32x2 nf = {-f, -f};
#pragma unroll
  for (int j = 0; j < NUM; j += 2) {
    f32x2 x = {h[j], h[j + 1]};
    x = __builtin_elementwise_fma(nf, f32x2{h[(j + 7) % NUM], h[(j + 8) % NUM]}, x);
    h[j] = x.x; h[j + 1] = x.y;
  }
}
template <int P> struct SweepFMA {
  static __device__ __forceinline__ void run(float (&h)[NUM], int lane) { step_fma<P>(h, lane); SweepFMA<P + 1>::run(h, lane); }
};
template <> struct SweepFMA<NUM> { static __device__ __forceinline__ void run(float (&)[NUM], int) {} };
// ---- D: hybrid broadcast: the first K columns through LDS, the rest by readlane (two pipes) ----
template <int P, int K>
__device__ __forceinline__ void step_hyb(float (&h)[NUM], int lane, float* col) {
  float* c = col + (P & 1) * 64;
  c[lane] = h[P];
  float rk[NUM];
#pragma unroll
  for (int j = K; j < NUM; j++) rk[j] = readlane_f(h[j], P);
#pragma unroll
  for (int j = 0; j < K; j += 4) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(c + j);
    rk[j] = v.x; rk[j + 1] = v.y; rk[j + 2] = v.z; rk[j + 3] = v.w;
  }
  const float inv = __builtin_amdgcn_rcpf(readlane_f(h[P], P));
  const bool piv = lane == P;
  const float hp = h[P];
  const float f = piv ? (1.f - inv) : hp * inv;
  const f32x2 nf = {-f, -f};
#pragma unroll
  for (int j = NUM - 2; j >= 0; j -= 2) {
    const f32x2 rr = {rk[j], rk[j + 1]};
    f32x2 x = {h[j], h[j + 1]};
    x = __builtin_elementwise_fma(nf, rr, x);
    h[j] = x.x; h[j + 1] = x.y;
  }
  h[P] = piv ? -inv : hp * inv;
}
template <int P, int K> struct SweepHyb {
  static __device__ __forceinline__ void run(float (&h)[NUM], int lane, float* col) { step_hyb<P, K>(h, lane, col); SweepHyb<P + 1, K>::run(h, lane, col); }
};
template <int K> struct SweepHyb<NUM, K> { static __device__ __forceinline__ void run(float (&)[NUM], int, float*) {} };
// ---- E: 2D layout: lane (ga, gb) of an 8 x 8 grid holds the S x S block (ga S.., gb S..) ----
// Pivot P: the lanes of row block P/S publish their row-P segment (S values, LDS segment stride
// 8); every lane reads the two segments it needs (its rows' pivot-column entries = row-P entries
// by symmetry, and its columns' row-P entries) and updates S x S entries.
constexpr int S2 = NUM / 8;
template <int P>
__device__ __forceinline__ void publish_2d(const float (&h)[S2][S2], int ga, int gb, float* prow) {
  constexpr int aP = P / S2, rP = P % S2;
  float* pr = prow + (P & 1) * 64;
  if (ga == aP) {
#pragma unroll
    for (int c = 0; c < S2; c++) pr[gb * 8 + c] = h[rP][c];
  }
  // the next step's reads must stay after these writes (LDS is in order within a wave; the
  // fences only stop the compiler from reordering and emit no wait)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// pivot P on the row published by the previous step; row P+1 is updated first and published
// before the rest of the update, so its LDS round trip overlaps the remaining FMAs
template <int P>
__device__ __forceinline__ void step_2d(float (&h)[S2][S2], int ga, int gb, float* prow) {
  constexpr int aP = P / S2, rP = P % S2;
  constexpr int P1 = P + 1, rP1 = P1 % S2;
  const float* pr = prow + (P & 1) * 64;
  float fr[S2], rk[S2];
#pragma unroll
  for (int r = 0; r < S2; r++) fr[r] = pr[ga * 8 + r];
#pragma unroll
  for (int c = 0; c < S2; c++) rk[c] = pr[gb * 8 + c];
  const float inv = __builtin_amdgcn_rcpf(pr[aP * 8 + rP]);
  float f[S2];
#pragma unroll
  for (int r = 0; r < S2; r++) f[r] = fr[r] * inv;
  f[rP] = (ga == aP) ? 1.f - inv : f[rP];
  rk[rP] = (gb == aP) ? rk[rP] - 1.f : rk[rP];
  if constexpr (P1 < NUM) {
#pragma unroll
    for (int c = 0; c < S2; c++) h[rP1][c] = fmaf(-f[rP1], rk[c], h[rP1][c]);
    publish_2d<P1>(h, ga, gb, prow);
  }
#pragma unroll
  for (int r = 0; r < S2; r++) {
    if (P1 < NUM && r == rP1) continue;
#pragma unroll
    for (int c = 0; c < S2; c++) h[r][c] = fmaf(-f[r], rk[c], h[r][c]);
  }
  h[rP][rP] = (ga == aP && gb == aP) ? -inv : h[rP][rP];
}
template <int P> struct Sweep2D {
  static __device__ __forceinline__ void run(float (&h)[S2][S2], int ga, int gb, float* pr) { step_2d<P>(h, ga, gb, pr); Sweep2D<P + 1>::run(h, ga, gb, pr); }
};
template <> struct Sweep2D<NUM> { static __device__ __forceinline__ void run(float (&)[S2][S2], int, int, float*) {} };

__global__ __launch_bounds__(64) void kern2d(const float* H, float* W, long long* cyc, int reps) {
  __shared__ __attribute__((aligned(16))) float prow[128];
  const int lane = threadIdx.x, b = blockIdx.x, ga = lane >> 3, gb = lane & 7;
  float h[S2][S2], acc = 0.f;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int rep = 0; rep < reps; rep++) {
#pragma unroll
    for (int r = 0; r < S2; r++)
#pragma unroll
      for (int c = 0; c < S2; c++) h[r][c] = H[((size_t)b * NUM + ga * S2 + r) * NUM + gb * S2 + c];
    publish_2d<0>(h, ga, gb, prow);
    Sweep2D<0>::run(h, ga, gb, prow);
#pragma unroll
    for (int r = 0; r < S2; r++)
#pragma unroll
      for (int c = 0; c < S2; c++) acc += h[r][c];
  }
  asm volatile("" ::"v"(acc));
  const long long t1 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int r = 0; r < S2; r++)
#pragma unroll
    for (int c = 0; c < S2; c++) W[((size_t)b * NUM + ga * S2 + r) * NUM + gb * S2 + c] = h[r][c];
  if (lane == 0) cyc[b] = t1 - t0;
}

template <int P> struct SweepRL {
  static __device__ __forceinline__ void run(float (&h)[NUM], int lane) { step_rl<P>(h, lane); SweepRL<P + 1>::run(h, lane); }
};
template <> struct SweepRL<NUM> { static __device__ __forceinline__ void run(float (&)[NUM], int) {} };

// ---- B: LDS broadcast of the pivot column (symmetric: column P = row P) ----
// LDS ops of one wave execute in order, so the column read after the write needs no barrier;
// BAR = 1 adds a scheduling barrier (no overlap of the next pivot's exchange with this update).
template <int P, int BAR>
__device__ __forceinline__ void step_lds(float (&h)[NUM], int lane, float* col) {
  float* c = col + (P & 1) * 64;
  c[lane] = h[P];
  if (BAR) { __builtin_amdgcn_s_waitcnt(0xc07f); __builtin_amdgcn_wave_barrier(); }
  float rk[NUM];
#pragma unroll
  for (int j = 0; j < NUM; j += 4) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(c + j);
    rk[j] = v.x; rk[j + 1] = v.y; rk[j + 2] = v.z; rk[j + 3] = v.w;
  }
  const float inv = __builtin_amdgcn_rcpf(rk[P]);
  const bool piv = lane == P;
  const float hp = h[P];
  const float f = piv ? (1.f - inv) : hp * inv;
  const f32x2 nf = {-f, -f};
#pragma unroll
  for (int j = 0; j < NUM; j += 2) {
    const f32x2 rr = {rk[j], rk[j + 1]};
    f32x2 x = {h[j], h[j + 1]};
    x = __builtin_elementwise_fma(nf, rr, x);
    h[j] = x.x; h[j + 1] = x.y;
  }
  h[P] = piv ? -inv : hp * inv;
}
template <int P, int BAR> struct SweepLDS {
  static __device__ __forceinline__ void run(float (&h)[NUM], int lane, float* col) { step_lds<P, BAR>(h, lane, col); SweepLDS<P + 1, BAR>::run(h, lane, col); }
};
template <int BAR> struct SweepLDS<NUM, BAR> { static __device__ __forceinline__ void run(float (&)[NUM], int, float*) {} };

// ---- C: two pivots per step through LDS (2x2 block pivot, rank-2 update) ----
// Sweeping P then P+1 equals one block sweep on {P, P+1}: with the 2x2 pivot block D and its
// inverse E, a_ij -= [a_iP a_iQ] E [a_Pj a_Qj]', the pivot rows/columns become E-scaled and
// the block becomes -E.
template <int P, int BAR>
__device__ __forceinline__ void step_lds2(float (&h)[NUM], int lane, float* col) {
  constexpr int Q = P + 1;
  float* c = col + ((P >> 1) & 1) * 128;
  c[lane] = h[P];
  c[64 + lane] = h[Q];
  if (BAR) { __builtin_amdgcn_s_waitcnt(0xc07f); __builtin_amdgcn_wave_barrier(); }
  float rp[NUM], rq[NUM];
#pragma unroll
  for (int j = 0; j < NUM; j += 4) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(c + j);
    const f32x4 w = *reinterpret_cast<const f32x4*>(c + 64 + j);
    rp[j] = v.x; rp[j + 1] = v.y; rp[j + 2] = v.z; rp[j + 3] = v.w;
    rq[j] = w.x; rq[j + 1] = w.y; rq[j + 2] = w.z; rq[j + 3] = w.w;
  }
  const float d00 = rp[P], d01 = rp[Q], d11 = rq[Q];
  const float idet = __builtin_amdgcn_rcpf(d00 * d11 - d01 * d01);
  const float e00 = d11 * idet, e01 = -d01 * idet, e11 = d00 * idet;
  const float hp = h[P], hq = h[Q];
  // row coefficients [a_iP a_iQ] E
  float fp = hp * e00 + hq * e01, fq = hp * e01 + hq * e11;
  const bool inP = lane == P, inQ = lane == Q;
  // pivot rows: a_Pj -> e00 a_Pj + e01 a_Qj, a_Qj -> e01 a_Pj + e11 a_Qj through the same FMA
  fp = inP ? 1.f - e00 : (inQ ? -e01 : fp);
  fq = inP ? -e01 : (inQ ? 1.f - e11 : fq);
  const f32x2 np = {-fp, -fp}, nq = {-fq, -fq};
#pragma unroll
  for (int j = 0; j < NUM; j += 2) {
    f32x2 x = {h[j], h[j + 1]};
    x = __builtin_elementwise_fma(np, f32x2{rp[j], rp[j + 1]}, x);
    x = __builtin_elementwise_fma(nq, f32x2{rq[j], rq[j + 1]}, x);
    h[j] = x.x; h[j + 1] = x.y;
  }
  // pivot columns: a_iP -> (row coeffs), block -> -E
  const float cp = hp * e00 + hq * e01, cq = hp * e01 + hq * e11;
  h[P] = inP ? -e00 : (inQ ? -e01 : cp);
  h[Q] = inP ? -e01 : (inQ ? -e11 : cq);
}
template <int P, int BAR> struct SweepLDS2 {
  static __device__ __forceinline__ void run(float (&h)[NUM], int lane, float* col) { step_lds2<P, BAR>(h, lane, col); SweepLDS2<P + 2, BAR>::run(h, lane, col); }
};
template <int BAR> struct SweepLDS2<NUM, BAR> { static __device__ __forceinline__ void run(float (&)[NUM], int, float*) {} };

__device__ __forceinline__ void load_row(float (&h)[NUM], const float* H, int b, int lane) {
#pragma unroll
  for (int j = 0; j < NUM; j++) h[j] = (lane < NUM) ? H[((size_t)b * NUM + lane) * NUM + j] : (j == lane ? 1.f : 0.f);
}
__device__ __forceinline__ void store_row(const float (&h)[NUM], float* W, int b, int lane) {
  if (lane < NUM)
#pragma unroll
    for (int j = 0; j < NUM; j++) W[((size_t)b * NUM + lane) * NUM + j] = h[j];
}

template <int V>
__global__ __launch_bounds__(64) void kern(const float* H, float* W, long long* cyc, int reps) {
  __shared__ __attribute__((aligned(16))) float col[256];
  const int lane = threadIdx.x, b = blockIdx.x;
  float h[NUM], acc[NUM];
#pragma unroll
  for (int j = 0; j < NUM; j++) acc[j] = 0.f;
  // the whole loop is timed (s_memtime is no scheduling barrier, so per-phase stamps can lie);
  // cost per sweep = (cycles(reps) - cycles(1)) / (reps - 1)
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; r++) {
    load_row(h, H, b, lane);
    if (V == 0) SweepRL<0>::run(h, lane);
    if (V == 1) SweepLDS<0, 1>::run(h, lane, col);
    if (V == 2) SweepLDS2<0, 1>::run(h, lane, col);
    if (V == 3) SweepLDS<0, 0>::run(h, lane, col);
    if (V == 4) SweepLDS2<0, 0>::run(h, lane, col);
    if (V == 5) SweepRLS<0>::run(h, lane);
    if (V == 6) SweepFMA<0>::run(h, lane);
    if (V == 7) SweepHyb<0, 8>::run(h, lane, col);
    if (V == 8) SweepHyb<0, 12>::run(h, lane, col);
    if (V == 9) SweepHyb<0, 16>::run(h, lane, col);
    if (V == 10) SweepHyb<0, 20>::run(h, lane, col);
    if (V == 11) SweepHyb<0, 24>::run(h, lane, col);
#pragma unroll
    for (int j = 0; j < NUM; j++) acc[j] += h[j];
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NUM; j++) s += acc[j];
  asm volatile("" ::"v"(s));
  const long long t1 = __builtin_amdgcn_s_memtime();
  store_row(h, W, b, lane);
  if (lane == 0) cyc[b] = t1 - t0;
}

int main() {
  const int B = 1024;
  std::vector<float> H((size_t)B * NUM * NUM);
  srand(1);
  for (int b = 0; b < B; b++) {
    std::vector<double> M(NUM * NUM);
    for (auto& m : M) m = (rand() / (double)RAND_MAX - 0.5);
    for (int i = 0; i < NUM; i++)
      for (int j = 0; j < NUM; j++) {
        double s = (i == j) ? 0.5 : 0.0;
        for (int k = 0; k < NUM; k++) s += M[k * NUM + i] * M[k * NUM + j] / NUM;
        H[((size_t)b * NUM + i) * NUM + j] = (float)s;
      }
  }
  float *dH, *dW;
  long long* dc;
  hipMalloc(&dH, H.size() * 4);
  hipMalloc(&dW, H.size() * 4);
  hipMalloc(&dc, B * 8);
  hipMemcpy(dH, H.data(), H.size() * 4, hipMemcpyHostToDevice);
  const char* names[13] = {"readlane", "lds", "lds2", "lds-nobar", "lds2-nobar", "rl-scalar", "fma-only", "hyb8", "hyb12", "hyb16", "hyb20", "hyb24", "2d"};
  for (int v = 0; v < 13; v++) {
    double meanr[2] = {0, 0}, maxr[2] = {0, 0};
    std::vector<float> W(H.size());
    for (int k = 0; k < 2; k++) {
      const int reps = k ? 9 : 1;
      for (int w = 0; w < 3; w++) {
        if (v == 0) hipLaunchKernelGGL(kern<0>, dim3(B), dim3(64), 0, 0, dH, dW, dc, reps);
        if (v == 1) hipLaunchKernelGGL(kern<1>, dim3(B), dim3(64), 0, 0, dH, dW, dc, reps);
        if (v == 2) hipLaunchKernelGGL(kern<2>, dim3(B), dim3(64), 0, 0, dH, dW, dc, reps);
        if (v == 3) hipLaunchKernelGGL(kern<3>, dim3(B), dim3(64), 0, 0, dH, dW, dc, reps);
        if (v == 4) hipLaunchKernelGGL(kern<4>, dim3(B), dim3(64), 0, 0, dH, dW, dc, reps);
        if (v == 5) hipLaunchKernelGGL(kern<5>, dim3(B), dim3(64), 0, 0, dH, dW, dc, reps);
        if (v == 6) hipLaunchKernelGGL(kern<6>, dim3(B), dim3(64), 0, 0, dH, dW, dc, reps);
        if (v == 7) hipLaunchKernelGGL(kern<7>, dim3(B), dim3(64), 0, 0, dH, dW, dc, reps);
        if (v == 8) hipLaunchKernelGGL(kern<8>, dim3(B), dim3(64), 0, 0, dH, dW, dc, reps);
        if (v == 9) hipLaunchKernelGGL(kern<9>, dim3(B), dim3(64), 0, 0, dH, dW, dc, reps);
        if (v == 10) hipLaunchKernelGGL(kern<10>, dim3(B), dim3(64), 0, 0, dH, dW, dc, reps);
        if (v == 11) hipLaunchKernelGGL(kern<11>, dim3(B), dim3(64), 0, 0, dH, dW, dc, reps);
        if (v == 12) hipLaunchKernelGGL(kern2d, dim3(B), dim3(64), 0, 0, dH, dW, dc, reps);
      }
      hipDeviceSynchronize();
      std::vector<long long> c(B);
      hipMemcpy(c.data(), dc, B * 8, hipMemcpyDeviceToHost);
      hipMemcpy(W.data(), dW, W.size() * 4, hipMemcpyDeviceToHost);
      for (int b = 0; b < B; b++) { meanr[k] += c[b] / (double)B; maxr[k] = fmax(maxr[k], (double)c[b]); }
    }
    double res = 0;
    for (int b = 0; b < 16; b++)  // || H (-W) - I ||_max
      for (int i = 0; i < NUM; i++)
        for (int j = 0; j < NUM; j++) {
          double s = 0;
          for (int k = 0; k < NUM; k++) s -= (double)H[((size_t)b * NUM + i) * NUM + k] * W[((size_t)b * NUM + k) * NUM + j];
          res = fmax(res, fabs(s - (i == j)));
        }
    printf("NUM=%d %-10s cycles/sweep mean %8.0f (max-based %8.0f)  residual %.2e\n", NUM, names[v],
           (meanr[1] - meanr[0]) / 8, (maxr[1] - maxr[0]) / 8, res);
  }
  return 0;
}
