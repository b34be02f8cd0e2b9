// contention.hip — does a one-wave-per-SIMD kernel slow down when the other SIMDs of its CU are
// busy? Each kernel is a fixed per-wave instruction stream; it is launched with 128, 256, 1024
// and 2048 one-wave workgroups (1 wave on half the CUs, 1 per CU, 1 per SIMD, 2 per SIMD) and
// reports the wall time per launch (events) and the mean per-wave s_memtime cycles.
// Build: hipcc --offload-arch=gfx950 -O3 contention.hip -o contention
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define STEPS 2048
#ifndef NREP
#define NREP 10
#endif

// 4 independent fp64 FMA chains
__global__ __launch_bounds__(64) void k_fp64(double* out, long long* cyc, double a, double b) {
  double x = threadIdx.x * 1e-3, y = x + 1, z = x + 2, w = x + 3;
  long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 32
  for (int i = 0; i < STEPS; i++) { x = fma(x, a, b); y = fma(y, a, b); z = fma(z, a, b); w = fma(w, a, b); }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = x + y + z + w;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
// 4 independent fp32 FMA chains
__global__ __launch_bounds__(64) void k_fp32(double* out, long long* cyc, double a, double b) {
  float x = threadIdx.x * 1e-3f, y = x + 1, z = x + 2, w = x + 3;
  const float fa = (float)a, fb = (float)b;
  long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 32
  for (int i = 0; i < STEPS; i++) { x = fmaf(x, fa, fb); y = fmaf(y, fa, fb); z = fmaf(z, fa, fb); w = fmaf(w, fa, fb); }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = x + y + z + w;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
// integer / select VALU (v_cndmask, v_add_u32)
__global__ __launch_bounds__(64) void k_int(double* out, long long* cyc, double a, double b) {
  unsigned x = threadIdx.x, y = x + 1, z = x + 2, w = x + 3;
  long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 32
  for (int i = 0; i < STEPS; i++) { x = x * 3u + 1u; y = y * 5u + 7u; z = z * 9u + 3u; w = w * 7u + 5u; }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = (double)(x + y + z + w);
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
// LDS: fp64 writes + reads (8 B / lane), the lane kernel's scratch pattern
__global__ __launch_bounds__(64) void k_lds(double* out, long long* cyc, double a, double b) {
  __shared__ double s[64 * 16];
  double acc = threadIdx.x;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < STEPS / 8; i++) {
#pragma unroll
    for (int e = 0; e < 8; e++) s[e * 64 + threadIdx.x] = acc + e;
#pragma unroll
    for (int e = 0; e < 8; e++) acc += s[((e + i) & 15) * 64 + threadIdx.x];
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// the fp64 loop again with 200 VGPRs allocated (occupancy 2 waves per SIMD, as the lane kernel),
// recording where each wave ran (HW_ID: wave, SIMD, CU, SH, SE)
__global__ __launch_bounds__(64) void k_fp64_fat(double* out, long long* cyc, double a, double b) {
  asm volatile("v_mov_b32 v199, 0" ::: "v199");
  double x = threadIdx.x * 1e-3, y = x + 1, z = x + 2, w = x + 3;
  long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 32
  for (int i = 0; i < STEPS; i++) { x = fma(x, a, b); y = fma(y, a, b); z = fma(z, a, b); w = fma(w, a, b); }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = x + y + z + w;
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
  if (threadIdx.x == 0) cyc[blockIdx.x] = ((t1 - t0) << 20) | (hw & 0xfffff);
}

// lane-kernel-like stage loop: fp64 chain with rcp, selects and a dependent LDS read per step;
// ACTIVE lanes only (8 of 64 when partial) — which ingredient slows with 4 waves per CU?
template <int MODE>
__global__ __launch_bounds__(64) void k_mix(double* out, long long* cyc, double a, double b) {
  asm volatile("v_mov_b32 v199, 0" ::: "v199");
  __shared__ double s[64 * 8];
  const int lane = threadIdx.x;
  double x = lane * 1e-3 + 1.0, y = x + 1, z = x + 2, w = x + 3;
  for (int i = lane; i < 64 * 8; i += 64) s[i] = 1.0 + i * 1e-6;
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  const bool act = (MODE & 1) ? lane < 8 : true;
  if (act) {
    for (int i = 0; i < STEPS / 8; i++) {
#pragma unroll
      for (int k = 0; k < 8; k++) {
        x = fma(x, a, b); y = fma(y, x, b); z = fma(z, a, y); w = fma(w, z, b);
        if (MODE & 2) x = x + __builtin_amdgcn_rcp(w) * 1e-9;
        if (MODE & 4) y = (w > 2.0) ? y : x;
        if (MODE & 8) z = z + s[((int)(x * 7.0) & 7) * 64 + lane] * 1e-9;
      }
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = x + y + z + w;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// same-address LDS writes: lanes write slot (lane % DUP) of each row (DUP = 64: no sharing)
template <int DUP>
__global__ __launch_bounds__(64) void k_ldsdup(double* out, long long* cyc, double a, double b) {
  __shared__ double s[64 * 16];
  const int lane = threadIdx.x, slot = lane % DUP;
  double acc = lane;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < STEPS / 8; i++) {
#pragma unroll
    for (int e = 0; e < 8; e++) s[e * 64 + slot] = acc + e;
#pragma unroll
    for (int e = 0; e < 8; e++) acc += s[((e + i) & 15) * 64 + slot];
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  double* d; long long* c;
  hipMalloc(&d, 4096 * 64 * 8); hipMalloc(&c, 4096 * 8);
  long long h[4096];
  struct { const char* n; void (*k)(double*, long long*, double, double); } ks[] = {
      {"fp64 fma x4", k_fp64}, {"fp32 fma x4", k_fp32}, {"int mad x4", k_int}, {"lds fp64 w/r", k_lds}};
  const int grids[] = {128, 256, 1024, 2048, 4096};
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (auto& k : ks) {
    if (getenv("SKIP_BASIC")) break;
    for (int g : grids) {
      hipLaunchKernelGGL(k.k, dim3(g), dim3(64), 0, 0, d, c, 1.0000001, 1e-9);
      hipDeviceSynchronize();
      hipEventRecord(e0);
      for (int r = 0; r < NREP; r++) hipLaunchKernelGGL(k.k, dim3(g), dim3(64), 0, 0, d, c, 1.0000001, 1e-9);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      hipMemcpy(h, c, g * 8, hipMemcpyDeviceToHost);
      double m = 0; for (int i = 0; i < g; i++) m += h[i]; m /= g;
      printf("%-14s grid %5d: %8.2f us/launch, %8.0f cycles/wave (%.2f per step-instr), clock %.2f GHz (last launch)\n", k.n, g,
             ms * 1000.0 / NREP, m, m / (4.0 * STEPS), m / (ms * 1e6 / NREP));
    }
  }
  {
    struct { const char* n; void (*k)(double*, long long*, double, double); } km[] = {
        {"mix chain", k_mix<0>}, {"mix 8 lanes", k_mix<1>}, {"mix +rcp", k_mix<2>}, {"mix +sel", k_mix<4>},
        {"mix +lds", k_mix<8>}, {"mix all", k_mix<14>}, {"mix all 8 lanes", k_mix<15>},
        {"lds dup 64", k_ldsdup<64>}, {"lds dup 8", k_ldsdup<8>}, {"lds dup 1", k_ldsdup<1>}};
    for (auto& k : km) {
      for (int g : {128, 1024}) {
        hipLaunchKernelGGL(k.k, dim3(g), dim3(64), 0, 0, d, c, 1.0000001, 1e-9);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        for (int r = 0; r < 10; r++) hipLaunchKernelGGL(k.k, dim3(g), dim3(64), 0, 0, d, c, 1.0000001, 1e-9);
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        hipMemcpy(h, c, g * 8, hipMemcpyDeviceToHost);
        double m = 0; for (int i = 0; i < g; i++) m += h[i]; m /= g;
        printf("%-16s grid %5d: %8.2f us/launch, %8.0f cycles/wave\n", k.n, g, ms * 100.0, m);
      }
    }
  }
  // placement of 1,024 one-wave workgroups of a 200-VGPR kernel
  for (int g : {256, 1024}) {
    hipLaunchKernelGGL(k_fp64_fat, dim3(g), dim3(64), 0, 0, d, c, 1.0000001, 1e-9);
    hipDeviceSynchronize();
    hipMemcpy(h, c, g * 8, hipMemcpyDeviceToHost);
    int simd_hist[4] = {0, 0, 0, 0};
    // waves per (SE, SH, CU, SIMD)
    static int per[4096];
    for (int i = 0; i < 4096; i++) per[i] = 0;
    double m = 0;
    for (int i = 0; i < g; i++) {
      const unsigned hw = (unsigned)(h[i] & 0xfffff);
      const int simd = (hw >> 4) & 3, cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
      simd_hist[simd]++;
      per[(((se * 2 + sh) * 16 + cu) * 4) + simd]++;
      m += (double)(h[i] >> 20);
    }
    int mx = 0, used = 0;
    for (int i = 0; i < 4096; i++) { if (per[i] > mx) mx = per[i]; if (per[i]) used++; }
    printf("fat fp64 grid %d: mean %.0f cycles/wave; waves on SIMD0..3: %d %d %d %d; slots used %d, max waves per slot %d\n",
           g, m / g, simd_hist[0], simd_hist[1], simd_hist[2], simd_hist[3], used, mx);
  }
  return 0;
}
