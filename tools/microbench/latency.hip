// latency.hip — gfx950 micro-benchmarks for the Riccati kernels' design: cycles per dependent
// fp64 / fp32 FMA, per fp64 quad-DPP exchange, per LDS load-to-use, per v_rcp_f64, with one
// wave per SIMD (the latency regime of small batches). Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHAIN 4096

__global__ void fma64(double* out, long long* cyc, double a, double b) {
  double x = threadIdx.x * 1e-3;
  long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 64
  for (int i = 0; i < CHAIN; i++) x = fma(x, a, b);
  long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
__global__ void fma64x4(double* out, long long* cyc, double a, double b) {  // 4 independent chains
  double x = threadIdx.x * 1e-3, y = x + 1, z = x + 2, w = x + 3;
  long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 64
  for (int i = 0; i < CHAIN; i++) { x = fma(x, a, b); y = fma(y, a, b); z = fma(z, a, b); w = fma(w, a, b); }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x + y + z + w;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
__global__ void fma32(float* out, long long* cyc, float a, float b) {
  float x = threadIdx.x * 1e-3f;
  long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 64
  for (int i = 0; i < CHAIN; i++) x = fmaf(x, a, b);
  long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
__global__ void dpp64(double* out, long long* cyc, double a, double b) {  // fma + quad bcast
  double x = threadIdx.x * 1e-3;
  long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 64
  for (int i = 0; i < CHAIN; i++) {
    int2 p = *reinterpret_cast<int2*>(&x);
    p.x = __builtin_amdgcn_mov_dpp(p.x, 0x55, 0xf, 0xf, false);
    p.y = __builtin_amdgcn_mov_dpp(p.y, 0x55, 0xf, 0xf, false);
    x = fma(*reinterpret_cast<double*>(&p), a, b);
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
__global__ void rcp64(double* out, long long* cyc, double a, double b) {
  double x = 1.5 + threadIdx.x * 1e-3;
  long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 64
  for (int i = 0; i < CHAIN; i++) x = __builtin_amdgcn_rcp(x) + b;
  long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
__global__ void lds64(double* out, long long* cyc, double a, double b) {  // pointer chase in LDS
  __shared__ int idx[64 * 64];
  for (int i = threadIdx.x; i < 64 * 64; i += 64) idx[i] = (i + 64) % (64 * 64);
  __syncthreads();
  int p = threadIdx.x;
  long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
  for (int i = 0; i < CHAIN; i++) p = idx[p];
  long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = p;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  double* d; long long* c; float* f;
  hipMalloc(&d, 64 * 8); hipMalloc(&c, 8 * 1024); hipMalloc(&f, 64 * 4);
  long long h[1];
  struct { const char* n; void (*k)(double*, long long*, double, double); } ks[] = {
      {"fp64 fma dependent", fma64}, {"fp64 fma 4 chains (per step)", fma64x4},
      {"fp64 quad-dpp + fma", dpp64}, {"fp64 rcp + add", rcp64}, {"lds b32 load chase", lds64}};
  for (auto& k : ks) {
    for (int rep = 0; rep < 3; rep++) {
      hipLaunchKernelGGL(k.k, dim3(1), dim3(64), 0, 0, d, c, 1.0000001, 1e-9);
      hipDeviceSynchronize();
    }
    hipMemcpy(h, c, 8, hipMemcpyDeviceToHost);
    printf("%-32s %6.2f cycles/step\n", k.n, (double)h[0] / CHAIN);
  }
  for (int rep = 0; rep < 3; rep++) {
    hipLaunchKernelGGL(fma32, dim3(1), dim3(64), 0, 0, f, c, 1.0000001f, 1e-9f);
    hipDeviceSynchronize();
  }
  hipMemcpy(h, c, 8, hipMemcpyDeviceToHost);
  printf("%-32s %6.2f cycles/step\n", "fp32 fma dependent", (double)h[0] / CHAIN);
  // s_memtime vs wall clock: one long fp64 chain kernel timed both ways
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int rep = 0; rep < 100; rep++) hipLaunchKernelGGL(fma64, dim3(1), dim3(64), 0, 0, d, c, 1.0000001, 1e-9);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  hipMemcpy(h, c, 8, hipMemcpyDeviceToHost);
  printf("fp64 chain kernel: %.2f us per launch (events), %lld memtime cycles in the chain\n", ms * 10, h[0]);
  return 0;
}
