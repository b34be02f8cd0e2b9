// mfma_wg.hip — the one measurement behind the MFMA decision:
// the grouped (C4) first pass Y = W * [g_1 .. g_G], one 2N x 2N W = H^-1 shared by the G = 120
// candidates of a scenario, N = 40 (2N = 80). Per scenario a (80 x 80) * (80 x 120) fp32 GEMM,
// 546 scenarios (C4's 65,536 candidates). Two kernels, one 256-thread workgroup per scenario,
// both staging W and G in LDS:
//   mfma : v_mfma_f32_16x16x4_f32 (exact f32: a k-ordered fmaf chain), 5 x 8 output tiles of
//          16 x 16, each wave owns 2 column tiles (10 accumulators), K = 80 in 20 steps;
//   valu : each thread one column j and 40 rows, v_pk_fma_f32 over row pairs, W broadcast from LDS.
// Times both with HIP events (µs per launch, TFLOP/s vs the 157.3 TF fp32 peak) and checks them
// against each other. Build: hipcc -O3 --offload-arch=gfx950 mfma_wg.hip -o mfma_wg
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

constexpr int NV = 80;    // 2N decision variables (N = 40)
constexpr int NG = 120;   // candidates per scenario (6 lanes x 20 steers)
constexpr int NGP = 128;  // padded to 8 column tiles
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void wg_mfma(const float* __restrict__ W, const float* __restrict__ G,
                                               float* __restrict__ Y) {
  __shared__ float sW[NV][NV + 1];
  __shared__ float sG[NV][NGP + 1];
  const int s = blockIdx.x, t = threadIdx.x;
  const float* w = W + (size_t)s * NV * NV;
  const float* g = G + (size_t)s * NV * NG;
  for (int e = t; e < NV * NV; e += 256) sW[e / NV][e % NV] = w[e];
  for (int e = t; e < NV * NGP; e += 256) {
    const int k = e / NGP, j = e % NGP;
    sG[k][j] = j < NG ? g[k * NG + j] : 0.f;
  }
  __syncthreads();
  const int wave = t >> 6, l = t & 63;
  f32x4 acc[5][2];
#pragma unroll
  for (int i = 0; i < 5; i++)
#pragma unroll
    for (int c = 0; c < 2; c++) acc[i][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int ct0 = 2 * wave;  // column tiles 2w, 2w+1
#pragma unroll 4
  for (int k0 = 0; k0 < NV; k0 += 4) {
    const int kk = k0 + (l >> 4);
    float a[5], b[2];
#pragma unroll
    for (int i = 0; i < 5; i++) a[i] = sW[16 * i + (l & 15)][kk];  // A[row][k]
#pragma unroll
    for (int c = 0; c < 2; c++) b[c] = sG[kk][16 * (ct0 + c) + (l & 15)];  // B[k][col]
#pragma unroll
    for (int i = 0; i < 5; i++)
#pragma unroll
      for (int c = 0; c < 2; c++) acc[i][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[c], acc[i][c], 0, 0, 0);
  }
  float* y = Y + (size_t)s * NV * NG;
#pragma unroll
  for (int i = 0; i < 5; i++)
#pragma unroll
    for (int c = 0; c < 2; c++) {
      const int col = 16 * (ct0 + c) + (l & 15);
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = 16 * i + 4 * (l >> 4) + r;  // C/D: col = l & 15, row = 4 (l >> 4) + r
        if (col < NG) y[row * NG + col] = acc[i][c][r];
      }
    }
}

__global__ __launch_bounds__(256) void wg_valu(const float* __restrict__ W, const float* __restrict__ G,
                                               float* __restrict__ Y) {
  __shared__ float sW[NV][NV];
  __shared__ float sG[NV][NGP];
  const int s = blockIdx.x, t = threadIdx.x;
  const float* w = W + (size_t)s * NV * NV;
  const float* g = G + (size_t)s * NV * NG;
  for (int e = t; e < NV * NV; e += 256) sW[e / NV][e % NV] = w[e];
  for (int e = t; e < NV * NGP; e += 256) {
    const int k = e / NGP, j = e % NGP;
    sG[k][j] = j < NG ? g[k * NG + j] : 0.f;
  }
  __syncthreads();
  const int j = t & 127, i0 = (t >> 7) * 40;  // one column, 40 rows
  f32x2 acc[20];
#pragma unroll
  for (int i = 0; i < 20; i++) acc[i] = f32x2{0.f, 0.f};
#pragma unroll 2
  for (int k = 0; k < NV; k++) {
    const float gk = sG[k][j];
    const f32x2 g2 = {gk, gk};
#pragma unroll
    for (int i = 0; i < 20; i++) {
      const f32x2 w2 = {sW[i0 + 2 * i][k], sW[i0 + 2 * i + 1][k]};  // wave-uniform: LDS broadcast
      acc[i] = __builtin_elementwise_fma(w2, g2, acc[i]);
    }
  }
  if (j < NG) {
    float* y = Y + (size_t)s * NV * NG;
#pragma unroll
    for (int i = 0; i < 20; i++) {
      y[(i0 + 2 * i) * NG + j] = acc[i].x;
      y[(i0 + 2 * i + 1) * NG + j] = acc[i].y;
    }
  }
}

int main(int argc, char** argv) {
  const int S = argc > 1 ? atoi(argv[1]) : 546;
  const int reps = argc > 2 ? atoi(argv[2]) : 50;
  std::vector<float> hW((size_t)S * NV * NV), hG((size_t)S * NV * NG);
  srand(7);
  for (auto& v : hW) v = (float)((double)rand() / RAND_MAX) - 0.5f;
  for (auto& v : hG) v = (float)((double)rand() / RAND_MAX) - 0.5f;
  float *dW, *dG, *dY1, *dY2;
  CK(hipMalloc(&dW, hW.size() * 4));
  CK(hipMalloc(&dG, hG.size() * 4));
  CK(hipMalloc(&dY1, hG.size() * 4));
  CK(hipMalloc(&dY2, hG.size() * 4));
  CK(hipMemcpy(dW, hW.data(), hW.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dG, hG.data(), hG.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const double flops = 2.0 * NV * NV * NG * S;
  float ms[2];
  for (int kind = 0; kind < 2; kind++) {
    float* y = kind ? dY2 : dY1;
    for (int w = 0; w < 3; w++) {
      if (kind) hipLaunchKernelGGL(wg_valu, dim3(S), dim3(256), 0, 0, dW, dG, y);
      else hipLaunchKernelGGL(wg_mfma, dim3(S), dim3(256), 0, 0, dW, dG, y);
    }
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; r++) {
      if (kind) hipLaunchKernelGGL(wg_valu, dim3(S), dim3(256), 0, 0, dW, dG, y);
      else hipLaunchKernelGGL(wg_mfma, dim3(S), dim3(256), 0, 0, dW, dG, y);
    }
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms[kind], a, b));
    ms[kind] /= reps;
  }
  std::vector<float> y1(hG.size()), y2(hG.size());
  CK(hipMemcpy(y1.data(), dY1, y1.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(y2.data(), dY2, y2.size() * 4, hipMemcpyDeviceToHost));
  // fp64 reference on scenario 0 and the max difference of the two kernels everywhere
  double e1 = 0, e2 = 0, d12 = 0;
  for (int i = 0; i < NV; i++)
    for (int j = 0; j < NG; j++) {
      double r = 0;
      for (int k = 0; k < NV; k++) r += (double)hW[i * NV + k] * hG[k * NG + j];
      e1 = fmax(e1, fabs(y1[i * NG + j] - r));
      e2 = fmax(e2, fabs(y2[i * NG + j] - r));
    }
  for (size_t e = 0; e < y1.size(); e++) d12 = fmax(d12, fabs((double)y1[e] - y2[e]));
  const char* nm[2] = {"mfma_f32_16x16x4", "valu_pk_fma_f32"};
  printf("{\"scenarios\": %d, \"gemm\": \"(80x80)*(80x120) fp32 per scenario\", \"flops_per_launch\": %.0f", S, flops);
  for (int k = 0; k < 2; k++)
    printf(", \"%s\": {\"us\": %.3f, \"tflops\": %.3f, \"frac_of_157.3\": %.4f}", nm[k], ms[k] * 1e3,
           flops / (ms[k] * 1e-3) / 1e12, flops / (ms[k] * 1e-3) / 1e12 / 157.3);
  printf(", \"max_abs_err_vs_fp64\": [%.3g, %.3g], \"max_abs_diff\": %.3g}\n", e1, e2, d12);
  return 0;
}
