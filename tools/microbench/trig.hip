// trig.hip — device fp64 cos/sin/sincos vs the host libm on the same arguments (ulp counts).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

__global__ void k(const float* a, double* c, double* s, double* c2, double* s2, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double x = (double)a[i];
  c[i] = cos(x);
  s[i] = sin(x);
  double ss, cc;
  sincos(x, &ss, &cc);
  c2[i] = cc;
  s2[i] = ss;
}

static long long ulps(double a, double b) {
  long long ia, ib;
  memcpy(&ia, &a, 8); memcpy(&ib, &b, 8);
  return llabs(ia - ib);
}

int main() {
  const int n = 1 << 20;
  float* ha = (float*)malloc(n * 4);
  srand(1);
  for (int i = 0; i < n; i++) ha[i] = (float)(((double)rand() / RAND_MAX) * 8.0 - 4.0);
  float* da; double *dc, *ds, *dc2, *ds2;
  hipMalloc(&da, n * 4); hipMalloc(&dc, n * 8); hipMalloc(&ds, n * 8); hipMalloc(&dc2, n * 8); hipMalloc(&ds2, n * 8);
  hipMemcpy(da, ha, n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, da, dc, ds, dc2, ds2, n);
  double *hc = (double*)malloc(n * 8), *hs = (double*)malloc(n * 8), *hc2 = (double*)malloc(n * 8), *hs2 = (double*)malloc(n * 8);
  hipMemcpy(hc, dc, n * 8, hipMemcpyDeviceToHost); hipMemcpy(hs, ds, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(hc2, dc2, n * 8, hipMemcpyDeviceToHost); hipMemcpy(hs2, ds2, n * 8, hipMemcpyDeviceToHost);
  long long h[4][4] = {{0}};
  for (int i = 0; i < n; i++) {
    const double x = (double)ha[i];
    const long long u[4] = {ulps(hc[i], cos(x)), ulps(hs[i], sin(x)), ulps(hc2[i], cos(x)), ulps(hs2[i], sin(x))};
    for (int j = 0; j < 4; j++) h[j][u[j] == 0 ? 0 : u[j] == 1 ? 1 : u[j] <= 16 ? 2 : 3]++;
  }
  const char* nm[4] = {"cos", "sin", "sincos.c", "sincos.s"};
  for (int j = 0; j < 4; j++)
    printf("%-9s exact %lld  1ulp %lld  2-16ulp %lld  >16ulp %lld\n", nm[j], h[j][0], h[j][1], h[j][2], h[j][3]);
  return 0;
}
