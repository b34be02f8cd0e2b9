// Launch-to-answer latency of a one-wave kernel: hipStreamSynchronize against the host spinning on
// a flag in pinned, coherent host memory that the kernel's last wave writes after a system-scope
// fence (single-QP latency). Build: hipcc --offload-arch=gfx950 -O2 flag_latency.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void work(float* out, int n, volatile unsigned* flag, unsigned seq) {
  float a = threadIdx.x;
  for (int i = 0; i < n; i++) a = a * 1.0000001f + 1e-7f;
  out[threadIdx.x] = a;
  if (flag) {
    __threadfence_system();
    if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 4);
  unsigned* flag;
  hipHostMalloc((void**)&flag, 64, hipHostMallocCoherent | hipHostMallocMapped);
  unsigned* dflag;
  hipHostGetDevicePointer((void**)&dflag, flag, 0);
  *flag = 0;
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  for (int n : {0, 20000}) {
    std::vector<double> a, b;
    for (int it = 0; it < 2200; it++) {
      auto t0 = std::chrono::steady_clock::now();
      hipLaunchKernelGGL(work, dim3(1), dim3(64), 0, s, out, n, nullptr, 0u);
      hipStreamSynchronize(s);
      auto t1 = std::chrono::steady_clock::now();
      if (it >= 200) a.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    for (unsigned it = 1; it <= 2200; it++) {
      auto t0 = std::chrono::steady_clock::now();
      hipLaunchKernelGGL(work, dim3(1), dim3(64), 0, s, out, n, dflag, it);
      while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != it) {
      }
      auto t1 = std::chrono::steady_clock::now();
      if (it > 200) b.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    hipStreamSynchronize(s);
    std::sort(a.begin(), a.end());
    std::sort(b.begin(), b.end());
    printf("{\"work_iters\": %d, \"sync_p50_us\": %.2f, \"sync_p99_us\": %.2f, \"flag_p50_us\": %.2f, \"flag_p99_us\": %.2f}\n",
           n, a[a.size() / 2], a[a.size() * 99 / 100], b[b.size() / 2], b[b.size() * 99 / 100]);
  }
  return 0;
}
