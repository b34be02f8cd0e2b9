// Semantics check of the gfx950 DPP wave shifts used by the segmented kernel's lane-adjacent
// segment layout: prints, for each control, the source lane every destination lane read (-1: the
// bound_ctrl zero / old value). Build: hipcc --offload-arch=gfx950 -O2 dpp_check.hip -o dpp_check
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CTRL>
__global__ void k(int* out) {
  const int lane = threadIdx.x;
  out[lane] = __builtin_amdgcn_update_dpp(-1, lane + 1000, CTRL, 0xF, 0xF, false) - 1000;
}

int main() {
  int* d;
  int h[64];
  hipMalloc(&d, 64 * sizeof(int));
  auto run = [&](auto kern, const char* name) {
    hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("%s:", name);
    for (int i = 0; i < 64; i++) printf(" %d", h[i] < -500 ? -1 : h[i]);
    printf("\n");
  };
  run(k<0x130>, "wave_shl1");
  run(k<0x138>, "wave_shr1");
  run(k<0x111>, "row_shr1");
  run(k<0x101>, "row_shl1");
  run(k<0x134>, "wave_rol1");
  run(k<0x13C>, "wave_ror1");
  hipFree(d);
  return 0;
}
