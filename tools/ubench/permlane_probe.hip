// Semantics probe (gfx950): v_permlane16_swap_b32 / v_permlane32_swap_b32
// on lane ids, both outputs of each, printed per 16-lane row.
//   hipcc --offload-arch=gfx950 -O3 -o permlane_probe tools/ubench/permlane_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* o) {
  unsigned v = threadIdx.x, w = threadIdx.x + 100;
  auto r = __builtin_amdgcn_permlane16_swap(v, w, false, false);
  auto s = __builtin_amdgcn_permlane32_swap(v, w, false, false);
  o[threadIdx.x] = r[0]; o[64 + threadIdx.x] = r[1]; o[128 + threadIdx.x] = s[0]; o[192 + threadIdx.x] = s[1];
}
int main() {
  unsigned *d, h[256];
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  const char* nm[4] = {"swap16.vdst(old=lane)", "swap16.src0(old=lane+100)", "swap32.vdst(old=lane)", "swap32.src0(old=lane+100)"};
  for (int q = 0; q < 4; q++) {
    printf("%s:", nm[q]);
    for (int r = 0; r < 4; r++) printf("  row%d=[%u..%u]", r, h[64 * q + 16 * r], h[64 * q + 16 * r + 15]);
    printf("\n");
  }
  return 0;
}
