// Carry-chain microbenchmark (gfx950): the centered field products of
// fd25519_fe.h (rounding carries, 64-bit adds in the chain) against the
// unsigned-limb forms (_u: floor carries, each column started from the
// previous column's carry).  Squaring chains of 1 (a decompression's
// exponentiation: one serial chain per lane) and 4 (a doubling's four
// independent squarings) per lane, and 3 interleaved products, at 2 waves
// per SIMD like the decode and dsm kernels (latency exposed: the interleave
// of the other wave is all that hides it) and at 8 (issue-bound).  The _u results are checked
// against the centered ones on the device (canonical bytes) first.
//
//   hipcc --offload-arch=gfx950 -O3 -I firedancer_amd/csrc -o fe_carry_ubench tools/ubench/fe_carry_ubench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include "fd25519_fe.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

__device__ void load_in(fe& a, const int32_t* in, int t, int c) {
  uint32_t w[8];
  for (int i = 0; i < 8; i++) w[i] = (uint32_t)in[(t * 4 + c) * 8 + i];
  fe_frombytes(a, w);
}

__global__ void __launch_bounds__(256, 2) k_check(const int32_t* in, int* bad, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  fe a, b, au, bu;
  load_in(a, in, t, 0);
  load_in(b, in, t, 1);
  au = a; bu = b;
  int err = 0;
  for (int it = 0; it < iters; it++) {
    fe s, su, m, mu, s2, s2u;
    fe_sq(s, a);     fe_sq_u(su, au);
    fe_mul(m, a, b); fe_mul_u(mu, au, bu);
    fe_sq2(s2, b);   fe_sq2_u(s2u, bu);
    uint32_t x[8], y[8];
    fe_tobytes(x, s);  fe_tobytes(y, su);  for (int i = 0; i < 8; i++) err |= x[i] != y[i];
    fe_tobytes(x, m);  fe_tobytes(y, mu);  for (int i = 0; i < 8; i++) err |= x[i] != y[i];
    fe_tobytes(x, s2); fe_tobytes(y, s2u); for (int i = 0; i < 8; i++) err |= x[i] != y[i];
    /* the _u outputs must stay within the unsigned bound */
    for (int i = 0; i < 10; i++) {
      const int32_t lim = (i & 1) ? (1 << 25) + 1024 : (1 << 26) + 1024;
      err |= (su.v[i] < -1024 || su.v[i] >= lim) | (mu.v[i] < -1024 || mu.v[i] >= lim);
    }
    /* next round: centered chain on centered values, _u chain on _u values,
       with a difference of two _u outputs (<= 2x) as one operand */
    a = s; au = su;
    fe_sub(b, m, s2); fe_sub(bu, mu, s2u);
  }
  if (err) atomicAdd(bad, 1);
}

template <int U, int CH>
__global__ void __launch_bounds__(256, 2) k_sq(const int32_t* in, int32_t* out, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  fe a[4];
  for (int c = 0; c < CH; c++) load_in(a[c], in, t, c);
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < CH; c++) {
      if (U) fe_sq_u(a[c], a[c]);
      else fe_sq(a[c], a[c]);
    }
  }
  int32_t s = 0;
  for (int c = 0; c < CH; c++) for (int i = 0; i < 10; i++) s ^= a[c].v[i];
  out[t] = s;
}

template <int U>
__global__ void __launch_bounds__(256, 2) k_mul(const int32_t* in, int32_t* out, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  fe a[3];
  for (int c = 0; c < 3; c++) load_in(a[c], in, t, c);
  for (int it = 0; it < iters; it++) {
    if (U) { fe_mul_u(a[0], a[0], a[1]); fe_mul_u(a[1], a[1], a[2]); fe_mul_u(a[2], a[2], a[0]); }
    else   { fe_mul(a[0], a[0], a[1]);   fe_mul(a[1], a[1], a[2]);   fe_mul(a[2], a[2], a[0]); }
  }
  int32_t s = 0;
  for (int c = 0; c < 3; c++) for (int i = 0; i < 10; i++) s ^= a[c].v[i];
  out[t] = s;
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int block = 256, max_lanes = cus * 8 * block;
  int32_t *in, *out;
  int* bad;
  CHECK(hipMalloc(&in, sizeof(int32_t) * max_lanes * 32));
  CHECK(hipMalloc(&out, sizeof(int32_t) * max_lanes));
  CHECK(hipMalloc(&bad, sizeof(int)));
  int32_t* h = (int32_t*)malloc(sizeof(int32_t) * max_lanes * 32);
  uint64_t x = 88172645463325252ull;
  for (long i = 0; i < (long)max_lanes * 32; i++) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; h[i] = (int32_t)x; }
  /* a few lanes at the top of the range (limbs near 2^w - 1) */
  for (int t = 0; t < 64; t++) for (int i = 0; i < 32; i++) h[t * 32 + i] = -1;
  CHECK(hipMemcpy(in, h, sizeof(int32_t) * max_lanes * 32, hipMemcpyHostToDevice));
  CHECK(hipMemset(bad, 0, sizeof(int)));
  hipLaunchKernelGGL(k_check, dim3(cus * 2), dim3(block), 0, 0, in, bad, 256);
  int hbad = -1;
  CHECK(hipMemcpy(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost));
  printf("unsigned-limb forms vs centered: %d of %d lanes differ (256 rounds)\n", hbad, cus * 2 * block);
  if (hbad) return 1;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  const int iters = 400;
  struct { const char* name; void (*f)(const int32_t*, int32_t*, int); double ops_per_iter; } ks[] = {
    {"fe_sq   x1 (centered)", k_sq<0, 1>, 1}, {"fe_sq_u x1 (unsigned)", k_sq<1, 1>, 1},
    {"fe_sq   x4 (centered)", k_sq<0, 4>, 4}, {"fe_sq_u x4 (unsigned)", k_sq<1, 4>, 4},
    {"fe_mul  x3 (centered)", k_mul<0>, 3},   {"fe_mul_u x3 (unsigned)", k_mul<1>, 3},
  };
  for (int wps : {2, 8}) {   /* resident waves per SIMD: grid of wps blocks of 4 waves per CU */
  const int grid = cus * wps, lanes = grid * block;
  printf("-- %d waves per SIMD\n", wps);
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.f, dim3(grid), dim3(block), 0, 0, in, out, iters);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(k.f, dim3(grid), dim3(block), 0, 0, in, out, iters);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    const double ops = (double)lanes * iters * k.ops_per_iter;
    printf("%-24s %8.3f ms  %7.2f G field ops/s  %6.1f SIMD-cycles per op per wave at 2.4 GHz\n", k.name, best,
           ops / (best * 1e-3) / 1e9, best * 1e-3 * 2.4e9 * cus * 4 / (ops / 64));
  }
  }
  return 0;
}
