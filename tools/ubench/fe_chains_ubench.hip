// Column-chain microbenchmark (gfx950): the unsigned-limb products of
// fd25519_fe.h split into NC independent column chains (NC = 2 is the
// shipped form: columns 0..4 and 5..9).  Each chain starts from zero and
// carries column to column through the first multiply-add's addend; the
// chains are joined at the end (carry into the next chain's first limb,
// re-split into the limb after it; the last chain's carry times 19 into
// limb 0).  More chains = more independent multiply-adds in flight per
// wave (the dsm kernel runs 2 waves per SIMD, decode 4), at the price of
// one join (~4 instructions) per extra chain.
//
// Also: two serial squaring chains per lane (decode A and R in one lane)
// against one, at 2..4 waves per SIMD.
//
//   hipcc --offload-arch=gfx950 -O3 -I firedancer_amd/csrc -o fe_chains_ubench tools/ubench/fe_chains_ubench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include "fd25519_fe.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

template <int NC> struct chains;
template <> struct chains<2> { static constexpr int s[3] = {0, 5, 10}; static constexpr int len = 5; };
template <> struct chains<3> { static constexpr int s[4] = {0, 4, 7, 10}; static constexpr int len = 4; };
template <> struct chains<4> { static constexpr int s[5] = {0, 3, 5, 8, 10}; static constexpr int len = 3; };

template <int NC>
__device__ __forceinline__ void join_c(int32_t (&u)[10], int64_t (&c)[4]) {
#pragma unroll
  for (int ch = 0; ch < NC; ch++) {
    if (ch + 1 < NC) {
      const int l = chains<NC>::s[ch + 1];
      const int w = (l & 1) ? 25 : 26;
      const int64_t t = c[ch] + (int64_t)(uint32_t)u[l];
      u[l] = (int32_t)t & ((1 << w) - 1);
      u[l + 1] += (int32_t)(t >> w);
    } else {
      const int64_t t = c[ch] * 19 + (int64_t)(uint32_t)u[0];
      u[0] = (int32_t)t & ((1 << 26) - 1);
      u[1] += (int32_t)(t >> 26);
    }
  }
}

template <int NC>
__device__ __forceinline__ void mul19_c(fe& h, const fe& f, const fe& g, const fe& g19) {
  int32_t u[10];
  int64_t c[4] = {0, 0, 0, 0};
#pragma unroll
  for (int t = 0; t < chains<NC>::len; t++) {
#pragma unroll
    for (int ch = 0; ch < NC; ch++) {
      const int k = chains<NC>::s[ch] + t;
      if (k >= chains<NC>::s[ch + 1]) continue;
      int64_t acc = c[ch];
#pragma unroll
      for (int n = 0; n < 10; n++) {
        const int i = n, j = (k - i + 10) % 10;
        const int32_t x = ((i & 1) && (j & 1)) ? 2 * f.v[i] : f.v[i];
        const int32_t y = (i + j >= 10) ? g19.v[j] : g.v[j];
        if (t == 0 && n == 0) acc = (int64_t)x * y;
        else acc += (int64_t)x * y;
        asm("" : "+v"(acc));
      }
      const int w = (k & 1) ? 25 : 26;
      u[k] = (int32_t)acc & ((1 << w) - 1);
      c[ch] = acc >> w;
    }
  }
  join_c<NC>(u, c);
  fe_launder_u(h, u);
}

template <int NC>
__device__ __forceinline__ void mul_c(fe& h, const fe& f, const fe& g) {
  fe g19;
  fe_19(g19, g);
  mul19_c<NC>(h, f, g, g19);
}

template <int NC, int S>
__device__ __forceinline__ void sqs_c(fe& h, const fe& f) {
  int32_t u[10];
  int64_t c[4] = {0, 0, 0, 0};
#pragma unroll
  for (int t = 0; t < chains<NC>::len; t++) {
#pragma unroll
    for (int ch = 0; ch < NC; ch++) {
      const int k = chains<NC>::s[ch] + t;
      if (k >= chains<NC>::s[ch + 1]) continue;
      int64_t acc = c[ch];
      bool first = (t == 0);
#pragma unroll
      for (int i = 0; i < 10; i++) {
#pragma unroll
        for (int j = i; j < 10; j++) {
          if ((i + j) % 10 != k) continue;
          const int m = (((i & 1) && (j & 1)) ? 2 : 1) * ((i + j >= 10) ? 19 : 1);
          const int32_t x = (i == j) ? S * f.v[i] : 2 * S * f.v[i];
          const int32_t y = m * f.v[j];
          if (first) acc = (int64_t)x * y;
          else acc += (int64_t)x * y;
          first = false;
          asm("" : "+v"(acc));
        }
      }
      const int w = (k & 1) ? 25 : 26;
      u[k] = (int32_t)acc & ((1 << w) - 1);
      c[ch] = acc >> w;
    }
  }
  join_c<NC>(u, c);
  fe_launder_u(h, u);
}

__device__ void load_in(fe& a, const int32_t* in, int t, int c) {
  uint32_t w[8];
  for (int i = 0; i < 8; i++) w[i] = (uint32_t)in[(t * 4 + c) * 8 + i];
  fe_frombytes(a, w);
}

template <int NC>
__global__ void __launch_bounds__(256, 2) k_check(const int32_t* in, int* bad, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  fe a, b, au, bu;
  load_in(a, in, t, 0);
  load_in(b, in, t, 1);
  au = a; bu = b;
  int err = 0;
  for (int it = 0; it < iters; it++) {
    fe s, su, m, mu, s2, s2u;
    fe_sq(s, a);     sqs_c<NC, 1>(su, au);
    fe_mul(m, a, b); mul_c<NC>(mu, au, bu);
    fe_sq2(s2, b);   sqs_c<NC, 2>(s2u, bu);
    uint32_t x[8], y[8];
    fe_tobytes(x, s);  fe_tobytes(y, su);  for (int i = 0; i < 8; i++) err |= x[i] != y[i];
    fe_tobytes(x, m);  fe_tobytes(y, mu);  for (int i = 0; i < 8; i++) err |= x[i] != y[i];
    fe_tobytes(x, s2); fe_tobytes(y, s2u); for (int i = 0; i < 8; i++) err |= x[i] != y[i];
    for (int i = 0; i < 10; i++) {
      const int32_t lim = (i & 1) ? (1 << 25) + (1 << 15) : (1 << 26) + (1 << 15);
      err |= (su.v[i] < -(1 << 15) || su.v[i] >= lim) | (mu.v[i] < -(1 << 15) || mu.v[i] >= lim);
    }
    a = s; au = su;
    fe_sub(b, m, s2); fe_sub(bu, mu, s2u);
  }
  if (err) atomicAdd(bad, 1);
}

/* CH serial squaring chains per lane */
template <int NC, int CH, int W>
__global__ void __launch_bounds__(256, W) k_sq(const int32_t* in, int32_t* out, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  fe a[4];
  for (int c = 0; c < CH; c++) load_in(a[c], in, t, c);
#pragma clang loop unroll(disable)
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < CH; c++) sqs_c<NC, 1>(a[c], a[c]);
  }
  int32_t s = 0;
  for (int c = 0; c < CH; c++) for (int i = 0; i < 10; i++) s ^= a[c].v[i];
  out[t] = s;
}

template <int NC, int W>
__global__ void __launch_bounds__(256, W) k_mul(const int32_t* in, int32_t* out, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  fe a[3];
  for (int c = 0; c < 3; c++) load_in(a[c], in, t, c);
#pragma clang loop unroll(disable)
  for (int it = 0; it < iters; it++) {
    mul_c<NC>(a[0], a[0], a[1]); mul_c<NC>(a[1], a[1], a[2]); mul_c<NC>(a[2], a[2], a[0]);
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
  for (int t = 0; t < 64; t++) for (int i = 0; i < 32; i++) h[t * 32 + i] = -1;
  CHECK(hipMemcpy(in, h, sizeof(int32_t) * max_lanes * 32, hipMemcpyHostToDevice));
  void (*checks[3])(const int32_t*, int*, int) = {k_check<2>, k_check<3>, k_check<4>};
  for (int v = 0; v < 3; v++) {
    CHECK(hipMemset(bad, 0, sizeof(int)));
    hipLaunchKernelGGL(checks[v], dim3(cus * 2), dim3(block), 0, 0, in, bad, 256);
    int hbad = -1;
    CHECK(hipMemcpy(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost));
    printf("%d chains vs centered: %d of %d lanes differ (256 rounds)\n", v + 2, hbad, cus * 2 * block);
    if (hbad) return 1;
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  const int iters = 400;
  struct { const char* name; void (*f)(const int32_t*, int32_t*, int); double ops_per_iter; int wps; } ks[] = {
    {"sq  2ch x1 w2", k_sq<2, 1, 2>, 1, 2}, {"sq  2ch x1 w3", k_sq<2, 1, 3>, 1, 3}, {"sq  2ch x1 w4", k_sq<2, 1, 4>, 1, 4},
    {"sq  2ch x2 w2", k_sq<2, 2, 2>, 2, 2}, {"sq  2ch x2 w3", k_sq<2, 2, 3>, 2, 3}, {"sq  2ch x2 w4", k_sq<2, 2, 4>, 2, 4},
    {"sq  2ch x4 w2", k_sq<2, 4, 2>, 4, 2}, {"sq  2ch x4 w3", k_sq<2, 4, 3>, 4, 3}, {"sq  2ch x4 w4", k_sq<2, 4, 4>, 4, 4},
    {"sq  2ch x1 w8", k_sq<2, 1, 8>, 1, 8}, {"sq  2ch x4 w8", k_sq<2, 4, 8>, 4, 8},
    {"mul 2ch x3 w2", k_mul<2, 2>, 3, 2}, {"mul 2ch x3 w3", k_mul<2, 3>, 3, 3}, {"mul 2ch x3 w4", k_mul<2, 4>, 3, 4},
    {"mul 2ch x3 w8", k_mul<2, 8>, 3, 8},
    {"sq  3ch x1 w2", k_sq<3, 1, 2>, 1, 2}, {"sq  3ch x1 w4", k_sq<3, 1, 4>, 1, 4},
    {"mul 3ch x3 w2", k_mul<3, 2>, 3, 2}, {"mul 3ch x3 w3", k_mul<3, 3>, 3, 3},
  };
  for (auto& k : ks) {
    const int grid = cus * k.wps, lanes = grid * block;
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
    printf("%-16s %8.3f ms  %7.2f G field ops/s  %6.1f SIMD-cycles per op per wave at 2.4 GHz\n", k.name, best,
           ops / (best * 1e-3) / 1e9, best * 1e-3 * 2.4e9 * cus * 4 / (ops / 64));
  }
  return 0;
}
