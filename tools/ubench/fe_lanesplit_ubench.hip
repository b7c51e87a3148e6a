// Lane-split field arithmetic microbenchmark (gfx950), VERDICT r4 next #2:
// is one GF(2^255-19) squaring / product faster when its columns are spread
// over the lanes of a row than when one lane runs it alone (the latency
// form's chains: decode's 250 dependent squarings, the quad kernels'
// doublings)?
//
//   serial  the production unsigned-limb radix-2^25.5 fe_sq_u / fe_mul_u
//           (firedancer_amd/csrc/fd25519_fe.h), one element per lane;
//   r16     one element per 16-lane DPP row, radix 2^16: lane c holds limb
//           c (loose, < 2^16.02) and computes column c of the product,
//             col_c = sum_t g_t * f_{c-t mod 16} * (c < t ? 38 : 1)
//           (2^256 = 38 mod p).  Per t one row broadcast of g_t
//           (v_mov_b32_dpp row_newbcast:t), one rotation of f times the
//           lane's wrap factor (v_mul_u32_u24 with row_ror:t folded in:
//           the factor is a per-lane constant) and one v_mad_u64_u32; then
//           three carry rounds, each moving the carries one lane up
//           (row_ror:1, lane 0 taking 38 x lane 15's).
//
// Each chain is dependent (x <- x^2, or x <- x*y), one wave per CU for the
// latency figure and a full chip for the throughput one.  The r16 results
// are reduced to canonical bytes and compared with the serial chain's on
// the device: a timing is only printed for a correct path.
//
//   hipcc --offload-arch=gfx950 -O3 -I firedancer_amd/csrc -o fe_lanesplit_ubench tools/ubench/fe_lanesplit_ubench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include "fd25519_fe.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

#define BC(x, t)  ((uint32_t)__builtin_amdgcn_mov_dpp((int)(x), 0x150 + (t), 0xf, 0xf, true))   /* row_newbcast:t */
#define ROR(x, t) ((uint32_t)__builtin_amdgcn_mov_dpp((int)(x), 0x120 + (t), 0xf, 0xf, true))   /* row_ror:t      */

/* three carry rounds: limbs back below 2^16 + 2^10 */
__device__ __forceinline__ uint32_t r16_carry(uint64_t acc, uint32_t m1) {
  uint32_t lo = (uint32_t)acc & 0xffffu;
  uint32_t hi = (uint32_t)(acc >> 16);           /* < 2^25.2 */
  uint32_t l = lo + ROR(hi, 1) * m1;             /* < 2^30.8 */
  hi = l >> 16; lo = l & 0xffffu;
  l = lo + __umul24(ROR(hi, 1), m1);             /* < 2^20.1 */
  hi = l >> 16; lo = l & 0xffffu;
  return lo + __umul24(ROR(hi, 1), m1);          /* < 2^16 + 38*17 */
}

#define STEP(a, t) a += (uint64_t)BC(g, t) * __umul24(ROR(f, t), m[t]);

/* h = f*g, one element per 16-lane row; ACC column accumulators (1: one
   dependent multiply-add chain, 2: even and odd t in two chains) */
template <int ACC>
__device__ __forceinline__ uint32_t r16_mul(uint32_t f, uint32_t g, const uint32_t (&m)[16]) {
  if (ACC == 1) {
    uint64_t acc = (uint64_t)BC(g, 0) * f;
    STEP(acc, 1) STEP(acc, 2) STEP(acc, 3) STEP(acc, 4) STEP(acc, 5) STEP(acc, 6) STEP(acc, 7) STEP(acc, 8)
    STEP(acc, 9) STEP(acc, 10) STEP(acc, 11) STEP(acc, 12) STEP(acc, 13) STEP(acc, 14) STEP(acc, 15)
    return r16_carry(acc, m[1]);
  } else {
    uint64_t acc = (uint64_t)BC(g, 0) * f, acc2 = (uint64_t)BC(g, 1) * __umul24(ROR(f, 1), m[1]);
    STEP(acc, 2) STEP(acc2, 3) STEP(acc, 4) STEP(acc2, 5) STEP(acc, 6) STEP(acc2, 7) STEP(acc, 8)
    STEP(acc2, 9) STEP(acc, 10) STEP(acc2, 11) STEP(acc, 12) STEP(acc2, 13) STEP(acc, 14) STEP(acc2, 15)
    return r16_carry(acc + acc2, m[1]);
  }
}

__device__ __forceinline__ void r16_consts(uint32_t (&m)[16]) {
  const uint32_t c = threadIdx.x & 15u;
#pragma unroll
  for (int t = 0; t < 16; t++) m[t] = c < (uint32_t)t ? 38u : 1u;
}

template <int ACC>
__global__ void __launch_bounds__(64) k_r16(const uint32_t* in, const uint32_t* yin, uint32_t* out, int n, int mul) {
  const uint32_t tid = blockIdx.x * 64u + threadIdx.x;
  uint32_t m[16];
  r16_consts(m);
  uint32_t f = in[tid];
  const uint32_t y = yin[tid];
  if (mul) {
#pragma clang loop unroll(disable)
    for (int i = 0; i < n; i++) f = r16_mul<ACC>(f, y, m);
  } else {
#pragma clang loop unroll(disable)
    for (int i = 0; i < n; i++) f = r16_mul<ACC>(f, f, m);
  }
  out[tid] = f;
}

/* the same chains in the production one-lane form; in/out as 8 words */
__global__ void __launch_bounds__(64) k_serial(const uint32_t* in, const uint32_t* yin, uint32_t* out, int n, int mul) {
  const uint32_t tid = blockIdx.x * 64u + threadIdx.x;
  uint32_t w[8], v[8];
#pragma unroll
  for (int k = 0; k < 8; k++) { w[k] = in[8 * tid + k]; v[k] = yin[8 * tid + k]; }
  fe x, y;
  fe_frombytes(x, w);
  fe_frombytes(y, v);
  if (mul) {
    fe y19;
    fe_19(y19, y);
#pragma clang loop unroll(disable)
    for (int i = 0; i < n; i++) fe_mul19_u(x, x, y, y19);
  } else {
#pragma clang loop unroll(disable)
    for (int i = 0; i < n; i++) fe_sq_u(x, x);
  }
  uint32_t s[8];
  fe_tobytes(s, x);
#pragma unroll
  for (int k = 0; k < 8; k++) out[8 * tid + k] = s[k];
}

/* a row's 16 loose limbs -> canonical bytes (one thread per row) */
__global__ void k_r16_canon(const uint32_t* limbs, uint32_t* out, int rows) {
  const int r = blockIdx.x * 64 + threadIdx.x;
  if (r >= rows) return;
  uint32_t d[16];
  uint64_t acc = 0;
  for (int c = 0; c < 16; c++) { acc += limbs[16 * r + c]; d[c] = (uint32_t)acc & 0xffffu; acc >>= 16; }
  for (int pass = 0; pass < 2; pass++) {   /* fold 2^256 (x 38) and bit 255 (x 19) into the low limbs */
    uint64_t top = acc * 38u + 19u * (d[15] >> 15);
    d[15] &= 0x7fffu;
    acc = top;
    for (int c = 0; c < 16; c++) { acc += d[c]; d[c] = (uint32_t)acc & 0xffffu; acc >>= 16; }
  }
  uint32_t w[8];
  for (int k = 0; k < 8; k++) w[k] = d[2 * k] | (d[2 * k + 1] << 16);
  fe x;
  fe_frombytes(x, w);
  uint32_t s[8];
  fe_tobytes(s, x);
  for (int k = 0; k < 8; k++) out[8 * r + k] = s[k];
}

static float time_kernel(void (*launch)(void*), void* ctx, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  launch(ctx);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < reps; i++) launch(ctx);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return ms / reps;
}

struct Launch { int r16, waves, n, mul; uint32_t *in, *yin, *out; };

static void do_launch(void* p) {
  Launch* l = (Launch*)p;
  if (l->r16 == 1) hipLaunchKernelGGL(k_r16<1>, dim3(l->waves), dim3(64), 0, 0, l->in, l->yin, l->out, l->n, l->mul);
  else if (l->r16 == 2) hipLaunchKernelGGL(k_r16<2>, dim3(l->waves), dim3(64), 0, 0, l->in, l->yin, l->out, l->n, l->mul);
  else hipLaunchKernelGGL(k_serial, dim3(l->waves), dim3(64), 0, 0, l->in, l->yin, l->out, l->n, l->mul);
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4000;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const double clk = prop.clockRate * 1e3;   /* Hz */
  const int cus = prop.multiProcessorCount;
  printf("{\"device\": \"%s\", \"cus\": %d, \"clock_mhz\": %.0f, \"chain\": %d}\n", prop.gcnArchName, cus, clk / 1e6, n);

  /* check: R rows of r16 against the same R values through the serial chain */
  const int R = 1024, chk_n = 257;
  std::vector<uint32_t> val(8 * R), yv(8 * R), limbs(16 * R), ylimbs(16 * R);
  srand(7);
  for (int i = 0; i < 8 * R; i++) { val[i] = ((uint32_t)rand() << 16) ^ (uint32_t)rand(); yv[i] = ((uint32_t)rand() << 16) ^ (uint32_t)rand(); }
  for (int r = 0; r < R; r++) {
    if (r == 0) for (int k = 0; k < 8; k++) val[8 * r + k] = 0xffffffffu;   /* 2^255 - 1: the widest limbs */
    val[8 * r + 7] &= 0x7fffffffu;
    yv[8 * r + 7] &= 0x7fffffffu;
    for (int c = 0; c < 16; c++) {
      limbs[16 * r + c] = (val[8 * r + c / 2] >> (16 * (c & 1))) & 0xffffu;
      ylimbs[16 * r + c] = (yv[8 * r + c / 2] >> (16 * (c & 1))) & 0xffffu;
    }
  }
  uint32_t *d_val, *d_yv, *d_limbs, *d_ylimbs, *d_out8, *d_outl, *d_canon;
  CHECK(hipMalloc(&d_val, 4 * val.size())); CHECK(hipMalloc(&d_yv, 4 * yv.size()));
  CHECK(hipMalloc(&d_limbs, 4 * limbs.size())); CHECK(hipMalloc(&d_ylimbs, 4 * ylimbs.size()));
  CHECK(hipMalloc(&d_out8, 4 * val.size())); CHECK(hipMalloc(&d_outl, 4 * limbs.size()));
  CHECK(hipMalloc(&d_canon, 4 * val.size()));
  CHECK(hipMemcpy(d_val, val.data(), 4 * val.size(), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_yv, yv.data(), 4 * yv.size(), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_limbs, limbs.data(), 4 * limbs.size(), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_ylimbs, ylimbs.data(), 4 * ylimbs.size(), hipMemcpyHostToDevice));
  int ok[2] = {0, 0};
  for (int mul = 0; mul < 2; mul++) {
    hipLaunchKernelGGL(k_serial, dim3(R / 64), dim3(64), 0, 0, d_val, d_yv, d_out8, chk_n, mul);
    for (int acc = 1; acc <= 2; acc++) {
      if (acc == 1) hipLaunchKernelGGL(k_r16<1>, dim3(R * 16 / 64), dim3(64), 0, 0, d_limbs, d_ylimbs, d_outl, chk_n, mul);
      else hipLaunchKernelGGL(k_r16<2>, dim3(R * 16 / 64), dim3(64), 0, 0, d_limbs, d_ylimbs, d_outl, chk_n, mul);
      hipLaunchKernelGGL(k_r16_canon, dim3(R / 64), dim3(64), 0, 0, d_outl, d_canon, R);
      CHECK(hipDeviceSynchronize());
      std::vector<uint32_t> a(8 * R), b(8 * R);
      CHECK(hipMemcpy(a.data(), d_out8, 4 * a.size(), hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(b.data(), d_canon, 4 * b.size(), hipMemcpyDeviceToHost));
      int bad = 0;
      for (int i = 0; i < 8 * R; i++) bad += a[i] != b[i];
      ok[mul] += bad == 0;
      printf("{\"check\": \"%s\", \"accumulators\": %d, \"elements\": %d, \"chain\": %d, \"words_differing\": %d}\n",
             mul ? "mul" : "sq", acc, R, chk_n, bad);
    }
  }
  if (ok[0] != 2 || ok[1] != 2) { printf("{\"error\": \"r16 differs from the production arithmetic: no timings\"}\n"); return 1; }

  /* timings: one wave per CU (latency: each wave's SIMD to itself), and the
     whole chip at 8 waves per CU (throughput) */
  const int big = cus * 8;
  uint32_t *t_in, *t_y, *t_out;
  CHECK(hipMalloc(&t_in, 4UL * 8 * 64 * big)); CHECK(hipMalloc(&t_y, 4UL * 8 * 64 * big));
  CHECK(hipMalloc(&t_out, 4UL * 8 * 64 * big));
  CHECK(hipMemset(t_in, 0x11, 4UL * 8 * 64 * big)); CHECK(hipMemset(t_y, 0x07, 4UL * 8 * 64 * big));
  for (int mul = 0; mul < 2; mul++) {
    for (int waves : {cus, big}) {
      Launch ls = {0, waves, n, mul, t_in, t_y, t_out}, lr = {1, waves, n, mul, t_in, t_y, t_out},
             lr2 = {2, waves, n, mul, t_in, t_y, t_out};
      float ms_s = time_kernel(do_launch, &ls, 3), ms_r = time_kernel(do_launch, &lr, 3);
      float ms_r2 = time_kernel(do_launch, &lr2, 3);
      const double cyc_s = ms_s * 1e-3 * clk / n, cyc_r = ms_r * 1e-3 * clk / n, cyc_r2 = ms_r2 * 1e-3 * clk / n;
      const double el_s = 64.0 * waves, el_r = 4.0 * waves;   /* elements per launch */
      printf("{\"op\": \"%s\", \"waves\": %d, \"waves_per_cu\": %d, \"serial_cycles_per_op\": %.1f, "
             "\"r16_cycles_per_op\": %.1f, \"r16_2acc_cycles_per_op\": %.1f, \"latency_ratio_serial_over_best_r16\": %.3f, "
             "\"serial_elem_ops_per_s\": %.4g, \"r16_elem_ops_per_s\": %.4g}\n",
             mul ? "mul" : "sq", waves, waves / cus, cyc_s, cyc_r, cyc_r2, cyc_s / (cyc_r < cyc_r2 ? cyc_r : cyc_r2),
             el_s * n / (ms_s * 1e-3), el_r * n / ((ms_r < ms_r2 ? ms_r : ms_r2) * 1e-3));
    }
  }
  return 0;
}
