// Field-multiplication microbenchmark (gfx950): the production radix-2^25.5
// fe_mul / fe_sq (firedancer_amd/csrc/fd25519_fe.h) against a radix-2^32
// prototype (8 unsigned limbs, product scanning with 96-bit column
// accumulators: v_mad_u64_u32 + v_addc_co_u32 per product, 38-fold).
// Each lane runs 3 (mul) or 4 (sq) independent chains -- the shape of the
// point formulas -- at 2 waves per SIMD, as the dsm kernel does.  The
// prototype's results are checked against the production arithmetic on the
// device (canonical bytes), so a timing is only printed for a correct path.
//
//   hipcc --offload-arch=gfx950 -O3 -I firedancer_amd/csrc -o fe_ubench tools/ubench/fe_ubench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include "fd25519_fe.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

struct fe32 { uint32_t w[8]; };

__device__ __forceinline__ void mac(uint64_t& lo, uint32_t& hi, uint32_t a, uint32_t b) {
  asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
               : "+v"(lo), "+v"(hi) : "v"(a), "v"(b) : "vcc");
}

/* r = t[0..8) + 38 t[8..16) folded to 8 words (value < 2^256, = t mod p) */
__device__ __forceinline__ void fe32_reduce(fe32& r, const uint32_t (&t)[16]) {
  uint64_t acc[8];
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = (uint64_t)t[8 + i] * 38u + t[i];   /* < 39 * 2^32 */
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    c += acc[i];
    r.w[i] = (uint32_t)c;
    c >>= 32;
  }
  /* c <= 39: add 38 c, once more if that wraps past 2^256 */
  uint64_t s = (uint64_t)r.w[0] + c * 38u;
  r.w[0] = (uint32_t)s;
  s >>= 32;
#pragma unroll
  for (int i = 1; i < 8; i++) {
    s += r.w[i];
    r.w[i] = (uint32_t)s;
    s >>= 32;
  }
  r.w[0] += (uint32_t)s * 38u;   /* s in {0,1}; then w0 < 38*39 + 38, no carry */
}

__device__ __forceinline__ void fe32_mul(fe32& r, const fe32& a, const fe32& b) {
  uint32_t t[16];
  uint64_t lo = 0;
  uint32_t hi = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j >= 0 && j < 8) mac(lo, hi, a.w[i], b.w[j]);
    }
    t[k] = (uint32_t)lo;
    lo = (lo >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  t[15] = (uint32_t)lo;
  fe32_reduce(r, t);
}

__device__ __forceinline__ void fe32_sq(fe32& r, const fe32& a) {
  uint32_t t[16];
  uint64_t lo = 0;
  uint32_t hi = 0;
  /* cross products i < j */
  t[0] = 0;
#pragma unroll
  for (int k = 1; k < 14; k++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (i < j && j < 8) mac(lo, hi, a.w[i], a.w[j]);
    }
    t[k] = (uint32_t)lo;
    lo = (lo >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  t[14] = (uint32_t)lo;
  t[15] = (uint32_t)(lo >> 32);
  /* double, add the diagonal */
  uint32_t u[16];
  u[0] = 0;
#pragma unroll
  for (int k = 1; k < 16; k++) u[k] = __builtin_amdgcn_alignbit(t[k], t[k - 1], 31);
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t d = (uint64_t)a.w[i] * a.w[i];
    c += (uint64_t)u[2 * i] + (uint32_t)d;
    u[2 * i] = (uint32_t)c;
    c >>= 32;
    c += (uint64_t)u[2 * i + 1] + (uint32_t)(d >> 32);
    u[2 * i + 1] = (uint32_t)c;
    c >>= 32;
  }
  fe32_reduce(r, u);
}

__device__ void fe32_from_fe(fe32& r, const fe& f) {
  uint32_t s[8];
  fe_tobytes(s, f);
  for (int i = 0; i < 8; i++) r.w[i] = s[i];
}

/* canonical bytes of a fe32 through the production arithmetic */
__device__ void fe32_canon(uint32_t (&s)[8], const fe32& a) {
  /* a = lo255 + 2^255 * top: value mod p = lo255 + 19 top */
  uint32_t w[8];
  for (int i = 0; i < 8; i++) w[i] = a.w[i];
  const uint32_t top = w[7] >> 31;
  w[7] &= 0x7fffffffu;
  fe f, g;
  fe_frombytes(f, w);
  fe_0(g);
  g.v[0] = 19 * (int32_t)top;
  fe_add(f, f, g);
  fe_tobytes(s, f);
}

__global__ void __launch_bounds__(256, 2) k_check(const uint32_t* in, int* bad, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t wa[8], wb[8];
  for (int i = 0; i < 8; i++) { wa[i] = in[t * 16 + i]; wb[i] = in[t * 16 + 8 + i]; }
  if (t & 1) for (int i = 0; i < 8; i++) wa[i] = 0xffffffffu - (uint32_t)(t >> 1) * i;  /* near 2^256 */
  wa[7] &= 0x7fffffffu; wb[7] &= 0x7fffffffu;
  fe fa, fb;
  fe_frombytes(fa, wa); fe_frombytes(fb, wb);
  fe32 xa, xb;
  for (int i = 0; i < 8; i++) { xa.w[i] = in[t * 16 + i]; xb.w[i] = wb[i]; }
  if (t & 1) for (int i = 0; i < 8; i++) xa.w[i] = 0xffffffffu - (uint32_t)(t >> 1) * i;
  /* the fe32 operand xa is the full 256-bit value; fa is its low 255 bits: add 19 * bit255 */
  { fe g; fe_0(g); g.v[0] = 19 * (int32_t)(xa.w[7] >> 31); fe_add(fa, fa, g); fe_carry(fa, fa); }
  int err = 0;
  for (int it = 0; it < iters; it++) {
    fe fm, fs;
    fe32 ym, ys;
    fe_mul(fm, fa, fb); fe32_mul(ym, xa, xb);
    fe_sq(fs, fa);      fe32_sq(ys, xa);
    uint32_t s1[8], s2[8], s3[8], s4[8];
    fe_tobytes(s1, fm); fe32_canon(s2, ym);
    fe_tobytes(s3, fs); fe32_canon(s4, ys);
    for (int i = 0; i < 8; i++) err |= (s1[i] != s2[i]) | (s3[i] != s4[i]);
    fa = fm; fb = fs; xa = ym; xb = ys;
  }
  if (err) atomicAdd(bad, 1);
}

template <int SQ>
__global__ void __launch_bounds__(256, 2) k_fe(const int32_t* in, int32_t* out, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  fe a[4];
  for (int c = 0; c < 4; c++) for (int i = 0; i < 10; i++) a[c].v[i] = in[(t * 4 + c) * 10 + i] & 0xffffff;
  for (int it = 0; it < iters; it++) {
    if (SQ) { fe_sq(a[0], a[0]); fe_sq(a[1], a[1]); fe_sq(a[2], a[2]); fe_sq(a[3], a[3]); }
    else    { fe_mul(a[0], a[0], a[1]); fe_mul(a[1], a[1], a[2]); fe_mul(a[2], a[2], a[0]); }
  }
  int32_t s = 0;
  for (int c = 0; c < 4; c++) for (int i = 0; i < 10; i++) s ^= a[c].v[i];
  out[t] = s;
}

template <int SQ>
__global__ void __launch_bounds__(256, 2) k_fe32(const int32_t* in, int32_t* out, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  fe32 a[4];
  for (int c = 0; c < 4; c++) for (int i = 0; i < 8; i++) a[c].w[i] = (uint32_t)in[(t * 4 + c) * 10 + i];
  for (int it = 0; it < iters; it++) {
    if (SQ) { fe32_sq(a[0], a[0]); fe32_sq(a[1], a[1]); fe32_sq(a[2], a[2]); fe32_sq(a[3], a[3]); }
    else    { fe32_mul(a[0], a[0], a[1]); fe32_mul(a[1], a[1], a[2]); fe32_mul(a[2], a[2], a[0]); }
  }
  uint32_t s = 0;
  for (int c = 0; c < 4; c++) for (int i = 0; i < 8; i++) s ^= a[c].w[i];
  out[t] = (int32_t)s;
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int block = 256, grid = cus * 2 * 4;   /* 2 blocks/CU x 4 rounds */
  const int lanes = grid * block;
  int32_t *in, *out;
  int* bad;
  CHECK(hipMalloc(&in, sizeof(int32_t) * lanes * 40));
  CHECK(hipMalloc(&out, sizeof(int32_t) * lanes));
  CHECK(hipMalloc(&bad, sizeof(int)));
  int32_t* h = (int32_t*)malloc(sizeof(int32_t) * lanes * 40);
  uint64_t x = 88172645463325252ull;
  for (long i = 0; i < (long)lanes * 40; i++) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; h[i] = (int32_t)x; }
  CHECK(hipMemcpy(in, h, sizeof(int32_t) * lanes * 40, hipMemcpyHostToDevice));
  CHECK(hipMemset(bad, 0, sizeof(int)));
  hipLaunchKernelGGL(k_check, dim3(cus * 2), dim3(block), 0, 0, (const uint32_t*)in, bad, 64);
  int hbad = -1;
  CHECK(hipMemcpy(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost));
  printf("radix-2^32 prototype vs production arithmetic: %d of %d lanes differ\n", hbad, cus * 2 * block);
  if (hbad) return 1;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  const int iters = 200;
  struct { const char* name; void (*f)(const int32_t*, int32_t*, int); double ops_per_iter; } ks[] = {
    {"fe_mul   (2^25.5)", k_fe<0>, 3}, {"fe32_mul (2^32)  ", k_fe32<0>, 3},
    {"fe_sq    (2^25.5)", k_fe<1>, 4}, {"fe32_sq  (2^32)  ", k_fe32<1>, 4},
  };
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.f, dim3(grid), dim3(block), 0, 0, in, out, iters);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 3; r++) {
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(k.f, dim3(grid), dim3(block), 0, 0, in, out, iters);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    const double ops = (double)lanes * iters * k.ops_per_iter;
    printf("%s %8.3f ms  %7.2f G field ops/s  %6.1f SIMD-cycles per op per wave at 2.4 GHz\n", k.name, best,
           ops / (best * 1e-3) / 1e9, best * 1e-3 * 2.4e9 * cus * 4 / (ops / 64));
  }
  return 0;
}
