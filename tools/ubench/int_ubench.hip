// Instruction-throughput microbenchmark for the big-integer primitives the
// ed25519 field arithmetic can be built from (gfx950).  Each lane runs
// NCHAIN independent dependency chains of one instruction inside a loop so the
// measurement is issue-throughput bound, not latency bound.
//
//   hipcc --offload-arch=gfx950 -O3 -o int_ubench int_ubench.hip
//
// Output: one line per instruction: wave-instructions per cycle per CU and
// lane-ops/s for the whole chip (sclk taken from hipDeviceProp clockRate).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int NCHAIN = 8;
constexpr int ITERS = 4096;

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

// v_mad_u64_u32: 32x32 -> 64 + 64
__global__ void k_mad_u64_u32(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x + seed, b = blockIdx.x * 7 + seed;
  uint64_t acc[NCHAIN];
#pragma unroll
  for (int i = 0; i < NCHAIN; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#define X(i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b) : "vcc");
    REP8(X)
#undef X
  }
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < NCHAIN; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mul_lo_u32(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x + seed;
  uint32_t acc[NCHAIN];
#pragma unroll
  for (int i = 0; i < NCHAIN; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#define X(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc[i]) : "v"(a));
    REP8(X)
#undef X
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < NCHAIN; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mul_hi_u32(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x + seed;
  uint32_t acc[NCHAIN];
#pragma unroll
  for (int i = 0; i < NCHAIN; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#define X(i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc[i]) : "v"(a));
    REP8(X)
#undef X
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < NCHAIN; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mad_u32_u24(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x + seed, b = blockIdx.x + seed;
  uint32_t acc[NCHAIN];
#pragma unroll
  for (int i = 0; i < NCHAIN; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#define X(i) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b));
    REP8(X)
#undef X
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < NCHAIN; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mul_hi_u32_u24(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x + seed;
  uint32_t acc[NCHAIN];
#pragma unroll
  for (int i = 0; i < NCHAIN; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#define X(i) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(acc[i]) : "v"(a));
    REP8(X)
#undef X
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < NCHAIN; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_add_u32(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x + seed;
  uint32_t acc[NCHAIN];
#pragma unroll
  for (int i = 0; i < NCHAIN; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#define X(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc[i]) : "v"(a));
    REP8(X)
#undef X
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < NCHAIN; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_add3_u32(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x + seed, b = seed * 3;
  uint32_t acc[NCHAIN];
#pragma unroll
  for (int i = 0; i < NCHAIN; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#define X(i) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(acc[i]) : "v"(a), "v"(b));
    REP8(X)
#undef X
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < NCHAIN; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// 64-bit add as the pair v_add_co_u32 / v_addc_co_u32 (2 VALU per 64-bit add)
__global__ void k_add_u64(uint64_t* out, uint32_t seed) {
  uint64_t a = threadIdx.x + seed;
  uint64_t acc[NCHAIN];
#pragma unroll
  for (int i = 0; i < NCHAIN; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#define X(i) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[i]) : "v"(a));
    REP8(X)
#undef X
  }
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < NCHAIN; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_fma_f64(uint64_t* out, uint32_t seed) {
  double a = threadIdx.x * 1e-3 + seed, b = 0.999;
  double acc[NCHAIN];
#pragma unroll
  for (int i = 0; i < NCHAIN; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#define X(i) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(acc[i]) : "v"(b), "v"(a));
    REP8(X)
#undef X
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < NCHAIN; i++) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

__global__ void k_fma_f32(uint64_t* out, uint32_t seed) {
  float a = threadIdx.x * 1e-3f + seed, b = 0.999f;
  float acc[NCHAIN];
#pragma unroll
  for (int i = 0; i < NCHAIN; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#define X(i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(acc[i]) : "v"(b), "v"(a));
    REP8(X)
#undef X
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < NCHAIN; i++) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

// mixed: one v_mad_u64_u32 followed by 2 plain adds -- shows whether VALU
// ops co-issue behind a multi-cycle multiply.
__global__ void k_mix_mad_add(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x + seed, b = blockIdx.x * 7 + seed;
  uint64_t acc[NCHAIN];
  uint32_t t[NCHAIN];
#pragma unroll
  for (int i = 0; i < NCHAIN; i++) { acc[i] = a + i; t[i] = b + i; }
  for (int it = 0; it < ITERS; it++) {
#define X(i) asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_add_u32 %1, %1, %2\n\tv_add_u32 %1, %1, %3" : "+v"(acc[i]), "+v"(t[i]) : "v"(a), "v"(b) : "vcc");
    REP8(X)
#undef X
  }
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < NCHAIN; i++) s ^= acc[i] ^ t[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}


// 32-bit ops used by SHA-512, the DPP exchanges and the carry chains
#define UB_K32(NAME, ASM)                                                        \
__global__ void NAME(uint64_t* out, uint32_t seed) {                               \
  uint32_t a = threadIdx.x + seed, b = seed * 3;                                   \
  uint32_t acc[NCHAIN];                                                            \
  _Pragma("unroll") for (int i = 0; i < NCHAIN; i++) acc[i] = a + i;                \
  for (int it = 0; it < ITERS; it++) {                                             \
    _Pragma("unroll") for (int i = 0; i < NCHAIN; i++)                             \
      asm volatile(ASM : "+v"(acc[i]) : "v"(a), "v"(b));                           \
  }                                                                                \
  uint32_t s = 0;                                                                  \
  _Pragma("unroll") for (int i = 0; i < NCHAIN; i++) s ^= acc[i];                  \
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                  \
}
UB_K32(k_alignbit, "v_alignbit_b32 %0, %0, %1, %2")
UB_K32(k_bitop3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")
UB_K32(k_xor, "v_xor_b32 %0, %0, %1")
UB_K32(k_lshl_add_u32, "v_lshl_add_u32 %0, %0, 3, %1")
UB_K32(k_dpp_qp, "v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
UB_K32(k_cndmask, "v_cndmask_b32_e64 %0, %0, %1, s[0:1]")

// 64-bit arithmetic shift (the carry extraction)
__global__ void k_ashr_i64(uint64_t* out, uint32_t seed) {
  int64_t a = threadIdx.x + seed;
  int64_t acc[NCHAIN];
#pragma unroll
  for (int i = 0; i < NCHAIN; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < NCHAIN; i++) asm volatile("v_ashrrev_i64 %0, 1, %0" : "+v"(acc[i]));
  }
  int64_t s = 0;
#pragma unroll
  for (int i = 0; i < NCHAIN; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

typedef void (*kfn)(uint64_t*, uint32_t);

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const double sclk = prop.clockRate * 1e3;  // Hz
  const int cus = prop.multiProcessorCount;
  printf("device %s  CUs %d  clockRate %.0f MHz\n", prop.gcnArchName, cus, sclk / 1e6);
  const int block = 256;
  const int grid = cus * 8;  // 8 blocks of 4 waves per CU: 8 waves/SIMD
  uint64_t* out;
  CHECK(hipMalloc(&out, sizeof(uint64_t) * grid * block));
  struct { const char* name; kfn f; int instr_per_chain_iter; } ks[] = {
      {"v_mad_u64_u32", k_mad_u64_u32, 1},
      {"v_mul_lo_u32", k_mul_lo_u32, 1},
      {"v_mul_hi_u32", k_mul_hi_u32, 1},
      {"v_mad_u32_u24", k_mad_u32_u24, 1},
      {"v_mul_hi_u32_u24", k_mul_hi_u32_u24, 1},
      {"v_add_u32", k_add_u32, 1},
      {"v_add3_u32", k_add3_u32, 1},
      {"v_lshl_add_u64", k_add_u64, 1},
      {"v_fma_f64", k_fma_f64, 1},
      {"v_fma_f32", k_fma_f32, 1},
      {"mad_u64+2add", k_mix_mad_add, 3},
      {"v_alignbit_b32", k_alignbit, 1},
      {"v_bitop3_b32", k_bitop3, 1},
      {"v_xor_b32", k_xor, 1},
      {"v_lshl_add_u32", k_lshl_add_u32, 1},
      {"v_mov_b32_dpp", k_dpp_qp, 1},
      {"v_cndmask_b32", k_cndmask, 1},
      {"v_ashrrev_i64", k_ashr_i64, 1},
  };
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.f, dim3(grid), dim3(block), 0, 0, out, 1u);  // warmup
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(k.f, dim3(grid), dim3(block), 0, 0, out, (uint32_t)r);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    double waves = (double)grid * block / 64;
    double wave_instr = waves * ITERS * NCHAIN * k.instr_per_chain_iter;
    double cycles = best * 1e-3 * sclk;
    double per_cu_cyc = wave_instr / cus / cycles;
    double lane_ops = wave_instr * 64 / (best * 1e-3);
    printf("%-18s %8.3f ms  wave-instr/cyc/CU %.3f  (cyc per wave-instr per SIMD %.2f)  chip %.2f Tops/s\n",
           k.name, best, per_cu_cyc, 4.0 / per_cu_cyc, lane_ops / 1e12);
  }
  CHECK(hipFree(out));
  return 0;
}
