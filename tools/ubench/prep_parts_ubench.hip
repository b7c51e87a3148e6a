// Where the latency form's hash -> scalar chain spends its time (gfx950):
// one wave (LANES active lanes, one signature each) runs the prep16 wave-0
// pieces in sequence -- SHA-512(R||A||M) of a 200-byte message, the
// reduction mod L, the half-size scalar search (Lehmer), the integer pair
// check, s' = d S mod L -- with s_memtime stamps between them.  The
// production device code is compiled in (fd_ed25519_kernels.hip), so the
// pieces are the kernels' own.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I firedancer_amd/csrc -o tools/ubench/prep_parts_ubench tools/ubench/prep_parts_ubench.hip
#include "../../firedancer_amd/csrc/fd_ed25519_kernels.hip"
#include "half_timed.inc"
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

__global__ void __launch_bounds__(64) k_parts(const uint8_t* sigs, const uint8_t* pubs, const uint8_t* msgs, int msz,
                                              int lanes, uint64_t* stamps, uint32_t* sink, uint64_t* htm) {
  const int j = threadIdx.x;
  if (j >= lanes) return;
  uint64_t t[6];
  t[0] = __builtin_amdgcn_s_memtime();
  uint32_t r[8], S[8], a[8];
  {
    const uint4* sg = reinterpret_cast<const uint4*>(sigs + 64 * j);
    const uint4* pk = reinterpret_cast<const uint4*>(pubs + 32 * j);
    const uint4 q0 = sg[0], q1 = sg[1], q2 = sg[2], q3 = sg[3], q4 = pk[0], q5 = pk[1];
    r[0] = q0.x; r[1] = q0.y; r[2] = q0.z; r[3] = q0.w; r[4] = q1.x; r[5] = q1.y; r[6] = q1.z; r[7] = q1.w;
    S[0] = q2.x; S[1] = q2.y; S[2] = q2.z; S[3] = q2.w; S[4] = q3.x; S[5] = q3.y; S[6] = q3.z; S[7] = q3.w;
    a[0] = q4.x; a[1] = q4.y; a[2] = q4.z; a[3] = q4.w; a[4] = q5.x; a[5] = q5.y; a[6] = q5.z; a[7] = q5.w;
  }
  uint32_t dig[16], k[8];
  sha_msg_src m;
  m.base = reinterpret_cast<const uint32_t*>(msgs + (size_t)msz * j);
  m.shift = 0;
  m.sz = (uint32_t)msz;
  sha512_ram(dig, r, a, m);
  asm volatile("" :: "v"(dig[0]), "v"(dig[15]));
  t[1] = __builtin_amdgcn_s_memtime();
  sc_reduce512(k, dig);
  asm volatile("" :: "v"(k[0]), "v"(k[7]));
  t[2] = __builtin_amdgcn_s_memtime();
  uint32_t cw[FD_HALF_TW], dm[FD_HALF_TW];
  int dneg = 0;
  uint64_t hq[6];
  const int found = half_scalars_timed(hq, k, cw, dm, &dneg, FD_HALF_DBITS_MAX);
  asm volatile("" :: "v"(cw[0]), "v"(dm[0]));
  t[3] = __builtin_amdgcn_s_memtime();
  const bool ok = found && half_pair_ok(k, cw, dm, dneg, FD_HALF_DBITS_MAX);
  asm volatile("" :: "v"((uint32_t)ok));
  t[4] = __builtin_amdgcn_s_memtime();
  uint32_t prod[16], sp[8];
#pragma unroll
  for (int w = 0; w < 16; w++) prod[w] = 0u;
#pragma unroll
  for (int x = 0; x < FD_HALF_TW; x++) {
    uint64_t carry = 0;
#pragma unroll
    for (int y = 0; y < 8; y++) {
      const uint64_t v = (uint64_t)dm[x] * S[y] + prod[x + y] + carry;
      prod[x + y] = (uint32_t)v;
      carry = v >> 32;
    }
    prod[x + 8] = (uint32_t)carry;
  }
  sc_reduce512(sp, prod);
  t[5] = __builtin_amdgcn_s_memtime();
  uint32_t acc = ok ? 1u : 0u;
#pragma unroll
  for (int w = 0; w < 8; w++) acc ^= sp[w] ^ k[w];
  sink[j] = acc;
  if (j == 0)
    for (int q = 0; q < 6; q++) stamps[q] = t[q];
  for (int q = 0; q < 6; q++) htm[6 * j + q] = hq[q];
}

int main(int argc, char** argv) {
  const int msz = 200;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  std::vector<uint8_t> h_sig(64 * 64), h_pub(32 * 64), h_msg((size_t)msz * 64);
  srand(7);
  for (auto& b : h_sig) b = (uint8_t)rand();
  for (auto& b : h_pub) b = (uint8_t)rand();
  for (auto& b : h_msg) b = (uint8_t)rand();
  for (int j = 0; j < 64; j++) h_sig[64 * j + 63] &= 0x0f;   /* S < 2^252 */
  uint8_t *d_sig, *d_pub, *d_msg;
  uint64_t* d_st;
  uint32_t* d_sink;
  uint64_t* d_htm;
  CHECK(hipMalloc(&d_htm, 64 * 6 * sizeof(uint64_t)));
  CHECK(hipMalloc(&d_sig, h_sig.size()));
  CHECK(hipMalloc(&d_pub, h_pub.size()));
  CHECK(hipMalloc(&d_msg, h_msg.size() + 64));
  CHECK(hipMalloc(&d_st, 6 * sizeof(uint64_t)));
  CHECK(hipMalloc(&d_sink, 64 * sizeof(uint32_t)));
  CHECK(hipMemcpy(d_sig, h_sig.data(), h_sig.size(), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_pub, h_pub.data(), h_pub.size(), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_msg, h_msg.data(), h_msg.size(), hipMemcpyHostToDevice));
  printf("{\"device\": \"%s\", \"clock_mhz\": %d, \"msg_sz\": %d}\n", prop.gcnArchName, prop.clockRate / 1000, msz);
  const char* nm[5] = {"sha512", "reduce_k", "half_scalars", "pair_check", "dS_mod_L"};
  for (int lanes : {1, 64}) {
    for (int rep = 0; rep < 6; rep++) {
      hipEvent_t a, b;
      CHECK(hipEventCreate(&a));
      CHECK(hipEventCreate(&b));
      CHECK(hipEventRecord(a));
      hipLaunchKernelGGL(k_parts, dim3(1), dim3(64), 0, 0, d_sig, d_pub, d_msg, msz, lanes, d_st, d_sink, d_htm);
      CHECK(hipEventRecord(b));
      CHECK(hipEventSynchronize(b));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, a, b));
      uint64_t st[6];
      CHECK(hipMemcpy(st, d_st, sizeof(st), hipMemcpyDeviceToHost));
      if (rep < 2) continue;   /* warm-up: code fetch, clocks */
      printf("{\"lanes\": %d, \"kernel_us\": %.2f", lanes, ms * 1e3);
      for (int q = 0; q < 5; q++) printf(", \"%s_clk\": %llu", nm[q], (unsigned long long)(st[q + 1] - st[q]));
      uint64_t hq[64 * 6];
      CHECK(hipMemcpy(hq, d_htm, sizeof(hq), hipMemcpyDeviceToHost));
      printf(", \"lehmer_clk\": %llu, \"single_clk\": %llu, \"final_clk\": %llu, \"rounds\": %llu, \"inner\": %llu, \"singles\": %llu",
             (unsigned long long)hq[0], (unsigned long long)hq[1], (unsigned long long)hq[2], (unsigned long long)hq[3],
             (unsigned long long)hq[4], (unsigned long long)hq[5]);
      if (lanes == 64) {
        uint64_t mx[6] = {0, 0, 0, 0, 0, 0};
        for (int j = 0; j < 64; j++) for (int q = 3; q < 6; q++) mx[q] = hq[6 * j + q] > mx[q] ? hq[6 * j + q] : mx[q];
        printf(", \"max_rounds\": %llu, \"max_inner\": %llu, \"max_singles\": %llu", (unsigned long long)mx[3],
               (unsigned long long)mx[4], (unsigned long long)mx[5]);
      }
      printf("}\n");
      CHECK(hipEventDestroy(a));
      CHECK(hipEventDestroy(b));
    }
  }
  return 0;
}
