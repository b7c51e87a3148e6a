// Where prep16's hash -> scalar chain spends its time (gfx950): one block
// of prep16's hash shape (two waves: wave 1 the message schedule into LDS,
// wave 0 the rounds) over LANES signatures of a 200-byte message, with
// s_memtime stamps on wave 0 after the rounds, after k mod L (hash_finish)
// and after the half-size search + s' (scalar_one); and, for comparison,
// one decode16 wave alone.  The production device code is compiled in.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I firedancer_amd/csrc -o tools/ubench/prep16_stamps_ubench tools/ubench/prep16_stamps_ubench.hip
#include "../../firedancer_amd/csrc/fd_ed25519_kernels.hip"
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

__global__ void __launch_bounds__(128) k_hash_stamped(fd_ed25519_verify_params_t p, uint64_t* st) {
  __shared__ uint64_t sched[2 * SHA2W_WORDS];
  uint64_t t[4];
  t[0] = __builtin_amdgcn_s_memtime();
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint64_t j0 = threadIdx.x & (SHA2W_LANES - 1u);
  const bool live = j0 < p.n && (threadIdx.x & 63u) < SHA2W_LANES;
  const uint64_t j = live ? j0 : p.n - 1u;
  uint32_t pre[16], S[8];
  {
    const uint4* sg = reinterpret_cast<const uint4*>(p.sigs + 64 * j);
    const uint4* pk = reinterpret_cast<const uint4*>(p.pubs + 32 * j);
    const uint4 q0 = sg[0], q1 = sg[1], q2 = sg[2], q3 = sg[3], q4 = pk[0], q5 = pk[1];
    pre[0] = q0.x; pre[1] = q0.y; pre[2] = q0.z; pre[3] = q0.w; pre[4] = q1.x; pre[5] = q1.y; pre[6] = q1.z;
    pre[7] = q1.w;
    pre[8] = q4.x; pre[9] = q4.y; pre[10] = q4.z; pre[11] = q4.w; pre[12] = q5.x; pre[13] = q5.y; pre[14] = q5.z;
    pre[15] = q5.w;
    S[0] = q2.x; S[1] = q2.y; S[2] = q2.z; S[3] = q2.w; S[4] = q3.x; S[5] = q3.y; S[6] = q3.z; S[7] = q3.w;
  }
  sha_msg_src m;
  const uintptr_t mp = reinterpret_cast<uintptr_t>(p.msgs + p.msg_off[j]);
  m.base = reinterpret_cast<const uint32_t*>(mp & ~(uintptr_t)3);
  m.shift = (uint32_t)(mp & 3);
  m.sz = p.msg_sz[j];
  const uint32_t nblk_wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)((m.sz + 64u + 17u + 127u) >> 7));
  if (wave == 1u) {
    sha512_sched_wave<16>(pre, m, nblk_wave, sched);
    return;
  }
  uint32_t dig[16];
  sha512_rounds_wave<16>(dig, m, nblk_wave, sched);
  asm volatile("" :: "v"(dig[0]), "v"(dig[15]));
  t[1] = __builtin_amdgcn_s_memtime();
  if (live) hash_finish(p, j, dig, S);
  t[2] = __builtin_amdgcn_s_memtime();
  if (live) scalar_one(p, j);
  t[3] = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0)
    for (int q = 0; q < 4; q++) st[q] = t[q];
}

__global__ void __launch_bounds__(64) k_decode_stamped(fd_ed25519_verify_params_t p, uint64_t* st) {
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  decode16_wave(p, 0);
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { st[4] = t0; st[5] = t1; }
}

int main() {
  const int msz = 200, cap = 64;
  std::vector<uint8_t> h_sig(64 * cap), h_pub(32 * cap), h_msg((size_t)msz * cap + 64);
  std::vector<uint64_t> h_off(cap);
  std::vector<uint32_t> h_sz(cap, msz);
  srand(7);
  for (auto& b : h_sig) b = (uint8_t)rand();
  for (auto& b : h_pub) b = (uint8_t)rand();
  for (auto& b : h_msg) b = (uint8_t)rand();
  for (int j = 0; j < cap; j++) { h_sig[64 * j + 63] &= 0x0f; h_off[j] = (uint64_t)msz * j; }
  fd_ed25519_verify_params_t p;
  memset(&p, 0, sizeof(p));
  uint8_t *d_sig, *d_pub, *d_msg, *d_work;
  int8_t* d_out;
  uint64_t *d_off, *d_st;
  uint32_t* d_sz;
  CHECK(hipMalloc(&d_sig, h_sig.size()));
  CHECK(hipMalloc(&d_pub, h_pub.size()));
  CHECK(hipMalloc(&d_msg, h_msg.size()));
  CHECK(hipMalloc(&d_off, cap * 8));
  CHECK(hipMalloc(&d_sz, cap * 4));
  CHECK(hipMalloc(&d_out, cap));
  CHECK(hipMalloc(&d_st, 8 * sizeof(uint64_t)));
  const size_t work = (size_t)cap * 1024;
  CHECK(hipMalloc(&d_work, work));
  CHECK(hipMemset(d_work, 0, work));
  CHECK(hipMemcpy(d_sig, h_sig.data(), h_sig.size(), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_pub, h_pub.data(), h_pub.size(), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_msg, h_msg.data(), h_msg.size(), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_off, h_off.data(), cap * 8, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_sz, h_sz.data(), cap * 4, hipMemcpyHostToDevice));
  p.msgs = d_msg; p.msg_off = d_off; p.msg_sz = d_sz; p.sigs = d_sig; p.pubs = d_pub; p.out = d_out;
  p.cap = cap;
  uint8_t* w = d_work;
  p.k = (uint32_t*)w;     w += 8 * 4 * cap;
  p.pts = (int32_t*)w;    w += 2 * 20 * 4 * cap;
  p.hs = (uint32_t*)w;    w += 19 * 4 * cap;
  p.sflag = w;            w += cap;
  p.pflag = w;            w += 2 * cap;
  p.hflag = w;            w += cap;
  p.half_dbits = FD_HALF_DBITS_MAX;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  printf("{\"device\": \"%s\", \"msg_sz\": %d, \"memtime\": \"s_memtime (100 MHz on gfx950 is NOT assumed: ratios only)\"}\n",
         prop.gcnArchName, msz);
  for (int n : {1, 32}) {
    p.n = n;
    for (int rep = 0; rep < 8; rep++) {
      hipEvent_t a, b, c;
      CHECK(hipEventCreate(&a));
      CHECK(hipEventCreate(&b));
      CHECK(hipEventCreate(&c));
      CHECK(hipEventRecord(a));
      hipLaunchKernelGGL(k_hash_stamped, dim3(1), dim3(128), 0, 0, p, d_st);
      CHECK(hipEventRecord(b));
      hipLaunchKernelGGL(k_decode_stamped, dim3(1), dim3(64), 0, 0, p, d_st);
      CHECK(hipEventRecord(c));
      CHECK(hipEventSynchronize(c));
      float ms_h = 0, ms_d = 0;
      CHECK(hipEventElapsedTime(&ms_h, a, b));
      CHECK(hipEventElapsedTime(&ms_d, b, c));
      uint64_t st[6];
      CHECK(hipMemcpy(st, d_st, sizeof(st), hipMemcpyDeviceToHost));
      if (rep < 3) continue;
      printf("{\"lanes\": %d, \"hash_kernel_us\": %.2f, \"decode_kernel_us\": %.2f, \"sha_clk\": %llu, "
             "\"reduce_k_clk\": %llu, \"scalar_one_clk\": %llu, \"decode16_clk\": %llu}\n",
             n, ms_h * 1e3, ms_d * 1e3, (unsigned long long)(st[1] - st[0]), (unsigned long long)(st[2] - st[1]),
             (unsigned long long)(st[3] - st[2]), (unsigned long long)(st[5] - st[4]));
      CHECK(hipEventDestroy(a));
      CHECK(hipEventDestroy(b));
      CHECK(hipEventDestroy(c));
    }
  }
  return 0;
}
