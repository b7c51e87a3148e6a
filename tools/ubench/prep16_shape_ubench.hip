// prep16's time by batch size and by part (gfx950): the production kernel
// (fd_ed25519_kernels.hip compiled in) launched as the engine launches it
// -- hash blocks of two waves per 32 messages, then decode blocks of two
// waves, four points a wave -- and with only its hash blocks, or only its
// decode blocks (hash_blocks = 0), over n signatures of 200-byte messages.
// HIP events around each launch (a few microseconds of event overhead in
// every figure alike).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I firedancer_amd/csrc -o tools/ubench/prep16_shape_ubench tools/ubench/prep16_shape_ubench.hip
#include "../../firedancer_amd/csrc/fd_ed25519_kernels.hip"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

int main() {
  const int msz = 200, cap = 512;
  std::vector<uint8_t> h_sig(64 * cap), h_pub(32 * cap), h_msg((size_t)msz * cap + 64);
  std::vector<uint64_t> h_off(cap);
  std::vector<uint32_t> h_sz(cap, msz);
  srand(11);
  for (auto& b : h_sig) b = (uint8_t)rand();
  for (auto& b : h_pub) b = (uint8_t)rand();
  for (auto& b : h_msg) b = (uint8_t)rand();
  for (int j = 0; j < cap; j++) { h_sig[64 * j + 63] &= 0x0f; h_off[j] = (uint64_t)msz * j; }
  fd_ed25519_verify_params_t p;
  memset(&p, 0, sizeof(p));
  uint8_t *d_sig, *d_pub, *d_msg, *d_work;
  int8_t* d_out;
  uint64_t* d_off;
  uint32_t* d_sz;
  CHECK(hipMalloc(&d_sig, h_sig.size()));
  CHECK(hipMalloc(&d_pub, h_pub.size()));
  CHECK(hipMalloc(&d_msg, h_msg.size()));
  CHECK(hipMalloc(&d_off, cap * 8));
  CHECK(hipMalloc(&d_sz, cap * 4));
  CHECK(hipMalloc(&d_out, cap));
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
  p.small = 3;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  printf("{\"device\": \"%s\", \"msg_sz\": %d}\n", prop.gcnArchName, msz);
  const char* part_name[3] = {"full", "hash_only", "decode_only"};
  for (int n : {1, 32, 64, 128, 256, 512}) {
    p.n = n;
    const uint32_t hb = (uint32_t)((n + SHA2W_LANES - 1) / SHA2W_LANES), dw = (uint32_t)((n + 1) / 2);
    for (int part = 0; part < 3; part++) {
      const uint32_t grid = part == 0 ? hb + (dw + 1) / 2 : part == 1 ? hb : (dw + 1) / 2;
      const uint32_t hbl = part == 2 ? 0u : hb;
      std::vector<float> us;
      for (int rep = 0; rep < 23; rep++) {
        hipEvent_t a, b;
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL(fd_ed25519_prep16_kernel, dim3(grid), dim3(128), 0, 0, p, hbl);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        if (rep >= 3) us.push_back(ms * 1e3f);
        CHECK(hipEventDestroy(a));
        CHECK(hipEventDestroy(b));
      }
      std::sort(us.begin(), us.end());
      printf("{\"n\": %d, \"part\": \"%s\", \"blocks\": %u, \"p50_us\": %.2f, \"min_us\": %.2f}\n", n, part_name[part],
             grid, us[us.size() / 2], us[0]);
    }
  }
  return 0;
}
