/* fd_ed25519_txn.hip -- raw transaction payloads straight to the verify
   phases (GPU-side fd_txn_parse).

   The host copies frags as they come (payload bytes + offset/size per
   transaction) and reads one byte per transaction: the signature count
   (byte 0; a payload fd_txn_parse accepts has 1..127 signatures there), to
   reserve its signature slots.  On the device, one lane per transaction:

     stage   fd_txn_parse (fd_txn_parse_core.h, the same source the host
             library compiles), with the first 64 bytes of its fd_txn_t
             (the trailer the tile publishes) and, if accepted, the gather of its
             signatures and signer keys into the aligned SoA the verify
             phases read, with every signature's message pointing at the
             payload's message bytes in place (message_off .. end,
             fd_verify.h:57-60)
     finish fd_ed25519_verify_batch_single_msg's combine per transaction,
             with FD_ED25519_TXN_PARSE_FAILED for payloads the parser
             rejected (after_frag's filter, fd_verify.c:117-121) */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/fd_ed25519_hip_tile.h"
#include "fd_ed25519_hip_internal.h"

#define FD_TXN_FN __device__ static inline
#include "fd_txn_parse_core.h"

/* FD_ED25519_SUCCESS / ERR_* come from fd_ed25519_hip.h (via the tile header) */
static_assert(FD_ED25519_TXN_PARSE_FAILED_CODE == FD_ED25519_HIP_TXN_CODE_PARSE_FAILED, "parse-failure code");

/* 16 bytes at any byte address, from dword-aligned loads (the payload
   buffer is readable 16 bytes past every payload, see the staging
   allocation) */
__device__ static inline uint4 load16_any(const uint8_t* src) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(src);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3);
  const uint32_t d0 = w[0], d1 = w[1], d2 = w[2], d3 = w[3], d4 = sh ? w[4] : 0u;
  return make_uint4(__builtin_amdgcn_alignbyte(d1, d0, sh), __builtin_amdgcn_alignbyte(d2, d1, sh),
                    __builtin_amdgcn_alignbyte(d3, d2, sh), __builtin_amdgcn_alignbyte(d4, d3, sh));
}

__global__ void __launch_bounds__(256)
fd_ed25519_txn_stage_kernel(fd_ed25519_txn_stage_params_t p) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= p.ntxn) return;
  const uint8_t* pay = p.payloads + p.pay_off[t];
  const uint32_t sz = p.pay_sz[t];
  fd_ed25519_hip_txn_t tx;
  const uint32_t cnt = p.txn_cnt[t];
  /* the host reserved cnt signature slots from its own read of the
     signature count; the copy parsed here may differ from that read when
     the payload sat in a room the tile can still write (zero-copy).  The
     slots are filled from this parse's offsets, so a count that disagrees
     with the host's -- or an account list shorter than it -- is a parse
     failure: nothing is read past what this parse validated */
  const int good = fd_txn_core_parse(pay, sz, &tx, p.trailer ? p.trailer + 64 * t : nullptr, 64) != 0 &&
                   (uint32_t)tx.signature_cnt == cnt && (uint32_t)tx.acct_addr_cnt >= cnt;
  p.parse_ok[t] = (uint8_t)good;
  const uint32_t slots = (cnt >= 1u && cnt <= 16u) ? cnt : 0u;  /* the host reserved these */
  const uint32_t first = p.txn_first[t];
  for (uint32_t j = 0; j < slots; j++) {
    const uint64_t k = first + j;
    uint4* sg = reinterpret_cast<uint4*>(p.sigs + 64 * k);
    uint4* pk = reinterpret_cast<uint4*>(p.pubs + 32 * k);
    if (good) {
      const uint8_t* s = pay + tx.signature_off + 64u * j;
      const uint8_t* a = pay + tx.acct_addr_off + 32u * j;
#pragma unroll
      for (int q = 0; q < 4; q++) sg[q] = load16_any(s + 16 * q);
      pk[0] = load16_any(a);
      pk[1] = load16_any(a + 16);
      p.msg_off[k] = p.pay_off[t] + tx.message_off;
      p.msg_sz[k] = sz - tx.message_off;
    } else {
      const uint4 z = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
      for (int q = 0; q < 4; q++) sg[q] = z;
      pk[0] = z;
      pk[1] = z;
      p.msg_off[k] = p.pay_off[t];
      p.msg_sz[k] = 0u;
    }
  }
}

/* per-transaction code: parse failure, else the batch_single_msg priority
   (the first phase-1 error in signature order, then ERR_MSG) */
__global__ void __launch_bounds__(256)
fd_ed25519_txn_finish_kernel(const int8_t* sig_codes, const uint32_t* txn_first, const uint32_t* txn_cnt,
                             const uint8_t* parse_ok, int8_t* out, uint64_t ntxn) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntxn) return;
  int code = FD_ED25519_SUCCESS;
  const uint32_t f = txn_first[t], n = txn_cnt[t];
  if (parse_ok && !parse_ok[t]) {
    code = FD_ED25519_TXN_PARSE_FAILED_CODE;
  } else if (n == 0u || n > 16u) {
    code = FD_ED25519_ERR_SIG;
  } else {
    bool msg_fail = false;
    for (uint32_t j = 0; j < n; j++) {
      const int c = sig_codes[f + j];
      if (c == FD_ED25519_ERR_MSG) msg_fail = true;
      else if (c != FD_ED25519_SUCCESS) { code = c; break; }
    }
    if (code == FD_ED25519_SUCCESS && msg_fail) code = FD_ED25519_ERR_MSG;
  }
  out[t] = (int8_t)code;
}

extern "C" int fd_ed25519_hip_launch_txn_stage(const fd_ed25519_txn_stage_params_t* p, void* stream) {
  if (!p->ntxn) return 0;
  const uint32_t blk = 256;
  hipLaunchKernelGGL(fd_ed25519_txn_stage_kernel, dim3((uint32_t)((p->ntxn + blk - 1) / blk)), dim3(blk), 0,
                     (hipStream_t)stream, *p);
  return (int)hipGetLastError();
}

extern "C" int fd_ed25519_hip_launch_txn_finish(const int8_t* d_sig_codes, const uint32_t* d_txn_first,
                                                const uint32_t* d_txn_cnt, const uint8_t* d_parse_ok,
                                                int8_t* d_txn_out, uint64_t ntxn, void* stream) {
  if (!ntxn) return 0;
  const uint32_t blk = 256;
  hipLaunchKernelGGL(fd_ed25519_txn_finish_kernel, dim3((uint32_t)((ntxn + blk - 1) / blk)), dim3(blk), 0,
                     (hipStream_t)stream, d_sig_codes, d_txn_first, d_txn_cnt, d_parse_ok, d_txn_out, ntxn);
  return (int)hipGetLastError();
}

/* fd_ed25519_hip_launch_pull (fd_ed25519_hip_internal.h): blockIdx.y picks
   the span, the x blocks stride over its 16-byte words; the last n % 16
   bytes are copied one by one (never a byte past the span: a span can end
   at the last byte of a registered mapping). */
__global__ void __launch_bounds__(256)
fd_ed25519_pull_kernel(fd_ed25519_pull_params_t p) {
  const uint32_t k = blockIdx.y;
  if (k >= p.cnt) return;
  const uint8_t* src = p.src[k];
  uint8_t* dst = p.dst[k];
  const uint64_t n = p.n[k], n16 = n / 16u;
  const uint4* s4 = reinterpret_cast<const uint4*>(src);
  uint4* d4 = reinterpret_cast<uint4*>(dst);
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
    d4[i] = s4[i];
  if (blockIdx.x == 0 && threadIdx.x < (n & 15u)) dst[16u * n16 + threadIdx.x] = src[16u * n16 + threadIdx.x];
}

extern "C" int fd_ed25519_hip_launch_pull(const fd_ed25519_pull_params_t* p, void* stream) {
  if (!p->cnt) return 0;
  uint64_t most = 0;
  for (uint32_t k = 0; k < p->cnt; k++) most = p->n[k] > most ? p->n[k] : most;
  /* ~8 words per thread, at most 256 blocks per span */
  uint64_t blocks = (most / 16u + 2047u) / 2048u;
  blocks = blocks < 1u ? 1u : blocks > 256u ? 256u : blocks;
  hipLaunchKernelGGL(fd_ed25519_pull_kernel, dim3((uint32_t)blocks, p->cnt), dim3(256), 0, (hipStream_t)stream, *p);
  return (int)hipGetLastError();
}
