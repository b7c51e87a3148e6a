/* fd_ed25519_gen.hip -- batched keygen / sign on gfx950 and the synthetic
   workload generator used by bench.py.

   fd_ed25519_sign_kernel restates fd_ed25519_public_from_private and
   fd_ed25519_sign (src/ballet/ed25519/fd_ed25519_user.c:4-132, RFC 8032
   5.1.5-5.1.6) one signature per lane:
     h = SHA-512(priv); a = clamp(h[0:32]); prefix = h[32:64]
     A = [a]B; r = SHA-512(prefix || M) mod L; R = [r]B
     k = SHA-512(R || A || M) mod L; S = (r + k a) mod L
   Signing is deterministic, so identical (priv, M) give byte-identical
   signatures to the reference (pinned by tests against the sign KATs).

   The generator derives every byte from a 64-bit seed with a counter-based
   mixer (splitmix64 finalizer), so any shard of a stream can be produced on
   any GPU, and the same bytes can be recomputed on the host
   (firedancer_amd/workload.py) for cross-checks. */
#include <hip/hip_runtime.h>
#include "fd25519_dsm.h"
#include "fd25519_sc.h"
#include "fd_sha512_dev.h"

#define GEN_GOLDEN 0x9E3779B97F4A7C15ULL
#define GEN_MSG_SALT 0xA0761D6478BD642FULL
#define GEN_BAD_SALT 0xE7037ED1A0B428DBULL

FD_DEV uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

/* message buffer byte b = byte (b % 8) of mix64((seed ^ MSG_SALT) + GOLDEN (b/8 + 1)) */
__global__ void fd_ed25519_fill_random_kernel(uint8_t* d, uint64_t nbytes, uint64_t seed) {
  const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t b0 = w * 8;
  if (b0 >= nbytes) return;
  const uint64_t x = mix64((seed ^ GEN_MSG_SALT) + GEN_GOLDEN * (w + 1));
  if (b0 + 8 <= nbytes && ((reinterpret_cast<uintptr_t>(d) & 7) == 0)) {
    reinterpret_cast<uint64_t*>(d)[w] = x;
  } else {
    for (int k = 0; k < 8 && b0 + k < nbytes; k++) d[b0 + k] = (uint8_t)(x >> (8 * k));
  }
}

/* 256 x 256 -> 512-bit product plus a 256-bit addend */
FD_DEV void mul256_add(uint32_t (&out)[16], const uint32_t (&a)[8], const uint32_t (&b)[8],
                       const uint32_t (&c)[8]) {
#pragma unroll
  for (int i = 0; i < 16; i++) out[i] = i < 8 ? c[i] : 0u;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint64_t t = (uint64_t)a[i] * b[j] + out[i + j] + carry;
      out[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
#pragma unroll
    for (int j = i + 8; j < 16; j++) {
      const uint64_t t = (uint64_t)out[j] + carry;
      out[j] = (uint32_t)t;
      carry = t >> 32;
    }
  }
}

__global__ void __launch_bounds__(256)
fd_ed25519_sign_kernel(fd_ed25519_sign_params_t p) {
  __shared__ int4 s_btab[FD_ED25519_BTAB_INTS / 4];
  const int4* g_btab = reinterpret_cast<const int4*>(p.btab);
  for (int t = threadIdx.x; t < FD_ED25519_BTAB_INTS / 4; t += blockDim.x) s_btab[t] = g_btab[t];
  __syncthreads();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;

  uint32_t priv[8];
  if (p.privs) {
    const uint4* src = reinterpret_cast<const uint4*>(p.privs + 32 * i);
    const uint4 q0 = src[0], q1 = src[1];
    priv[0] = q0.x; priv[1] = q0.y; priv[2] = q0.z; priv[3] = q0.w;
    priv[4] = q1.x; priv[5] = q1.y; priv[6] = q1.z; priv[7] = q1.w;
  } else {
    const uint64_t g = p.index_base + i;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint64_t x = mix64(p.seed + GEN_GOLDEN * (4 * g + q + 1));
      priv[2 * q] = (uint32_t)x;
      priv[2 * q + 1] = (uint32_t)(x >> 32);
    }
  }

  sha_msg_src none;
  none.base = reinterpret_cast<const uint32_t*>(p.msgs);
  none.shift = 0;
  none.sz = 0;
  uint32_t h[16];
  sha512_pre<8>(h, priv, none);
  uint32_t a[8], prefix[8];
#pragma unroll
  for (int w = 0; w < 8; w++) {
    a[w] = h[w];
    prefix[w] = h[8 + w];
  }
  a[0] &= 0xFFFFFFF8u;
  a[7] &= 0x7FFFFFFFu;
  a[7] |= 0x40000000u;

  uint32_t enc_a[8], enc_r[8];
  {
    uint32_t wide[16], amod[8];
#pragma unroll
    for (int w = 0; w < 16; w++) wide[w] = w < 8 ? a[w] : 0u;
    sc_reduce512(amod, wide);
    ge_p2 Q;
    ge_scalarmult_base(Q, amod, s_btab);
    ge_encode(enc_a, Q);
  }

  const uintptr_t mp = reinterpret_cast<uintptr_t>(p.msgs + p.msg_off[i]);
  sha_msg_src m;
  m.base = reinterpret_cast<const uint32_t*>(mp & ~(uintptr_t)3);
  m.shift = (uint32_t)(mp & 3);
  m.sz = p.msg_sz[i];

  uint32_t r[8];
  {
    uint32_t rh[16];
    sha512_pre<8>(rh, prefix, m);
    sc_reduce512(r, rh);
    ge_p2 Q;
    ge_scalarmult_base(Q, r, s_btab);
    ge_encode(enc_r, Q);
  }
  uint32_t S[8];
  {
    uint32_t kh[16], k[8], prod[16];
    sha512_ram(kh, enc_r, enc_a, m);
    sc_reduce512(k, kh);
    mul256_add(prod, k, a, r);
    sc_reduce512(S, prod);
  }
  uint4* sg = reinterpret_cast<uint4*>(p.sigs + 64 * i);
  uint4* pk = reinterpret_cast<uint4*>(p.pubs + 32 * i);
  sg[0] = make_uint4(enc_r[0], enc_r[1], enc_r[2], enc_r[3]);
  sg[1] = make_uint4(enc_r[4], enc_r[5], enc_r[6], enc_r[7]);
  sg[2] = make_uint4(S[0], S[1], S[2], S[3]);
  sg[3] = make_uint4(S[4], S[5], S[6], S[7]);
  pk[0] = make_uint4(enc_a[0], enc_a[1], enc_a[2], enc_a[3]);
  pk[1] = make_uint4(enc_a[4], enc_a[5], enc_a[6], enc_a[7]);
}

/* ------------------------------------------------------------------------
   Invalid-signature injection (SURVEY.md §8(d) C2 classes).  For signature
   g = index_base + i, x = mix64((seed ^ BAD_SALT) + GOLDEN (g+1)); it is
   corrupted iff x % 10^6 < ppm, with class 1 + (x >> 32) % 7 and the code
   the reference's AVX-512 build returns for that class:

     1 S += L                          -> ERR_SIG
     2 A := small-order encoding       -> ERR_PUBKEY
     3 R := small-order encoding       -> ERR_SIG
     4 A := undecodable encoding       -> ERR_SIG   (portable build: ERR_PUBKEY)
     5 R := undecodable encoding       -> ERR_SIG
     6 A := non-canonical y (p, p+1)   -> ERR_PUBKEY (decodes to a small-order point)
     7 flip one message bit            -> ERR_MSG                               */

__constant__ uint32_t gen_small_order[8][8] = {
  {0x00000001u, 0, 0, 0, 0, 0, 0, 0x00000000u},
  {0xffffffecu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu},
  {0, 0, 0, 0, 0, 0, 0, 0},
  {0, 0, 0, 0, 0, 0, 0, 0x80000000u},
  {0x8f95e826u, 0xb027b2c2u, 0x89f4c345u, 0xf098eff2u, 0x05acdfd5u, 0x3933c6d3u, 0x880238b1u, 0x05fc536du},
  {0x8f95e826u, 0xb027b2c2u, 0x89f4c345u, 0xf098eff2u, 0x05acdfd5u, 0x3933c6d3u, 0x880238b1u, 0x85fc536du},
  {0x706a17c7u, 0x4fd84d3du, 0x760b3cbau, 0x0f67100du, 0xfa53202au, 0xc6cc392cu, 0x77fdc74eu, 0x7a03ac92u},
  {0x706a17c7u, 0x4fd84d3du, 0x760b3cbau, 0x0f67100du, 0xfa53202au, 0xc6cc392cu, 0x77fdc74eu, 0xfa03ac92u},
};
/* no square root: 02..00 and b898e00f...7447 (src/ballet/ed25519/test_ed25519.c:646-650) */
__constant__ uint32_t gen_undecodable[2][8] = {
  {0x00000002u, 0, 0, 0, 0, 0, 0, 0},
  {0x0fe098b8u, 0x58f76d6fu, 0x5ca0f9b3u, 0x5fb173bfu, 0x08a092d3u, 0xd417a4a9u, 0xc178c171u, 0x47748cb2u},
};
/* y = p and y = p + 1, sign 0 */
__constant__ uint32_t gen_noncanon[2][8] = {
  {0xffffffedu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu},
  {0xffffffeeu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu},
};

FD_DEV void put8(uint8_t* dst, const uint32_t* w) {
  uint4* d = reinterpret_cast<uint4*>(dst);
  d[0] = make_uint4(w[0], w[1], w[2], w[3]);
  d[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

__global__ void fd_ed25519_corrupt_kernel(fd_ed25519_corrupt_params_t p) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  const uint64_t x = mix64((p.seed ^ GEN_BAD_SALT) + GEN_GOLDEN * (p.index_base + i + 1));
  int cls = 0;
  if ((uint32_t)(x % 1000000ULL) < p.ppm) cls = 1 + (int)((x >> 32) % 7ULL);
  const uint32_t sel = (uint32_t)(x >> 40);
  int expect = FD_ED25519_SUCCESS;
  uint8_t* sig = p.sigs + 64 * i;
  uint8_t* pub = p.pubs + 32 * i;
  switch (cls) {
  case 1: {  /* S += L */
    uint32_t* S = reinterpret_cast<uint32_t*>(sig + 32);
    const uint32_t l[8] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu, 0u, 0u, 0u, 0x10000000u};
    uint64_t c = 0;
    for (int w = 0; w < 8; w++) {
      const uint64_t t = (uint64_t)S[w] + l[w] + c;
      S[w] = (uint32_t)t;
      c = t >> 32;
    }
    expect = -1;
  } break;
  case 2: put8(pub, gen_small_order[sel & 7]); expect = -2; break;
  case 3: put8(sig, gen_small_order[sel & 7]); expect = -1; break;
  case 4: put8(pub, gen_undecodable[sel & 1]); expect = -1; break;
  case 5: put8(sig, gen_undecodable[sel & 1]); expect = -1; break;
  case 6: put8(pub, gen_noncanon[sel & 1]); expect = -2; break;
  case 7: {
    const uint32_t sz = p.msg_sz[i];
    if (sz) {
      const uint32_t bit = sel % (8u * sz);
      p.msgs[p.msg_off[i] + (bit >> 3)] ^= (uint8_t)(1u << (bit & 7));
      expect = -3;
    } else {
      cls = 0;
    }
  } break;
  default: break;
  }
  if (p.expect) p.expect[i] = (int8_t)expect;
  if (p.cls) p.cls[i] = (uint8_t)cls;
}

extern "C" int fd_ed25519_hip_launch_fill_random(uint8_t* d, uint64_t nbytes, uint64_t seed, void* stream) {
  if (!nbytes) return 0;
  const uint64_t words = (nbytes + 7) / 8;
  hipLaunchKernelGGL(fd_ed25519_fill_random_kernel, dim3((uint32_t)((words + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, d, nbytes, seed);
  return (int)hipGetLastError();
}

extern "C" int fd_ed25519_hip_launch_sign(const fd_ed25519_sign_params_t* p, void* stream) {
  if (!p->n) return 0;
  hipLaunchKernelGGL(fd_ed25519_sign_kernel, dim3((uint32_t)((p->n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, *p);
  return (int)hipGetLastError();
}

extern "C" int fd_ed25519_hip_launch_corrupt(const fd_ed25519_corrupt_params_t* p, void* stream) {
  if (!p->n) return 0;
  hipLaunchKernelGGL(fd_ed25519_corrupt_kernel, dim3((uint32_t)((p->n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, *p);
  return (int)hipGetLastError();
}
