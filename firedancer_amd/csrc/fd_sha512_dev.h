/* fd_sha512_dev.h -- SHA-512 of R || A || M for gfx950, one message per lane.

   Computes the challenge hash of the verify equation,
   k = SHA-512(R || A || M), as fd_ed25519_verify does with
   fd_sha512_init/append/fini (src/ballet/ed25519/fd_ed25519_user.c:203-205;
   core src/ballet/sha512/fd_sha512.c:128-231).  FIPS 180-4: 80 rounds of
   64-bit big-endian arithmetic per 128-byte block; ceil((81+sz)/128)
   blocks for a message of sz bytes.

   Message bytes are read straight from the SoA message buffer in HBM with
   dword-aligned 16-byte loads (any message byte offset is accepted) and
   realigned in registers (v_alignbyte_b32); the next block's loads are in
   flight while the current block is compressed.  Padding (0x80, zeros,
   128-bit length) is synthesized in registers. */
#pragma once
#include "fd25519_fe.h"

__constant__ uint64_t fd_sha512_dev_k[80] = {
  0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
  0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
  0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
  0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
  0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
  0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
  0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
  0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
  0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
  0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
  0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
  0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
  0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
  0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
  0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
  0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
  0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
  0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
  0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
  0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL,
};

/* 64-bit words live in VGPR pairs; the rotations, shifts and 3-input
   boolean functions are written on the 32-bit halves so that each costs
   one full-rate op per half: a rotation is two v_alignbit_b32 (funnel
   shifts), xor3 / maj / ch one v_bitop3_b32 each (gfx950's 3-input LUT op,
   truth-table index = a<<2 | b<<1 | c).  Left to itself LLVM builds the
   rotations from 64-bit shifts and ors. */
#ifndef FD_SHA_OPAQUE_PAIR
#define FD_SHA_OPAQUE_PAIR 1
#endif
FD_DEV uint32_t sha_lo(uint64_t x) { return (uint32_t)x; }
FD_DEV uint32_t sha_hi(uint64_t x) { return (uint32_t)(x >> 32); }
FD_DEV uint64_t sha_pair(uint32_t hi, uint32_t lo) {
  uint64_t x = ((uint64_t)hi << 32) | lo;
#if FD_SHA_OPAQUE_PAIR
  asm("" : "+v"(x));
#endif
  return x;
}

FD_DEV uint64_t sha_ror(uint64_t x, int n) {
  const uint32_t lo = sha_lo(x), hi = sha_hi(x);
  if (n < 32) return sha_pair(__builtin_amdgcn_alignbit(lo, hi, n), __builtin_amdgcn_alignbit(hi, lo, n));
  return sha_pair(__builtin_amdgcn_alignbit(hi, lo, n - 32), __builtin_amdgcn_alignbit(lo, hi, n - 32));
}

FD_DEV uint64_t sha_shr(uint64_t x, int n) {  /* n < 32 */
  const uint32_t lo = sha_lo(x), hi = sha_hi(x);
  return sha_pair(hi >> n, __builtin_amdgcn_alignbit(hi, lo, n));
}

template <int LUT>
FD_DEV uint64_t sha_bitop3(uint64_t a, uint64_t b, uint64_t c) {
  return sha_pair(__builtin_amdgcn_bitop3_b32(sha_hi(a), sha_hi(b), sha_hi(c), LUT),
                  __builtin_amdgcn_bitop3_b32(sha_lo(a), sha_lo(b), sha_lo(c), LUT));
}
#define SHA_XOR3 0x96
#define SHA_MAJ  0xE8
#define SHA_CH   0xCA

FD_DEV uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

/* One compression: h <- h + F(h, w).  The schedule is kept as a rolling
   16-word window; rounds are unrolled 16 at a time with the round constants
   read through the scalar cache. */
template <bool SCHED>
FD_DEV void sha512_rounds16(uint64_t (&v)[8], uint64_t (&w)[16], int r0) {
  uint64_t a = v[0], b = v[1], c = v[2], d = v[3], e = v[4], f = v[5], g = v[6], hh = v[7];
#pragma unroll
  for (int r = 0; r < 16; r++) {
    if (SCHED) {
      const uint64_t w15 = w[(r + 1) & 15], w2 = w[(r + 14) & 15];
      const uint64_t s0 = sha_bitop3<SHA_XOR3>(sha_ror(w15, 1), sha_ror(w15, 8), sha_shr(w15, 7));
      const uint64_t s1 = sha_bitop3<SHA_XOR3>(sha_ror(w2, 19), sha_ror(w2, 61), sha_shr(w2, 6));
      w[r] += s0 + w[(r + 9) & 15] + s1;
    }
    const uint64_t S1 = sha_bitop3<SHA_XOR3>(sha_ror(e, 14), sha_ror(e, 18), sha_ror(e, 41));
    const uint64_t ch = sha_bitop3<SHA_CH>(e, f, g);
    const uint64_t t1 = hh + S1 + ch + fd_sha512_dev_k[r0 + r] + w[r];
    const uint64_t S0 = sha_bitop3<SHA_XOR3>(sha_ror(a, 28), sha_ror(a, 34), sha_ror(a, 39));
    const uint64_t mj = sha_bitop3<SHA_MAJ>(a, b, c);
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;
  }
  v[0] = a; v[1] = b; v[2] = c; v[3] = d; v[4] = e; v[5] = f; v[6] = g; v[7] = hh;
}

/* rounds 0..15 on the block's words, then 4 x 16 with the schedule (a
   loop with no per-round test) */
FD_DEV void sha512_block(uint64_t (&h)[8], uint64_t (&w)[16]) {
  uint64_t v[8];
#pragma unroll
  for (int i = 0; i < 8; i++) v[i] = h[i];
  sha512_rounds16<false>(v, w, 0);
#pragma clang loop unroll(disable)
  for (int r0 = 16; r0 < 80; r0 += 16) sha512_rounds16<true>(v, w, r0);
#pragma unroll
  for (int i = 0; i < 8; i++) h[i] += v[i];
}

/* A lane's message: base is the aligned dword holding message byte 0,
   which is byte `shift` of it. */
struct sha_msg_src {
  const uint32_t* base;
  uint32_t shift;
  uint32_t sz;
};

/* 16-byte load of base dwords [j, j+4); skipped (zero) unless it holds a
   message byte.  Dword-aligned global_load_dwordx4 (gfx950 unaligned mode).
   A chunk that holds the last message byte may read up to 15 bytes past
   the message; callers keep message buffers readable that far (the
   engine's staging and generator buffers are padded). */
FD_DEV uint4 sha_chunk(const sha_msg_src& m, int j) {
  uint4 v = make_uint4(0u, 0u, 0u, 0u);
  if (j >= 0 && 4u * (uint32_t)j < m.shift + m.sz) __builtin_memcpy(&v, m.base + j, 16);
  return v;
}

/* Message dword at message byte position p (p % 4 == 0), from the two base
   dwords covering it, padded: bytes >= sz are zero except byte sz = 0x80.
   Little-endian (memory) byte order. */
FD_DEV uint32_t sha_msg_dword(const sha_msg_src& m, int p, uint32_t lo, uint32_t hi) {
  uint32_t d = __builtin_amdgcn_alignbyte(hi, lo, m.shift);
  const int n = (int)m.sz - p;
  const uint32_t keep = n >= 4 ? 0xffffffffu : (n > 0 ? (1u << (8 * n)) - 1u : 0u);
  const uint32_t pad = (n >= 0 && n < 4) ? (0x80u << (8 * n)) : 0u;
  return (d & keep) | pad;
}

#define SHA_CHUNKS 9  /* 36 dwords cover a 128-byte block at any byte shift */

FD_DEV void sha_load_block(uint4 (&c)[SHA_CHUNKS], const sha_msg_src& m, int j0) {
#pragma unroll
  for (int q = 0; q < SHA_CHUNKS; q++) c[q] = sha_chunk(m, j0 + 4 * q);
}

FD_DEV uint32_t sha_chunk_dword(const uint4 (&c)[SHA_CHUNKS], int i) {
  const uint4 v = c[i >> 2];
  return (i & 3) == 0 ? v.x : (i & 3) == 1 ? v.y : (i & 3) == 2 ? v.z : v.w;
}

/* digest (as 16 little-endian words of the 64-byte output) of
   PRE || M(sz), where PRE is NPRE 32-bit words (8: a 32-byte prefix, e.g.
   the signing nonce prefix; 16: R || A) held in registers as little-endian
   words.  Block b covers stream dwords [32 b, 32 b + 32), i.e. message
   dwords from j0 = 32 b - NPRE; its 9 chunk loads are issued before the
   previous block is compressed, so the load latency hides under 80 rounds. */
/* Message schedule words of block b from its chunks (and, for the first
   block, the register prefix), with padding and the length in the last. */
/* FULL: every byte of the block is a message byte (blocks b + 2 < nblk), so
   no padding masks and no length words. */
template <int NPRE, bool FIRST, bool FULL = false>
FD_DEV void sha_build_w(uint64_t (&w)[16], const uint4 (&c)[SHA_CHUNKS], const uint32_t (&pre)[NPRE],
                        const sha_msg_src& m, uint32_t b, uint32_t nblk, uint64_t bitlen) {
  constexpr int PB = 4 * NPRE;
  constexpr int PW = NPRE / 2;
  const int p0 = 128 * (int)b - PB;  /* message byte position of word 0 */
#pragma unroll
  for (int t = 0; t < 16; t++) {
    uint32_t d0, d1;
    if (FIRST && t < PW) {
      d0 = pre[2 * t];
      d1 = pre[2 * t + 1];
    } else if (FULL) {
      /* realign and byte-swap in one v_perm_b32: byte k of the big-endian
         word is byte shift + 3 - k of {hi, lo} */
      const uint32_t sel = 0x00010203u + m.shift * 0x01010101u;
      const uint32_t e0 = __builtin_amdgcn_perm(sha_chunk_dword(c, 2 * t + 1), sha_chunk_dword(c, 2 * t), sel);
      const uint32_t e1 = __builtin_amdgcn_perm(sha_chunk_dword(c, 2 * t + 2), sha_chunk_dword(c, 2 * t + 1), sel);
      w[t] = ((uint64_t)e0 << 32) | (uint64_t)e1;
      continue;
    } else {
      const int p = p0 + 8 * t;
      d0 = sha_msg_dword(m, p, sha_chunk_dword(c, 2 * t), sha_chunk_dword(c, 2 * t + 1));
      d1 = sha_msg_dword(m, p + 4, sha_chunk_dword(c, 2 * t + 1), sha_chunk_dword(c, 2 * t + 2));
    }
    uint64_t word = ((uint64_t)bswap32(d0) << 32) | (uint64_t)bswap32(d1);
    if (!FULL && b + 1 == nblk) {
      if (t == 14) word = 0;
      if (t == 15) word = bitlen;
    }
    w[t] = word;
  }
}

/* digest (as 16 little-endian words of the 64-byte output) of
   PRE || M(sz), where PRE is NPRE 32-bit words (8: a 32-byte prefix, e.g.
   the signing nonce prefix; 16: R || A) held in registers as little-endian
   words.  Block b covers stream dwords [32 b, 32 b + 32), i.e. message
   dwords from j0 = 32 b - NPRE.  Once a block's schedule is built, its chunk
   registers receive the next block's loads, in flight during the 80
   rounds.  The first block (prefix + message head) is peeled so the prefix
   registers die before the loop. */
template <int NPRE>
FD_DEV void sha512_pre(uint32_t (&out)[16], const uint32_t (&pre)[NPRE], const sha_msg_src& m) {
  static_assert(NPRE == 8 || NPRE == 16, "prefix is 32 or 64 bytes");
  constexpr int PB = 4 * NPRE;   /* prefix bytes */
  uint64_t h[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                   0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                   0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  const uint32_t nblk = (m.sz + PB + 17u + 127u) >> 7;
  const uint64_t bitlen = (uint64_t)(PB + m.sz) << 3;
  uint4 cur[SHA_CHUNKS];
  uint64_t w[16];
  sha_load_block(cur, m, -NPRE);
  sha_build_w<NPRE, true>(w, cur, pre, m, 0u, nblk, bitlen);
  if (nblk > 1) sha_load_block(cur, m, 32 - NPRE);
  sha512_block(h, w);
  for (uint32_t b = 1; b < nblk; b++) {
    if (b + 2 < nblk) sha_build_w<NPRE, false, true>(w, cur, pre, m, b, nblk, bitlen);
    else sha_build_w<NPRE, false>(w, cur, pre, m, b, nblk, bitlen);
    if (b + 1 < nblk) sha_load_block(cur, m, 32 * (int)(b + 1) - NPRE);
    sha512_block(h, w);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    out[2 * i] = bswap32((uint32_t)(h[i] >> 32));
    out[2 * i + 1] = bswap32((uint32_t)h[i]);
  }
}

/* ---- the hash over two waves (the latency form's prep16) ----------------

   A lane's hash is a chain of 80 rounds per block, and at one wave per
   SIMD the wave issues every instruction of it in turn: the message
   schedule (~20 of the ~50 VALU operations of a round) sits in that
   chain only because the same lane computes it.  Here a second wave of
   the block builds each block's 80 schedule words into LDS (one buffer
   per block parity) while the first runs the rounds of the block before
   from the other buffer; one workgroup barrier per block hands a buffer
   over.  Same digest, bit for bit (the words and rounds are the
   one-wave form's).  32 messages per pair of waves (lanes 32..63 repeat
   lanes 0..31), so the two buffers are 40 KiB and four blocks fit a CU. */
#define SHA2W_LANES 32
#define SHA2W_WORDS (80 * SHA2W_LANES)   /* one buffer: [word][lane], 64-bit */

/* wave 1: the schedules of blocks 0 .. nblk_wave - 1 of this lane's
   PRE || M, block b into buf[b & 1], a barrier after each */
template <int NPRE>
FD_DEV void sha512_sched_wave(const uint32_t (&pre)[NPRE], const sha_msg_src& m, uint32_t nblk_wave, uint64_t* lds) {
  constexpr int PB = 4 * NPRE;
  const uint32_t lane = threadIdx.x & (SHA2W_LANES - 1u);
  const bool writer = (threadIdx.x & 63u) < SHA2W_LANES;
  const uint32_t nblk = (m.sz + PB + 17u + 127u) >> 7;
  const uint64_t bitlen = (uint64_t)(PB + m.sz) << 3;
  if (!nblk_wave) return;
  uint4 cur[SHA_CHUNKS];
  uint64_t w[16];
  sha_load_block(cur, m, -NPRE);
#pragma clang loop unroll(disable)
  for (uint32_t b = 0; b < nblk_wave; b++) {
    if (b == 0) sha_build_w<NPRE, true>(w, cur, pre, m, 0u, nblk, bitlen);
    else if (b + 2 < nblk) sha_build_w<NPRE, false, true>(w, cur, pre, m, b, nblk, bitlen);
    else sha_build_w<NPRE, false>(w, cur, pre, m, b, nblk, bitlen);
    if (b + 1 < nblk) sha_load_block(cur, m, 32 * (int)(b + 1) - NPRE);
    uint64_t* dst = lds + (b & 1u) * SHA2W_WORDS + lane;
#pragma unroll
    for (int t = 0; t < 16; t++)
      if (writer) dst[SHA2W_LANES * t] = w[t];
#pragma unroll 16
    for (int t = 16; t < 80; t++) {
      const uint64_t w15 = w[(t + 1) & 15], w2 = w[(t + 14) & 15];
      const uint64_t s0 = sha_bitop3<SHA_XOR3>(sha_ror(w15, 1), sha_ror(w15, 8), sha_shr(w15, 7));
      const uint64_t s1 = sha_bitop3<SHA_XOR3>(sha_ror(w2, 19), sha_ror(w2, 61), sha_shr(w2, 6));
      w[t & 15] += s0 + w[(t + 9) & 15] + s1;
      if (writer) dst[SHA2W_LANES * t] = w[t & 15];
    }
    __syncthreads();
  }
}

/* wave 0: 80 rounds per block from the schedule in LDS, a barrier before
   each; the digest of this lane's PRE || M as sha512_pre returns it
   (blocks past the lane's own count are run and dropped) */
template <int NPRE>
FD_DEV void sha512_rounds_wave(uint32_t (&out)[16], const sha_msg_src& m, uint32_t nblk_wave, const uint64_t* lds) {
  constexpr int PB = 4 * NPRE;
  const uint32_t lane = threadIdx.x & (SHA2W_LANES - 1u);
  const uint32_t nblk = (m.sz + PB + 17u + 127u) >> 7;
  uint64_t h[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                   0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                   0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
#pragma clang loop unroll(disable)
  for (uint32_t b = 0; b < nblk_wave; b++) {
    __syncthreads();
    const uint64_t* src = lds + (b & 1u) * SHA2W_WORDS + lane;
    uint64_t v[8];
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = h[i];
#pragma clang loop unroll(disable)
    for (int r0 = 0; r0 < 80; r0 += 16) {
      uint64_t w[16];
#pragma unroll
      for (int r = 0; r < 16; r++) w[r] = src[SHA2W_LANES * (r0 + r)];
      sha512_rounds16<false>(v, w, r0);
    }
    const bool mine = b < nblk;
#pragma unroll
    for (int i = 0; i < 8; i++) h[i] += mine ? v[i] : 0ull;
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    out[2 * i] = bswap32((uint32_t)(h[i] >> 32));
    out[2 * i + 1] = bswap32((uint32_t)h[i]);
  }
}

/* digest of R(32) || A(32) || M(sz): the verify challenge */
FD_DEV void sha512_ram(uint32_t (&out)[16], const uint32_t (&r)[8], const uint32_t (&a)[8],
                       const sha_msg_src& m) {
  uint32_t pre[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    pre[i] = r[i];
    pre[8 + i] = a[i];
  }
  sha512_pre<16>(out, pre, m);
}
