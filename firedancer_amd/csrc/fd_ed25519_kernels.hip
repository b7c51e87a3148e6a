/* fd_ed25519_kernels.hip -- gfx950 kernels behind libfd_ed25519_hip.

   Verification of a batch: every step of fd_ed25519_verify
   (src/ballet/ed25519/fd_ed25519_user.c:134-229) for every signature, with
   the verdict computed as data (no early exits, so a wave never diverges on
   an invalid signature), in four phase kernels (see "Phase kernels"):

     1. S < L                          (fd_curve25519_scalar_validate)
     2. decode A and R, reject on no square root (and, in AVX-512 code mode,
        x == 0 with the sign bit set)  (fd_ed25519_point_frombytes_2x)
     3. small-order A, then R          (fd_ed25519_affine_is_small_order)
     4. k = SHA-512(R||A||M) mod L     (fd_sha512_*, fd_curve25519_scalar_reduce)
     5. the group equation [S]B - R - [k]A == 0, cofactorless, as the
        reference's R' = [k](-A) + [S]B == R (fd_ed25519_double_scalar_mul_base,
        fd_ed25519_point_eq_z1)

   R is decoded (step 2, the decode kernel) and enters the equation as a
   point.  Step 5 runs, for all but ~1e-6 of signatures, in the half-size
   form: with c == d k (mod 8L), d odd (the scalar kernel, fd25519_half.h,
   every pair re-checked with integers only), [c](-A) + [|d|](-+R) +
   [s_lo]B + [s_hi][2^144]B == 0 in a four-scalar Straus loop of 33 signed
   4-bit windows (dsm_half_one), exactly equivalent since [d] is invertible
   on the group of order 8L; the rest in the full-length form
   [k](-A) + [S]B == R (dsm_full_one).  Fixed windows instead of the
   reference's sliding wNAF make every lane of a wave execute the same
   additions; the group element is the same, so the verdict is
   bit-identical.

   Tables: per-lane [1..8](-A) and [1..8](-+R) in an HBM scratch of the
   persistent dsm grid (dynamically scheduled, 64 items per wave); the base
   tables [0..2^24)B and [0..2^24)[2^144]B (or the compact radix-2^16 pair)
   and [0..2^15]B (full-length form) in HBM, shared by the engines of a
   device; [0..128]B in LDS for the signing kernels only. */
#include <hip/hip_runtime.h>
#include "fd25519_dsm.h"
#include "fd25519_ge4.h"
#include "fd25519_sc.h"
#include "fd_sha512_dev.h"
#define FD_HALF_FN __device__ static inline
#define FD_HALF_RCP(y) __builtin_amdgcn_rcp(y)
#define FD_HALF_RCPF(y) __builtin_amdgcn_rcpf(y)
#include "fd25519_half.h"


/* ------------------------------------------------------------------------
   Phase kernels.  A batch is verified by four phases on one stream, each
   kernel with its own register budget, handing ~280 B per signature
   through the work arrays in HBM (fd_ed25519_verify_params_t):

     hash    one lane per signature: S < L, k = SHA-512(R||A||M) mod L
     scalar  one lane per signature: half-size scalars c, d (c == d k mod
             8L) and s' = d S mod L
     decode  one lane per point (A, R): decompression and the reference's
             acceptance / small-order rules
     dsm     persistent, dynamically scheduled: the group equation as
             [c](-A) + [d](-R) + [dS]B == 0, and the full-length form for
             the ~0.13% of signatures whose k has no half-size pair */

#define FD_PF_FAIL  1u
#define FD_PF_SMALL 2u
#define FD_HF_DNEG  1u   /* hflag: d < 0                        */
#define FD_HF_FULL  2u   /* hflag: no (verified) half-size pair, full form */

/* ------------------------------------------------------------------------
   Length sort for the hash phase.  A wave runs as many SHA-512 blocks as
   its longest message; on C2 (64-1232 B) the wave maximum is ~11 blocks
   against a mean of 6.5.  A counting sort of the chunk by block count
   (64 buckets, the last one open-ended) gives every hash wave equal trip
   counts.  Order inside a bucket is arbitrary; results are written by
   signature index, so the output does not depend on it. */

FD_DEV uint32_t nblk_bucket(uint32_t sz) {
  const uint32_t b = (sz + 208u) >> 7;  /* SHA-512 blocks of R||A||M */
  return b < (FD_ED25519_SORT_BUCKETS - 1) ? b : (FD_ED25519_SORT_BUCKETS - 1);
}

/* Each block sorts FD_SORT_PER_BLOCK signatures (FD_SORT_PER_THREAD per
   lane), so a bucket's global counter takes one atomic per 4096 signatures
   (one per 256 had the same-address atomics at the L2 serialize: ~49 us
   per kernel at 1M).  Inside a wave, lanes of one bucket are counted
   together (a ballot per distinct bucket, one LDS atomic by the first
   such lane), and a lane's rank is its group's offset plus the lanes of
   the group below it. */
#define FD_SORT_PER_THREAD 16
#define FD_SORT_PER_BLOCK (256 * FD_SORT_PER_THREAD)

/* adds this lane's element (bucket b, if `valid`) to cnt[]; returns its rank
   among the block's elements of that bucket */
FD_DEV uint32_t sort_wave_count(uint32_t* cnt, uint32_t b, bool valid) {
  const uint32_t lane = threadIdx.x & 63u;
  uint64_t active = __ballot(valid);
  uint32_t r = 0;
  while (active) {
    const int lead = __ffsll((unsigned long long)active) - 1;
    const uint32_t bl = (uint32_t)__shfl((int)b, lead);
    const uint64_t grp = __ballot(valid && b == bl) & active;
    uint32_t off = 0;
    if ((int)lane == lead) off = atomicAdd(&cnt[bl], (uint32_t)__popcll(grp));
    off = (uint32_t)__shfl((int)off, lead);
    if ((grp >> lane) & 1ull) r = off + (uint32_t)__popcll(grp & ((1ull << lane) - 1ull));
    active &= ~grp;
  }
  return r;
}

__global__ void __launch_bounds__(256) fd_ed25519_sort_hist_kernel(fd_ed25519_verify_params_t p) {
  __shared__ uint32_t h[FD_ED25519_SORT_BUCKETS];
  if (threadIdx.x < FD_ED25519_SORT_BUCKETS) h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t j0 = (uint64_t)blockIdx.x * FD_SORT_PER_BLOCK + threadIdx.x;
#pragma unroll
  for (int e = 0; e < FD_SORT_PER_THREAD; e++) {
    const uint64_t j = j0 + (uint64_t)e * 256u;
    const bool v = j < p.n;
    sort_wave_count(h, v ? nblk_bucket(p.msg_sz[p.base + j]) : 0u, v);
  }
  __syncthreads();
  if (threadIdx.x < FD_ED25519_SORT_BUCKETS && h[threadIdx.x]) atomicAdd(&p.hist[threadIdx.x], h[threadIdx.x]);
}

#ifndef FD_ED25519_SORT_DESC
#define FD_ED25519_SORT_DESC 1   /* longest hashes first: hash 1.05 -> 1.01 ms per 1M */
#endif

__global__ void fd_ed25519_sort_scan_kernel(fd_ed25519_verify_params_t p) {
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int i = 0; i < FD_ED25519_SORT_BUCKETS; i++) {
      const int b = FD_ED25519_SORT_DESC ? FD_ED25519_SORT_BUCKETS - 1 - i : i;
      p.hist[FD_ED25519_SORT_BUCKETS + b] = acc;  /* cursor = exclusive prefix */
      acc += p.hist[b];
    }
  }
}

__global__ void __launch_bounds__(256) fd_ed25519_sort_scatter_kernel(fd_ed25519_verify_params_t p) {
  __shared__ uint32_t cnt[FD_ED25519_SORT_BUCKETS], base[FD_ED25519_SORT_BUCKETS];
  if (threadIdx.x < FD_ED25519_SORT_BUCKETS) cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t j0 = (uint64_t)blockIdx.x * FD_SORT_PER_BLOCK + threadIdx.x;
  uint32_t b[FD_SORT_PER_THREAD], r[FD_SORT_PER_THREAD];
#pragma unroll
  for (int e = 0; e < FD_SORT_PER_THREAD; e++) {
    const uint64_t j = j0 + (uint64_t)e * 256u;
    const bool v = j < p.n;
    b[e] = v ? nblk_bucket(p.msg_sz[p.base + j]) : 0u;
    r[e] = sort_wave_count(cnt, b[e], v);
  }
  __syncthreads();
  if (threadIdx.x < FD_ED25519_SORT_BUCKETS && cnt[threadIdx.x])
    base[threadIdx.x] = atomicAdd(&p.hist[FD_ED25519_SORT_BUCKETS + threadIdx.x], cnt[threadIdx.x]);
  __syncthreads();
#pragma unroll
  for (int e = 0; e < FD_SORT_PER_THREAD; e++) {
    const uint64_t j = j0 + (uint64_t)e * 256u;
    if (j < p.n) p.perm[base[b[e]] + r[e]] = (uint32_t)j;
  }
}

/* k = digest mod L and the S < L flag, into the work arrays */
FD_DEV void hash_finish(const fd_ed25519_verify_params_t& p, uint64_t j, const uint32_t (&dig)[16],
                        const uint32_t (&S)[8]) {
  uint32_t k[8];
  sc_reduce512(k, dig);
#pragma unroll
  for (int w = 0; w < 8; w++) p.k[(uint64_t)w * p.cap + j] = k[w];
  p.sflag[j] = sc_is_canonical(S) ? 1 : 0;
}

FD_DEV void hash_one(const fd_ed25519_verify_params_t& p, uint64_t j) {
  const uint64_t i = p.base + j;
  uint32_t r[8], S[8], a[8];
  {
    const uint4* sg = reinterpret_cast<const uint4*>(p.sigs + 64 * i);
    const uint4* pk = reinterpret_cast<const uint4*>(p.pubs + 32 * i);
    const uint4 q0 = sg[0], q1 = sg[1], q2 = sg[2], q3 = sg[3], q4 = pk[0], q5 = pk[1];
    r[0] = q0.x; r[1] = q0.y; r[2] = q0.z; r[3] = q0.w; r[4] = q1.x; r[5] = q1.y; r[6] = q1.z; r[7] = q1.w;
    S[0] = q2.x; S[1] = q2.y; S[2] = q2.z; S[3] = q2.w; S[4] = q3.x; S[5] = q3.y; S[6] = q3.z; S[7] = q3.w;
    a[0] = q4.x; a[1] = q4.y; a[2] = q4.z; a[3] = q4.w; a[4] = q5.x; a[5] = q5.y; a[6] = q5.z; a[7] = q5.w;
  }
  uint32_t dig[16];
  if (p.digests) {
    /* the caller hashed R||A||M (a message the device path's 32-bit sizes
       cannot carry, fd_ed25519_hip_verify_digests_dev): a uniform branch,
       the whole launch takes one side */
    const uint4* dg = reinterpret_cast<const uint4*>(p.digests + 64 * i);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint4 v = dg[q];
      dig[4 * q] = v.x; dig[4 * q + 1] = v.y; dig[4 * q + 2] = v.z; dig[4 * q + 3] = v.w;
    }
  } else {
    const uintptr_t mp = reinterpret_cast<uintptr_t>(p.msgs + p.msg_off[i]);
    sha_msg_src m;
    m.base = reinterpret_cast<const uint32_t*>(mp & ~(uintptr_t)3);
    m.shift = (uint32_t)(mp & 3);
    m.sz = p.msg_sz[i];
    sha512_ram(dig, r, a, m);
  }
  hash_finish(p, j, dig, S);
}

__global__ void __launch_bounds__(256, FD_ED25519_HASH_WAVES_PER_SIMD)
fd_ed25519_hash_kernel(fd_ed25519_verify_params_t p) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= p.n) return;
  hash_one(p, p.perm ? (uint64_t)p.perm[t] : t);
}

/* One lane per point (2n lanes: A, then R): decompression with the
   reference's acceptance rules (fd_ed25519_point_frombytes_2x) and the
   small-order test (fd_ed25519_affine_is_small_order). */
FD_DEV void decode_one(const fd_ed25519_verify_params_t& p, int which /* 0: A (public key), 1: R */, uint64_t j) {
  const uint64_t i = p.base + j;
  uint32_t s[8];
  {
    const uint4* src = which ? reinterpret_cast<const uint4*>(p.sigs + 64 * i)
                             : reinterpret_cast<const uint4*>(p.pubs + 32 * i);
    const uint4 q0 = src[0], q1 = src[1];
    s[0] = q0.x; s[1] = q0.y; s[2] = q0.z; s[3] = q0.w; s[4] = q1.x; s[5] = q1.y; s[6] = q1.z; s[7] = q1.w;
  }
  decoded_pt d;
  ge_decode(d, s, !p.codes_portable);
  int32_t* dst = p.pts + (uint64_t)which * 20 * p.cap + j;
#pragma unroll
  for (int l = 0; l < 10; l++) {
    dst[(uint64_t)l * p.cap] = d.x.v[l];
    dst[(uint64_t)(10 + l) * p.cap] = d.y.v[l];
  }
  p.pflag[(uint64_t)which * p.cap + j] = (uint8_t)((d.fail ? FD_PF_FAIL : 0u) | (d.small ? FD_PF_SMALL : 0u));
}

__global__ void __launch_bounds__(256, FD_ED25519_DECODE_WAVES_PER_SIMD)
fd_ed25519_decode_kernel(fd_ed25519_verify_params_t p) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 2 * p.n) return;
  const int which = t >= p.n;
  decode_one(p, which, which ? t - p.n : t);
}

FD_DEV void load_fe(fe& x, const int32_t* src, uint64_t cap) {
#pragma unroll
  for (int l = 0; l < 10; l++) x.v[l] = src[(uint64_t)l * cap];
}

FD_DEV void load_pt(fe& x, fe& y, const fd_ed25519_verify_params_t& p, int which, uint64_t j) {
  const int32_t* src = p.pts + (uint64_t)which * 20 * p.cap + j;
  load_fe(x, src, p.cap);
  load_fe(y, src + 10 * p.cap, p.cap);
}

/* The reference's checks before the group equation, in its order
   (fd_ed25519_user.c:134-229): S < L; A and R decode (an undecodable A is
   ERR_SIG with AVX-512 codes, ERR_PUBKEY with portable ones; R: ERR_SIG);
   A small order (ERR_PUBKEY); R small order (ERR_SIG).  1 = pending. */
#define FD_PENDING 1
FD_DEV int precheck(const fd_ed25519_verify_params_t& p, uint64_t j) {
  const uint32_t s_ok = p.sflag[j];
  const uint32_t af = p.pflag[j], rf = p.pflag[p.cap + j];
  if (!s_ok) return FD_ED25519_ERR_SIG;
  if (af & FD_PF_FAIL) return p.codes_portable ? FD_ED25519_ERR_PUBKEY : FD_ED25519_ERR_SIG;
  if (rf & FD_PF_FAIL) return FD_ED25519_ERR_SIG;
  if (af & FD_PF_SMALL) return FD_ED25519_ERR_PUBKEY;
  if (rf & FD_PF_SMALL) return FD_ED25519_ERR_SIG;
  return FD_PENDING;
}

/* [0..8](sign P) in cached form for the affine point (x, y), into a lane's
   9-entry table; NT: the entries hold -2dT (ge_add<true>) */
template <bool NT>
FD_DEV void table_store(int4* tab, int e, ge_cached c) {
  if (NT) fe_neg(c.T2d, c.T2d);
  atab_store(tab, e, c);
}

/* The cached identity (Y+X = Y-X = 1, 2Z = 2, T = 0) that a zero digit
   reads from the half-size form's [1..8] lane tables: one 160-byte
   entry shared by every lane, L2-resident. */
__device__ const int4 fd_ident_cached[10] = {{1, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 0}, {0, 0, 0, 0},
                                             {2, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};

/* the entry for digit e: [|e|] of the lane's table (IDENT: [1..8] at 0..7,
   the shared identity for e == 0) */
template <bool IDENT>
FD_DEV const int4* tab_entry(const int4* tab, int e) {
  const int a = e < 0 ? -e : e;
  if (IDENT) return a == 0 ? fd_ident_cached : tab + (a - 1) * 10;
  return tab + a * 10;
}

/* IDENT: [1..8] at entries 0..7, no identity entry */
template <bool NT, bool IDENT = false>
FD_DEV void table_build(int4* tab, const fe& x, const fe& y, bool negate) {
  ge_p3 P0;
  fe xn;
  fe_neg(xn, x);
  fe_select(P0.X, x, xn, negate);
  P0.Y = y;
  fe_1(P0.Z);
  fe_mul(P0.T, P0.X, y);
  ge_cached c1, c;
  if (!IDENT) {
    c.YplusX = P0.Z; c.YminusX = P0.Z; fe_add(c.Z2, P0.Z, P0.Z); fe_0(c.T2d);  /* identity */
    atab_store(tab, 0, c);
  }
  ge_p3_to_cached(c1, P0);
  table_store<NT>(tab, IDENT ? 0 : 1, c1);
  /* P0 is affine: the multiples by mixed additions (3 multiplications) */
  ge_precomp pre;
  pre.yplusx = c1.YplusX; pre.yminusx = c1.YminusX; pre.xy2d = c1.T2d;
  ge_p3 cur = P0;
  ge_p1p1 sum;
#pragma clang loop unroll(disable)
  for (int e = 2; e <= 8; e++) {
    ge_madd(sum, cur, pre);
    ge_p1p1_to_p3_uxyt(cur, sum);   /* Z centered: the next mixed addition doubles it */
    ge_p3_to_cached<true>(c, cur);
    table_store<NT>(tab, IDENT ? e - 1 : e, c);
  }
}

FD_DEV void table_add(ge_p1p1& Rt, const ge_p3& P, const int4* tab, int e) {
  ge_cached c;
  atab_load(c, tab, e < 0 ? -e : e);
  ge_cached_cneg(c, e < 0);
  ge_add(Rt, P, c);
}

FD_DEV void btab_add(ge_p1p1& Rt, const ge_p3& P, ge_precomp& b, int f) {
  ge_precomp_cneg(b, f < 0);
  ge_madd(Rt, P, b);
}

/* ------------------------------------------------------------------------
   The invariant the half-size verdict rests on, re-checked with integer
   arithmetic only.  fd_half_scalars (fd25519_half.h) finds (c, d) with a
   Euclid whose quotients come from exact-integer double-precision steps; a
   wrong quotient there, or a compiler change to that sequence, must never
   reach the group equation.  So every pair is checked before use:

       d odd,  0 <= c < 2^131,  |d| < 2^dbits,  c == d k (mod 8L)

   the congruence as X = |d| k + (d < 0 ? c : 8L - c) == 0 (mod 8L), i.e.
   X == 0 (mod 8) and X / 8 == 0 (mod L) (sc_reduce512: X < 2^406).  A pair
   that fails goes to the full-length form, whose verdict is the
   reference's equation itself (fd_ed25519_user.c:209-226). */

FD_DEV bool half_pair_ok(const uint32_t (&k)[8], const uint32_t (&c)[FD_HALF_TW], const uint32_t (&dm)[FD_HALF_TW],
                         int dneg, int dbits) {
  uint32_t x[16];
#pragma unroll
  for (int w = 0; w < 16; w++) x[w] = 0u;
#pragma unroll
  for (int a = 0; a < FD_HALF_TW; a++) {   /* |d| k: 160 x 256 bits */
    uint64_t carry = 0;
#pragma unroll
    for (int b = 0; b < 8; b++) {
      const uint64_t t = (uint64_t)dm[a] * k[b] + x[a + b] + carry;
      x[a + b] = (uint32_t)t;
      carry = t >> 32;
    }
    x[a + 8] = (uint32_t)carry;
  }
  const uint32_t n8l[8] = FD_HALF_N8L;
  uint32_t add[8];
  {
    uint64_t br = 0;
#pragma unroll
    for (int w = 0; w < 8; w++) {
      const uint32_t cv = w < FD_HALF_TW ? c[w] : 0u;
      const uint64_t t = (uint64_t)n8l[w] - cv - br;   /* 8L - c: c < 2^160 < 8L */
      br = (t >> 63) & 1u;
      add[w] = dneg ? cv : (uint32_t)t;
    }
  }
  {
    uint64_t carry = 0;
#pragma unroll
    for (int w = 0; w < 15; w++) {
      const uint64_t t = (uint64_t)x[w] + (w < 8 ? add[w] : 0u) + carry;
      x[w] = (uint32_t)t;
      carry = t >> 32;
    }
  }
  const uint32_t low = x[0] & 7u;
#pragma unroll
  for (int w = 0; w < 15; w++) x[w] = __builtin_amdgcn_alignbit(x[w + 1], x[w], 3);
  x[15] >>= 3;
  uint32_t r[8];
  sc_reduce512(r, x);
  uint32_t nz = low;
#pragma unroll
  for (int w = 0; w < 8; w++) nz |= r[w];
  return nz == 0u && (dm[0] & 1u) && fd_half_bitlen<FD_HALF_TW>(c) <= FD_HALF_BITS &&
         fd_half_bitlen<FD_HALF_TW>(dm) <= dbits;
}

/* Compile-time fault injection (-DFD_ED25519_HALF_FAULT=1, a test build
   only: libfd_ed25519_hip_faultinj.so): a bit of c flipped for 1/8 of the
   items and a bit of |d| above bit 0 for another 1/8, after the search and
   before the check, so that the check -- not luck -- keeps the verdicts
   bit-exact (tests/test_gpu_halfcheck.py). */
#ifndef FD_ED25519_AB_LDS_BASE
#define FD_ED25519_AB_LDS_BASE 0
#endif
#ifndef FD_ED25519_HALF_FAULT
#define FD_ED25519_HALF_FAULT 0
#endif

FD_DEV int half_scalars_checked(const uint32_t (&k)[8], uint32_t (&c)[FD_HALF_TW], uint32_t (&dm)[FD_HALF_TW],
                                int* dneg, int dbits, uint64_t tag) {
  const int found = fd_half_scalars(k, c, dm, dneg, dbits);
#if FD_ED25519_HALF_FAULT
  {
    const uint32_t h = (uint32_t)(tag * 0x9E3779B97F4A7C15ull >> 32);
    const uint32_t sel = h >> 29, w = (h >> 8) & 3u, b = h & 31u;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      if (sel == 1u && i == (int)w) c[i] ^= 1u << b;
      if (sel == 2u && i == (int)w) dm[i] ^= (i == 0 && b == 0) ? 2u : (1u << b);
    }
  }
#else
  (void)tag;
#endif
  return found && half_pair_ok(k, c, dm, *dneg, dbits);
}

/* ------------------------------------------------------------------------
   scalar: the half-size scalars (fd25519_half.h) of every signature, one
   lane per signature, before the points are decoded:

       c == d k (mod 8L), d odd, 0 <= c < 2^131, |d| < 2^half_dbits,
       s' = d S mod L = s_lo + 2^144 s_hi

   written to hs[19][cap] (c, |d|, s_lo: 5 words each, s_hi: 4) with d's
   sign in hflag.  Signatures whose k has no such pair (~1e-6 of random k
   at 151 bits, ~0.16% at 131) are flagged and queued on fix_list for the
   full-length form. */

FD_DEV void scalar_one(const fd_ed25519_verify_params_t& p, uint64_t j) {
  const uint64_t i = p.base + j;
  uint32_t k[8], S[8];
#pragma unroll
  for (int w = 0; w < 8; w++) k[w] = p.k[(uint64_t)w * p.cap + j];
  {
    const uint4* sg = reinterpret_cast<const uint4*>(p.sigs + 64 * i);
    const uint4 q2 = sg[2], q3 = sg[3];
    S[0] = q2.x; S[1] = q2.y; S[2] = q2.z; S[3] = q2.w; S[4] = q3.x; S[5] = q3.y; S[6] = q3.z; S[7] = q3.w;
  }
  uint32_t cw[FD_HALF_TW], dm[FD_HALF_TW];
  int dneg = 0;
  int ok = half_scalars_checked(k, cw, dm, &dneg, p.half_dbits, j);
  if (!p.sflag[j]) ok = 1;   /* S >= L: decided without the equation, any scalars do */

  /* s' = d S mod L */
  uint32_t sp[8];
  {
    uint32_t prod[16];
#pragma unroll
    for (int w = 0; w < 16; w++) prod[w] = 0u;
#pragma unroll
    for (int a = 0; a < FD_HALF_TW; a++) {
      uint64_t carry = 0;
#pragma unroll
      for (int b = 0; b < 8; b++) {
        const uint64_t t = (uint64_t)dm[a] * S[b] + prod[a + b] + carry;
        prod[a + b] = (uint32_t)t;
        carry = t >> 32;
      }
      prod[a + 8] = (uint32_t)carry;
    }
    sc_reduce512(sp, prod);
    if (dneg) {   /* L - sp (mod L) */
      const uint32_t l[8] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu, 0u, 0u, 0u, 0x10000000u};
      uint32_t nz = 0;
#pragma unroll
      for (int w = 0; w < 8; w++) nz |= sp[w];
      uint64_t br = 0;
#pragma unroll
      for (int w = 0; w < 8; w++) {
        const uint64_t t = (uint64_t)l[w] - sp[w] - br;
        br = (t >> 63) & 1u;
        sp[w] = nz ? (uint32_t)t : 0u;
      }
    }
  }
  uint32_t* hs = p.hs + j;
  const uint64_t c = p.cap;
  static_assert(FD_ED25519_BTABW_SHIFT == 144, "s_lo is words 0..3 and the low half of word 4");
#pragma unroll
  for (int w = 0; w < 5; w++) {
    hs[(uint64_t)w * c] = cw[w];
    hs[(uint64_t)(5 + w) * c] = dm[w];
    hs[(uint64_t)(10 + w) * c] = w < 4 ? sp[w] : (sp[4] & 0xffffu);            /* bits 0..143   */
  }
#pragma unroll
  for (int w = 0; w < 4; w++)                                                  /* bits 144..252 */
    hs[(uint64_t)(15 + w) * c] = __builtin_amdgcn_alignbit(w + 5 < 8 ? sp[w + 5] : 0u, sp[w + 4], 16);
  p.hflag[j] = (uint8_t)((dneg ? FD_HF_DNEG : 0u) | (ok ? 0u : FD_HF_FULL));
  if (!ok && !p.small) {   /* small chunks: the dsm scan finds them by hflag */
    const uint32_t slot = atomicAdd(p.fix_cnt, 1u);
    p.fix_list[slot] = (uint32_t)j;
  }
}

__global__ void __launch_bounds__(256, FD_ED25519_SCALAR_WAVES_PER_SIMD)
fd_ed25519_scalar_kernel(fd_ed25519_verify_params_t p) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= p.n) return;
  scalar_one(p, j);
}

/* Small chunks (the latency regime): hash, scalar and decode in one launch,
   specialised by wave so no wave diverges: per 64 signatures, wave 0 hashes
   and then finds the half-size scalars, waves 1 and 2 decode A and R, all
   three at once on different SIMDs (the path is the longer of the two
   chains instead of their sum, and two launches and the counting sort are
   gone). */
__global__ void __launch_bounds__(192) fd_ed25519_prep_kernel(fd_ed25519_verify_params_t p) {
  const uint32_t w = threadIdx.x >> 6;
  const uint64_t t = (uint64_t)blockIdx.x * 64u + (threadIdx.x & 63u);
  if (t >= p.n) return;
  if (w == 0) {
    const uint64_t j = p.perm ? (uint64_t)p.perm[t] : t;   /* hash order (length-sorted) */
    hash_one(p, j);
    scalar_one(p, j);
  } else {
    decode_one(p, (int)w - 1, t);
  }
}

/* x << SH for a 160-bit value known to stay below 2^160 */
template <int SH>
FD_DEV void shl160(uint32_t (&out)[5], const uint32_t (&x)[5]) {
  constexpr int W = SH / 32, B = SH % 32;
#pragma unroll
  for (int i = 4; i >= 0; i--) {
    const uint32_t hi = i - W >= 0 ? x[i - W] : 0u;
    const uint32_t lo = i - W - 1 >= 0 ? x[i - W - 1] : 0u;
    out[i] = B ? __builtin_amdgcn_alignbit(hi, lo, 32 - B) : hi;
  }
}

/* x << s for 0 < s < 32 (wave-uniform s), the value staying below 2^160 */
FD_DEV void shl160v(uint32_t (&out)[5], const uint32_t (&x)[5], int s) {
#pragma unroll
  for (int i = 4; i > 0; i--) out[i] = __builtin_amdgcn_alignbit(x[i], x[i - 1], 32 - s);
  out[0] = x[0] << s;
}

/* signed recoding of a 160-bit value in radix 2^BITS, digits packed as
   BITS-bit two's complement (the carry out of the top digit is dropped:
   the caller reads the top digit unsigned where it may reach 2^(BITS-1)) */
template <int BITS>
FD_DEV void recode160(uint32_t (&out)[5], const uint32_t (&x)[5]) {
  constexpr uint32_t M = (1u << BITS) - 1u;
  constexpr int PER = 32 / BITS;
  int carry = 0;
#pragma unroll
  for (int w = 0; w < 5; w++) {
    uint32_t packed = 0;
#pragma unroll
    for (int q = 0; q < PER; q++) {
      int e = (int)((x[w] >> (BITS * q)) & M) + carry;
      carry = (e + (1 << (BITS - 1))) >> BITS;
      e -= carry << BITS;
      packed |= ((uint32_t)e & M) << (BITS * q);
    }
    out[w] = packed;
  }
}

template <int BITS>
FD_DEV uint32_t pop160u(uint32_t (&d)[5]) {
  const uint32_t v = d[4] >> (32 - BITS);
#pragma unroll
  for (int w = 4; w > 0; w--) d[w] = __builtin_amdgcn_alignbit(d[w], d[w - 1], 32 - BITS);
  d[0] <<= BITS;
  return v;
}

template <int BITS>
FD_DEV int pop160(uint32_t (&d)[5]) {
  const int v = ((int32_t)d[4]) >> (32 - BITS);
#pragma unroll
  for (int w = 4; w > 0; w--) d[w] = __builtin_amdgcn_alignbit(d[w], d[w - 1], 32 - BITS);
  d[0] <<= BITS;
  return v;
}

FD_DEV void load_hs(uint32_t (&x)[5], const fd_ed25519_verify_params_t& p, int row, int words, uint64_t j) {
#pragma unroll
  for (int w = 0; w < 5; w++) x[w] = w < words ? p.hs[(uint64_t)(row + w) * p.cap + j] : 0u;
}

/* base digits of s_lo and s_hi in radix 2^BW: digit m sits at bits BW m,
   i.e. window (BW/4) m, top-aligned in 160 bits for pop160u.  BW = 24 (the
   wide tables: s_lo's 6 and s_hi's 5 digits at windows 30, 24, .., 0 and
   24, .., 0) or 16 (the compact tables, FD_ED25519_HIP_FLAG_COMPACT_TABLES:
   9 and 7 digits at windows 32, 28, .., 0 and 24, .., 0). */
template <int BW>
struct fd_bw {
  static constexpr int STEP   = BW / 4;
  static constexpr int LO_N   = FD_ED25519_BTABW_SHIFT / BW;
  static constexpr int HI_N   = (253 - FD_ED25519_BTABW_SHIFT + BW - 1) / BW;
  static constexpr int LO_SHL = 160 - LO_N * BW;
  static constexpr int HI_SHL = 160 - HI_N * BW;
  static_assert(BW % 4 == 0, "base digits start at window boundaries");
  static_assert(LO_N * BW == FD_ED25519_BTABW_SHIFT, "s_lo digits cover bits 0..SHIFT-1");
  static_assert(HI_N * BW >= 253 - FD_ED25519_BTABW_SHIFT, "s_hi digits cover s' >> SHIFT");
  static_assert(STEP * (LO_N - 1) <= 32, "every base digit falls within the 33 windows");
  FD_DEV static bool lo_at(int it) { return it <= STEP * (LO_N - 1) && it % STEP == 0; }
  FD_DEV static bool hi_at(int it) { return it <= STEP * (HI_N - 1) && it % STEP == 0; }
};

/* ------------------------------------------------------------------------
   dsm: the group equation with half-size scalars.

   E = [S]B - R - [k]A == 0 is tested as [d]E == 0, i.e.

       [c](-A) + [|d|](-sign(d) R) + [s_lo]B + [s_hi]B' == 0,   B' = [2^144]B

   exactly equivalent (fd25519_half.h: the group has order 8L and [d] is
   invertible on it).  A four-scalar Straus loop over W signed 4-bit
   windows, W = 33 unless a lane of the wave has |d| >= 2^131 (~0.16% of
   signatures; then up to 38, the same W for the whole wave, the other
   lanes' top digits being 0): 4(W-1) = 128 doublings (against 252 for the
   reference's double-scalar form), W additions from each lane's
   [1..8](-A) and [1..8](-+R) tables (a zero digit adds the shared identity entry)
   (HBM, lane-contiguous 160-byte entries) and 6 + 5 mixed additions from
   the two unsigned radix-2^24 base tables [0..2^24)B and [0..2^24)B'
   (2 GiB each, HBM) -- or, with BW = 16, 9 + 7 from the compact
   [0..2^16) tables (8 MiB each).  Every table entry is loaded
   one step ahead of its use: the -A entry before the window's doublings,
   the R entry before the -A addition, the base entries before the R
   addition.  The result is compared with the identity (X == 0, Y == Z). */

template <int BW>
FD_DEV int dsm_half_one(const fd_ed25519_verify_params_t& p, uint64_t j, int4* tabA, int4* tabR) {
  int code = precheck(p, j);
  const uint32_t hf = p.hflag[j];

  /* lane tables: [1..8](-A) and [1..8](-sign(d) R) */
  {
    fe x, y;
    load_pt(x, y, p, 0, j);
    table_build<true, true>(tabA, x, y, true);
    load_pt(x, y, p, 1, j);
    table_build<true, true>(tabR, x, y, !(hf & FD_HF_DNEG));
  }
  /* digits, most significant first, top-aligned in 160 bits: c, |d| in
     radix 16 (W signed digits, the top one in [0,8]), s_lo, s_hi in
     radix 2^24 (6 and 5 unsigned digits: no recoding, no negation) */
  uint32_t cd[5], dd[5], ld[5], hd[5];
  int W = 33;
  {
    uint32_t x[5], t[5];
    load_hs(x, p, 5, 5, j);
    /* windows this lane needs: |d| < 2^(4W-1); the wave takes the max */
    const int wl = (fd_half_bitlen<5>(x) + 4) >> 2;
#pragma unroll
    for (int w = 34; w <= (FD_HALF_DBITS_MAX + 4) / 4; w++) W += __ballot(wl >= w) != 0ull;
    const int sh = 160 - 4 * W;
    shl160v(t, x, sh); recode160<4>(dd, t);
    load_hs(x, p, 0, 5, j);  shl160v(t, x, sh); recode160<4>(cd, t);
    load_hs(x, p, 10, 5, j); shl160<fd_bw<BW>::LO_SHL>(ld, x);
    load_hs(x, p, 15, 4, j); shl160<fd_bw<BW>::HI_SHL>(hd, x);
  }
  const int4* g_btab = reinterpret_cast<const int4*>(p.btab_lo);
  const int4* g_btab2 = reinterpret_cast<const int4*>(p.btab_hi);

  ge_p3 P;
  ge_p3_0(P);
  ge_p1p1 Rt;
  ge_p2 Q;
#pragma clang loop unroll(disable)
  for (int it = W - 1; it >= 0; it--) {
    int ea = pop160<4>(cd), er = pop160<4>(dd);
    if (it == W - 1) { ea &= 15; er &= 15; }   /* top digits in [0,8] */
    ge_cached ca, cr;
    const bool blo = fd_bw<BW>::lo_at(it), bhi = fd_bw<BW>::hi_at(it);
    ge_precomp b1, b2;
    atab_load(ca, tab_entry<true>(tabA, ea), 0);
    if (it != W - 1) {
#pragma clang loop unroll(disable)
      for (int dbl = 0; dbl < 4; dbl++) {
        ge_p2_dbl(Rt, Q);
        if (dbl < 3) ge_p1p1_to_p2(Q, Rt);
      }
      ge_p1p1_to_p3_u(P, Rt);
    }
    atab_load(cr, tab_entry<true>(tabR, er), 0);
    ge_cached_cneg(ca, ea < 0);
    ge_add<true>(Rt, P, ca);
    ge_p1p1_to_p3_u(P, Rt);
    if (blo) btab16_load(b1, g_btab, (int)pop160u<BW>(ld));
    if (bhi) btab16_load(b2, g_btab2, (int)pop160u<BW>(hd));
    ge_cached_cneg(cr, er < 0);
    ge_add<true>(Rt, P, cr);
    if (blo) {
      ge_p1p1_to_p3_uxyt(P, Rt);
      ge_madd(Rt, P, b1);
    }
    if (bhi) {
      ge_p1p1_to_p3_uxyt(P, Rt);
      ge_madd(Rt, P, b2);
    }
    ge_p1p1_to_p2(Q, Rt);
  }
  /* identity: X == 0 and Y == Z */
  fe t;
  fe_sub(t, Q.Y, Q.Z);
  const bool ident = fe_iszero(Q.X) && fe_iszero(t);
  if (code == FD_PENDING) code = ident ? FD_ED25519_SUCCESS : FD_ED25519_ERR_MSG;
  return code;
}

#if FD_ED25519_AB_LDS_BASE
/* A/B build only ("tables staged in LDS"): the base
   tables in LDS.  2 x 256 entries x 128 B = 64 KiB per block, i.e. radix
   2^8: s' = s_lo + 2^144 s_hi is re-split at 2^136 into 17 + 15 unsigned
   8-bit digits at windows 32, 30, .., 0 and 28, .., 0 -- 32 mixed
   additions from LDS against 11 from the 2 x 2 GiB HBM tables.  Same
   lane tables, doublings and identity test as dsm_half_one. */
FD_DEV int dsm_half_one_lds(const fd_ed25519_verify_params_t& p, uint64_t j, int4* tabA, int4* tabR,
                            const int4* s_lo8, const int4* s_hi8) {
  int code = precheck(p, j);
  const uint32_t hf = p.hflag[j];
  {
    fe x, y;
    load_pt(x, y, p, 0, j);
    table_build<true, true>(tabA, x, y, true);
    load_pt(x, y, p, 1, j);
    table_build<true, true>(tabR, x, y, !(hf & FD_HF_DNEG));
  }
  uint32_t cd[5], dd[5], ld[5], hd[5];
  int W = 33;
  {
    uint32_t x[5], t[5], sl[5], sh[5];
    load_hs(x, p, 5, 5, j);
    const int wl = (fd_half_bitlen<5>(x) + 4) >> 2;
#pragma unroll
    for (int w = 34; w <= (FD_HALF_DBITS_MAX + 4) / 4; w++) W += __ballot(wl >= w) != 0ull;
    const int shv = 160 - 4 * W;
    shl160v(t, x, shv); recode160<4>(dd, t);
    load_hs(x, p, 0, 5, j);  shl160v(t, x, shv); recode160<4>(cd, t);
    load_hs(sl, p, 10, 5, j);
    load_hs(sh, p, 15, 4, j);
    static_assert(FD_ED25519_BTABW_SHIFT - FD_ED25519_BTAB8_SHIFT == 8, "re-split of s' by one byte");
    uint32_t lo[5] = {sl[0], sl[1], sl[2], sl[3], sl[4] & 0xffu};
    uint32_t hi[5] = {(sl[4] >> 8) | (sh[0] << 8), (sh[0] >> 24) | (sh[1] << 8), (sh[1] >> 24) | (sh[2] << 8),
                      (sh[2] >> 24) | (sh[3] << 8), sh[3] >> 24};
    shl160<160 - 17 * 8>(ld, lo);
    shl160<160 - 15 * 8>(hd, hi);
  }
  ge_p3 P;
  ge_p3_0(P);
  ge_p1p1 Rt;
  ge_p2 Q;
#pragma clang loop unroll(disable)
  for (int it = W - 1; it >= 0; it--) {
    int ea = pop160<4>(cd), er = pop160<4>(dd);
    if (it == W - 1) { ea &= 15; er &= 15; }
    ge_cached ca, cr;
    const bool blo = it <= 32 && !(it & 1), bhi = it <= 28 && !(it & 1);
    ge_precomp b1, b2;
    atab_load(ca, tab_entry<true>(tabA, ea), 0);
    if (it != W - 1) {
#pragma clang loop unroll(disable)
      for (int dbl = 0; dbl < 4; dbl++) {
        ge_p2_dbl(Rt, Q);
        if (dbl < 3) ge_p1p1_to_p2(Q, Rt);
      }
      ge_p1p1_to_p3_u(P, Rt);
    }
    atab_load(cr, tab_entry<true>(tabR, er), 0);
    ge_cached_cneg(ca, ea < 0);
    ge_add<true>(Rt, P, ca);
    ge_p1p1_to_p3_u(P, Rt);
    if (blo) btab16_load(b1, s_lo8, (int)pop160u<8>(ld));
    if (bhi) btab16_load(b2, s_hi8, (int)pop160u<8>(hd));
    ge_cached_cneg(cr, er < 0);
    ge_add<true>(Rt, P, cr);
    if (blo) {
      ge_p1p1_to_p3_uxyt(P, Rt);
      ge_madd(Rt, P, b1);
    }
    if (bhi) {
      ge_p1p1_to_p3_uxyt(P, Rt);
      ge_madd(Rt, P, b2);
    }
    ge_p1p1_to_p2(Q, Rt);
  }
  fe t;
  fe_sub(t, Q.Y, Q.Z);
  const bool ident = fe_iszero(Q.X) && fe_iszero(t);
  if (code == FD_PENDING) code = ident ? FD_ED25519_SUCCESS : FD_ED25519_ERR_MSG;
  return code;
}
#endif

/* The reference's own form, for the few signatures whose k has no
   half-size pair: R' = [k](-A) + [S]B with k in radix 16 (252 doublings,
   64 additions of [0..8](-A)) and S in radix 2^16 (16 mixed additions),
   then R' == R projectively (fd_ed25519_point_eq_z1: X' == x_R Z',
   Y' == y_R Z'). */
FD_DEV int dsm_full_core(const fd_ed25519_verify_params_t& p, uint64_t j, int4* tabA, int code, const fe& ax,
                         const fe& ay, const fe& rx, const fe& ry) {
  const uint64_t i = p.base + j;
  table_build<false>(tabA, ax, ay, true);
  uint32_t kd[8], sd[8];
  {
    uint32_t k[8], S[8];
#pragma unroll
    for (int w = 0; w < 8; w++) k[w] = p.k[(uint64_t)w * p.cap + j];
    const uint4* sg = reinterpret_cast<const uint4*>(p.sigs + 64 * i);
    const uint4 q2 = sg[2], q3 = sg[3];
    S[0] = q2.x; S[1] = q2.y; S[2] = q2.z; S[3] = q2.w; S[4] = q3.x; S[5] = q3.y; S[6] = q3.z; S[7] = q3.w;
    recode_radix16(kd, k);
    recode_radix65536(sd, S);
  }
  const int4* g_btab = reinterpret_cast<const int4*>(p.btab16);
  ge_p3 P;
  ge_p3_0(P);
  ge_p1p1 Rt;
  ge_p2 Q;
#pragma clang loop unroll(disable)
  for (int it = 63; it >= 0; it--) {
    const bool badd = (it & 3) == 0;
    int f = 0;
    ge_precomp b;
    if (badd) {
      f = pop_digit<16>(sd);
      btab16_load(b, g_btab, f < 0 ? -f : f);
    }
    if (it != 63) {
#pragma clang loop unroll(disable)
      for (int dbl = 0; dbl < 4; dbl++) {
        ge_p2_dbl(Rt, Q);
        if (dbl < 3) ge_p1p1_to_p2(Q, Rt);
      }
      ge_p1p1_to_p3_u(P, Rt);
    }
    table_add(Rt, P, tabA, pop_digit<4>(kd));
    if (badd) {
      ge_p1p1_to_p3_uxyt(P, Rt);
      btab_add(Rt, P, b, f);
    }
    ge_p1p1_to_p2(Q, Rt);
  }
  fe t1, t2;
  fe_mul(t1, rx, Q.Z);
  fe_sub(t1, t1, Q.X);
  fe_mul(t2, ry, Q.Z);
  fe_sub(t2, t2, Q.Y);
  const bool eq = fe_iszero(t1) && fe_iszero(t2);
  if (code != FD_PENDING) return code;
  return eq ? FD_ED25519_SUCCESS : FD_ED25519_ERR_MSG;
}

FD_DEV int dsm_full_one(const fd_ed25519_verify_params_t& p, uint64_t j, int4* tabA) {
  fe ax, ay, rx, ry;
  load_pt(ax, ay, p, 0, j);
  load_pt(rx, ry, p, 1, j);
  return dsm_full_core(p, j, tabA, precheck(p, j), ax, ay, rx, ry);
}

/* Persistent over fix_cnt (rounded up to whole waves) + n items, handed
   out 64 at a time (one atomic per wave): the full-length items first, in
   waves of their own (a wave mixing both forms would run both), then the
   chunk's signatures (those queued as full-length skipped), so the ~2x
   longer full-length work is spread over the grid instead of forming a
   tail. */
template <int BW>
__global__ void __launch_bounds__(FD_ED25519_VERIFY_BLOCK, FD_ED25519_DSM_WAVES_PER_SIMD)
fd_ed25519_dsm_kernel(fd_ed25519_verify_params_t p) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  int4* tabA = reinterpret_cast<int4*>(static_cast<char*>(p.atab) + wave * FD_ED25519_ATAB_BYTES_PER_WAVE) +
               lane * (2 * FD_ED25519_ATAB_STRIDE * 10);
  int4* tabR = tabA + FD_ED25519_ATAB_STRIDE * 10;   /* the full-length form uses tabA's 9 entries, into tabR's space */
#if FD_ED25519_AB_LDS_BASE
  __shared__ int4 s_b8[2 * 256 * (FD_ED25519_BTAB16_STRIDE / 4)];
  {
    const int4* g_lo = reinterpret_cast<const int4*>(p.btab8_lo);
    const int4* g_hi = reinterpret_cast<const int4*>(p.btab8_hi);
    constexpr int N = 256 * (FD_ED25519_BTAB16_STRIDE / 4);
    for (int i = threadIdx.x; i < N; i += blockDim.x) { s_b8[i] = g_lo[i]; s_b8[N + i] = g_hi[i]; }
    __syncthreads();
  }
#endif
  if (p.small) {
    /* after dsm4: the full-length items only, found by their flag (a
       static stride: the work counter is not reset for small chunks) */
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < p.n; t += stride)
      if (p.hflag[t] & FD_HF_FULL) p.out[p.base + t] = (int8_t)dsm_full_one(p, t, tabA);
    return;
  }
  const uint64_t nfix = *p.fix_cnt;
  const uint64_t head = (nfix + 63u) & ~(uint64_t)63u;
  const uint64_t total = head + p.n;
  for (;;) {
    uint32_t b = 0u;
    if (lane == 0u) b = atomicAdd(p.work_ctr, 64u);
    b = (uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl((int)b, 0));
    if ((uint64_t)b >= total) break;
    const uint64_t t = (uint64_t)b + lane;
    if (t < nfix) {
      const uint64_t j = p.fix_list[t];
      p.out[p.base + j] = (int8_t)dsm_full_one(p, j, tabA);
    } else if (t >= head && t < total) {
      const uint64_t j = t - head;
#if FD_ED25519_AB_LDS_BASE
      if (!(p.hflag[j] & FD_HF_FULL))
        p.out[p.base + j] = (int8_t)dsm_half_one_lds(p, j, tabA, tabR, s_b8, s_b8 + 256 * (FD_ED25519_BTAB16_STRIDE / 4));
#else
      if (!(p.hflag[j] & FD_HF_FULL)) p.out[p.base + j] = (int8_t)dsm_half_one<BW>(p, j, tabA, tabR);
#endif
    }
  }
}

/* ------------------------------------------------------------------------
   dsm4: the same half-size group equation with a quad of lanes per
   signature (fd25519_ge4.h), for small chunks: the verify tile's latency
   mode, where a one-lane-per-signature launch leaves the chip idle and the
   batch waits for one lane's serial chain.  Same digits, tables (in qc
   layout: each lane stores its coordinate of every entry, 48-byte entries,
   FD_ED25519_QUAD_LANE_BYTES per lane) and addition order as
   dsm_half_one, each group operation in one multiplication's time.  A
   negative table digit adds -Q as -((-P) + Q) (negating P costs no DPP,
   swapping Q's coordinates would).  Full-length items are left to the dsm
   kernel (launched after this one in fix-only mode). */

FD_DEV void tab4_store(int4* tab, int e, const fe& c) {
  int4* d = tab + 3 * e;
  d[0] = make_int4(c.v[0], c.v[1], c.v[2], c.v[3]);
  d[1] = make_int4(c.v[4], c.v[5], c.v[6], c.v[7]);
  d[2] = make_int4(c.v[8], c.v[9], 0, 0);
}

FD_DEV void tab4_load(fe& c, const int4* tab, int e) {
  const int4* s = tab + 3 * e;
  const int4 a = s[0], b = s[1], d = s[2];
  c.v[0] = a.x; c.v[1] = a.y; c.v[2] = a.z; c.v[3] = a.w;
  c.v[4] = b.x; c.v[5] = b.y; c.v[6] = b.z; c.v[7] = b.w;
  c.v[8] = d.x; c.v[9] = d.y;
}

/* this lane's coordinate of base entry e as qc: (y-x, y+x, 2dxy, 2) */
FD_DEV void btab4_load(fe& c, const int32_t* g_btab, int e, const qmask_t& m) {
  const int off = m.l0 ? 10 : (m.l1 ? 0 : 20);
  const int2* s = reinterpret_cast<const int2*>(g_btab + (size_t)e * FD_ED25519_BTAB16_STRIDE + off);
#pragma unroll
  for (int q = 0; q < 5; q++) {
    const int2 x = s[q];
    c.v[2 * q] = x.x;
    c.v[2 * q + 1] = x.y;
  }
#pragma unroll
  for (int i = 0; i < 10; i++) c.v[i] = m.l3 ? (i == 0 ? 2 : 0) : c.v[i];
}

/* [0..8](sign P) as qc entries for the affine point (x, y) */
FD_DEV void table4_build(int4* tab, const fe& x, const fe& y, bool negate, const qmask_t& m) {
  fe xs, xy, p0, c1, c, r, cur;
#pragma unroll
  for (int i = 0; i < 10; i++) xs.v[i] = negate ? -x.v[i] : x.v[i];
  fe_mul(xy, xs, y);
#pragma unroll
  for (int i = 0; i < 10; i++) {
    p0.v[i] = m.l0 ? xs.v[i] : (m.l1 ? y.v[i] : (m.l2 ? (i == 0 ? 1 : 0) : xy.v[i]));
    c.v[i] = i == 0 ? (m.l2 ? 0 : (m.l3 ? 2 : 1)) : 0;   /* the identity (1, 1, 0, 2) */
  }
  tab4_store(tab, 0, c);
  ge4_to_qc(c1, p0, m);
  tab4_store(tab, 1, c1);
  cur = p0;
#pragma clang loop unroll(disable)
  for (int e = 2; e <= 8; e++) {
    ge4_add(r, cur, c1, m);
    ge4_to_p3(cur, r);
    ge4_to_qc(c, cur, m);
    tab4_store(tab, e, c);
  }
}

template <int BW>
__global__ void __launch_bounds__(256) fd_ed25519_dsm4_kernel(fd_ed25519_verify_params_t p) {
  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t j = gid >> 2;   /* a quad per signature: all four lanes take the same branches */
  if (j >= p.n) return;
  const uint32_t hf = p.hflag[j];
  if (hf & FD_HF_FULL) return;   /* the dsm kernel's (full-length form) */
  const qmask_t m = quad_masks();
  int4* tabA = reinterpret_cast<int4*>(static_cast<char*>(p.atab) + gid * FD_ED25519_QUAD_LANE_BYTES);
  int4* tabR = tabA + 27;
  int code = precheck(p, j);
  {
    fe x, y;
    load_pt(x, y, p, 0, j);
    table4_build(tabA, x, y, true, m);
    load_pt(x, y, p, 1, j);
    table4_build(tabR, x, y, !(hf & FD_HF_DNEG), m);
  }
  uint32_t cd[5], dd[5], ld[5], hd[5];
  int W = 33;
  {
    uint32_t x[5], t[5];
    load_hs(x, p, 5, 5, j);
    const int wl = (fd_half_bitlen<5>(x) + 4) >> 2;
#pragma unroll
    for (int w = 34; w <= (FD_HALF_DBITS_MAX + 4) / 4; w++) W += __ballot(wl >= w) != 0ull;
    const int sh = 160 - 4 * W;
    shl160v(t, x, sh); recode160<4>(dd, t);
    load_hs(x, p, 0, 5, j);  shl160v(t, x, sh); recode160<4>(cd, t);
    load_hs(x, p, 10, 5, j); shl160<fd_bw<BW>::LO_SHL>(ld, x);
    load_hs(x, p, 15, 4, j); shl160<fd_bw<BW>::HI_SHL>(hd, x);
  }
  fe P, Rt;
#pragma unroll
  for (int i = 0; i < 10; i++) P.v[i] = (i == 0 && (m.l1 | m.l2)) ? 1 : 0;   /* identity (0, 1, 1, 0) */
#pragma clang loop unroll(disable)
  for (int it = W - 1; it >= 0; it--) {
    int ea = pop160<4>(cd), er = pop160<4>(dd);
    if (it == W - 1) { ea &= 15; er &= 15; }
    const bool blo = fd_bw<BW>::lo_at(it), bhi = fd_bw<BW>::hi_at(it);
    fe ca, cr, b1, b2;
    tab4_load(ca, tabA, ea < 0 ? -ea : ea);
    if (it != W - 1) {
#pragma clang loop unroll(disable)
      for (int dbl = 0; dbl < 4; dbl++) {
        ge4_dbl(Rt, P, m);
        ge4_to_p3(P, Rt);
      }
    }
    tab4_load(cr, tabR, er < 0 ? -er : er);
    ge4_cneg(P, m.l03, ea < 0);
    ge4_add(Rt, P, ca, m);
    ge4_cneg(Rt, m.l0, ea < 0);
    ge4_to_p3(P, Rt);
    if (blo) btab4_load(b1, p.btab_lo, (int)pop160u<BW>(ld), m);
    if (bhi) btab4_load(b2, p.btab_hi, (int)pop160u<BW>(hd), m);
    ge4_cneg(P, m.l03, er < 0);
    ge4_add(Rt, P, cr, m);
    ge4_cneg(Rt, m.l0, er < 0);
    ge4_to_p3(P, Rt);
    if (blo) {
      ge4_add(Rt, P, b1, m);
      ge4_to_p3(P, Rt);
    }
    if (bhi) {
      ge4_add(Rt, P, b2, m);
      ge4_to_p3(P, Rt);
    }
  }
  /* identity: X == 0 and Y == Z (on lane 0) */
  fe y1, z1, t;
  fe_qp<FD_QP(1, 1, 1, 1)>(y1, P);
  fe_qp<FD_QP(2, 2, 2, 2)>(z1, P);
  fe_sub(t, y1, z1);
  const bool ident = fe_iszero(P) && fe_iszero(t);
  if (code == FD_PENDING) code = ident ? FD_ED25519_SUCCESS : FD_ED25519_ERR_MSG;
  if (m.l0) p.out[p.base + j] = (int8_t)code;
}

/* dsm8: two quads per signature for the smallest chunks.  The four-scalar
   sum splits into two Straus halves over the same windows,

       quad 0: [c](-A) + [s_lo]B        quad 1: [|d|](-+R) + [s_hi]B',

   each quad building only its own [0..8] table and doing one table
   addition (plus one base addition every 6th window) per 4 doublings;
   quad 1 then hands its point to quad 0 (DPP row shift) for one last
   addition and the identity test.  ~22% less latency than dsm4 for ~57%
   more lane work. */
template <int BW>
__global__ void __launch_bounds__(256) fd_ed25519_dsm8_kernel(fd_ed25519_verify_params_t p) {
  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t j = gid >> 3;                 /* 8 lanes per signature, the same branches */
  if (j >= p.n) return;
  const uint32_t hf = p.hflag[j];
  if (hf & FD_HF_FULL) return;   /* the dsm kernel's (full-length form) */
  const int half = (int)((threadIdx.x >> 2) & 1u);   /* 0: -A and B, 1: -+R and B' */
  const qmask_t m = quad_masks();
  int4* tab = reinterpret_cast<int4*>(static_cast<char*>(p.atab) + gid * (FD_ED25519_QUAD_LANE_BYTES / 2));
  int code = precheck(p, j);
  {
    fe x, y;
    load_pt(x, y, p, half, j);
    table4_build(tab, x, y, half ? !(hf & FD_HF_DNEG) : true, m);
  }
  uint32_t sd[5], bd[5];
  int W = 33;
  {
    uint32_t x[5], t[5];
    load_hs(x, p, 5, 5, j);
    const int wl = (fd_half_bitlen<5>(x) + 4) >> 2;
#pragma unroll
    for (int w = 34; w <= (FD_HALF_DBITS_MAX + 4) / 4; w++) W += __ballot(wl >= w) != 0ull;
    if (!half) load_hs(x, p, 0, 5, j);
    shl160v(t, x, 160 - 4 * W); recode160<4>(sd, t);
    if (half) {
      load_hs(x, p, 15, 4, j);
      shl160<fd_bw<BW>::HI_SHL>(bd, x);
    } else {
      load_hs(x, p, 10, 5, j);
      shl160<fd_bw<BW>::LO_SHL>(bd, x);
    }
  }
  const int32_t* btab = half ? p.btab_hi : p.btab_lo;
  fe P, Rt;
#pragma unroll
  for (int i = 0; i < 10; i++) P.v[i] = (i == 0 && (m.l1 | m.l2)) ? 1 : 0;   /* identity (0, 1, 1, 0) */
#pragma clang loop unroll(disable)
  for (int it = W - 1; it >= 0; it--) {
    int e = pop160<4>(sd);
    if (it == W - 1) e &= 15;
    const bool badd = half ? fd_bw<BW>::hi_at(it) : fd_bw<BW>::lo_at(it);
    fe ce, b;
    tab4_load(ce, tab, e < 0 ? -e : e);
    if (it != W - 1) {
#pragma clang loop unroll(disable)
      for (int dbl = 0; dbl < 4; dbl++) {
        ge4_dbl(Rt, P, m);
        ge4_to_p3(P, Rt);
      }
    }
    if (badd) btab4_load(b, btab, (int)pop160u<BW>(bd), m);
    ge4_cneg(P, m.l03, e < 0);
    ge4_add(Rt, P, ce, m);
    ge4_cneg(Rt, m.l0, e < 0);
    ge4_to_p3(P, Rt);
    if (badd) {
      ge4_add(Rt, P, b, m);
      ge4_to_p3(P, Rt);
    }
  }
  /* quad 1's point as an addend, moved 4 lanes down */
  fe q, qs;
  ge4_to_qc(q, P, m);
#pragma unroll
  for (int i = 0; i < 10; i++) qs.v[i] = __shfl_down(q.v[i], 4);
  ge4_add(Rt, P, qs, m);
  ge4_to_p3(P, Rt);
  /* identity: X == 0 and Y == Z (on lane 0 of quad 0) */
  fe y1, z1, t;
  fe_qp<FD_QP(1, 1, 1, 1)>(y1, P);
  fe_qp<FD_QP(2, 2, 2, 2)>(z1, P);
  fe_sub(t, y1, z1);
  const bool ident = fe_iszero(P) && fe_iszero(t);
  if (code == FD_PENDING) code = ident ? FD_ED25519_SUCCESS : FD_ED25519_ERR_MSG;
  if (m.l0 && !half) p.out[p.base + j] = (int8_t)code;
}

/* ------------------------------------------------------------------------
   dsm16: the same equation with the field arithmetic spread over the
   lanes (fd25519_r16.h), for the smallest chunks -- a drop-in call, a
   latency-mode batch of a few hundred signatures -- where dsm8 leaves most
   SIMDs idle and each batch waits for one lane's serial chain of products.
   Two waves per signature, one per Straus half as in dsm8 (wave 0: [c](-A)
   + [s_lo]B, wave 1: [|d|](-+R) + [s_hi]B'), a point per wave (row q =
   coordinate q, lane c = limb c), the [0..8] table in nine registers and
   every digit wave-uniform (one signature per wave), so a table lookup is
   a scalar branch.  Base entries are the wide / compact tables' (radix
   2^25.5, converted per lane).  Wave 1 hands its point to wave 0 through
   LDS for the last addition and the identity test.  Same digits, windows,
   tables, additions and order as dsm8. */
#include "fd25519_r16.h"

/* base entry e's coordinate for this lane's row, fetched (btab16_fetch,
   issued a window ahead of its use: the wide tables are 2 GiB, so the
   load usually misses the TLB) and then converted to this lane's r16 limb
   of the qc form (y-x, y+x, 2dxy, 2) */
FD_DEV fe btab16_fetch(const int32_t* g_btab, int e, const r16ctx& k) {
  const int off = (int)((k.r0 & 10u) | (k.r2 & 20u));   /* row 3 loads row 1's (y+x) and drops it */
  const int2* src = reinterpret_cast<const int2*>(g_btab + (size_t)e * FD_ED25519_BTAB16_STRIDE + off);
  fe c;
#pragma unroll
  for (int q = 0; q < 5; q++) {
    const int2 x = src[q];
    c.v[2 * q] = x.x;
    c.v[2 * q + 1] = x.y;
  }
  return c;
}
FD_DEV uint32_t btab16_r16(const fe& c, const r16ctx& k) {
  return (r16_from_fe(c, k) & ~k.r3) | (r16_small(2u, k) & k.r3);
}

/* params.go: one lane of the block polls the page-locked word (a relaxed
   atomic load at system scope: a vector load that goes to the host's
   memory each time, never a cached copy), sleeping between polls, and
   takes the acquire fence once it is set (one cache invalidate per block,
   not one per poll); 0 after the bound */
FD_DEV uint32_t wait_go(const uint32_t* go) {
  for (uint32_t spin = 0u; spin < FD_ED25519_GO_SPIN_MAX; spin++) {
    const uint32_t g = __hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (g != 0u) {
      __atomic_thread_fence(__ATOMIC_ACQUIRE);
      return g;
    }
    __builtin_amdgcn_s_sleep(8);
  }
  return 0u;
}

template <int BW>
__global__ void __launch_bounds__(128) fd_ed25519_dsm16_kernel(fd_ed25519_verify_params_t p) {
  const uint64_t j = blockIdx.x;   /* a block (two waves) per signature: every return below is block-uniform */
  if (j >= p.n) return;
  if (p.go) {   /* launched ahead of the host's scalars and points */
    __shared__ uint32_t go;
    if (threadIdx.x == 0u) go = wait_go(p.go);
    __syncthreads();
    if (go != FD_ED25519_GO_RUN) return;
  }
  const uint32_t hf = p.hflag[j];
  const int half = (int)(threadIdx.x >> 6);   /* 0: -A and B, 1: -+R and B' */
  /* the scalars loaded first, used after the table build: with host
     scalars (p.hs_host) they sit in page-locked host memory, and their
     link round trips then overlap the table build instead of following it */
  uint32_t hd[5], hx[5], hb[5];
  load_hs(hd, p, 5, 5, j);                    /* |d|                     */
  load_hs(hx, p, half ? 5 : 0, 5, j);         /* c (wave 0), |d| (wave 1) */
  load_hs(hb, p, half ? 15 : 10, half ? 4 : 5, j);   /* s_hi / s_lo        */
  if (hf & FD_HF_FULL) return;     /* the dsm kernel's (full-length form) */
  r16ctx k;
  r16_init(k);
  const uint32_t d2 = r16_from_fe(fe{FE_D2}, k);
  uint32_t tab[9];
  {
    fe x, y;
    load_pt(x, y, p, half, j);
    table16_build(tab, r16_from_fe(x, k), r16_from_fe(y, k), half ? !(hf & FD_HF_DNEG) : true, d2, k);
  }
  uint32_t sd[5], bd[5];
  int W = 33;
  {
    uint32_t t[5];
    W = (fd_half_bitlen<5>(hd) + 4) >> 2;
    W = W < 33 ? 33 : W;
    shl160v(t, hx, 160 - 4 * W); recode160<4>(sd, t);
    if (half) shl160<fd_bw<BW>::HI_SHL>(bd, hb);
    else      shl160<fd_bw<BW>::LO_SHL>(bd, hb);
  }
  W = __builtin_amdgcn_readfirstlane(W);
  const int32_t* btab = half ? p.btab_hi : p.btab_lo;
  const uint32_t one = r16_small(1u, k);
  uint32_t P = one & k.r12;   /* identity (0, 1, 1, 0) */
#pragma clang loop unroll(disable)
  for (int it = W - 1; it >= 0; it--) {
    int e = pop160<4>(sd);
    if (it == W - 1) e &= 15;
    e = __builtin_amdgcn_readfirstlane(e);
    const bool badd = half ? fd_bw<BW>::hi_at(it) : fd_bw<BW>::lo_at(it);
    const uint32_t bdig = (uint32_t)__builtin_amdgcn_readfirstlane((int)(badd ? pop160u<BW>(bd) : 0u));
    const uint32_t ce = table16_at(tab, e < 0 ? -e : e);
    fe braw;
    if (badd) braw = btab16_fetch(btab, (int)bdig, k);   /* in flight during the doublings */
    if (it != W - 1) {
      P = ge16_dbl2<false, false>(P, k);   /* (X, Y, Z, X) between doublings: T only before an addition */
      P = ge16_dbl2<true, false>(P, k);
      P = ge16_dbl2<true, false>(P, k);
      P = ge16_dbl2<true, true>(P, k);
    }
    uint32_t b = 0u;
    if (badd) b = btab16_r16(braw, k);
    if (e != 0) {   /* a zero digit (~1 in 16) adds the identity: skipped, the digit is wave-uniform */
      P = ge16_cneg4(P, k.r03, e < 0, k);
      P = ge16_add2<true>(P, ce, e < 0, k);
    }
    if (badd) P = ge16_add2<true>(P, b, false, k);
  }
  /* wave 1's point as an addend of wave 0's */
  __shared__ uint32_t hand[64];
  if (half) hand[threadIdx.x & 63u] = ge16_to_qc(P, d2, k);
  __syncthreads();
  if (half) return;
  P = ge16_add2<true>(P, hand[threadIdx.x], false, k);
  /* identity: X == 0 (row 0) and Y == Z (row 1: Y + 4p - Z) */
  const uint32_t z = r16_rp<2, 2, 2, 2>(P, k);
  const bool zero = r16_iszero(P + ((k.p4 - z) & k.r1));
  const uint64_t bal = __ballot(zero);
  const bool ident = (bal & 1ull) && (bal & (1ull << 16));
  int code = precheck(p, j);   /* S < L, decode failures, small order: the reference's order */
  if (code == FD_PENDING) code = ident ? FD_ED25519_SUCCESS : FD_ED25519_ERR_MSG;
  /* Write-code-last invariant: a signature's code is the last thing any
     kernel of its launch does with that signature; no kernel reads the
     inputs (or anything else in the drop-in's pinned block) after the code
     is written.  The drop-in's direct launches return once every code has
     landed in that block (host/fd_ed25519_hip_engine.c, dropin_run) and the
     next call restages it; a kernel added after dsm16 that reads the block
     would break that silently. */
  if (threadIdx.x == 0u) p.out[p.base + j] = (int8_t)code;
}

/* ------------------------------------------------------------------------
   dsm16s<S>: dsm16's equation over S = 4 or 8 waves, for the launches
   whose points the host computed (host/fd_ed25519_hip_hsdec.cc).  With
   H = S/2 parts per half-size scalar, split every G = 66 (S = 4) or 33
   (S = 8) bits -- c = sum c_i 2^(G i), |d| = sum d_i 2^(G i) -- and the
   points doubled by the host too, A_i = [2^(G i)]A, R_i = [2^(G i)]R, and
   s' in S chunks of CB = 72 or 32 bits:

     sum_i [c_i](-A_i) + sum_i [d_i](-+R_i) + sum_q [s'_q][2^(CB q)]B == 0

   exactly (A_i and R_i are the points themselves doubled, so no reduction
   of c or d is involved).  Wave q = H side + i holds one variable-base
   term (side 0: A, 1: R) and base chunk q: W = 17 (S = 4) or 9 (S = 8)
   windows of 4 doublings instead of 33 (more for the rare |d| >= 2^131),
   the base digits radix 2^16 from compact tables at offsets 2^(CB q)
   (params.btabq), CB/16 of them (rounded up) at windows .., 4, 0.  The
   waves' points meet in LDS by halves (log2 S rounds of additions), wave
   0 tests the identity.  Inputs (host memory, params.go's launch-ahead):
   pts [S][40][cap] (row 2i + side: A, R, A_1, R_1, ..; A and R affine
   (x, y) in the first 20, the doubled points extended (X, Y, Z, T) -- the
   host never inverts), pflag [2][cap],
   sflag, hflag [cap], hs [24][cap]: rows KW q .. KW q + KW-1 the scalar of
   wave q (KW = 3 or 2 words), rows S KW + BWORDS q .. its chunk of s'. */
template <int S>
__global__ void __launch_bounds__(64 * S) fd_ed25519_dsm16s_kernel(fd_ed25519_verify_params_t p) {
  static_assert(S == 4 || S == 8, "four or eight waves");
  constexpr int H = S / 2, KW = S == 4 ? 3 : 2, CB = S == 4 ? 72 : 32, BWORDS = (CB + 31) / 32;
  constexpr int NB = (CB + 15) / 16, WMIN = S == 4 ? 17 : 9, SH0 = S == 4 ? 64 : 96;
  const uint64_t j = blockIdx.x;   /* a block (S waves) per signature: every return below is block-uniform */
  if (j >= p.n) return;
  if (p.go) {
    __shared__ uint32_t go;
    if (threadIdx.x == 0u) go = wait_go(p.go);
    __syncthreads();
    if (go != FD_ED25519_GO_RUN) return;
  }
  const uint32_t hf = p.hflag[j];
  const int q = (int)(threadIdx.x >> 6), side = q / H, part = q % H;
  uint32_t hk[5] = {0u, 0u, 0u, 0u, 0u}, hb[5] = {0u, 0u, 0u, 0u, 0u};
#pragma unroll
  for (int w = 0; w < KW; w++) hk[w] = p.hs[(uint64_t)(KW * q + w) * p.cap + j];
#pragma unroll
  for (int w = 0; w < BWORDS; w++) hb[w] = p.hs[(uint64_t)(S * KW + BWORDS * q + w) * p.cap + j];
  /* the block's window count: the longest of the S scalars (every wave
     reads them all, so W is the same in each without a barrier) */
  int W = WMIN;
#pragma unroll
  for (int t = 0; t < S; t++) {
    uint32_t x[5] = {0u, 0u, 0u, 0u, 0u};
#pragma unroll
    for (int w = 0; w < KW; w++) x[w] = p.hs[(uint64_t)(KW * t + w) * p.cap + j];
    const int wt = (fd_half_bitlen<5>(x) + 4) >> 2;
    W = wt > W ? wt : W;
  }
  W = __builtin_amdgcn_readfirstlane(W);
  r16ctx k;
  r16_init(k);
  const uint32_t d2 = r16_from_fe(fe{FE_D2}, k);
  uint32_t tab[9];
  {
    const bool negate = side == 0 ? true : !(hf & FD_HF_DNEG);
    const int32_t* src = p.pts + (uint64_t)(2 * part + side) * 40 * p.cap + j;
    if (part == 0) {   /* A or R as decoded: affine (x, y) */
      fe x, y;
      load_fe(x, src, p.cap);
      load_fe(y, src + 10 * p.cap, p.cap);
      table16_build(tab, r16_from_fe(x, k), r16_from_fe(y, k), negate, d2, k);
    } else {           /* doubled on the host: extended (X, Y, Z, T), no inversion; row r loads coordinate r */
      fe c;
      load_fe(c, src + (uint64_t)k.row * 10 * p.cap, p.cap);
      table16_build_p3(tab, ge16_cneg4(r16_from_fe(c, k), k.r03, negate, k), d2, k);
    }
  }
  uint32_t sd[5], bd[5];
  {
    uint32_t t[5], u[5];
    shl160<SH0>(u, hk);                      /* 160 - 4W - SH0 in [8, 28] for every W that occurs */
    shl160v(t, u, 160 - 4 * W - SH0);
    recode160<4>(sd, t);
    shl160<160 - 16 * NB>(bd, hb);           /* the chunk's 16-bit digits, the top one first */
  }
  const int32_t* btab = p.btabq[q];
  const uint32_t one = r16_small(1u, k);
  uint32_t P = one & k.r12;   /* identity (0, 1, 1, 0) */
#pragma clang loop unroll(disable)
  for (int it = W - 1; it >= 0; it--) {
    int e = pop160<4>(sd);
    if (it == W - 1) e &= 15;
    e = __builtin_amdgcn_readfirstlane(e);
    const bool badd = it < 4 * NB && (it & 3) == 0;
    const uint32_t bdig = (uint32_t)__builtin_amdgcn_readfirstlane((int)(badd ? pop160u<16>(bd) : 0u));
    const uint32_t ce = table16_at(tab, e < 0 ? -e : e);
    fe braw;
    if (badd) braw = btab16_fetch(btab, (int)bdig, k);
    if (it != W - 1) {
      P = ge16_dbl2<false, false>(P, k);
      P = ge16_dbl2<true, false>(P, k);
      P = ge16_dbl2<true, false>(P, k);
      P = ge16_dbl2<true, true>(P, k);
    }
    uint32_t b = 0u;
    if (badd) b = btab16_r16(braw, k);
    if (e != 0) {
      P = ge16_cneg4(P, k.r03, e < 0, k);
      P = ge16_add2<true>(P, ce, e < 0, k);
    }
    if (badd) P = ge16_add2<true>(P, b, false, k);
  }
  /* the waves' points summed by halves: waves [h, 2h) hand theirs to
     [0, h); every wave reaches every barrier */
  __shared__ uint32_t hand[S / 2][64];
#pragma unroll
  for (int h = S / 2; h >= 1; h >>= 1) {
    if (q >= h && q < 2 * h) hand[q - h][threadIdx.x & 63u] = ge16_to_qc(P, d2, k);
    __syncthreads();
    if (q < h) P = ge16_add2<true>(P, hand[q][threadIdx.x & 63u], false, k);
    __syncthreads();
  }
  if (q) return;
  const uint32_t z = r16_rp<2, 2, 2, 2>(P, k);
  const bool zero = r16_iszero(P + ((k.p4 - z) & k.r1));
  const uint64_t bal = __ballot(zero);
  const bool ident = (bal & 1ull) && (bal & (1ull << 16));
  int code = precheck(p, j);
  if (code == FD_PENDING) code = ident ? FD_ED25519_SUCCESS : FD_ED25519_ERR_MSG;
  /* the code last (dsm16's write-code-last invariant) */
  if (threadIdx.x == 0u) p.out[p.base + j] = (int8_t)code;
}

extern "C" int fd_ed25519_hip_launch_dsm16s(const fd_ed25519_verify_params_t* p, int waves, void* stream) {
  if (!p->n) return 0;
  if (waves != 4 && waves != 8) return (int)hipErrorInvalidValue;
  for (int q = 0; q < waves; q++)
    if (!p->btabq[q]) return (int)hipErrorInvalidValue;
  if (waves == 4)
    hipLaunchKernelGGL(fd_ed25519_dsm16s_kernel<4>, dim3((uint32_t)p->n), dim3(256), 0, (hipStream_t)stream, *p);
  else
    hipLaunchKernelGGL(fd_ed25519_dsm16s_kernel<8>, dim3((uint32_t)p->n), dim3(512), 0, (hipStream_t)stream, *p);
  return (int)hipGetLastError();
}

/* ------------------------------------------------------------------------
   prep16: the dsm16 chunks' prep, with the decompressions spread over the
   lanes as dsm16's products are.  The one-lane decode is a chain of 250
   dependent squarings (~490 cycles each, fe_sq_u); a row of 16 lanes runs
   one in ~300 (profiles/r5_lanesplit_ubench.txt), so a wave decodes four
   points (row q: point 4w + q, A and R of two signatures) in about 60% of
   the time.  One wave per block: the first hash_waves blocks hash and find
   the half-size scalars of 64 signatures each (prep's wave 0), the others
   decode.  Outputs are decode_one's: x in fe_mul's carried form with its
   sign applied, y as fe_frombytes of the encoding, the flags. */
FD_DEV void decode16_wave(const fd_ed25519_verify_params_t& p, uint64_t dw) {
  r16ctx k;
  r16_init(k);
  const uint64_t pt = 4u * dw + k.row;
  const int which = (int)(pt & 1u);   /* 0: A (public key), 1: R */
  const bool live = (pt >> 1) < p.n;
  const uint64_t j = live ? pt >> 1 : p.n - 1u;   /* an idle row repeats a live point, its result dropped */
  const uint64_t i = p.base + j;
  const uint32_t* src = which ? reinterpret_cast<const uint32_t*>(p.sigs + 64 * i)
                              : reinterpret_cast<const uint32_t*>(p.pubs + 32 * i);
  const uint32_t wd = src[k.c >> 1], w7 = src[7];
  uint32_t y = (k.c & 1u) ? wd >> 16 : wd & 0xffffu;
  y &= k.c == 15u ? 0x7fffu : 0xffffu;
  const uint32_t d = r16_from_fe(fe{FE_D}, k), sqrtm1 = r16_from_fe(fe{FE_SQRTM1}, k);
  r16_dec o;
  decode16(o, y, w7 >> 31, !p.codes_portable, d, sqrtm1, k);
  if (live && k.c == 0u) {
    uint32_t s[8];
#pragma unroll
    for (int q = 0; q < 8; q++) s[q] = src[q];
    fe x, fy, t;
    fe_frombytes(t, o.x);
    fe_carry(x, t);
    if (o.neg) fe_neg(x, x);
    fe_frombytes(fy, s);
    int32_t* dst = p.pts + (uint64_t)which * 20 * p.cap + j;
#pragma unroll
    for (int l = 0; l < 10; l++) {
      dst[(uint64_t)l * p.cap] = x.v[l];
      dst[(uint64_t)(10 + l) * p.cap] = fy.v[l];
    }
    p.pflag[(uint64_t)which * p.cap + j] = (uint8_t)((o.fail ? FD_PF_FAIL : 0u) | (o.small ? FD_PF_SMALL : 0u));
  }
}

/* The hash blocks: 128 threads for 32 signatures, wave 1 building the
   message schedules into LDS, wave 0 running the rounds from them
   (sha512_sched_wave / sha512_rounds_wave), then k and the half-size
   scalars.  Every lane of both waves reaches every barrier: lanes past the
   chunk repeat the last signature and store nothing. */
FD_DEV void hash16_block(const fd_ed25519_verify_params_t& p, uint64_t* sched) {
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint64_t t = (uint64_t)blockIdx.x * SHA2W_LANES + (threadIdx.x & (SHA2W_LANES - 1u));
  const bool live = t < p.n && (threadIdx.x & 63u) < SHA2W_LANES;
  const uint64_t j = live ? t : p.n - 1u;
  const uint64_t i = p.base + j;
  uint32_t pre[16], S[8];
  {
    const uint4* sg = reinterpret_cast<const uint4*>(p.sigs + 64 * i);
    const uint4* pk = reinterpret_cast<const uint4*>(p.pubs + 32 * i);
    const uint4 q0 = sg[0], q1 = sg[1], q2 = sg[2], q3 = sg[3], q4 = pk[0], q5 = pk[1];
    pre[0] = q0.x; pre[1] = q0.y; pre[2] = q0.z; pre[3] = q0.w; pre[4] = q1.x; pre[5] = q1.y; pre[6] = q1.z;
    pre[7] = q1.w;
    pre[8] = q4.x; pre[9] = q4.y; pre[10] = q4.z; pre[11] = q4.w; pre[12] = q5.x; pre[13] = q5.y; pre[14] = q5.z;
    pre[15] = q5.w;
    S[0] = q2.x; S[1] = q2.y; S[2] = q2.z; S[3] = q2.w; S[4] = q3.x; S[5] = q3.y; S[6] = q3.z; S[7] = q3.w;
  }
  sha_msg_src m = {nullptr, 0u, 0u};
  uint32_t nblk = 0u;
  if (!p.digests) {
    const uintptr_t mp = reinterpret_cast<uintptr_t>(p.msgs + p.msg_off[i]);
    m.base = reinterpret_cast<const uint32_t*>(mp & ~(uintptr_t)3);
    m.shift = (uint32_t)(mp & 3);
    m.sz = p.msg_sz[i];
    nblk = (m.sz + 64u + 17u + 127u) >> 7;
  }
  /* the wave's largest block count, the same in both waves: the barrier count */
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t o = (uint32_t)__shfl_xor((int)nblk, off);
    nblk = o > nblk ? o : nblk;
  }
  const uint32_t nblk_wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)nblk);
  if (wave == 1u) {
    sha512_sched_wave<16>(pre, m, nblk_wave, sched);
    return;
  }
  uint32_t dig[16];
  if (p.digests) {
    const uint4* dg = reinterpret_cast<const uint4*>(p.digests + 64 * i);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint4 v = dg[q];
      dig[4 * q] = v.x; dig[4 * q + 1] = v.y; dig[4 * q + 2] = v.z; dig[4 * q + 3] = v.w;
    }
  } else {
    sha512_rounds_wave<16>(dig, m, nblk_wave, sched);
  }
  if (!live) return;
  hash_finish(p, j, dig, S);
  scalar_one(p, j);
#if FD_ED25519_FULL_IN_PREP
  /* the rare signature without a half-size pair (~1e-6): the full-length
     form right here, on points this lane decodes itself (decode16's
     blocks write the same points concurrently, in another
     representation), so that no flag-scan launch follows dsm16 */
  if (p.full_in_prep && (p.hflag[j] & FD_HF_FULL)) {
    const bool avx = !p.codes_portable;
    uint32_t sa[8], sr[8];
#pragma unroll
    for (int w = 0; w < 8; w++) { sa[w] = pre[8 + w]; sr[w] = pre[w]; }
    decoded_pt da, dr;
    ge_decode(da, sa, avx);
    ge_decode(dr, sr, avx);
    int code = FD_PENDING;   /* precheck's order, from this lane's own flags */
    if (!p.sflag[j]) code = FD_ED25519_ERR_SIG;
    else if (da.fail) code = p.codes_portable ? FD_ED25519_ERR_PUBKEY : FD_ED25519_ERR_SIG;
    else if (dr.fail) code = FD_ED25519_ERR_SIG;
    else if (da.small) code = FD_ED25519_ERR_PUBKEY;
    else if (dr.small) code = FD_ED25519_ERR_SIG;
    int4* tabA = reinterpret_cast<int4*>(static_cast<char*>(p.atab) + (j >> 6) * FD_ED25519_ATAB_BYTES_PER_WAVE) +
                 (j & 63u) * (2 * FD_ED25519_ATAB_STRIDE * 10);
    /* the code last: see the write-code-last invariant at dsm16's end */
    p.out[p.base + j] = (int8_t)dsm_full_core(p, j, tabA, code, da.x, da.y, dr.x, dr.y);
  }
#endif
}

__global__ void __launch_bounds__(128) fd_ed25519_prep16_kernel(fd_ed25519_verify_params_t p, uint32_t hash_blocks) {
  __shared__ uint64_t sched[2 * SHA2W_WORDS];
  if (blockIdx.x < hash_blocks) {
    hash16_block(p, sched);
    return;
  }
  decode16_wave(p, 2u * (blockIdx.x - hash_blocks) + (threadIdx.x >> 6));
}

/* ------------------------------------------------------------------------
   Base tables [0..entries)B as (y+x, y-x, 2dxy), one entry per lane:
   [e]B by double-and-add over `bits` bits, then affine. */

__global__ void fd_ed25519_gen_btab_kernel(int32_t* btab, int entries, int stride, int bits, int base_dbl) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= entries) return;
  ge_p3 B, P;
  const fe bx = {FE_BX}, by = {FE_BY}, d2 = {FE_D2};
  B.X = bx; B.Y = by; fe_1(B.Z); fe_mul(B.T, bx, by);
  for (int i = 0; i < base_dbl; i++) {   /* the table's base: [2^base_dbl]B */
    ge_p1p1 t2;
    ge_p3_dbl(t2, B);
    ge_p1p1_to_p3(B, t2);
  }
  ge_cached cb;
  ge_p3_to_cached(cb, B);
  ge_p3_0(P);
  ge_p1p1 t;
  for (int bit = bits - 1; bit >= 0; bit--) {
    ge_p3_dbl(t, P);
    ge_p1p1_to_p3(P, t);
    if ((e >> bit) & 1) {
      ge_add(t, P, cb);
      ge_p1p1_to_p3(P, t);
    }
  }
  fe zi, x, y, ypx, ymx, xy2d;
  fe_invert(zi, P.Z);
  fe_mul(x, P.X, zi);
  fe_mul(y, P.Y, zi);
  fe_add(ypx, y, x); fe_carry(ypx, ypx);
  fe_sub(ymx, y, x); fe_carry(ymx, ymx);
  fe_mul(xy2d, x, y);
  fe_mul(xy2d, xy2d, d2);
  int32_t* o = btab + (int64_t)e * stride;
  for (int i = 0; i < 10; i++) {
    o[i] = ypx.v[i];
    o[10 + i] = ymx.v[i];
    o[20 + i] = xy2d.v[i];
  }
  for (int i = 30; i < stride; i++) o[i] = 0;
}

/* Wide unsigned-digit tables [0..2^bits)[2^base_dbl]B (bits 24, or 16 for
   the compact tables).  The base is computed
   once (gen_base), then each thread produces a run of consecutive entries
   by additions and puts them in affine form with one inversion per run
   (Montgomery's trick: prefix products of Z in `scratch`). */
#define FD_BTAB_RUN 32

__global__ void fd_ed25519_gen_base_kernel(int32_t* base, int base_dbl) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  ge_p3 B;
  const fe bx = {FE_BX}, by = {FE_BY};
  B.X = bx; B.Y = by; fe_1(B.Z); fe_mul(B.T, bx, by);
  for (int i = 0; i < base_dbl; i++) {
    ge_p1p1 t2;
    ge_p3_dbl(t2, B);
    ge_p1p1_to_p3(B, t2);
  }
  for (int i = 0; i < 10; i++) {
    base[i] = B.X.v[i]; base[10 + i] = B.Y.v[i]; base[20 + i] = B.Z.v[i]; base[30 + i] = B.T.v[i];
  }
}

FD_DEV void fe_st(int32_t* o, const fe& a) {
  for (int i = 0; i < 10; i++) o[i] = a.v[i];
}
FD_DEV void fe_ld(fe& a, const int32_t* o) {
  for (int i = 0; i < 10; i++) a.v[i] = o[i];
}

__global__ void __launch_bounds__(256)
fd_ed25519_gen_btab_run_kernel(int32_t* tab, int entries, int bits, const int32_t* base, int32_t* scratch) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int e0 = t * FD_BTAB_RUN;
  if (e0 >= entries) return;
  const int e1 = e0 + FD_BTAB_RUN < entries ? e0 + FD_BTAB_RUN : entries;
  ge_p3 B, P;
  fe_ld(B.X, base); fe_ld(B.Y, base + 10); fe_ld(B.Z, base + 20); fe_ld(B.T, base + 30);
  ge_cached cb;
  ge_p3_to_cached(cb, B);
  ge_p3_0(P);
  ge_p1p1 r;
  for (int bit = bits - 1; bit >= 0; bit--) {   /* P = [e0] base */
    ge_p3_dbl(r, P);
    ge_p1p1_to_p3(P, r);
    if ((e0 >> bit) & 1) {
      ge_add(r, P, cb);
      ge_p1p1_to_p3(P, r);
    }
  }
  fe acc;
  fe_1(acc);
  for (int e = e0; e < e1; e++) {   /* projective entries, prefix products of Z */
    int32_t* o = tab + (int64_t)e * FD_ED25519_BTAB16_STRIDE;
    fe_st(o, P.X); fe_st(o + 10, P.Y); fe_st(o + 20, P.Z);
    fe_mul(acc, acc, P.Z);
    fe_st(scratch + (int64_t)e * 10, acc);
    ge_add(r, P, cb);
    ge_p1p1_to_p3(P, r);
  }
  fe inv;
  fe_invert(inv, acc);
  const fe d2 = {FE_D2};
  for (int e = e1 - 1; e >= e0; e--) {
    int32_t* o = tab + (int64_t)e * FD_ED25519_BTAB16_STRIDE;
    fe X, Y, Z, zi, x, y, ypx, ymx, xy2d;
    fe_ld(X, o); fe_ld(Y, o + 10); fe_ld(Z, o + 20);
    if (e > e0) {
      fe prev;
      fe_ld(prev, scratch + (int64_t)(e - 1) * 10);
      fe_mul(zi, inv, prev);
    } else {
      zi = inv;
    }
    fe_mul(inv, inv, Z);
    fe_mul(x, X, zi);
    fe_mul(y, Y, zi);
    fe_add(ypx, y, x); fe_carry(ypx, ypx);
    fe_sub(ymx, y, x); fe_carry(ymx, ymx);
    fe_mul(xy2d, x, y);
    fe_mul(xy2d, xy2d, d2);
    fe_st(o, ypx); fe_st(o + 10, ymx); fe_st(o + 20, xy2d);
    o[30] = 0; o[31] = 0;
  }
}

/* Self-check of a wide base table: entry e + 1 == entry e + entry 1 for
   every e (entry 0 the identity), one lane per e; mismatches counted with a
   vector atomic.  With entry 1 (and a few others) compared against an
   independent [s]B on the host, this proves every entry
   (fd_ed25519_hip_engine_check_base_tables, tests/test_gpu_parity.py). */
FD_DEV void btab_entry_p3(ge_p3& P, const int32_t* o) {
  const fe dinv = {FE_DINV};
  fe ypx, ymx, xy2d;
  fe_ld(ypx, o); fe_ld(ymx, o + 10); fe_ld(xy2d, o + 20);
  fe_sub(P.X, ypx, ymx);          /* 2x */
  fe_add(P.Y, ypx, ymx);          /* 2y */
  fe_0(P.Z); P.Z.v[0] = 2;        /* 2  */
  fe_mul(P.T, xy2d, dinv);        /* 2xy = X Y / Z */
}

__global__ void __launch_bounds__(256)
fd_ed25519_check_btabw_kernel(const int32_t* tab, int entries, uint32_t* bad) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e + 1 >= entries) return;
  const int32_t* o = tab + (int64_t)e * FD_ED25519_BTAB16_STRIDE;
  const int32_t* n = o + FD_ED25519_BTAB16_STRIDE;
  const int32_t* b = tab + FD_ED25519_BTAB16_STRIDE;
  ge_p3 P;
  btab_entry_p3(P, o);
  ge_precomp q;
  fe_ld(q.yplusx, b); fe_ld(q.yminusx, b + 10); fe_ld(q.xy2d, b + 20);
  ge_p1p1 r;
  ge_madd(r, P, q);                /* x = r.X / r.Z, y = r.Y / r.T */
  fe ypx, ymx, d, t, u;
  fe_ld(ypx, n); fe_ld(ymx, n + 10);
  fe_sub(d, ypx, ymx);             /* 2x' */
  fe_mul(t, d, r.Z);
  fe_add(u, r.X, r.X);
  fe_sub(t, t, u);
  bool ok = fe_iszero(t);
  fe_add(d, ypx, ymx);             /* 2y' */
  fe_mul(t, d, r.T);
  fe_add(u, r.Y, r.Y);
  fe_sub(t, t, u);
  ok = ok && fe_iszero(t);
  if (e == 0) {                    /* entry 0: the identity (1, 1, 0) */
    bool id = o[0] == 1 && o[10] == 1 && o[20] == 0;
    for (int i = 1; i < 10; i++) id = id && o[i] == 0 && o[10 + i] == 0 && o[20 + i] == 0;
    ok = ok && id;
  }
  if (!ok) atomicAdd(bad, 1u);
}

extern "C" int fd_ed25519_hip_launch_check_btabw(const int32_t* d_tab, int entries, uint32_t* d_bad, void* stream) {
  hipLaunchKernelGGL(fd_ed25519_check_btabw_kernel, dim3((entries + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     d_tab, entries, d_bad);
  return (int)hipGetLastError();
}

/* ------------------------------------------------------------------------
   Per-transaction combine (fd_ed25519_verify_batch_single_msg priority). */

__global__ void fd_ed25519_txn_combine_kernel(const int8_t* sig_codes, const uint32_t* txn_first,
                                              const uint32_t* txn_cnt, int8_t* out, uint64_t ntxn) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntxn) return;
  const uint32_t f = txn_first[t], n = txn_cnt[t];
  int code = FD_ED25519_SUCCESS;
  if (n == 0u || n > 16u) {
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

#if FD_ED25519_HALF_FAULT
/* Fault-injection build only (tests/test_gpu_service_fault.py): a stand-in
   for a hung batch.  One wave sleeps until `ticks` of the constant-rate
   wall clock have passed since it started, then exits: every wave reaches
   that exit, so the grid always drains (a bounded stall, never a real
   hang). */
__global__ void fd_ed25519_stall_kernel(uint64_t ticks) {
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

extern "C" int fd_ed25519_hip_launch_stall(unsigned ms, void* stream) {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
      khz <= 0)
    khz = 100000;
  if (ms > 10000u) ms = 10000u;   /* bounded whatever the caller asks */
  hipLaunchKernelGGL(fd_ed25519_stall_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (uint64_t)ms * (uint64_t)khz);
  return (int)hipGetLastError();
}
#endif

/* ------------------------------------------------------------------------
   C-ABI launchers */

extern "C" int fd_ed25519_hip_launch_gen_btab(int32_t* d_btab, void* stream) {
  hipLaunchKernelGGL(fd_ed25519_gen_btab_kernel, dim3(3), dim3(64), 0, (hipStream_t)stream, d_btab,
                     FD_ED25519_BTAB_ENTRIES, FD_ED25519_BTAB_STRIDE, 8, 0);
  return (int)hipGetLastError();
}

extern "C" int fd_ed25519_hip_launch_gen_btab8(int32_t* d_tab, int base_dbl, void* stream) {
  hipLaunchKernelGGL(fd_ed25519_gen_btab_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, d_tab, 256,
                     FD_ED25519_BTAB16_STRIDE, 8, base_dbl);
  return (int)hipGetLastError();
}

extern "C" int fd_ed25519_hip_launch_gen_btab16(int32_t* d_btab16, int base_dbl, void* stream) {
  const int entries = FD_ED25519_BTAB16_ENTRIES;
  hipLaunchKernelGGL(fd_ed25519_gen_btab_kernel, dim3((entries + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     d_btab16, entries, FD_ED25519_BTAB16_STRIDE, 16, base_dbl);
  return (int)hipGetLastError();
}

__global__ void __launch_bounds__(256) fd_ed25519_diag_half_kernel(const uint32_t* kin, uint32_t* out, uint64_t n,
                                                                   int dbits) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8], c[FD_HALF_TW], d[FD_HALF_TW];
  for (int w = 0; w < 8; w++) k[w] = kin[8 * i + w];
  int neg = 0;
  const int ok = half_scalars_checked(k, c, d, &neg, dbits, i);
  uint32_t* o = out + 12 * i;
  o[0] = (uint32_t)ok;
  o[1] = (uint32_t)neg;
  for (int w = 0; w < FD_HALF_TW; w++) { o[2 + w] = c[w]; o[7 + w] = d[w]; }
}

extern "C" int fd_ed25519_hip_launch_diag_half(const uint32_t* d_k, uint32_t* d_out, uint64_t n, int dbits,
                                               void* stream) {
  if (!n) return 0;
  hipLaunchKernelGGL(fd_ed25519_diag_half_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     d_k, d_out, n, dbits);
  return (int)hipGetLastError();
}

extern "C" int fd_ed25519_hip_launch_gen_btabw(int32_t* d_tab, int base_dbl, int bits, int32_t* d_scratch,
                                               void* stream) {
  if (bits != FD_ED25519_BTABW_BITS && bits != FD_ED25519_BTABC_BITS) return (int)hipErrorInvalidValue;
  const int entries = 1 << bits;
  int32_t* base = d_scratch + (size_t)entries * 10;   /* 40 ints after the prefix products */
  hipLaunchKernelGGL(fd_ed25519_gen_base_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, base, base_dbl);
  const int threads = (entries + FD_BTAB_RUN - 1) / FD_BTAB_RUN;
  hipLaunchKernelGGL(fd_ed25519_gen_btab_run_kernel, dim3((threads + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     d_tab, entries, bits, (const int32_t*)base, d_scratch);
  return (int)hipGetLastError();
}

extern "C" int fd_ed25519_hip_launch_phase(const fd_ed25519_verify_params_t* p, int phase, uint32_t grid,
                                           void* stream) {
  if (!p->n) return 0;
  hipStream_t st = (hipStream_t)stream;
  const uint32_t blk = 256;
  switch (phase) {
  case FD_ED25519_PHASE_HASH: {
    if (p->small == 3) {   /* dsm16 chunks: the decompressions lane-split too, the hash over two waves */
      const uint32_t hb = p->hs_host ? 0u : (uint32_t)((p->n + SHA2W_LANES - 1) / SHA2W_LANES),
                     dw = (uint32_t)((p->n + 1) / 2);
      hipLaunchKernelGGL(fd_ed25519_prep16_kernel, dim3(hb + (dw + 1) / 2), dim3(128), 0, st, *p, hb);
      break;
    }
    if (p->small) {
      hipLaunchKernelGGL(fd_ed25519_prep_kernel, dim3((uint32_t)((p->n + 63) / 64)), dim3(192), 0, st, *p);
      break;
    }
    const dim3 g((uint32_t)((p->n + blk - 1) / blk));
    if (p->perm) {
      const hipError_t e = hipMemsetAsync(p->hist, 0, 2 * FD_ED25519_SORT_BUCKETS * sizeof(uint32_t), st);
      if (e != hipSuccess) return (int)e;
      const dim3 gs((uint32_t)((p->n + FD_SORT_PER_BLOCK - 1) / FD_SORT_PER_BLOCK));
      hipLaunchKernelGGL(fd_ed25519_sort_hist_kernel, gs, dim3(blk), 0, st, *p);
      hipLaunchKernelGGL(fd_ed25519_sort_scan_kernel, dim3(1), dim3(64), 0, st, *p);
      hipLaunchKernelGGL(fd_ed25519_sort_scatter_kernel, gs, dim3(blk), 0, st, *p);
    }
    hipLaunchKernelGGL(fd_ed25519_hash_kernel, g, dim3(blk), 0, st, *p);
  } break;
  case FD_ED25519_PHASE_SCALAR: {
    if (p->small) break;   /* in the prep kernel */
    /* fix_cnt and the dsm work counter, adjacent words */
    const hipError_t e = hipMemsetAsync(p->fix_cnt, 0, 2 * sizeof(uint32_t), st);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(fd_ed25519_scalar_kernel, dim3((uint32_t)((p->n + blk - 1) / blk)), dim3(blk), 0, st, *p);
  } break;
  case FD_ED25519_PHASE_DECODE:
    if (p->small) break;   /* in the prep kernel */
    hipLaunchKernelGGL(fd_ed25519_decode_kernel, dim3((uint32_t)((2 * p->n + blk - 1) / blk)), dim3(blk), 0, st,
                       *p);
    break;
  case FD_ED25519_PHASE_DSM: {
    if (p->small) {
      /* a quad / two quads / two waves per signature, then the (rare)
         full-length items, found by a scan of the flags -- unless prep16
         ran them (full_in_prep) */
      const bool compact = p->bw_bits == FD_ED25519_BTABC_BITS;
      const dim3 g8((uint32_t)((8 * p->n + 255) / 256)), g4((uint32_t)((4 * p->n + 255) / 256));
      if (p->small == 3) {
        const dim3 g16((uint32_t)p->n);
        if (compact) hipLaunchKernelGGL(fd_ed25519_dsm16_kernel<FD_ED25519_BTABC_BITS>, g16, dim3(128), 0, st, *p);
        else         hipLaunchKernelGGL(fd_ed25519_dsm16_kernel<FD_ED25519_BTABW_BITS>, g16, dim3(128), 0, st, *p);
        if (p->full_in_prep || p->hs_host) break;   /* the full-length items were done in prep16, or there are
                                                       none (host scalars): no scan */
      } else if (p->small == 2) {
        if (compact) hipLaunchKernelGGL(fd_ed25519_dsm8_kernel<FD_ED25519_BTABC_BITS>, g8, dim3(256), 0, st, *p);
        else         hipLaunchKernelGGL(fd_ed25519_dsm8_kernel<FD_ED25519_BTABW_BITS>, g8, dim3(256), 0, st, *p);
      } else {
        if (compact) hipLaunchKernelGGL(fd_ed25519_dsm4_kernel<FD_ED25519_BTABC_BITS>, g4, dim3(256), 0, st, *p);
        else         hipLaunchKernelGGL(fd_ed25519_dsm4_kernel<FD_ED25519_BTABW_BITS>, g4, dim3(256), 0, st, *p);
      }
      const uint64_t need = (p->n + FD_ED25519_VERIFY_BLOCK - 1) / FD_ED25519_VERIFY_BLOCK;
      const uint32_t g = (uint32_t)(need < grid ? need : grid);
      if (compact) hipLaunchKernelGGL(fd_ed25519_dsm_kernel<FD_ED25519_BTABC_BITS>, dim3(g), dim3(FD_ED25519_VERIFY_BLOCK), 0, st, *p);
      else         hipLaunchKernelGGL(fd_ed25519_dsm_kernel<FD_ED25519_BTABW_BITS>, dim3(g), dim3(FD_ED25519_VERIFY_BLOCK), 0, st, *p);
      break;
    }
    /* one wave more than the chunk needs: the full-length items (counted on
       the device) run in waves of their own, in parallel with the rest */
    const uint64_t need = (p->n + 64 + FD_ED25519_VERIFY_BLOCK - 1) / FD_ED25519_VERIFY_BLOCK;
    const uint32_t g = (uint32_t)(need < grid ? need : grid);
    if (p->bw_bits == FD_ED25519_BTABC_BITS)
      hipLaunchKernelGGL(fd_ed25519_dsm_kernel<FD_ED25519_BTABC_BITS>, dim3(g), dim3(FD_ED25519_VERIFY_BLOCK), 0, st, *p);
    else
      hipLaunchKernelGGL(fd_ed25519_dsm_kernel<FD_ED25519_BTABW_BITS>, dim3(g), dim3(FD_ED25519_VERIFY_BLOCK), 0, st, *p);
  } break;
  default:
    return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

extern "C" int fd_ed25519_hip_launch_verify(const fd_ed25519_verify_params_t* p, uint32_t grid, void* stream) {
  for (int ph = 0; ph < FD_ED25519_PHASE_CNT; ph++) {
    const int err = fd_ed25519_hip_launch_phase(p, ph, grid, stream);
    if (err) return err;
  }
  return 0;
}

extern "C" unsigned long fd_ed25519_hip_atab_bytes_per_wave(void) { return FD_ED25519_ATAB_BYTES_PER_WAVE; }

extern "C" int fd_ed25519_hip_verify_occupancy(int* blocks_per_cu) {
  return (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, fd_ed25519_dsm_kernel<FD_ED25519_BTABW_BITS>,
                                                           FD_ED25519_VERIFY_BLOCK, 0);
}

extern "C" int fd_ed25519_hip_launch_txn_combine(const int8_t* d_sig_codes, const uint32_t* d_txn_first,
                                                 const uint32_t* d_txn_cnt, int8_t* d_txn_out, uint64_t ntxn,
                                                 void* stream) {
  if (!ntxn) return 0;
  const uint32_t blk = 256;
  const uint32_t grid = (uint32_t)((ntxn + blk - 1) / blk);
  hipLaunchKernelGGL(fd_ed25519_txn_combine_kernel, dim3(grid), dim3(blk), 0, (hipStream_t)stream,
                     d_sig_codes, d_txn_first, d_txn_cnt, d_txn_out, ntxn);
  return (int)hipGetLastError();
}
