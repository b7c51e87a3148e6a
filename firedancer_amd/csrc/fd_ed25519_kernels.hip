/* fd_ed25519_kernels.hip -- gfx950 kernels behind libfd_ed25519_hip.

   Verification of a batch: every step of fd_ed25519_verify
   (src/ballet/ed25519/fd_ed25519_user.c:134-229) for every signature, with
   the verdict computed as data (no early exits, so a wave never diverges on
   an invalid signature), in three phase kernels (see "Phase kernels"):

     1. S < L                          (fd_curve25519_scalar_validate)
     2. decode A and R, reject on no square root (and, in AVX-512 code mode,
        x == 0 with the sign bit set)  (fd_ed25519_point_frombytes_2x)
     3. small-order A, then R          (fd_ed25519_affine_is_small_order)
     4. k = SHA-512(R||A||M) mod L     (fd_sha512_*, fd_curve25519_scalar_reduce)
     5. R' = [k](-A) + [S]B            (fd_ed25519_double_scalar_mul_base)
     6. R' == R projectively           (fd_ed25519_point_eq_z1)

   Steps 2-3 for R and step 6 are done together, without decompressing R,
   by comparing the encoding of R' with R's bytes (fin, below).

   Step 5 uses fixed signed windows instead of the reference's sliding
   wNAF so that every lane of a wave executes the same additions: k in
   radix 16 (64 digits in [-8,8], table [0..8](-A) per lane in HBM) and S in
   radix 256 (32 digits in [-128,128], table [0..128]B shared in LDS).  The
   group element computed is the same, so the verdict is bit-identical.

   The dsm kernel is persistent: its grid is sized to the resident occupancy
   and each lane strides over signatures, so the per-lane -A table lives in
   a fixed HBM scratch of waves x 90 KiB. */
#include <hip/hip_runtime.h>
#include "fd25519_dsm.h"
#include "fd25519_sc.h"
#include "fd_sha512_dev.h"


/* ------------------------------------------------------------------------
   Phase kernels.  A batch is verified by four phases on one stream, each
   kernel with its own register budget, handing ~240 B per signature
   through the work arrays in HBM (fd_ed25519_verify_params_t):

     hash    one lane per signature: S < L, k = SHA-512(R||A||M) mod L
     decode  one lane per public key A: decompression and the reference's
             acceptance / small-order rules
     dsm     one lane per signature, persistent: R' = [k](-A) + [S]B,
             written projective with the S / A status
     fin     R' in affine by per-lane batched inversion, compared with R's
             encoding; rfix decodes R for the few signatures that need it */

#define FD_PF_FAIL  1u
#define FD_PF_SMALL 2u

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

__global__ void __launch_bounds__(256) fd_ed25519_sort_hist_kernel(fd_ed25519_verify_params_t p) {
  __shared__ uint32_t h[FD_ED25519_SORT_BUCKETS];
  if (threadIdx.x < FD_ED25519_SORT_BUCKETS) h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < p.n) atomicAdd(&h[nblk_bucket(p.msg_sz[p.base + j])], 1u);
  __syncthreads();
  if (threadIdx.x < FD_ED25519_SORT_BUCKETS && h[threadIdx.x]) atomicAdd(&p.hist[threadIdx.x], h[threadIdx.x]);
}

__global__ void fd_ed25519_sort_scan_kernel(fd_ed25519_verify_params_t p) {
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int b = 0; b < FD_ED25519_SORT_BUCKETS; b++) {
      p.hist[FD_ED25519_SORT_BUCKETS + b] = acc;  /* cursor = exclusive prefix */
      acc += p.hist[b];
    }
  }
}

__global__ void __launch_bounds__(256) fd_ed25519_sort_scatter_kernel(fd_ed25519_verify_params_t p) {
  __shared__ uint32_t cnt[FD_ED25519_SORT_BUCKETS], base[FD_ED25519_SORT_BUCKETS];
  if (threadIdx.x < FD_ED25519_SORT_BUCKETS) cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t b = 0, r = 0;
  if (j < p.n) {
    b = nblk_bucket(p.msg_sz[p.base + j]);
    r = atomicAdd(&cnt[b], 1u);
  }
  __syncthreads();
  if (threadIdx.x < FD_ED25519_SORT_BUCKETS && cnt[threadIdx.x])
    base[threadIdx.x] = atomicAdd(&p.hist[FD_ED25519_SORT_BUCKETS + threadIdx.x], cnt[threadIdx.x]);
  __syncthreads();
  if (j < p.n) p.perm[base[b] + r] = (uint32_t)j;
}

__global__ void __launch_bounds__(256, FD_ED25519_HASH_WAVES_PER_SIMD)
fd_ed25519_hash_kernel(fd_ed25519_verify_params_t p) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= p.n) return;
  const uint64_t j = p.perm ? (uint64_t)p.perm[t] : t;
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
  const uintptr_t mp = reinterpret_cast<uintptr_t>(p.msgs + p.msg_off[i]);
  sha_msg_src m;
  m.base = reinterpret_cast<const uint32_t*>(mp & ~(uintptr_t)3);
  m.shift = (uint32_t)(mp & 3);
  m.sz = p.msg_sz[i];
  uint32_t dig[16], k[8];
  sha512_ram(dig, r, a, m);
  sc_reduce512(k, dig);
#pragma unroll
  for (int w = 0; w < 8; w++) p.k[(uint64_t)w * p.cap + j] = k[w];
  p.sflag[j] = sc_is_canonical(S) ? 1 : 0;
}

/* One lane per public key A: decompression with the reference's acceptance
   rules and the small-order test.  R is never decompressed on the common
   path: fin compares the encoding of R' = [k](-A) + [S]B with R's bytes
   (see fd_ed25519_fin_kernel). */
__global__ void __launch_bounds__(256, FD_ED25519_DECODE_WAVES_PER_SIMD)
fd_ed25519_decode_kernel(fd_ed25519_verify_params_t p) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= p.n) return;
  const uint64_t i = p.base + j;
  uint32_t s[8];
  {
    const uint4* src = reinterpret_cast<const uint4*>(p.pubs + 32 * i);
    const uint4 q0 = src[0], q1 = src[1];
    s[0] = q0.x; s[1] = q0.y; s[2] = q0.z; s[3] = q0.w; s[4] = q1.x; s[5] = q1.y; s[6] = q1.z; s[7] = q1.w;
  }
  decoded_pt d;
  ge_decode(d, s, !p.codes_portable);
  int32_t* dst = p.pts + j;
#pragma unroll
  for (int l = 0; l < 10; l++) {
    dst[(uint64_t)l * p.cap] = d.x.v[l];
    dst[(uint64_t)(10 + l) * p.cap] = d.y.v[l];
  }
  p.pflag[j] = (uint8_t)((d.fail ? FD_PF_FAIL : 0u) | (d.small ? FD_PF_SMALL : 0u));
}

FD_DEV void load_fe(fe& x, const int32_t* src, uint64_t cap) {
#pragma unroll
  for (int l = 0; l < 10; l++) x.v[l] = src[(uint64_t)l * cap];
}

FD_DEV void store_fe(int32_t* dst, uint64_t cap, const fe& x) {
#pragma unroll
  for (int l = 0; l < 10; l++) dst[(uint64_t)l * cap] = x.v[l];
}

/* R' = [k](-A) + [S]B for signature j, written to proj as (X:Y:Z), plus the
   status that fin finishes.  The reference's checks in order
   (fd_ed25519_user.c:134-229): S < L, A and R decode (an undecodable A is
   ERR_SIG with AVX-512 codes, ERR_PUBKEY with portable ones; R: ERR_SIG),
   A small order (ERR_PUBKEY), R small order (ERR_SIG), the group equation
   (ERR_MSG).  Here S and A are decided; everything about R is left to fin. */
FD_DEV void dsm_one(const fd_ed25519_verify_params_t& p, uint64_t j, int4* lane_tab, const int4* s_btab) {
  const uint64_t i = p.base + j;
  const uint32_t s_ok = p.sflag[j];
  const uint32_t af = p.pflag[j];
  int st;
  if (!s_ok) st = FD_ED25519_ERR_SIG;
  else if (af & FD_PF_FAIL) st = p.codes_portable ? FD_ED25519_ERR_PUBKEY : FD_ED25519_ERR_SIG;
  else if (af & FD_PF_SMALL) st = FD_ST_ASMALL;
  else st = FD_ST_CHECK;

  /* table [0..8](-A), cached form, in this lane's HBM slot */
  {
    fe ax, ay;
    load_fe(ax, p.pts + j, p.cap);
    load_fe(ay, p.pts + 10 * p.cap + j, p.cap);
    ge_p3 nA;
    fe_neg(nA.X, ax);
    nA.Y = ay;
    fe_1(nA.Z);
    fe t;
    fe_mul(t, ax, ay);
    fe_neg(nA.T, t);
    ge_cached c1, c;
    c.YplusX = nA.Z; c.YminusX = nA.Z; c.Z = nA.Z; fe_0(c.T2d);  /* identity */
    atab_store(lane_tab, 0, c);
    ge_p3_to_cached(c1, nA);
    atab_store(lane_tab, 1, c1);
    ge_p3 cur = nA;
    ge_p1p1 sum;
#pragma clang loop unroll(disable)
    for (int e = 2; e <= 8; e++) {
      ge_add(sum, cur, c1);
      ge_p1p1_to_p3(cur, sum);
      ge_p3_to_cached(c, cur);
      atab_store(lane_tab, e, c);
    }
  }

  uint32_t kd[8], sd[8];
  {
    uint32_t k[8], S[8];
#pragma unroll
    for (int w = 0; w < 8; w++) k[w] = p.k[(uint64_t)w * p.cap + j];
    const uint4* sg = reinterpret_cast<const uint4*>(p.sigs + 64 * i);
    const uint4 q2 = sg[2], q3 = sg[3];
    S[0] = q2.x; S[1] = q2.y; S[2] = q2.z; S[3] = q2.w; S[4] = q3.x; S[5] = q3.y; S[6] = q3.z; S[7] = q3.w;
    /* a rejected S may be >= L; keep the recoding in range (the verdict is
       already decided for this lane) */
    if (!s_ok) {
#pragma unroll
      for (int w = 0; w < 8; w++) S[w] = 0;
    }
    recode_radix16(kd, k);
#if FD_ED25519_BWIN == 16
    recode_radix65536(sd, S);
#else
    recode_radix256(sd, S);
#endif
  }
#if FD_ED25519_BWIN == 16
  const int4* g_btab16 = reinterpret_cast<const int4*>(p.btab16);
#endif

  ge_p3 P;
  ge_p3_0(P);
  ge_p1p1 Rt;
  ge_p2 Q;
#pragma clang loop unroll(disable)
  for (int it = 63; it >= 0; it--) {
#if FD_ED25519_BWIN == 16
    /* every 4th k-window adds a B entry: its HBM/L2 load is issued here,
       before the window's doublings, so their ~28 field operations cover
       the latency */
    const bool badd = (it & 3) == 0;
    int f = 0;
    ge_precomp b;
    if (badd) {
      f = pop_digit<16>(sd);
      btab16_load(b, g_btab16, f < 0 ? -f : f);
    }
#else
    const bool badd = (it & 1) == 0;
#endif
    if (it != 63) {
#pragma clang loop unroll(disable)
      for (int dd = 0; dd < 4; dd++) {
        ge_p2_dbl(Rt, Q);
        if (dd < 3) ge_p1p1_to_p2(Q, Rt);
      }
      ge_p1p1_to_p3(P, Rt);
    }
    {
      const int e = pop_digit<4>(kd);
      ge_cached c;
      atab_load(c, lane_tab, e < 0 ? -e : e);
      ge_cached_cneg(c, e < 0);
      ge_add(Rt, P, c);
    }
    if (badd) {
      ge_p1p1_to_p3(P, Rt);
#if FD_ED25519_BWIN != 16
      const int f = pop_digit<8>(sd);
      ge_precomp b;
      btab_load(b, s_btab, f < 0 ? -f : f);
#endif
      ge_precomp_cneg(b, f < 0);
      ge_madd(Rt, P, b);
    }
    ge_p1p1_to_p2(Q, Rt);
  }

  /* A decided lane publishes Z = 1 so that it cannot zero fin's batched
     inversion (an undecodable A is not a curve point, so its R' is not
     either).  For a curve point the complete formulas never give Z = 0. */
  if (st < 0) {
    fe_0(Q.X);
    fe_1(Q.Y);
    fe_1(Q.Z);
  }
  int32_t* dst = p.proj + j;
  store_fe(dst, p.cap, Q.X);
  store_fe(dst + 10 * p.cap, p.cap, Q.Y);
  store_fe(dst + 20 * p.cap, p.cap, Q.Z);
  p.st[j] = (int8_t)st;
}

__global__ void __launch_bounds__(FD_ED25519_VERIFY_BLOCK, FD_ED25519_DSM_WAVES_PER_SIMD)
fd_ed25519_dsm_kernel(fd_ed25519_verify_params_t p) {
#if FD_ED25519_BWIN == 16
  const int4* s_btab = nullptr;  /* the wide table is read from global memory */
#else
  __shared__ int4 s_btab[FD_ED25519_BTAB_INTS / 4];
  const int4* g_btab = reinterpret_cast<const int4*>(p.btab);
  for (int t = threadIdx.x; t < FD_ED25519_BTAB_INTS / 4; t += blockDim.x) s_btab[t] = g_btab[t];
  __syncthreads();
#endif

  const uint64_t gtid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  int4* lane_tab = reinterpret_cast<int4*>(static_cast<char*>(p.atab) +
                                           (gtid >> 6) * FD_ED25519_ATAB_BYTES_PER_WAVE) + (threadIdx.x & 63) * 90;
  for (uint64_t j = gtid; j < p.n; j += stride) dsm_one(p, j, lane_tab, s_btab);
}

/* ------------------------------------------------------------------------
   fin: the group equation without decompressing R.

   The reference decodes R (a square root, ~265 field operations) and tests
   R' == R projectively (fd_ed25519_point_eq_z1).  Equivalently: R decodes
   to R' exactly when R's bytes are the encoding of R' with y taken mod p
   (decoding y gives x up to sign; R' on the curve proves the root exists;
   the sign bit picks x's parity -- x = 0 with the sign bit set never
   matches, which is the AVX-512 decoder's rejection).  So each signature
   needs R' in affine form, and the inversions are batched per lane with
   Montgomery's trick: FIN_M signatures share one inversion (3 (M-1)
   multiplications + 1 inversion instead of M inversions).

   If the encodings match, R is decodable and equal to R': the verdict is
   ERR_SIG if R has small order (y in {0, 1, -1, y0, y1} -- x = 0 iff
   y = +-1 on the curve) and SUCCESS otherwise.  Otherwise -- and whenever A
   has small order, where the verdict depends on whether R decodes -- the
   signature goes to fix_list and rfix decodes R the reference's way.  Only
   invalid signatures take that path. */

FD_DEV bool r_encoding_small(const uint32_t (&y)[8]) {
  const uint32_t y0[8] = {0x8f95e826u, 0xb027b2c2u, 0x89f4c345u, 0xf098eff2u,
                          0x05acdfd5u, 0x3933c6d3u, 0x880238b1u, 0x05fc536du};
  const uint32_t y1[8] = {0x706a17c7u, 0x4fd84d3du, 0x760b3cbau, 0x0f67100du,
                          0xfa53202au, 0xc6cc392cu, 0x77fdc74eu, 0x7a03ac92u};
  uint32_t hi = 0, e0 = 0, e1 = 0, ones = 0;
#pragma unroll
  for (int w = 0; w < 8; w++) {
    if (w) hi |= y[w];
    e0 |= y[w] ^ y0[w];
    e1 |= y[w] ^ y1[w];
    if (w && w < 7) ones |= ~y[w];
  }
  const bool y01 = hi == 0u && y[0] <= 1u;                               /* 0, 1  */
  const bool ym1 = ones == 0u && y[7] == 0x7fffffffu && y[0] == 0xffffffecu;  /* p - 1 */
  return y01 || ym1 || e0 == 0u || e1 == 0u;
}

__global__ void __launch_bounds__(256)
fd_ed25519_fin_kernel(fd_ed25519_verify_params_t p) {
  constexpr int M = FD_ED25519_FIN_M;
  const uint64_t lanes = (p.n + M - 1) / M;
  const uint64_t L = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (L >= lanes) return;
  const int32_t* PX = p.proj;
  const int32_t* PY = p.proj + 10 * p.cap;
  const int32_t* PZ = p.proj + 20 * p.cap;

  fe pre[M];  /* prefix products of Z */
#pragma unroll
  for (int t = 0; t < M; t++) {
    const uint64_t j = L + (uint64_t)t * lanes;
    fe z;
    if (j < p.n) load_fe(z, PZ + j, p.cap);
    else fe_1(z);
    if (t == 0) pre[0] = z;
    else fe_mul(pre[t], pre[t - 1], z);
  }
  fe inv;
  fe_invert(inv, pre[M - 1]);

#pragma unroll
  for (int t = M - 1; t >= 0; t--) {
    const uint64_t j = L + (uint64_t)t * lanes;
    const bool live = j < p.n;
    fe zi;
    if (t > 0) {
      fe_mul(zi, inv, pre[t - 1]);
      fe z;
      if (live) load_fe(z, PZ + j, p.cap);
      else fe_1(z);
      fe_mul(inv, inv, z);
    } else {
      zi = inv;
    }
    if (!live) continue;
    const int st = p.st[j];
    int code;
    if (st < 0) {
      code = st;
    } else if (st == FD_ST_ASMALL) {
      code = 1;  /* R decode needed */
    } else {
      fe x, y, X, Y;
      load_fe(X, PX + j, p.cap);
      load_fe(Y, PY + j, p.cap);
      fe_mul(x, X, zi);
      fe_mul(y, Y, zi);
      uint32_t xb[8], yb[8], r[8];
      fe_tobytes(xb, x);
      fe_tobytes(yb, y);
      {
        const uint4* sg = reinterpret_cast<const uint4*>(p.sigs + 64 * (p.base + j));
        const uint4 q0 = sg[0], q1 = sg[1];
        r[0] = q0.x; r[1] = q0.y; r[2] = q0.z; r[3] = q0.w; r[4] = q1.x; r[5] = q1.y; r[6] = q1.z; r[7] = q1.w;
      }
      const uint32_t sign = r[7] >> 31;
      r[7] &= 0x7fffffffu;
      /* y >= p (only 2^255-19 .. 2^255-1) is taken mod p, as the decoder does */
      uint32_t allf = 0xffffffffu;
#pragma unroll
      for (int w = 1; w < 7; w++) allf &= r[w];
      const bool ge_p = allf == 0xffffffffu && r[7] == 0x7fffffffu && r[0] >= 0xffffffedu;
      if (ge_p) {
        r[0] -= 0xffffffedu;
#pragma unroll
        for (int w = 1; w < 8; w++) r[w] = 0u;
      }
      uint32_t diff = (xb[0] & 1u) ^ sign;
#pragma unroll
      for (int w = 0; w < 8; w++) diff |= yb[w] ^ r[w];
      if (diff == 0u) code = r_encoding_small(yb) ? FD_ED25519_ERR_SIG : FD_ED25519_SUCCESS;
      else code = 1;
    }
    if (code == 1) {
      const uint32_t slot = atomicAdd(p.fix_cnt, 1u);
      p.fix_list[slot] = (uint32_t)j;
    } else {
      p.out[p.base + j] = (int8_t)code;
    }
  }
}

/* rfix: decode R the reference's way for the signatures fin could not
   settle (invalid ones, and those with a small-order A).  Persistent grid;
   the list length is read on the device. */
__global__ void __launch_bounds__(256, FD_ED25519_DECODE_WAVES_PER_SIMD)
fd_ed25519_rfix_kernel(fd_ed25519_verify_params_t p) {
  const uint32_t cnt = *p.fix_cnt;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < cnt;
       t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t j = p.fix_list[t];
    uint32_t s[8];
    {
      const uint4* sg = reinterpret_cast<const uint4*>(p.sigs + 64 * (p.base + j));
      const uint4 q0 = sg[0], q1 = sg[1];
      s[0] = q0.x; s[1] = q0.y; s[2] = q0.z; s[3] = q0.w; s[4] = q1.x; s[5] = q1.y; s[6] = q1.z; s[7] = q1.w;
    }
    decoded_pt d;
    ge_decode(d, s, !p.codes_portable);
    int code;
    if (d.fail) code = FD_ED25519_ERR_SIG;
    else if (p.st[j] == FD_ST_ASMALL) code = FD_ED25519_ERR_PUBKEY;
    else if (d.small) code = FD_ED25519_ERR_SIG;
    else code = FD_ED25519_ERR_MSG;  /* R decodes, is not small, and R' != R */
    p.out[p.base + j] = (int8_t)code;
  }
}

/* ------------------------------------------------------------------------
   Base tables [0..entries)B as (y+x, y-x, 2dxy), one entry per lane:
   [e]B by double-and-add over `bits` bits, then affine. */

__global__ void fd_ed25519_gen_btab_kernel(int32_t* btab, int entries, int stride, int bits) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= entries) return;
  ge_p3 B, P;
  const fe bx = {FE_BX}, by = {FE_BY}, d2 = {FE_D2};
  B.X = bx; B.Y = by; fe_1(B.Z); fe_mul(B.T, bx, by);
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

/* ------------------------------------------------------------------------
   C-ABI launchers */

extern "C" int fd_ed25519_hip_launch_gen_btab(int32_t* d_btab, void* stream) {
  hipLaunchKernelGGL(fd_ed25519_gen_btab_kernel, dim3(3), dim3(64), 0, (hipStream_t)stream, d_btab,
                     FD_ED25519_BTAB_ENTRIES, FD_ED25519_BTAB_STRIDE, 8);
  return (int)hipGetLastError();
}

extern "C" int fd_ed25519_hip_launch_gen_btab16(int32_t* d_btab16, void* stream) {
  const int entries = FD_ED25519_BTAB16_ENTRIES;
  hipLaunchKernelGGL(fd_ed25519_gen_btab_kernel, dim3((entries + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     d_btab16, entries, FD_ED25519_BTAB16_STRIDE, 16);
  return (int)hipGetLastError();
}

extern "C" int fd_ed25519_hip_launch_phase(const fd_ed25519_verify_params_t* p, int phase, uint32_t grid,
                                           void* stream) {
  if (!p->n) return 0;
  hipStream_t st = (hipStream_t)stream;
  const uint32_t blk = 256;
  switch (phase) {
  case FD_ED25519_PHASE_HASH: {
    const dim3 g((uint32_t)((p->n + blk - 1) / blk));
    if (p->perm) {
      const hipError_t e = hipMemsetAsync(p->hist, 0, 2 * FD_ED25519_SORT_BUCKETS * sizeof(uint32_t), st);
      if (e != hipSuccess) return (int)e;
      hipLaunchKernelGGL(fd_ed25519_sort_hist_kernel, g, dim3(blk), 0, st, *p);
      hipLaunchKernelGGL(fd_ed25519_sort_scan_kernel, dim3(1), dim3(64), 0, st, *p);
      hipLaunchKernelGGL(fd_ed25519_sort_scatter_kernel, g, dim3(blk), 0, st, *p);
    }
    hipLaunchKernelGGL(fd_ed25519_hash_kernel, g, dim3(blk), 0, st, *p);
  } break;
  case FD_ED25519_PHASE_DECODE:
    hipLaunchKernelGGL(fd_ed25519_decode_kernel, dim3((uint32_t)((p->n + blk - 1) / blk)), dim3(blk), 0, st, *p);
    break;
  case FD_ED25519_PHASE_DSM: {
    const uint64_t need = (p->n + FD_ED25519_VERIFY_BLOCK - 1) / FD_ED25519_VERIFY_BLOCK;
    const uint32_t g = (uint32_t)(need < grid ? need : grid);
    hipLaunchKernelGGL(fd_ed25519_dsm_kernel, dim3(g), dim3(FD_ED25519_VERIFY_BLOCK), 0, st, *p);
  } break;
  case FD_ED25519_PHASE_FIN: {
    const hipError_t e = hipMemsetAsync(p->fix_cnt, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return (int)e;
    const uint64_t lanes = (p->n + FD_ED25519_FIN_M - 1) / FD_ED25519_FIN_M;
    hipLaunchKernelGGL(fd_ed25519_fin_kernel, dim3((uint32_t)((lanes + blk - 1) / blk)), dim3(blk), 0, st, *p);
    const uint64_t need = (p->n + blk - 1) / blk;
    hipLaunchKernelGGL(fd_ed25519_rfix_kernel, dim3((uint32_t)(need < 1024 ? need : 1024)), dim3(blk), 0, st, *p);
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

extern "C" int fd_ed25519_hip_verify_occupancy(int* blocks_per_cu) {
  return (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, fd_ed25519_dsm_kernel,
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
