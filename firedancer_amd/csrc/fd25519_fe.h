/* fd25519_fe.h -- GF(2^255-19) arithmetic for gfx950, one field element
   per lane in ten signed 32-bit limbs (radix 2^25.5: limb i holds bits
   [ceil(25.5 i), ceil(25.5 (i+1)) ), 26 bits for even i, 25 for odd).

   Why this shape on MI355X: the products are 32x32->64 signed
   multiply-accumulates, which hipcc lowers to one v_mad_i64_i32 each (a
   VOP3 op that issues at half the rate of a plain VALU add on gfx950,
   measured in tools/ubench/int_ubench.hip -- the same issue cost as a
   24-bit multiply and cheaper than an f64 FMA).  A full product is 100 of
   them plus a 12-step carry chain; a square 55.  Nothing here is a dense
   contraction, so MFMA is not used.

   Semantics follow the field API of the reference
   (src/ballet/ed25519/fd_f25519.h:46-253): frombytes ignores bit 255 and
   accepts non-canonical values (>= p), comparisons are on canonical
   encodings.

   Bound discipline (|limb| relative to 2^25 even / 2^24 odd):
     tight  (outputs of mul/sq/carry, constants)  <= 1.01x
     add/sub of two tight values                   <= 2.02x
     add/sub of a tight and a 2.02x value          <= 3.03x
   mul/sq accept inputs <= 3.3x (|limb| < 1.65*2^26 / 1.65*2^25): every
   product term fits in a signed 32-bit operand (19*1.65*2^26 < 2^31) and
   every 64-bit column sum stays below 2^63. */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define FD_DEV __device__ __forceinline__

struct fe { int32_t v[10]; };

/* Constants in centered limbs (tight). */
#define FE_D      {-10913610, 13857413, -15372611, 6949391, 114729, -8787816, -6275908, -3247719, -18696448, -12055116}
#define FE_D2     {-21827239, -5839606, -30745221, 13898782, 229458, 15978800, -12551817, -6495438, 29715968, 9444199}
#define FE_DINV   {30013526, 3972531, -24787780, 12719051, 2979674, -4599962, -15693209, -3644061, 18959709, -16629253}
#define FE_SQRTM1 {-32595792, -7943725, 9377950, 3500415, 12389472, -272473, -25146209, -2005654, 326686, 11406482}
#define FE_BX     {-14297830, -7645148, 16144683, -16471763, 27570974, -2696100, -26142465, 8378389, 20764389, 8758491}
#define FE_BY     {-26843541, -6710886, 13421773, -13421773, 26843546, 6710886, -13421773, 13421773, -26843546, -6710886}

FD_DEV void fe_set_const(fe& h, const int32_t (&c)[10]) {
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = c[i];
}

FD_DEV void fe_0(fe& h) {
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = 0;
}

FD_DEV void fe_1(fe& h) {
  fe_0(h);
  h.v[0] = 1;
}

FD_DEV void fe_add(fe& h, const fe& f, const fe& g) {
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = f.v[i] + g.v[i];
}

FD_DEV void fe_sub(fe& h, const fe& f, const fe& g) {
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = f.v[i] - g.v[i];
}

FD_DEV void fe_neg(fe& h, const fe& f) {
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = -f.v[i];
}

/* h = c ? g : f  (per-lane select, no branch) */
FD_DEV void fe_select(fe& h, const fe& f, const fe& g, bool c) {
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = c ? g.v[i] : f.v[i];
}

/* Rounding bias of column k: the carry out of a centered limb is
   (a + 2^(w-1)) >> w.  Accumulators start at this bias (it rides along the
   multiply-accumulate chain for free), so each carry step is one 64-bit
   shift and one 64-bit add, and the limb is (low bits) - bias. */
#define FE_BIAS(k) (((k) & 1) ? (1LL << 24) : (1LL << 25))

/* One 32x32->64 signed multiply-accumulate, v_mad_i64_i32, written as
   inline asm so that LLVM cannot reassociate the column sums: left to
   itself it moves the (constant) bias of every column to a separate 64-bit
   add, one extra v_lshl_add_u64 per column and product.  fe_mad_init
   starts a column with its bias as the addend (an SGPR pair).  The carry-out
   SGPR pair the instruction writes is a dead scratch output.
   FE_ASM_MAD=0 restores the plain C (for A/B builds). */
#ifndef FE_ASM_MAD
#define FE_ASM_MAD 1
#endif

/* How the unsigned-limb forms (below) pin their accumulation order.
   FE_USE_BARRIER=0: asm("" : "+v"(acc)) after each multiply-add, like the
   centered forms.  FE_USE_BARRIER=1: a use-only asm (acc is read, not
   redefined).  Both keep every partial sum as its own value, so LLVM
   cannot reassociate the column; but an asm that *defines* a VGPR counts
   as a possible dst-forwarding producer for gfx950's hazard recognizer,
   which then puts an s_nop before the next instruction that reads it (one
   per multiply-add pair wherever the scheduler groups two barriers: 2353
   in the dsm kernel, 821 in decode).  The use-only form leaves 141 and
   122: dsm 7.82 -> 7.75 ms per 1M, decode unchanged (interleaved A/B x3,
   profiles/r3_ab_use_barrier.txt).  The centered forms keep the defining
   barrier: the use-only form there makes decode spill 3.4 KB per lane. */
#ifndef FE_USE_BARRIER
#define FE_USE_BARRIER 1
#endif
#if FE_USE_BARRIER
#define FE_ACC_BARRIER_U(acc) asm volatile("" ::"v"(acc))
#else
#define FE_ACC_BARRIER_U(acc) asm("" : "+v"(acc))
#endif

FD_DEV void fe_mad(int64_t& acc, int32_t x, int32_t y) {
  acc += (int64_t)x * y;
#if FE_ASM_MAD
  asm("" : "+v"(acc));
#endif
}

FD_DEV void fe_mad_init(int64_t& acc, int32_t x, int32_t y, int k) {
  acc = FE_BIAS(k) + (int64_t)x * y;
#if FE_ASM_MAD
  asm("" : "+v"(acc));
#endif
}

/* Column sums a[k] (each pre-biased with FE_BIAS(k)) of a 10x10 product,
   reduced to tight centered limbs in two interleaved chains (limbs 4 and 0
   are carried twice; between their two carries they are kept in biased
   form, so the result equals carrying (a + 2^(w-1)) >> w step by step). */
FD_DEV void fe_carry_wide(fe& h, int64_t (&a)[10]) {
  const int64_t m26 = (1LL << 26) - 1, m25 = (1LL << 25) - 1;
  int64_t c;
  c = a[0] >> 26; a[1] += c; a[0] &= m26;                    /* a0 stays biased */
  c = a[4] >> 26; a[5] += c; a[4] &= m26;                    /* a4 stays biased */
  c = a[1] >> 25; a[2] += c; h.v[1] = (int32_t)(a[1] & m25) - (1 << 24);
  c = a[5] >> 25; a[6] += c; h.v[5] = (int32_t)(a[5] & m25) - (1 << 24);
  c = a[2] >> 26; a[3] += c; h.v[2] = (int32_t)(a[2] & m26) - (1 << 25);
  c = a[6] >> 26; a[7] += c; h.v[6] = (int32_t)(a[6] & m26) - (1 << 25);
  c = a[3] >> 25; a[4] += c; h.v[3] = (int32_t)(a[3] & m25) - (1 << 24);
  c = a[7] >> 25; a[8] += c; h.v[7] = (int32_t)(a[7] & m25) - (1 << 24);
  c = a[4] >> 26; h.v[5] += (int32_t)c; h.v[4] = (int32_t)(a[4] & m26) - (1 << 25);
  c = a[8] >> 26; a[9] += c; h.v[8] = (int32_t)(a[8] & m26) - (1 << 25);
  c = a[9] >> 25; a[0] += c * 19; h.v[9] = (int32_t)(a[9] & m25) - (1 << 24);
  c = a[0] >> 26; h.v[1] += (int32_t)c; h.v[0] = (int32_t)(a[0] & m26) - (1 << 25);
}

/* h = f*g.  Term (i,j) lands in column (i+j) mod 10; it is doubled when i
   and j are both odd (the half-bit of the 25.5 radix) and multiplied by 19
   when it wraps (2^255 = 19 mod p). */
FD_DEV void fe_mul(fe& h, const fe& f, const fe& g) {
  int64_t a[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
#pragma unroll
    for (int j = 0; j < 10; j++) {
      const int k = i + j;
      const int32_t x = ((i & 1) && (j & 1)) ? 2 * f.v[i] : f.v[i];
      const int32_t y = (k >= 10) ? 19 * g.v[j] : g.v[j];
      if (i == 0) fe_mad_init(a[k], x, y, k);
      else fe_mad(a[k >= 10 ? k - 10 : k], x, y);
    }
  }
  fe_carry_wide(h, a);
}

/* 19 g (limbs 1..9; limb 0 never wraps), for products that share g */
FD_DEV void fe_19(fe& g19, const fe& g) {
  g19.v[0] = 0;
#pragma unroll
  for (int j = 1; j < 10; j++) g19.v[j] = 19 * g.v[j];
}

/* h = f*g with 19 g given */
FD_DEV void fe_mul19(fe& h, const fe& f, const fe& g, const fe& g19) {
  int64_t a[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
#pragma unroll
    for (int j = 0; j < 10; j++) {
      const int k = i + j;
      const int32_t x = ((i & 1) && (j & 1)) ? 2 * f.v[i] : f.v[i];
      const int32_t y = (k >= 10) ? g19.v[j] : g.v[j];
      if (i == 0) fe_mad_init(a[k], x, y, k);
      else fe_mad(a[k >= 10 ? k - 10 : k], x, y);
    }
  }
  fe_carry_wide(h, a);
}

/* h = f^2 (55 products): off-diagonal terms carry the factor 2 on the
   left operand, the odd/odd and wrap factors (2, 19, 38) on the right. */
FD_DEV void fe_sq(fe& h, const fe& f) {
  int64_t a[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
#pragma unroll
    for (int j = i; j < 10; j++) {
      const int k = i + j;
      const int m = (((i & 1) && (j & 1)) ? 2 : 1) * ((k >= 10) ? 19 : 1);
      const int32_t x = (i == j) ? f.v[i] : 2 * f.v[i];
      const int32_t y = m * f.v[j];
      if (i == 0) fe_mad_init(a[k], x, y, k);
      else fe_mad(a[k >= 10 ? k - 10 : k], x, y);
    }
  }
  fe_carry_wide(h, a);
}

/* h = 2 f^2 */
FD_DEV void fe_sq2(fe& h, const fe& f) {
  int64_t a[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
#pragma unroll
    for (int j = i; j < 10; j++) {
      const int k = i + j;
      const int m = (((i & 1) && (j & 1)) ? 2 : 1) * ((k >= 10) ? 19 : 1);
      const int32_t x = (i == j) ? 2 * f.v[i] : 4 * f.v[i];
      const int32_t y = m * f.v[j];
      if (i == 0) fe_mad_init(a[k], x, y, k);
      else fe_mad(a[k >= 10 ? k - 10 : k], x, y);
    }
  }
  fe_carry_wide(h, a);
}

/* ------------------------------------------------------------------------
   Unsigned-limb forms (suffix _u): the same products, reduced with floor
   carries, so the output limbs are the plain digits, in [0, 2^w) (limbs 1
   and 6 within 2^10 of that range): <= 2.0x in the units above, i.e.
   "tight" only in magnitude, not centered.

   Without a rounding bias no column needs a constant, so each column's
   accumulation starts from the previous column's carry -- the carry is the
   addend of the column's first multiply-add -- and the 64-bit add of every
   carry step disappears (9 v_lshl_add_u64 per product), as do the ten
   bias subtractions.  The columns run in two chains (0..4 and 5..9) so two
   multiply-add streams are in flight; the chains are joined by two short
   steps: column 4's carry into limb 5 (re-split into limb 6) and 19 times
   column 9's carry into limb 0 (re-split into limb 1).

   Inputs as for fe_mul / fe_sq (the 19-side <= 3.3x).  The callers keep
   every sum fed to a product within that bound (fd25519_ge.h). */
FD_DEV void fe_join_u(int32_t (&u)[10], int64_t c4, int64_t c9) {
  {
    const int64_t t = c4 + (int64_t)(uint32_t)u[5];
    u[5] = (int32_t)t & ((1 << 25) - 1);
    u[6] += (int32_t)(t >> 25);
  }
  {
    const int64_t t = c9 * 19 + (int64_t)(uint32_t)u[0];
    u[0] = (int32_t)t & ((1 << 26) - 1);
    u[1] += (int32_t)(t >> 26);
  }
}

/* The digits are known non-negative to the compiler, which then splits a
   later signed product into an unsigned multiply-add plus a correction of
   the high word (two instructions and moves instead of one
   v_mad_i64_i32); hiding the range keeps every product one instruction. */
FD_DEV void fe_launder_u(fe& h, int32_t (&u)[10]) {
#pragma unroll
  for (int i = 0; i < 10; i++) {
    asm("" : "+v"(u[i]));
    h.v[i] = u[i];
  }
}

FD_DEV void fe_mul19_u(fe& h, const fe& f, const fe& g, const fe& g19) {
  int32_t u[10];
  int64_t cA = 0, cB = 0;
#pragma unroll
  for (int s = 0; s < 5; s++) {
#pragma unroll
    for (int half = 0; half < 2; half++) {
      const int k = s + 5 * half;
      int64_t acc = half ? cB : cA;
#pragma unroll
      for (int n = 0; n < 10; n++) {
        const int i = n, j = (k - i + 10) % 10;
        const int32_t x = ((i & 1) && (j & 1)) ? 2 * f.v[i] : f.v[i];
        const int32_t y = (i + j >= 10) ? g19.v[j] : g.v[j];
        if (s == 0 && n == 0) acc = (int64_t)x * y;
        else acc += (int64_t)x * y;
#if FE_ASM_MAD
        FE_ACC_BARRIER_U(acc);
#endif
      }
      const int w = (k & 1) ? 25 : 26;
      u[k] = (int32_t)acc & ((1 << w) - 1);
      if (half) cB = acc >> w;
      else cA = acc >> w;
    }
  }
  fe_join_u(u, cA, cB);
  fe_launder_u(h, u);
}

FD_DEV void fe_mul_u(fe& h, const fe& f, const fe& g) {
  fe g19;
  fe_19(g19, g);
  fe_mul19_u(h, f, g, g19);
}

/* h = S f^2, S = 1 or 2 */
template <int S>
FD_DEV void fe_sqs_u(fe& h, const fe& f) {
  int32_t u[10];
  int64_t cA = 0, cB = 0;
#pragma unroll
  for (int s = 0; s < 5; s++) {
#pragma unroll
    for (int half = 0; half < 2; half++) {
      const int k = s + 5 * half;
      int64_t acc = half ? cB : cA;
      bool first = (s == 0);
#pragma unroll
      for (int i = 0; i < 10; i++) {
#pragma unroll
        for (int j = i; j < 10; j++) {
          if ((i + j) % 10 != k) continue;
          const int m = (((i & 1) && (j & 1)) ? 2 : 1) * ((i + j >= 10) ? 19 : 1);
          const int32_t x = (i == j) ? S * f.v[i] : 2 * S * f.v[i];
          const int32_t y = m * f.v[j];
          if (first) acc = (int64_t)x * y;
          else acc += (int64_t)x * y;
          first = false;
#if FE_ASM_MAD
          FE_ACC_BARRIER_U(acc);
#endif
        }
      }
      const int w = (k & 1) ? 25 : 26;
      u[k] = (int32_t)acc & ((1 << w) - 1);
      if (half) cB = acc >> w;
      else cA = acc >> w;
    }
  }
  fe_join_u(u, cA, cB);
  fe_launder_u(h, u);
}

FD_DEV void fe_sq_u(fe& h, const fe& f) { fe_sqs_u<1>(h, f); }
FD_DEV void fe_sq2_u(fe& h, const fe& f) { fe_sqs_u<2>(h, f); }

/* Re-tighten a 32-bit-limb element (e.g. the result of adds/subs). */
FD_DEV void fe_carry(fe& h, const fe& f) {
  int64_t a[10];
#pragma unroll
  for (int i = 0; i < 10; i++) a[i] = (int64_t)f.v[i] + FE_BIAS(i);
  fe_carry_wide(h, a);
}

/* Load 32 little-endian bytes given as 8 words; bit 255 is ignored and
   values >= p are accepted (reduced implicitly by the arithmetic). */
FD_DEV void fe_frombytes(fe& h, const uint32_t (&w)[8]) {
  /* limb offsets 0,26,51,77,102,128,153,179,204,230 */
  const uint32_t m26 = (1u << 26) - 1u, m25 = (1u << 25) - 1u;
  h.v[0] = (int32_t)(w[0] & m26);
  h.v[1] = (int32_t)(__builtin_amdgcn_alignbit(w[1], w[0], 26) & m25);
  h.v[2] = (int32_t)(__builtin_amdgcn_alignbit(w[2], w[1], 19) & m26);
  h.v[3] = (int32_t)(__builtin_amdgcn_alignbit(w[3], w[2], 13) & m25);
  h.v[4] = (int32_t)((w[3] >> 6) & m26);
  h.v[5] = (int32_t)(w[4] & m25);
  h.v[6] = (int32_t)(__builtin_amdgcn_alignbit(w[5], w[4], 25) & m26);
  h.v[7] = (int32_t)(__builtin_amdgcn_alignbit(w[6], w[5], 19) & m25);
  h.v[8] = (int32_t)(__builtin_amdgcn_alignbit(w[7], w[6], 12) & m26);
  h.v[9] = (int32_t)((w[7] >> 6) & m25);
}

/* Canonical little-endian encoding (value mod p, < p) as 8 words.  Any
   input within the mul bounds is accepted: it is re-tightened first so the
   quotient estimate below (valid for |h| < 2^254) is exact. */
FD_DEV void fe_carry(fe& h, const fe& f);
FD_DEV void fe_tobytes(uint32_t (&s)[8], const fe& f) {
  fe g;
  fe_carry(g, f);
  int32_t h[10];
#pragma unroll
  for (int i = 0; i < 10; i++) h[i] = g.v[i];
  /* q = floor(h / p) in {0,1} once h is folded to [0, 2p) */
  int32_t q = (19 * h[9] + (1 << 24)) >> 25;
#pragma unroll
  for (int i = 0; i < 10; i++) q = (h[i] + q) >> ((i & 1) ? 25 : 26);
  h[0] += 19 * q;
  int32_t c;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int sh = (i & 1) ? 25 : 26;
    c = h[i] >> sh;
    h[i + 1] += c;
    h[i] -= c * (1 << sh);
  }
  c = h[9] >> 25;
  h[9] -= c * (1 << 25);
  /* pack: limbs are now in [0, 2^w) */
  const uint32_t u0 = (uint32_t)h[0], u1 = (uint32_t)h[1], u2 = (uint32_t)h[2], u3 = (uint32_t)h[3],
                 u4 = (uint32_t)h[4], u5 = (uint32_t)h[5], u6 = (uint32_t)h[6], u7 = (uint32_t)h[7],
                 u8 = (uint32_t)h[8], u9 = (uint32_t)h[9];
  s[0] = u0 | (u1 << 26);
  s[1] = (u1 >> 6) | (u2 << 19);
  s[2] = (u2 >> 13) | (u3 << 13);
  s[3] = (u3 >> 19) | (u4 << 6);
  s[4] = u5 | (u6 << 25);
  s[5] = (u6 >> 7) | (u7 << 19);
  s[6] = (u7 >> 13) | (u8 << 12);
  s[7] = (u8 >> 20) | (u9 << 6);
}

FD_DEV bool fe_iszero(const fe& f) {
  uint32_t s[8];
  fe_tobytes(s, f);
  return (s[0] | s[1] | s[2] | s[3] | s[4] | s[5] | s[6] | s[7]) == 0u;
}

/* parity of the canonical value (fd_f25519_sgn) */
FD_DEV int fe_isodd(const fe& f) {
  uint32_t s[8];
  fe_tobytes(s, f);
  return (int)(s[0] & 1u);
}

/* z^(2^252-3) -- same addition chain as fd_f25519_pow22523
   (src/ballet/ed25519/fd_f25519.c:11-59): 250 squarings, 11 products, all
   in the unsigned-limb forms (a chain of products only: every input is a
   previous output, <= 2x; the result is unsigned, <= 2x). */
FD_DEV void fe_sqn(fe& h, const fe& f, int n) {
  fe_sq_u(h, f);
#pragma clang loop unroll(disable)
  for (int i = 1; i < n; i++) fe_sq_u(h, h);
}

FD_DEV void fe_pow22523(fe& out, const fe& z) {
  fe t0, t1, t2;
  fe_sq_u(t0, z);
  fe_sqn(t1, t0, 2);
  fe_mul_u(t1, z, t1);
  fe_mul_u(t0, t0, t1);
  fe_sq_u(t0, t0);
  fe_mul_u(t0, t1, t0);
  fe_sqn(t1, t0, 5);
  fe_mul_u(t0, t1, t0);
  fe_sqn(t1, t0, 10);
  fe_mul_u(t1, t1, t0);
  fe_sqn(t2, t1, 20);
  fe_mul_u(t1, t2, t1);
  fe_sqn(t1, t1, 10);
  fe_mul_u(t0, t1, t0);
  fe_sqn(t1, t0, 50);
  fe_mul_u(t1, t1, t0);
  fe_sqn(t2, t1, 100);
  fe_mul_u(t1, t2, t1);
  fe_sqn(t1, t1, 50);
  fe_mul_u(t0, t1, t0);
  fe_sqn(t0, t0, 2);
  fe_mul_u(out, t0, z);
}

/* 1/z = z^(p-2) = (z^(2^252-3))^8 * z^3 */
FD_DEV void fe_invert(fe& out, const fe& z) {
  fe t, z2, z3;
  fe_pow22523(t, z);
  fe_sqn(t, t, 3);
  fe_sq(z2, z);
  fe_mul(z3, z2, z);
  fe_mul(out, t, z3);
}
