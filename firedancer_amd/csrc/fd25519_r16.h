/* fd25519_r16.h -- GF(2^255-19) and edwards25519 spread over the lanes of a
   wave, for the latency form's smallest batches (fd_ed25519_dsm16_kernel).

   One field element per 16-lane DPP row, radix 2^16: lane c (= threadIdx &
   15) holds limb c, an unsigned 32-bit value; the element is
   sum_c l_c 2^(16c) mod p.  A product's column c is computed by lane c,

       col_c = sum_t g_t * f_(c-t mod 16) * (c < t ? 38 : 1)     (2^256 = 38 mod p)

   with, per t, one row broadcast of g_t (v_mov_b32_dpp row_newbcast:t),
   one rotation of f scaled by the lane's wrap factor (v_mul_u32_u24 with
   row_ror:t folded in) and one v_mad_u64_u32 -- 16 multiply-adds per lane
   instead of the one-lane form's 55 (squaring) or 100 (product) -- then
   three carry rounds that move each lane's carry one lane up (row_ror:1,
   lane 0 taking 38 x lane 15's).  Measured on gfx950 with one wave per
   SIMD (tools/ubench/fe_lanesplit_ubench.hip, profiles/r5_lanesplit_ubench.txt):
   a dependent squaring 301 cycles against 485 for fe_sq_u, a product 336
   against 682 for fe_mul_u -- but 10x the lane-work, so only where the
   chip would otherwise idle.

   A point is four rows of one wave: row q holds coordinate q, as lane q of
   a quad does in fd25519_ge4.h.  Each group operation is two rounds of
   four products (one per row); between them every row gets all four
   products of the first round (gfx950's permlane swaps, ge16_dbl2 /
   ge16_add2) and picks its operands with per-row bit selects (ds_bpermute,
   r16_rp, only for the final identity test).

   Bounds (every limb is unsigned; "tight" = < 2^16 + 64):
     r16_mul / r16_sq take limbs < 2^19 and return tight limbs:
       col_c < 571 x 2^38 < 2^47.2; round 1 leaves < 2^16 + 571 x 2^38 / 2^16
       < 2^31.2 in lanes 1..15 and < 2^16 + 38 x 16 x 2^38 / 2^16 < 2^31.3 in
       lane 0 (lane 15's column has no wrapped term); round 2 < 2^16 + 38 x
       2^15.3 in lane 0, < 2^17 elsewhere; round 3 < 2^16 + 38 (lane 0),
       < 2^16 + 2^6 (lane 1), < 2^16 + 1 elsewhere.
     x - y is x + 4p - y for tight y (4p's limbs are 2^17 - 2, lane 0
       2^17 - 76: all above a tight limb, so nothing wraps below zero), and
       x + 8p - y for y < 2^18 - 152 (8p: 2^18 - 4, lane 0 2^18 - 152).
   Each formula below states the bound of what it forms; all stay < 2^19.
   tests/test_r16_model.py restates the arithmetic on Python integers with
   these bounds asserted. */
#pragma once
#include "fd25519_fe.h"

#define R16_BC(x, t)  ((uint32_t)__builtin_amdgcn_mov_dpp((int)(x), 0x150 + (t), 0xf, 0xf, true))   /* row_newbcast:t */
#define R16_ROR(x, t) ((uint32_t)__builtin_amdgcn_mov_dpp((int)(x), 0x120 + (t), 0xf, 0xf, true))   /* row_ror:t      */

/* per-lane constants, made once per kernel.  Everything that differs by
   row is selected with these masks (and, or): a branch on the row would
   make the wave run each row's side in turn. */
struct r16ctx {
  uint32_t m[16];     /* m[t] = 38 if c < t else 1: the wrap factor of term t in lane c */
  uint32_t p4, p8;    /* limb c of 4p / 8p (all limbs positive, above any tight / < 2^18 - 152 limb) */
  uint32_t c;         /* lane in row */
  uint32_t row;       /* row (coordinate) in the wave */
  uint32_t r0, r1, r2, r3, r03, r12;   /* all ones in rows 0 / 1 / 2 / 3 / 0 and 3 / 1 and 2, else 0 */
};

FD_DEV void r16_init(r16ctx& k) {
  k.c = threadIdx.x & 15u;
  k.row = (threadIdx.x >> 4) & 3u;
#pragma unroll
  for (int t = 0; t < 16; t++) k.m[t] = k.c < (uint32_t)t ? 38u : 1u;
  k.p4 = k.c ? (1u << 17) - 2u : (1u << 17) - 76u;
  k.p8 = k.c ? (1u << 18) - 4u : (1u << 18) - 152u;
  k.r0 = 0u - (uint32_t)(k.row == 0u); k.r1 = 0u - (uint32_t)(k.row == 1u);
  k.r2 = 0u - (uint32_t)(k.row == 2u); k.r3 = 0u - (uint32_t)(k.row == 3u);
  k.r03 = k.r0 | k.r3; k.r12 = k.r1 | k.r2;
}

/* three carry rounds of a column sum < 2^47.2 (see the header) */
FD_DEV uint32_t r16_carry(uint64_t acc, const r16ctx& k) {
  uint32_t lo = (uint32_t)acc & 0xffffu;
  uint32_t hi = (uint32_t)(acc >> 16);
  uint32_t l = lo + R16_ROR(hi, 1) * k.m[1];
  hi = l >> 16; lo = l & 0xffffu;
  l = lo + __umul24(R16_ROR(hi, 1), k.m[1]);
  hi = l >> 16; lo = l & 0xffffu;
  return lo + __umul24(R16_ROR(hi, 1), k.m[1]);
}

#define R16_STEP(a, t) a += (uint64_t)R16_BC(g, t) * __umul24(R16_ROR(f, t), k.m[t]);

/* f*g, limbs < 2^19 in, tight out.  Two accumulators in the source; LLVM
   merges them into one dependent chain of multiply-adds, and keeping them
   apart (use-only asm barriers) or four chains measured no faster
   (profiles/r5_ab_r16_routing.txt): the chain is issue-bound. */
FD_DEV uint32_t r16_mul(uint32_t f, uint32_t g, const r16ctx& k) {
  uint64_t acc = (uint64_t)R16_BC(g, 0) * f, acc2 = (uint64_t)R16_BC(g, 1) * __umul24(R16_ROR(f, 1), k.m[1]);
  R16_STEP(acc, 2) R16_STEP(acc2, 3) R16_STEP(acc, 4) R16_STEP(acc2, 5) R16_STEP(acc, 6) R16_STEP(acc2, 7)
  R16_STEP(acc, 8) R16_STEP(acc2, 9) R16_STEP(acc, 10) R16_STEP(acc2, 11) R16_STEP(acc, 12) R16_STEP(acc2, 13)
  R16_STEP(acc, 14) R16_STEP(acc2, 15)
  return r16_carry(acc + acc2, k);
}

FD_DEV uint32_t r16_sq(uint32_t f, const r16ctx& k) { return r16_mul(f, f, k); }

/* row r of the result = row SRC[r] of x (ds_bpermute: any permutation or
   broadcast of the four rows, one instruction) */
template <int S0, int S1, int S2, int S3>
FD_DEV uint32_t r16_rp(uint32_t x, const r16ctx& k) {
  constexpr uint32_t PACK = (uint32_t)(S0 | (S1 << 2) | (S2 << 4) | (S3 << 6));
  const uint32_t src = (PACK >> (2u * k.row)) & 3u;
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)((src << 6) | (k.c << 2)), (int)x);
}

/* Row moves without LDS: gfx950's v_permlane16_swap / v_permlane32_swap
   with both operands x (measured, tools/ubench/permlane_probe.hip):
     swap16 -> e = (x0, x0, x2, x2), o = (x1, x1, x3, x3)
     swap32 -> l = (x0, x1, x0, x1), h = (x2, x3, x2, x3)
   (xq = row q of x), combined with per-row bit selects (v_bfi_b32).  A
   VALU op each, where a ds_bpermute waits on the LDS pipe. */
struct r16_eo { uint32_t e, o; };
struct r16_lh { uint32_t l, h; };

FD_DEV r16_eo r16_swap16(uint32_t x) {
  const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  return {(uint32_t)r[0], (uint32_t)r[1]};
}
FD_DEV r16_lh r16_swap32(uint32_t x) {
  const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return {(uint32_t)r[0], (uint32_t)r[1]};
}

/* bits of a where m, of b elsewhere */
FD_DEV uint32_t r16_bsel(uint32_t m, uint32_t a, uint32_t b) { return (a & m) | (b & ~m); }

/* (x1, x0, x3, x2) */
FD_DEV uint32_t r16_xor1(uint32_t x, const r16ctx& k) {
  const r16_eo s = r16_swap16(x);
  return r16_bsel(k.r1 | k.r3, s.e, s.o);
}

/* ---- conversions with the one-lane radix-2^25.5 form ------------------- */

/* limb c of f's canonical value (every lane runs fe_tobytes: the selects
   pick this lane's 16 bits) */
FD_DEV uint32_t r16_from_fe(const fe& f, const r16ctx& k) {
  uint32_t s[8];
  fe_tobytes(s, f);
  const uint32_t w = k.c >> 1;
  const uint32_t a = (w & 1u) ? s[1] : s[0], b = (w & 1u) ? s[3] : s[2];
  const uint32_t d = (w & 1u) ? s[5] : s[4], e = (w & 1u) ? s[7] : s[6];
  const uint32_t ab = (w & 2u) ? b : a, de = (w & 2u) ? e : d;
  const uint32_t v = (w & 4u) ? de : ab;
  return (k.c & 1u) ? (v >> 16) : (v & 0xffffu);
}

/* 1 in the lanes of rows whose element (limbs < 2^19) is 0 mod p */
FD_DEV bool r16_iszero(uint32_t x) {
  uint32_t l[16];
  l[0] = R16_BC(x, 0); l[1] = R16_BC(x, 1); l[2] = R16_BC(x, 2); l[3] = R16_BC(x, 3);
  l[4] = R16_BC(x, 4); l[5] = R16_BC(x, 5); l[6] = R16_BC(x, 6); l[7] = R16_BC(x, 7);
  l[8] = R16_BC(x, 8); l[9] = R16_BC(x, 9); l[10] = R16_BC(x, 10); l[11] = R16_BC(x, 11);
  l[12] = R16_BC(x, 12); l[13] = R16_BC(x, 13); l[14] = R16_BC(x, 14); l[15] = R16_BC(x, 15);
  /* digits of the value (< 2^259): carry once, fold 2^256 (x 38) and bit 255 (x 19) twice */
  uint64_t acc = 0;
#pragma unroll
  for (int c = 0; c < 16; c++) { acc += l[c]; l[c] = (uint32_t)acc & 0xffffu; acc >>= 16; }
#pragma unroll
  for (int pass = 0; pass < 2; pass++) {
    acc = acc * 38u + 19u * (l[15] >> 15);
    l[15] &= 0x7fffu;
#pragma unroll
    for (int c = 0; c < 16; c++) { acc += l[c]; l[c] = (uint32_t)acc & 0xffffu; acc >>= 16; }
  }
  /* now < 2^255 + 2^6: zero mod p iff it is 0 or p (digits ffed, ffff x 14, 7fff) */
  uint32_t z = 0u, q = (l[0] ^ 0xffedu) | (l[15] ^ 0x7fffu);
#pragma unroll
  for (int c = 0; c < 16; c++) z |= l[c];
#pragma unroll
  for (int c = 1; c < 15; c++) q |= l[c] ^ 0xffffu;
  return z == 0u || q == 0u;
}

/* ---- group operations with broadcast routing (round 5) -----------------

   Each group operation ends in the four products that finish it (a p1p1 to
   a p3, one product per row).  Their operands are linear combinations of
   the previous four products (the squarings of a doubling, the products
   of an addition): instead of moving rows pairwise into place (a swap, a
   select and a register copy per move, ~30 operations per doubling),
   r16_bcast4 spreads the four products over every row with three swaps,
   every lane forms the few combinations it needs, and two selects per
   operand pick its row's. */

/* rows (x0, x1, x2, x3) of x, each broadcast over the wave */
struct r16_b4 { uint32_t v0, v1, v2, v3; };
FD_DEV r16_b4 r16_bcast4(uint32_t x) {
  const r16_eo e = r16_swap16(x);                        /* (x0, x0, x2, x2), (x1, x1, x3, x3) */
  const r16_lh a = r16_swap32(e.e), b = r16_swap32(e.o);
  return {a.l, b.l, a.h, b.h};
}

/* 2P (dbl-2008-hwcd, a = -1).  P is a p3 (X, Y, Z, T) or, LX, (X, Y, Z, X);
   tight in, tight out.  The squarings f g = (X^2, Y^2, Z^2, XY) with
   f = (X, Y, Z, X), g = (X, Y, Z, Y); then, every square in every row,
     E = 2XY,  G = Y^2 - X^2,  -H = X^2 + Y^2,  -F = 2Z^2 - G
   (< 2^17.1, 2^17.6, 2^17.1, 2^18.6: G < 2^18 - 152), and the products
   (E -F, G -H, -F G, E -H) = -(X3, Y3, Z3, T3): the same point; or, not
   WANT_T, (X3, Y3, Z3, X3) negated, for the next doubling. */
template <bool LX, bool WANT_T>
FD_DEV uint32_t ge16_dbl2(uint32_t p, const r16ctx& k) {
  const uint32_t f = LX ? p : r16_bsel(k.r3, r16_swap32(r16_swap16(p).e).l, p);   /* row 3 <- X */
  const uint32_t g = r16_bsel(k.r3, r16_swap32(p).l, p);                          /* row 3 <- Y */
  const r16_b4 q = r16_bcast4(r16_mul(f, g, k));
  const uint32_t nh = q.v0 + q.v1;
  const uint32_t gg = q.v1 + k.p4 - q.v0;
  const uint32_t e = q.v3 + q.v3;
  const uint32_t nf = q.v2 + q.v2 + k.p8 - gg;
  const uint32_t a = r16_bsel(k.r1, gg, r16_bsel(k.r2, nf, e));                   /* (E, G, -F, E)        */
  const uint32_t b = r16_bsel(k.r1, nh, r16_bsel(k.r2, gg, WANT_T ? r16_bsel(k.r3, nh, nf) : nf));
  return r16_mul(a, b, k);                                                         /* b: (-F, -H, G, -H|-F) */
}

/* P + Q, P a p3 with limbs < 2^17 (tight, or 4p - tight where ge16_cneg4
   negated it), Q in qc form (Y2 - X2, Y2 + X2, 2dT2, 2Z2), < 2^19: the
   products (Y-X)(Y2-X2), (Y+X)(Y2+X2), T 2dT2, Z 2Z2 = (b, a, c, t), then
   R = (a - b, a + b, t + c, t - c) (< 2^17.6; NEG: b - a in the first,
   which with X and T of P negated adds -Q) and the products
   (R0 R3, R1 R2, R2 R3, R0 R1) = (X3, Y3, Z3, T3) -- ge16_add then
   ge16_to_p3 -- or (X3, Y3, Z3, X3) without WANT_T */
template <bool WANT_T>
FD_DEV uint32_t ge16_add2(uint32_t p, uint32_t qc, bool neg, const r16ctx& k) {
  const uint32_t v = r16_xor1(p, k);                                              /* Y, X, T, Z */
  const uint32_t o = v + (((k.p4 - p) & k.r0) | (p & k.r1));                      /* < 2^18     */
  const r16_b4 q = r16_bcast4(r16_mul(o, qc, k));
  const uint32_t r0 = neg ? q.v0 + k.p4 - q.v1 : q.v1 + k.p4 - q.v0;
  const uint32_t r1 = q.v1 + q.v0, r2 = q.v3 + q.v2, r3 = q.v3 + k.p4 - q.v2;
  const uint32_t a = r16_bsel(k.r1, r1, r16_bsel(k.r2, r2, r0));                  /* (R0, R1, R2, R0)    */
  const uint32_t b = r16_bsel(k.r1, r2, WANT_T ? r16_bsel(k.r3, r1, r3) : r3);    /* (R3, R2, R3, R1|R3) */
  return r16_mul(a, b, k);
}

/* limb c of the constant 1 / 2 (row-independent) */
FD_DEV uint32_t r16_small(uint32_t v, const r16ctx& k) { return k.c ? 0u : v; }

/* the canonical 16-bit digits of the row's element (limbs < 2^19), in every
   lane of the row: r16_iszero's folds, then value - p when value >= p
   (value + 19 reaches bit 255) */
FD_DEV void r16_digits(uint32_t (&l)[16], uint32_t x) {
  l[0] = R16_BC(x, 0); l[1] = R16_BC(x, 1); l[2] = R16_BC(x, 2); l[3] = R16_BC(x, 3);
  l[4] = R16_BC(x, 4); l[5] = R16_BC(x, 5); l[6] = R16_BC(x, 6); l[7] = R16_BC(x, 7);
  l[8] = R16_BC(x, 8); l[9] = R16_BC(x, 9); l[10] = R16_BC(x, 10); l[11] = R16_BC(x, 11);
  l[12] = R16_BC(x, 12); l[13] = R16_BC(x, 13); l[14] = R16_BC(x, 14); l[15] = R16_BC(x, 15);
  uint64_t acc = 0;
#pragma unroll
  for (int c = 0; c < 16; c++) { acc += l[c]; l[c] = (uint32_t)acc & 0xffffu; acc >>= 16; }
#pragma unroll
  for (int pass = 0; pass < 2; pass++) {
    acc = acc * 38u + 19u * (l[15] >> 15);
    l[15] &= 0x7fffu;
#pragma unroll
    for (int c = 0; c < 16; c++) { acc += l[c]; l[c] = (uint32_t)acc & 0xffffu; acc >>= 16; }
  }
  /* < 2^255 + 2^6 */
  uint32_t t[16], a = 19u;
#pragma unroll
  for (int c = 0; c < 16; c++) { a += l[c]; t[c] = a & 0xffffu; a >>= 16; }
  const bool ge = (t[15] >> 15) != 0u;
  t[15] &= 0x7fffu;
#pragma unroll
  for (int c = 0; c < 16; c++) l[c] = ge ? t[c] : l[c];
}

/* digits -> 8 little-endian words */
FD_DEV void r16_words(uint32_t (&w)[8], const uint32_t (&l)[16]) {
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = l[2 * i] | (l[2 * i + 1] << 16);
}

FD_DEV uint32_t r16_sqn(uint32_t x, int n, const r16ctx& k) {
#pragma clang loop unroll(disable)
  for (int i = 0; i < n; i++) x = r16_sq(x, k);
  return x;
}

/* z^(2^252-3): fe_pow22523's chain (fd_f25519_pow22523,
   src/ballet/ed25519/fd_f25519.c:11-59), 250 squarings and 11 products */
FD_DEV uint32_t r16_pow22523(uint32_t z, const r16ctx& k) {
  uint32_t t0 = r16_sq(z, k);
  uint32_t t1 = r16_sqn(t0, 2, k);
  t1 = r16_mul(z, t1, k);
  t0 = r16_mul(t0, t1, k);
  t0 = r16_sq(t0, k);
  t0 = r16_mul(t1, t0, k);
  t1 = r16_sqn(t0, 5, k);
  t0 = r16_mul(t1, t0, k);
  t1 = r16_sqn(t0, 10, k);
  t1 = r16_mul(t1, t0, k);
  uint32_t t2 = r16_sqn(t1, 20, k);
  t1 = r16_mul(t2, t1, k);
  t1 = r16_sqn(t1, 10, k);
  t0 = r16_mul(t1, t0, k);
  t1 = r16_sqn(t0, 50, k);
  t1 = r16_mul(t1, t0, k);
  t2 = r16_sqn(t1, 100, k);
  t1 = r16_mul(t2, t1, k);
  t1 = r16_sqn(t1, 50, k);
  t0 = r16_mul(t1, t0, k);
  t0 = r16_sqn(t0, 2, k);
  return r16_mul(t0, z, k);
}

/* ---- point decompression, a row per point (fd25519_dsm.h ge_decode) -----

   y: the row's encoding as limbs (lane c: bits 16c..16c+15, bit 255
   cleared), sign: bit 255.  Returns x's canonical words before its sign is
   applied (the caller negates when `neg`), and ge_decode's fail / small
   verdicts: x = u v^3 (u v^7)^((p-5)/8), u = y^2 - 1, v = d y^2 + 1; a root
   when v x^2 = u, times sqrt(-1) when v x^2 = -u, else no root; the
   AVX-512 rule also rejects x = 0 with the sign set; small order on the
   canonical y (x = 0, y = 0 or y = the order-8 points' y).  Every operand
   stays < 2^19: u + 4p - 1 < 2^17.6, v + 1 < 2^16 + 65, v x^2 + 8p - u
   (u < 2^18 - 152) < 2^18.4, v x^2 + u < 2^17.7. */
struct r16_dec {
  uint32_t x[8];
  bool neg, fail, small;
};

FD_DEV void decode16(r16_dec& o, uint32_t y, uint32_t sign, bool avx_rule, uint32_t d, uint32_t sqrtm1,
                     const r16ctx& k) {
  const uint32_t one = r16_small(1u, k);
  uint32_t u = r16_sq(y, k);
  uint32_t v = r16_mul(u, d, k) + one;                          /* d y^2 + 1  */
  u = u + k.p4 - one;                                           /* y^2 - 1    */
  const uint32_t v3 = r16_mul(r16_sq(v, k), v, k);              /* v^3        */
  uint32_t x = r16_mul(r16_mul(r16_sq(v3, k), v, k), u, k);     /* u v^7      */
  x = r16_pow22523(x, k);
  x = r16_mul(r16_mul(x, v3, k), u, k);
  const uint32_t vxx = r16_mul(r16_sq(x, k), v, k);
  uint32_t l[16];
  uint32_t z = 0u;
  r16_digits(l, vxx + k.p8 - u);
#pragma unroll
  for (int c = 0; c < 16; c++) z |= l[c];
  const bool root = z == 0u;
  z = 0u;
  r16_digits(l, vxx + u);
#pragma unroll
  for (int c = 0; c < 16; c++) z |= l[c];
  const bool iroot = z == 0u;
  const uint32_t xi = r16_mul(x, sqrtm1, k);
  r16_digits(l, root ? x : xi);
  z = 0u;
#pragma unroll
  for (int c = 0; c < 16; c++) z |= l[c];
  const bool x0 = z == 0u;
  r16_words(o.x, l);
  o.fail = !(root || iroot) || (avx_rule && x0 && sign);
  o.neg = (l[0] & 1u) != sign;
  /* small order on the canonical y */
  r16_digits(l, y);
  uint32_t yw[8];
  r16_words(yw, l);
  const uint32_t y0[8] = {0x8f95e826u, 0xb027b2c2u, 0x89f4c345u, 0xf098eff2u,
                          0x05acdfd5u, 0x3933c6d3u, 0x880238b1u, 0x05fc536du};
  const uint32_t y1[8] = {0x706a17c7u, 0x4fd84d3du, 0x760b3cbau, 0x0f67100du,
                          0xfa53202au, 0xc6cc392cu, 0x77fdc74eu, 0x7a03ac92u};
  uint32_t zy = 0u, e0 = 0u, e1 = 0u;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    zy |= yw[i];
    e0 |= yw[i] ^ y0[i];
    e1 |= yw[i] ^ y1[i];
  }
  o.small = x0 || zy == 0u || e0 == 0u || e1 == 0u;
}

/* ---- negation, cached form, tables ------------------------------------ */

/* -x in the rows of the mask `rows` when neg (wave-uniform): 4p - x for
   tight x (a p3's X and T: -P before ge16_add2 with neg) */
FD_DEV uint32_t ge16_cneg4(uint32_t x, uint32_t rows, bool neg, const r16ctx& k) {
  return neg ? (x ^ ((x ^ (k.p4 - x)) & rows)) : x;
}

/* qc of a p3 (limbs < 2^17): (Y-X, Y+X, 2dT, 2Z), < 2^18 */
FD_DEV uint32_t ge16_to_qc(uint32_t p, uint32_t d2, const r16ctx& k) {
  const uint32_t v = r16_xor1(p, k);                            /* Y, X, T, Z        */
  const uint32_t t = r16_mul(v, d2, k);                         /* row 2: 2d T       */
  return ((v + k.p4 - p) & k.r0) | ((v + p) & k.r1) | (t & k.r2) | ((v + v) & k.r3);
}

/* [0..8](sign P) as qc entries, one register per entry (the lane's limb
   of its row's coordinate), for the affine point (x, y) given as r16
   limbs (tight) in every row; negate: -P (fd25519_ge4.h table4_build) */
FD_DEV void table16_build(uint32_t (&tab)[9], uint32_t x, uint32_t y, bool negate, uint32_t d2, const r16ctx& k) {
  const uint32_t xs = negate ? k.p4 - x : x;                    /* < 2^17 */
  const uint32_t xy = r16_mul(xs, y, k);
  const uint32_t one = r16_small(1u, k);
  const uint32_t p0 = (xs & k.r0) | (y & k.r1) | (one & k.r2) | (xy & k.r3);   /* (x, y, 1, xy) */
  /* the identity (1, 1, 0, 2) */
  tab[0] = (one & (k.r0 | k.r1)) | (r16_small(2u, k) & k.r3);
  const uint32_t c1 = ge16_to_qc(p0, d2, k);
  tab[1] = c1;
  uint32_t cur = p0;
#pragma unroll
  for (int e = 2; e <= 8; e++) {
    cur = ge16_add2<true>(cur, c1, false, k);
    tab[e] = ge16_to_qc(cur, d2, k);
  }
}

/* ... for a point given in extended coordinates: p0 is the lane's limb
   of its row's coordinate of P (X, Y, Z, T; tight), already negated when
   the table is for -P (ge16_cneg4 on rows 0 and 3) */
FD_DEV void table16_build_p3(uint32_t (&tab)[9], uint32_t p0, uint32_t d2, const r16ctx& k) {
  const uint32_t one = r16_small(1u, k);
  tab[0] = (one & (k.r0 | k.r1)) | (r16_small(2u, k) & k.r3);
  const uint32_t c1 = ge16_to_qc(p0, d2, k);
  tab[1] = c1;
  uint32_t cur = p0;
#pragma unroll
  for (int e = 2; e <= 8; e++) {
    cur = ge16_add2<true>(cur, c1, false, k);
    tab[e] = ge16_to_qc(cur, d2, k);
  }
}

/* entry e of the table, e wave-uniform (a branch on a scalar) */
FD_DEV uint32_t table16_at(const uint32_t (&tab)[9], int e) {
  switch (e) {
  case 0: return tab[0];
  case 1: return tab[1];
  case 2: return tab[2];
  case 3: return tab[3];
  case 4: return tab[4];
  case 5: return tab[5];
  case 6: return tab[6];
  case 7: return tab[7];
  default: return tab[8];
  }
}
