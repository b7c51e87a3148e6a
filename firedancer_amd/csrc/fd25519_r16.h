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
   a quad does in fd25519_ge4.h, whose formulas (same products, same order)
   are followed step for step; operands move between rows with
   ds_bpermute (r16_rp).

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

/* per-lane constants, made once per kernel */
struct r16ctx {
  uint32_t m[16];     /* m[t] = 38 if c < t else 1: the wrap factor of term t in lane c */
  uint32_t p4, p8;    /* limb c of 4p / 8p (all limbs positive, above any tight / < 2^18 - 152 limb) */
  uint32_t c;         /* lane in row */
  uint32_t row;       /* row (coordinate) in the wave */
};

FD_DEV void r16_init(r16ctx& k) {
  k.c = threadIdx.x & 15u;
  k.row = (threadIdx.x >> 4) & 3u;
#pragma unroll
  for (int t = 0; t < 16; t++) k.m[t] = k.c < (uint32_t)t ? 38u : 1u;
  k.p4 = k.c ? (1u << 17) - 2u : (1u << 17) - 76u;
  k.p8 = k.c ? (1u << 18) - 4u : (1u << 18) - 152u;
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

/* f*g, limbs < 2^19 in, tight out; two accumulators (even / odd t) so that
   two multiply-add chains are in flight */
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
  const uint32_t src = k.row == 0u ? (uint32_t)S0 : k.row == 1u ? (uint32_t)S1 : k.row == 2u ? (uint32_t)S2 : (uint32_t)S3;
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((src << 4) | k.c) << 2), (int)x);
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

/* ---- group operations (fd25519_ge4.h's, a row per coordinate) ---------- */

/* x in rows where sel, else y */
FD_DEV uint32_t r16_sel(bool sel, uint32_t x, uint32_t y) { return sel ? x : y; }

/* p1p1 -> p3 (or p2): (X T, Y Z, Z T, X Y); r < 2^19 in, tight out */
FD_DEV uint32_t ge16_to_p3(uint32_t r, const r16ctx& k) {
  const uint32_t a = r16_rp<0, 1, 2, 0>(r, k), b = r16_rp<3, 2, 3, 1>(r, k);
  return r16_mul(a, b, k);
}

/* r = 2p (p2 or p3 in, tight; p1p1 out): squares X^2, Y^2, (X+Y)^2, 2Z^2 in
   rows 0..3, then (X+Y)^2 - (X^2+Y^2), X^2+Y^2, Y^2-X^2, 2Z^2-(Y^2-X^2)
   (ge4_dbl, ge_p2_dbl) */
FD_DEV uint32_t ge16_dbl(uint32_t p, const r16ctx& k) {
  const uint32_t a = r16_rp<0, 1, 0, 2>(p, k), b = r16_rp<0, 0, 1, 0>(p, k);
  const uint32_t u = a + (k.row == 2u ? b : 0u);                /* X, Y, X+Y, Z      < 2^17.1 */
  uint32_t s = r16_sq(u, k);                                    /* tight             */
  s = k.row == 3u ? s + s : s;                                  /* 2Z^2              < 2^17.1 */
  const uint32_t w = r16_rp<1, 0, 3, 2>(s, k);                  /* s1, s0, s3, s2    */
  /* row 0: s0 + s1 (< 2^17.1), row 1: s1 - s0 (s1 + 4p - s0 < 2^17.6), rows 2, 3: s2, s3 */
  const uint32_t t = k.row == 0u ? s + w : k.row == 1u ? s + k.p4 - w : s;
  const uint32_t x = r16_rp<2, 0, 1, 3>(t, k);                  /* s2, t0, t1, s3    */
  const uint32_t y = r16_rp<0, 0, 0, 1>(t, k);                  /* t0 (row 0), t1 (row 3) */
  /* row 0: s2 + 8p - t0, row 3: s3 + 8p - t1 (t0, t1 < 2^17.6 < 2^18 - 152): < 2^18.6 */
  return (k.row == 0u || k.row == 3u) ? x + k.p8 - y : x;
}

/* r = p + q (p3 in, tight; q in qc form (Y-X, Y+X, 2dT, 2Z), < 2^19; p1p1
   out): b = (Y-X)(Y2-X2), a = (Y+X)(Y2+X2), c = T 2dT2, t = Z 2Z2 in rows
   0..3, then (a - b, a + b, t + c, t - c) (ge4_add) */
FD_DEV uint32_t ge16_add(uint32_t p, uint32_t qc, const r16ctx& k) {
  const uint32_t v = r16_rp<1, 0, 3, 2>(p, k);                  /* Y, X, T, Z        */
  /* row 0: Y + 4p - X (< 2^17.6), row 1: X + Y (< 2^17.1), rows 2, 3: T, Z */
  const uint32_t o = k.row == 0u ? v + k.p4 - p : k.row == 1u ? v + p : v;
  const uint32_t pr = r16_mul(o, qc, k);                        /* b, a, c, t: tight */
  const uint32_t w = r16_rp<1, 0, 3, 2>(pr, k);                 /* a, b, t, c        */
  /* row 0: a + 4p - b, row 1: a + b, row 2: c + t, row 3: t + 4p - c: < 2^17.6 */
  return k.row == 0u ? w + k.p4 - pr : k.row == 3u ? pr + k.p4 - w : w + pr;
}

/* -P in the rows of `rows` when neg: 4p - x for tight x (p3), 8p - x for
   x < 2^18 - 152 (a p1p1's row 0) */
FD_DEV uint32_t ge16_cneg4(uint32_t x, bool rows, bool neg, const r16ctx& k) {
  return (rows && neg) ? k.p4 - x : x;
}
FD_DEV uint32_t ge16_cneg8(uint32_t x, bool rows, bool neg, const r16ctx& k) {
  return (rows && neg) ? k.p8 - x : x;
}

/* qc of a p3 (tight): (Y-X, Y+X, 2dT, 2Z), < 2^17.6 */
FD_DEV uint32_t ge16_to_qc(uint32_t p, uint32_t d2, const r16ctx& k) {
  const uint32_t v = r16_rp<1, 0, 3, 2>(p, k);                  /* Y, X, T, Z        */
  const uint32_t t = r16_mul(v, d2, k);                         /* row 2: 2d T       */
  return k.row == 0u ? v + k.p4 - p : k.row == 1u ? v + p : k.row == 2u ? t : v + v;
}

/* limb c of the constant 1 / 2 (row-independent) */
FD_DEV uint32_t r16_small(uint32_t v, const r16ctx& k) { return k.c ? 0u : v; }

/* [0..8](sign P) as qc entries, one register per entry (the lane's limb
   of its row's coordinate), for the affine point (x, y) given as r16
   limbs (tight) in every row; negate: -P (fd25519_ge4.h table4_build) */
FD_DEV void table16_build(uint32_t (&tab)[9], uint32_t x, uint32_t y, bool negate, uint32_t d2, const r16ctx& k) {
  const uint32_t xs = negate ? k.p4 - x : x;                    /* < 2^17 */
  const uint32_t xy = r16_mul(xs, y, k);
  const uint32_t one = r16_small(1u, k);
  const uint32_t p0 = k.row == 0u ? xs : k.row == 1u ? y : k.row == 2u ? one : xy;   /* (x, y, 1, xy) */
  /* the identity (1, 1, 0, 2) */
  tab[0] = k.row == 2u ? 0u : k.row == 3u ? r16_small(2u, k) : one;
  const uint32_t c1 = ge16_to_qc(p0, d2, k);
  tab[1] = c1;
  uint32_t cur = p0;
#pragma unroll
  for (int e = 2; e <= 8; e++) {
    cur = ge16_to_p3(ge16_add(cur, c1, k), k);
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
