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
   are followed step for step; operands move between rows with gfx950's
   permlane swaps and per-row bit selects (ds_bpermute, r16_rp, only for
   the final identity test).

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

/* ---- group operations (fd25519_ge4.h's, a row per coordinate) ---------- */

/* p1p1 -> p3 (or p2): (X T, Y Z, Z T, X Y); r < 2^19 in, tight out */
FD_DEV uint32_t ge16_to_p3(uint32_t r, const r16ctx& k) {
  /* a = (r0, r1, r2, r0): row 3 takes the broadcast of r0 (swap32 of swap16's e) */
  const uint32_t b0 = r16_swap32(r16_swap16(r).e).l;
  const uint32_t a = r16_bsel(k.r3, b0, r);
  /* b = (r3, r2, r3, r1): the broadcasts of r2, r3 (swap16 of swap32's h), r1 from swap32's l */
  const r16_lh s = r16_swap32(r);
  const r16_eo t = r16_swap16(s.h);
  const uint32_t b = r16_bsel(k.r3, s.l, r16_bsel(k.r1, t.e, t.o));
  return r16_mul(a, b, k);
}

/* r = 2p (p2 or p3 in, tight; p1p1 out): squares X^2, Y^2, (X+Y)^2, 2Z^2 in
   rows 0..3, then (X+Y)^2 - (X^2+Y^2), X^2+Y^2, Y^2-X^2, 2Z^2-(Y^2-X^2)
   (ge4_dbl, ge_p2_dbl) */
FD_DEV uint32_t ge16_dbl(uint32_t p, const r16ctx& k) {
  /* u = (X, Y, X+Y, Z): swap32's l is (X, Y, X, Y), the broadcast of Y
     (swap32 of swap16's o) is added in row 2, row 3 takes swap16's e (Z) */
  const r16_eo pe = r16_swap16(p);
  const uint32_t by = r16_swap32(pe.o).l;
  const uint32_t u = r16_bsel(k.r3, pe.e, r16_swap32(p).l + (by & k.r2));   /* < 2^17.1 */
  uint32_t s = r16_sq(u, k);                                    /* tight             */
  s += s & k.r3;                                                /* 2Z^2              < 2^17.1 */
  const uint32_t w = r16_xor1(s, k);                            /* s1, s0, s3, s2    */
  /* row 0: s0 + s1 (< 2^17.1), row 1: s1 - s0 (s1 + 4p - s0 < 2^17.6), rows 2, 3: s2, s3 */
  const uint32_t t = s + ((w & k.r0) | ((k.p4 - w) & k.r1));
  /* x = (t2, t0, t1, t3): swap32's h, swap16's e, the broadcast of t1, t;
     y = (t0, -, -, t1) = swap32's l */
  const r16_lh tl = r16_swap32(t);
  const r16_eo te = r16_swap16(t);
  const uint32_t b1 = r16_swap32(te.o).l;
  const uint32_t x = r16_bsel(k.r0, tl.h, r16_bsel(k.r1, te.e, r16_bsel(k.r2, b1, t)));
  const uint32_t y = tl.l;
  /* row 0: s2 + 8p - t0, row 3: s3 + 8p - t1 (t0, t1 < 2^17.6 < 2^18 - 152): < 2^18.6 */
  return x + ((k.p8 - y) & k.r03);
}

/* r = p + q (p3 in, limbs < 2^17 -- tight, or 4p - tight where negated;
   q in qc form (Y-X, Y+X, 2dT, 2Z), < 2^19; p1p1 out): b = (Y-X)(Y2-X2),
   a = (Y+X)(Y2+X2), c = T 2dT2, t = Z 2Z2 in rows 0..3, then
   (a - b, a + b, t + c, t - c) (ge4_add) */
FD_DEV uint32_t ge16_add(uint32_t p, uint32_t qc, const r16ctx& k) {
  const uint32_t v = r16_xor1(p, k);                            /* Y, X, T, Z        */
  /* row 0: Y + 4p - X (< 2^18), row 1: X + Y (< 2^18), rows 2, 3: T, Z */
  const uint32_t o = v + (((k.p4 - p) & k.r0) | (p & k.r1));
  const uint32_t pr = r16_mul(o, qc, k);                        /* b, a, c, t: tight */
  const uint32_t w = r16_xor1(pr, k);                           /* a, b, t, c        */
  /* row 0: a + 4p - b, row 1: a + b, row 2: c + t, row 3: t + 4p - c: < 2^17.6 */
  return ((w + pr) & k.r12) | ((w + k.p4 - pr) & k.r0) | ((pr + k.p4 - w) & k.r3);
}

/* -x in the rows of the mask `rows` when neg (wave-uniform): 4p - x for
   tight x (p3), 8p - x for x < 2^18 - 152 (a p1p1's row 0) */
FD_DEV uint32_t ge16_cneg4(uint32_t x, uint32_t rows, bool neg, const r16ctx& k) {
  return neg ? (x ^ ((x ^ (k.p4 - x)) & rows)) : x;
}
FD_DEV uint32_t ge16_cneg8(uint32_t x, uint32_t rows, bool neg, const r16ctx& k) {
  return neg ? (x ^ ((x ^ (k.p8 - x)) & rows)) : x;
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
