/* fd25519_dsm.h -- device helpers shared by the verify and generator
   kernels: point decoding with the reference's acceptance rules, signed
   fixed-window scalar recoding, and the table accessors: per-lane -A / -+R
   tables and the base tables in HBM (verify), [0..128]B in LDS (signing). */
#pragma once
#include "fd25519_ge.h"
#include "fd_ed25519_hip_internal.h"

/* reference codes, src/ballet/ed25519/fd_ed25519.h:11-14 */
#define FD_ED25519_SUCCESS 0
#define FD_ED25519_ERR_SIG -1
#define FD_ED25519_ERR_PUBKEY -2
#define FD_ED25519_ERR_MSG -3

/* ------------------------------------------------------------------------
   Point decoding with the reference's acceptance rules. */

struct decoded_pt {
  fe x, y;
  bool fail;   /* no square root, or (AVX-512 rule) x == 0 with sign set */
  bool small;  /* small order: x == 0, y == 0, y == y0 or y == y1       */
};

FD_DEV void ge_decode(decoded_pt& d, const uint32_t (&s)[8], bool avx_rule) {
  const fe one = {{1, 0, 0, 0, 0, 0, 0, 0, 0, 0}};
  const fe cd = {FE_D}, sqrtm1 = {FE_SQRTM1};
  fe u, v, v3, x, vxx, t;
  fe_frombytes(d.y, s);
  const uint32_t sign = s[7] >> 31;
  fe_sq(u, d.y);
  fe_mul(v, u, cd);
  fe_sub(u, u, one);  /* u = y^2 - 1  */
  fe_add(v, v, one);  /* v = d y^2 + 1 */
  fe_sq(v3, v);
  fe_mul(v3, v3, v);  /* v^3 */
  fe_sq(x, v3);
  fe_mul(x, x, v);
  fe_mul(x, x, u);    /* u v^7 */
  fe_pow22523(x, x);
  fe_mul(x, x, v3);
  fe_mul(x, x, u);    /* x = u v^3 (u v^7)^((p-5)/8) */
  fe_sq(vxx, x);
  fe_mul(vxx, vxx, v);
  fe_sub(t, vxx, u);
  const bool root = fe_iszero(t);
  fe_add(t, vxx, u);
  const bool iroot = fe_iszero(t);
  fe xi;
  fe_mul(xi, x, sqrtm1);
  fe_select(x, x, xi, !root);
  uint32_t xb[8];
  fe_tobytes(xb, x);
  const bool x0 = (xb[0] | xb[1] | xb[2] | xb[3] | xb[4] | xb[5] | xb[6] | xb[7]) == 0u;
  const uint32_t par = xb[0] & 1u;
  d.fail = !(root || iroot) || (avx_rule && x0 && sign);
  fe xn;
  fe_neg(xn, x);
  fe_select(d.x, x, xn, par != sign);
  /* small order on the canonical y */
  uint32_t yb[8];
  fe_tobytes(yb, d.y);
  const uint32_t y0[8] = {0x8f95e826u, 0xb027b2c2u, 0x89f4c345u, 0xf098eff2u,
                          0x05acdfd5u, 0x3933c6d3u, 0x880238b1u, 0x05fc536du};
  const uint32_t y1[8] = {0x706a17c7u, 0x4fd84d3du, 0x760b3cbau, 0x0f67100du,
                          0xfa53202au, 0xc6cc392cu, 0x77fdc74eu, 0x7a03ac92u};
  uint32_t z = 0, e0 = 0, e1 = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    z |= yb[i];
    e0 |= yb[i] ^ y0[i];
    e1 |= yb[i] ^ y1[i];
  }
  d.small = x0 || z == 0u || e0 == 0u || e1 == 0u;
}

/* ------------------------------------------------------------------------
   Signed fixed-window recoding, packed so the main loop can pop the most
   significant digit with a shift (no dynamically indexed register arrays). */

/* k < L < 2^253 -> 64 digits e_i in [-8,7] (e_63 in [0,2]), 4 bits each */
FD_DEV void recode_radix16(uint32_t (&out)[8], const uint32_t (&k)[8]) {
  int carry = 0;
#pragma unroll
  for (int w = 0; w < 8; w++) {
    uint32_t packed = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      int e = (int)((k[w] >> (4 * j)) & 15u) + carry;
      carry = (e + 8) >> 4;
      e -= carry * 16;
      packed |= ((uint32_t)e & 15u) << (4 * j);
    }
    out[w] = packed;
  }
}

/* S < L -> 32 digits f_j in [-128,127] (f_31 in [0,17]), 8 bits each */
FD_DEV void recode_radix256(uint32_t (&out)[8], const uint32_t (&s)[8]) {
  int carry = 0;
#pragma unroll
  for (int w = 0; w < 8; w++) {
    uint32_t packed = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      int f = (int)((s[w] >> (8 * j)) & 255u) + carry;
      carry = (f + 128) >> 8;
      f -= carry * 256;
      packed |= ((uint32_t)f & 255u) << (8 * j);
    }
    out[w] = packed;
  }
}

/* S < L -> 16 digits g_j in [-2^15, 2^15] (g_15 in [0, 2^13+1]), 16 bits each */
FD_DEV void recode_radix65536(uint32_t (&out)[8], const uint32_t (&s)[8]) {
  int carry = 0;
#pragma unroll
  for (int w = 0; w < 8; w++) {
    uint32_t packed = 0;
#pragma unroll
    for (int j = 0; j < 2; j++) {
      int g = (int)((s[w] >> (16 * j)) & 0xffffu) + carry;
      carry = (g + 32768) >> 16;
      g -= carry * 65536;
      packed |= ((uint32_t)g & 0xffffu) << (16 * j);
    }
    out[w] = packed;
  }
}

/* pop the top `bits` of the 256-bit value as a signed digit */
template <int BITS>
FD_DEV int pop_digit(uint32_t (&d)[8]) {
  const int v = ((int32_t)d[7]) >> (32 - BITS);
#pragma unroll
  for (int w = 7; w > 0; w--) d[w] = __builtin_amdgcn_alignbit(d[w], d[w - 1], 32 - BITS);
  d[0] <<= BITS;
  return v;
}

/* ------------------------------------------------------------------------
   Tables */

FD_DEV void atab_store(int4* lane_tab, int e, const ge_cached& c) {
  int v[40];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    v[i] = c.YplusX.v[i];
    v[10 + i] = c.YminusX.v[i];
    v[20 + i] = c.Z2.v[i];
    v[30 + i] = c.T2d.v[i];
  }
#pragma unroll
  for (int q = 0; q < 10; q++)
    lane_tab[e * 10 + q] = make_int4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
}

FD_DEV void atab_load(ge_cached& c, const int4* lane_tab, int e) {
  int v[40];
#pragma unroll
  for (int q = 0; q < 10; q++) {
    const int4 x = lane_tab[e * 10 + q];
    v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
  }
#pragma unroll
  for (int i = 0; i < 10; i++) {
    c.YplusX.v[i] = v[i];
    c.YminusX.v[i] = v[10 + i];
    c.Z2.v[i] = v[20 + i];
    c.T2d.v[i] = v[30 + i];
  }
}

FD_DEV void btab_load(ge_precomp& b, const int4* s_btab, int e) {
  int v[32];
  const int4* src = s_btab + e * (FD_ED25519_BTAB_STRIDE / 4);
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const int4 x = src[q];
    v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
  }
#pragma unroll
  for (int i = 0; i < 10; i++) {
    b.yplusx.v[i] = v[i];
    b.yminusx.v[i] = v[10 + i];
    b.xy2d.v[i] = v[20 + i];
  }
}

/* entry e of the wide B table in global memory (128-byte entries) */
FD_DEV void btab16_load(ge_precomp& b, const int4* g_btab, int e) {
  int v[32];
  const int4* src = g_btab + e * (FD_ED25519_BTAB16_STRIDE / 4);
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const int4 x = src[q];
    v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
  }
#pragma unroll
  for (int i = 0; i < 10; i++) {
    b.yplusx.v[i] = v[i];
    b.yminusx.v[i] = v[10 + i];
    b.xy2d.v[i] = v[20 + i];
  }
}

/* ------------------------------------------------------------------------
   Fixed-base scalar multiplication [s]B, s < L, with the [0..128]B table in
   LDS (radix-256 signed digits: 248 doublings, 32 mixed additions), and
   point encoding (canonical y with the parity of x in bit 255, as
   fd_ed25519_point_tobytes, src/ballet/ed25519/fd_curve25519.c:64-76). */

FD_DEV void ge_scalarmult_base(ge_p2& Q, const uint32_t (&s)[8], const int4* s_btab) {
  uint32_t sd[8];
  recode_radix256(sd, s);
  ge_p3 P;
  ge_p3_0(P);
  ge_p1p1 Rt;
#pragma clang loop unroll(disable)
  for (int j = 31; j >= 0; j--) {
    if (j != 31) {
#pragma clang loop unroll(disable)
      for (int dd = 0; dd < 8; dd++) {
        ge_p2_dbl(Rt, Q);
        if (dd < 7) ge_p1p1_to_p2(Q, Rt);
      }
      ge_p1p1_to_p3(P, Rt);
    }
    const int f = pop_digit<8>(sd);
    ge_precomp b;
    btab_load(b, s_btab, f < 0 ? -f : f);
    ge_precomp_cneg(b, f < 0);
    ge_madd(Rt, P, b);
    ge_p1p1_to_p2(Q, Rt);
  }
}

FD_DEV void ge_encode(uint32_t (&out)[8], const ge_p2& Q) {
  fe zi, x, y;
  fe_invert(zi, Q.Z);
  fe_mul(x, Q.X, zi);
  fe_mul(y, Q.Y, zi);
  uint32_t xb[8];
  fe_tobytes(xb, x);
  fe_tobytes(out, y);
  out[7] |= (xb[0] & 1u) << 31;
}
