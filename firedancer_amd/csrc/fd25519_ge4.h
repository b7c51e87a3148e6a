/* fd25519_ge4.h -- edwards25519 group operations spread over a quad of
   lanes: one point per 4 consecutive lanes, lane q of the quad holding
   coordinate q.  The verify tile's latency mode hands the GPU batches of a
   few hundred signatures; one lane per signature leaves the chip idle and
   the batch waits for one lane's whole serial chain of field operations.
   The a = -1 extended-coordinate formulas (fd25519_ge.h) have exactly four
   independent multiplications per step, so a quad performs each group
   operation in the time of one multiplication (doubling: one squaring +
   one multiplication), exchanging operands with DPP quad permutations
   (no LDS, no barrier).

   Layouts (lane q = threadIdx & 3 holds the q-th entry):
     p3    (X, Y, Z, T)            also p2 (lane 3's T is then ignored)
     p1p1  (X, Y, Z, T)            completed: x = X/Z, y = Y/T
     qc    (Y-X, Y+X, 2dT, 2Z)     right operand of an addition; a base
                                   table entry (y+x, y-x, 2dxy) is
                                   (y-x, y+x, 2dxy, 2)

   Every step below produces what fd25519_ge.h's serial step produces
   (same formulas, same products), so the bounds of fd25519_fe.h carry
   over: products tight, the sums formed <= 3.03x. */
#pragma once
#include "fd25519_fe.h"

#define FD_QP(a, b, c, d) ((a) | ((b) << 2) | ((c) << 4) | ((d) << 6))

/* h = f of the lane selected by CTRL (a DPP quad permutation) */
template <int CTRL>
FD_DEV void fe_qp(fe& h, const fe& f) {
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = __builtin_amdgcn_mov_dpp(f.v[i], CTRL, 0xf, 0xf, true);
}

/* per-lane masks of a quad (all 0 or -1) */
struct qmask_t {
  int32_t l0, l1, l2, l3;   /* lane q */
  int32_t l01, l03;         /* lanes 0,1 / 0,3 */
};

FD_DEV qmask_t quad_masks() {
  const int q = (int)(threadIdx.x & 3u);
  qmask_t m;
  m.l0 = q == 0 ? -1 : 0;
  m.l1 = q == 1 ? -1 : 0;
  m.l2 = q == 2 ? -1 : 0;
  m.l3 = q == 3 ? -1 : 0;
  m.l01 = q < 2 ? -1 : 0;
  m.l03 = (q == 0 || q == 3) ? -1 : 0;
  return m;
}

/* x if n == 0, -x if n == -1 */
FD_DEV int32_t cneg32(int32_t x, int32_t n) { return (x ^ n) - n; }

/* h = f^2, times 2 on lanes with sh == 1 (the factor folded into the left
   operands as in fe_sq2: inputs tight there, so the bounds hold) */
FD_DEV void fe_sq_sh(fe& h, const fe& f, int sh) {
  int32_t f2[10];
#pragma unroll
  for (int i = 0; i < 10; i++) f2[i] = f.v[i] << sh;
  int64_t a[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
#pragma unroll
    for (int j = i; j < 10; j++) {
      const int k = i + j;
      const int m = (((i & 1) && (j & 1)) ? 2 : 1) * ((k >= 10) ? 19 : 1);
      const int32_t x = (i == j) ? f2[i] : 2 * f2[i];
      const int32_t y = m * f.v[j];
      if (i == 0) fe_mad_init(a[k], x, y, k);
      else fe_mad(a[k >= 10 ? k - 10 : k], x, y);
    }
  }
  fe_carry_wide(h, a);
}

/* p1p1 -> p3 (or p2): (X T, Y Z, Z T, X Y), one product per lane */
FD_DEV void ge4_to_p3(fe& p, const fe& r) {
  fe a, b;
  fe_qp<FD_QP(0, 1, 2, 0)>(a, r);
  fe_qp<FD_QP(3, 2, 3, 1)>(b, r);
  fe_mul(p, a, b);
}

/* r = 2p (p2 or p3 in, p1p1 out): squares X^2, Y^2, (X+Y)^2, 2Z^2 on
   lanes 0..3, then (X+Y)^2 - (Y^2+X^2), Y^2+X^2, Y^2-X^2, 2Z^2-(Y^2-X^2)
   (ge_p2_dbl) */
FD_DEV void ge4_dbl(fe& r, const fe& p, const qmask_t& m) {
  fe a, b, u, s, w, t, x, y;
  fe_qp<FD_QP(0, 1, 0, 2)>(a, p);   /* X, Y, X, Z */
  fe_qp<FD_QP(0, 0, 1, 0)>(b, p);   /* lane 2: Y */
#pragma unroll
  for (int i = 0; i < 10; i++) u.v[i] = a.v[i] + (b.v[i] & m.l2);
  fe_sq_sh(s, u, m.l3 & 1);
  fe_qp<FD_QP(1, 0, 3, 2)>(w, s);   /* s1, s0, s3, s2 */
  /* lane 0: s0 + s1, lane 1: s1 - s0, lanes 2, 3: unchanged */
#pragma unroll
  for (int i = 0; i < 10; i++) t.v[i] = s.v[i] + cneg32(w.v[i] & m.l01, m.l1);
  fe_qp<FD_QP(2, 0, 1, 3)>(x, t);   /* s2, Y, Z, s3 */
  fe_qp<FD_QP(0, 0, 0, 1)>(y, t);   /* lane 0: Y, lane 3: Z */
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = x.v[i] - (y.v[i] & m.l03);
}

/* r = p + q (p3 in, p1p1 out; ge_add / ge_madd): the products
   b = (Y-X)(Y2-X2), a = (Y+X)(Y2+X2), c = T 2dT2, t = Z 2Z2 on lanes 0..3,
   then (a - b, a + b, t + c, t - c) */
FD_DEV void ge4_add(fe& r, const fe& p, const fe& qc, const qmask_t& m) {
  fe v, o, pr, w;
  fe_qp<FD_QP(1, 0, 3, 2)>(v, p);   /* Y, X, T, Z */
#pragma unroll
  for (int i = 0; i < 10; i++) o.v[i] = v.v[i] + cneg32(p.v[i] & m.l01, m.l0);   /* Y-X, Y+X, T, Z */
  fe_mul(pr, o, qc);
  fe_qp<FD_QP(1, 0, 3, 2)>(w, pr);
  /* lane 0: m1 - m0, lane 1: m1 + m0, lane 2: m2 + m3, lane 3: m3 - m2 */
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = cneg32(pr.v[i], m.l0) + cneg32(w.v[i], m.l3);
}

/* -P for a p3 (lanes 0, 3 negate) or, with l0 only, a p1p1 */
FD_DEV void ge4_cneg(fe& p, int32_t lanes, bool neg) {
  const int32_t n = neg ? lanes : 0;
#pragma unroll
  for (int i = 0; i < 10; i++) p.v[i] = cneg32(p.v[i], n);
}

/* qc of a p3: (Y-X, Y+X, 2dT, 2Z) */
FD_DEV void ge4_to_qc(fe& c, const fe& p, const qmask_t& m) {
  const fe d2 = {FE_D2};
  fe v, t;
  fe_qp<FD_QP(1, 0, 3, 2)>(v, p);   /* Y, X, T, Z */
  fe_mul(t, v, d2);
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const int32_t s = v.v[i] + (cneg32(p.v[i], m.l0) & m.l01) + (v.v[i] & m.l3);
    c.v[i] = m.l2 ? t.v[i] : s;
  }
}
