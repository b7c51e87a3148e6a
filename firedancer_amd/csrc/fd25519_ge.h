/* fd25519_ge.h -- edwards25519 group operations for gfx950 (one point per
   lane), a = -1 twisted Edwards in extended coordinates.

   Representations
     ge_p2      (X:Y:Z)            projective, x = X/Z, y = Y/Z
     ge_p3      (X:Y:Z:T)          extended, additionally xy = T/Z
     ge_p1p1    ((X:Z),(Y:T))      "completed", x = X/Z, y = Y/T
     ge_cached  (Y+X, Y-X, 2Z, 2dT) right operand of a general addition
                                  (tables may hold -2dT: ge_add<true>)
     ge_precomp (y+x, y-x, 2dxy)   right operand of a mixed addition (Z=1)

   The addition/doubling laws are the complete formulas for a = -1
   (Hisil-Wong-Carter-Dawson 2008, "add-2008-hwcd-3" / "dbl-2008-hwcd");
   they are complete on edwards25519, so the double-scalar multiplication
   can add the identity for zero digits without branching.  The reference
   uses the same laws (src/ballet/ed25519/ref/fd_curve25519.h:144-211,
   src/ballet/ed25519/ref/fd_curve25519.c:25-179).

   Bounds: every coordinate produced by a conversion (a mul) is tight; the
   sums/differences formed inside stay <= 3.03x tight (fd25519_fe.h). */
#pragma once
#include "fd25519_fe.h"

struct ge_p2 { fe X, Y, Z; };
struct ge_p3 { fe X, Y, Z, T; };
struct ge_p1p1 { fe X, Y, Z, T; };
struct ge_cached { fe YplusX, YminusX, Z2, T2d; };
struct ge_precomp { fe yplusx, yminusx, xy2d; };

FD_DEV void ge_p3_0(ge_p3& h) {
  fe_0(h.X); fe_1(h.Y); fe_1(h.Z); fe_0(h.T);
}

/* Bounds (fd25519_fe.h units): centered products (C) are <= 1.01x,
   unsigned-limb products (U, the _u forms) lie in [0, 2x].  A product's
   19-side operand must stay <= 3.3x, its other operand may be larger.
   Every completed point these formulas produce has X, Z, T within 3x and
   Y within [-1x, 4x], so the conversions below take X, Z (and T) as
   19-sides and Y (and T: ge_add<true>) only as the other operand.

   The conversions share each 19-side between two products, so its
   19-multiples (the wrapped terms) are computed once.  Swapping the
   operands of a product does not change its column sums, so the choice of
   side changes no result. */

/* -> projective, unsigned (the doublings' input) */
FD_DEV void ge_p1p1_to_p2(ge_p2& r, const ge_p1p1& p) {
  fe x19, z19;
  fe_19(x19, p.X);
  fe_19(z19, p.Z);
  fe_mul19_u(r.X, p.T, p.X, x19);
  fe_mul19_u(r.Y, p.Y, p.Z, z19);
  fe_mul19_u(r.Z, p.T, p.Z, z19);
}

/* -> extended.  UXYT: X, Y, T unsigned (an addition's input: they only
   enter sums and differences fed to 19-free sides), UZ: Z unsigned too
   (a general addition's input; a mixed addition doubles Z into a 19-free
   sum with a centered product, so it needs Z centered).  Tables keep all
   four centered (their sums Y+X are 19-sides). */
template <bool UXYT, bool UZ>
FD_DEV void ge_p1p1_to_p3_t(ge_p3& r, const ge_p1p1& p) {
  fe x19, z19;
  fe_19(x19, p.X);
  fe_19(z19, p.Z);
  if (UXYT) {
    fe_mul19_u(r.X, p.T, p.X, x19);
    fe_mul19_u(r.T, p.Y, p.X, x19);
    fe_mul19_u(r.Y, p.Y, p.Z, z19);
  } else {
    fe_mul19(r.X, p.T, p.X, x19);
    fe_mul19(r.T, p.Y, p.X, x19);
    fe_mul19(r.Y, p.Y, p.Z, z19);
  }
  if (UZ) fe_mul19_u(r.Z, p.T, p.Z, z19);
  else fe_mul19(r.Z, p.T, p.Z, z19);
}

FD_DEV void ge_p1p1_to_p3(ge_p3& r, const ge_p1p1& p) { ge_p1p1_to_p3_t<false, false>(r, p); }
/* before a general addition */
FD_DEV void ge_p1p1_to_p3_u(ge_p3& r, const ge_p1p1& p) { ge_p1p1_to_p3_t<true, true>(r, p); }
/* before a mixed addition */
FD_DEV void ge_p1p1_to_p3_uxyt(ge_p3& r, const ge_p1p1& p) { ge_p1p1_to_p3_t<true, false>(r, p); }

/* r = 2p  (4 squarings), |X|, |Y|, |Z| <= 2x.  dbl-2008-hwcd with
   2XY = X^2 + Y^2 - (X-Y)^2; X^2 centered, the other squares unsigned:
     r.Y = Y^2 + X^2            in [-1x, 3x]
     r.Z = Y^2 - X^2            in [-1x, 3x]
     r.X = r.Y - (X-Y)^2        in [-3x, 3x]
     r.T = 2Z^2 - r.Z           in [-3x, 3x] */
FD_DEV void ge_p2_dbl(ge_p1p1& r, const ge_p2& p) {
  fe xx, yy, b, a, aa;
  fe_sq(xx, p.X);
  fe_sq_u(yy, p.Y);
  fe_sq2_u(b, p.Z);
  fe_sub(a, p.X, p.Y);
  fe_sq_u(aa, a);
  fe_add(r.Y, yy, xx);
  fe_sub(r.Z, yy, xx);
  fe_sub(r.X, r.Y, aa);
  fe_sub(r.T, b, r.Z);
}

FD_DEV void ge_p3_dbl(ge_p1p1& r, const ge_p3& p) {
  ge_p2 q;
  q.X = p.X; q.Y = p.Y; q.Z = p.Z;
  ge_p2_dbl(r, q);
}

/* |X|, |Y| <= 1x (centered) or in [0, 2x] (unsigned), |Z| <= 1x: the
   entry's Y+X, Y-X and 2Z are 19-sides of the addition, so Y+X of two
   unsigned coordinates ([0, 4x]) is moved by p (limbs ~2x each, value 0)
   into [-2x, 2x] */
#define FE_P_LIMBS {(1 << 26) - 19, (1 << 25) - 1, (1 << 26) - 1, (1 << 25) - 1, (1 << 26) - 1, \
                    (1 << 25) - 1, (1 << 26) - 1, (1 << 25) - 1, (1 << 26) - 1, (1 << 25) - 1}
template <bool UXY = false>
FD_DEV void ge_p3_to_cached(ge_cached& r, const ge_p3& p) {
  const fe d2 = {FE_D2};
  if (UXY) {
    const fe pl = {FE_P_LIMBS};
#pragma unroll
    for (int i = 0; i < 10; i++) r.YplusX.v[i] = p.Y.v[i] + p.X.v[i] - pl.v[i];
  } else {
    fe_add(r.YplusX, p.Y, p.X);
  }
  fe_sub(r.YminusX, p.Y, p.X);
  fe_add(r.Z2, p.Z, p.Z);
  fe_mul_u(r.T2d, p.T, d2);
}

/* r = p + q (add-2008-hwcd-3, k = 2d, with 2 Z1 Z2 formed by the product
   against the entry's 2Z).  The products into r.X, r.Y and 2 Z1 Z2 are
   unsigned (U), so
     r.X = a - b in [-2x, 2x],  r.Y = a + b in [0, 4x];
   NT = false: q.T2d = 2dT, c = 2dT1T2 centered,
     r.Z = 2Z1Z2 + c, r.T = 2Z1Z2 - c in [-1x, 3x];
   NT = true: the table holds -2dT, c' = -2dT1T2 unsigned too,
     r.Z = 2Z1Z2 - c' in [-2x, 2x], r.T = 2Z1Z2 + c' in [0, 4x] --
   T then enters only the 19-free side of the next product (every
   conversion below takes X and Z as its 19-sides). */
template <bool NT = false>
FD_DEV void ge_add(ge_p1p1& r, const ge_p3& p, const ge_cached& q) {
  fe a, b, c, zz2;
  fe_add(a, p.Y, p.X);
  fe_sub(b, p.Y, p.X);
  fe_mul_u(a, a, q.YplusX);
  fe_mul_u(b, b, q.YminusX);
  fe_mul_u(zz2, p.Z, q.Z2);
  if (NT) fe_mul_u(c, q.T2d, p.T);
  else fe_mul(c, q.T2d, p.T);
  fe_sub(r.X, a, b);
  fe_add(r.Y, a, b);
  if (NT) {
    fe_sub(r.Z, zz2, c);
    fe_add(r.T, zz2, c);
  } else {
    fe_add(r.Z, zz2, c);
    fe_sub(r.T, zz2, c);
  }
}

/* r = p + q, q affine */
FD_DEV void ge_madd(ge_p1p1& r, const ge_p3& p, const ge_precomp& q) {
  fe a, b, c, t0;
  fe_add(a, p.Y, p.X);
  fe_sub(b, p.Y, p.X);
  fe_mul_u(a, a, q.yplusx);
  fe_mul_u(b, b, q.yminusx);
  fe_mul(c, q.xy2d, p.T);
  fe_add(t0, p.Z, p.Z);       /* p.Z centered: r.Z, r.T within 3x */
  fe_sub(r.X, a, b);
  fe_add(r.Y, a, b);
  fe_add(r.Z, t0, c);
  fe_sub(r.T, t0, c);
}

/* q <- neg ? -q : q for a cached point (swap Y+X/Y-X, negate 2dT) */
FD_DEV void ge_cached_cneg(ge_cached& q, bool neg) {
  fe t;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const int32_t a = q.YplusX.v[i], b = q.YminusX.v[i];
    q.YplusX.v[i] = neg ? b : a;
    q.YminusX.v[i] = neg ? a : b;
    t.v[i] = -q.T2d.v[i];
    q.T2d.v[i] = neg ? t.v[i] : q.T2d.v[i];
  }
}

FD_DEV void ge_precomp_cneg(ge_precomp& q, bool neg) {
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const int32_t a = q.yplusx.v[i], b = q.yminusx.v[i];
    q.yplusx.v[i] = neg ? b : a;
    q.yminusx.v[i] = neg ? a : b;
    const int32_t t = q.xy2d.v[i];
    q.xy2d.v[i] = neg ? -t : t;
  }
}
