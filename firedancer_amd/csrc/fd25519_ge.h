/* fd25519_ge.h -- edwards25519 group operations for gfx950 (one point per
   lane), a = -1 twisted Edwards in extended coordinates.

   Representations
     ge_p2      (X:Y:Z)            projective, x = X/Z, y = Y/Z
     ge_p3      (X:Y:Z:T)          extended, additionally xy = T/Z
     ge_p1p1    ((X:Z),(Y:T))      "completed", x = X/Z, y = Y/T
     ge_cached  (Y+X, Y-X, Z, 2dT) right operand of a general addition
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
struct ge_cached { fe YplusX, YminusX, Z, T2d; };
struct ge_precomp { fe yplusx, yminusx, xy2d; };

FD_DEV void ge_p3_0(ge_p3& h) {
  fe_0(h.X); fe_1(h.Y); fe_1(h.Z); fe_0(h.T);
}

#ifndef FD_GE_SHARE19
#define FD_GE_SHARE19 1
#endif

/* The conversions share each right operand between two products, so its
   19-multiples (the wrapped terms) are computed once. */
FD_DEV void ge_p1p1_to_p2(ge_p2& r, const ge_p1p1& p) {
#if FD_GE_SHARE19
  fe t19;
  fe_19(t19, p.T);
  fe_mul19(r.X, p.X, p.T, t19);
  fe_mul19(r.Z, p.Z, p.T, t19);
  fe_mul(r.Y, p.Y, p.Z);
#else
  fe_mul(r.X, p.X, p.T);
  fe_mul(r.Y, p.Y, p.Z);
  fe_mul(r.Z, p.Z, p.T);
#endif
}

FD_DEV void ge_p1p1_to_p3(ge_p3& r, const ge_p1p1& p) {
#if FD_GE_SHARE19
  fe t19, y19;
  fe_19(t19, p.T);
  fe_mul19(r.X, p.X, p.T, t19);
  fe_mul19(r.Z, p.Z, p.T, t19);
  fe_19(y19, p.Y);
  fe_mul19(r.Y, p.Z, p.Y, y19);
  fe_mul19(r.T, p.X, p.Y, y19);
#else
  fe_mul(r.X, p.X, p.T);
  fe_mul(r.Y, p.Y, p.Z);
  fe_mul(r.Z, p.Z, p.T);
  fe_mul(r.T, p.X, p.Y);
#endif
}

/* r = 2p  (4 squarings) */
FD_DEV void ge_p2_dbl(ge_p1p1& r, const ge_p2& p) {
  fe xx, yy, b, a, aa;
  fe_sq(xx, p.X);
  fe_sq(yy, p.Y);
  fe_sq2(b, p.Z);
  fe_add(a, p.X, p.Y);
  fe_sq(aa, a);
  fe_add(r.Y, yy, xx);
  fe_sub(r.Z, yy, xx);
  fe_sub(r.X, aa, r.Y);
  fe_sub(r.T, b, r.Z);
}

FD_DEV void ge_p3_dbl(ge_p1p1& r, const ge_p3& p) {
  ge_p2 q;
  q.X = p.X; q.Y = p.Y; q.Z = p.Z;
  ge_p2_dbl(r, q);
}

FD_DEV void ge_p3_to_cached(ge_cached& r, const ge_p3& p) {
  const fe d2 = {FE_D2};
  fe_add(r.YplusX, p.Y, p.X);
  fe_sub(r.YminusX, p.Y, p.X);
  r.Z = p.Z;
  fe_mul(r.T2d, p.T, d2);
}

/* the cached point back in extended form, scaled by 2:
   (Y+X) - (Y-X) = 2X, (Y+X) + (Y-X) = 2Y, 2Z, 2dT / d = 2T */
FD_DEV void ge_cached_to_p3(ge_p3& r, const ge_cached& c) {
  const fe dinv = {FE_DINV};
  fe t;
  fe_sub(t, c.YplusX, c.YminusX);
  fe_carry(r.X, t);
  fe_add(t, c.YplusX, c.YminusX);
  fe_carry(r.Y, t);
  fe_add(t, c.Z, c.Z);
  fe_carry(r.Z, t);
  fe_mul(r.T, c.T2d, dinv);
}

/* r = p + q */
FD_DEV void ge_add(ge_p1p1& r, const ge_p3& p, const ge_cached& q) {
  fe a, b, c, zz, t0;
  fe_add(a, p.Y, p.X);
  fe_sub(b, p.Y, p.X);
  fe_mul(a, a, q.YplusX);
  fe_mul(b, b, q.YminusX);
  fe_mul(c, q.T2d, p.T);
  fe_mul(zz, p.Z, q.Z);
  fe_add(t0, zz, zz);
  fe_sub(r.X, a, b);
  fe_add(r.Y, a, b);
  fe_add(r.Z, t0, c);
  fe_sub(r.T, t0, c);
}

/* r = p + q, q affine */
FD_DEV void ge_madd(ge_p1p1& r, const ge_p3& p, const ge_precomp& q) {
  fe a, b, c, t0;
  fe_add(a, p.Y, p.X);
  fe_sub(b, p.Y, p.X);
  fe_mul(a, a, q.yplusx);
  fe_mul(b, b, q.yminusx);
  fe_mul(c, q.xy2d, p.T);
  fe_add(t0, p.Z, p.Z);
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
