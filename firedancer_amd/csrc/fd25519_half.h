/* fd25519_half.h -- half-size scalars for the verification equation.

   The reference checks E = [S]B - R - [k]A == 0 exactly (cofactorless,
   fd_ed25519_verify, src/ballet/ed25519/fd_ed25519_user.c:209-226).  The
   group of curve points has order 8L and is cyclic, so for any integers
   c, d with

       c == d k  (mod 8L),   d odd,   0 < |d| < L

   [d] is an automorphism of the group and [dk]P = [c]P for every point P,
   hence

       [d]E = [dS mod L]B - [d]R - [c]A,   and   E == 0  <=>  [d]E == 0.

   (B has order L, so its scalar may be reduced mod L; the odd d keeps the
   torsion components of A and R exactly as the reference sees them.)  With
   0 <= c, |d| < 2^131 the double-scalar multiplication becomes a
   four-scalar one whose scalars are all ~131 bits (dS mod L is split at
   2^132 with a second base table for [2^132]B): half the doublings.

   (c, d) is a short vector of the lattice {(c, d) : c == d k mod 8L}, found
   by the extended Euclidean algorithm on (8L, k): remainders r_i satisfy
   r_i == t_i k (mod 8L) and |t_i| <= 8L / r_{i-1}.  At the first remainder
   r_i below 2^131, (r_i, t_i) is taken if t_i is odd and short; otherwise
   (t_i even: t_{i-1} is odd, consecutive t being coprime) the vector
   (r_{i-1} - m r_i, t_{i-1} - m t_i) with the least m that brings the
   first coordinate below 2^131 (every t of that family is odd, and the
   least m gives the smallest |t|).  That |d| may exceed 2^131 (~0.16% of
   random k: the lattice is unbalanced, its short vector has an even d);
   the caller states how long a d it accepts (dbits: 131 for the strict
   half-size form, up to FD_HALF_DBITS_MAX for the extended one, whose
   multiplication simply runs a few more windows) and falls back to the
   full-length multiplication beyond that (~1e-6 of random k at 151 bits).

   The Euclidean steps run Lehmer-style (Knuth, TAOCP 4.5.2, Algorithm L):
   quotients are found from 52 leading bits, every value an exact integer
   in double precision (FMA remainders), and verified by the two-sided
   test, the cofactor matrix is
   applied to the full-length values once per round; the last steps near
   2^131 and rounds with an unverifiable quotient use single conservative
   steps (a quotient estimate never above the true one, so a step may be
   partial; the remainder sequence and its invariant are unchanged).

   Plain C++ on 32-bit limbs (compiled for the device by hipcc and for the
   host by g++ in the tests). */
#ifndef FD25519_HALF_H
#define FD25519_HALF_H

#include <stdint.h>

#ifndef FD_HALF_FN
#define FD_HALF_FN static inline
#endif

#define FD_HALF_BITS 131   /* 0 <= c < 2^FD_HALF_BITS, |d| < 2^dbits, dbits >= FD_HALF_BITS */
#define FD_HALF_DBITS_MAX 151  /* longest |d| the dsm kernel takes (38 windows of 4 bits) */
#define FD_HALF_TW   5     /* t values: 160-bit two's complement */
#ifndef FD_HALF_LEHMER_MARGIN
#define FD_HALF_LEHMER_MARGIN 0  /* Lehmer rounds stop this many bits above 2^FD_HALF_BITS (0: measured fastest, same fallback rate) */
#endif

/* 8L, little-endian 32-bit words */
#define FD_HALF_N8L {0xe7ae9f68u, 0xc09318d2u, 0x17bce6b2u, 0xa6f7cef5u, 0u, 0u, 0u, 0x80000000u}

template <int N>
FD_HALF_FN int fd_half_bitlen(const uint32_t (&x)[N]) {
  int r = 0;
#pragma unroll
  for (int i = 0; i < N; i++)
    if (x[i]) r = 32 * i + 32 - __builtin_clz(x[i]);
  return r;
}

/* (x >> s) truncated to 64 bits, 0 <= s < 256; select chains, no dynamic
   register indexing */
FD_HALF_FN uint64_t fd_half_shr64(const uint32_t (&x)[8], int s) {
  const int w = s >> 5, sh = s & 31;
  uint32_t x0 = 0u, x1 = 0u, x2 = 0u;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    x0 = i == w ? x[i] : x0;
    x1 = i == w + 1 ? x[i] : x1;
    x2 = i == w + 2 ? x[i] : x2;
  }
  const uint64_t lo = (((uint64_t)x1 << 32) | x0) >> sh;
  const uint64_t hi = (((uint64_t)x2 << 32) | x1) >> sh;
  return (lo & 0xffffffffu) | (hi << 32);
}

FD_HALF_FN int fd_half_lt(const uint32_t (&a)[8], const uint32_t (&b)[8]) {
  int r = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r = a[i] != b[i] ? (a[i] < b[i]) : r;
  return r;
}

/* out = m x mod 2^(32N), m < 2^64 */
template <int N>
FD_HALF_FN void fd_half_mul_small(uint32_t (&out)[N], const uint32_t (&x)[N], uint64_t m) {
  const uint64_t m0 = m & 0xffffffffu, m1 = m >> 32;
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    const uint64_t t = (uint64_t)x[i] * m0 + c;
    out[i] = (uint32_t)t;
    c = t >> 32;
  }
  c = 0;
#pragma unroll
  for (int i = 0; i + 1 < N; i++) {
    const uint64_t t = (uint64_t)x[i] * m1 + out[i + 1] + c;
    out[i + 1] = (uint32_t)t;
    c = t >> 32;
  }
}

/* out = A x + B y mod 2^(32N) for signed A, B with |A|, |B| < 2^63 */
template <int N>
FD_HALF_FN void fd_half_lin(uint32_t (&out)[N], const uint32_t (&x)[N], const uint32_t (&y)[N], int64_t A,
                            int64_t B) {
  uint32_t px[N], py[N];
  fd_half_mul_small<N>(px, x, (uint64_t)(A < 0 ? -A : A));
  fd_half_mul_small<N>(py, y, (uint64_t)(B < 0 ? -B : B));
  /* out = (+-px) + (+-py): negation as complement + 1 folded into the sum */
  const uint32_t fx = A < 0 ? 0xffffffffu : 0u, fy = B < 0 ? 0xffffffffu : 0u;
  uint64_t c = (uint64_t)(A < 0) + (uint64_t)(B < 0);
#pragma unroll
  for (int i = 0; i < N; i++) {
    const uint64_t t = (uint64_t)(px[i] ^ fx) + (uint64_t)(py[i] ^ fy) + c;
    out[i] = (uint32_t)t;
    c = t >> 32;
  }
}

/* a -= q b and t_a -= q t_b (mod 2^160), q < 2^64, q b <= a */
FD_HALF_FN void fd_half_step(uint32_t (&a)[8], const uint32_t (&b)[8], uint32_t (&ta)[FD_HALF_TW],
                             const uint32_t (&tb)[FD_HALF_TW], uint64_t q) {
  uint32_t p[8], pt[FD_HALF_TW];
  fd_half_mul_small<8>(p, b, q);
  fd_half_mul_small<FD_HALF_TW>(pt, tb, q);
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t t = (uint64_t)a[i] - p[i] - br;
    a[i] = (uint32_t)t;
    br = (t >> 63) & 1u;
  }
  br = 0;
#pragma unroll
  for (int i = 0; i < FD_HALF_TW; i++) {
    const uint64_t t = (uint64_t)ta[i] - pt[i] - br;
    ta[i] = (uint32_t)t;
    br = (t >> 63) & 1u;
  }
}

/* conservative quotient estimate: 1 <= q <= floor(a / b), for a >= b > 0 */
FD_HALF_FN uint64_t fd_half_quot(const uint32_t (&a)[8], const uint32_t (&b)[8]) {
  const int la = fd_half_bitlen<8>(a);
  const int s = la > 52 ? la - 52 : 0;
  const uint64_t ah = fd_half_shr64(a, s), bh = fd_half_shr64(b, s);
  /* a / b >= ah / (bh + 1); shrink by 2^-40 so rounding never overshoots */
  const double r = (double)ah / (double)(bh + 1u) * (1.0 - 0x1p-40);
  const uint64_t q = (uint64_t)r;
  return q ? q : 1u;
}

FD_HALF_FN void fd_half_swap(uint32_t (&a)[8], uint32_t (&b)[8], uint32_t (&ta)[FD_HALF_TW],
                             uint32_t (&tb)[FD_HALF_TW], int cond) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t x = a[i], y = b[i];
    a[i] = cond ? y : x;
    b[i] = cond ? x : y;
  }
#pragma unroll
  for (int i = 0; i < FD_HALF_TW; i++) {
    const uint32_t x = ta[i], y = tb[i];
    ta[i] = cond ? y : x;
    tb[i] = cond ? x : y;
  }
}

/* one conservative Euclidean step on (a, b), a >= b > 0, keeping a > b */
FD_HALF_FN void fd_half_single(uint32_t (&a)[8], uint32_t (&b)[8], uint32_t (&ta)[FD_HALF_TW],
                               uint32_t (&tb)[FD_HALF_TW]) {
  fd_half_step(a, b, ta, tb, fd_half_quot(a, b));
  fd_half_swap(a, b, ta, tb, fd_half_lt(a, b));
}

/* floor(x / y) for integers 0 <= x < 2^53, 0 < y < 2^53 held in doubles:
   an estimate from a refined reciprocal, then exact remainder corrections
   (fma(-q, y, x) is exact on these integers) */
#ifndef FD_HALF_RCP
#define FD_HALF_RCP(y) (1.0 / (y))
#endif
FD_HALF_FN double fd_half_fdiv(double x, double y) {
  double r = FD_HALF_RCP(y);
  r = __builtin_fma(r, __builtin_fma(-y, r, 1.0), r);
  double q = __builtin_floor(x * r);
#pragma unroll
  for (int i = 0; i < 2; i++) {
    const double rem = __builtin_fma(-q, y, x);
    q = rem < 0.0 ? q - 1.0 : (rem >= y ? q + 1.0 : q);
  }
  return q;
}

/* floor(x / y) for integers 0 <= x, 0 < y < 2^53 held in doubles, from a
   single-precision estimate (relative error < 2^-21.4: off by at most one
   below quotients of 2^20) and one exact correction (fma(-q, y, x) is
   exact here); -1 when the result is still not exact -- a quotient too
   large for the estimate, which ends the caller's Lehmer round */
#ifndef FD_HALF_RCPF
#define FD_HALF_RCPF(y) (1.0f / (y))
#endif
FD_HALF_FN double fd_half_fdiv32(double x, double y) {
  double q = __builtin_floor((double)((float)x * FD_HALF_RCPF((float)y)));
  double rem = __builtin_fma(-q, y, x);
  q = rem < 0.0 ? q - 1.0 : (rem >= y ? q + 1.0 : q);
  rem = __builtin_fma(-q, y, x);
  return (rem >= 0.0 && rem < y) ? q : -1.0;
}

/* floor(x / y) as fd_half_fdiv32, with the exactness test replaced by a
   bound on the estimate that makes one correction exact: below 2^20 the
   estimate is within 0.4 of x / y (relative error < 2^-21.4), so its floor
   is off by at most one; at or above 2^20 (and for y <= 0, x < 0, inf or
   NaN operands, whose results the caller discards) -1, which ends the
   caller's Lehmer round.  The test no longer waits on the corrected
   remainder: one fma and its compares fewer on the step's chain. */
FD_HALF_FN double fd_half_fdiv20(double x, double y) {
  const double e = (double)((float)x * FD_HALF_RCPF((float)y));
  double q = __builtin_floor(e);
  const double rem = __builtin_fma(-q, y, x);
  q = rem < 0.0 ? q - 1.0 : (rem >= y ? q + 1.0 : q);
  return e < 0x1p20 ? q : -1.0;
}

/* the Lehmer inner step's form: 0 the two-branch double-precision
   division (fd_half_fdiv), 1 one branch per step with fd_half_fdiv,
   2 one branch with fd_half_fdiv32, 3 one branch with fd_half_fdiv20 on
   unguarded operands (the operand checks only in the branch) and the
   cofactor updates ahead of it, 4 as 3 with two steps per branch */
#ifndef FD_HALF_INNER
#define FD_HALF_INNER 4
#endif
#if FD_HALF_INNER >= 3
#define FD_HALF_QUOT(x, y) fd_half_fdiv20((x), (y))
#elif FD_HALF_INNER == 2
#define FD_HALF_QUOT(x, y) fd_half_fdiv32((x), (y))
#else
#define FD_HALF_QUOT(x, y) fd_half_fdiv((x), (y))
#endif

/* |x| of a 160-bit two's complement value into mag, returns the sign */
FD_HALF_FN int fd_half_abs(uint32_t (&mag)[FD_HALF_TW], const uint32_t (&x)[FD_HALF_TW]) {
  const int neg = (int)(x[FD_HALF_TW - 1] >> 31);
  const uint32_t f = neg ? 0xffffffffu : 0u;
  uint64_t c = (uint64_t)neg;
#pragma unroll
  for (int i = 0; i < FD_HALF_TW; i++) {
    const uint64_t t = (uint64_t)(x[i] ^ f) + c;
    mag[i] = (uint32_t)t;
    c = t >> 32;
  }
  return neg;
}

/* Finds c, d with c == d k (mod 8L), d odd, 0 <= c < 2^131, |d| < 2^dbits
   (FD_HALF_BITS <= dbits <= FD_HALF_DBITS_MAX), for 0 <= k < L.  Returns 1
   and c (5 words), |d| (5 words), d's sign; 0 if no such pair was found
   within the bounds / iteration caps. */
FD_HALF_FN int fd_half_scalars(const uint32_t (&k)[8], uint32_t (&c)[FD_HALF_TW], uint32_t (&dmag)[FD_HALF_TW],
                               int* dneg, int dbits) {
  uint32_t a[8] = FD_HALF_N8L, b[8];
  uint32_t ta[FD_HALF_TW] = {0u, 0u, 0u, 0u, 0u}, tb[FD_HALF_TW] = {1u, 0u, 0u, 0u, 0u};
#pragma unroll
  for (int i = 0; i < 8; i++) b[i] = k[i];
  int ok = 1, it = 0;
  /* invariant: a > b >= 0, (a, ta), (b, tb) consecutive remainders with
     their cofactors (or a partially reduced one after a conservative step) */

  /* Lehmer rounds down to ~2^(131 + margin) */
  while (fd_half_bitlen<8>(b) > FD_HALF_BITS + FD_HALF_LEHMER_MARGIN) {
    if (++it > 200) { ok = 0; break; }
    const int s = fd_half_bitlen<8>(a) - 52;   /* a > 2^137: s > 0 */
    /* leading 52 bits and the cosequences, all exact integers in doubles */
    double uh = (double)fd_half_shr64(a, s), vh = (double)fd_half_shr64(b, s);
    /* the emulated remainder must stay above the margin (Knuth L with a floor) */
    const int fl = FD_HALF_BITS + FD_HALF_LEHMER_MARGIN - s;
    const double floor_v = fl > 0 ? (double)((uint64_t)1 << (fl < 62 ? fl : 62)) : 0.0;
    double Af = 1.0, Bf = 0.0, Cf = 0.0, Df = 1.0;
    for (int inner = 0; inner < 64; inner++) {
      const double x1 = uh + Af, y1 = vh + Cf, x2 = uh + Bf, y2 = vh + Df;
#if FD_HALF_INNER == 0
      if (!(y1 > 0.0 && y2 > 0.0 && x1 >= 0.0 && x2 >= 0.0)) break;
      const double q = fd_half_fdiv(x1, y1);
      if (q != fd_half_fdiv(x2, y2)) break;
      const double nv = __builtin_fma(-q, vh, uh);
      if (nv < floor_v) break;
#elif FD_HALF_INNER == 4
      /* two steps per branch: the second computed from the first's
         state as if the first passed; on a failed test the state falls
         back to the last step that passed */
      const bool valid = (y1 > 0.0) & (y2 > 0.0) & (x1 >= 0.0) & (x2 >= 0.0);
      const double q = fd_half_fdiv20(x1, y1), q2 = fd_half_fdiv20(x2, y2);
      const double nv = __builtin_fma(-q, vh, uh);
      const double nC = __builtin_fma(-q, Cf, Af), nD = __builtin_fma(-q, Df, Bf);
      const bool ok1 = valid & (q >= 0.0) & (q == q2) & (nv >= floor_v);
      /* step 2 on (vh, nv, Cf, nC, Df, nD) */
      const double x1b = vh + Cf, y1b = nv + nC, x2b = vh + Df, y2b = nv + nD;
      const bool validb = (y1b > 0.0) & (y2b > 0.0) & (x1b >= 0.0) & (x2b >= 0.0);
      const double qb = fd_half_fdiv20(x1b, y1b), q2b = fd_half_fdiv20(x2b, y2b);
      const double nvb = __builtin_fma(-qb, nv, vh);
      const double nCb = __builtin_fma(-qb, nC, Cf), nDb = __builtin_fma(-qb, nD, Df);
      const bool ok2 = validb & (qb >= 0.0) & (qb == q2b) & (nvb >= floor_v);
      if (!(ok1 & ok2)) {
        if (ok1) { Af = Cf; Cf = nC; Bf = Df; Df = nD; uh = vh; vh = nv; }
        break;
      }
      Af = nC; Cf = nCb; Bf = nD; Df = nDb;
      uh = nv; vh = nvb;
      inner++;
      continue;
#elif FD_HALF_INNER == 3
      /* the quotients straight from the operands: when an operand check
         fails, whatever they are is discarded with the step */
      const bool valid = (y1 > 0.0) & (y2 > 0.0) & (x1 >= 0.0) & (x2 >= 0.0);
      const double q = FD_HALF_QUOT(x1, y1), q2 = FD_HALF_QUOT(x2, y2);
      const double nv = __builtin_fma(-q, vh, uh);
      const double nC = __builtin_fma(-q, Cf, Af), nD = __builtin_fma(-q, Df, Bf);
      if (!(valid & (q >= 0.0) & (q == q2) & (nv >= floor_v))) break;
      Af = Cf; Cf = nC; Bf = Df; Df = nD;
      uh = vh; vh = nv;
      continue;
#else
      /* every test of the step folded into one branch, both quotients
         computed side by side (the step is a latency chain at one wave) */
      const bool valid = (y1 > 0.0) & (y2 > 0.0) & (x1 >= 0.0) & (x2 >= 0.0);
      const double q = FD_HALF_QUOT(x1, valid ? y1 : 1.0), q2 = FD_HALF_QUOT(x2, valid ? y2 : 1.0);
      const double nv = __builtin_fma(-q, vh, uh);
      if (!(valid & (q >= 0.0) & (q == q2) & (nv >= floor_v))) break;
#endif
      double T = __builtin_fma(-q, Cf, Af); Af = Cf; Cf = T;
      T = __builtin_fma(-q, Df, Bf); Bf = Df; Df = T;
      uh = vh; vh = nv;
    }
    const int64_t A = (int64_t)Af, B = (int64_t)Bf, C = (int64_t)Cf, D = (int64_t)Df;
    if (B == 0) {
      fd_half_single(a, b, ta, tb);
    } else {
      uint32_t na[8], nb[8], nta[FD_HALF_TW], ntb[FD_HALF_TW];
      fd_half_lin<8>(na, a, b, A, B);
      fd_half_lin<8>(nb, a, b, C, D);
      fd_half_lin<FD_HALF_TW>(nta, ta, tb, A, B);
      fd_half_lin<FD_HALF_TW>(ntb, ta, tb, C, D);
#pragma unroll
      for (int i = 0; i < 8; i++) { a[i] = na[i]; b[i] = nb[i]; }
#pragma unroll
      for (int i = 0; i < FD_HALF_TW; i++) { ta[i] = nta[i]; tb[i] = ntb[i]; }
    }
  }
  /* single steps to the first remainder below 2^131 */
  while (ok && fd_half_bitlen<8>(b) > FD_HALF_BITS) {
    if (++it > 400) { ok = 0; break; }
    fd_half_single(a, b, ta, tb);
  }
  uint32_t cw[8], dw[FD_HALF_TW];
  if (tb[0] & 1u) {
    /* (r_i, t_i) */
#pragma unroll
    for (int i = 0; i < 8; i++) cw[i] = b[i];
#pragma unroll
    for (int i = 0; i < FD_HALF_TW; i++) dw[i] = tb[i];
  } else {
    /* (r_{i-1} - m r_i, t_{i-1} - m t_i), m = ceil((a - 2^131 + 1) / b) */
    uint32_t x[8], dummy[FD_HALF_TW] = {0u, 0u, 0u, 0u, 0u};
    const uint32_t zt[FD_HALF_TW] = {0u, 0u, 0u, 0u, 0u};
    /* x = a - 2^131 (a >= 2^131 unless the rounds overshot; then m = 0) */
    const int big = fd_half_bitlen<8>(a) > FD_HALF_BITS;
    uint64_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint32_t sub = i == FD_HALF_BITS / 32 ? (1u << (FD_HALF_BITS % 32)) : 0u;
      const uint64_t t = (uint64_t)a[i] - sub - br;
      x[i] = (uint32_t)t;
      br = (t >> 63) & 1u;
    }
    /* m = floor(x / b) + 1 (then a - m b < 2^131 <= a - (m-1) b) */
    uint64_t m = 0;
    const int zb = fd_half_bitlen<8>(b) == 0;
    if (zb || fd_half_bitlen<8>(a) - fd_half_bitlen<8>(b) > 60) ok = 0;
    int guard = 0;
    while (ok && big && !fd_half_lt(x, b)) {
      if (++guard > 8) { ok = 0; break; }
      const uint64_t q = fd_half_quot(x, b);
      fd_half_step(x, b, dummy, zt, q);
      m += q;
    }
    if (big) m += 1;
    /* |t_{i-1} - m t_i| = |t_{i-1}| + m |t_i| must not wrap the 160-bit t
       (|t_{i-1}| <= |t_i| < 2^125): require m |t_i| < 2^155 */
    {
      uint32_t tm[FD_HALF_TW];
      fd_half_abs(tm, tb);
      const int mb = m ? 64 - __builtin_clzll(m) : 0;
      if (mb + fd_half_bitlen<FD_HALF_TW>(tm) > 155) ok = 0;
    }
    fd_half_lin<8>(cw, a, b, 1, -(int64_t)m);
    fd_half_lin<FD_HALF_TW>(dw, ta, tb, 1, -(int64_t)m);
  }
#pragma unroll
  for (int i = 0; i < FD_HALF_TW; i++) c[i] = cw[i];
  *dneg = fd_half_abs(dmag, dw);
  uint32_t chi = 0u;
#pragma unroll
  for (int i = FD_HALF_TW; i < 8; i++) chi |= cw[i];
  if (chi || fd_half_bitlen<FD_HALF_TW>(c) > FD_HALF_BITS || fd_half_bitlen<FD_HALF_TW>(dmag) > dbits ||
      !(dw[0] & 1u))
    ok = 0;
  return ok;
}

#endif
