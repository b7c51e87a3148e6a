/* fd25519_sc.h -- scalars mod L = 2^252 + 27742317777372353535851937790883648493
   on gfx950, one scalar per lane, as 8 little-endian 32-bit words.

   sc_is_canonical restates fd_curve25519_scalar_validate
   (src/ballet/ed25519/fd_curve25519_scalar.h:57-73): S is accepted iff
   S <= L-1 as a 256-bit little-endian integer.

   sc_reduce512 computes a 512-bit little-endian value mod L (the role of
   fd_curve25519_scalar_reduce, src/ballet/ed25519/fd_curve25519_scalar.c:3-110):
   the value is split into 24 signed 21-bit digits in 64-bit registers and
   digits of weight >= 2^252 are folded down with
   2^252 = -(L - 2^252) = sum m_i 2^(21 i) (mod L),
   m = (666643, 470296, 654183, -997805, 136657, -683901), followed by
   centered carries; two final passes fold the last overflow and
   canonicalize with floor carries.  Each fold is six v_mad_i64_i32. */
#pragma once
#include "fd25519_fe.h"

FD_DEV bool sc_is_canonical(const uint32_t (&s)[8]) {
  const uint32_t l[8] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu, 0u, 0u, 0u, 0x10000000u};
  bool lt = false, eq = true;
#pragma unroll
  for (int i = 7; i >= 0; i--) {
    lt = lt || (eq && s[i] < l[i]);
    eq = eq && (s[i] == l[i]);
  }
  return lt;
}

FD_DEV void sc_fold(int64_t (&s)[24], int k) {
  const int64_t x = s[k];
  s[k - 12] += x * 666643;
  s[k - 11] += x * 470296;
  s[k - 10] += x * 654183;
  s[k - 9] -= x * 997805;
  s[k - 8] += x * 136657;
  s[k - 7] -= x * 683901;
  s[k] = 0;
}

FD_DEV void sc_carry_c(int64_t (&s)[24], int i) {  /* centered */
  const int64_t c = (s[i] + (1LL << 20)) >> 21;
  s[i + 1] += c;
  s[i] -= c * (1LL << 21);
}

FD_DEV void sc_carry_f(int64_t (&s)[24], int i) {  /* floor */
  const int64_t c = s[i] >> 21;
  s[i + 1] += c;
  s[i] -= c * (1LL << 21);
}

FD_DEV void sc_reduce512(uint32_t (&out)[8], const uint32_t (&in)[16]) {
  int64_t s[24];
  const uint32_t m21 = (1u << 21) - 1u;
#pragma unroll
  for (int i = 0; i < 23; i++) {
    const int bit = 21 * i, w = bit >> 5, sh = bit & 31;
    const uint32_t lo = in[w], hi = (w + 1 < 16) ? in[w + 1] : 0u;
    s[i] = (int64_t)(__builtin_amdgcn_alignbit(hi, lo, sh) & m21);
  }
  s[23] = (int64_t)(in[15] >> 3);  /* bits 483..511 */

#pragma unroll
  for (int k = 23; k >= 18; k--) sc_fold(s, k);
#pragma unroll
  for (int i = 6; i <= 16; i += 2) sc_carry_c(s, i);
#pragma unroll
  for (int i = 7; i <= 15; i += 2) sc_carry_c(s, i);
#pragma unroll
  for (int k = 17; k >= 12; k--) sc_fold(s, k);
#pragma unroll
  for (int i = 0; i <= 10; i += 2) sc_carry_c(s, i);
#pragma unroll
  for (int i = 1; i <= 11; i += 2) sc_carry_c(s, i);
  sc_fold(s, 12);
#pragma unroll
  for (int i = 0; i <= 11; i++) sc_carry_f(s, i);
  sc_fold(s, 12);
#pragma unroll
  for (int i = 0; i <= 10; i++) sc_carry_f(s, i);

  /* pack 12 digits of 21 bits (s[i] in [0,2^21)) */
  uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const uint32_t v = (uint32_t)s[i];
    const int bit = 21 * i, wi = bit >> 5, sh = bit & 31;
    w[wi] |= v << sh;
    if (sh + 21 > 32 && wi + 1 < 8) w[wi + 1] |= v >> (32 - sh);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = w[i];
}
