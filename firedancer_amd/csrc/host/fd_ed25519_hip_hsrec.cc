/* fd_ed25519_hip_hsrec.cc -- the scalar part of one signature's verify on
   the calling thread, for the drop-in's direct launches of a few
   signatures (host/fd_ed25519_hip_engine.c, dropin_run).

   What prep16's hash blocks compute on the device (fd_ed25519_kernels.hip:
   hash16_block -> hash_finish, scalar_one), here in host C++:

     k      = SHA-512( R || A || M ) mod L     (fd_ed25519_user.c:193-203)
     sflag  = S < L                             (fd_curve25519_scalar.h:57-73)
     c, d   : c == d k (mod 8L), d odd, 0 <= c < 2^131, |d| < 2^dbits
              (the product's half-size search, fd25519_half.h, compiled for
              the host; the pair is checked here as the device checks it)
     s'     = d S mod L, split at 2^144

   packed as the device's work arrays take them (one 32-word record:
   k[8], hs[19], sflag, hflag, 3 words of padding).  A prep16 launch given
   the records (fd_ed25519_verify_params_t.hsrec) runs only its decode
   blocks and copies the records into the work arrays, so a one-signature
   launch's critical path loses the hash -> search chain of one lane
   (~60 us of ~120, profiles/r5_prep_parts_ubench.txt) and keeps the
   decompressions (~44 us).  The pair found here may differ from the one
   the device's search would find (its quotient estimates use an
   approximate reciprocal); any pair that passes the check gives the same
   verdict. */
#include <stdint.h>
#include <string.h>

#include "../fd25519_half.h"

extern "C" void fd_ed25519_hip_private_challenge( unsigned char const sig[ 64 ], unsigned char const pub[ 32 ],
                                                  unsigned char const * msg, unsigned long msg_sz,
                                                  unsigned char out[ 64 ] );

namespace {

/* L = 2^252 + 27742317777372353535851937790883648493, 32-bit words */
const uint32_t L32[ 8 ] = { 0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu, 0u, 0u, 0u, 0x10000000u };

/* x (n little-endian 32-bit words) mod L.  Word by word from the top:
   r = (r 2^32 + w) mod L with t = r 2^32 + w < 2^285, q = t >> 252 is
   floor(t / L) or one more (t / 2^252 - t / L < 2^-90), so one conditional
   add of L fixes it. */
void
mod_l( uint32_t out[ 8 ], uint32_t const * x, int n ) {
  uint32_t r[ 8 ] = { 0 };
  for( int i=n-1; i>=0; i-- ) {
    uint32_t t[ 9 ];
    t[ 0 ] = x[ i ];
    for( int w=0; w<8; w++ ) t[ w+1 ] = r[ w ];
    /* q = t >> 252: bits 252..284 of the 288-bit t (words 7, 8) */
    uint64_t q = ( (uint64_t)t[ 8 ] << 4 ) | ( t[ 7 ] >> 28 );
    /* t -= q L (9 words), tracking the signed result */
    int64_t borrow = 0;
    unsigned __int128 carry = 0;   /* q < 2^33: q L_w + carry needs 66 bits */
    for( int w=0; w<9; w++ ) {
      unsigned __int128 ql = (unsigned __int128)q * ( w<8 ? L32[ w ] : 0u ) + carry;
      carry = ql >> 32;
      int64_t d = (int64_t)t[ w ] - (int64_t)(uint32_t)ql - borrow;
      borrow = d<0;
      t[ w ] = (uint32_t)d;
    }
    if( borrow ) {   /* q was one too many: add L back */
      uint64_t c = 0;
      for( int w=0; w<9; w++ ) {
        uint64_t s = (uint64_t)t[ w ] + ( w<8 ? L32[ w ] : 0u ) + c;
        t[ w ] = (uint32_t)s;
        c = s >> 32;
      }
    }
    for( int w=0; w<8; w++ ) r[ w ] = t[ w ];
  }
  memcpy( out, r, 32 );
}

/* a (na words) * b (nb words) -> out (na + nb words) */
void
mul_words( uint32_t * out, uint32_t const * a, int na, uint32_t const * b, int nb ) {
  memset( out, 0, 4UL*(unsigned long)( na + nb ) );
  for( int i=0; i<na; i++ ) {
    uint64_t c = 0;
    for( int j=0; j<nb; j++ ) {
      uint64_t t = (uint64_t)a[ i ] * b[ j ] + out[ i+j ] + c;
      out[ i+j ] = (uint32_t)t;
      c = t >> 32;
    }
    out[ i+nb ] = (uint32_t)c;
  }
}

bool
is_zero( uint32_t const * x, int n ) {
  uint32_t z = 0u;
  for( int i=0; i<n; i++ ) z |= x[ i ];
  return !z;
}

bool
lt_l( uint32_t const s[ 8 ] ) {   /* S < L, from the top word down */
  for( int i=7; i>=0; i-- ) {
    if( s[ i ]<L32[ i ] ) return true;
    if( s[ i ]>L32[ i ] ) return false;
  }
  return false;
}

/* c == d k (mod 8L) with d = (dneg ? -1 : 1) dm, d odd, and the size bounds:
   |d| k + (dneg ? c : 8L - c) is a multiple of 8L */
bool
pair_ok( uint32_t const k[ 8 ], uint32_t const ( &c )[ FD_HALF_TW ], uint32_t const ( &dm )[ FD_HALF_TW ], int dneg,
         int dbits ) {
  uint32_t x[ 8 + FD_HALF_TW + 1 ];
  mul_words( x, dm, FD_HALF_TW, k, 8 );
  x[ 8 + FD_HALF_TW ] = 0u;
  uint32_t add[ 8 ];
  if( dneg ) {
    for( int w=0; w<8; w++ ) add[ w ] = w<FD_HALF_TW ? c[ w ] : 0u;
  } else {   /* 8L - c */
    uint32_t l8[ 8 ];
    uint32_t cc = 0u;
    for( int w=0; w<8; w++ ) { l8[ w ] = ( L32[ w ] << 3 ) | cc; cc = L32[ w ] >> 29; }
    int64_t br = 0;
    for( int w=0; w<8; w++ ) {
      int64_t d = (int64_t)l8[ w ] - (int64_t)( w<FD_HALF_TW ? c[ w ] : 0u ) - br;
      br = d<0;
      add[ w ] = (uint32_t)d;
    }
  }
  uint64_t cy = 0;
  for( int w=0; w<8 + FD_HALF_TW + 1; w++ ) {
    uint64_t t = (uint64_t)x[ w ] + ( w<8 ? add[ w ] : 0u ) + cy;
    x[ w ] = (uint32_t)t;
    cy = t >> 32;
  }
  if( x[ 0 ] & 7u ) return false;
  for( int w=0; w<8 + FD_HALF_TW; w++ ) x[ w ] = ( x[ w ] >> 3 ) | ( x[ w+1 ] << 29 );
  x[ 8 + FD_HALF_TW ] >>= 3;
  uint32_t r[ 8 ];
  mod_l( r, x, 8 + FD_HALF_TW + 1 );
  return is_zero( r, 8 ) && ( dm[ 0 ] & 1u ) && fd_half_bitlen<FD_HALF_TW>( c )<=FD_HALF_BITS &&
         fd_half_bitlen<FD_HALF_TW>( dm )<=dbits;
}

} /* namespace */

/* 1: rec holds the signature's record; 0: its k has no half-size pair
   within dbits (about 1e-6 of signatures at 151 bits): the caller takes the
   device's own path for that launch (whose full-length form handles it). */
extern "C" int
fd_ed25519_hip_private_hsrec( unsigned char const sig[ 64 ], unsigned char const pub[ 32 ],
                              unsigned char const * msg, unsigned long msg_sz, int dbits, uint32_t rec[ 32 ] ) {
  unsigned char dig[ 64 ];
  fd_ed25519_hip_private_challenge( sig, pub, msg, msg_sz, dig );
  uint32_t h[ 16 ], k[ 8 ], S[ 8 ];
  for( int w=0; w<16; w++ ) h[ w ] = (uint32_t)dig[ 4*w ] | (uint32_t)dig[ 4*w+1 ] << 8 |
                                     (uint32_t)dig[ 4*w+2 ] << 16 | (uint32_t)dig[ 4*w+3 ] << 24;
  for( int w=0; w<8; w++ ) S[ w ] = (uint32_t)sig[ 32+4*w ] | (uint32_t)sig[ 33+4*w ] << 8 |
                                    (uint32_t)sig[ 34+4*w ] << 16 | (uint32_t)sig[ 35+4*w ] << 24;
  mod_l( k, h, 16 );
  int sflag = lt_l( S );
  uint32_t c[ FD_HALF_TW ], dm[ FD_HALF_TW ];
  int dneg = 0;
  int ok = fd_half_scalars( k, c, dm, &dneg, dbits ) && pair_ok( k, c, dm, dneg, dbits );
  if( !ok && sflag ) return 0;
  if( !ok ) {   /* S >= L: decided before the equation, any scalars do (scalar_one) */
    memset( c, 0, sizeof(c) ); memset( dm, 0, sizeof(dm) ); dm[ 0 ] = 1u; dneg = 0;
  }
  /* s' = d S mod L */
  uint32_t prod[ 8 + FD_HALF_TW ], sp[ 8 ];
  mul_words( prod, dm, FD_HALF_TW, S, 8 );
  mod_l( sp, prod, 8 + FD_HALF_TW );
  if( dneg && !is_zero( sp, 8 ) ) {
    int64_t br = 0;
    for( int w=0; w<8; w++ ) {
      int64_t d = (int64_t)L32[ w ] - (int64_t)sp[ w ] - br;
      br = d<0;
      sp[ w ] = (uint32_t)d;
    }
  }
  memset( rec, 0, 32UL*4UL );
  for( int w=0; w<8; w++ ) rec[ w ] = k[ w ];
  for( int w=0; w<5; w++ ) {
    rec[ 8 + w ]      = c[ w ];
    rec[ 8 + 5 + w ]  = dm[ w ];
    rec[ 8 + 10 + w ] = w<4 ? sp[ w ] : ( sp[ 4 ] & 0xffffu );                    /* bits 0..143   */
  }
  for( int w=0; w<4; w++ )                                                       /* bits 144..252 */
    rec[ 8 + 15 + w ] = ( sp[ w+4 ] >> 16 ) | ( ( w+5<8 ? sp[ w+5 ] : 0u ) << 16 );
  rec[ 27 ] = (uint32_t)sflag;
  rec[ 28 ] = dneg ? 1u : 0u;   /* FD_HF_DNEG; never FD_HF_FULL here */
  return 1;
}
