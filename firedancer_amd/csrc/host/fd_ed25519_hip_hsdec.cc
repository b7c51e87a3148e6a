/* fd_ed25519_hip_hsdec.cc -- a point decompression on the calling thread,
   for the launches of a few signatures that also take their scalars from it
   (host/fd_ed25519_hip_hsrec.cc; host/fd_ed25519_hip_engine.c dropin_run,
   host/fd_ed25519_hip_tile.c pipe_submit_hs).

   Why on the host: a decompression is one chain of ~265 dependent field
   operations (x = u v^3 (u v^7)^((p-5)/8)).  A row of 16 lanes runs it in
   ~44 us on the device (prep16's decode blocks, ~300 cycles a squaring,
   profiles/r5_lanesplit_ubench.txt); one host core with 64x64->128
   products runs it in a few us.  For a launch of one signature that chain
   is on the call's critical path and nothing else can hide it; for the
   throughput path (thousands of signatures a launch) the device's decode
   kernels stay.

   Same acceptance rules and the same output as decode16_wave
   (fd_ed25519_kernels.hip) / ge_decode (fd25519_dsm.h), the reference's
   fd_ed25519_point_frombytes + fd_ed25519_affine_is_small_order
   (src/ballet/ed25519/fd_curve25519.h:104-170, fd_ed25519_user.c:150-175):
     fail  : no square root, or (the AVX-512 rule) x == 0 with the sign set
     small : x == 0, y == 0, or y one of the order-8 points' y (canonical y)
   and the work arrays' representation: x as fe_carry of its canonical
   bytes with the sign applied (fd25519_fe.h's centered radix-2^25.5 limbs,
   limb for limb what the device writes), y as fe_frombytes of the encoding
   (bit 255 dropped, values >= p kept as they are). */
#include <stdint.h>
#include <string.h>

namespace {

typedef unsigned __int128 u128;
const uint64_t M51 = ( 1ULL << 51 ) - 1ULL;

/* GF(2^255-19) in five unsigned 51-bit limbs (carried: each < 2^52) */
struct f51 { uint64_t v[ 5 ]; };

const f51 F_D      = { { 0x34dca135978a3ULL, 0x1a8283b156ebdULL, 0x5e7a26001c029ULL, 0x739c663a03cbbULL, 0x52036cee2b6ffULL } };
const f51 F_SQRTM1 = { { 0x61b274a0ea0b0ULL, 0xd5a5fc8f189dULL, 0x7ef5e9cbd0c60ULL, 0x78595a6804c9eULL, 0x2b8324804fc1dULL } };

inline uint64_t ld64( unsigned char const * p ) { uint64_t x; memcpy( &x, p, 8 ); return x; }

/* bit 255 ignored, values >= p accepted */
f51 frombytes( unsigned char const s[ 32 ] ) {
  uint64_t w0 = ld64( s ), w1 = ld64( s+8 ), w2 = ld64( s+16 ), w3 = ld64( s+24 );
  f51 h;
  h.v[ 0 ] = w0 & M51;
  h.v[ 1 ] = ( ( w0 >> 51 ) | ( w1 << 13 ) ) & M51;
  h.v[ 2 ] = ( ( w1 >> 38 ) | ( w2 << 26 ) ) & M51;
  h.v[ 3 ] = ( ( w2 >> 25 ) | ( w3 << 39 ) ) & M51;
  h.v[ 4 ] = ( w3 >> 12 ) & M51;
  return h;
}

/* column sums (each < 2^115) -> carried limbs (< 2^51, limb 1 < 2^51 + 2^15) */
inline f51 carry( u128 const ( &t )[ 5 ] ) {
  f51 h;
  u128 t1 = t[ 1 ], t2 = t[ 2 ], t3 = t[ 3 ], t4 = t[ 4 ];
  h.v[ 0 ] = (uint64_t)t[ 0 ] & M51; t1 += t[ 0 ] >> 51;
  h.v[ 1 ] = (uint64_t)t1 & M51;     t2 += t1 >> 51;
  h.v[ 2 ] = (uint64_t)t2 & M51;     t3 += t2 >> 51;
  h.v[ 3 ] = (uint64_t)t3 & M51;     t4 += t3 >> 51;
  h.v[ 4 ] = (uint64_t)t4 & M51;
  u128 w = (u128)h.v[ 0 ] + ( t4 >> 51 ) * 19U;
  h.v[ 0 ] = (uint64_t)w & M51;
  h.v[ 1 ] += (uint64_t)( w >> 51 );
  return h;
}

f51 mul( f51 const & f, f51 const & g ) {
  uint64_t const * a = f.v, * b = g.v;
  uint64_t b1 = b[ 1 ]*19ULL, b2 = b[ 2 ]*19ULL, b3 = b[ 3 ]*19ULL, b4 = b[ 4 ]*19ULL;
  u128 t[ 5 ];
  t[ 0 ] = (u128)a[ 0 ]*b[ 0 ] + (u128)a[ 1 ]*b4 + (u128)a[ 2 ]*b3 + (u128)a[ 3 ]*b2 + (u128)a[ 4 ]*b1;
  t[ 1 ] = (u128)a[ 0 ]*b[ 1 ] + (u128)a[ 1 ]*b[ 0 ] + (u128)a[ 2 ]*b4 + (u128)a[ 3 ]*b3 + (u128)a[ 4 ]*b2;
  t[ 2 ] = (u128)a[ 0 ]*b[ 2 ] + (u128)a[ 1 ]*b[ 1 ] + (u128)a[ 2 ]*b[ 0 ] + (u128)a[ 3 ]*b4 + (u128)a[ 4 ]*b3;
  t[ 3 ] = (u128)a[ 0 ]*b[ 3 ] + (u128)a[ 1 ]*b[ 2 ] + (u128)a[ 2 ]*b[ 1 ] + (u128)a[ 3 ]*b[ 0 ] + (u128)a[ 4 ]*b4;
  t[ 4 ] = (u128)a[ 0 ]*b[ 4 ] + (u128)a[ 1 ]*b[ 3 ] + (u128)a[ 2 ]*b[ 2 ] + (u128)a[ 3 ]*b[ 1 ] + (u128)a[ 4 ]*b[ 0 ];
  return carry( t );
}

f51 sq( f51 const & f ) {
  uint64_t const * a = f.v;
  uint64_t a0_2 = a[ 0 ]*2ULL, a1_2 = a[ 1 ]*2ULL, a1_38 = a[ 1 ]*38ULL, a2_38 = a[ 2 ]*38ULL,
           a3_38 = a[ 3 ]*38ULL, a3_19 = a[ 3 ]*19ULL, a4_19 = a[ 4 ]*19ULL;
  u128 t[ 5 ];
  t[ 0 ] = (u128)a[ 0 ]*a[ 0 ] + (u128)a1_38*a[ 4 ] + (u128)a2_38*a[ 3 ];
  t[ 1 ] = (u128)a0_2*a[ 1 ] + (u128)a2_38*a[ 4 ] + (u128)a3_19*a[ 3 ];
  t[ 2 ] = (u128)a0_2*a[ 2 ] + (u128)a[ 1 ]*a[ 1 ] + (u128)a3_38*a[ 4 ];
  t[ 3 ] = (u128)a0_2*a[ 3 ] + (u128)a1_2*a[ 2 ] + (u128)a4_19*a[ 4 ];
  t[ 4 ] = (u128)a0_2*a[ 4 ] + (u128)a1_2*a[ 3 ] + (u128)a[ 2 ]*a[ 2 ];
  return carry( t );
}

f51 add( f51 const & f, f51 const & g ) {
  f51 h;
  for( int i=0; i<5; i++ ) h.v[ i ] = f.v[ i ] + g.v[ i ];
  return h;
}

/* f - g + 4p, limb-wise non-negative for carried g (< 2^52) */
f51 sub( f51 const & f, f51 const & g ) {
  const uint64_t p4_0 = 0x1fffffffffffb4ULL, p4_i = 0x1ffffffffffffcULL;
  f51 h;
  h.v[ 0 ] = f.v[ 0 ] + p4_0 - g.v[ 0 ];
  for( int i=1; i<5; i++ ) h.v[ i ] = f.v[ i ] + p4_i - g.v[ i ];
  u128 t[ 5 ] = { h.v[ 0 ], h.v[ 1 ], h.v[ 2 ], h.v[ 3 ], h.v[ 4 ] };
  return carry( t );
}

f51 one() { f51 h = { { 1ULL, 0ULL, 0ULL, 0ULL, 0ULL } }; return h; }

/* f - g + 8p without the carry, for a value that only feeds mul / sq: g's
   limbs < 2^54 - 152, the result's < f's + 2^54 (mul and sq take limbs up
   to 2^55.5: b 19 < 2^64, five products < 2^118) */
f51 sub_lazy( f51 const & f, f51 const & g ) {
  const uint64_t p8_0 = 0x3fffffffffff68ULL, p8_i = 0x3ffffffffffff8ULL;
  f51 h;
  h.v[ 0 ] = f.v[ 0 ] + p8_0 - g.v[ 0 ];
  for( int i=1; i<5; i++ ) h.v[ i ] = f.v[ i ] + p8_i - g.v[ i ];
  return h;
}

/* canonical little-endian words (value mod p) */
void tobytes( uint32_t out[ 8 ], f51 const & f ) {
  u128 t[ 5 ] = { f.v[ 0 ], f.v[ 1 ], f.v[ 2 ], f.v[ 3 ], f.v[ 4 ] };
  f51 h = carry( t );   /* h < 2^255 + 2^67 < 2p */
  /* q = floor(h / p) in {0, 1}: h + 19 reaches 2^255 exactly when h >= p
     (the chain is exact carry propagation whatever the limb sizes); then
     h + 19 q mod 2^255 = h - q p */
  uint64_t q = ( h.v[ 0 ] + 19ULL ) >> 51;
  q = ( h.v[ 1 ] + q ) >> 51;
  q = ( h.v[ 2 ] + q ) >> 51;
  q = ( h.v[ 3 ] + q ) >> 51;
  q = ( h.v[ 4 ] + q ) >> 51;
  h.v[ 0 ] += 19ULL * q;
  h.v[ 1 ] += h.v[ 0 ] >> 51; h.v[ 0 ] &= M51;
  h.v[ 2 ] += h.v[ 1 ] >> 51; h.v[ 1 ] &= M51;
  h.v[ 3 ] += h.v[ 2 ] >> 51; h.v[ 2 ] &= M51;
  h.v[ 4 ] += h.v[ 3 ] >> 51; h.v[ 3 ] &= M51;
  h.v[ 4 ] &= M51;
  uint64_t w[ 4 ] = { h.v[ 0 ] | ( h.v[ 1 ] << 51 ), ( h.v[ 1 ] >> 13 ) | ( h.v[ 2 ] << 38 ),
                      ( h.v[ 2 ] >> 26 ) | ( h.v[ 3 ] << 25 ), ( h.v[ 3 ] >> 39 ) | ( h.v[ 4 ] << 12 ) };
  for( int i=0; i<4; i++ ) { out[ 2*i ] = (uint32_t)w[ i ]; out[ 2*i+1 ] = (uint32_t)( w[ i ] >> 32 ); }
}

bool iszero( f51 const & f ) {
  uint32_t b[ 8 ];
  tobytes( b, f );
  uint32_t z = 0u;
  for( int i=0; i<8; i++ ) z |= b[ i ];
  return !z;
}

/* z^(2^252 - 3) for N independent elements at once: the chain is latency
   bound (each squaring waits for the last), so N chains side by side keep
   the core's multipliers busy -- a launch's A and R decompress in about the
   time of one */
template< int N >
void sqn_n( f51 ( &f )[ N ], int n ) {
  for( int k=0; k<n; k++ ) for( int i=0; i<N; i++ ) f[ i ] = sq( f[ i ] );
}

template< int N >
void mul_n( f51 ( &h )[ N ], f51 const ( &f )[ N ], f51 const ( &g )[ N ] ) {
  for( int i=0; i<N; i++ ) h[ i ] = mul( f[ i ], g[ i ] );
}

template< int N >
void pow22523_n( f51 ( &z )[ N ] ) {
  f51 t0[ N ], t1[ N ], t2[ N ];
  for( int i=0; i<N; i++ ) { t0[ i ] = sq( z[ i ] ); t1[ i ] = t0[ i ]; }   /* 2         */
  sqn_n( t1, 2 );                                                            /* 8         */
  mul_n( t1, z, t1 );                                                        /* 9         */
  mul_n( t0, t0, t1 );                                                       /* 11        */
  sqn_n( t0, 1 );                                                            /* 22        */
  mul_n( t0, t1, t0 );                                                       /* 2^5 - 1   */
  for( int i=0; i<N; i++ ) t1[ i ] = t0[ i ];
  sqn_n( t1, 5 );   mul_n( t0, t1, t0 );                                     /* 2^10 - 1  */
  for( int i=0; i<N; i++ ) t1[ i ] = t0[ i ];
  sqn_n( t1, 10 );  mul_n( t1, t1, t0 );                                     /* 2^20 - 1  */
  for( int i=0; i<N; i++ ) t2[ i ] = t1[ i ];
  sqn_n( t2, 20 );  mul_n( t1, t2, t1 );                                     /* 2^40 - 1  */
  sqn_n( t1, 10 );  mul_n( t0, t1, t0 );                                     /* 2^50 - 1  */
  for( int i=0; i<N; i++ ) t1[ i ] = t0[ i ];
  sqn_n( t1, 50 );  mul_n( t1, t1, t0 );                                     /* 2^100 - 1 */
  for( int i=0; i<N; i++ ) t2[ i ] = t1[ i ];
  sqn_n( t2, 100 ); mul_n( t1, t2, t1 );                                     /* 2^200 - 1 */
  sqn_n( t1, 50 );  mul_n( t0, t1, t0 );                                     /* 2^250 - 1 */
  sqn_n( t0, 2 );                                                            /* 2^252 - 4 */
  mul_n( z, t0, z );                                                         /* 2^252 - 3 */
}

/* fd25519_fe.h fe_frombytes: limb i = bits [ceil(25.5 i), ceil(25.5 (i+1))) */
void limbs_frombytes( int32_t h[ 10 ], uint32_t const w[ 8 ] ) {
  uint64_t v[ 4 ];
  for( int i=0; i<4; i++ ) v[ i ] = (uint64_t)w[ 2*i ] | ( (uint64_t)w[ 2*i+1 ] << 32 );
  static const int off[ 10 ] = { 0, 26, 51, 77, 102, 128, 153, 179, 204, 230 };
  for( int i=0; i<10; i++ ) {
    int o = off[ i ], wd = ( i & 1 ) ? 25 : 26;
    uint64_t lo = v[ o >> 6 ] >> ( o & 63 );
    if( ( o & 63 ) + wd > 64 ) lo |= v[ ( o >> 6 ) + 1 ] << ( 64 - ( o & 63 ) );
    h[ i ] = (int32_t)( lo & ( ( 1ULL << wd ) - 1ULL ) );
  }
}

/* fd25519_fe.h fe_carry (fe_carry_wide on biased columns), step for step */
void limbs_carry( int32_t h[ 10 ], int32_t const f[ 10 ] ) {
  int64_t a[ 10 ];
  for( int i=0; i<10; i++ ) a[ i ] = (int64_t)f[ i ] + ( ( i & 1 ) ? ( 1LL << 24 ) : ( 1LL << 25 ) );
  const int64_t m26 = ( 1LL << 26 ) - 1, m25 = ( 1LL << 25 ) - 1;
  int64_t c;
  c = a[ 0 ] >> 26; a[ 1 ] += c; a[ 0 ] &= m26;
  c = a[ 4 ] >> 26; a[ 5 ] += c; a[ 4 ] &= m26;
  c = a[ 1 ] >> 25; a[ 2 ] += c; h[ 1 ] = (int32_t)( a[ 1 ] & m25 ) - ( 1 << 24 );
  c = a[ 5 ] >> 25; a[ 6 ] += c; h[ 5 ] = (int32_t)( a[ 5 ] & m25 ) - ( 1 << 24 );
  c = a[ 2 ] >> 26; a[ 3 ] += c; h[ 2 ] = (int32_t)( a[ 2 ] & m26 ) - ( 1 << 25 );
  c = a[ 6 ] >> 26; a[ 7 ] += c; h[ 6 ] = (int32_t)( a[ 6 ] & m26 ) - ( 1 << 25 );
  c = a[ 3 ] >> 25; a[ 4 ] += c; h[ 3 ] = (int32_t)( a[ 3 ] & m25 ) - ( 1 << 24 );
  c = a[ 7 ] >> 25; a[ 8 ] += c; h[ 7 ] = (int32_t)( a[ 7 ] & m25 ) - ( 1 << 24 );
  c = a[ 4 ] >> 26; h[ 5 ] += (int32_t)c; h[ 4 ] = (int32_t)( a[ 4 ] & m26 ) - ( 1 << 25 );
  c = a[ 8 ] >> 26; a[ 9 ] += c; h[ 8 ] = (int32_t)( a[ 8 ] & m26 ) - ( 1 << 25 );
  c = a[ 9 ] >> 25; a[ 0 ] += c * 19; h[ 9 ] = (int32_t)( a[ 9 ] & m25 ) - ( 1 << 24 );
  c = a[ 0 ] >> 26; h[ 1 ] += (int32_t)c; h[ 0 ] = (int32_t)( a[ 0 ] & m26 ) - ( 1 << 25 );
}

const uint32_t Y0[ 8 ] = { 0x8f95e826u, 0xb027b2c2u, 0x89f4c345u, 0xf098eff2u,
                           0x05acdfd5u, 0x3933c6d3u, 0x880238b1u, 0x05fc536du };
const uint32_t Y1[ 8 ] = { 0x706a17c7u, 0x4fd84d3du, 0x760b3cbau, 0x0f67100du,
                           0xfa53202au, 0xc6cc392cu, 0x77fdc74eu, 0x7a03ac92u };

/* one point's decompression around the shared exponentiation */
struct dec_state {
  uint32_t sign;
  f51 y, u, v, v3;
};

void dec_pre( dec_state & d, f51 & x, unsigned char const enc[ 32 ] ) {
  uint32_t w7;
  memcpy( &w7, enc + 28, 4 );
  d.sign = w7 >> 31;
  d.y = frombytes( enc );
  f51 u = sq( d.y );
  d.v  = add( mul( u, F_D ), one() );          /* d y^2 + 1 */
  d.u  = sub( u, one() );                      /* y^2 - 1   */
  d.v3 = mul( sq( d.v ), d.v );                /* v^3       */
  x = mul( mul( sq( d.v3 ), d.v ), d.u );      /* u v^7     */
}

unsigned dec_post( dec_state const & d, f51 x, unsigned char const enc[ 32 ], int avx_rule, int32_t pt[ 20 ],
                   f51 * xs ) {
  x = mul( mul( x, d.v3 ), d.u );              /* u v^3 (u v^7)^((p-5)/8) */
  f51 vxx = mul( sq( x ), d.v );
  const bool root  = iszero( sub( vxx, d.u ) );
  const bool iroot = iszero( add( vxx, d.u ) );
  if( !root ) x = mul( x, F_SQRTM1 );
  uint32_t xb[ 8 ];
  tobytes( xb, x );
  uint32_t z = 0u;
  for( int i=0; i<8; i++ ) z |= xb[ i ];
  const bool x0 = !z;
  const bool fail = !( root || iroot ) || ( avx_rule && x0 && d.sign );
  const bool neg = ( xb[ 0 ] & 1u ) != d.sign;
  /* small order on the canonical y */
  uint32_t yb[ 8 ];
  tobytes( yb, d.y );
  uint32_t zy = 0u, e0 = 0u, e1 = 0u;
  for( int i=0; i<8; i++ ) { zy |= yb[ i ]; e0 |= yb[ i ] ^ Y0[ i ]; e1 |= yb[ i ] ^ Y1[ i ]; }
  const bool small = x0 || !zy || !e0 || !e1;
  /* the device's representation (decode16_wave's stores) */
  int32_t t[ 10 ];
  limbs_frombytes( t, xb );
  limbs_carry( pt, t );
  if( neg ) for( int i=0; i<10; i++ ) pt[ i ] = -pt[ i ];
  if( xs ) *xs = neg ? sub( f51{ { 0ULL, 0ULL, 0ULL, 0ULL, 0ULL } }, x ) : x;
  uint32_t ew[ 8 ];
  memcpy( ew, enc, 32 );
  ew[ 7 ] &= 0x7fffffffu;   /* fe_frombytes drops bit 255 (limb 9 is 25 bits wide) */
  limbs_frombytes( pt + 10, ew );
  return ( fail ? 1u : 0u ) | ( small ? 2u : 0u );
}

/* [2^(step m)](x, y) for m = 1 .. nx (nx <= 3), for N points at once
   (extended coordinates without T, dbl-2008-hwcd for a = -1), returned in
   extended coordinates (X Z, Y Z, Z^2, X Y) -- no inversion: ox[ i nx +
   m-1 ][ 4 ] */
template< int N >
void dbl_n( f51 const ( &x )[ N ], f51 const ( &y )[ N ], int step, int nx, f51 ( *ox )[ 4 ] ) {
  const f51 zero = { { 0ULL, 0ULL, 0ULL, 0ULL, 0ULL } };
  f51 X[ N ], Y[ N ], Z[ N ];
  for( int i=0; i<N; i++ ) { X[ i ] = x[ i ]; Y[ i ] = y[ i ]; Z[ i ] = one(); }
  for( int m=0; m<nx; m++ ) {
    for( int r=0; r<step; r++ ) {
      for( int i=0; i<N; i++ ) {
        /* A, B, Z2 carried (< 2^52); every difference below only feeds a
           product, so none is carried: E, F < 2^55.2, G, H < 2^54.3 */
        f51 A = sq( X[ i ] ), B = sq( Y[ i ] ), Z2 = sq( Z[ i ] );
        f51 C = add( Z2, Z2 );                                      /* < 2^53   */
        f51 E = sub_lazy( sub_lazy( sq( add( X[ i ], Y[ i ] ) ), A ), B );
        f51 G = sub_lazy( B, A );               /* D + B, D = -A */
        f51 F = sub_lazy( G, C );
        f51 H = sub_lazy( zero, add( A, B ) );  /* D - B         */
        X[ i ] = mul( E, F ); Y[ i ] = mul( G, H ); Z[ i ] = mul( F, G );
      }
    }
    for( int i=0; i<N; i++ ) {
      f51 * o = ox[ i*nx + m ];
      o[ 0 ] = mul( X[ i ], Z[ i ] ); o[ 1 ] = mul( Y[ i ], Z[ i ] ); o[ 2 ] = sq( Z[ i ] ); o[ 3 ] = mul( X[ i ], Y[ i ] );
    }
  }
}

/* the device's tight limbs of one coordinate (fe_carry of its canonical
   bytes) */
void limbs_coord( int32_t out[ 10 ], f51 const & v ) {
  uint32_t b[ 8 ];
  int32_t t[ 10 ];
  tobytes( b, v );
  limbs_frombytes( t, b );
  limbs_carry( out, t );
}

template< int N >
void dec_n( unsigned char const * const * enc, int avx_rule, int32_t * pt, unsigned char * flags, int32_t * ptx,
            int nx, int step ) {
  dec_state d[ N ];
  f51 x[ N ];
  for( int i=0; i<N; i++ ) dec_pre( d[ i ], x[ i ], enc[ i ] );
  pow22523_n< N >( x );
  f51 xs[ N ], ys[ N ];
  for( int i=0; i<N; i++ ) {
    flags[ i ] = (unsigned char)dec_post( d[ i ], x[ i ], enc[ i ], avx_rule, pt + 20*i, &xs[ i ] );
    ys[ i ] = d[ i ].y;
  }
  if( !ptx || nx<1 ) return;
  f51 ox[ N*3 ][ 4 ];
  dbl_n< N >( xs, ys, step, nx, ox );
  for( int t=0; t<N*nx; t++ ) for( int c=0; c<4; c++ ) limbs_coord( ptx + 40*t + 10*c, ox[ t ][ c ] );
}

} /* namespace */

/* enc[i]: n 32-byte point encodings (public keys and Rs).  pt: n x 20
   int32, the work arrays' limbs of (x, y) per point; flags[i]: 1
   FD_PF_FAIL, 2 FD_PF_SMALL (fd_ed25519_hip_internal.h).  avx_rule: the
   AVX-512 build's codes (an engine without
   FD_ED25519_HIP_FLAG_CODES_PORTABLE).  ptx (when not NULL): each point
   also doubled step, 2 step, .. nx step times (nx <= 3), in extended
   coordinates (X, Y, Z, T: 40 limbs, each coordinate as the device's tight
   limbs) -- ptx[(i nx + m-1) 40 ..] = [2^(step m)]P_i, the split forms'
   A_i and R_i (a failed decode's are any values: its code is the
   decode's). */
extern "C" void
fd_ed25519_hip_private_hsdec3_n( unsigned char const * const * enc, unsigned long n, int avx_rule, int32_t * pt,
                                 int32_t * ptx, int nx, int step, unsigned char * flags ) {
  if( nx>3 ) nx = 3;
  unsigned long i = 0UL;
#define HSDEC_GROUP( N ) dec_n< N >( enc + i, avx_rule, pt + 20UL*i, flags + i, \
                                     ptx ? ptx + 40UL*(unsigned long)nx*i : NULL, nx, step )
  for( ; i+4UL<=n; i+=4UL ) HSDEC_GROUP( 4 );
  if( n-i==3UL ) HSDEC_GROUP( 3 );
  if( n-i==2UL ) HSDEC_GROUP( 2 );
  if( n-i==1UL ) HSDEC_GROUP( 1 );
#undef HSDEC_GROUP
}

extern "C" void
fd_ed25519_hip_private_hsdec_n( unsigned char const * const * enc, unsigned long n, int avx_rule, int32_t * pt,
                                unsigned char * flags ) {
  fd_ed25519_hip_private_hsdec3_n( enc, n, avx_rule, pt, NULL, 0, 0, flags );
}

/* the split forms' scalars from a host record (hsrec's layout: c
   rec[8..12], |d| rec[13..17], s' = rec[18..22] (bits 0..143) + rec[23..26]
   << 144), at column j of stride cap:
     waves 4: rows 3q..3q+2 = c0, c1, d0, d1 (c and |d| split at bit 66),
              rows 12+3q..14+3q = bits [72 q, 72 q + 72) of s';
     waves 8: rows 2q, 2q+1 = c0..c3, d0..d3 (split every 33 bits, the
              last part the rest), row 16+q = bits [32 q, 32 q + 32). */
extern "C" void
fd_ed25519_hip_private_hssplit( uint32_t const rec[ 32 ], int waves, uint32_t * hq, unsigned long cap, unsigned long j ) {
  const int H = waves==8 ? 4 : 2, G = waves==8 ? 33 : 66, KW = waves==8 ? 2 : 3;
  for( int side=0; side<2; side++ ) {
    uint32_t const * w = rec + ( side ? 13 : 8 );   /* 160 bits */
    for( int i=0; i<H; i++ ) {
      /* bits [G i, G (i+1)) of the value -- the last part all the rest -- as KW words */
      for( int o=0; o<KW; o++ ) {
        int b = G*i + 32*o;
        uint32_t x = 0u;
        if( b<160 ) {
          int wi = b >> 5, sh = b & 31;
          uint64_t v = (uint64_t)w[ wi ] | ( wi+1<5 ? (uint64_t)w[ wi+1 ] << 32 : 0ULL );
          x = (uint32_t)( v >> sh );
        }
        int keep = i<H-1 ? G - 32*o : 160;   /* bits of this word that belong to the part */
        if( keep<=0 ) x = 0u;
        else if( keep<32 ) x &= ( 1u << keep ) - 1u;
        hq[ (unsigned long)( KW*( H*side + i ) + o )*cap + j ] = x;
      }
    }
  }
  /* s' (253 bits) from its two halves */
  uint32_t sw[ 9 ];
  for( int o=0; o<4; o++ ) sw[ o ] = rec[ 18 + o ];
  sw[ 4 ] = ( rec[ 22 ] & 0xffffu ) | ( rec[ 23 ] << 16 );
  for( int o=5; o<8; o++ ) sw[ o ] = ( rec[ 18 + o ] >> 16 ) | ( rec[ 19 + o ] << 16 );
  sw[ 8 ] = rec[ 26 ] >> 16;
  if( waves==8 ) {
    for( int q=0; q<8; q++ ) hq[ (unsigned long)( 16 + q )*cap + j ] = sw[ q ];
    return;
  }
  for( int q=0; q<4; q++ ) {
    for( int o=0; o<3; o++ ) {   /* bits 72q + 32o .. +31 of s', masked to the chunk's 72 */
      int b = 72*q + 32*o, wi = b >> 5, sh = b & 31;
      uint64_t v = (uint64_t)sw[ wi ] | ( wi+1<9 ? (uint64_t)sw[ wi+1 ] << 32 : 0ULL );
      uint32_t x = (uint32_t)( v >> sh );
      if( o==2 ) x &= 0xffu;   /* 64 + 8 bits */
      hq[ (unsigned long)( 12 + 3*q + o )*cap + j ] = x;
    }
  }
}

/* one point: returns its flags */
extern "C" unsigned
fd_ed25519_hip_private_hsdec( unsigned char const enc[ 32 ], int avx_rule, int32_t pt[ 20 ] ) {
  unsigned char f;
  fd_ed25519_hip_private_hsdec_n( &enc, 1UL, avx_rule, pt, &f );
  return f;
}
