/* fd_ed25519_oracle.c -- CPU restatement of Firedancer's ed25519 verify path.

   TEST INFRASTRUCTURE ONLY.  This file is the parity oracle for the MI355X
   engine (firedancer_amd).  Only tests/, __graft_entry__.smoke() and
   bench.py's cpu_baseline leg may load it, and only as the checker.  The
   product path never links, loads or falls back to it.

   It restates, in plain C with its own radix-2^51 field arithmetic (the GPU
   engine uses radix 2^25.5, so the two implementations share no code), the
   reference algorithm of tigarcia/firedancer @ 2025-01-17:

     fd_ed25519_verify                  src/ballet/ed25519/fd_ed25519_user.c:134-229
     fd_ed25519_verify_batch_single_msg src/ballet/ed25519/fd_ed25519_user.c:231-309
     fd_ed25519_strerror                src/ballet/ed25519/fd_ed25519_user.c:311-321
     fd_ed25519_public_from_private     src/ballet/ed25519/fd_ed25519_user.c:4-60
     fd_ed25519_sign                    src/ballet/ed25519/fd_ed25519_user.c:62-132

   Error codes have two flavours: the reference's
   AVX-512 backend maps any point-decode failure to ERR_SIG and also rejects
   x==0 with sign bit 1 (src/ballet/ed25519/avx512/fd_r43x6_ge.c:139-140,
   241-251); the portable backend maps a public-key decode failure to
   ERR_PUBKEY (src/ballet/ed25519/ref/fd_curve25519.c:209-224 via
   fd_ed25519_user.c:190-192).  `codes` selects: 0 = AVX-512 (production),
   1 = portable.  Accept/reject verdicts are identical in both.

   Parity is pinned by tests/test_oracle_golden.py against the reference's
   own vectors (wycheproof, cctv, malleability, sign KAT) and against
   outputs of the reference compiled from its sources (oracle/_ref). */

#include <stdint.h>
#include <string.h>
#include <pthread.h>
#include <stdlib.h>

#define ORACLE_SUCCESS     ( 0)
#define ORACLE_ERR_SIG     (-1)
#define ORACLE_ERR_PUBKEY  (-2)
#define ORACLE_ERR_MSG     (-3)

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------------
   SHA-512 (FIPS 180-4).  Follows fd_sha512_core_ref
   src/ballet/sha512/fd_sha512.c:128-231 and init/append/fini :265-390. */

static const uint64_t sha512_k[80] = {
  0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
  0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
  0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
  0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
  0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
  0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
  0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
  0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
  0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
  0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
  0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
  0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
  0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
  0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
  0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
  0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
  0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
  0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
  0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
  0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL,
};

static const uint64_t sha512_iv[8] = {
  0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
  0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL,
};

typedef struct {
  uint64_t h[8];
  uint8_t  buf[128];
  uint64_t buf_used;
  uint64_t bit_cnt;   /* message length in bits (messages here are < 2^61 B) */
} oracle_sha512_t;

static inline uint64_t ror64( uint64_t x, int n ) { return (x>>n) | (x<<(64-n)); }

static void
sha512_block( uint64_t h[8], uint8_t const blk[128] ) {
  uint64_t w[80];
  for( int i=0; i<16; i++ ) {
    uint64_t x = 0;
    for( int b=0; b<8; b++ ) x = (x<<8) | blk[8*i+b];   /* big endian */
    w[i] = x;
  }
  for( int i=16; i<80; i++ ) {
    uint64_t s0 = ror64( w[i-15], 1 ) ^ ror64( w[i-15], 8 ) ^ (w[i-15]>>7);
    uint64_t s1 = ror64( w[i-2], 19 ) ^ ror64( w[i-2], 61 ) ^ (w[i-2]>>6);
    w[i] = w[i-16] + s0 + w[i-7] + s1;
  }
  uint64_t a=h[0], b=h[1], c=h[2], d=h[3], e=h[4], f=h[5], g=h[6], hh=h[7];
  for( int i=0; i<80; i++ ) {
    uint64_t S1 = ror64( e, 14 ) ^ ror64( e, 18 ) ^ ror64( e, 41 );
    uint64_t ch = (e & f) ^ (~e & g);
    uint64_t t1 = hh + S1 + ch + sha512_k[i] + w[i];
    uint64_t S0 = ror64( a, 28 ) ^ ror64( a, 34 ) ^ ror64( a, 39 );
    uint64_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint64_t t2 = S0 + mj;
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0]+=a; h[1]+=b; h[2]+=c; h[3]+=d; h[4]+=e; h[5]+=f; h[6]+=g; h[7]+=hh;
}

static void
sha512_init( oracle_sha512_t * s ) {
  memcpy( s->h, sha512_iv, sizeof(sha512_iv) );
  s->buf_used = 0UL;
  s->bit_cnt  = 0UL;
}

static void
sha512_append( oracle_sha512_t * s, void const * data, uint64_t sz ) {
  uint8_t const * p = (uint8_t const *)data;
  s->bit_cnt += sz<<3;
  while( sz ) {
    uint64_t take = 128UL - s->buf_used;
    if( take>sz ) take = sz;
    memcpy( s->buf + s->buf_used, p, take );
    s->buf_used += take; p += take; sz -= take;
    if( s->buf_used==128UL ) { sha512_block( s->h, s->buf ); s->buf_used = 0UL; }
  }
}

static void
sha512_fini( oracle_sha512_t * s, uint8_t out[64] ) {
  uint64_t bits = s->bit_cnt;
  uint8_t pad = 0x80;
  sha512_append( s, &pad, 1 );
  uint8_t zero = 0;
  while( s->buf_used!=112UL ) sha512_append( s, &zero, 1 );
  uint8_t len[16] = {0};
  for( int i=0; i<8; i++ ) len[15-i] = (uint8_t)(bits>>(8*i));   /* 128-bit BE length, high 64 bits zero */
  sha512_append( s, len, 16 );
  for( int i=0; i<8; i++ ) for( int b=0; b<8; b++ ) out[8*i+b] = (uint8_t)(s->h[i]>>(56-8*b));
}

void
oracle_sha512( uint8_t out[64], void const * data, uint64_t sz ) {
  oracle_sha512_t s[1];
  sha512_init( s ); sha512_append( s, data, sz ); sha512_fini( s, out );
}

/* ------------------------------------------------------------------------
   Scalars mod L = 2^252 + 27742317777372353535851937790883648493.
   Restates fd_curve25519_scalar_validate (fd_curve25519_scalar.h:57-73),
   fd_curve25519_scalar_reduce (fd_curve25519_scalar.c:3-110) and
   fd_curve25519_scalar_muladd.  The reduction here is a plain
   shift-and-subtract long division (slow, obviously correct); any exact
   reduction yields the same residue. */

static const uint64_t L_limb[4] = {
  0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0x0000000000000000ULL, 0x1000000000000000ULL
};

static inline uint64_t ld64( uint8_t const * p ) { uint64_t x; memcpy( &x, p, 8 ); return x; }
static inline void     st64( uint8_t * p, uint64_t x ) { memcpy( p, &x, 8 ); }

/* returns 1 if S < L (canonical), 0 otherwise */
int
oracle_scalar_validate( uint8_t const s[32] ) {
  for( int i=3; i>=0; i-- ) {
    uint64_t si = ld64( s+8*i );
    if( si<L_limb[i] ) return 1;
    if( si>L_limb[i] ) return 0;
  }
  return 0; /* equal to L */
}

/* r (4 limbs, r<L) = x (nlimb limbs, little endian) mod L */
static void
scalar_mod_l( uint64_t r[4], uint64_t const * x, int nlimb ) {
  uint64_t acc[5] = {0,0,0,0,0};   /* acc < 2L < 2^254 always fits 4 limbs; 5th as slack */
  for( int i=nlimb*64-1; i>=0; i-- ) {
    uint64_t bit = (x[i>>6]>>(i&63)) & 1UL;
    /* acc = 2*acc + bit */
    for( int j=4; j>0; j-- ) acc[j] = (acc[j]<<1) | (acc[j-1]>>63);
    acc[0] = (acc[0]<<1) | bit;
    /* if acc >= L: acc -= L */
    int ge = acc[4]!=0;
    if( !ge ) {
      ge = 1;
      for( int j=3; j>=0; j-- ) {
        if( acc[j]>L_limb[j] ) { ge = 1; break; }
        if( acc[j]<L_limb[j] ) { ge = 0; break; }
      }
    }
    if( ge ) {
      u128 borrow = 0;
      for( int j=0; j<4; j++ ) {
        u128 d = (u128)acc[j] - L_limb[j] - borrow;
        acc[j] = (uint64_t)d;
        borrow = (d>>64) ? 1 : 0;
      }
      acc[4] -= (uint64_t)borrow;
    }
  }
  for( int j=0; j<4; j++ ) r[j] = acc[j];
}

void
oracle_scalar_reduce( uint8_t out[32], uint8_t const in[64] ) {
  uint64_t x[8], r[4];
  for( int i=0; i<8; i++ ) x[i] = ld64( in+8*i );
  scalar_mod_l( r, x, 8 );
  for( int i=0; i<4; i++ ) st64( out+8*i, r[i] );
}

/* out = (a*b + c) mod L */
static void
scalar_muladd( uint8_t out[32], uint8_t const a[32], uint8_t const b[32], uint8_t const c[32] ) {
  uint64_t A[4], B[4], C[4], P[9] = {0};
  for( int i=0; i<4; i++ ) { A[i] = ld64( a+8*i ); B[i] = ld64( b+8*i ); C[i] = ld64( c+8*i ); }
  for( int i=0; i<4; i++ ) {
    u128 carry = 0;
    for( int j=0; j<4; j++ ) {
      u128 t = (u128)A[i]*B[j] + P[i+j] + carry;
      P[i+j] = (uint64_t)t; carry = t>>64;
    }
    P[i+4] += (uint64_t)carry;
  }
  u128 carry = 0;
  for( int i=0; i<9; i++ ) {
    u128 t = (u128)P[i] + (i<4 ? C[i] : 0) + carry;
    P[i] = (uint64_t)t; carry = t>>64;
  }
  uint64_t r[4];
  scalar_mod_l( r, P, 9 );
  for( int i=0; i<4; i++ ) st64( out+8*i, r[i] );
}

/* ------------------------------------------------------------------------
   GF(p), p = 2^255-19, 5 limbs of 51 bits (u64).  Restates the field API of
   src/ballet/ed25519/fd_f25519.h:46-253 with the ref backend semantics of
   src/ballet/ed25519/ref/fd_f25519.h:34-324 (frombytes ignores bit 255 and
   does NOT reject values >= p; comparisons are on canonical encodings). */

typedef struct { uint64_t v[5]; } fe;
#define M51 ((1ULL<<51)-1ULL)

static void fe_0( fe * h ) { memset( h, 0, sizeof(fe) ); }
static void fe_1( fe * h ) { fe_0( h ); h->v[0] = 1; }

static void
fe_frombytes( fe * h, uint8_t const s[32] ) {
  uint64_t w0 = ld64( s ), w1 = ld64( s+8 ), w2 = ld64( s+16 ), w3 = ld64( s+24 ) & 0x7fffffffffffffffULL;
  h->v[0] =  w0                  & M51;
  h->v[1] = ((w0>>51)|(w1<<13))  & M51;
  h->v[2] = ((w1>>38)|(w2<<26))  & M51;
  h->v[3] = ((w2>>25)|(w3<<39))  & M51;
  h->v[4] =  (w3>>12);
}

static void
fe_carry( fe * h ) {
  uint64_t c;
  c = h->v[0]>>51; h->v[0] &= M51; h->v[1] += c;
  c = h->v[1]>>51; h->v[1] &= M51; h->v[2] += c;
  c = h->v[2]>>51; h->v[2] &= M51; h->v[3] += c;
  c = h->v[3]>>51; h->v[3] &= M51; h->v[4] += c;
  c = h->v[4]>>51; h->v[4] &= M51; h->v[0] += 19*c;
  c = h->v[0]>>51; h->v[0] &= M51; h->v[1] += c;
}

static void
fe_tobytes( uint8_t s[32], fe const * f ) {
  fe h = *f;
  fe_carry( &h ); fe_carry( &h );
  /* h < 2^255 + small < 2p: subtract p once if h >= p */
  uint64_t q = (h.v[0] + 19) >> 51;
  q = (h.v[1] + q) >> 51;
  q = (h.v[2] + q) >> 51;
  q = (h.v[3] + q) >> 51;
  q = (h.v[4] + q) >> 51;
  h.v[0] += 19*q;
  uint64_t c;
  c = h.v[0]>>51; h.v[0] &= M51; h.v[1] += c;
  c = h.v[1]>>51; h.v[1] &= M51; h.v[2] += c;
  c = h.v[2]>>51; h.v[2] &= M51; h.v[3] += c;
  c = h.v[3]>>51; h.v[3] &= M51; h.v[4] += c;
  h.v[4] &= M51;
  st64( s,    h.v[0]      | (h.v[1]<<51) );
  st64( s+8,  (h.v[1]>>13)| (h.v[2]<<38) );
  st64( s+16, (h.v[2]>>26)| (h.v[3]<<25) );
  st64( s+24, (h.v[3]>>39)| (h.v[4]<<12) );
}

static void fe_add( fe * h, fe const * f, fe const * g ) {
  for( int i=0; i<5; i++ ) h->v[i] = f->v[i] + g->v[i];
  fe_carry( h );
}

static void fe_sub( fe * h, fe const * f, fe const * g ) {
  /* f + 4p - g; inputs carried (limbs < 2^52) */
  h->v[0] = f->v[0] + 0x1FFFFFFFFFFFB4ULL - g->v[0];
  for( int i=1; i<5; i++ ) h->v[i] = f->v[i] + 0x1FFFFFFFFFFFFCULL - g->v[i];
  fe_carry( h );
}

static void fe_neg( fe * h, fe const * f ) { fe z; fe_0( &z ); fe_sub( h, &z, f ); }

static void
fe_mul( fe * h, fe const * f, fe const * g ) {
  uint64_t f0=f->v[0], f1=f->v[1], f2=f->v[2], f3=f->v[3], f4=f->v[4];
  uint64_t g0=g->v[0], g1=g->v[1], g2=g->v[2], g3=g->v[3], g4=g->v[4];
  uint64_t g1_19 = 19*g1, g2_19 = 19*g2, g3_19 = 19*g3, g4_19 = 19*g4;
  u128 r0 = (u128)f0*g0 + (u128)f1*g4_19 + (u128)f2*g3_19 + (u128)f3*g2_19 + (u128)f4*g1_19;
  u128 r1 = (u128)f0*g1 + (u128)f1*g0    + (u128)f2*g4_19 + (u128)f3*g3_19 + (u128)f4*g2_19;
  u128 r2 = (u128)f0*g2 + (u128)f1*g1    + (u128)f2*g0    + (u128)f3*g4_19 + (u128)f4*g3_19;
  u128 r3 = (u128)f0*g3 + (u128)f1*g2    + (u128)f2*g1    + (u128)f3*g0    + (u128)f4*g4_19;
  u128 r4 = (u128)f0*g4 + (u128)f1*g3    + (u128)f2*g2    + (u128)f3*g1    + (u128)f4*g0;
  uint64_t c;
  c = (uint64_t)(r0>>51); r1 += c; uint64_t h0 = (uint64_t)r0 & M51;
  c = (uint64_t)(r1>>51); r2 += c; uint64_t h1 = (uint64_t)r1 & M51;
  c = (uint64_t)(r2>>51); r3 += c; uint64_t h2 = (uint64_t)r2 & M51;
  c = (uint64_t)(r3>>51); r4 += c; uint64_t h3 = (uint64_t)r3 & M51;
  c = (uint64_t)(r4>>51);          uint64_t h4 = (uint64_t)r4 & M51;
  h0 += 19*c;
  c = h0>>51; h0 &= M51; h1 += c;
  h->v[0]=h0; h->v[1]=h1; h->v[2]=h2; h->v[3]=h3; h->v[4]=h4;
}

static void fe_sq( fe * h, fe const * f ) { fe_mul( h, f, f ); }

static int fe_eq( fe const * a, fe const * b ) {
  uint8_t x[32], y[32]; fe_tobytes( x, a ); fe_tobytes( y, b );
  return !memcmp( x, y, 32 );
}
static int fe_is_zero( fe const * a ) { fe z; fe_0( &z ); return fe_eq( a, &z ); }
static int fe_sgn( fe const * a ) { uint8_t x[32]; fe_tobytes( x, a ); return x[0] & 1; }

static fe fe_d, fe_d2, fe_sqrtm1, fe_y0, fe_y1;

/* a^(2^252-3): fd_f25519_pow22523, src/ballet/ed25519/fd_f25519.c:11-59 */
static void
fe_pow22523( fe * r, fe const * a ) {
  fe t0, t1, t2; int i;
  fe_sq( &t0, a );
  fe_sq( &t1, &t0 ); fe_sq( &t1, &t1 );
  fe_mul( &t1, a, &t1 );
  fe_mul( &t0, &t0, &t1 );
  fe_sq( &t0, &t0 );
  fe_mul( &t0, &t1, &t0 );
  fe_sq( &t1, &t0 ); for( i=1; i<5;   i++ ) fe_sq( &t1, &t1 );
  fe_mul( &t0, &t1, &t0 );
  fe_sq( &t1, &t0 ); for( i=1; i<10;  i++ ) fe_sq( &t1, &t1 );
  fe_mul( &t1, &t1, &t0 );
  fe_sq( &t2, &t1 ); for( i=1; i<20;  i++ ) fe_sq( &t2, &t2 );
  fe_mul( &t1, &t2, &t1 );
  fe_sq( &t1, &t1 ); for( i=1; i<10;  i++ ) fe_sq( &t1, &t1 );
  fe_mul( &t0, &t1, &t0 );
  fe_sq( &t1, &t0 ); for( i=1; i<50;  i++ ) fe_sq( &t1, &t1 );
  fe_mul( &t1, &t1, &t0 );
  fe_sq( &t2, &t1 ); for( i=1; i<100; i++ ) fe_sq( &t2, &t2 );
  fe_mul( &t1, &t2, &t1 );
  fe_sq( &t1, &t1 ); for( i=1; i<50;  i++ ) fe_sq( &t1, &t1 );
  fe_mul( &t0, &t1, &t0 );
  fe_sq( &t0, &t0 ); fe_sq( &t0, &t0 );
  fe_mul( r, &t0, a );
}

/* 1/a = a^(p-2): fd_f25519_inv, src/ballet/ed25519/fd_f25519.c:62-104 */
static void
fe_inv( fe * r, fe const * a ) {
  /* a^(p-2) = a^(2^255-21) = (a^(2^252-3))^8 * a^3 */
  fe t, a2, a3;
  fe_pow22523( &t, a );
  fe_sq( &t, &t ); fe_sq( &t, &t ); fe_sq( &t, &t );
  fe_sq( &a2, a ); fe_mul( &a3, &a2, a );
  fe_mul( r, &t, &a3 );
}

/* ------------------------------------------------------------------------
   Points: extended twisted Edwards (X:Y:Z:T), x=X/Z, y=Y/Z, xy=T/Z.
   Restates the group API of src/ballet/ed25519/fd_curve25519.h and
   src/ballet/ed25519/ref/fd_curve25519.{h,c} with the complete a=-1
   formulas (add-2008-hwcd-3 / dbl-2008-hwcd). */

typedef struct { fe X, Y, Z, T; } ge;

static void ge_zero( ge * r ) { fe_0( &r->X ); fe_1( &r->Y ); fe_1( &r->Z ); fe_0( &r->T ); }

static void
ge_add( ge * r, ge const * p, ge const * q ) {
  fe a, b, c, d, e, f, g, h, t;
  fe_sub( &a, &p->Y, &p->X ); fe_sub( &t, &q->Y, &q->X ); fe_mul( &a, &a, &t );
  fe_add( &b, &p->Y, &p->X ); fe_add( &t, &q->Y, &q->X ); fe_mul( &b, &b, &t );
  fe_mul( &c, &p->T, &q->T ); fe_mul( &c, &c, &fe_d2 );
  fe_mul( &d, &p->Z, &q->Z ); fe_add( &d, &d, &d );
  fe_sub( &e, &b, &a );
  fe_sub( &f, &d, &c );
  fe_add( &g, &d, &c );
  fe_add( &h, &b, &a );
  fe_mul( &r->X, &e, &f );
  fe_mul( &r->Y, &g, &h );
  fe_mul( &r->T, &e, &h );
  fe_mul( &r->Z, &f, &g );
}

static void
ge_dbl( ge * r, ge const * p ) {
  fe a, b, c, e, f, g, h, t;
  fe_sq( &a, &p->X );
  fe_sq( &b, &p->Y );
  fe_sq( &c, &p->Z ); fe_add( &c, &c, &c );
  fe_add( &t, &p->X, &p->Y ); fe_sq( &t, &t );
  fe_add( &h, &a, &b );              /* h = A+B           */
  fe_sub( &e, &h, &t );              /* e = A+B-(X+Y)^2 = -E_hwcd */
  fe_sub( &g, &a, &b );              /* g = A-B = -G_hwcd  */
  fe_add( &f, &c, &g );              /* f = C+A-B = -F_hwcd */
  /* hwcd with a=-1: E=(X+Y)^2-A-B, G=B-A, F=G-C, H=-A-B.
     Here e=-E, g=-G, f=-F, h=-H; products of two negated terms are equal. */
  fe_mul( &r->X, &e, &f );
  fe_mul( &r->Y, &g, &h );
  fe_mul( &r->T, &e, &h );
  fe_mul( &r->Z, &f, &g );
}

static void
ge_neg( ge * r, ge const * p ) {
  fe_neg( &r->X, &p->X ); r->Y = p->Y; r->Z = p->Z; fe_neg( &r->T, &p->T );
}

/* fd_ed25519_point_eq_z1, src/ballet/ed25519/ref/fd_curve25519.h:132-139 */
static int
ge_eq_z1( ge const * a, ge const * b ) {
  fe x1, y1;
  fe_mul( &x1, &b->X, &a->Z );
  fe_mul( &y1, &b->Y, &a->Z );
  return fe_eq( &x1, &a->X ) & fe_eq( &y1, &a->Y );
}

/* fd_ed25519_affine_is_small_order, src/ballet/ed25519/fd_curve25519.h:81-111 */
static int
ge_affine_is_small_order( ge const * a ) {
  return fe_is_zero( &a->X ) | fe_is_zero( &a->Y ) | fe_eq( &a->Y, &fe_y0 ) | fe_eq( &a->Y, &fe_y1 );
}

/* Point decode.  Follows fd_ed25519_point_frombytes,
   src/ballet/ed25519/fd_curve25519.c:25-62 (sqrt via fd_f25519_sqrt_ratio,
   src/ballet/ed25519/fd_f25519.c:107-143).  With codes==0 (AVX-512
   backend) it additionally fails on x==0 with sign bit set, as
   fd_r43x6_ge_decode does (src/ballet/ed25519/avx512/fd_r43x6_ge.c:139-140,
   226-228).  Returns 0 on success, -1 on failure. */
static int
ge_frombytes( ge * r, uint8_t const buf[32], int codes ) {
  fe y, u, v, v3, vxx, check, x;
  fe_frombytes( &y, buf );
  int sign = buf[31]>>7;
  fe one; fe_1( &one );
  fe_sq( &u, &y );
  fe_mul( &v, &u, &fe_d );
  fe_sub( &u, &u, &one );            /* u = y^2-1  */
  fe_add( &v, &v, &one );            /* v = dy^2+1 */
  /* x = u v^3 (u v^7)^((p-5)/8) */
  fe_sq( &v3, &v ); fe_mul( &v3, &v3, &v );              /* v^3 */
  fe_sq( &x, &v3 ); fe_mul( &x, &x, &v ); fe_mul( &x, &x, &u ); /* u v^7 */
  fe_pow22523( &x, &x );
  fe_mul( &x, &x, &v3 ); fe_mul( &x, &x, &u );
  fe_sq( &vxx, &x ); fe_mul( &vxx, &vxx, &v );
  fe_sub( &check, &vxx, &u );
  if( !fe_is_zero( &check ) ) {
    fe_add( &check, &vxx, &u );
    if( !fe_is_zero( &check ) ) return -1;
    fe_mul( &x, &x, &fe_sqrtm1 );
  }
  if( codes==0 && fe_is_zero( &x ) && sign ) return -1;
  if( fe_sgn( &x )!=sign ) fe_neg( &x, &x );
  r->X = x; r->Y = y; fe_1( &r->Z ); fe_mul( &r->T, &x, &y );
  return 0;
}

static void
ge_tobytes( uint8_t out[32], ge const * p ) {
  fe zi, x, y;
  fe_inv( &zi, &p->Z );
  fe_mul( &x, &p->X, &zi );
  fe_mul( &y, &p->Y, &zi );
  fe_tobytes( out, &y );
  out[31] ^= (uint8_t)(fe_sgn( &x )<<7);
}

/* wNAF recoding.  Follows fd_curve25519_scalar_wnaf,
   src/ballet/ed25519/fd_curve25519_scalar.c:277-360: odd digits in
   [-(2^w-1), 2^w-1], bit 255 of the input ignored. */
static void
scalar_wnaf( int16_t t[256], uint8_t const s[32], int w ) {
  int16_t max = (int16_t)((1<<w)-1);
  for( int i=0; i<255; i++ ) t[i] = (int16_t)((s[i>>3]>>(i&7)) & 1);
  t[255] = 0;
  int i = 0;
  while( i<256 && !t[i] ) i++;
  while( i<256 ) {
    int16_t ti = 1;
    int j;
    for( j=i+1; j<256; j++ ) {
      if( !t[j] ) continue;
      int sh = j-i; if( sh>14 ) sh = 14;
      int16_t delta = (int16_t)(1<<sh);
      if( delta>2*max ) break;
      if( ti+delta<=max ) { ti = (int16_t)(ti+delta); t[j] = 0; continue; }
      if( ti-delta>=-max ) {
        ti = (int16_t)(ti-delta); t[j] = 0;
        for(;;) { j++; if( !t[j] ) { t[j] = 1; break; } t[j] = 0; }
        break;
      }
      break;
    }
    t[i] = ti;
    i = j;
  }
}

static ge  ge_base;
static ge  ge_base_odd[128];   /* [1,3,5,...,255] B, cf. fd_ed25519_base_point_wnaf_table */
static pthread_once_t oracle_once = PTHREAD_ONCE_INIT;

/* fd_ed25519_double_scalar_mul_base, src/ballet/ed25519/fd_curve25519.c:122-166:
   r = [n1] A + [n2] B with w=4 wNAF for n1 and w=8 wNAF for n2. */
static void
ge_double_scalar_mul_base( ge * r, uint8_t const n1[32], ge const * a, uint8_t const n2[32] ) {
  int16_t s1[256], s2[256];
  scalar_wnaf( s1, n1, 4 );
  scalar_wnaf( s2, n2, 8 );
  ge ai[8], a2, t;
  ai[0] = *a;
  ge_dbl( &a2, a );
  for( int i=1; i<8; i++ ) ge_add( &ai[i], &a2, &ai[i-1] );
  ge_zero( r );
  int i;
  for( i=255; i>=0; i-- ) if( s1[i] || s2[i] ) break;
  for( ; i>=0; i-- ) {
    ge_dbl( r, r );
    if( s1[i]>0 ) ge_add( r, r, &ai[ s1[i]/2] );
    else if( s1[i]<0 ) { ge_neg( &t, &ai[(-s1[i])/2] ); ge_add( r, r, &t ); }
    if( s2[i]>0 ) ge_add( r, r, &ge_base_odd[ s2[i]/2] );
    else if( s2[i]<0 ) { ge_neg( &t, &ge_base_odd[(-s2[i])/2] ); ge_add( r, r, &t ); }
  }
}

static void
fe_from_hex_le( fe * h, char const * hex ) {
  uint8_t b[32];
  for( int i=0; i<32; i++ ) {
    unsigned v; char tmp[3] = { hex[2*i], hex[2*i+1], 0 };
    v = (unsigned)strtoul( tmp, NULL, 16 );
    b[i] = (uint8_t)v;
  }
  fe_frombytes( h, b );
}

static void
oracle_init( void ) {
  /* d = -121665/121666, 2d, sqrt(-1), order-8 y's (fd_f25519_table_ref.c;
     fd_curve25519_table_ref.c:18-27), base point (compressed 0x58666...) */
  fe_from_hex_le( &fe_d,      "a3785913ca4deb75abd841414d0a700098e879777940c78c73fe6f2bee6c0352" );
  fe_from_hex_le( &fe_d2,     "59f1b226949bd6eb56b183829a14e00030d1f3eef2808e19e7fcdf56dcd90624" );
  fe_from_hex_le( &fe_sqrtm1, "b0a00e4a271beec478e42fad0618432fa7d7fb3d99004d2b0bdfc14f8024832b" );
  fe_from_hex_le( &fe_y0,     "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05" );
  fe_from_hex_le( &fe_y1,     "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a" );
  uint8_t bb[32]; bb[0] = 0x58; for( int i=1; i<32; i++ ) bb[i] = 0x66;
  ge_frombytes( &ge_base, bb, 1 );
  ge b2; ge_dbl( &b2, &ge_base );
  ge_base_odd[0] = ge_base;
  for( int i=1; i<128; i++ ) ge_add( &ge_base_odd[i], &ge_base_odd[i-1], &b2 );
}

static void ensure_init( void ) { pthread_once( &oracle_once, oracle_init ); }

/* [s] B by the same machinery (n1 = 0) */
static void
ge_scalarmult_base( ge * r, uint8_t const s[32] ) {
  uint8_t zero[32] = {0};
  ge dummy; ge_zero( &dummy );
  ge_double_scalar_mul_base( r, zero, &dummy, s );
}

/* ------------------------------------------------------------------------
   Public API (restating fd_ed25519_user.c) */

/* encoding of [s]B, s < L (test infrastructure: anchors the GPU's base
   tables, tests/test_gpu_parity.py) */
void
oracle_base_mul_encode( uint8_t out[32], uint8_t const s[32] ) {
  ensure_init();
  ge r;
  ge_scalarmult_base( &r, s );
  ge_tobytes( out, &r );
}

int
oracle_ed25519_verify( uint8_t const * msg, uint64_t msg_sz, uint8_t const sig[64],
                       uint8_t const pub[32], int codes ) {
  ensure_init();
  uint8_t const * r = sig;
  uint8_t const * S = sig+32;
  if( !oracle_scalar_validate( S ) ) return ORACLE_ERR_SIG;
  ge A, R;
  if( ge_frombytes( &A, pub, codes ) ) return codes==0 ? ORACLE_ERR_SIG : ORACLE_ERR_PUBKEY;
  if( ge_frombytes( &R, r,   codes ) ) return ORACLE_ERR_SIG;
  if( ge_affine_is_small_order( &A ) ) return ORACLE_ERR_PUBKEY;
  if( ge_affine_is_small_order( &R ) ) return ORACLE_ERR_SIG;
  oracle_sha512_t sh[1];
  uint8_t h[64], k[32];
  sha512_init( sh );
  sha512_append( sh, r, 32 ); sha512_append( sh, pub, 32 ); sha512_append( sh, msg, msg_sz );
  sha512_fini( sh, h );
  oracle_scalar_reduce( k, h );
  ge nA, Rc;
  ge_neg( &nA, &A );
  ge_double_scalar_mul_base( &Rc, k, &nA, S );
  return ge_eq_z1( &Rc, &R ) ? ORACLE_SUCCESS : ORACLE_ERR_MSG;
}

int
oracle_ed25519_verify_batch_single_msg( uint8_t const * msg, uint64_t msg_sz,
                                        uint8_t const * sigs, uint8_t const * pubs,
                                        uint32_t batch_sz, int codes ) {
  ensure_init();
  if( batch_sz==0 || batch_sz>16 ) return ORACLE_ERR_SIG;
  ge A[16], R[16];
  uint8_t k[16][32];
  for( uint32_t j=0; j<batch_sz; j++ ) {
    uint8_t const * r   = sigs + 64*j;
    uint8_t const * S   = sigs + 64*j + 32;
    uint8_t const * pub = pubs + 32*j;
    if( !oracle_scalar_validate( S ) ) return ORACLE_ERR_SIG;
    if( ge_frombytes( &A[j], pub, codes ) ) return codes==0 ? ORACLE_ERR_SIG : ORACLE_ERR_PUBKEY;
    if( ge_frombytes( &R[j], r,   codes ) ) return ORACLE_ERR_SIG;
    if( ge_affine_is_small_order( &A[j] ) ) return ORACLE_ERR_PUBKEY;
    if( ge_affine_is_small_order( &R[j] ) ) return ORACLE_ERR_SIG;
    oracle_sha512_t sh[1];
    uint8_t h[64];
    sha512_init( sh );
    sha512_append( sh, r, 32 ); sha512_append( sh, pub, 32 ); sha512_append( sh, msg, msg_sz );
    sha512_fini( sh, h );
    oracle_scalar_reduce( k[j], h );
  }
  for( uint32_t j=0; j<batch_sz; j++ ) {
    ge nA, Rc;
    ge_neg( &nA, &A[j] );
    ge_double_scalar_mul_base( &Rc, k[j], &nA, sigs + 64*j + 32 );
    if( !ge_eq_z1( &Rc, &R[j] ) ) return ORACLE_ERR_MSG;
  }
  return ORACLE_SUCCESS;
}

char const *
oracle_ed25519_strerror( int err ) {
  switch( err ) {
  case ORACLE_SUCCESS:    return "success";
  case ORACLE_ERR_SIG:    return "bad signature";
  case ORACLE_ERR_PUBKEY: return "bad public key";
  case ORACLE_ERR_MSG:    return "bad message";
  default: break;
  }
  return "unknown";
}

void
oracle_ed25519_public_from_private( uint8_t pub[32], uint8_t const priv[32] ) {
  ensure_init();
  uint8_t h[64];
  oracle_sha512( h, priv, 32 );
  h[0] &= 0xF8; h[31] &= 0x7F; h[31] |= 0x40;
  ge A; ge_scalarmult_base( &A, h );
  ge_tobytes( pub, &A );
}

void
oracle_ed25519_sign( uint8_t sig[64], uint8_t const * msg, uint64_t msg_sz,
                     uint8_t const pub[32], uint8_t const priv[32] ) {
  ensure_init();
  uint8_t h[64], r[32], rr[64], k[64], kk[32];
  oracle_sha512( h, priv, 32 );
  h[0] &= 0xF8; h[31] &= 0x7F; h[31] |= 0x40;
  oracle_sha512_t sh[1];
  sha512_init( sh ); sha512_append( sh, h+32, 32 ); sha512_append( sh, msg, msg_sz ); sha512_fini( sh, rr );
  oracle_scalar_reduce( r, rr );
  ge R; ge_scalarmult_base( &R, r );
  ge_tobytes( sig, &R );
  sha512_init( sh ); sha512_append( sh, sig, 32 ); sha512_append( sh, pub, 32 ); sha512_append( sh, msg, msg_sz ); sha512_fini( sh, k );
  oracle_scalar_reduce( kk, k );
  scalar_muladd( sig+32, kk, h, r );
}

/* Bulk helpers (SoA, one verify per element), multi-threaded. */

typedef struct {
  uint64_t n, i0, i1;
  uint8_t const * msgs; uint64_t const * off; uint32_t const * sz;
  uint8_t const * sigs; uint8_t const * pubs; int8_t * out; int codes;
} oracle_job_t;

static void *
oracle_verify_worker( void * arg ) {
  oracle_job_t * j = (oracle_job_t *)arg;
  for( uint64_t i=j->i0; i<j->i1; i++ )
    j->out[i] = (int8_t)oracle_ed25519_verify( j->msgs + j->off[i], j->sz[i], j->sigs + 64*i, j->pubs + 32*i, j->codes );
  return NULL;
}

int
oracle_verify_many( uint64_t n, uint8_t const * msgs, uint64_t const * off, uint32_t const * sz,
                    uint8_t const * sigs, uint8_t const * pubs, int8_t * out, int codes, int nthreads ) {
  ensure_init();
  if( nthreads<1 ) nthreads = 1;
  if( nthreads>256 ) nthreads = 256;
  pthread_t th[256]; oracle_job_t jobs[256];
  for( int t=0; t<nthreads; t++ ) {
    jobs[t] = (oracle_job_t){ n, n*(uint64_t)t/(uint64_t)nthreads, n*(uint64_t)(t+1)/(uint64_t)nthreads,
                              msgs, off, sz, sigs, pubs, out, codes };
    if( pthread_create( &th[t], NULL, oracle_verify_worker, &jobs[t] ) ) return -1;
  }
  for( int t=0; t<nthreads; t++ ) pthread_join( th[t], NULL );
  return 0;
}
