/* fd_ed25519_hip_sha512.c -- SHA-512 on the host, for the one case the
   device path cannot take: the drop-in verify of a message whose size does
   not fit the device path's 32-bit message sizes (4 GiB and more; the
   reference takes any ulong size, src/ballet/ed25519/fd_ed25519.h:96-101).
   The caller's thread hashes R || A || M (fd_ed25519_user.c:199-205's
   challenge) and the device takes the digest from there
   (fd_ed25519_hip_verify_digests_dev): reduction mod L, decompression and
   the group equation stay on the GPU.

   FIPS 180-4 SHA-512, the same function as src/ballet/sha512/fd_sha512.c's
   core (fd_sha512_core_ref) -- written here from the standard, plain C,
   one 128-byte block at a time.  tests/test_abi.py checks it against
   hashlib. */
#include "../../../include/fd_ed25519_hip.h"

#include <stdint.h>
#include <string.h>

static uint64_t const K512[ 80 ] = {
  0x428a2f98d728ae22UL, 0x7137449123ef65cdUL, 0xb5c0fbcfec4d3b2fUL, 0xe9b5dba58189dbbcUL, 0x3956c25bf348b538UL,
  0x59f111f1b605d019UL, 0x923f82a4af194f9bUL, 0xab1c5ed5da6d8118UL, 0xd807aa98a3030242UL, 0x12835b0145706fbeUL,
  0x243185be4ee4b28cUL, 0x550c7dc3d5ffb4e2UL, 0x72be5d74f27b896fUL, 0x80deb1fe3b1696b1UL, 0x9bdc06a725c71235UL,
  0xc19bf174cf692694UL, 0xe49b69c19ef14ad2UL, 0xefbe4786384f25e3UL, 0x0fc19dc68b8cd5b5UL, 0x240ca1cc77ac9c65UL,
  0x2de92c6f592b0275UL, 0x4a7484aa6ea6e483UL, 0x5cb0a9dcbd41fbd4UL, 0x76f988da831153b5UL, 0x983e5152ee66dfabUL,
  0xa831c66d2db43210UL, 0xb00327c898fb213fUL, 0xbf597fc7beef0ee4UL, 0xc6e00bf33da88fc2UL, 0xd5a79147930aa725UL,
  0x06ca6351e003826fUL, 0x142929670a0e6e70UL, 0x27b70a8546d22ffcUL, 0x2e1b21385c26c926UL, 0x4d2c6dfc5ac42aedUL,
  0x53380d139d95b3dfUL, 0x650a73548baf63deUL, 0x766a0abb3c77b2a8UL, 0x81c2c92e47edaee6UL, 0x92722c851482353bUL,
  0xa2bfe8a14cf10364UL, 0xa81a664bbc423001UL, 0xc24b8b70d0f89791UL, 0xc76c51a30654be30UL, 0xd192e819d6ef5218UL,
  0xd69906245565a910UL, 0xf40e35855771202aUL, 0x106aa07032bbd1b8UL, 0x19a4c116b8d2d0c8UL, 0x1e376c085141ab53UL,
  0x2748774cdf8eeb99UL, 0x34b0bcb5e19b48a8UL, 0x391c0cb3c5c95a63UL, 0x4ed8aa4ae3418acbUL, 0x5b9cca4f7763e373UL,
  0x682e6ff3d6b2b8a3UL, 0x748f82ee5defb2fcUL, 0x78a5636f43172f60UL, 0x84c87814a1f0ab72UL, 0x8cc702081a6439ecUL,
  0x90befffa23631e28UL, 0xa4506cebde82bde9UL, 0xbef9a3f7b2c67915UL, 0xc67178f2e372532bUL, 0xca273eceea26619cUL,
  0xd186b8c721c0c207UL, 0xeada7dd6cde0eb1eUL, 0xf57d4f7fee6ed178UL, 0x06f067aa72176fbaUL, 0x0a637dc5a2c898a6UL,
  0x113f9804bef90daeUL, 0x1b710b35131c471bUL, 0x28db77f523047d84UL, 0x32caab7b40c72493UL, 0x3c9ebe0a15c9bebcUL,
  0x431d67c49c100d4cUL, 0x4cc5d4becb3e42b6UL, 0x597f299cfc657e2aUL, 0x5fcb6fab3ad6faecUL, 0x6c44198c4a475817UL };

#define ROR( x, n ) ( ((x)>>(n)) | ((x)<<(64-(n))) )

static inline uint64_t
load_be64( unsigned char const * p ) {
  uint64_t x;
  memcpy( &x, p, 8UL );
  return __builtin_bswap64( x );
}

static void
sha512_blocks( uint64_t h[ 8 ], unsigned char const * p, unsigned long blk_cnt ) {
  for( unsigned long b=0UL; b<blk_cnt; b++, p+=128 ) {
    uint64_t w[ 80 ];
    for( int t=0; t<16; t++ ) w[ t ] = load_be64( p + 8*t );
    for( int t=16; t<80; t++ ) {
      uint64_t s0 = ROR( w[t-15], 1 ) ^ ROR( w[t-15], 8 ) ^ ( w[t-15]>>7 );
      uint64_t s1 = ROR( w[t-2], 19 ) ^ ROR( w[t-2], 61 ) ^ ( w[t-2]>>6 );
      w[ t ] = w[t-16] + s0 + w[t-7] + s1;
    }
    uint64_t a = h[0], bb = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for( int t=0; t<80; t++ ) {
      uint64_t t1 = hh + ( ROR( e, 14 ) ^ ROR( e, 18 ) ^ ROR( e, 41 ) ) + ( (e & f) ^ (~e & g) ) + K512[ t ] + w[ t ];
      uint64_t t2 = ( ROR( a, 28 ) ^ ROR( a, 34 ) ^ ROR( a, 39 ) ) + ( (a & bb) ^ (a & c) ^ (bb & c) );
      hh = g; g = f; f = e; e = d + t1; d = c; c = bb; bb = a; a = t1 + t2;
    }
    h[0] += a; h[1] += bb; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
}

typedef struct {
  uint64_t      h[ 8 ];
  unsigned char buf[ 128 ];
  unsigned long buf_used;
  unsigned long total;      /* bytes; messages here stay far below 2^64 bits / 8 */
} host_sha512_t;

static void
sha512_init( host_sha512_t * s ) {
  static uint64_t const iv[ 8 ] = { 0x6a09e667f3bcc908UL, 0xbb67ae8584caa73bUL, 0x3c6ef372fe94f82bUL,
                                    0xa54ff53a5f1d36f1UL, 0x510e527fade682d1UL, 0x9b05688c2b3e6c1fUL,
                                    0x1f83d9abfb41bd6bUL, 0x5be0cd19137e2179UL };
  memcpy( s->h, iv, sizeof(iv) );
  s->buf_used = 0UL;
  s->total    = 0UL;
}

static void
sha512_append( host_sha512_t * s, unsigned char const * p, unsigned long sz ) {
  s->total += sz;
  if( s->buf_used ) {
    unsigned long take = 128UL - s->buf_used;
    if( take>sz ) take = sz;
    memcpy( s->buf + s->buf_used, p, take );
    s->buf_used += take; p += take; sz -= take;
    if( s->buf_used<128UL ) return;
    sha512_blocks( s->h, s->buf, 1UL );
    s->buf_used = 0UL;
  }
  unsigned long blk = sz>>7;
  if( blk ) { sha512_blocks( s->h, p, blk ); p += blk<<7; sz -= blk<<7; }
  if( sz ) { memcpy( s->buf, p, sz ); s->buf_used = sz; }
}

static void
sha512_fini( host_sha512_t * s, unsigned char out[ 64 ] ) {
  unsigned char pad[ 256 ];
  unsigned long used = s->buf_used;
  memcpy( pad, s->buf, used );
  pad[ used++ ] = 0x80;
  unsigned long len = used<=112UL ? 128UL : 256UL;
  memset( pad + used, 0, len - used );
  uint64_t bits_hi = s->total>>61, bits_lo = s->total<<3;
  for( int i=0; i<8; i++ ) {
    pad[ len - 16 + i ] = (unsigned char)( bits_hi>>(56-8*i) );
    pad[ len -  8 + i ] = (unsigned char)( bits_lo>>(56-8*i) );
  }
  sha512_blocks( s->h, pad, len>>7 );
  for( int i=0; i<8; i++ ) {
    uint64_t be = __builtin_bswap64( s->h[ i ] );
    memcpy( out + 8*i, &be, 8UL );
  }
}

void
fd_ed25519_hip_sha512( void const * data, unsigned long sz, unsigned char out[ 64 ] ) {
  host_sha512_t s;
  sha512_init( &s );
  sha512_append( &s, (unsigned char const *)data, sz );
  sha512_fini( &s, out );
}

/* the verify challenge's digest, SHA-512( R || A || M ) */
void
fd_ed25519_hip_private_challenge( unsigned char const sig[ 64 ], unsigned char const pub[ 32 ],
                                  unsigned char const * msg, unsigned long msg_sz, unsigned char out[ 64 ] ) {
  host_sha512_t s;
  sha512_init( &s );
  sha512_append( &s, sig, 32UL );
  sha512_append( &s, pub, 32UL );
  if( msg_sz ) sha512_append( &s, msg, msg_sz );
  sha512_fini( &s, out );
}
