/* ref_harness.c -- TEST INFRASTRUCTURE ONLY.

   Thin driver around the reference's own fd_ed25519 objects, compiled
   from /root/reference/src by oracle/Makefile into oracle/_ref/.  It
   exposes SoA bulk entry points (multi-threaded with pthreads) so that the
   tests can generate golden fixtures and bench.py can time the reference
   CPU path (cpu_baseline kind "reference") on the GPU box's host cores.

   Entry points wrap:
     fd_ed25519_verify                  src/ballet/ed25519/fd_ed25519.h:96-101
     fd_ed25519_verify_batch_single_msg src/ballet/ed25519/fd_ed25519.h:124-130
     fd_ed25519_sign / public_from_private src/ballet/ed25519/fd_ed25519.h:41-73 */

#include "ballet/ed25519/fd_ed25519.h"
#include <pthread.h>
#include <time.h>

/* One sha512 state per thread, as the verify tile owns one per call site
   (src/app/fdctl/run/tiles/fd_verify.c:169-173). */
static __thread fd_sha512_t * tl_sha;
static __thread uchar         tl_sha_mem[ 16 ][ FD_SHA512_FOOTPRINT ] __attribute__((aligned(FD_SHA512_ALIGN)));
static __thread fd_sha512_t * tl_shas[ 16 ];

static fd_sha512_t *
tsha( void ) {
  if( FD_UNLIKELY( !tl_sha ) ) {
    for( int i=0; i<16; i++ ) tl_shas[i] = fd_sha512_join( fd_sha512_new( tl_sha_mem[i] ) );
    tl_sha = tl_shas[0];
  }
  return tl_sha;
}

int
fdref_verify( uchar const * msg, ulong sz, uchar const * sig, uchar const * pub ) {
  return fd_ed25519_verify( msg, sz, sig, pub, tsha() );
}

int
fdref_verify_batch_single_msg( uchar const * msg, ulong sz, uchar const * sigs, uchar const * pubs, uint n ) {
  tsha();
  return fd_ed25519_verify_batch_single_msg( msg, sz, sigs, pubs, tl_shas, (uchar)n );
}

void
fdref_public_from_private( uchar * pub, uchar const * priv ) {
  fd_ed25519_public_from_private( pub, priv, tsha() );
}

void
fdref_sign( uchar * sig, uchar const * msg, ulong sz, uchar const * pub, uchar const * priv ) {
  fd_ed25519_sign( sig, msg, sz, pub, priv, tsha() );
}

typedef struct {
  ulong i0, i1, reps;
  uchar const * msgs; ulong const * off; uint const * sz;
  uchar const * sigs; uchar const * pubs; schar * out;
} job_t;

static void *
verify_worker( void * arg ) {
  job_t * j = (job_t *)arg;
  fd_sha512_t * sha = tsha();
  for( ulong r=0UL; r<j->reps; r++ )
    for( ulong i=j->i0; i<j->i1; i++ )
      j->out[i] = (schar)fd_ed25519_verify( j->msgs + j->off[i], j->sz[i], j->sigs + 64UL*i, j->pubs + 32UL*i, sha );
  return NULL;
}

/* Verifies n signatures (SoA) on nthreads pthreads, `reps` passes over the
   slice each.  Returns wall time in ns (so bench.py can time it without
   Python overhead), or -1 on thread creation failure. */
long
fdref_verify_many( ulong n, uchar const * msgs, ulong const * off, uint const * sz,
                   uchar const * sigs, uchar const * pubs, schar * out, int nthreads, ulong reps ) {
  if( nthreads<1 ) nthreads = 1;
  if( nthreads>512 ) nthreads = 512;
  static pthread_t th[512]; static job_t jobs[512];
  struct timespec t0, t1;
  clock_gettime( CLOCK_MONOTONIC, &t0 );
  for( int t=0; t<nthreads; t++ ) {
    jobs[t] = (job_t){ n*(ulong)t/(ulong)nthreads, n*(ulong)(t+1)/(ulong)nthreads, reps, msgs, off, sz, sigs, pubs, out };
    if( pthread_create( &th[t], NULL, verify_worker, &jobs[t] ) ) return -1L;
  }
  for( int t=0; t<nthreads; t++ ) pthread_join( th[t], NULL );
  clock_gettime( CLOCK_MONOTONIC, &t1 );
  return (t1.tv_sec - t0.tv_sec)*1000000000L + (t1.tv_nsec - t0.tv_nsec);
}
