/* ref_harness.c -- TEST INFRASTRUCTURE ONLY.

   Thin driver around the reference's own fd_ed25519 objects, compiled
   from /root/reference/src by oracle/Makefile into oracle/_ref/.  It
   exposes SoA bulk entry points (multi-threaded with pthreads) so that the
   tests can generate golden fixtures and bench.py can time the reference
   CPU path (cpu_baseline kind "reference") on the GPU box's host cores.

   Entry points wrap:
     fd_ed25519_verify                  src/ballet/ed25519/fd_ed25519.h:96-101
     fd_ed25519_verify_batch_single_msg src/ballet/ed25519/fd_ed25519.h:124-130
     fd_ed25519_sign / public_from_private src/ballet/ed25519/fd_ed25519.h:41-73
     fd_txn_parse                       src/ballet/txn/fd_txn.h, fd_txn_parse.c
     the verify tile's after_frag + fd_txn_verify, sequentially
                                        src/app/fdctl/run/tiles/fd_verify.c:85-155,
                                        src/app/fdctl/run/tiles/fd_verify.h:43-88 */

#include "ballet/ed25519/fd_ed25519.h"
#include "ballet/txn/fd_txn.h"
#include "tango/tcache/fd_tcache.h"
#include <stdlib.h>
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

/* fd_txn_parse of one payload: returns the footprint (0 = rejected) and the
   parsed fields the verify tile uses in fields[0..12]. */
ulong
fdref_txn_parse( uchar const * payload, ulong sz, ulong * fields ) {
  static __thread uchar buf[ FD_TXN_MAX_SZ ] __attribute__((aligned(16)));
  ulong r = fd_txn_parse( payload, sz, buf, NULL );
  if( !r ) return 0UL;
  fd_txn_t const * t = (fd_txn_t const *)buf;
  fields[ 0] = t->transaction_version;   fields[ 1] = t->signature_cnt;        fields[ 2] = t->signature_off;
  fields[ 3] = t->message_off;           fields[ 4] = t->readonly_signed_cnt;  fields[ 5] = t->readonly_unsigned_cnt;
  fields[ 6] = t->acct_addr_cnt;         fields[ 7] = t->acct_addr_off;        fields[ 8] = t->recent_blockhash_off;
  fields[ 9] = t->instr_cnt;             fields[10] = t->addr_table_lookup_cnt;
  fields[11] = t->addr_table_adtl_writable_cnt;                                 fields[12] = t->addr_table_adtl_cnt;
  return r;
}

/* The verify tile over n frags in order, as one tile sees them: after_frag's
   parse filter (-3), then fd_txn_verify: tcache query (-2 DEDUP), batch
   verify (-1 FAILED), tcache insert (-2 DEDUP on a duplicate, else 0). */
void
fdref_vtile_seq( ulong n, uchar const * payloads, ulong const * off, uint const * sz, ulong depth, ulong map_cnt,
                 schar * verdict, ulong * tag_out ) {
  ulong * ring = (ulong *)calloc( depth, sizeof(ulong) );
  ulong * map  = (ulong *)calloc( map_cnt, sizeof(ulong) );
  ulong oldest = 0UL;
  static __thread uchar buf[ FD_TXN_MAX_SZ ] __attribute__((aligned(16)));
  tsha();
  for( ulong i=0UL; i<n; i++ ) {
    uchar const * p = payloads + off[i];
    tag_out[i] = 0UL;
    if( !fd_txn_parse( p, sz[i], buf, NULL ) ) { verdict[i] = -3; continue; }
    fd_txn_t const * t = (fd_txn_t const *)buf;
    uchar const * signatures = p + t->signature_off;
    ulong tag = *(ulong const *)signatures;
    tag_out[i] = tag;
    int dup; ulong map_idx;
    FD_TCACHE_QUERY( dup, map_idx, map, map_cnt, tag );
    (void)map_idx;
    if( dup ) { verdict[i] = -2; continue; }
    int res = fd_ed25519_verify_batch_single_msg( p + t->message_off, (ulong)sz[i] - t->message_off, signatures,
                                                  p + t->acct_addr_off, tl_shas, t->signature_cnt );
    if( res!=FD_ED25519_SUCCESS ) { verdict[i] = -1; continue; }
    FD_TCACHE_INSERT( dup, oldest, ring, depth, map, map_cnt, tag );
    verdict[i] = dup ? (schar)-2 : (schar)0;
  }
  free( ring ); free( map );
}

/* fd_txn_parse's output itself: the fd_txn_t bytes (FD_TXN_MAX_SZ buffer,
   zeroed first); returns the footprint, 0 = rejected. */
ulong
fdref_txn_parse_raw( uchar const * payload, ulong sz, uchar * out ) {
  fd_memset( out, 0, FD_TXN_MAX_SZ );
  return fd_txn_parse( payload, sz, out, NULL );
}

/* after_frag's trailer (src/app/fdctl/run/tiles/fd_verify.c:102-133),
   restated step by step on a zeroed FD_TPU_DCACHE_MTU buffer: the payload
   as during_frag copied it, fd_txn_t at the payload size aligned up to 2,
   then the payload size as a ushort.  Returns new_sz, 0 if the parse
   filter drops the frag. */
#define REF_TPU_DCACHE_MTU (1232UL + FD_TXN_MAX_SZ + 2UL)
ulong
fdref_after_frag( uchar const * payload, ulong payload_sz, uchar * out ) {
  fd_memset( out, 0, REF_TPU_DCACHE_MTU );
  fd_memcpy( out, payload, payload_sz );
  ulong txnt_off = fd_ulong_align_up( payload_sz, 2UL );
  fd_txn_t * txn_t = (fd_txn_t *)( out + txnt_off );
  ulong txn_t_sz = fd_txn_parse( out, payload_sz, txn_t, NULL );
  if( !txn_t_sz ) return 0UL;
  ushort * payload_sz_p = (ushort *)( (ulong)txn_t + txn_t_sz );
  *payload_sz_p = (ushort)payload_sz;
  return ( (ulong)payload_sz_p + sizeof(ushort) ) - (ulong)out;
}

/* fdref_vtile_seq plus the frag each SUCCESS transaction publishes:
   frags[i*REF_TPU_DCACHE_MTU ..] and frag_sz[i] (0 when filtered). */
void
fdref_vtile_seq_frags( ulong n, uchar const * payloads, ulong const * off, uint const * sz, ulong depth, ulong map_cnt,
                       schar * verdict, ulong * tag_out, uchar * frags, ulong * frag_sz ) {
  fdref_vtile_seq( n, payloads, off, sz, depth, map_cnt, verdict, tag_out );
  for( ulong i=0UL; i<n; i++ ) {
    frag_sz[i] = 0UL;
    if( verdict[i]!=0 ) continue;
    frag_sz[i] = fdref_after_frag( payloads + off[i], sz[i], frags + i*REF_TPU_DCACHE_MTU );
  }
}
