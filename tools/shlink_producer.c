/* shlink_producer -- the verify tile's side of the sandboxed integration,
   standalone: maps two shared-memory links (txn frags out, verdict frags
   in), then enters seccomp strict mode (only read, write, _exit and
   sigreturn remain -- stricter than the verify tile's write/fsync policy,
   src/app/fdctl/run/tiles/verify.seccomppolicy) and runs the whole stream
   with memory operations only.  Any other system call would kill it.

     shlink_producer IN_LINK OUT_LINK PAYLOAD_FILE [--no-sandbox] [--stale-ms MS] [--profile]

   PAYLOAD_FILE: u64 n, n x u32 sizes, the payloads back to back.  Frag i
   carries sig = i; after the last one an EOS frag.  Verdict frags are
   consumed whenever a publish finds no credit, and after the EOS until
   the service's EOS (and, as the tile's after_credit does, every 16
   frags).  Output on stdout, via write(2): n verdict bytes in
   frag order (checked against the sig of every verdict frag), then for
   each SUCCESS verdict the frag the verify tile publishes, assembled as the
   tile does from its own payload and the trailer the service returned
   (fd_ed25519_hip_frag_assemble: u32 size, then the bytes); exit status 0, or
   2 on a protocol error, 3 if strict mode is unavailable, 4 if the service
   stopped: its heartbeat on OUT_LINK unchanged for MS milliseconds
   (default 1000; 60 s before its first tick) or a link marked failed
   (fd_cnc's heartbeat check, src/tango/cnc/fd_cnc.h:63-65,129-130).  Strict
   mode leaves no clock -- not even the time-stamp counter, which the kernel
   disables for it -- so time is counted in pause instructions, their rate
   measured before the sandbox (the waits only run longer than that, so the
   bound is a lower bound on the time waited).  --profile (implies
   --no-sandbox: strict mode disables the time-stamp counter) prints the
   cycles per transaction spent publishing, taking verdicts (with the frag
   assembly) and waiting, to stderr at the end. */
#define _GNU_SOURCE
#include "../include/fd_ed25519_hip_tile.h"

#include <linux/seccomp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/prctl.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>
#include <x86intrin.h>

static void
leave( int status ) {   /* exit(2) itself: exit_group is not allowed in strict mode */
  syscall( SYS_exit, status );
  for(;;) {}
}

/* the service's liveness, checked while waiting on it */
typedef struct {
  fd_ed25519_hip_shlink_t * txl;
  fd_ed25519_hip_shlink_t * vdl;
  unsigned long hb_last;
  unsigned long since;       /* pauses since hb_last changed */
  unsigned long stale, boot; /* bounds in pauses */
  unsigned long spin;
} watch_t;

static void
say( char const * msg ) {
  long k = write( 2, msg, strlen( msg ) );
  (void)k;
}

static void
watch( watch_t * w ) {
  _mm_pause();
  w->since++;
  if( (++w->spin & 255UL) ) return;
  if( fd_ed25519_hip_shlink_status( w->vdl ) || fd_ed25519_hip_shlink_status( w->txl ) ) {
    say( "shlink_producer: the verify service marked a link failed\n" );
    leave( 4 );
  }
  unsigned long hb = fd_ed25519_hip_shlink_heartbeat_query( w->vdl );
  if( hb!=w->hb_last ) { w->hb_last = hb; w->since = 0UL; return; }
  if( w->since > (hb ? w->stale : w->boot) ) {
    say( "shlink_producer: the verify service's heartbeat is stale\n" );
    leave( 4 );
  }
}

static double
now_ns( void ) {
  struct timespec ts; clock_gettime( CLOCK_MONOTONIC, &ts );
  return 1e9*(double)ts.tv_sec + (double)ts.tv_nsec;
}

typedef struct {
  unsigned char * mem;   /* preallocated: no allocation after seccomp */
  unsigned long   cap, used;
} frags_t;

typedef struct {
  unsigned char const * pay;
  unsigned long const * off;
  unsigned int const *  sz;
} stream_t;

static int
take_verdicts( fd_ed25519_hip_shlink_t * in, unsigned char * buf, signed char * verdict, unsigned long n,
               unsigned long * next, int * eos, frags_t * fr, stream_t const * st ) {
  for(;;) {
    unsigned long sz = 0UL, sig = 0UL;
    unsigned int ctl = 0U;
    int r = fd_ed25519_hip_shlink_consume( in, buf, &sz, &sig, &ctl );
    if( r==1 ) return 0;
    if( r ) return -1;
    if( ctl & FD_ED25519_HIP_SHLINK_CTL_EOS ) { *eos = 1; return 0; }
    if( sz<1UL || sig!=*next || *next>=n ) return -1;
    signed char v = (signed char)buf[ 0 ];
    if( (v==FD_ED25519_HIP_TXN_VERIFY_SUCCESS) != (sz>1UL) ) return -1;   /* a frag with every SUCCESS, only then */
    if( sz>1UL ) {
      /* assembled at a cache-line boundary, as the tile assembles into its
         out dcache's 64-byte chunks (packed for stdout after the stream) */
      unsigned long k = *next;
      if( fr->used + 64UL + FD_ED25519_HIP_TPU_DCACHE_MTU > fr->cap ) return -1;
      unsigned int fsz = (unsigned int)fd_ed25519_hip_frag_assemble( fr->mem + fr->used + 64UL, st->pay + st->off[ k ],
                                                                     st->sz[ k ], buf + 1, sz - 1UL );
      if( !fsz ) return -1;
      memcpy( fr->mem + fr->used, &fsz, 4UL );
      fr->used += 64UL + ( ( fsz + 63UL ) & ~63UL );
    }
    verdict[ (*next)++ ] = v;
  }
}

int
main( int argc, char ** argv ) {
  if( argc<4 ) { fprintf( stderr, "usage: %s IN_LINK OUT_LINK PAYLOAD_FILE [--no-sandbox] [--stale-ms MS]\n", argv[0] ); return 1; }
  int sandbox = 1, profile = 0;
  double stale_ms = 1000.0;
  for( int a=4; a<argc; a++ ) {
    if(      !strcmp( argv[a], "--no-sandbox" ) ) sandbox = 0;
    else if( !strcmp( argv[a], "--profile" ) ) { profile = 1; sandbox = 0; }
    else if( !strcmp( argv[a], "--stale-ms" ) && a+1<argc ) stale_ms = strtod( argv[++a], NULL );
    else { fprintf( stderr, "bad argument %s\n", argv[a] ); return 1; }
  }
  FILE * f = fopen( argv[3], "rb" );
  if( !f ) { perror( "payload file" ); return 1; }
  unsigned long n = 0UL;
  if( fread( &n, 8, 1, f )!=1 ) return 1;
  unsigned int * sz = (unsigned int *)malloc( 4UL*(n+1UL) );
  unsigned long * off = (unsigned long *)malloc( 8UL*(n+1UL) );
  if( !sz || !off || fread( sz, 4, n, f )!=n ) return 1;
  unsigned long total = 0UL;
  for( unsigned long i=0UL; i<n; i++ ) { off[ i ] = total; total += sz[ i ]; }
  unsigned char * pay = (unsigned char *)malloc( total + 1UL );
  if( !pay || fread( pay, 1, total, f )!=total ) return 1;
  fclose( f );
  signed char * verdict = (signed char *)malloc( n + 1UL );
  unsigned char * buf = (unsigned char *)malloc( FD_ED25519_HIP_SHLINK_MTU );
  frags_t fr;
  fr.cap = total + n*(FD_ED25519_HIP_TXN_MAX_SZ + 8UL + 128UL) + FD_ED25519_HIP_TPU_DCACHE_MTU + 64UL;   /* every payload + pad,
                                                      trailer, size line, alignment; one frag's room */
  fr.used = 0UL;
  fr.mem = (unsigned char *)aligned_alloc( 64UL, ( fr.cap + 63UL ) & ~63UL );
  if( !fr.mem ) return 1;
  /* touched before the stream: page faults of the output buffers would
     otherwise land inside it (a tile publishes into its out dcache, which
     is mapped and warm) */
  memset( fr.mem, 0, fr.cap );
  fd_ed25519_hip_shlink_t * txl = fd_ed25519_hip_shlink_join( argv[1] );
  fd_ed25519_hip_shlink_t * vdl = fd_ed25519_hip_shlink_join( argv[2] );
  if( !verdict || !buf || !txl || !vdl ) { fprintf( stderr, "cannot join the links\n" ); return 1; }
  memset( verdict, 0x7f, n + 1UL );
  /* pauses per ns, measured before the sandbox */
  double n0 = now_ns();
  for( unsigned long k=0UL; k<(1UL<<20); k++ ) _mm_pause();
  double pause_per_ns = (double)(1UL<<20) / (now_ns() - n0);
  watch_t wt = { txl, vdl, fd_ed25519_hip_shlink_heartbeat_query( vdl ), 0UL,
                 (unsigned long)(pause_per_ns * stale_ms * 1e6), (unsigned long)(pause_per_ns * 60e9), 0UL };
  fflush( stdout ); fflush( stderr );

  if( sandbox && prctl( PR_SET_SECCOMP, SECCOMP_MODE_STRICT ) ) { perror( "seccomp strict" ); return 3; }

  /* from here on: memory operations, write(2) and _exit(2) only */
  unsigned long i = 0UL, got = 0UL;
  int eos = 0;
  stream_t st = { pay, off, sz };
  unsigned long long pf_pub = 0ULL, pf_take = 0ULL, pf_wait = 0ULL, pf_c = profile ? __rdtsc() : 0ULL, pf_n;
#define PF( acc ) do { if( profile ) { pf_n = __rdtsc(); acc += pf_n - pf_c; pf_c = pf_n; } } while(0)
  /* unanswered frags stay below the txn link's depth, as the tile's cap
     does (integration/fd_verify_hip.c): a zero-copy service hands credits
     back when it stages a frag, and the room itself is reused only after
     the verdict, so a producer limited by credits alone could overwrite a
     payload before its batch reached the GPU */
  unsigned long depth = fd_ed25519_hip_shlink_depth( txl );
  while( i<n ) {
    if( i - got>=depth ) {
      if( take_verdicts( vdl, buf, verdict, n, &got, &eos, &fr, &st ) || eos ) leave( 2 );
      PF( pf_take );
      if( i - got>=depth ) { watch( &wt ); PF( pf_wait ); }
      continue;
    }
    int r = fd_ed25519_hip_shlink_publish( txl, pay + off[ i ], sz[ i ], i, 0U );
    PF( pf_pub );
    if( r==0 ) {
      /* as the tile's mux loop does (after_credit between frags): the
         verdicts that are back are taken every 16 frags, not only when the
         txn link runs out of credits */
      if( !(++i & 15UL) && ( take_verdicts( vdl, buf, verdict, n, &got, &eos, &fr, &st ) || eos ) ) leave( 2 );
      PF( pf_take );
      continue;
    }
    if( r!=1 ) leave( 2 );
    if( take_verdicts( vdl, buf, verdict, n, &got, &eos, &fr, &st ) || eos ) leave( 2 );
    PF( pf_take );
    watch( &wt );
    PF( pf_wait );
  }
  while( fd_ed25519_hip_shlink_publish( txl, NULL, 0UL, n, FD_ED25519_HIP_SHLINK_CTL_EOS )==1 ) {
    if( take_verdicts( vdl, buf, verdict, n, &got, &eos, &fr, &st ) || eos ) leave( 2 );
    watch( &wt );
  }
  while( !eos ) {
    if( take_verdicts( vdl, buf, verdict, n, &got, &eos, &fr, &st ) ) leave( 2 );
    watch( &wt );
  }
  if( got!=n ) leave( 2 );
  if( profile ) {
    char line[ 200 ];
    int k = snprintf( line, sizeof(line), "shlink_producer profile: cycles per txn: publish %.0f, take verdicts %.0f, "
                      "wait (no credit) %.0f\n", (double)pf_pub/(double)n, (double)pf_take/(double)n,
                      (double)pf_wait/(double)n );
    if( k>0 ) say( line );
  }
  unsigned long w = 0UL;
  while( w<n ) {
    long k = write( 1, verdict + w, n - w );
    if( k<=0 ) leave( 2 );
    w += (unsigned long)k;
  }
  /* packed in place: u32 size, then the frag */
  unsigned long packed = 0UL;
  for( unsigned long e=0UL; e<fr.used; ) {
    unsigned int fsz;
    memcpy( &fsz, fr.mem + e, 4UL );
    memmove( fr.mem + packed, fr.mem + e, 4UL );
    memmove( fr.mem + packed + 4UL, fr.mem + e + 64UL, fsz );
    packed += 4UL + fsz;
    e      += 64UL + ( ( fsz + 63UL ) & ~63UL );
  }
  w = 0UL;
  while( w<packed ) {
    long k = write( 1, fr.mem + w, packed - w );
    if( k<=0 ) leave( 2 );
    w += (unsigned long)k;
  }
  leave( 0 );
  return 0;
}
