/* fd_verify_hip_service -- the GPU process behind sandboxed verify tiles.

   The verify tile runs under a write/fsync-only seccomp policy
   (src/app/fdctl/run/tiles/verify.seccomppolicy) and cannot drive a GPU;
   its accelerated form (integration/fd_verify_hip.c) hands transaction
   payloads to this process over two shared-memory links per tile and
   publishes the verdict frags that come back.  One service process serves
   every verify tile of one GPU, so the device's 4 GiB of base tables exist
   once per GPU, not once per tile (fd_ed25519_hip_vservice_serve).

     fd_verify_hip_service --prefix NAME --tiles K [--gpu G] [--depth D]
                           [--slots S] [--batch B] [--gpu-parse | --zero-copy] [--codes portable|avx512]
                           [--tile-stale-ms T] [--gpu-hang-ms H] [--no-parent-watch] [--links-per-thread L]
                           [--cpus LIST] [--hw-queues N] [--split-waves 2|4|8]

   creates, for k in [0,K), the links NAME<k>_txn (tile -> service) and
   NAME<k>_vd (service -> tile), each of D lines (default 16384), prints
   "ready K" on stdout once they exist and every link pair can serve (its
   engines and the base tables built, every kernel launched once), and
   serves them until every link has ended.  A link left behind by a service that was killed is reclaimed
   (fd_ed25519_hip_shlink_create); one whose creator still runs is not.

   Lifecycle (fd_topo_run's supervision, src/disco/topo/fd_topo_run.c:
   50-100; fd_cnc's heartbeat, src/tango/cnc/fd_cnc.h:63-65,129-130):
     - a tile whose txn-link heartbeat stops for T ms (default 5000) is
       gone: its links end and its engines and device memory are freed;
       once every tile has ended the service exits and unlinks the links;
     - SIGTERM / SIGINT / SIGHUP end every link (marked STOPPED);
     - the service exits the same way when the process that started it
       dies (PR_SET_PDEATHSIG, and its parent pid watched), so a validator
       that is gone never leaves an orphan holding HBM and shm links;
     - a batch the GPU has not completed after H ms (default 30000) is a
       hung GPU and ends every link (marked FD_ED25519_HIP_ERR_TIMEOUT,
       or STOPPED for the other tiles'); the service then exits with
       status 2 at once, without freeing its engines or running the HIP
       runtime's teardown (both would wait on the hung device).

   --gpu-parse: the transactions are parsed on the GPU (the service copies
   each payload out of the link into a batch); --zero-copy: the same, and
   the payloads are DMA'd from the txn links' rooms as they lie (the links
   page-locked with the GPU, FD_ED25519_HIP_VSERVICE_ZERO_COPY): the host
   reads two bytes per transaction and copies none.

   --links-per-thread L: one service thread serves L tiles' link pairs in
   turn (default 1, a thread per tile); a pass over a pair never waits for
   the GPU, so the pairs of a thread do not hold each other up, and a
   service whose threads would mostly spin idle takes fewer cores.
   --cpus LIST (e.g. 8-15 or 8,10,12): service thread t runs on the t-th
   CPU of the list (cyclically), as fdctl pins each tile to a core.

   Exit status: 0 every tile ended its stream (EOS); 1 bad arguments, or a
   link name a live process already holds; 2 the device failed (GPU,
   launch or allocation failure, hang) -- every link marked failed; 3 the
   device was fine but not every link ended with EOS (tiles gone or broke
   the protocol, or a signal / the parent's death stopped the service).
   The links are removed on every exit path but a SIGKILL (which the next
   service's create reclaims).

   Each link pair runs slot_cnt engines with one stream each, and a HIP
   process gets GPU_MAX_HW_QUEUES hardware queues (4 by default): engines
   beyond that share queues, and a batch on a shared queue waits for the
   one ahead of it (8 slots on 4 queues: +0.13 ms p50 on the deployed path,
   none on 8).  --hw-queues N sets GPU_MAX_HW_QUEUES for the service before
   its first HIP call; without it the service takes tiles x slots (at least
   4, at most 16), or the environment's value if that is larger. */
#define _GNU_SOURCE
#include "../../../include/fd_ed25519_hip_tile.h"

#include <errno.h>
#include <pthread.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/prctl.h>
#include <time.h>
#include <unistd.h>

static volatile int g_stop;           /* read by every link thread (opts.stop) */
static volatile int g_stop_signal;

static void
on_signal( int sig ) {
  g_stop_signal = sig;
  g_stop        = 1;
}

/* the parent's death: PR_SET_PDEATHSIG delivers SIGTERM when the thread
   that started us exits; the pid watch covers a parent that died before
   the prctl and a launcher thread that is not the parent process's last */
static pid_t g_parent;

static void *
parent_watch( void * arg ) {
  (void)arg;
  struct timespec ts = { 0, 50L*1000L*1000L };
  while( !g_stop ) {
    if( getppid()!=g_parent ) { g_stop_signal = -1; g_stop = 1; break; }
    nanosleep( &ts, NULL );
  }
  return NULL;
}

/* the service's "ready" line: once every link pair can serve (engines,
   tables, kernels loaded), so a tile's first frags never wait on set-up */
static void
announce_ready( void * ctx ) {
  printf( "ready %u\n", *(unsigned const *)ctx );
  fflush( stdout );
}

static void
usage( char const * argv0 ) {
  fprintf( stderr, "usage: %s --prefix NAME --tiles K [--gpu G] [--depth D] [--slots S] [--batch B] "
                   "[--gpu-parse | --zero-copy] [--codes portable|avx512] [--tile-stale-ms T] [--gpu-hang-ms H] "
                   "[--no-parent-watch] [--links-per-thread L] [--cpus LIST] [--hw-queues N] [--split-waves W]\n", argv0 );
}

/* "a,b,c-d" -> cpus (at most max); the count, or -1 on a malformed list */
static int
parse_cpus( char const * s, int * cpus, int max ) {
  int n = 0;
  while( *s ) {
    char * e;
    long a = strtol( s, &e, 10 );
    if( e==s || a<0 || a>=CPU_SETSIZE ) return -1;
    long b = a;
    if( *e=='-' ) {
      s = e + 1;
      b = strtol( s, &e, 10 );
      if( e==s || b<a || b>=CPU_SETSIZE ) return -1;
    }
    for( long c=a; c<=b; c++ ) { if( n>=max ) return -1; cpus[ n++ ] = (int)c; }
    if( *e==',' ) e++;
    else if( *e ) return -1;
    s = e;
  }
  return n;
}

int
main( int argc, char ** argv ) {
  g_parent = getppid();
  char const *  prefix = NULL;
  unsigned      tiles  = 0U, slots = 3U, per_thread = 1U, hw_queues = 0U;
  int           cpus[ 256 ];
  int           cpu_cnt = 0;
  int           gpu    = 0, flags = 0, parent_watch_on = 1;
  unsigned long depth  = 16384UL, batch = 4096UL;
  long          stale_ms = 0L, hang_ms = 0L;
  for( int i=1; i<argc; i++ ) {
    char const * a = argv[ i ];
    char const * v = i+1<argc ? argv[ i+1 ] : NULL;
    if(      !strcmp( a, "--prefix" ) && v ) { prefix = v; i++; }
    else if( !strcmp( a, "--tiles"  ) && v ) { tiles = (unsigned)strtoul( v, NULL, 0 ); i++; }
    else if( !strcmp( a, "--gpu"    ) && v ) { gpu = (int)strtol( v, NULL, 0 ); i++; }
    else if( !strcmp( a, "--depth"  ) && v ) { depth = strtoul( v, NULL, 0 ); i++; }
    else if( !strcmp( a, "--slots"  ) && v ) { slots = (unsigned)strtoul( v, NULL, 0 ); i++; }
    else if( !strcmp( a, "--batch"  ) && v ) { batch = strtoul( v, NULL, 0 ); i++; }
    else if( !strcmp( a, "--tile-stale-ms" ) && v ) { stale_ms = strtol( v, NULL, 0 ); i++; }
    else if( !strcmp( a, "--gpu-hang-ms" ) && v ) { hang_ms = strtol( v, NULL, 0 ); i++; }
    else if( !strcmp( a, "--no-parent-watch" ) ) { parent_watch_on = 0; }
    else if( !strcmp( a, "--links-per-thread" ) && v ) { per_thread = (unsigned)strtoul( v, NULL, 0 ); i++; }
    else if( !strcmp( a, "--hw-queues" ) && v ) { hw_queues = (unsigned)strtoul( v, NULL, 0 ); i++; }
    else if( !strcmp( a, "--split-waves" ) && v ) {   /* small batches' group equation: 2, 4 or 8 waves */
      fd_ed25519_hip_pipe_set_split_waves( (int)strtol( v, NULL, 0 ) ); i++;
    }
    else if( !strcmp( a, "--cpus" ) && v ) {
      cpu_cnt = parse_cpus( v, cpus, 256 );
      if( cpu_cnt<=0 ) { fprintf( stderr, "fd_verify_hip_service: bad --cpus list %s\n", v ); return 1; }
      i++;
    }
    else if( !strcmp( a, "--gpu-parse" ) )   { flags |= FD_ED25519_HIP_VTILE_GPU_PARSE; }
    else if( !strcmp( a, "--zero-copy" ) )   { flags |= FD_ED25519_HIP_VTILE_GPU_PARSE | FD_ED25519_HIP_VSERVICE_ZERO_COPY; }
    else if( !strcmp( a, "--codes" ) && v ) {
      if(      !strcmp( v, "portable" ) ) flags |= FD_ED25519_HIP_FLAG_CODES_PORTABLE;
      else if( strcmp( v, "avx512" ) ) { usage( argv[0] ); return 1; }
      i++;
    }
    else { usage( argv[0] ); return 1; }
  }
  if( !prefix || !tiles || tiles>FD_ED25519_HIP_VSERVICE_LINK_MAX || strlen( prefix )>96 || hw_queues>32U || !slots || slots>8U ) { usage( argv[0] ); return 1; }
  /* read by the HIP runtime when it starts, at the service's first HIP call (below) */
  {
    unsigned long q = hw_queues;
    if( !q ) {   /* a queue per slot, within [4,16], or more if the environment names more */
      q = (unsigned long)tiles*(unsigned long)slots;
      q = q<4UL ? 4UL : q>16UL ? 16UL : q;
      char const * e = getenv( "GPU_MAX_HW_QUEUES" );
      unsigned long qe = e ? strtoul( e, NULL, 10 ) : 0UL;
      if( qe>q && qe<=32UL ) q = qe;
    }
    char qs[ 16 ];
    snprintf( qs, sizeof(qs), "%lu", q );
    setenv( "GPU_MAX_HW_QUEUES", qs, 1 );
    /* kernel arguments in host memory (unless the environment says
       otherwise): a batch's five launches then take the link thread ~7 us
       instead of ~15 us (device-memory kernargs need a write over the link
       and a flush per launch), and the GPU fetches the few hundred bytes
       itself (profiles/r6_c5_launch_bump.txt) */
    setenv( "HIP_FORCE_DEV_KERNARG", "0", 0 );
  }
  if( fd_ed25519_hip_abi_check( FD_ED25519_HIP_ABI_VERSION, sizeof(fd_ed25519_hip_slot_t), sizeof(fd_ed25519_hip_info_t),
                                sizeof(fd_ed25519_hip_vservice_stats_t) ) ) {
    fprintf( stderr, "fd_verify_hip_service: %s\n", fd_ed25519_hip_last_error() );
    return 1;
  }

  struct sigaction sa;
  memset( &sa, 0, sizeof(sa) );
  sa.sa_handler = on_signal;
  sigemptyset( &sa.sa_mask );
  sigaction( SIGTERM, &sa, NULL );
  sigaction( SIGINT,  &sa, NULL );
  sigaction( SIGHUP,  &sa, NULL );
  signal( SIGPIPE, SIG_IGN );   /* a launcher that died with our stdout: still end cleanly */
  pthread_t watcher;
  int watching = 0;
  if( parent_watch_on ) {
    prctl( PR_SET_PDEATHSIG, SIGTERM );
    if( getppid()!=g_parent ) { fprintf( stderr, "fd_verify_hip_service: the parent exited at start-up\n" ); return 3; }
    watching = !pthread_create( &watcher, NULL, parent_watch, NULL );
  }

  fd_ed25519_hip_shlink_t * in [ FD_ED25519_HIP_VSERVICE_LINK_MAX ];
  fd_ed25519_hip_shlink_t * out[ FD_ED25519_HIP_VSERVICE_LINK_MAX ];
  memset( in, 0, sizeof(in) ); memset( out, 0, sizeof(out) );
  int rc = 0;
  for( unsigned k=0U; k<tiles; k++ ) {
    char name[ 128 ];
    snprintf( name, sizeof(name), "%s%u_txn", prefix, k );
    in[ k ] = fd_ed25519_hip_shlink_create( name, depth );
    int e = errno;
    snprintf( name, sizeof(name), "%s%u_vd", prefix, k );
    if( in[ k ] ) { out[ k ] = fd_ed25519_hip_shlink_create( name, depth ); e = errno; }
    if( !in[ k ] || !out[ k ] ) {
      fprintf( stderr, "fd_verify_hip_service: cannot create the links of tile %u (%s*): %s\n", k, prefix,
               e==EEXIST ? "a running process holds them" : strerror( e ) );
      rc = 1;
      break;
    }
  }
  if( !rc ) {
    char const * q = getenv( "GPU_MAX_HW_QUEUES" );
    unsigned long queues = q && *q ? strtoul( q, NULL, 0 ) : 4UL;
    if( (unsigned long)tiles*slots>queues )
      fprintf( stderr, "fd_verify_hip_service: note: %u tiles x %u slots = %u engine streams on %lu hardware queues "
                       "(GPU_MAX_HW_QUEUES, at most 32): streams share queues\n", tiles, slots, tiles*slots, queues );
    fd_ed25519_hip_vservice_stats_t st[ FD_ED25519_HIP_VSERVICE_LINK_MAX ];
    memset( st, 0, sizeof(st) );
    fd_ed25519_hip_vservice_opts_t opts;
    memset( &opts, 0, sizeof(opts) );
    opts.stop          = &g_stop;
    opts.tile_stale_ns = stale_ms>0L ? stale_ms*1000000L : stale_ms<0L ? -1L : 0L;
    opts.gpu_hang_ns   = hang_ms>0L ? hang_ms*1000000L : 0L;
    opts.ready         = announce_ready;
    opts.ready_ctx     = &tiles;
    opts.links_per_thread = per_thread;
    opts.link_cpus        = cpu_cnt ? cpus : NULL;
    opts.link_cpu_cnt     = (unsigned)cpu_cnt;
    int err = fd_ed25519_hip_vservice_serve( gpu, slots, batch, flags, in, out, tiles, st, &opts );
    /* one JSON line for tools and tests: per-tile device memory, how each
       link ended, and the base tables this one process holds for all */
    unsigned long shared = 0UL;
    for( unsigned k=0U; k<tiles; k++ ) if( st[ k ].shared_device_bytes>shared ) shared = st[ k ].shared_device_bytes;
    printf( "{\"tiles\": %u, \"shared_device_bytes\": %lu, \"tile_device_bytes\": [", tiles, shared );
    for( unsigned k=0U; k<tiles; k++ ) printf( "%s%lu", k ? ", " : "", st[ k ].device_bytes );
    printf( "], \"txns\": [" );
    for( unsigned k=0U; k<tiles; k++ ) printf( "%s%lu", k ? ", " : "", st[ k ].txn_cnt );
    printf( "], \"end_codes\": [" );
    for( unsigned k=0U; k<tiles; k++ ) printf( "%s%d", k ? ", " : "", st[ k ].end_code );
    unsigned leaked = 0U;
    for( unsigned k=0U; k<tiles; k++ ) leaked |= st[ k ].leaked_on_hang;
    printf( "], \"signal\": %d, \"rc\": %d, \"gpu_hang\": %s}\n", g_stop_signal, err, leaked ? "true" : "false" );
    fflush( stdout );
    if( leaked ) {
      /* a hung GPU: the link pairs left their engines as they were (freeing
         them would wait on the device), and so would the HIP runtime's own
         teardown at exit.  Remove the links' names, say why, and leave
         without running any exit handler: the kernel reclaims the process's
         device memory and queues. */
      fprintf( stderr, "fd_verify_hip_service: FAILED: %s (%d): %s; every link is marked failed, exiting without "
                       "device teardown\n", fd_ed25519_hip_strerror( err ), err, fd_ed25519_hip_last_error() );
      for( unsigned k=0U; k<tiles; k++ ) {
        char name[ 128 ];
        snprintf( name, sizeof(name), "%s%u_txn", prefix, k ); shm_unlink( name );
        snprintf( name, sizeof(name), "%s%u_vd",  prefix, k ); shm_unlink( name );
      }
      _exit( 2 );
    }
    int device = err && err!=FD_ED25519_HIP_SHLINK_FAIL_PROTOCOL && err!=FD_ED25519_HIP_SHLINK_FAIL_STOPPED &&
                 err!=FD_ED25519_HIP_SHLINK_FAIL_TILE_GONE;
    if( device ) {
      fprintf( stderr, "fd_verify_hip_service: FAILED: %s (%d): %s; every link is marked failed\n",
               fd_ed25519_hip_strerror( err ), err, fd_ed25519_hip_last_error() );
      rc = 2;
    } else {
      for( unsigned k=0U; k<tiles; k++ )
        fprintf( stderr, "fd_verify_hip_service: tile %u: %lu txns in %lu batches, %.3f s, %lu device bytes, %s (%d)\n", k,
                 st[ k ].txn_cnt, st[ k ].batches, st[ k ].seconds, st[ k ].device_bytes,
                 !st[ k ].end_code ? "ended" : st[ k ].end_code==FD_ED25519_HIP_SHLINK_FAIL_TILE_GONE ? "tile gone" :
                 st[ k ].end_code==FD_ED25519_HIP_SHLINK_FAIL_STOPPED ? "stopped" : "tile broke the protocol",
                 st[ k ].end_code );
      rc = err ? 3 : 0;
    }
  }
  g_stop = 1;
  if( watching ) pthread_join( watcher, NULL );
  for( unsigned k=0U; k<tiles; k++ ) {
    fd_ed25519_hip_shlink_leave( in [ k ], 1 );
    fd_ed25519_hip_shlink_leave( out[ k ], 1 );
  }
  return rc;
}
