/* mux_harness.c -- TEST INFRASTRUCTURE ONLY (oracle/Makefile ref-mux).

   Runs verify tiles -- the reference's own fd_tile_verify
   (src/app/fdctl/run/tiles/fd_verify.c:230-244, compiled from its sources,
   CPU verify) or the accelerated fd_tile_verify_hip
   (integration/fd_verify_hip.c, GPU service behind shared-memory links) --
   inside the reference's tile runtime, the way fd_topo_run_tile starts a
   tile (src/disco/topo/fd_topo_run.c:56-180):

     privileged_init -> the tile's own seccomp filter
     (populate_allowed_seccomp) installed on the tile's thread ->
     fd_metrics_register -> unprivileged_init -> fd_mux_tile (the
     reference's run loop, src/disco/mux/fd_mux.c:90-710) with the tile's
     mux_flags, burst and callbacks,

   over the topology fdctl builds for them (src/app/fdctl/topology.c: one
   quic -> verify link that every verify tile reads, each with its own
   reliable fseq, keeping the frags with seq % verify_tile_count == its
   kind id, fd_verify.c:36-47; one verify -> dedup link per verify tile,
   all read by the dedup tile).  A producer thread is the quic tile: it
   publishes the payloads of a file into the shared link with the
   reference's fd_mcache_publish (sig = seq, at an optional rate), its
   credits the minimum over every verify tile's fseq (fd_fctl's rule for
   reliable consumers).  A consumer thread is the dedup tile's side: it
   polls every verify -> dedup link in turn, reads each published frag (sig,
   sz, bytes) and returns credits through that link's fseq.

     mux_harness verify|verify_hip|filter_all|publish_only PAYLOADS OUT [--app NAME] [--depth D]
                 [--tiles K | --rr-cnt N --rr-idx I] [--no-sandbox]
                 [--rate TXN_PER_S] [--timeout S] [--lat-out FILE]
                 [--cpus LIST]

   filter_all runs the reference's fd_mux_tile with a tile that filters
   every frag in before_frag (the run loop's own per-frag cost, no verify
   behind it); publish_only runs the producer alone (its publish rate with
   no reader): together they say whether the multi-tile deployed rate is
   the run loop's or the producer's.

   --tiles K: K verify tiles (kind ids 0..K-1) each run on a thread of its
   own (default 1).  --rr-cnt N --rr-idx I: the topology has N verify tiles
   and only the one of kind id I runs (it sees every frag and keeps its
   share; the producer's credits are that tile's).  --cpus LIST (e.g.
   8-19 or 8,9,12): the producer, the consumer and tile k run on the 1st,
   2nd and (k+3)-th CPU of the list, as fdctl pins each tile to a core.

   PAYLOADS: u64 n, n x u32 sizes, the payloads.  OUT: every published frag
   in the order the consumer took it (per out link in order, the links
   interleaved as polled) as u64 sig, u32 sz, sz bytes.  stdout: one JSON
   line of counts.  The run ends when every tile has consumed every frag and
   has nothing pending (fd_verify_hip_pending for the accelerated tile), the
   consumer has drained every out link, and every tile has halted on its
   cnc; each accelerated tile's txn link then carries the end-of-stream
   frag, so the GPU service exits.  A tile that stops (FD_LOG_ERR inside the
   sandbox) ends the process; exit status 3 on the harness's own timeout.

   Latency (SURVEY.md §8(d) C5 on the deployed path): each frag's tsorig
   is its due time -- the producer's start plus seq / rate, or its publish
   time when unpaced -- so a producer held back by credits does not hide
   the wait (no coordinated omission).  Both tiles publish the frag's
   tsorig with the verified frag (fd_verify.c:152-153; the accelerated tile
   echoes it through the service), and the consumer, the dedup tile's
   side, takes now - fd_frag_meta_ts_decomp( tsorig ) for every frag it
   receives: due time -> verified frag on the out link.  The JSON line
   carries p50 / p99 / max in microseconds; --lat-out writes every sample
   (u32 nanoseconds, in the order received). */

#define _GNU_SOURCE
#include "disco/tiles.h"
#include "disco/metrics/fd_metrics.h"
#include "fd_ed25519_hip_tile.h"

#include <linux/filter.h>
#include <linux/seccomp.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/prctl.h>
#include <time.h>
#include <unistd.h>

extern fd_topo_run_tile_t fd_tile_verify;
extern fd_topo_run_tile_t fd_tile_verify_hip;
ulong fd_verify_hip_pending( void const * ctx );
fd_ed25519_hip_shlink_t * fd_verify_hip_txn_link( void * ctx );

#define OUT_BURST (16UL)
#define TILE_MAX  (16UL)

/* filter_all: the reference's fd_mux_tile loop with a tile whose
   before_frag filters every frag -- what the run loop
   alone costs per frag of the shared quic -> verify link, with no verify
   work behind it (fd_mux.c:387 calls before_frag on every frag; the
   verify tiles keep seq % verify_tile_count, fd_verify.c:36-47) */
static ulong filter_all_align( void ) { return 128UL; }
static ulong filter_all_footprint( fd_topo_tile_t const * tile ) { (void)tile; return 128UL; }
static void
filter_all_before_frag( void * ctx, ulong in_idx, ulong seq, ulong sig, int * opt_filter ) {
  (void)ctx; (void)in_idx; (void)seq; (void)sig;
  *opt_filter = 1;
}
static fd_topo_run_tile_t fd_tile_filter_all = {
  .name              = "filter",
  .mux_flags         = FD_MUX_FLAG_COPY | FD_MUX_FLAG_MANUAL_PUBLISH,
  .burst             = 1UL,
  .mux_before_frag   = filter_all_before_frag,
  .scratch_align     = filter_all_align,
  .scratch_footprint = filter_all_footprint,
};

static double
now_s( void ) {
  struct timespec ts; clock_gettime( CLOCK_MONOTONIC, &ts );
  return (double)ts.tv_sec + 1e-9*(double)ts.tv_nsec;
}

/* bump allocator over the one region that serves as the workspace: the
   tiles translate chunks relative to its base (fd_chunk_to_laddr) */
static uchar * g_mem;
static ulong   g_used, g_cap;

static void *
walloc( ulong align, ulong sz ) {
  if( align<4096UL ) align = 4096UL;
  ulong off = fd_ulong_align_up( g_used, align );
  FD_TEST( off + sz<=g_cap );
  g_used = off + sz;
  return g_mem + off;
}

static ulong
woff( void const * p ) {
  return (ulong)((uchar const *)p - g_mem);
}

typedef struct harness harness_t;

typedef struct {               /* one running verify tile */
  harness_t *          h;
  ulong                k;      /* its kind id */
  fd_topo_tile_t *     tile;
  fd_frag_meta_t *     out_mcache;  uchar * out_dcache;  ulong * out_fseq;
  ulong *              in_fseq;
  fd_cnc_t *           cnc;
  void *               scratch;
  void *               mux_scratch;
  void *               ctx;
  int                  cpu;
  volatile int         halted;
  ulong                out_seq;   /* consumer: next out seq expected on this tile's link */
} tile_run_t;

struct harness {
  /* input */
  ulong            n;
  uchar const *    pay;
  ulong const *    off;
  uint const *     sz;
  double           rate;
  /* the shared quic -> verify link */
  fd_frag_meta_t * in_mcache;   ulong in_depth;  uchar * in_dcache;
  ulong            out_depth;
  /* tiles */
  fd_topo_t *          topo;
  fd_topo_run_tile_t * run;
  tile_run_t           t[ TILE_MAX ];
  ulong                t_cnt;
  int                  sandbox;
  int                  cpu_prod, cpu_cons;
  /* consumer output */
  uchar *          res;
  ulong            res_used, res_cap;
  uint *           lat_ns;       /* per published frag: now - tsorig */
  double           tick_per_ns;
  volatile ulong   res_cnt;
  volatile int     producer_done;
  volatile int     stop;
  volatile int     consumer_err;
  ulong            credit_spins;   /* producer: pauses waiting for the tiles' fseqs (a tile is behind) */
  ulong            idle_spins;     /* consumer: passes over every out link with nothing published */
  long             last_recv_tick; /* consumer: when it took the last frag it received */
  long             prod_k0;        /* producer: its start (frag 0's due time)           */
};

static void
pin_cpu( int cpu ) {
  if( cpu<0 ) return;
  cpu_set_t set;
  CPU_ZERO( &set );
  CPU_SET( cpu, &set );
  if( pthread_setaffinity_np( pthread_self(), sizeof(set), &set ) ) FD_LOG_ERR(( "cannot run on CPU %d", cpu ));
}

/* the slowest tile's fseq: the producer's credits (fd_fctl, reliable consumers) */
static ulong
min_fseq( harness_t const * h ) {
  if( !h->t_cnt ) return h->n;   /* publish_only: no reader, no credit limit */
  ulong m = fd_fseq_query( h->t[0].in_fseq );
  for( ulong k=1UL; k<h->t_cnt; k++ ) {
    ulong q = fd_fseq_query( h->t[k].in_fseq );
    if( fd_seq_lt( q, m ) ) m = q;
  }
  return m;
}

static void *
producer_main( void * arg ) {
  harness_t * h = (harness_t *)arg;
  pin_cpu( h->cpu_prod );
  ulong chunk0 = fd_dcache_compact_chunk0( g_mem, h->in_dcache );
  ulong wmark  = fd_dcache_compact_wmark ( g_mem, h->in_dcache, FD_TPU_MTU );
  ulong chunk  = chunk0;
  double t0 = now_s();
  long   k0 = fd_tickcount();
  h->prod_k0 = k0;   /* the stream's start: frag seq is due at k0 + seq / rate */
  double tick_per_s = h->tick_per_ns*1e9;
  ulong  cr = 0UL;   /* seq up to which the tiles have room (refreshed when used up) */
  for( ulong seq=0UL; seq<h->n && !h->stop; seq++ ) {
    long due = 0L;
    if( h->rate>0.0 ) {
      while( now_s() < t0 + (double)seq/h->rate ) FD_SPIN_PAUSE();
      due = k0 + (long)( (double)seq/h->rate*tick_per_s );
    }
    /* credits: never more than depth frags ahead of the slowest tile */
    while( fd_seq_ge( seq, cr ) ) {
      cr = min_fseq( h ) + h->in_depth;
      if( fd_seq_lt( seq, cr ) ) break;
      if( h->stop ) return NULL;
      h->credit_spins++;
      FD_SPIN_PAUSE();
    }
    ulong sz = h->sz[ seq ];
    fd_memcpy( fd_chunk_to_laddr( g_mem, chunk ), h->pay + h->off[ seq ], sz );
    long  now   = fd_tickcount();
    ulong ts    = (ulong)fd_frag_meta_ts_comp( now );
    ulong tsorig = h->rate>0.0 ? (ulong)fd_frag_meta_ts_comp( due ) : ts;   /* the frag's due time */
    fd_mcache_publish( h->in_mcache, h->in_depth, seq, seq, chunk, sz, fd_frag_meta_ctl( 0UL, 1, 1, 0 ), tsorig, ts );
    chunk = fd_dcache_compact_next( chunk, sz, chunk0, wmark );
  }
  h->producer_done = 1;
  return NULL;
}

/* the dedup tile's side of the out links: every frag of each, in order */
static void *
consumer_main( void * arg ) {
  harness_t * h = (harness_t *)arg;
  pin_cpu( h->cpu_cons );
  while( !h->stop ) {
    int took = 0;
    for( ulong k=0UL; k<h->t_cnt; k++ ) {
      tile_run_t * t = &h->t[k];
      ulong seq = t->out_seq;
      fd_frag_meta_t const * m = t->out_mcache + fd_mcache_line_idx( seq, h->out_depth );
      ulong s0 = FD_VOLATILE_CONST( m->seq );
      long d = fd_seq_diff( s0, seq );
      if( d<0L ) continue;
      if( d>0L ) { h->consumer_err = 1; return NULL; }       /* overrun: the tile ignored our credits */
      FD_COMPILER_MFENCE();
      ulong sig = m->sig, chunk = m->chunk, sz = m->sz, tsorig = m->tsorig;
      FD_COMPILER_MFENCE();
      if( sz>FD_TPU_DCACHE_MTU || h->res_used + 12UL + sz>h->res_cap ) { h->consumer_err = 2; return NULL; }
      uchar * r = h->res + h->res_used;
      fd_memcpy( r, &sig, 8UL ); uint usz = (uint)sz; fd_memcpy( r+8, &usz, 4UL );
      fd_memcpy( r+12, fd_chunk_to_laddr_const( g_mem, chunk ), sz );
      FD_COMPILER_MFENCE();
      if( FD_VOLATILE_CONST( m->seq )!=s0 ) { h->consumer_err = 3; return NULL; }
      h->res_used += 12UL + sz;
      long lat = fd_tickcount() - fd_frag_meta_ts_decomp( tsorig, fd_tickcount() );
      double ns = (double)lat / h->tick_per_ns;
      h->lat_ns[ h->res_cnt ] = ns<0.0 ? 0U : ns>4e9 ? 4000000000U : (uint)ns;
      h->res_cnt++;
      h->last_recv_tick = fd_tickcount();
      seq++;
      FD_VOLATILE( t->out_seq ) = seq;
      fd_fseq_update( t->out_fseq, seq );
      took = 1;
    }
    if( !took ) { h->idle_spins++; FD_SPIN_PAUSE(); }
  }
  return NULL;
}

/* fd_topo_run_tile's sequence on this thread (src/disco/topo/fd_topo_run.c) */
static void *
tile_main( void * arg ) {
  tile_run_t * t = (tile_run_t *)arg;
  harness_t *  h = t->h;
  pin_cpu( t->cpu );   /* before the sandbox: the affinity call is not in the tile's policy */
  fd_log_cpu_set( NULL );
  fd_log_thread_set( h->run==&fd_tile_verify ? "verify:ref" : h->run==&fd_tile_filter_all ? "filter" : "verify:hip" );
  FD_LOG_NOTICE(( "booting tile %lu", t->k ));   /* as fd_topo_run_tile does: warms the logger (thread state, time zone) before the sandbox */

  if( h->sandbox && h->run->populate_allowed_seccomp ) {
    struct sock_filter filter[ 128 ];
    ulong cnt = h->run->populate_allowed_seccomp( t->scratch, 128UL, filter );
    struct sock_fprog prog = { .len = (ushort)cnt, .filter = filter };
    /* this thread only (no TSYNC): the harness's other threads stay free to
       write the result; the tile itself runs under exactly its policy */
    if( prctl( PR_SET_NO_NEW_PRIVS, 1, 0, 0, 0 ) || prctl( PR_SET_SECCOMP, SECCOMP_MODE_FILTER, &prog ) )
      FD_LOG_ERR(( "seccomp filter install failed" ));
  }

  fd_metrics_register( (ulong *)t->tile->metrics );
  if( h->run->unprivileged_init ) h->run->unprivileged_init( h->topo, t->tile, t->scratch );

  fd_mux_callbacks_t callbacks = {
    .during_housekeeping = h->run->mux_during_housekeeping,
    .before_credit       = h->run->mux_before_credit,
    .after_credit        = h->run->mux_after_credit,
    .before_frag         = h->run->mux_before_frag,
    .during_frag         = h->run->mux_during_frag,
    .after_frag          = h->run->mux_after_frag,
    .metrics_write       = h->run->mux_metrics_write,
  };
  fd_frag_meta_t const * in_mcache[1] = { h->in_mcache };
  ulong *                in_fseq[1]   = { t->in_fseq };
  ulong *                out_fseq[1]  = { t->out_fseq };
  fd_rng_t rng[1];
  int ret = fd_mux_tile( t->cnc, h->run->mux_flags, 1UL, in_mcache, in_fseq, t->out_mcache, 1UL, out_fseq,
                         h->run->burst, 0UL, 0L, fd_rng_join( fd_rng_new( rng, (uint)t->k, 0UL ) ), t->mux_scratch,
                         t->ctx, &callbacks );
  t->halted = ret ? -1 : 1;
  /* a sandboxed thread may not even exit: park until the process ends */
  for(;;) FD_SPIN_PAUSE();
  return NULL;
}

static double
calibrate_ticks( void ) {
  /* fd_tempo_tick_per_ns, measured before the sandbox (it sleeps) */
  long t0 = fd_log_wallclock(); long k0 = fd_tickcount();
  struct timespec ts = { 0, 50L*1000L*1000L }; nanosleep( &ts, NULL );
  long t1 = fd_log_wallclock(); long k1 = fd_tickcount();
  double tpn = (double)(k1-k0)/(double)(t1-t0);
  fd_tempo_set_tick_per_ns( tpn, 0.0 );
  return tpn;
}

static int
cmp_uint( void const * a, void const * b ) {
  uint x = *(uint const *)a, y = *(uint const *)b;
  return x<y ? -1 : x>y;
}

/* "a,b,c-d" -> cpus (at most max); the count, or -1 */
static int
parse_cpus( char const * s, int * cpus, int max ) {
  int n = 0;
  while( *s ) {
    char * e;
    long a = strtol( s, &e, 10 ), b = a;
    if( e==s || a<0 ) return -1;
    if( *e=='-' ) { s = e + 1; b = strtol( s, &e, 10 ); if( e==s || b<a ) return -1; }
    for( long c=a; c<=b; c++ ) { if( n>=max ) return -1; cpus[ n++ ] = (int)c; }
    if( *e==',' ) e++;
    else if( *e ) return -1;
    s = e;
  }
  return n;
}

int
main( int argc, char ** argv ) {
  fd_log_private_boot( &argc, &argv );
  if( argc<4 ) FD_LOG_ERR(( "usage: %s verify|verify_hip|filter_all|publish_only PAYLOADS OUT [--app NAME] [--depth D] [--tiles K | --rr-cnt N "
                            "--rr-idx I] [--no-sandbox] [--rate TXN_PER_S] [--timeout S] [--lat-out FILE] [--cpus LIST]",
                            argv[0] ));
  harness_t * h = (harness_t *)calloc( 1, sizeof(harness_t) );
  char const * kind = argv[1];
  int publish_only = 0;   /* the producer alone: no tile reads the link (its publish rate) */
  if(      !strcmp( kind, "verify"       ) ) h->run = &fd_tile_verify;
  else if( !strcmp( kind, "verify_hip"   ) ) h->run = &fd_tile_verify_hip;
  else if( !strcmp( kind, "filter_all"   ) ) h->run = &fd_tile_filter_all;
  else if( !strcmp( kind, "publish_only" ) ) { h->run = &fd_tile_filter_all; publish_only = 1; }
  else FD_LOG_ERR(( "unknown tile %s", kind ));
  char const * app = "harness";
  char const * lat_out = NULL;
  ulong depth = 4096UL, rr_cnt = 0UL, rr_idx = 0UL, tiles = 0UL;
  double timeout = 120.0;
  int cpus[ 64 ];
  int cpu_cnt = 0;
  h->sandbox = 1;
  for( int i=4; i<argc; i++ ) {
    char const * a = argv[i]; char const * v = i+1<argc ? argv[i+1] : NULL;
    if(      !strcmp( a, "--app"     ) && v ) { app = v; i++; }
    else if( !strcmp( a, "--depth"   ) && v ) { depth = strtoul( v, NULL, 0 ); i++; }
    else if( !strcmp( a, "--tiles"   ) && v ) { tiles = strtoul( v, NULL, 0 ); i++; }
    else if( !strcmp( a, "--rr-cnt"  ) && v ) { rr_cnt = strtoul( v, NULL, 0 ); i++; }
    else if( !strcmp( a, "--rr-idx"  ) && v ) { rr_idx = strtoul( v, NULL, 0 ); i++; }
    else if( !strcmp( a, "--rate"    ) && v ) { h->rate = strtod( v, NULL ); i++; }
    else if( !strcmp( a, "--timeout" ) && v ) { timeout = strtod( v, NULL ); i++; }
    else if( !strcmp( a, "--no-sandbox" ) ) h->sandbox = 0;
    else if( !strcmp( a, "--lat-out" ) && v ) { lat_out = v; i++; }
    else if( !strcmp( a, "--cpus" ) && v ) {
      cpu_cnt = parse_cpus( v, cpus, 64 );
      if( cpu_cnt<=0 ) FD_LOG_ERR(( "bad --cpus list %s", v ));
      i++;
    }
    else FD_LOG_ERR(( "bad argument %s", a ));
  }
  if( tiles && rr_cnt ) FD_LOG_ERR(( "--tiles and --rr-cnt exclude each other" ));
  ulong first = 0UL;               /* kind id of the first tile that runs */
  if( tiles ) { rr_cnt = tiles; h->t_cnt = tiles; }
  else if( rr_cnt ) { h->t_cnt = 1UL; first = rr_idx; }
  else { rr_cnt = 1UL; h->t_cnt = 1UL; }
  if( publish_only ) h->t_cnt = 0UL;
  FD_TEST( rr_cnt>=1UL && rr_cnt<=TILE_MAX && first<rr_cnt && fd_ulong_is_pow2( depth ) );
  h->cpu_prod = cpu_cnt>0 ? cpus[0] : -1;
  h->cpu_cons = cpu_cnt>1 ? cpus[1] : -1;

  /* payloads */
  FILE * f = fopen( argv[2], "rb" );
  if( !f ) FD_LOG_ERR(( "cannot open %s", argv[2] ));
  FD_TEST( fread( &h->n, 8UL, 1UL, f )==1UL );
  uint *  sz  = (uint  *)malloc( 4UL*(h->n+1UL) );
  ulong * off = (ulong *)malloc( 8UL*(h->n+1UL) );
  FD_TEST( fread( sz, 4UL, h->n, f )==h->n );
  ulong total = 0UL;
  for( ulong i=0UL; i<h->n; i++ ) { off[i] = total; total += sz[i]; FD_TEST( sz[i]<=FD_TPU_MTU ); }
  uchar * pay = (uchar *)malloc( total+1UL );
  FD_TEST( fread( pay, 1UL, total, f )==total );
  fclose( f );
  h->pay = pay; h->off = off; h->sz = sz;

  h->tick_per_ns = calibrate_ticks();

  /* the workspace region and the objects in it */
  ulong K = h->t_cnt;
  ulong out_depth = depth;
  ulong in_data  = fd_dcache_req_data_sz( FD_TPU_MTU,        depth,     1UL,       1 );
  ulong out_data = fd_dcache_req_data_sz( FD_TPU_DCACHE_MTU, out_depth, OUT_BURST, 1 );
  g_cap = 64UL*1024UL*1024UL + fd_dcache_footprint( in_data, 0UL ) + fd_mcache_footprint( depth, 0UL ) +
          K*( fd_dcache_footprint( out_data, 0UL ) + fd_mcache_footprint( out_depth, 0UL ) +
              h->run->scratch_footprint( NULL ) + FD_MUX_TILE_SCRATCH_FOOTPRINT( 1UL, 1UL ) + 6UL*4096UL +
              FD_METRICS_FOOTPRINT( 1UL, 1UL ) );
  FD_TEST( !posix_memalign( (void **)&g_mem, 4096UL, g_cap ) );
  fd_memset( g_mem, 0, g_cap );

  h->in_depth   = depth;
  h->out_depth  = out_depth;
  h->in_mcache  = fd_mcache_join( fd_mcache_new( walloc( fd_mcache_align(), fd_mcache_footprint( depth, 0UL ) ), depth, 0UL, 0UL ) );
  h->in_dcache  = fd_dcache_join( fd_dcache_new( walloc( fd_dcache_align(), fd_dcache_footprint( in_data, 0UL ) ), in_data, 0UL ) );
  FD_TEST( h->in_mcache && h->in_dcache );

  /* the topology the tiles' init reads: objects 0, 1 the shared in link,
     2+2k, 3+2k tile k's out link */
  fd_topo_t * topo = (fd_topo_t *)calloc( 1, sizeof(fd_topo_t) );
  h->topo = topo;
  FD_TEST( fd_cstr_printf_check( topo->app_name, sizeof(topo->app_name), NULL, "%s", app ) );
  topo->wksp_cnt = 1UL;
  topo->workspaces[0].id = 0UL;
  strcpy( topo->workspaces[0].name, "harness" );
  topo->workspaces[0].wksp = (fd_wksp_t *)g_mem;
  topo->objs[0].id = 0UL; topo->objs[0].wksp_id = 0UL; topo->objs[0].offset = woff( h->in_mcache );
  topo->objs[1].id = 1UL; topo->objs[1].wksp_id = 0UL; topo->objs[1].offset = woff( h->in_dcache );
  topo->link_cnt = 1UL;
  fd_topo_link_t * lin = &topo->links[0];
  lin->id = 0UL; strcpy( lin->name, "quic_verify" ); lin->depth = depth; lin->mtu = FD_TPU_MTU; lin->burst = 1UL;
  lin->mcache_obj_id = 0UL; lin->dcache_obj_id = 1UL; lin->mcache = h->in_mcache; lin->dcache = h->in_dcache;
  topo->tile_cnt = rr_cnt;
  topo->obj_cnt  = 2UL;
  for( ulong k=0UL; k<rr_cnt; k++ ) {
    fd_topo_tile_t * tt = &topo->tiles[k];
    tt->id = k; strcpy( tt->name, "verify" ); tt->kind_id = k;
    tt->in_cnt = 1UL; tt->in_link_id[0] = 0UL; tt->in_link_reliable[0] = 1; tt->in_link_poll[0] = 1;
  }
  for( ulong j=0UL; j<K; j++ ) {
    tile_run_t * t = &h->t[j];
    t->h = h; t->k = first + j;
    t->cpu = cpu_cnt ? cpus[ (2 + (int)j) % cpu_cnt ] : -1;
    t->out_mcache = fd_mcache_join( fd_mcache_new( walloc( fd_mcache_align(), fd_mcache_footprint( out_depth, 0UL ) ), out_depth, 0UL, 0UL ) );
    t->out_dcache = fd_dcache_join( fd_dcache_new( walloc( fd_dcache_align(), fd_dcache_footprint( out_data, 0UL ) ), out_data, 0UL ) );
    t->out_fseq   = fd_fseq_join( fd_fseq_new( walloc( fd_fseq_align(), fd_fseq_footprint() ), 0UL ) );
    t->in_fseq    = fd_fseq_join( fd_fseq_new( walloc( fd_fseq_align(), fd_fseq_footprint() ), 0UL ) );
    t->cnc        = fd_cnc_join( fd_cnc_new( walloc( fd_cnc_align(), fd_cnc_footprint( 64UL ) ), 64UL, 0UL, fd_tickcount() ) );
    ulong * metrics = fd_metrics_new( walloc( FD_METRICS_ALIGN, FD_METRICS_FOOTPRINT( 1UL, 1UL ) ), 1UL, 1UL );
    t->scratch     = walloc( h->run->scratch_align(), h->run->scratch_footprint( NULL ) );
    t->mux_scratch = walloc( FD_MUX_TILE_SCRATCH_ALIGN, FD_MUX_TILE_SCRATCH_FOOTPRINT( 1UL, 1UL ) );
    FD_TEST( t->out_mcache && t->out_dcache && t->out_fseq && t->in_fseq && t->cnc && metrics );
    ulong o = topo->obj_cnt;
    topo->objs[o  ].id = o;   topo->objs[o  ].wksp_id = 0UL; topo->objs[o  ].offset = woff( t->out_mcache );
    topo->objs[o+1].id = o+1; topo->objs[o+1].wksp_id = 0UL; topo->objs[o+1].offset = woff( t->out_dcache );
    topo->obj_cnt += 2UL;
    ulong li = topo->link_cnt++;
    fd_topo_link_t * lout = &topo->links[li];
    lout->id = li; strcpy( lout->name, "verify_dedup" ); lout->kind_id = j; lout->depth = out_depth;
    lout->mtu = FD_TPU_DCACHE_MTU; lout->burst = OUT_BURST; lout->mcache_obj_id = o; lout->dcache_obj_id = o+1;
    lout->mcache = t->out_mcache; lout->dcache = t->out_dcache;
    fd_topo_tile_t * tt = &topo->tiles[ t->k ];
    tt->out_link_id_primary = li;
    tt->in_link_fseq[0] = t->in_fseq;
    tt->cnc = t->cnc; tt->metrics = metrics;
    t->tile = tt;
  }

  h->res_cap = 64UL + h->n*(12UL + FD_TPU_DCACHE_MTU);
  h->res     = (uchar *)malloc( h->res_cap );
  h->lat_ns  = (uint *)malloc( 4UL*(h->n+1UL) );
  FD_TEST( h->res && h->lat_ns );
  /* both touched before the stream: the consumer appends every published
     frag to res, and a first-touch fault there (a 2 MiB huge page zeroed
     every ~6K frags) held it for a few hundred us at a time, which every
     frag it then read late carried as latency */
  fd_memset( h->lat_ns, 0, 4UL*(h->n+1UL) );
  fd_memset( h->res, 0, h->res_cap );

  /* privileged_init (maps the accelerated tiles' links), then the threads */
  for( ulong j=0UL; j<K; j++ ) {
    if( h->run->privileged_init ) h->run->privileged_init( topo, h->t[j].tile, h->t[j].scratch );
    h->t[j].ctx = h->run->mux_ctx ? h->run->mux_ctx( h->t[j].scratch ) : NULL;
  }
  double t_start = now_s();
  pthread_t tp, tc, tt[ TILE_MAX ];
  FD_TEST( !pthread_create( &tc, NULL, consumer_main, h ) );
  for( ulong j=0UL; j<K; j++ ) FD_TEST( !pthread_create( &tt[j], NULL, tile_main, &h->t[j] ) );
  for( ulong j=0UL; j<K; j++ ) {
    while( fd_cnc_signal_query( h->t[j].cnc )!=FD_CNC_SIGNAL_RUN ) {
      if( now_s() - t_start > timeout ) { printf( "{\"error\": \"tile did not boot\"}\n" ); fflush( stdout ); _exit( 3 ); }
      FD_SPIN_PAUSE();
    }
  }
  double t0 = now_s();
  FD_TEST( !pthread_create( &tp, NULL, producer_main, h ) );

  /* quiescence: every frag consumed by every tile, nothing pending inside
     them, the consumer caught up with what each published */
  int hip = h->run==&fd_tile_verify_hip;
  for(;;) {
    if( now_s() - t_start > timeout ) { printf( "{\"error\": \"timeout\", \"published\": %lu}\n", h->res_cnt ); fflush( stdout ); _exit( 3 ); }
    if( h->consumer_err ) { printf( "{\"error\": \"consumer %d\"}\n", h->consumer_err ); fflush( stdout ); _exit( 4 ); }
    if( !h->producer_done || fd_seq_lt( min_fseq( h ), h->n ) ) { FD_SPIN_PAUSE(); continue; }
    int busy = 0;
    for( ulong j=0UL; j<K && !busy; j++ ) busy = hip && fd_verify_hip_pending( h->t[j].ctx );
    if( busy ) { FD_SPIN_PAUSE(); continue; }
    /* all of the tiles' publishes happened before what was just read; the
       consumer has them once each link's next line is still unpublished */
    FD_COMPILER_MFENCE();
    int behind = 0;
    for( ulong j=0UL; j<K && !behind; j++ ) {
      ulong seq = FD_VOLATILE_CONST( h->t[j].out_seq );
      fd_frag_meta_t const * m = h->t[j].out_mcache + fd_mcache_line_idx( seq, h->out_depth );
      behind = fd_seq_diff( FD_VOLATILE_CONST( m->seq ), seq )>=0L;
    }
    if( behind ) { FD_SPIN_PAUSE(); continue; }
    break;
  }
  double t1 = now_s();
  for( ulong j=0UL; j<K; j++ ) fd_cnc_signal( h->t[j].cnc, FD_CNC_SIGNAL_HALT );
  for( ulong j=0UL; j<K; j++ ) {
    while( !h->t[j].halted ) {
      if( now_s() - t_start > timeout ) { printf( "{\"error\": \"halt timeout\"}\n" ); fflush( stdout ); _exit( 3 ); }
      FD_SPIN_PAUSE();
    }
  }
  h->stop = 1;
  pthread_join( tc, NULL );
  pthread_join( tp, NULL );
  if( hip ) {   /* end each service stream */
    for( ulong j=0UL; j<K; j++ ) {
      fd_ed25519_hip_shlink_t * txl = fd_verify_hip_txn_link( h->t[j].ctx );
      while( fd_ed25519_hip_shlink_publish( txl, NULL, 0UL, 0UL, FD_ED25519_HIP_SHLINK_CTL_EOS )==1 ) {
        if( now_s() - t_start > timeout ) break;
        FD_SPIN_PAUSE();
      }
    }
  }

  FILE * o = fopen( argv[3], "wb" );
  FD_TEST( o && fwrite( h->res, 1UL, h->res_used, o )==h->res_used );
  fclose( o );
  ulong nl = h->res_cnt;
  if( lat_out ) {
    FILE * lo = fopen( lat_out, "wb" );
    FD_TEST( lo && fwrite( h->lat_ns, 4UL, nl, lo )==nl );
    fclose( lo );
  }
  qsort( h->lat_ns, nl, 4UL, cmp_uint );
  double p50 = nl ? 1e-3*(double)h->lat_ns[ (nl-1UL)/2UL ] : 0.0;
  double p99 = nl ? 1e-3*(double)h->lat_ns[ (ulong)((double)(nl-1UL)*0.99) ] : 0.0;
  double pmx = nl ? 1e-3*(double)h->lat_ns[ nl-1UL ] : 0.0;
  int halted_ok = 1;
  for( ulong j=0UL; j<K; j++ ) halted_ok &= h->t[j].halted==1;
  /* the stream's own span: the producer's start (frag 0 due) to the last
     verified frag delivered -- not the thread's start-up before it, nor the
     quiescence check after it, which waits up to a housekeeping interval of
     each tile for its fseq */
  double delivered_s = h->last_recv_tick && h->prod_k0 ? (double)(h->last_recv_tick - h->prod_k0) / h->tick_per_ns * 1e-9
                                                        : t1 - t0;
  printf( "{\"tile\": \"%s\", \"frags\": %lu, \"published\": %lu, \"seconds\": %.6f, \"txn_per_s\": %.1f, "
          "\"delivered_seconds\": %.6f, \"txn_per_s_delivered\": %.1f, "
          "\"rr_cnt\": %lu, \"rr_idx\": %lu, \"tiles_running\": %lu, \"threads\": %lu, \"pinned\": %d, \"sandbox\": %d, "
          "\"rate\": %.1f, \"lat_p50_us\": %.2f, \"lat_p99_us\": %.2f, \"lat_max_us\": %.2f, "
          "\"producer_credit_spins\": %lu, \"consumer_idle_spins\": %lu}\n",
          kind, h->n, h->res_cnt, t1-t0, (double)h->n/(t1-t0), delivered_s, (double)h->n/delivered_s,
          rr_cnt, first, K, K + 2UL, cpu_cnt>0, h->sandbox,
          h->rate, p50, p99, pmx, h->credit_spins, h->idle_spins );
  fflush( stdout );
  _exit( halted_ok ? 0 : 5 );
}
