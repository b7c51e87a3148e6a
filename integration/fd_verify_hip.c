/* fd_verify_hip.c -- the verify tile with its signature verification on an
   MI355X.  Drop-in source for src/app/fdctl/run/tiles/ next to the
   reference's fd_verify.c (src/app/fdctl/run/tiles/fd_verify.c:1-244); it is
   built against the reference's own headers (the include paths below are
   relative to src/).

   Same place in the topology, same callbacks, same output: frags arrive
   from the quic tile round-robin over the verify tiles (before_frag's
   seq % round_robin_cnt), are bounds checked and copied in during_frag,
   and every transaction that parses, has valid signatures and is not an
   HA duplicate is published to dedup as after_frag's frag (payload, pad,
   fd_txn_t, payload_sz) with sig = the dedup tag -- byte for byte and in
   frag order what fd_tile_verify publishes (tests/test_mux_tile.py runs
   both under the reference's fd_mux_tile on the same stream).

   What moves: the tile stays in its write/fsync-only seccomp sandbox
   (src/app/fdctl/run/tiles/verify.seccomppolicy, populate_allowed_seccomp
   below is the reference's, unchanged) and never touches the GPU.  The
   parse, the HA dedup tcache, fd_ed25519_verify_batch_single_msg and the
   construction of the published frag run in the GPU verify service
   (firedancer_amd/csrc/host/fd_verify_service_main.c, one process per GPU
   for all its verify tiles), which this tile reaches through two
   shared-memory links mapped in privileged_init
   (include/fd_ed25519_hip_tile.h, shlink):

     during_frag   the payload is copied straight into the txn link's next
                   dcache room (fd_ed25519_hip_shlink_prepare)
     after_frag    ... and handed over (commit); sig = (frag count << 32) |
                   tsorig, which the service echoes with the verdict
     after_credit  up to `burst` verdict frags are taken back in frag order;
                   a SUCCESS verdict carries the published frag's trailer
                   (fd_txn_t, payload_sz), which the tile appends to its own
                   payload (still in the txn link's dcache) in the out dcache
                   (fd_ed25519_hip_frag_assemble) and publishes with
                   fd_mux_publish (the mux guarantees `burst` credits here,
                   src/disco/mux/fd_mux.c:548-559); the others are filtered
                   -- publishing moves from after_frag to after_credit, which
                   FD_MUX_FLAG_COPY|MANUAL_PUBLISH allow (fd_verify.c:232)

   Flow control: at most `cap` (the txn link's depth, at most
   FD_VERIFY_HIP_RING) frags are unanswered, so the payload of every one of
   them is still intact in the txn link's dcache (a room is reused only
   depth+1 frags later).  The mux runs after_credit before each frag it
   processes, one frag per pass (fd_mux.c:548-559), so after_credit keeps
   the count below cap: when it is at cap, it waits for the oldest verdict,
   which the service produces without ever waiting on the tile (it keeps
   verdicts it cannot publish yet).  The wait ends while the service lives;
   during_frag then always finds room, and the mux's own backpressure (no
   after_credit, no new frags while dedup is behind) bounds the rest.

   Liveness (fd_cnc's heartbeat, src/tango/cnc/fd_cnc.h:63-65,129-130):
   the service ticks the heartbeat of the verdict link; during housekeeping
   and while waiting for room, the tile checks it and both links' status.
   A heartbeat unchanged for FD_VERIFY_HIP_STALE_NS (FD_VERIFY_HIP_BOOT_NS
   before the service's first tick), or a link the service marked failed,
   ends the tile with FD_LOG_ERR -- the reference's reaction to a fatal
   condition in a tile (e.g. fd_verify.c:68), which takes the validator
   down instead of leaving the tile blocked forever.  A verdict frag that
   breaks the protocol (out of order, bad size, bad verdict) marks the txn
   link failed (so the service stops too) and ends the tile the same way.

   The out link's dcache must have room for `burst` frags beyond its depth
   (link burst >= FD_VERIFY_HIP_BURST in the topology). */

#include "disco/tiles.h"
#include "disco/quic/fd_tpu.h"
#include "app/fdctl/run/tiles/generated/verify_seccomp.h"

#include "fd_ed25519_hip_tile.h"

#include <errno.h>
#include <linux/unistd.h>

#define FD_VERIFY_HIP_BURST    (16UL)
#define FD_VERIFY_HIP_RING     (16384UL)                  /* unanswered frags at most (power of 2) */
#define FD_VERIFY_HIP_STALE_NS (1000L*1000L*1000L)        /* 1 s without a heartbeat: the service is gone */
#define FD_VERIFY_HIP_BOOT_NS  (60L*1000L*1000L*1000L)    /* the service's first tick (tables, engines)   */

typedef struct {
  fd_wksp_t * mem;
  ulong       chunk0;
  ulong       wmark;
} fd_verify_hip_in_ctx_t;

typedef struct {
  ulong round_robin_idx;
  ulong round_robin_cnt;

  fd_verify_hip_in_ctx_t in[ 32 ];

  fd_wksp_t * out_mem;
  ulong       out_chunk0;
  ulong       out_wmark;
  ulong       out_chunk;

  fd_ed25519_hip_shlink_t * txl;   /* tile -> service: payloads */
  fd_ed25519_hip_shlink_t * vdl;   /* service -> tile: verdict byte (+ the frag to publish) */
  uchar *                   room;  /* during_frag's copy in the txn link, committed by after_frag */
  ulong                     cap;   /* unanswered frags at most: min( txn link depth, FD_VERIFY_HIP_RING ) */

  ulong sent;                      /* frags handed to the service */
  ulong answered;                  /* verdicts taken back */
  ulong published;                 /* SUCCESS frags published downstream */

  ulong hb_last;                   /* the service's last heartbeat seen */
  long  hb_tick;                   /* fd_tickcount() when it changed */
  long  stale_ticks;
  long  boot_ticks;
  ulong beat;                      /* this tile's own heartbeat on the txn link */

  struct {                         /* the payload of unanswered frag k, in the txn link's dcache */
    uchar const * p;
    ulong         sz;
  } pay[ FD_VERIFY_HIP_RING ];     /* at k & (FD_VERIFY_HIP_RING-1) */
} fd_verify_hip_ctx_t;

FD_FN_CONST static inline ulong
scratch_align( void ) {
  return 128UL;
}

FD_FN_PURE static inline ulong
scratch_footprint( fd_topo_tile_t const * tile ) {
  (void)tile;
  ulong l = FD_LAYOUT_INIT;
  l = FD_LAYOUT_APPEND( l, alignof( fd_verify_hip_ctx_t ), sizeof( fd_verify_hip_ctx_t ) );
  return FD_LAYOUT_FINI( l, scratch_align() );
}

FD_FN_CONST static inline void *
mux_ctx( void * scratch ) {
  return (void*)fd_ulong_align_up( (ulong)scratch, alignof( fd_verify_hip_ctx_t ) );
}

/* The service is alive and healthy, or the tile ends. */
static void
check_service( fd_verify_hip_ctx_t * ctx ) {
  int st = fd_ed25519_hip_shlink_status( ctx->vdl );
  if( !st ) st = fd_ed25519_hip_shlink_status( ctx->txl );
  if( FD_UNLIKELY( st ) )
    FD_LOG_ERR(( "verify service failed (link status %d); verify tile %lu stops", st, ctx->round_robin_idx ));
  ulong hb  = fd_ed25519_hip_shlink_heartbeat_query( ctx->vdl );
  long  now = fd_tickcount();
  if( FD_LIKELY( hb!=ctx->hb_last ) ) { ctx->hb_last = hb; ctx->hb_tick = now; return; }
  long bound = hb ? ctx->stale_ticks : ctx->boot_ticks;
  if( FD_UNLIKELY( now - ctx->hb_tick > bound ) )
    FD_LOG_ERR(( "verify service heartbeat stale (%s for %li ms); verify tile %lu stops",
                 hb ? "unchanged" : "never started",
                 (long)((double)(now - ctx->hb_tick) / fd_tempo_tick_per_ns( NULL ) / 1e6), ctx->round_robin_idx ));
}

static void
protocol_error( fd_verify_hip_ctx_t * ctx,
                char const *          what ) {
  fd_ed25519_hip_shlink_fail( ctx->txl, FD_ED25519_HIP_SHLINK_FAIL_PROTOCOL );
  FD_LOG_ERR(( "verify service broke the frag protocol (%s, verdict %lu); verify tile %lu stops",
               what, ctx->answered, ctx->round_robin_idx ));
}

static void
during_housekeeping( void * _ctx ) {
  fd_verify_hip_ctx_t * ctx = (fd_verify_hip_ctx_t *)_ctx;
  fd_ed25519_hip_shlink_heartbeat( ctx->txl, ++ctx->beat );
  check_service( ctx );
}

/* Reference tile plumbing, kept verbatim so the tile sits in the same
   topology position: src/app/fdctl/run/tiles/fd_verify.c:36-47. */
static void
before_frag( void * _ctx,
             ulong  in_idx,
             ulong  seq,
             ulong  sig,
             int *  opt_filter ) {
  (void)in_idx;
  (void)sig;

  fd_verify_hip_ctx_t * ctx = (fd_verify_hip_ctx_t *)_ctx;
  if( FD_LIKELY( (seq % ctx->round_robin_cnt) != ctx->round_robin_idx ) ) *opt_filter = 1;
}

/* The reference tile's check (fd_verify.c:67-68), then the copy goes
   straight into the txn link, waiting for room if the service is behind. */
static inline void
during_frag( void * _ctx,
             ulong in_idx,
             ulong seq,
             ulong sig,
             ulong chunk,
             ulong sz,
             int * opt_filter ) {
  (void)seq;
  (void)sig;
  (void)opt_filter;

  fd_verify_hip_ctx_t * ctx = (fd_verify_hip_ctx_t *)_ctx;

  /* verbatim: src/app/fdctl/run/tiles/fd_verify.c:67-68 */
  if( FD_UNLIKELY( chunk<ctx->in[in_idx].chunk0 || chunk>ctx->in[in_idx].wmark || sz>FD_TPU_MTU ) )
    FD_LOG_ERR(( "chunk %lu %lu corrupt, not in range [%lu,%lu]", chunk, sz, ctx->in[in_idx].chunk0, ctx->in[in_idx].wmark ));

  uchar * dst = fd_ed25519_hip_shlink_prepare( ctx->txl );
  if( FD_UNLIKELY( !dst ) ) {
    for( ulong spin=1UL;; spin++ ) {
      dst = fd_ed25519_hip_shlink_prepare( ctx->txl );
      if( FD_LIKELY( dst ) ) break;
      if( !(spin & 1023UL) ) { fd_ed25519_hip_shlink_heartbeat( ctx->txl, ++ctx->beat ); check_service( ctx ); }
      FD_SPIN_PAUSE();
    }
  }
  uchar const * src = (uchar const *)fd_chunk_to_laddr_const( ctx->in[in_idx].mem, chunk );
  fd_memcpy( dst, src, sz );
  ctx->room = dst;
}

static inline void
after_frag( void *             _ctx,
            ulong              in_idx,
            ulong              seq,
            ulong *            opt_sig,
            ulong *            opt_chunk,
            ulong *            opt_sz,
            ulong *            opt_tsorig,
            int *              opt_filter,
            fd_mux_context_t * mux ) {
  (void)in_idx;
  (void)seq;
  (void)opt_sig;
  (void)opt_chunk;
  (void)opt_filter;
  (void)mux;

  fd_verify_hip_ctx_t * ctx = (fd_verify_hip_ctx_t *)_ctx;

  /* the service echoes this sig with the verdict: the frag's position in
     this tile's stream (checked on the way back) and its tsorig (what the
     reference publishes downstream, fd_verify.c:153) */
  ulong cookie = ( (ctx->sent & 0xffffffffUL)<<32 ) | ( *opt_tsorig & 0xffffffffUL );
  if( FD_UNLIKELY( !ctx->room || fd_ed25519_hip_shlink_commit( ctx->txl, *opt_sz, cookie, 0U ) ) )
    FD_LOG_CRIT(( "txn link commit failed (sz %lu)", *opt_sz ));
  ctx->pay[ ctx->sent & (FD_VERIFY_HIP_RING-1UL) ].p  = ctx->room;
  ctx->pay[ ctx->sent & (FD_VERIFY_HIP_RING-1UL) ].sz = *opt_sz;
  ctx->room = NULL;
  ctx->sent++;
  /* not filtered and not published here: its verdict comes back through
     after_credit, which publishes it (SUCCESS) or drops it */
}

/* The next verdict frag, if the service has published it: 1 taken (and
   published or filtered), 0 none yet.  A verdict frag is the fd_txn_verify
   / after_frag outcome as one byte (FD_TXN_VERIFY_SUCCESS 0, FAILED -1,
   DEDUP -2, fd_txn_parse failed -3), followed for SUCCESS by the published
   frag's trailer.  The service is trusted for verdicts (it computes them),
   not for memory safety: every size is checked before a byte lands in the
   out dcache. */
static int
take_verdict( fd_verify_hip_ctx_t * ctx,
              fd_mux_context_t *    mux ) {
  ulong sz; ulong sig; uint ctl; int err;
  uchar const * v = fd_ed25519_hip_shlink_peek( ctx->vdl, &sz, &sig, &ctl, &err );
  if( FD_LIKELY( !v ) ) {
    if( FD_UNLIKELY( err<0 ) ) protocol_error( ctx, "verdict link overrun or line out of bounds" );
    return 0;
  }
  if( FD_UNLIKELY( (ctl & FD_ED25519_HIP_SHLINK_CTL_EOS) || ctx->answered==ctx->sent ) ) protocol_error( ctx, "unexpected frag" );
  if( FD_UNLIKELY( (sig>>32)!=(ctx->answered & 0xffffffffUL) || !sz ) ) protocol_error( ctx, "verdict out of order" );
  schar verdict = (schar)v[ 0 ];
  ulong tsorig  = sig & 0xffffffffUL;

  if( FD_LIKELY( verdict==FD_ED25519_HIP_TXN_VERIFY_SUCCESS ) ) {
    ulong         k   = ctx->answered & (FD_VERIFY_HIP_RING-1UL);
    uchar const * pay = ctx->pay[ k ].p;
    ulong         psz = ctx->pay[ k ].sz;
    uchar * dst = (uchar *)fd_chunk_to_laddr( ctx->out_mem, ctx->out_chunk );
    ulong new_sz = fd_ed25519_hip_frag_assemble( dst, pay, psz, v+1, sz-1UL );
    if( FD_UNLIKELY( !new_sz || new_sz>FD_TPU_DCACHE_MTU ) ) protocol_error( ctx, "published frag trailer" );
    if( FD_UNLIKELY( fd_ed25519_hip_shlink_advance( ctx->vdl ) ) ) protocol_error( ctx, "verdict frag overwritten" );

    /* the publish sig is fd_txn_verify's txn_sig, the HA dedup tag: the
       first 8 bytes of the first signature (fd_verify.h:65), found
       through the frag's own fd_txn_t (fd_verify.c:102-128 layout) */
    ulong txnt_off = fd_ulong_align_up( psz, 2UL );
    if( FD_UNLIKELY( txnt_off + sizeof(fd_txn_t) + 2UL>new_sz ) ) protocol_error( ctx, "published frag layout" );
    fd_txn_t const * txn_t = (fd_txn_t const *)( dst + txnt_off );
    ulong signature_off = (ulong)txn_t->signature_off;
    if( FD_UNLIKELY( signature_off + 8UL>psz ) ) protocol_error( ctx, "published frag signature offset" );
    ulong txn_sig = FD_LOAD( ulong, dst + signature_off );

    ulong tspub = (ulong)fd_frag_meta_ts_comp( fd_tickcount() );
    fd_mux_publish( mux, txn_sig, ctx->out_chunk, new_sz, 0UL, tsorig, tspub );
    ctx->out_chunk = fd_dcache_compact_next( ctx->out_chunk, new_sz, ctx->out_chunk0, ctx->out_wmark );
    ctx->published++;
  } else {
    if( FD_UNLIKELY( sz!=1UL || verdict<FD_ED25519_HIP_TXN_PARSE_FAILED || verdict>FD_ED25519_HIP_TXN_VERIFY_FAILED ) )
      protocol_error( ctx, "verdict value" );
    if( FD_UNLIKELY( fd_ed25519_hip_shlink_advance( ctx->vdl ) ) ) protocol_error( ctx, "verdict frag overwritten" );
    /* filtered, as fd_verify.c:119 / :148 */
  }
  ctx->answered++;
  return 1;
}

/* Up to FD_VERIFY_HIP_BURST verdicts, in frag order; then, if cap frags
   are unanswered, wait for the oldest (the frag the mux processes next
   needs room, and every unanswered payload must stay intact).  At most
   one frag arrives between two calls, so the wait takes one verdict and
   the burst is never exceeded. */
static void
after_credit( void *             _ctx,
              fd_mux_context_t * mux ) {
  fd_verify_hip_ctx_t * ctx = (fd_verify_hip_ctx_t *)_ctx;

  ulong n = 0UL;
  while( n<FD_VERIFY_HIP_BURST && take_verdict( ctx, mux ) ) n++;
  for( ulong spin=1UL; ctx->sent - ctx->answered>=ctx->cap; spin++ ) {
    if( take_verdict( ctx, mux ) ) continue;
    /* alive while it waits: the service ends the links of a tile whose
       heartbeat stops (fd_ed25519_hip_vservice_serve) */
    if( !(spin & 1023UL) ) { fd_ed25519_hip_shlink_heartbeat( ctx->txl, ++ctx->beat ); check_service( ctx ); }
    FD_SPIN_PAUSE();
  }
}

/* The service names its links <prefix><kind_id>_txn / _vd with prefix
   "/fd_vhip_<app_name>_" (fd_verify_hip_service --prefix). */
static void
link_name( char *                   out,
           ulong                    out_sz,
           fd_topo_t const *        topo,
           fd_topo_tile_t const *   tile,
           char const *             dir ) {
  FD_TEST( fd_cstr_printf_check( out, out_sz, NULL, "/fd_vhip_%.48s_%lu_%s", topo->app_name, tile->kind_id, dir ) );
}

static void
privileged_init( fd_topo_t *      topo,
                 fd_topo_tile_t * tile,
                 void *           scratch ) {
  FD_SCRATCH_ALLOC_INIT( l, scratch );
  fd_verify_hip_ctx_t * ctx = FD_SCRATCH_ALLOC_APPEND( l, alignof( fd_verify_hip_ctx_t ), sizeof( fd_verify_hip_ctx_t ) );
  fd_memset( ctx, 0, sizeof( fd_verify_hip_ctx_t ) );

  /* map both links before the sandbox: afterwards they are memory only.
     The tile links the link code only (no HIP, so no
     fd_ed25519_hip_abi_check): join itself refuses a link whose frag
     protocol is not this build's (FD_ED25519_HIP_SHLINK_PROTO), so a tile
     and a service of different revisions never exchange frags. */
  char name[ 128 ];
  for( int k=0; k<2; k++ ) {
    link_name( name, sizeof(name), topo, tile, k ? "vd" : "txn" );
    fd_ed25519_hip_shlink_t * l = fd_ed25519_hip_shlink_join( name );
    if( FD_UNLIKELY( !l ) ) {
      if( errno==EPROTO )
        FD_LOG_ERR(( "cannot join %s: the service speaks another frag protocol (this tile: %lu); rebuild both from one "
                     "revision", name, (ulong)FD_ED25519_HIP_SHLINK_PROTO ));
      FD_LOG_ERR(( "cannot join %s (%s): is fd_verify_hip_service running for this GPU?", name, fd_io_strerror( errno ) ));
    }
    if( k ) ctx->vdl = l; else ctx->txl = l;
  }
  ctx->cap = fd_ulong_min( fd_ed25519_hip_shlink_depth( ctx->txl ), FD_VERIFY_HIP_RING );
}

static void
unprivileged_init( fd_topo_t *      topo,
                   fd_topo_tile_t * tile,
                   void *           scratch ) {
  FD_SCRATCH_ALLOC_INIT( l, scratch );
  fd_verify_hip_ctx_t * ctx = FD_SCRATCH_ALLOC_APPEND( l, alignof( fd_verify_hip_ctx_t ), sizeof( fd_verify_hip_ctx_t ) );

  /* in / out link setup verbatim from src/app/fdctl/run/tiles/fd_verify.c:181-200 */
  ctx->round_robin_cnt = fd_topo_tile_name_cnt( topo, tile->name );
  ctx->round_robin_idx = tile->kind_id;

  for( ulong i=0; i<tile->in_cnt; i++ ) {
    fd_topo_link_t * link = &topo->links[ tile->in_link_id[ i ] ];

    if( FD_UNLIKELY( link->is_reasm ) ) {
      fd_topo_wksp_t * link_wksp = &topo->workspaces[ topo->objs[ link->reasm_obj_id ].wksp_id ];
      ctx->in[i].mem = link_wksp->wksp;
      ctx->in[i].chunk0 = fd_laddr_to_chunk( ctx->in[i].mem, link->reasm );
      ctx->in[i].wmark  = ctx->in[i].chunk0 + (link->depth+link->burst-1) * FD_TPU_REASM_CHUNK_MTU;
    } else {
      fd_topo_wksp_t * link_wksp = &topo->workspaces[ topo->objs[ link->dcache_obj_id ].wksp_id ];
      ctx->in[i].mem = link_wksp->wksp;
      ctx->in[i].chunk0 = fd_dcache_compact_chunk0( ctx->in[i].mem, link->dcache );
      ctx->in[i].wmark  = fd_dcache_compact_wmark ( ctx->in[i].mem, link->dcache, link->mtu );
    }
  }

  ctx->out_mem    = topo->workspaces[ topo->objs[ topo->links[ tile->out_link_id_primary ].dcache_obj_id ].wksp_id ].wksp;
  ctx->out_chunk0 = fd_dcache_compact_chunk0( ctx->out_mem, topo->links[ tile->out_link_id_primary ].dcache );
  ctx->out_wmark  = fd_dcache_compact_wmark ( ctx->out_mem, topo->links[ tile->out_link_id_primary ].dcache, topo->links[ tile->out_link_id_primary ].mtu );
  ctx->out_chunk  = ctx->out_chunk0;

  double tick_per_ns = fd_tempo_tick_per_ns( NULL );
  ctx->stale_ticks = (long)( tick_per_ns * (double)FD_VERIFY_HIP_STALE_NS );
  ctx->boot_ticks  = (long)( tick_per_ns * (double)FD_VERIFY_HIP_BOOT_NS  );
  ctx->hb_last     = fd_ed25519_hip_shlink_heartbeat_query( ctx->vdl );
  ctx->hb_tick     = fd_tickcount();

  /* verbatim: src/app/fdctl/run/tiles/fd_verify.c:202-204 */
  ulong scratch_top = FD_SCRATCH_ALLOC_FINI( l, 1UL );
  if( FD_UNLIKELY( scratch_top > (ulong)scratch + scratch_footprint( tile ) ) )
    FD_LOG_ERR(( "scratch overflow %lu %lu %lu", scratch_top - (ulong)scratch - scratch_footprint( tile ), scratch_top, (ulong)scratch + scratch_footprint( tile ) ));
}

/* The reference tile's sandbox, unchanged (the tile needs nothing more):
   verbatim from src/app/fdctl/run/tiles/fd_verify.c:207-228. */
static ulong
populate_allowed_seccomp( void *               scratch,
                          ulong                out_cnt,
                          struct sock_filter * out ) {
  (void)scratch;
  populate_sock_filter_policy_verify( out_cnt, out, (uint)fd_log_private_logfile_fd() );
  return sock_filter_policy_verify_instr_cnt;
}

static ulong
populate_allowed_fds( void * scratch,
                      ulong  out_fds_cnt,
                      int *  out_fds ) {
  (void)scratch;
  if( FD_UNLIKELY( out_fds_cnt < 2 ) ) FD_LOG_ERR(( "out_fds_cnt %lu", out_fds_cnt ));

  ulong out_cnt = 0;
  out_fds[ out_cnt++ ] = 2; /* stderr */
  if( FD_LIKELY( -1!=fd_log_private_logfile_fd() ) )
    out_fds[ out_cnt++ ] = fd_log_private_logfile_fd(); /* logfile */
  return out_cnt;
}

/* Transactions handed to the service whose verdicts have not come back
   (test harness and monitoring; oracle/mux_harness.c). */
ulong
fd_verify_hip_pending( void const * _ctx ) {
  fd_verify_hip_ctx_t const * ctx = (fd_verify_hip_ctx_t const *)_ctx;
  return FD_VOLATILE_CONST( ctx->sent ) - FD_VOLATILE_CONST( ctx->answered );
}

/* The tile's txn link (the harness ends the service's stream with it once
   the tile has halted). */
fd_ed25519_hip_shlink_t *
fd_verify_hip_txn_link( void * _ctx ) {
  return ((fd_verify_hip_ctx_t *)_ctx)->txl;
}

fd_topo_run_tile_t fd_tile_verify_hip = {
  .name                     = "verify",
  .mux_flags                = FD_MUX_FLAG_COPY | FD_MUX_FLAG_MANUAL_PUBLISH,
  .burst                    = FD_VERIFY_HIP_BURST,
  .mux_ctx                  = mux_ctx,
  .mux_during_housekeeping  = during_housekeeping,
  .mux_after_credit         = after_credit,
  .mux_before_frag          = before_frag,
  .mux_during_frag          = during_frag,
  .mux_after_frag           = after_frag,
  .populate_allowed_seccomp = populate_allowed_seccomp,
  .populate_allowed_fds     = populate_allowed_fds,
  .scratch_align            = scratch_align,
  .scratch_footprint        = scratch_footprint,
  .privileged_init          = privileged_init,
  .unprivileged_init        = unprivileged_init,
};
