/* fd_ed25519_hip_tile.c -- host runtime between Firedancer's verify tile
   and the GPU engine (include/fd_ed25519_hip_tile.h): the asynchronous
   pipe, the transaction parser and tcache the verify tile needs, the
   batched verify-tile core, a tango-style ring for the latency mode, and
   the multi-GPU pool with one feeder thread per device.  Plain C11 +
   pthreads over the HIP runtime. */

#define _GNU_SOURCE
#include "../../../include/fd_ed25519_hip_tile.h"
#include "../fd_ed25519_hip_internal.h"

#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <sched.h>
#include <stdatomic.h>
#ifdef FD_ED25519_HIP_AB_SERVICE_PROFILE
#include <x86intrin.h>
#endif
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* engine.c's error buffer is thread-local there; this file reports through
   its own setter so that fd_ed25519_hip_last_error() sees both */
extern char const * fd_ed25519_hip_last_error( void );
void fd_ed25519_hip_private_set_error( char const * msg );

static double
now_s( void ) {
  struct timespec ts;
  clock_gettime( CLOCK_MONOTONIC, &ts );
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static int
tile_fail( char const * what, hipError_t err ) {
  char buf[ 256 ];
  snprintf( buf, sizeof(buf), "%s: %s (%d)", what, hipGetErrorString( err ), (int)err );
  fd_ed25519_hip_private_set_error( buf );
  return FD_ED25519_HIP_ERR_HIP - (int)err;
}

#define TCHK( call, what ) do {                       \
    hipError_t _e = (call);                           \
    if( _e!=hipSuccess ) return tile_fail( what, _e ); \
  } while(0)

unsigned
fd_ed25519_hip_abi_version( void ) {
  return FD_ED25519_HIP_ABI_VERSION;
}

int
fd_ed25519_hip_abi_check( unsigned version, unsigned long slot_sz, unsigned long info_sz,
                          unsigned long vservice_stats_sz ) {
  if( version!=FD_ED25519_HIP_ABI_VERSION || slot_sz!=sizeof(fd_ed25519_hip_slot_t) ||
      info_sz!=sizeof(fd_ed25519_hip_info_t) || vservice_stats_sz!=sizeof(fd_ed25519_hip_vservice_stats_t) ) {
    char buf[ 200 ];
    snprintf( buf, sizeof(buf), "ABI mismatch: caller v%u (%lu, %lu, %lu), library v%u (%lu, %lu, %lu)",
              version, slot_sz, info_sz, vservice_stats_sz, FD_ED25519_HIP_ABI_VERSION,
              (unsigned long)sizeof(fd_ed25519_hip_slot_t), (unsigned long)sizeof(fd_ed25519_hip_info_t),
              (unsigned long)sizeof(fd_ed25519_hip_vservice_stats_t) );
    fd_ed25519_hip_private_set_error( buf );
    return FD_ED25519_HIP_ERR_INVAL;
  }
  return FD_ED25519_HIP_OK;
}

/* ======================================================================
   pipe */

#define PIPE_SLOT_MAX 8

/* Staged payloads start on a cache line: a copy into cold lines that
   starts mid-line costs the host about twice as much (split stores and
   partial-line fills; the staging ring is megabytes, far out of L2), and
   the few bytes of padding per payload cost the link nothing that matters. */
#define STAGE_ALIGN( off ) ( ( (off) + 63UL ) & ~63UL )


#ifdef FD_ED25519_HIP_AB_SERVICE_PROFILE
/* A/B build only: host cycles inside each part of a batch submit */
static __thread unsigned long long pf_sub_h2d, pf_sub_launch, pf_sub_d2h, pf_sub_n, pf_sub_wait;
#define PF_SUB( acc, stmt ) do { unsigned long long c_ = __rdtsc(); stmt; acc += __rdtsc() - c_; } while(0)
#else
#define PF_SUB( acc, stmt ) do { stmt; } while(0)
#endif

#ifdef FD_ED25519_HIP_AB_STAGE_TRACE
/* A/B build only (tools/stage_trace_probe.py): per batch, the host time of
   each stage of its round trip -- submit entered, last launch enqueued,
   poll saw it done, its records resolved -- and the slots in flight when
   it went out; per frag of a latency run, when the producer actually
   published it and when the tile pulled it.  Read with
   fd_ed25519_hip_stage_trace_read. */
#define STAGE_TRACE_MAX (1UL<<18)
typedef struct {
  double t_submit, t_enq, t_done, t_resolved;
  double seq, sig_cnt, txn_cnt, in_flight;
} stage_rec_t;
static stage_rec_t   stage_rec[ STAGE_TRACE_MAX ];
static unsigned long stage_cnt;
static double *        stage_frag_due;    /* per frag: its due time (latency counts from here) */
static double *        stage_frag_pub;    /* per frag: producer's publish time   */
static double *        stage_frag_pull;   /* per frag: the tile's pull time      */
static unsigned long * stage_frag_batch;  /* per frag: the batch (pipe seq) it went into */

void
fd_ed25519_hip_stage_trace_frags( double * t_due, double * t_pub, double * t_pull, unsigned long * batch ) {
  stage_frag_due = t_due; stage_frag_pub = t_pub; stage_frag_pull = t_pull; stage_frag_batch = batch;
}

unsigned long
fd_ed25519_hip_stage_trace_read( double * out, unsigned long max, int reset ) {
  unsigned long n = stage_cnt < max ? stage_cnt : max;
  memcpy( out, stage_rec, n*sizeof(stage_rec_t) );
  if( reset ) stage_cnt = 0UL;
  return n;
}
#endif

/* May a partial batch (the input drained before the batch filled) go out
   with in_flight batches already on the GPU?  Only while a slot stays free
   for a full one, and only while fewer than VTILE_PARTIAL_MAX are in
   flight: at a low offered load every transaction would otherwise leave
   alone on its own slot, and eight slots' kernel chains on eight hardware
   queues at once made each batch's round trip twice as long (in-process
   latency mode at 28K txn/s: p50 0.36 ms with 8 slots, 0.18 ms with 4,
   profiles/r5_latency_low_load.txt; at most 2 / 3 / 4 / 7 in flight:
   p50 0.21 / 0.19 / 0.18 / 0.31-0.35 ms).  Full batches are not limited. */
#ifndef VTILE_PARTIAL_MAX
#define VTILE_PARTIAL_MAX 4U
#endif
static inline int
partial_ok( unsigned in_flight, unsigned slot_cnt ) {
  return in_flight+1U<slot_cnt && in_flight<VTILE_PARTIAL_MAX;
}

#define SLOT_FREE 0
#define SLOT_FILL 1
#define SLOT_BUSY 2
#define SLOT_DONE 3

typedef struct {
  fd_ed25519_hip_slot_t     pub;     /* first member: the public handle */
  fd_ed25519_hip_engine_t * eng;
  hipEvent_t                ev;
  hipEvent_t                ev_h2d;    /* the slot's batch has crossed the link */
  int                       state;
#ifdef FD_ED25519_HIP_AB_STAGE_TRACE
  double                    t_enq;         /* the batch's last launch enqueued */
  unsigned                  in_flight0;    /* batches in flight when it went out */
#endif
  /* staging: the public host arrays live in one pinned block laid out as
     [sigs | pubs | msg_off | msg_sz | txn_first | txn_sig_cnt | msgs], its
     device mirror has the same layout, so a batch goes over in one copy;
     the codes come back the same way ([sig_out | txn_out]) */
  unsigned char *           h_in;
  unsigned char *           d_in;
  unsigned long             in_msgs;    /* offset of msgs in both blocks */
  unsigned long             out_trl;    /* offset of the trailers in both output blocks */
  signed char *             h_outb;
  signed char *             d_outb;
  unsigned char *           d_msgs;
  unsigned long *           d_off;
  unsigned int *            d_sz;
  unsigned char *           d_sigs;
  unsigned char *           d_pubs;
  signed char *             d_out;
  unsigned int *            d_tfirst;
  unsigned int *            d_tcnt;
  signed char *             d_tout;
  unsigned char *           d_trailer; /* raw mode: 64 bytes of fd_txn_t per transaction       */
  unsigned long *           d_soff;    /* raw mode: per-signature message offset (device-made) */
  unsigned int *            d_ssz;     /* raw mode: per-signature message size             */
  unsigned char *           d_pok;     /* raw mode: fd_txn_parse accepted                  */
  unsigned long             dev_bytes; /* the staging mirrors' device bytes                */
  /* raw mode, zero-copy (the verify service): the payloads are DMA'd from
     up to two spans of page-locked memory the caller owns (a shared txn
     link's dcache) instead of the staging block, txn_sig_cnt filled by the
     caller; reset at acquire */
  unsigned char const *     ext_src[ 2 ];
  unsigned char const *     ext_dev[ 2 ];   /* ... the same spans' device-visible addresses */
  unsigned long             ext_len[ 2 ];
  int                       ext_counts;
  unsigned char *           h_in_dev;       /* h_in's device-visible address   */
  unsigned char *           h_outb_dev;     /* h_outb's device-visible address */
  /* host-scalar batches (at most PIPE_HS_MAX signatures, pipe_submit_hs):
     sflag [sig_cap], hflag [sig_cap], hs [19][sig_cap] written by the
     submitting thread and read in place by dsm16; the transactions' codes
     combined on the host when the batch completes */
  unsigned char *           h_hs;
  unsigned char *           h_hs_dev;
  int                       host_combine;
} pipe_slot_t;

/* Batches of at most this many signatures (a verify tile at a low load:
   one or two transactions each) take their scalars from the submitting
   thread (host/fd_ed25519_hip_hsrec.cc, ~8 us a signature) while the GPU
   decompresses A and R, read their signatures and keys from the staging
   block in place, write their codes into the page-locked output block, and
   have their transactions' codes combined on the host: two launches
   (prep16's decode blocks, dsm16) instead of five (pull, prep16, dsm16,
   combine, push).  0 turns it off (fd_ed25519_hip_pipe_set_host_scalars). */
#ifndef PIPE_HS_MAX
#define PIPE_HS_MAX 4UL
#endif
static unsigned long pipe_hs_max = PIPE_HS_MAX;

void
fd_ed25519_hip_pipe_set_host_scalars( unsigned long max_sigs ) {
  pipe_hs_max = max_sigs;
}

/* ... and batches of at most this many also decompress A and R on the
   submitting thread (host/fd_ed25519_hip_hsdec.cc, a few us a signature,
   against the decode blocks' ~44 us): one launch (dsm16, reading the
   points in place) instead of two.  At the reference tile's 95% load
   (54K txn/s, batches of 1.3-1.7 transactions) 4 beats 2: p50 0.108 /
   p99 0.146 ms against 0.137 / 0.239 (profiles/r6_pipe_host_decode.jsonl).
   0 turns it off (fd_ed25519_hip_pipe_set_host_decode). */
#ifndef PIPE_HD_MAX
#define PIPE_HD_MAX 4UL
#endif
#define PIPE_HD_CAP 4UL
static unsigned long pipe_hd_max = PIPE_HD_MAX;

/* ... in a split form's four or eight waves (dsm16s) or dsm16's two (2,
   the default): the split forms put the doublings of A and R on the
   submitting thread, which is the tile's own -- at the reference tile's
   loads four waves lost (p50 0.092 / 0.130 / 0.171 ms against 0.086 /
   0.086 / 0.103 at 29K / 46K / 54K txn/s, the batches growing as the tile
   thread fell behind, profiles/r6_pipe_quarter.jsonl) while the
   synchronous drop-in, whose caller waits anyway, gains
   (fd_ed25519_hip_dropin_set_split_waves) */
static int pipe_split = 2;

/* ... and only for batches of at most this many signatures: each one
   more puts its doublings on the tile thread too */
#ifndef PIPE_SPLIT_MAX_SIGS
#define PIPE_SPLIT_MAX_SIGS 1UL
#endif

void
fd_ed25519_hip_pipe_set_split_waves( int waves ) {
  pipe_split = waves==4 || waves==8 ? waves : 2;
}

void
fd_ed25519_hip_pipe_set_host_decode( unsigned long max_sigs ) {
  pipe_hd_max = max_sigs>PIPE_HD_CAP ? PIPE_HD_CAP : max_sigs;
}

/* the page-locked host-scalar block: sflag [cap], hflag [cap], hs [24][cap]
   words (dsm16: 19 rows; dsm16s: 24), pts [8][40][cap] words (dsm16: rows
   of 20 limbs, A and R; dsm16s: rows of 40, the doubled points' extended
   coordinates too), pflag [2][cap], the go word (params.go) */
#define HS_O_HS( cap )  ( 2UL*(cap) )
#define HS_O_PTS( cap ) ( ( 2UL + 24UL*4UL )*(cap) )
#define HS_O_PFL( cap ) ( ( 2UL + 24UL*4UL + 8UL*40UL*4UL )*(cap) )
#define HS_O_GO( cap )  ( ( ( 2UL + 24UL*4UL + 8UL*40UL*4UL + 2UL )*(cap) + 15UL ) & ~15UL )
#define HS_BYTES( cap ) ( HS_O_GO( cap ) + 16UL )

struct fd_ed25519_hip_pipe {
  int           device;
  unsigned      slot_cnt;
  unsigned long next_acq;    /* ring index of the next slot to acquire */
  unsigned long next_poll;   /* ring index of the oldest submitted slot */
  unsigned long seq;
  unsigned      in_flight;
  hipEvent_t    h2d_tail;    /* ev_h2d of the last batch submitted (one batch on the link at a time, as the pool) */
  int           err;         /* sticky: a batch failed on the GPU (FD_ED25519_HIP_ERR_HIP - hipError_t) */
  int           warming;     /* vt_warm's dummy batches (not the stream's) */
  pipe_slot_t   slot[ PIPE_SLOT_MAX ];
};

static void
pipe_slot_free( pipe_slot_t * s ) {
  hipHostFree( s->h_in ); hipHostFree( s->h_outb ); hipHostFree( s->h_hs );
  hipFree( s->d_in ); hipFree( s->d_outb );
  hipFree( s->d_soff ); hipFree( s->d_ssz ); hipFree( s->d_pok );
  if( s->ev ) hipEventDestroy( s->ev );
  if( s->ev_h2d ) hipEventDestroy( s->ev_h2d );
  if( s->eng ) fd_ed25519_hip_engine_delete( s->eng );
}

void
fd_ed25519_hip_pipe_delete( fd_ed25519_hip_pipe_t * pipe ) {
  if( !pipe ) return;
  hipSetDevice( pipe->device );
  for( unsigned i=0U; i<pipe->slot_cnt; i++ ) {
    if( pipe->slot[i].eng ) fd_ed25519_hip_engine_sync( pipe->slot[i].eng );
    pipe_slot_free( &pipe->slot[i] );
  }
  free( pipe );
}

static int
pipe_slot_init( pipe_slot_t * s, int device, unsigned long sig_cap, unsigned long msg_cap, unsigned long txn_cap,
                int flags ) {
  s->eng = fd_ed25519_hip_engine_new( device, sig_cap, flags | FD_ED25519_HIP_FLAG_ONE_STREAM );
  if( !s->eng ) return FD_ED25519_HIP_ERR_INVAL;
  fd_ed25519_hip_slot_t * p = &s->pub;
  p->sig_cap = sig_cap; p->msg_cap = msg_cap; p->txn_cap = txn_cap;
  unsigned long tc = txn_cap ? txn_cap : 1UL;
  /* per-signature (and, raw mode, per-transaction) offsets and sizes share
     the msg_off / msg_sz arrays: size them for the larger count */
  unsigned long oc = sig_cap > tc ? sig_cap : tc;
  unsigned long o_sigs = 0UL;
  unsigned long o_pubs = o_sigs + 64UL*sig_cap;
  unsigned long o_off  = o_pubs + 32UL*sig_cap;
  unsigned long o_sz   = (o_off + 8UL*oc + 15UL) & ~15UL;
  unsigned long o_tf   = (o_sz  + 4UL*oc + 15UL) & ~15UL;
  unsigned long o_tc   = (o_tf  + 4UL*tc + 15UL) & ~15UL;
  unsigned long o_msgs = (o_tc  + 4UL*tc + 255UL) & ~255UL;
  unsigned long in_sz  = o_msgs + msg_cap + 64UL;
  s->in_msgs = o_msgs;
  /* codes out: [sig_out | txn_out | trailers (64 B per transaction)] */
  s->out_trl = (sig_cap + tc + 63UL) & ~63UL;
  unsigned long out_sz = s->out_trl + 64UL*tc;
  TCHK( hipHostMalloc( (void **)&s->h_in,   in_sz,  hipHostMallocDefault ), "hipHostMalloc" );
  TCHK( hipHostMalloc( (void **)&s->h_outb, out_sz, hipHostMallocCoherent ), "hipHostMalloc" );
  TCHK( hipMalloc(     (void **)&s->d_in,   in_sz                        ), "hipMalloc" );
  TCHK( hipHostGetDevicePointer( (void **)&s->h_in_dev, s->h_in, 0U ), "hipHostGetDevicePointer" );
  TCHK( hipHostGetDevicePointer( (void **)&s->h_outb_dev, s->h_outb, 0U ), "hipHostGetDevicePointer" );
  /* the device-decode layout at the work arrays' stride (no points), or the
     host-decode one at the small stride: room for the larger */
  TCHK( hipHostMalloc( (void **)&s->h_hs, HS_O_PTS( sig_cap )>HS_BYTES( FD_ED25519_HS_STRIDE ) ? HS_O_PTS( sig_cap )
                                                                                               : HS_BYTES( FD_ED25519_HS_STRIDE ),
                       hipHostMallocCoherent ), "hipHostMalloc" );
  TCHK( hipHostGetDevicePointer( (void **)&s->h_hs_dev, s->h_hs, 0U ), "hipHostGetDevicePointer" );
  TCHK( hipMalloc(     (void **)&s->d_outb, out_sz                       ), "hipMalloc" );
  p->sigs        = s->h_in + o_sigs;                   s->d_sigs   = s->d_in + o_sigs;
  p->pubs        = s->h_in + o_pubs;                   s->d_pubs   = s->d_in + o_pubs;
  p->msg_off     = (unsigned long *)(s->h_in + o_off); s->d_off    = (unsigned long *)(s->d_in + o_off);
  p->msg_sz      = (unsigned int  *)(s->h_in + o_sz);  s->d_sz     = (unsigned int  *)(s->d_in + o_sz);
  p->txn_first   = (unsigned int  *)(s->h_in + o_tf);  s->d_tfirst = (unsigned int  *)(s->d_in + o_tf);
  p->txn_sig_cnt = (unsigned int  *)(s->h_in + o_tc);  s->d_tcnt   = (unsigned int  *)(s->d_in + o_tc);
  p->msgs        = s->h_in + o_msgs;                   s->d_msgs   = s->d_in + o_msgs;
  p->sig_out     = s->h_outb;                          s->d_out    = s->d_outb;
  p->txn_out     = s->h_outb + sig_cap;                s->d_tout   = s->d_outb + sig_cap;
  p->txn_trailer = (unsigned char *)s->h_outb + s->out_trl;  s->d_trailer = (unsigned char *)s->d_outb + s->out_trl;
  TCHK( hipMalloc( (void **)&s->d_soff, 8UL*sig_cap ), "hipMalloc" );
  TCHK( hipMalloc( (void **)&s->d_ssz,  4UL*sig_cap ), "hipMalloc" );
  TCHK( hipMalloc( (void **)&s->d_pok,  tc          ), "hipMalloc" );
  s->dev_bytes = in_sz + out_sz + 12UL*sig_cap + tc;
  TCHK( hipEventCreateWithFlags( &s->ev, hipEventDisableTiming ), "hipEventCreate" );
  TCHK( hipEventCreateWithFlags( &s->ev_h2d, hipEventDisableTiming ), "hipEventCreate" );
  s->state = SLOT_FREE;
  return FD_ED25519_HIP_OK;
}

fd_ed25519_hip_pipe_t *
fd_ed25519_hip_pipe_new( int device, unsigned slot_cnt, unsigned long sig_cap, unsigned long msg_cap,
                         unsigned long txn_cap, int flags ) {
  if( slot_cnt<1U || slot_cnt>PIPE_SLOT_MAX || !sig_cap ) {
    fd_ed25519_hip_private_set_error( "pipe_new: slot_cnt must be 1..8 and sig_cap > 0" );
    return NULL;
  }
  fd_ed25519_hip_pipe_t * pipe = (fd_ed25519_hip_pipe_t *)calloc( 1, sizeof(fd_ed25519_hip_pipe_t) );
  if( !pipe ) { fd_ed25519_hip_private_set_error( "pipe_new: calloc failed" ); return NULL; }
  pipe->device   = device;
  pipe->slot_cnt = slot_cnt;
  if( hipSetDevice( device )!=hipSuccess ) { tile_fail( "hipSetDevice", hipErrorInvalidDevice ); free( pipe ); return NULL; }
  for( unsigned i=0U; i<slot_cnt; i++ ) {
    if( pipe_slot_init( &pipe->slot[i], device, sig_cap, msg_cap, txn_cap, flags ) ) {
      fd_ed25519_hip_pipe_delete( pipe );
      return NULL;
    }
  }
  return pipe;
}

/* H2D of a batch: one copy of the staging block's prefix (every array at
   full capacity, then the used message bytes) unless the unused capacity
   would cost more to move than the per-array copies' overhead; sig_cnt
   counts the signature arrays in use, oc_cnt the msg_off/msg_sz entries. */
#define SLOT_ONE_COPY_SLACK (256UL << 10)

typedef struct {
  unsigned char const * src;   /* host address (page-locked) */
  unsigned char const * dev;   /* ... as the device sees it  */
  unsigned char *       dst;
  unsigned long         n;
} h2d_span_t;

/* the staging block's spans a batch moves: its prefix whole, or the arrays
   in use one by one; returns the count (at most 7) */
static unsigned
slot_h2d_spans( pipe_slot_t * s, unsigned long sig_cnt, unsigned long txn_cnt, unsigned long msg_bytes,
                h2d_span_t * sp ) {
  fd_ed25519_hip_slot_t * p = &s->pub;
  unsigned long oc_cnt = sig_cnt > txn_cnt ? sig_cnt : txn_cnt;
  unsigned long used = 96UL*sig_cnt + 12UL*oc_cnt + 8UL*txn_cnt + msg_bytes;
  unsigned long whole = s->in_msgs + msg_bytes;
  unsigned k = 0U;
#define SPAN( host, dptr, bytes ) do { sp[ k ].src = (unsigned char const *)(host);                                  \
                                       sp[ k ].dev = s->h_in_dev + ( (unsigned char const *)(host) - s->h_in );      \
                                       sp[ k ].dst = (unsigned char *)(dptr); sp[ k ].n = (bytes); k++; } while(0)
  if( whole - used <= SLOT_ONE_COPY_SLACK ) {
    SPAN( s->h_in, s->d_in, whole ? whole : 1UL );
    return k;
  }
  if( msg_bytes ) SPAN( p->msgs, s->d_msgs, msg_bytes );
  if( oc_cnt ) {
    SPAN( p->msg_off, s->d_off, 8UL*oc_cnt );
    SPAN( p->msg_sz,  s->d_sz,  4UL*oc_cnt );
  }
  if( sig_cnt ) {
    SPAN( p->sigs, s->d_sigs, 64UL*sig_cnt );
    SPAN( p->pubs, s->d_pubs, 32UL*sig_cnt );
  }
  if( txn_cnt ) {
    SPAN( p->txn_first,   s->d_tfirst, 4UL*txn_cnt );
    SPAN( p->txn_sig_cnt, s->d_tcnt,   4UL*txn_cnt );
  }
#undef SPAN
  return k;
}

/* H2D of a batch after the previous batch's copies (two batches on the
   link at once move fewer bytes than one: DESIGN.md 3b; the batch's
   kernels still overlap the next batch's copy): the staging block's spans
   and, zero-copy, the payload spans from the caller's page-locked memory
   (the second at a 64-byte boundary after the first). */
/* Batches of at most this many signatures skip that ordering: their copy
   is a few tens of KB, and the event that orders it sits on the batch's
   own path (≈6 µs between the copy and the first kernel, rocprofv3) */
#ifndef FD_ED25519_HIP_PIPE_H2D_ORDER_MIN
#define FD_ED25519_HIP_PIPE_H2D_ORDER_MIN 1024UL
#endif
static int
slot_h2d( fd_ed25519_hip_pipe_t * pipe, pipe_slot_t * s, hipStream_t st, unsigned long sig_cnt,
          unsigned long txn_cnt, unsigned long msg_bytes ) {
  int ordered = sig_cnt>FD_ED25519_HIP_PIPE_H2D_ORDER_MIN;
#ifndef FD_ED25519_HIP_AB_POOL_PARALLEL_H2D
  if( ordered && pipe->h2d_tail ) {
    hipError_t we_;
    PF_SUB( pf_sub_wait, we_ = hipStreamWaitEvent( st, pipe->h2d_tail, 0U ) );
    TCHK( we_, "hipStreamWaitEvent(h2d)" );
  }
#endif
  h2d_span_t sp[ 9 ];
  unsigned k = slot_h2d_spans( s, sig_cnt, txn_cnt, s->ext_src[0] ? 0UL : msg_bytes, sp );
  for( int g=0; g<2 && s->ext_src[g] && s->ext_len[g]; g++ ) {   /* zero-copy payloads */
    sp[ k ].src = s->ext_src[g]; sp[ k ].dev = s->ext_dev[g]; sp[ k ].n = s->ext_len[g];
    sp[ k ].dst = s->d_msgs + ( g ? STAGE_ALIGN( s->ext_len[0] ) : 0UL );
    k++;
  }
#ifndef FD_ED25519_HIP_AB_COPY_ENGINES
  for( unsigned i0=0U; i0<k; i0+=FD_ED25519_PULL_SPAN_MAX ) {   /* one launch moves up to 8 spans (9 at most here) */
    fd_ed25519_pull_params_t pp;
    memset( &pp, 0, sizeof(pp) );
    for( unsigned i=i0; i<k && i-i0<FD_ED25519_PULL_SPAN_MAX; i++ ) {
      pp.src[ pp.cnt ] = sp[ i ].dev; pp.dst[ pp.cnt ] = sp[ i ].dst; pp.n[ pp.cnt ] = sp[ i ].n; pp.cnt++;
    }
    int le = fd_ed25519_hip_launch_pull( &pp, st );
    if( le ) return tile_fail( "H2D pull launch", (hipError_t)le );
  }
#else
  for( unsigned i=0U; i<k; i++ )
    TCHK( hipMemcpyAsync( sp[ i ].dst, sp[ i ].src, sp[ i ].n, hipMemcpyHostToDevice, st ), "H2D batch" );
#endif
  if( ordered ) {
    TCHK( hipEventRecord( s->ev_h2d, st ), "hipEventRecord(h2d)" );
    pipe->h2d_tail = s->ev_h2d;
  }
  return FD_ED25519_HIP_OK;
}

/* D2H of the codes: [sig_out | txn_out] in one copy when transactions are
   combined (txn_out sits after sig_cap signature codes), else sig_out;
   with the device-parsed trailers too (raw mode).  Like the H2D, a launch
   that writes the page-locked block through its device-visible address,
   not a copy-engine copy: a hipMemcpyAsync here held the service's link
   thread for the copy. */
static int
slot_d2h( pipe_slot_t * s, hipStream_t st, unsigned long sig_cnt, unsigned long txn_cnt, int trailers ) {
  unsigned long n = trailers ? s->out_trl + 64UL*txn_cnt : (txn_cnt ? s->pub.sig_cap + txn_cnt : sig_cnt);
  if( !n ) return FD_ED25519_HIP_OK;
#ifndef FD_ED25519_HIP_AB_COPY_ENGINES
  fd_ed25519_pull_params_t pp;
  memset( &pp, 0, sizeof(pp) );
  pp.src[0] = (unsigned char const *)s->d_outb; pp.dst[0] = s->h_outb_dev; pp.n[0] = n; pp.cnt = 1U;
  int le = fd_ed25519_hip_launch_pull( &pp, st );
  if( le ) return tile_fail( "D2H push launch", (hipError_t)le );
#else
  TCHK( hipMemcpyAsync( s->h_outb, s->d_outb, n, hipMemcpyDeviceToHost, st ), "D2H codes" );
#endif
  return FD_ED25519_HIP_OK;
}

fd_ed25519_hip_slot_t *
fd_ed25519_hip_pipe_acquire( fd_ed25519_hip_pipe_t * pipe ) {
  pipe_slot_t * s = &pipe->slot[ pipe->next_acq % pipe->slot_cnt ];
  if( s->state!=SLOT_FREE ) return NULL;
  s->state = SLOT_FILL;
  pipe->next_acq++;
  s->pub.sig_cnt = 0UL; s->pub.msg_bytes = 0UL; s->pub.txn_cnt = 0UL;
  s->ext_src[0] = s->ext_src[1] = NULL; s->ext_dev[0] = s->ext_dev[1] = NULL;
  s->ext_len[0] = s->ext_len[1] = 0UL; s->ext_counts = 0;
  return &s->pub;
}

/* The kernels read what the staged offsets point at, with no bounds of
   their own: a message range past the staged bytes, or a transaction's
   signature range past the staged signatures, would be an out-of-bounds
   device read.  Checked on the host before anything is copied (a few ns
   per signature). */
static int
slot_check( fd_ed25519_hip_slot_t const * slot, unsigned long sig_cnt, unsigned long msg_bytes,
            unsigned long txn_cnt ) {
  for( unsigned long i=0UL; i<sig_cnt; i++ ) {
    if( slot->msg_off[ i ]>msg_bytes || slot->msg_sz[ i ]>msg_bytes - slot->msg_off[ i ] ) {
      fd_ed25519_hip_private_set_error( "pipe_submit: a signature's message lies outside the staged bytes" );
      return FD_ED25519_HIP_ERR_INVAL;
    }
  }
  for( unsigned long t=0UL; t<txn_cnt; t++ ) {
    unsigned long c = slot->txn_sig_cnt[ t ];
    if( c>=1UL && c<=16UL && ( slot->txn_first[ t ]>sig_cnt || c>sig_cnt - slot->txn_first[ t ] ) ) {
      fd_ed25519_hip_private_set_error( "pipe_submit: a transaction's signatures lie outside the staged ones" );
      return FD_ED25519_HIP_ERR_INVAL;
    }
  }
  return FD_ED25519_HIP_OK;
}

/* A host-scalar batch (PIPE_HS_MAX above): the decompressions launched
   first, the scalars computed meanwhile, then dsm16 writing the signature
   codes into the page-locked output block -- or (PIPE_HD_MAX) dsm16
   launched first, waiting on the go word, and the scalars and
   decompressions computed while it is dispatched.  1: submitted; 0: a
   signature has no half-size pair (~1e-6), nothing but the decode launch
   (or a cancelled dsm16) was queued and the caller takes the device's own
   path; < 0: a launch failed. */
static int
pipe_submit_hs( fd_ed25519_hip_pipe_t * pipe, pipe_slot_t * s, hipStream_t st ) {
  fd_ed25519_hip_slot_t * slot = &s->pub;
  unsigned long n = slot->sig_cnt, cap = slot->sig_cap;
  unsigned long o_sigs = (unsigned long)( slot->sigs - s->h_in ), o_pubs = (unsigned long)( slot->pubs - s->h_in );
  int err, hd = n<=pipe_hd_max;
  int split = hd && n<=PIPE_SPLIT_MAX_SIGS && pipe_split>2 && fd_ed25519_hip_private_want_dsms( s->eng, pipe_split )
              ? pipe_split : 0;
  /* the host block's stride: the work arrays' when the device decodes, a
     small one when every array is this thread's (FD_ED25519_HS_STRIDE) */
  unsigned long sc = hd ? FD_ED25519_HS_STRIDE : cap;
  volatile uint32_t * go = (volatile uint32_t *)( s->h_hs + HS_O_GO( sc ) );
  if( !hd ) {
    PF_SUB( pf_sub_launch, err = fd_ed25519_hip_private_hs_decode( s->eng, n, s->h_in_dev + o_sigs, s->h_in_dev + o_pubs,
                                                                   (signed char *)s->h_outb_dev, st ) );
    if( err ) return err;
  } else {
    /* dsm16 first, waiting on the go word while this thread computes
       (params.go); every path below stores RUN or CANCEL */
    *go = 0U;
    if( split ) {
      PF_SUB( pf_sub_launch, err = fd_ed25519_hip_private_hs_dsms( s->eng, split, n, s->h_in_dev + o_sigs, s->h_in_dev + o_pubs,
                                                                   (signed char *)s->h_outb_dev, s->h_hs_dev,
                                                                   s->h_hs_dev + sc,
                                                                   (unsigned int const *)( s->h_hs_dev + HS_O_HS( sc ) ),
                                                                   (int const *)( s->h_hs_dev + HS_O_PTS( sc ) ),
                                                                   s->h_hs_dev + HS_O_PFL( sc ),
                                                                   (unsigned int const *)( s->h_hs_dev + HS_O_GO( sc ) ), st ) );
    } else {
      PF_SUB( pf_sub_launch, err = fd_ed25519_hip_private_hs_dsm( s->eng, n, s->h_in_dev + o_sigs, s->h_in_dev + o_pubs,
                                                                  (signed char *)s->h_outb_dev, s->h_hs_dev,
                                                                  s->h_hs_dev + sc,
                                                                  (unsigned int const *)( s->h_hs_dev + HS_O_HS( sc ) ),
                                                                  (int const *)( s->h_hs_dev + HS_O_PTS( sc ) ),
                                                                  s->h_hs_dev + HS_O_PFL( sc ),
                                                                  (unsigned int const *)( s->h_hs_dev + HS_O_GO( sc ) ), st ) );
    }
    if( err ) return err;
  }
  unsigned char * hsf = s->h_hs, * hhf = s->h_hs + sc;
  uint32_t *      hs  = (uint32_t *)( s->h_hs + HS_O_HS( sc ) );
  int dbits = fd_ed25519_hip_private_half_dbits( s->eng );
  for( unsigned long i=0UL; i<n; i++ ) {
    uint32_t rec[ 32 ];
    if( !fd_ed25519_hip_private_hsrec( slot->sigs + 64UL*i, slot->pubs + 32UL*i, slot->msgs + slot->msg_off[ i ],
                                       slot->msg_sz[ i ], dbits, rec ) ) {
      if( hd ) __atomic_store_n( go, FD_ED25519_GO_CANCEL, __ATOMIC_RELEASE );
      return 0;
    }
    if( split ) fd_ed25519_hip_private_hssplit( rec, split, hs, sc, i );
    else for( int w=0; w<19; w++ ) hs[ (unsigned long)w*sc + i ] = rec[ 8 + w ];
    hsf[ i ] = (unsigned char)rec[ 27 ];
    hhf[ i ] = (unsigned char)rec[ 28 ];
  }
  if( hd ) {   /* A and R of each signature, side by side */
    unsigned char const * enc[ 2UL*PIPE_HD_CAP ];
    int32_t       pt[ 2UL*PIPE_HD_CAP ][ 20 ], ptx[ 2UL*PIPE_HD_CAP*3UL ][ 40 ];
    unsigned char fl[ 2UL*PIPE_HD_CAP ];
    int nx = split ? split/2 - 1 : 0, step = split==4 ? 66 : 33;
    for( unsigned long i=0UL; i<n; i++ ) { enc[ 2UL*i ] = slot->pubs + 32UL*i; enc[ 2UL*i+1UL ] = slot->sigs + 64UL*i; }
    fd_ed25519_hip_private_hsdec3_n( enc, 2UL*n, !fd_ed25519_hip_private_codes_portable( s->eng ), &pt[0][0],
                                     split ? &ptx[0][0] : NULL, nx, step, fl );
    int32_t * pts = (int32_t *)( s->h_hs + HS_O_PTS( sc ) );
    unsigned char * pfl = s->h_hs + HS_O_PFL( sc );
    unsigned long rs = split ? 40UL : 20UL;   /* the row stride in limbs: dsm16s's, dsm16's */
    for( unsigned long i=0UL; i<n; i++ )
      for( unsigned long side=0UL; side<2UL; side++ ) {   /* rows 2i + side: A, R, A_1, R_1, .. */
        unsigned long pi = 2UL*i + side;
        for( unsigned long l=0UL; l<20UL; l++ ) pts[ ( side*rs + l )*sc + i ] = pt[ pi ][ l ];
        for( int m=1; m<=nx; m++ )
          for( unsigned long l=0UL; l<40UL; l++ )
            pts[ ( ( 2UL*(unsigned long)m + side )*40UL + l )*sc + i ] = ptx[ pi*(unsigned long)nx + (unsigned long)(m-1) ][ l ];
        pfl[ side*sc + i ] = fl[ pi ];
      }
  }
  if( hd ) {
    __atomic_store_n( go, FD_ED25519_GO_RUN, __ATOMIC_RELEASE );
  } else {
    PF_SUB( pf_sub_launch, err = fd_ed25519_hip_private_hs_dsm( s->eng, n, s->h_in_dev + o_sigs, s->h_in_dev + o_pubs,
                                                                (signed char *)s->h_outb_dev, s->h_hs_dev,
                                                                s->h_hs_dev + sc,
                                                                (unsigned int const *)( s->h_hs_dev + HS_O_HS( sc ) ),
                                                                NULL, NULL, NULL, st ) );
    if( err ) return err;
  }
  s->host_combine = slot->txn_cnt ? 1 : 0;
  TCHK( hipEventRecord( s->ev, st ), "hipEventRecord" );
#ifdef FD_ED25519_HIP_AB_STAGE_TRACE
  s->t_enq = now_s(); s->in_flight0 = pipe->in_flight;
#endif
  s->state = SLOT_BUSY;
  pipe->in_flight++;
  return 1;
}

/* batch_single_msg's rule per transaction (fd_ed25519_user.c:231-309, the
   device's fd_ed25519_txn_combine_kernel): 0 or > 16 signatures ERR_SIG;
   else the first error other than ERR_MSG in signature order, else ERR_MSG
   if any signature had it, else SUCCESS */
static void
host_combine( fd_ed25519_hip_slot_t * slot ) {
  for( unsigned long t=0UL; t<slot->txn_cnt; t++ ) {
    unsigned int f = slot->txn_first[ t ], n = slot->txn_sig_cnt[ t ];
    int code = FD_ED25519_SUCCESS, msg_fail = 0;
    if( n==0U || n>16U ) code = FD_ED25519_ERR_SIG;
    else for( unsigned int j=0U; j<n; j++ ) {
      int c = slot->sig_out[ f + j ];
      if( c==FD_ED25519_ERR_MSG ) msg_fail = 1;
      else if( c!=FD_ED25519_SUCCESS ) { code = c; break; }
    }
    if( code==FD_ED25519_SUCCESS && msg_fail ) code = FD_ED25519_ERR_MSG;
    slot->txn_out[ t ] = (signed char)code;
  }
}

int
fd_ed25519_hip_pipe_submit( fd_ed25519_hip_pipe_t * pipe, fd_ed25519_hip_slot_t * slot,
                            unsigned long sig_cnt, unsigned long msg_bytes, unsigned long txn_cnt ) {
  pipe_slot_t * s = (pipe_slot_t *)slot;
  if( s->state!=SLOT_FILL || sig_cnt>slot->sig_cap || msg_bytes>slot->msg_cap || txn_cnt>slot->txn_cap )
    return FD_ED25519_HIP_ERR_INVAL;
  if( slot_check( slot, sig_cnt, msg_bytes, txn_cnt ) ) return FD_ED25519_HIP_ERR_INVAL;
  TCHK( hipSetDevice( pipe->device ), "hipSetDevice" );
  hipStream_t st = (hipStream_t)fd_ed25519_hip_engine_stream( s->eng );
  slot->sig_cnt = sig_cnt; slot->msg_bytes = msg_bytes; slot->txn_cnt = txn_cnt;
  slot->seq = pipe->seq++;
  slot->t_submit = now_s();
  s->host_combine = 0;
  int err;
  if( sig_cnt && sig_cnt<=pipe_hs_max && !s->ext_src[0] && !pipe->warming ) {
    err = pipe_submit_hs( pipe, s, st );
    if( err<0 ) return err;
    if( err==1 ) return FD_ED25519_HIP_OK;   /* 0: a signature without a half-size pair, the device's own path below */
  }
  PF_SUB( pf_sub_h2d, err = slot_h2d( pipe, s, st, sig_cnt, txn_cnt, msg_bytes ) );
  if( err ) return err;
#ifdef FD_ED25519_HIP_HOST_FAULT
  /* test build only (tests/test_gpu_service_fault.py): the stream's third
     batch's launch fails after its copies are enqueued -- or, with
     $FD_ED25519_HIP_FAULT_STALL_MS, is held on the device that long (a
     bounded stand-in for a hung GPU) before its kernels */
  if( slot->seq==2UL && !pipe->warming ) {
    char const * stall = getenv( "FD_ED25519_HIP_FAULT_STALL_MS" );
    if( stall && *stall ) {
      err = fd_ed25519_hip_launch_stall( (unsigned)strtoul( stall, NULL, 10 ), st );
      if( err ) return tile_fail( "stall launch", (hipError_t)err );
    } else {
      fd_ed25519_hip_private_set_error( "pipe: injected launch failure (fault-injection build)" );
      return FD_ED25519_HIP_ERR_HIP - (int)hipErrorLaunchFailure;
    }
  }
#endif
  if( sig_cnt ) {
    PF_SUB( pf_sub_launch, err = fd_ed25519_hip_verify_dev( s->eng, sig_cnt, s->d_msgs, s->d_off, s->d_sz, s->d_sigs,
                                                             s->d_pubs, s->d_out, st ) );
    if( err ) return err;
  }
  if( txn_cnt ) {
    PF_SUB( pf_sub_launch, err = fd_ed25519_hip_txn_combine_dev( s->eng, txn_cnt, s->d_out, s->d_tfirst, s->d_tcnt,
                                                                 s->d_tout, st ) );
    if( err ) return err;
  }
  PF_SUB( pf_sub_d2h, err = slot_d2h( s, st, sig_cnt, txn_cnt, 0 ) );
  if( err ) return err;
#ifdef FD_ED25519_HIP_AB_SERVICE_PROFILE
  pf_sub_n++;
#endif
  TCHK( hipEventRecord( s->ev, st ), "hipEventRecord" );
#ifdef FD_ED25519_HIP_AB_STAGE_TRACE
  s->t_enq = now_s(); s->in_flight0 = pipe->in_flight;
#endif
  s->state = SLOT_BUSY;
  pipe->in_flight++;
  return FD_ED25519_HIP_OK;
}

int
fd_ed25519_hip_pipe_submit_txns( fd_ed25519_hip_pipe_t * pipe, fd_ed25519_hip_slot_t * slot,
                                 unsigned long txn_cnt, unsigned long payload_bytes ) {
  pipe_slot_t * s = (pipe_slot_t *)slot;
  if( s->state!=SLOT_FILL || txn_cnt>slot->txn_cap || txn_cnt>slot->sig_cap || payload_bytes>slot->msg_cap )
    return FD_ED25519_HIP_ERR_INVAL;
  /* signature slots from byte 0 of each payload (its signature count if
     fd_txn_parse accepts it; 0 or > 16 reserve none) */
  unsigned long slots = 0UL;
  if( s->ext_src[0] && payload_bytes!=( s->ext_len[1] ? STAGE_ALIGN( s->ext_len[0] ) + s->ext_len[1] : s->ext_len[0] ) )
    return FD_ED25519_HIP_ERR_INVAL;
  for( unsigned long t=0UL; t<txn_cnt; t++ ) {
    if( slot->msg_off[ t ]>payload_bytes || slot->msg_sz[ t ]>payload_bytes - slot->msg_off[ t ] ) {
      fd_ed25519_hip_private_set_error( "pipe_submit_txns: a payload lies outside the staged bytes" );
      return FD_ED25519_HIP_ERR_INVAL;
    }
    /* the count from payload byte 0 (zero-copy: the caller read it) */
    unsigned int c = s->ext_counts ? slot->txn_sig_cnt[ t ] : slot->msg_sz[ t ] ? slot->msgs[ slot->msg_off[ t ] ] : 0U;
    slot->txn_first  [ t ] = (unsigned int)slots;
    slot->txn_sig_cnt[ t ] = c;
    if( c>=1U && c<=16U ) slots += c;
  }
  if( slots>slot->sig_cap ) return FD_ED25519_HIP_ERR_INVAL;
  TCHK( hipSetDevice( pipe->device ), "hipSetDevice" );
  hipStream_t st = (hipStream_t)fd_ed25519_hip_engine_stream( s->eng );
  slot->sig_cnt = slots; slot->msg_bytes = payload_bytes; slot->txn_cnt = txn_cnt;
  slot->seq = pipe->seq++;
  slot->t_submit = now_s();
  s->host_combine = 0;   /* the device combines raw batches (txn_finish) */
  if( txn_cnt ) {
    /* the per-transaction offsets / sizes travel in msg_off / msg_sz; the
       device writes the per-signature ones (and the signatures and keys)
       into arrays of its own */
    int err;
    PF_SUB( pf_sub_h2d, err = slot_h2d( pipe, s, st, 0UL, txn_cnt, payload_bytes ) );
    if( err ) return err;
    fd_ed25519_txn_stage_params_t sp;
    sp.payloads = s->d_msgs; sp.pay_off = s->d_off; sp.pay_sz = s->d_sz; sp.txn_first = s->d_tfirst;
    sp.txn_cnt = s->d_tcnt; sp.ntxn = txn_cnt; sp.sigs = s->d_sigs; sp.pubs = s->d_pubs; sp.msg_off = s->d_soff;
    sp.msg_sz = s->d_ssz; sp.parse_ok = s->d_pok; sp.trailer = s->d_trailer;
    PF_SUB( pf_sub_launch, err = fd_ed25519_hip_launch_txn_stage( &sp, st ) );
    if( err ) return tile_fail( "txn_stage launch", (hipError_t)err );
    if( slots ) {
        PF_SUB( pf_sub_launch, err = fd_ed25519_hip_verify_dev( s->eng, slots, s->d_msgs, s->d_soff, s->d_ssz, s->d_sigs,
                                                               s->d_pubs, s->d_out, st ) );
      if( err ) return err;
    }
    PF_SUB( pf_sub_launch, err = fd_ed25519_hip_launch_txn_finish( s->d_out, s->d_tfirst, s->d_tcnt, s->d_pok, s->d_tout,
                                                                   txn_cnt, st ) );
    if( err ) return tile_fail( "txn_finish launch", (hipError_t)err );
    PF_SUB( pf_sub_d2h, err = slot_d2h( s, st, slots, txn_cnt, 1 ) );
    if( err ) return err;
#ifdef FD_ED25519_HIP_AB_SERVICE_PROFILE
    pf_sub_n++;
#endif
  }
  TCHK( hipEventRecord( s->ev, st ), "hipEventRecord" );
#ifdef FD_ED25519_HIP_AB_STAGE_TRACE
  s->t_enq = now_s(); s->in_flight0 = pipe->in_flight;
#endif
  s->state = SLOT_BUSY;
  pipe->in_flight++;
  return FD_ED25519_HIP_OK;
}

fd_ed25519_hip_slot_t *
fd_ed25519_hip_pipe_poll( fd_ed25519_hip_pipe_t * pipe, int wait ) {
  pipe_slot_t * s = &pipe->slot[ pipe->next_poll % pipe->slot_cnt ];
  if( s->state!=SLOT_BUSY ) return NULL;
  hipError_t e = wait ? hipEventSynchronize( s->ev ) : hipEventQuery( s->ev );
  if( e==hipErrorNotReady ) return NULL;
  if( e!=hipSuccess ) {
    /* a failed batch is unrecoverable for the pipe: the error sticks (no
       later batch is trusted either), the caller decides what to do
       (the verify service marks its links failed and stops) */
    char what[ 64 ];
    snprintf( what, sizeof(what), "batch %lu failed on the GPU", s->pub.seq );
    if( !pipe->err ) pipe->err = tile_fail( what, e );
    return NULL;
  }
  s->pub.t_done = now_s();
  if( s->host_combine ) host_combine( &s->pub );
  s->state = SLOT_DONE;
  pipe->next_poll++;
  pipe->in_flight--;
  return &s->pub;
}

void
fd_ed25519_hip_pipe_release( fd_ed25519_hip_pipe_t * pipe, fd_ed25519_hip_slot_t * slot ) {
  (void)pipe;
  pipe_slot_t * s = (pipe_slot_t *)slot;
  if( s->state==SLOT_DONE ) s->state = SLOT_FREE;
}

unsigned
fd_ed25519_hip_pipe_in_flight( fd_ed25519_hip_pipe_t const * pipe ) {
  return pipe->in_flight;
}

int
fd_ed25519_hip_pipe_error( fd_ed25519_hip_pipe_t const * pipe ) {
  return pipe->err;
}

unsigned long
fd_ed25519_hip_pipe_device_bytes( fd_ed25519_hip_pipe_t const * pipe ) {
  unsigned long b = 0UL;
  for( unsigned i=0U; i<pipe->slot_cnt; i++ ) {
    fd_ed25519_hip_info_t info;
    if( !fd_ed25519_hip_engine_info( pipe->slot[i].eng, &info ) ) b += info.device_bytes;
    b += pipe->slot[i].dev_bytes;
  }
  return b;
}

/* ======================================================================
   txn: fd_txn_parse restated once in fd_txn_parse_core.h (shared with the
   device staging kernel, fd_ed25519_txn.hip). */

#include "../fd_txn_parse_core.h"

int
fd_ed25519_hip_txn_parse( unsigned char const * p, unsigned long sz, fd_ed25519_hip_txn_t * out ) {
  return fd_txn_core_parse( p, sz, out, NULL, 0UL ) ? 1 : 0;
}

unsigned long
fd_ed25519_hip_txn_parse_full( unsigned char const * p, unsigned long sz, void * out_txn ) {
  return fd_txn_core_parse( p, sz, NULL, (unsigned char *)out_txn, FD_ED25519_HIP_TXN_MAX_SZ );
}

/* [payload | pad to 2 | fd_txn_t | u16 payload_sz] (fd_verify.c:102-133) */
static unsigned long
txn_frag_core( unsigned char const * p, unsigned long sz, unsigned char * out, fd_ed25519_hip_txn_t * t ) {
  if( sz>FD_ED25519_HIP_TXN_MTU ) return 0UL;
  unsigned long toff = (sz + 1UL) & ~1UL;
  unsigned long foot = fd_txn_core_parse( p, sz, t, out + toff, FD_ED25519_HIP_TXN_MAX_SZ );
  if( !foot ) return 0UL;
  memcpy( out, p, sz );
  if( toff>sz ) out[ sz ] = 0;
  out[ toff + foot     ] = (unsigned char)sz;
  out[ toff + foot + 1 ] = (unsigned char)(sz >> 8);
  return toff + foot + 2UL;
}

unsigned long
fd_ed25519_hip_txn_frag( unsigned char const * p, unsigned long sz, unsigned char * out ) {
  fd_ed25519_hip_txn_t t;
  return txn_frag_core( p, sz, out, &t );
}

/* ======================================================================
   tcache: a ring of the last `depth` tags plus an open-addressed map
   (linear probing from tag & (map_cnt-1), tag 0 = empty slot), with the
   reference's semantics (src/tango/tcache/fd_tcache.h:259-404): query stops
   at the tag or at an empty slot -- so tag 0 always "hits" an empty slot;
   insert of a present tag changes nothing; otherwise the tag goes in and
   the tag `depth` inserts older is removed from the map with backward-shift
   deletion. */

struct fd_ed25519_hip_tcache {
  unsigned long depth, map_cnt, oldest;
  unsigned long * ring;
  unsigned long * map;
};

fd_ed25519_hip_tcache_t *
fd_ed25519_hip_tcache_new( unsigned long depth, unsigned long map_cnt ) {
  if( !depth || !map_cnt || (map_cnt & (map_cnt-1UL)) || map_cnt<depth+2UL ) return NULL;
  fd_ed25519_hip_tcache_t * tc = (fd_ed25519_hip_tcache_t *)calloc( 1, sizeof(*tc) );
  if( !tc ) return NULL;
  tc->depth = depth; tc->map_cnt = map_cnt;
  tc->ring = (unsigned long *)calloc( depth, sizeof(unsigned long) );
  tc->map  = (unsigned long *)calloc( map_cnt, sizeof(unsigned long) );
  if( !tc->ring || !tc->map ) { fd_ed25519_hip_tcache_delete( tc ); return NULL; }
  return tc;
}

void
fd_ed25519_hip_tcache_delete( fd_ed25519_hip_tcache_t * tc ) {
  if( !tc ) return;
  free( tc->ring ); free( tc->map ); free( tc );
}

static unsigned long
tc_probe( fd_ed25519_hip_tcache_t const * tc, unsigned long tag, int * found ) {
  unsigned long m = tc->map_cnt - 1UL, idx = tag & m;
  for( ;; ) {
    unsigned long t = tc->map[ idx ];
    if( t==tag ) { *found = 1; return idx; }
    if( !t )     { *found = 0; return idx; }
    idx = (idx+1UL) & m;
  }
}

int
fd_ed25519_hip_tcache_query( fd_ed25519_hip_tcache_t const * tc, unsigned long tag ) {
  int found;
  tc_probe( tc, tag, &found );
  return found;
}

static void
tc_remove( fd_ed25519_hip_tcache_t * tc, unsigned long tag ) {
  if( !tag ) return;
  int found;
  unsigned long slot = tc_probe( tc, tag, &found );
  if( !found ) return;
  unsigned long m = tc->map_cnt - 1UL;
  for( ;; ) {
    tc->map[ slot ] = 0UL;
    unsigned long hole = slot;
    for( ;; ) {
      slot = (slot+1UL) & m;
      unsigned long t = tc->map[ slot ];
      if( !t ) return;
      unsigned long home = t & m;
      /* t may stay iff its home lies cyclically in (hole, slot] */
      int stays = hole<=slot ? (hole<home && home<=slot) : (hole<home || home<=slot);
      if( !stays ) break;
    }
    tc->map[ hole ] = tc->map[ slot ];
  }
}

int
fd_ed25519_hip_tcache_insert( fd_ed25519_hip_tcache_t * tc, unsigned long tag ) {
  int found;
  unsigned long idx = tc_probe( tc, tag, &found );
  if( found ) return 1;
  tc->map[ idx ] = tag;
  unsigned long evict = tc->ring[ tc->oldest ];
  tc->ring[ tc->oldest ] = tag;
  tc->oldest = tc->oldest+1UL==tc->depth ? 0UL : tc->oldest+1UL;
  tc_remove( tc, evict );
  return 0;
}

/* ======================================================================
   vtile: fd_txn_verify batched.

   Every frag becomes a record in a FIFO.  Parse failures are answered at
   once (after_frag filters them, fd_verify.c:117-121); parsed transactions
   are staged into the open pipe slot.  When a batch completes, its records
   are resolved in frag order with exactly fd_txn_verify's sequence
   (fd_verify.h:65-87): tcache query -> DEDUP; else batch_single_msg code !=
   SUCCESS -> FAILED; else tcache insert -> DEDUP if it was a duplicate, else
   SUCCESS.  Because batches complete in submission order and no frag's
   outcome is decided before the ones ahead of it, the verdict stream is the
   one the reference tile produces on the same frags.

   Each SUCCESS transaction also yields the frag the reference tile
   publishes (after_frag, fd_verify.c:102-133: payload, pad, fd_txn_t,
   payload_sz), built in an output arena at resolve time from the
   payload copy in the batch and the fd_txn_t trailer its parse left there
   (64 bytes per transaction, written by the host parse or -- GPU-parse
   mode -- the device's; a host parse only for the rare fd_txn_t longer
   than that).  Arena bytes are handed out by vtile_poll_frags in frag
   order and reclaimed as records are polled. */

typedef struct {
  unsigned long cookie;
  unsigned long tag;
  unsigned char const * pay;  /* zero-copy: the payload in the caller's (shared) memory */
  unsigned long slot_seq;   /* submission seq of its batch (pending)  */
  unsigned long arena_off;  /* its frag in the output arena            */
  unsigned      arena_len;  /* bytes reserved there (0: none)          */
  unsigned      txn_idx;    /* index in its batch                      */
  unsigned short frag_sz;   /* the frag's size (new_sz), 0: none       */
  signed char   verdict;
  unsigned char resolved;
} vrec_t;

struct fd_ed25519_hip_vtile {
  fd_ed25519_hip_pipe_t *   pipe;
  fd_ed25519_hip_tcache_t * tc;
  fd_ed25519_hip_slot_t *   open;       /* acquired, not yet submitted */
  unsigned long             open_seq;   /* seq the open slot will get   */
  unsigned long             batch_sigs;
  int                       gpu_parse;  /* FD_ED25519_HIP_VTILE_GPU_PARSE: raw payloads to the device */
  int                       trailer_only;   /* the arena holds each frag's trailer only (fd_txn_t, payload_sz):
                                               the verify service, whose tile keeps the payload */
  int                       err;        /* sticky failure: nothing more is staged or resolved */
  vrec_t *                  q;          /* circular FIFO of records */
  unsigned long             q_cap, q_head, q_cnt;
  unsigned long             resolved_head;  /* records [q_head, q_head+resolved_head) are resolved */
  unsigned char *           oa;         /* output arena: a ring of frags, [oa_head, oa_tail) cyclically */
  unsigned long             oa_cap, oa_head, oa_tail, oa_live;
  /* the verify service's waits (internal): while every slot is in flight
     the vtile polls the oldest batch instead of blocking in the runtime,
     calling idle between polls (heartbeats, link watch: nonzero aborts the
     wait with that code), and fails with FD_ED25519_HIP_ERR_TIMEOUT when
     the batch has not completed after hang_s (a hung GPU) */
  int                    (* idle)( void * );
  void *                    idle_ctx;
  double                    hang_s;
  /* zero-copy GPU-parse mode (the verify service, vt_frag_zc): payloads
     stay in the caller's page-locked memory (the txn link's dcache, base /
     size below) and the open batch DMAs them from there as up to two
     spans (the dcache is a ring: one wrap per batch at most) */
  int                       zero_copy;
  unsigned char const *     zc_base;
  unsigned char const *     zc_dev;       /* zc_base as the device sees it */
  unsigned long             zc_size;
  unsigned long             zc_start[ 2 ], zc_end[ 2 ];   /* the open batch's spans, offsets in the dcache */
  int                       zc_seg;                       /* spans in use: 0 (empty), 1 or 2 */
};

fd_ed25519_hip_vtile_t *
fd_ed25519_hip_vtile_new( int device, unsigned slot_cnt, unsigned long batch_sigs, unsigned long tcache_depth,
                          unsigned long tcache_map_cnt, int flags ) {
  fd_ed25519_hip_vtile_t * vt = (fd_ed25519_hip_vtile_t *)calloc( 1, sizeof(*vt) );
  if( !vt ) return NULL;
  /* a transaction stages up to 16 signatures into one batch: a smaller
     batch could not hold it (its signatures would run past the slot) */
  vt->batch_sigs = !batch_sigs ? 4096UL : batch_sigs<16UL ? 16UL : batch_sigs;
  vt->gpu_parse  = !!(flags & FD_ED25519_HIP_VTILE_GPU_PARSE);
  vt->pipe = fd_ed25519_hip_pipe_new( device, slot_cnt, vt->batch_sigs, vt->batch_sigs*FD_ED25519_HIP_TXN_MTU,
                                      vt->batch_sigs, flags & FD_ED25519_HIP_FLAG_CODES_PORTABLE );
  vt->tc   = fd_ed25519_hip_tcache_new( tcache_depth, tcache_map_cnt );
  vt->q_cap = 1024UL;
  vt->q = (vrec_t *)malloc( vt->q_cap*sizeof(vrec_t) );
  vt->oa_cap = 1UL<<20;
  vt->oa = (unsigned char *)malloc( vt->oa_cap );
  if( !vt->pipe || !vt->tc || !vt->q || !vt->oa ) {
    if( !vt->tc ) fd_ed25519_hip_private_set_error( "vtile_new: bad tcache geometry" );
    fd_ed25519_hip_vtile_delete( vt );
    return NULL;
  }
  /* touched now, not on the first frags (first-touch faults in the stream) */
  memset( vt->q, 0, vt->q_cap*sizeof(vrec_t) );
  memset( vt->oa, 0, vt->oa_cap );
  return vt;
}

void
fd_ed25519_hip_vtile_delete( fd_ed25519_hip_vtile_t * vt ) {
  if( !vt ) return;
  fd_ed25519_hip_pipe_delete( vt->pipe );
  fd_ed25519_hip_tcache_delete( vt->tc );
  free( vt->q );
  free( vt->oa );
  free( vt );
}

static vrec_t *
vq_at( fd_ed25519_hip_vtile_t * vt, unsigned long k ) {
  return &vt->q[ (vt->q_head + k) & (vt->q_cap - 1UL) ];   /* q_cap: a power of 2 */
}

static vrec_t *
vq_push( fd_ed25519_hip_vtile_t * vt ) {
  if( vt->q_cnt==vt->q_cap ) {
    unsigned long ncap = 2UL*vt->q_cap;
    vrec_t * nq = (vrec_t *)malloc( ncap*sizeof(vrec_t) );
    if( !nq ) {
      fd_ed25519_hip_private_set_error( "vtile: queue allocation failed" );
      vt->err = FD_ED25519_HIP_ERR_NOMEM;
      return NULL;
    }
    for( unsigned long k=0UL; k<vt->q_cnt; k++ ) nq[k] = *vq_at( vt, k );
    free( vt->q );
    vt->q = nq; vt->q_cap = ncap; vt->q_head = 0UL;
  }
  vrec_t * r = &vt->q[ (vt->q_head + vt->q_cnt) & (vt->q_cap - 1UL) ];
  vt->q_cnt++;
  memset( r, 0, sizeof(*r) );
  return r;
}

/* The output arena is a ring of frags in record order: live bytes run
   from oa_head to oa_tail, cyclically (oa_live tells a full ring from an
   empty one); a frag never straddles the end (the tail wraps to 0 when the
   end is short, the skipped bytes come free with the record before).  It
   grows -- frags copied in order to a new ring, offsets rebased -- only
   when full.  `need` bytes at a 64-byte aligned offset: */
static unsigned long
oa_reserve( fd_ed25519_hip_vtile_t * vt, unsigned long need ) {
  need = (need + 63UL) & ~63UL;   /* oa_commit's aligned length never exceeds it */
  if( !vt->oa_live ) vt->oa_head = vt->oa_tail = 0UL;
  if( vt->oa_tail>=vt->oa_head ) {                        /* free: [tail, cap) and [0, head) */
    if( vt->oa_cap - vt->oa_tail>=need ) return vt->oa_tail;
    if( vt->oa_head>need ) return 0UL;                    /* wrap */
  } else if( vt->oa_head - vt->oa_tail>need ) {           /* free: [tail, head) */
    return vt->oa_tail;
  }
  /* full: a ring twice as large (or more), the live frags copied over in
     record order */
  unsigned long ncap = 2UL*vt->oa_cap;
  while( ncap < 2UL*need ) ncap *= 2UL;
  unsigned char * n = (unsigned char *)malloc( ncap );
  if( !n ) {
    fd_ed25519_hip_private_set_error( "vtile: arena allocation failed" );
    vt->err = FD_ED25519_HIP_ERR_NOMEM;
    return ~0UL;
  }
  unsigned long pos = 0UL;
  for( unsigned long k=0UL; k<vt->q_cnt; k++ ) {
    vrec_t * r = vq_at( vt, k );
    if( !r->arena_len ) continue;
    memcpy( n + pos, vt->oa + r->arena_off, r->arena_len );
    r->arena_off = pos;
    pos += r->arena_len;
  }
  free( vt->oa );
  vt->oa = n; vt->oa_cap = ncap; vt->oa_head = 0UL; vt->oa_tail = pos;
  return pos;
}

static unsigned
oa_commit( fd_ed25519_hip_vtile_t * vt, unsigned long off, unsigned long used ) {
  unsigned long len = (used + 63UL) & ~63UL;
  vt->oa_tail = off + len;
  vt->oa_live++;
  return (unsigned)len;
}

/* advance resolved_head over the resolved prefix of the FIFO */
static void
vt_advance( fd_ed25519_hip_vtile_t * vt ) {
  while( vt->resolved_head<vt->q_cnt && vq_at( vt, vt->resolved_head )->resolved ) vt->resolved_head++;
}

/* resolve the records of a completed batch, in frag order (records ahead
   of them are resolved already: earlier batches completed first, parse
   failures at once) */
/* where record r's payload starts in its batch (the frag is built from it) */
static inline unsigned char const *
vt_payload( fd_ed25519_hip_vtile_t const * vt, fd_ed25519_hip_slot_t const * s, vrec_t const * r ) {
  unsigned long ti = r->txn_idx;
  if( vt->gpu_parse ) return s->msgs + s->msg_off[ ti ];
  unsigned long k = s->txn_first[ ti ];
  return s->msgs + s->msg_off[ k ] - ( 1UL + 64UL*s->txn_sig_cnt[ ti ] );
}

static void
vt_resolve( fd_ed25519_hip_vtile_t * vt, fd_ed25519_hip_slot_t * s ) {
  for( unsigned long k=vt->resolved_head; k<vt->q_cnt; k++ ) {
    vrec_t * r = vq_at( vt, k );
    if( r->resolved ) continue;
    if( r->slot_seq!=s->seq ) break;
    /* the payload a few records ahead is read into the cache while this
       one resolves (the batch's bytes were staged a few batches ago) */
    if( vt->gpu_parse && k+4UL<vt->q_cnt ) {
      vrec_t const * a = vq_at( vt, k+4UL );
      if( !a->resolved && a->slot_seq==s->seq && s->txn_sig_cnt[ a->txn_idx ]-1U<16U ) {
        if( !vt->trailer_only ) {   /* the frag is built from the payload (a service sends the trailer only) */
          unsigned char const * pp = vt_payload( vt, s, a );
          for( unsigned long l=0UL; l<448UL; l+=64UL ) __builtin_prefetch( pp + l, 0, 3 );
        }
        __builtin_prefetch( s->txn_trailer + 64UL*a->txn_idx, 0, 3 );
      }
    }
    int code = s->txn_out[ r->txn_idx ];
    int v;
    if( code==FD_ED25519_HIP_TXN_CODE_PARSE_FAILED )          v = FD_ED25519_HIP_TXN_PARSE_FAILED;  /* device parse */
    else if( fd_ed25519_hip_tcache_query( vt->tc, r->tag ) )  v = FD_ED25519_HIP_TXN_VERIFY_DEDUP;
    else if( code!=FD_ED25519_SUCCESS )                       v = FD_ED25519_HIP_TXN_VERIFY_FAILED;
    else if( fd_ed25519_hip_tcache_insert( vt->tc, r->tag ) ) v = FD_ED25519_HIP_TXN_VERIFY_DEDUP;
    else                                                      v = FD_ED25519_HIP_TXN_VERIFY_SUCCESS;
    r->verdict  = (signed char)v;
    r->resolved = 1;
    if( v!=FD_ED25519_HIP_TXN_VERIFY_SUCCESS ) continue;   /* filtered: not published */
    if( !vt->gpu_parse ) continue;                         /* its frag was built with the frag (vtile_frag) */
    {
      /* the published frag from the payload in the slot and the fd_txn_t
         trailer its parse left in the slot (the device's in GPU-parse
         mode; a host parse when it exceeds the 64-byte trailer slot) */
      unsigned long ti = r->txn_idx, poff, psz;
      if( vt->gpu_parse ) {
        poff = s->msg_off[ ti ];
        psz  = s->msg_sz [ ti ];
      } else {   /* the signatures' message pointer, back over the signatures (signature_off is 1) */
        unsigned long k = s->txn_first[ ti ], mo = 1UL + 64UL*s->txn_sig_cnt[ ti ];
        poff = s->msg_off[ k ] - mo;
        psz  = s->msg_sz [ k ] + mo;
      }
      unsigned char const * pay = vt->zero_copy ? r->pay : s->msgs + poff;
      unsigned char const * tr  = s->txn_trailer + 64UL*ti;
      unsigned long foot = FD_ED25519_HIP_TXN_FOOTPRINT( (unsigned long)tr[18] | ((unsigned long)tr[19]<<8),
                                                         (unsigned long)tr[14] );
      unsigned long toff = vt->trailer_only ? 0UL : (psz + 1UL) & ~1UL;
      unsigned long aoff = oa_reserve( vt, toff + FD_ED25519_HIP_TXN_MAX_SZ + 2UL );
      if( aoff==~0UL ) return;   /* vt->err is set: nothing more resolves */
      unsigned char * o = vt->oa + aoff;
      unsigned long fsz;
      if( vt->trailer_only ) {
        if( foot>64UL ) {
          /* an fd_txn_t longer than the device's 64-byte trailer slot: parsed
             here, from a private copy (zero-copy: the payload is in memory
             another process shares) */
          unsigned char priv[ FD_ED25519_HIP_TXN_MTU ];
          fd_ed25519_hip_txn_t t;
          if( vt->zero_copy ) { memcpy( priv, pay, psz ); pay = priv; }
          foot = fd_txn_core_parse( pay, psz, &t, o, FD_ED25519_HIP_TXN_MAX_SZ );
          if( !foot ) { r->verdict = (signed char)FD_ED25519_HIP_TXN_PARSE_FAILED; continue; }   /* changed under us */
        } else {
          memcpy( o, tr, foot );
        }
        o[ foot ] = (unsigned char)psz; o[ foot + 1 ] = (unsigned char)(psz >> 8);
        fsz = foot + 2UL;
      } else if( foot<=64UL ) {
        memcpy( o, pay, psz );
        if( toff>psz ) o[ psz ] = 0;
        memcpy( o + toff, tr, foot );
        o[ toff + foot ] = (unsigned char)psz; o[ toff + foot + 1 ] = (unsigned char)(psz >> 8);
        fsz = toff + foot + 2UL;
      } else {
        fd_ed25519_hip_txn_t t;
        fsz = txn_frag_core( pay, psz, o, &t );
      }
      r->arena_off = aoff;
      r->arena_len = oa_commit( vt, aoff, fsz );
      r->frag_sz   = (unsigned short)fsz;
    }
  }
  vt_advance( vt );
}

#ifdef FD_ED25519_HIP_AB_SERVICE_PROFILE
static __thread unsigned long long vt_wait_cycles, vt_resolve_cycles, vt_blocks;   /* A/B build only */
static __thread unsigned long long vt_submit_cycles, vt_submits, vt_rtt_n;
static __thread double             vt_rtt_s, vt_rtt_max_s;
#endif

static int
vt_drain_one( fd_ed25519_hip_vtile_t * vt, int wait ) {
  if( vt->err ) return 0;
#ifdef FD_ED25519_HIP_AB_SERVICE_PROFILE
  unsigned long long w0 = __rdtsc();
#endif
  fd_ed25519_hip_slot_t * s = fd_ed25519_hip_pipe_poll( vt->pipe, wait );
#ifdef FD_ED25519_HIP_AB_SERVICE_PROFILE
  unsigned long long w1 = __rdtsc();
  if( wait ) { vt_wait_cycles += w1 - w0; vt_blocks++; }
#endif
  if( !s ) {
    if( fd_ed25519_hip_pipe_error( vt->pipe ) ) vt->err = fd_ed25519_hip_pipe_error( vt->pipe );
    return 0;
  }
#ifdef FD_ED25519_HIP_AB_SERVICE_PROFILE
  { double rt = s->t_done - s->t_submit; vt_rtt_s += rt; vt_rtt_n++; if( rt>vt_rtt_max_s ) vt_rtt_max_s = rt; }
#endif
  vt_resolve( vt, s );
#ifdef FD_ED25519_HIP_AB_STAGE_TRACE
  if( stage_cnt<STAGE_TRACE_MAX ) {
    pipe_slot_t const * ps = (pipe_slot_t const *)s;
    stage_rec_t * r = &stage_rec[ stage_cnt++ ];
    r->t_submit = s->t_submit; r->t_enq = ps->t_enq; r->t_done = s->t_done; r->t_resolved = now_s();
    r->seq = (double)s->seq; r->sig_cnt = (double)s->sig_cnt; r->txn_cnt = (double)s->txn_cnt;
    r->in_flight = (double)ps->in_flight0;
  }
#endif
  fd_ed25519_hip_pipe_release( vt->pipe, s );
#ifdef FD_ED25519_HIP_AB_SERVICE_PROFILE
  vt_resolve_cycles += __rdtsc() - w1;
#endif
  return 1;
}

static int
vt_submit_open( fd_ed25519_hip_vtile_t * vt ) {
  fd_ed25519_hip_slot_t * s = vt->open;
  if( !s || !s->txn_cnt ) return 0;
  if( vt->zero_copy ) {
    pipe_slot_t * ps = (pipe_slot_t *)s;
    ps->ext_counts = 1;
    for( int g=0; g<vt->zc_seg; g++ ) {
      ps->ext_src[ g ] = vt->zc_base + vt->zc_start[ g ];
      ps->ext_dev[ g ] = vt->zc_dev  + vt->zc_start[ g ];
      ps->ext_len[ g ] = vt->zc_end[ g ] - vt->zc_start[ g ];
    }
    vt->zc_seg = 0;
  }
#ifdef FD_ED25519_HIP_AB_SERVICE_PROFILE
  unsigned long long sc0 = __rdtsc();
#endif
  int err = vt->gpu_parse ? fd_ed25519_hip_pipe_submit_txns( vt->pipe, s, s->txn_cnt, s->msg_bytes )
                          : fd_ed25519_hip_pipe_submit( vt->pipe, s, s->sig_cnt, s->msg_bytes, s->txn_cnt );
#ifdef FD_ED25519_HIP_AB_SERVICE_PROFILE
  vt_submit_cycles += __rdtsc() - sc0; vt_submits++;
#endif
  if( err ) {   /* a launch failed: the batch's transactions have no verdicts, and the vtile stops */
    vt->err = err;
    return 0;
  }
  vt->open = NULL;
  return 1;
}

static inline void spin_pause( void );

/* every slot in flight: wait for the oldest batch (1: one completed and
   resolved, 0: vt->err is set) -- blocking in the runtime, or, with an idle
   hook (the verify service), polling it with the hook between polls and a
   bound on how long a batch may take */
static int
vt_wait_oldest( fd_ed25519_hip_vtile_t * vt ) {
  if( !vt->idle ) return vt_drain_one( vt, 1 );
  double t0 = now_s();
  for( unsigned long spin=1UL;; spin++ ) {
    if( vt_drain_one( vt, 0 ) ) return 1;
    if( vt->err ) return 0;
    if( !(spin & 63UL) ) {
      int r = vt->idle( vt->idle_ctx );
      if( r ) { vt->err = r; return 0; }
      if( vt->hang_s>0.0 && now_s() - t0>vt->hang_s ) {
        char buf[ 128 ];
        snprintf( buf, sizeof(buf), "vtile: batch %lu did not complete within %.1f s (GPU hang)",
                  vt->pipe->seq - fd_ed25519_hip_pipe_in_flight( vt->pipe ), vt->hang_s );
        fd_ed25519_hip_private_set_error( buf );
        vt->err = FD_ED25519_HIP_ERR_TIMEOUT;
        return 0;
      }
    }
    spin_pause();
  }
}

/* 0, or the vtile's sticky error (the open slot is then NULL) */
static int
vt_open( fd_ed25519_hip_vtile_t * vt ) {
  if( vt->err ) return vt->err;
  if( vt->open ) return 0;
  for( ;; ) {
    vt->open = fd_ed25519_hip_pipe_acquire( vt->pipe );  /* counts start at 0 */
    if( vt->open ) break;
    if( !vt_wait_oldest( vt ) && vt->err ) return vt->err;
  }
  vt->open_seq = vt->pipe->seq;
  return 0;
}

/* GPU-parse mode: the payload goes to the device as is; the host reads
   only byte 0 (the signature count, to reserve slots) and bytes 1..8 (the
   dedup tag, valid whenever the device's parse accepts the payload). */
static int
vt_frag_raw( fd_ed25519_hip_vtile_t * vt, unsigned char const * payload, unsigned long payload_sz,
             unsigned long cookie ) {
  if( vt->err ) return vt->err;
  if( !payload_sz || payload_sz>FD_ED25519_HIP_TXN_MTU ) {   /* fd_txn_parse rejects these before reading */
    vrec_t * r = vq_push( vt );
    if( !r ) return vt->err;
    r->cookie = cookie; r->verdict = FD_ED25519_HIP_TXN_PARSE_FAILED; r->resolved = 1;
    vt_advance( vt );
    return 0;
  }
  unsigned long c = payload[0], nsig = (c>=1UL && c<=16UL) ? c : 0UL;
  if( vt_open( vt ) ) return vt->err;
  fd_ed25519_hip_slot_t * s = vt->open;
  if( s->txn_cnt && ( s->sig_cnt+nsig>s->sig_cap || s->txn_cnt+1UL>s->txn_cap ||
                      STAGE_ALIGN( s->msg_bytes )+payload_sz>s->msg_cap ) ) {
    vt_submit_open( vt );
    if( vt_open( vt ) ) return vt->err;
    s = vt->open;
  }
  unsigned long ti = s->txn_cnt++, poff = STAGE_ALIGN( s->msg_bytes );
  memcpy( s->msgs + poff, payload, payload_sz );
  s->msg_off[ ti ] = poff;
  s->msg_sz [ ti ] = (unsigned int)payload_sz;
  s->msg_bytes = poff + payload_sz;
  s->sig_cnt   += nsig;
  vrec_t * r = vq_push( vt );
  if( !r ) return vt->err;
  r->cookie = cookie;
  if( payload_sz>=9UL ) memcpy( &r->tag, payload + 1, 8UL );
  r->slot_seq = vt->open_seq;
  r->txn_idx  = (unsigned)ti;
  if( s->sig_cnt>=s->sig_cap || s->txn_cnt>=s->txn_cap ) vt_submit_open( vt );
  return 1;
}

/* Zero-copy GPU-parse mode (the verify service): the payload is read in
   place in the caller's page-locked memory [zc_base, zc_base+zc_size) --
   byte 0 (the signature count, to reserve slots) and bytes 1..8 (the dedup
   tag) only -- and DMA'd to the device with its batch's span at submit;
   the device parses it (fd_txn_parse's acceptance) exactly as in GPU-parse
   mode.  The bytes must stay in place until the frag's verdict is taken
   (the verify tile's txn link guarantees it: a room is reused only after
   its frag is answered, integration/fd_verify_hip.c).  Payloads must come
   in the order they lie in the memory ring (a wrap to its start allowed);
   a payload out of that order closes the batch. */
static int
vt_frag_zc( fd_ed25519_hip_vtile_t * vt, unsigned char const * payload, unsigned long payload_sz,
            unsigned long cookie ) {
  if( vt->err ) return vt->err;
  if( !payload_sz || payload_sz>FD_ED25519_HIP_TXN_MTU ) {   /* fd_txn_parse rejects these before reading */
    vrec_t * r = vq_push( vt );
    if( !r ) return vt->err;
    r->cookie = cookie; r->verdict = FD_ED25519_HIP_TXN_PARSE_FAILED; r->resolved = 1;
    vt_advance( vt );
    return 0;
  }
  unsigned long o = (unsigned long)( payload - vt->zc_base ), e = o + payload_sz;
  if( payload<vt->zc_base || e>vt->zc_size ) { vt->err = FD_ED25519_HIP_ERR_INVAL; return vt->err; }
  unsigned long c = payload[0], nsig = (c>=1UL && c<=16UL) ? c : 0UL;
#ifdef FD_ED25519_HIP_HOST_FAULT
  /* test build only (tests/test_gpu_service_fault.py): with
     $FD_ED25519_HIP_FAULT_ZC_COUNT=k every 5th frag's signature count reads
     as k here, as if the tile had rewritten byte 0 of the room between this
     read and the batch's DMA (and back): the device's parse must reject
     the transaction instead of staging k signatures from it */
  {
    static unsigned long fault_zc_n;
    char const * f = getenv( "FD_ED25519_HIP_FAULT_ZC_COUNT" );
    if( f && *f && (fault_zc_n++ % 5UL)==2UL ) { c = strtoul( f, NULL, 10 ); nsig = (c>=1UL && c<=16UL) ? c : 0UL; }
  }
#endif
  for( int pass=0;; pass++ ) {
    if( vt_open( vt ) ) return vt->err;
    fd_ed25519_hip_slot_t * s = vt->open;
    /* where this payload goes in the batch's spans */
    int seg = -1;
    unsigned long len0 = vt->zc_seg>=1 ? vt->zc_end[0] - vt->zc_start[0] : 0UL;
    unsigned long len1 = vt->zc_seg>=2 ? vt->zc_end[1] - vt->zc_start[1] : 0UL;
    if( !vt->zc_seg ) seg = 0;
    else if( o>=vt->zc_end[ vt->zc_seg-1 ] && o - vt->zc_end[ vt->zc_seg-1 ]<64UL ) seg = vt->zc_seg-1;   /* the next room */
    else if( vt->zc_seg==1 && e<=vt->zc_start[0] ) seg = 1;                                           /* the ring wrapped */
    /* the batch's payload bytes with this one: span 0, then span 1 from a
       64-byte boundary (slot_h2d) */
    unsigned long need = seg<0 ? 0UL : !vt->zc_seg ? payload_sz : seg==vt->zc_seg ? STAGE_ALIGN( len0 ) + payload_sz :
                         seg==0 ? e - vt->zc_start[0] : STAGE_ALIGN( len0 ) + ( e - vt->zc_start[1] );
    (void)len1;
    int fits = seg>=0 && ( !s->txn_cnt || ( s->sig_cnt+nsig<=s->sig_cap && s->txn_cnt+1UL<=s->txn_cap &&
                                            need<=s->msg_cap ) );
    if( !fits ) {
      if( pass || !s->txn_cnt ) { vt->err = FD_ED25519_HIP_ERR_INVAL; return vt->err; }
      vt_submit_open( vt );   /* a full batch, or a payload out of ring order: a new batch */
      continue;
    }
    unsigned long moff;
    if( !vt->zc_seg ) { vt->zc_start[0] = o; vt->zc_end[0] = e; vt->zc_seg = 1; moff = 0UL; }
    else if( seg==vt->zc_seg ) { vt->zc_start[1] = o; vt->zc_end[1] = e; vt->zc_seg = 2; moff = STAGE_ALIGN( len0 ); }
    else { moff = ( seg ? STAGE_ALIGN( len0 ) + ( o - vt->zc_start[1] ) : o - vt->zc_start[0] ); vt->zc_end[ seg ] = e; }
    unsigned long ti = s->txn_cnt++;
    s->msg_off    [ ti ] = moff;
    s->msg_sz     [ ti ] = (unsigned int)payload_sz;
    s->txn_sig_cnt[ ti ] = (unsigned int)c;
    s->msg_bytes = vt->zc_seg==2 ? STAGE_ALIGN( vt->zc_end[0] - vt->zc_start[0] ) + ( vt->zc_end[1] - vt->zc_start[1] )
                                 : vt->zc_end[0] - vt->zc_start[0];
    s->sig_cnt  += nsig;
    vrec_t * r = vq_push( vt );
    if( !r ) return vt->err;
    r->cookie = cookie;
    if( payload_sz>=9UL ) memcpy( &r->tag, payload + 1, 8UL );
    r->pay      = payload;
    r->slot_seq = vt->open_seq;
    r->txn_idx  = (unsigned)ti;
    if( s->sig_cnt>=s->sig_cap || s->txn_cnt>=s->txn_cap ) vt_submit_open( vt );
    return 1;
  }
}

int
fd_ed25519_hip_vtile_frag( fd_ed25519_hip_vtile_t * vt, unsigned char const * payload, unsigned long payload_sz,
                           unsigned long cookie ) {
  if( vt->gpu_parse ) return vt_frag_raw( vt, payload, payload_sz, cookie );
  if( vt->err ) return vt->err;
  /* during_frag + after_frag: the payload goes into the open batch whole,
     and the frag the tile publishes if the transaction succeeds (payload,
     pad, fd_txn_t, payload_sz) is built now, while the payload is in the
     cache, into the output arena: the parse writes fd_txn_t there directly.
     Resolving a batch then only decides verdicts (a frag whose transaction
     fails stays unpublished and comes free in record order). */
  if( vt_open( vt ) ) return vt->err;
  fd_ed25519_hip_slot_t * s = vt->open;
  unsigned long aoff = oa_reserve( vt, ( vt->trailer_only ? 0UL : (payload_sz + 1UL) & ~1UL ) +
                                       FD_ED25519_HIP_TXN_MAX_SZ + 2UL );
  if( aoff==~0UL ) return vt->err;
  fd_ed25519_hip_txn_t t;
  unsigned long fsz;
  if( vt->trailer_only ) {   /* the trailer only: fd_txn_t, then payload_sz */
    unsigned char * o = vt->oa + aoff;
    unsigned long foot = payload_sz>FD_ED25519_HIP_TXN_MTU ? 0UL :
                         fd_txn_core_parse( payload, payload_sz, &t, o, FD_ED25519_HIP_TXN_MAX_SZ );
    if( foot ) { o[ foot ] = (unsigned char)payload_sz; o[ foot + 1 ] = (unsigned char)(payload_sz >> 8); }
    fsz = foot ? foot + 2UL : 0UL;
  } else {
    fsz = txn_frag_core( payload, payload_sz, vt->oa + aoff, &t );
  }
  if( !fsz ) {
    vrec_t * r = vq_push( vt );
    if( !r ) return vt->err;
    r->cookie = cookie; r->verdict = FD_ED25519_HIP_TXN_PARSE_FAILED; r->resolved = 1;
    vt_advance( vt );
    return 0;
  }
  unsigned long nsig = (t.signature_cnt>=1U && t.signature_cnt<=16U) ? t.signature_cnt : 0UL;
  if( s->txn_cnt && ( s->sig_cnt+nsig>s->sig_cap || s->txn_cnt+1UL>s->txn_cap ||
                      STAGE_ALIGN( s->msg_bytes )+payload_sz>s->msg_cap ) ) {
    vt_submit_open( vt );
    if( vt_open( vt ) ) return vt->err;
    s = vt->open;
  }
  unsigned long poff   = STAGE_ALIGN( s->msg_bytes );
  unsigned long moff   = poff + t.message_off;
  unsigned long msg_sz = payload_sz - t.message_off;
  memcpy( s->msgs + poff, payload, payload_sz );
  s->msg_bytes = poff + payload_sz;
  unsigned long first = s->sig_cnt;
  for( unsigned long j=0UL; j<nsig; j++ ) {
    unsigned long k = first + j;
    s->msg_off[ k ] = moff;
    s->msg_sz [ k ] = (unsigned int)msg_sz;
    memcpy( s->sigs + 64UL*k, payload + t.signature_off + 64UL*j, 64UL );
    memcpy( s->pubs + 32UL*k, payload + t.acct_addr_off + 32UL*j, 32UL );
  }
  s->sig_cnt += nsig;
  unsigned long ti = s->txn_cnt++;
  s->txn_first  [ ti ] = (unsigned int)first;
  s->txn_sig_cnt[ ti ] = t.signature_cnt;   /* 17..127 -> ERR_SIG, no signatures staged */
  vrec_t * r = vq_push( vt );
  if( !r ) return vt->err;
  r->cookie    = cookie;
  memcpy( &r->tag, payload + t.signature_off, 8UL );  /* ha_dedup_tag, fd_verify.h:65 */
  r->slot_seq = vt->open_seq;
  r->txn_idx  = (unsigned)ti;
  r->arena_off = aoff;
  r->arena_len = oa_commit( vt, aoff, fsz );
  r->frag_sz   = (unsigned short)fsz;
  if( s->sig_cnt>=s->sig_cap || s->txn_cnt>=s->txn_cap ) vt_submit_open( vt );
  return 1;
}

int
fd_ed25519_hip_vtile_flush( fd_ed25519_hip_vtile_t * vt, int wait ) {
  (void)wait;
  return vt_submit_open( vt );
}

unsigned long
fd_ed25519_hip_vtile_poll_frags( fd_ed25519_hip_vtile_t * vt, int wait, unsigned long max, unsigned long * cookie,
                                 signed char * verdict, unsigned long * tag, unsigned long * frag_off,
                                 unsigned long * frag_sz, unsigned char * frag_buf, unsigned long frag_buf_sz ) {
  while( vt_drain_one( vt, 0 ) ) {}
  if( wait && !vt->resolved_head && vt->q_cnt && fd_ed25519_hip_pipe_in_flight( vt->pipe ) ) vt_drain_one( vt, 1 );
  unsigned long n = 0UL, bo = 0UL;
  while( n<max && vt->resolved_head ) {
    vrec_t * r = vq_at( vt, 0UL );
    unsigned long fsz = r->verdict==FD_ED25519_HIP_TXN_VERIFY_SUCCESS ? r->frag_sz : 0UL;
    if( frag_buf && fsz ) {
      if( bo + fsz > frag_buf_sz ) break;   /* the caller's buffer is full */
      memcpy( frag_buf + bo, vt->oa + r->arena_off, fsz );
    }
    if( frag_off ) frag_off[ n ] = bo;
    if( frag_sz  ) frag_sz [ n ] = fsz;
    if( frag_buf && fsz ) bo += (fsz + 63UL) & ~63UL;
    if( cookie  ) cookie [ n ] = r->cookie;
    if( verdict ) verdict[ n ] = r->verdict;
    if( tag     ) tag    [ n ] = r->tag;
    if( r->arena_len ) {   /* arena bytes come free in record order */
      vt->oa_head = r->arena_off + r->arena_len;
      vt->oa_live--;
    }
    n++;
    vt->q_head = (vt->q_head+1UL) & (vt->q_cap - 1UL);
    vt->q_cnt--;
    vt->resolved_head--;
  }
  return n;
}

/* The service's path (vsvc_pass): resolved records are published
   straight from the output arena, without poll_frags' copy into a caller
   buffer.  vt_head returns the oldest record once it is resolved (its frag,
   for SUCCESS, at vt->oa + arena_off, frag_sz bytes), vt_pop retires it. */
static vrec_t const *
vt_head( fd_ed25519_hip_vtile_t * vt ) {
  return vt->resolved_head ? vq_at( vt, 0UL ) : NULL;
}

static void
vt_pop( fd_ed25519_hip_vtile_t * vt ) {
  vrec_t const * r = vq_at( vt, 0UL );
  if( r->arena_len ) {   /* arena bytes come free in record order */
    vt->oa_head = r->arena_off + r->arena_len;
    vt->oa_live--;
  }
  vt->q_head = (vt->q_head+1UL) & (vt->q_cap - 1UL);
  vt->q_cnt--;
  vt->resolved_head--;
}

unsigned long
fd_ed25519_hip_vtile_poll( fd_ed25519_hip_vtile_t * vt, int wait, unsigned long max, unsigned long * cookie,
                           signed char * verdict, unsigned long * tag ) {
  return fd_ed25519_hip_vtile_poll_frags( vt, wait, max, cookie, verdict, tag, NULL, NULL, NULL, 0UL );
}

unsigned long
fd_ed25519_hip_vtile_pending( fd_ed25519_hip_vtile_t const * vt ) {
  return vt->q_cnt;
}

int
fd_ed25519_hip_vtile_error( fd_ed25519_hip_vtile_t const * vt ) {
  return vt->err;
}

unsigned long
fd_ed25519_hip_vtile_device_bytes( fd_ed25519_hip_vtile_t const * vt ) {
  return fd_ed25519_hip_pipe_device_bytes( vt->pipe );
}

/* ======================================================================
   ring: a single-producer single-consumer tango-style mcache / dcache.
   The frag metadata is fd_frag_meta_t's layout (src/tango/fd_tango_base.h:
   123-203, 32 bytes: seq, sig, chunk, sz, ctl, tsorig, tspub); the producer
   invalidates a line (seq-1), writes the body, then publishes seq with
   release order; the consumer reads seq with acquire order, copies the
   payload, and re-reads seq to detect being overrun.  Payloads live in a
   dcache of 64-byte chunks, allocated compactly with wrap-around. */

typedef struct {
  _Atomic uint64_t seq;
  uint64_t         sig;
  uint32_t         chunk;
  uint16_t         sz;
  uint16_t         ctl;
  uint32_t         tsorig;
  uint32_t         tspub;
} ring_meta_t;

typedef struct {
  ring_meta_t *   mcache;
  unsigned long   depth;
  unsigned char * dcache;
  unsigned long   chunk_cnt;
} ring_t;

#define RING_CHUNK 64UL
#define RING_MTU_CHUNKS ((FD_ED25519_HIP_TXN_MTU + RING_CHUNK - 1UL) / RING_CHUNK)

typedef struct {
  ring_t *              ring;
  unsigned char const * payloads;
  unsigned long const * off;
  unsigned int const *  sz;
  unsigned long         n;
  double                rate;
  double *              t_pub;
  _Atomic int           go;
  _Atomic int           stop;       /* the consumer gave up (its vtile failed) */
  _Atomic uint64_t      consumed;   /* frags the consumer has taken (credits) */
  double                t0;
  int                   cpu;        /* pinned to this CPU (-1: not pinned) */
} producer_t;

/* CPUs for latency_run's producer and tile threads (-1: unpinned):
   fd_ed25519_hip_latency_set_cpus */
static int lat_cpu_prod = -1, lat_cpu_tile = -1;

static int
pin_self( int cpu ) {
  if( cpu<0 ) return 0;
  cpu_set_t set;
  CPU_ZERO( &set );
  CPU_SET( cpu, &set );
  return pthread_setaffinity_np( pthread_self(), sizeof(set), &set );
}

int
fd_ed25519_hip_latency_set_cpus( int producer_cpu, int tile_cpu ) {
  if( producer_cpu>=CPU_SETSIZE || tile_cpu>=CPU_SETSIZE || ( producer_cpu>=0 && producer_cpu==tile_cpu ) )
    return FD_ED25519_HIP_ERR_INVAL;
  lat_cpu_prod = producer_cpu < 0 ? -1 : producer_cpu;
  lat_cpu_tile = tile_cpu < 0 ? -1 : tile_cpu;
  return FD_ED25519_HIP_OK;
}

static void *
producer_main( void * arg ) {
  producer_t * pr = (producer_t *)arg;
  ring_t * rg = pr->ring;
  pin_self( pr->cpu );
  while( !atomic_load_explicit( &pr->go, memory_order_acquire ) ) {}
  unsigned long chunk = 0UL;
  double t0 = now_s();
  pr->t0 = t0;
  for( unsigned long i=0UL; i<pr->n; i++ ) {
    /* the time frag i is due: latency counts from here, so time a frag
       waits for credits is part of it (no coordinated omission) */
    double due = t0;
    if( pr->rate>0.0 ) {
      due = t0 + (double)i / pr->rate;
      while( now_s()<due ) {}
    } else {
      due = now_s();
    }
    while( i - atomic_load_explicit( &pr->consumed, memory_order_acquire ) >= rg->depth ) {
      if( atomic_load_explicit( &pr->stop, memory_order_relaxed ) ) return NULL;
    }
    unsigned long sz = pr->sz[ i ];
    unsigned long nch = (sz + RING_CHUNK - 1UL) / RING_CHUNK;
    if( chunk + RING_MTU_CHUNKS > rg->chunk_cnt ) chunk = 0UL;   /* compact wrap */
    ring_meta_t * m = &rg->mcache[ i & (rg->depth-1UL) ];
    atomic_store_explicit( &m->seq, i-1UL, memory_order_relaxed );
    atomic_thread_fence( memory_order_release );
    memcpy( rg->dcache + chunk*RING_CHUNK, pr->payloads + pr->off[ i ], sz );
    m->sig = i; m->chunk = (uint32_t)chunk; m->sz = (uint16_t)sz; m->ctl = 0; m->tsorig = 0; m->tspub = 0;
    pr->t_pub[ i ] = due;
    atomic_store_explicit( &m->seq, i, memory_order_release );
#ifdef FD_ED25519_HIP_AB_STAGE_TRACE
    if( stage_frag_pub ) { stage_frag_pub[ i ] = now_s(); stage_frag_due[ i ] = due; }
#endif
    chunk += nch;
  }
  return NULL;
}

static int
latency_run( int device, unsigned slot_cnt, unsigned long batch_sigs, unsigned char const * payloads,
             unsigned long const * payload_off, unsigned int const * payload_sz, unsigned long txn_cnt,
             double offered_txn_per_s, unsigned long ring_depth, int flags, double * lat_s, signed char * verdict,
             fd_ed25519_hip_latency_result_t * res, int cpu_prod );

/* One tile: the calling thread is the tile, pinned for the run when
   fd_ed25519_hip_latency_set_cpus named a CPU (its affinity restored after). */
int
fd_ed25519_hip_latency_run( int device, unsigned slot_cnt, unsigned long batch_sigs,
                            unsigned char const * payloads, unsigned long const * payload_off,
                            unsigned int const * payload_sz, unsigned long txn_cnt, double offered_txn_per_s,
                            unsigned long ring_depth, int flags, double * lat_s, signed char * verdict,
                            fd_ed25519_hip_latency_result_t * res ) {
  cpu_set_t saved;
  int restore = lat_cpu_tile>=0 && !pthread_getaffinity_np( pthread_self(), sizeof(saved), &saved );
  if( restore && pin_self( lat_cpu_tile ) ) restore = 0;
  int err = latency_run( device, slot_cnt, batch_sigs, payloads, payload_off, payload_sz, txn_cnt, offered_txn_per_s,
                         ring_depth, flags, lat_s, verdict, res, lat_cpu_prod );
  if( restore ) pthread_setaffinity_np( pthread_self(), sizeof(saved), &saved );
  return err;
}

static int
latency_run( int device, unsigned slot_cnt, unsigned long batch_sigs, unsigned char const * payloads,
             unsigned long const * payload_off, unsigned int const * payload_sz, unsigned long txn_cnt,
             double offered_txn_per_s, unsigned long ring_depth, int flags, double * lat_s, signed char * verdict,
             fd_ed25519_hip_latency_result_t * res, int cpu_prod ) {
  if( !txn_cnt || !ring_depth || (ring_depth & (ring_depth-1UL)) || !lat_s || !verdict || !res )
    return FD_ED25519_HIP_ERR_INVAL;
  for( unsigned long i=0UL; i<txn_cnt; i++ )
    if( payload_sz[ i ]>FD_ED25519_HIP_TXN_MTU ) return FD_ED25519_HIP_ERR_INVAL;
  memset( res, 0, sizeof(*res) );
  fd_ed25519_hip_vtile_t * vt = fd_ed25519_hip_vtile_new( device, slot_cnt, batch_sigs, 16UL, 64UL, flags );
  if( !vt ) return FD_ED25519_HIP_ERR_INVAL;
  ring_t rg;
  rg.depth     = ring_depth;
  rg.chunk_cnt = (ring_depth + 2UL) * RING_MTU_CHUNKS;
  rg.mcache    = (ring_meta_t *)aligned_alloc( 64, ring_depth*sizeof(ring_meta_t) );
  rg.dcache    = (unsigned char *)aligned_alloc( 64, rg.chunk_cnt*RING_CHUNK );
  double * t_pub = (double *)malloc( txn_cnt*sizeof(double) );
  unsigned long * ck = (unsigned long *)malloc( 4096UL*sizeof(unsigned long) );
  signed char *   vd = (signed char *)malloc( 4096UL );
  unsigned char * buf = (unsigned char *)malloc( FD_ED25519_HIP_TXN_MTU );
  if( !rg.mcache || !rg.dcache || !t_pub || !ck || !vd || !buf ) {
    free( rg.mcache ); free( rg.dcache ); free( t_pub ); free( ck ); free( vd ); free( buf );
    fd_ed25519_hip_vtile_delete( vt );
    return FD_ED25519_HIP_ERR_NOMEM;
  }
  for( unsigned long k=0UL; k<ring_depth; k++ ) atomic_store( &rg.mcache[k].seq, (uint64_t)(k - ring_depth) );
  /* every page the timed run writes is touched now: a first-touch fault
     (a huge page zeroed, or compaction on a freshly started host) inside
     the run would stall the producer or the tile for milliseconds and show
     up as latency */
  memset( rg.dcache, 0, rg.chunk_cnt*RING_CHUNK );
  memset( t_pub, 0, txn_cnt*sizeof(double) );
  memset( ck, 0, 4096UL*sizeof(unsigned long) );
  memset( vd, 0, 4096UL );
  for( unsigned long i=0UL; i<txn_cnt; i++ ) { lat_s[ i ] = -1.0; verdict[ i ] = 0; }

  producer_t pr;
  memset( &pr, 0, sizeof(pr) );
  pr.ring = &rg; pr.payloads = payloads; pr.off = payload_off; pr.sz = payload_sz; pr.n = txn_cnt;
  pr.rate = offered_txn_per_s; pr.t_pub = t_pub; pr.cpu = cpu_prod;
  pthread_t th;
  if( pthread_create( &th, NULL, producer_main, &pr ) ) {
    free( rg.mcache ); free( rg.dcache ); free( t_pub ); free( ck ); free( vd ); free( buf );
    fd_ed25519_hip_vtile_delete( vt );
    return FD_ED25519_HIP_ERR_NOMEM;
  }
  atomic_store_explicit( &pr.go, 1, memory_order_release );

  unsigned long next = 0UL, done = 0UL, sigs = 0UL;
  unsigned long batches0 = 0UL;
  int err = 0;
  while( done<txn_cnt ) {
    if( (err = fd_ed25519_hip_vtile_error( vt )) ) {   /* the GPU failed: stop the producer, report */
      atomic_store_explicit( &pr.stop, 1, memory_order_release );
      break;
    }
    /* pull every frag that is ready (after_frag) */
    int pulled = 0;
    while( next<txn_cnt ) {
      ring_meta_t * m = &rg.mcache[ next & (ring_depth-1UL) ];
      uint64_t s0 = atomic_load_explicit( &m->seq, memory_order_acquire );
      if( (int64_t)(s0 - next)<0 ) break;                 /* not yet published */
      if( s0!=next ) { res->ring_overruns++; verdict[ next ] = FD_ED25519_HIP_TXN_PARSE_FAILED; lat_s[ next ] = -1.0;
                       next++; done++; continue; }
      unsigned long sz = m->sz, cookie = m->sig;
      memcpy( buf, rg.dcache + (unsigned long)m->chunk*RING_CHUNK, sz );
      atomic_thread_fence( memory_order_acquire );
      if( atomic_load_explicit( &m->seq, memory_order_relaxed )!=s0 ) {
        res->ring_overruns++; verdict[ next ] = FD_ED25519_HIP_TXN_PARSE_FAILED; lat_s[ next ] = -1.0;
        next++; done++; continue;
      }
      if( sz && buf[0]<=16U ) sigs += buf[0];
      fd_ed25519_hip_vtile_frag( vt, buf, sz, cookie );
#ifdef FD_ED25519_HIP_AB_STAGE_TRACE
      if( stage_frag_pull ) {
        stage_frag_pull [ next ] = now_s();
        stage_frag_batch[ next ] = vt->open ? vt->open_seq : vt->pipe->seq - 1UL;
      }
#endif
      next++;
      atomic_store_explicit( &pr.consumed, next, memory_order_release );
      pulled = 1;
      if( vt->pipe->seq!=batches0 ) break;                /* a full batch went out: go collect */
    }
    batches0 = vt->pipe->seq;
    /* ring drained: send the open batch if a slot can take it */
    if( !pulled && vt->open && vt->open->txn_cnt &&
        ( slot_cnt==1U || partial_ok( fd_ed25519_hip_pipe_in_flight( vt->pipe ), slot_cnt ) || next==txn_cnt ) )
      fd_ed25519_hip_vtile_flush( vt, 0 );
    unsigned long got = fd_ed25519_hip_vtile_poll( vt, 0, 4096UL, ck, vd, NULL );
    double t = now_s();
    for( unsigned long k=0UL; k<got; k++ ) {
      lat_s  [ ck[k] ] = t - t_pub[ ck[k] ];
      verdict[ ck[k] ] = vd[k];
    }
    done += got;
  }
  double t_end = now_s();
  pthread_join( th, NULL );
  if( err ) {
    free( rg.mcache ); free( rg.dcache ); free( t_pub ); free( ck ); free( vd ); free( buf );
    fd_ed25519_hip_vtile_delete( vt );
    return err;
  }
  res->offered_txn_per_s  = offered_txn_per_s;
  res->seconds            = t_end - pr.t0;
  res->txn_cnt            = txn_cnt;
  res->sig_cnt            = sigs;
  res->achieved_txn_per_s = (double)txn_cnt / res->seconds;
  res->achieved_sig_per_s = (double)sigs / res->seconds;
  res->batches            = vt->pipe->seq;
  free( rg.mcache ); free( rg.dcache ); free( t_pub ); free( ck ); free( vd ); free( buf );
  fd_ed25519_hip_vtile_delete( vt );
  return FD_ED25519_HIP_OK;
}

/* ======================================================================
   several verify tiles: one thread per tile, each a whole latency_run on
   its round-robin share of the transactions */

typedef struct {
  int                   device;
  unsigned              slot_cnt;
  unsigned long         batch_sigs, ring_depth, n;
  unsigned char const * payloads;
  unsigned long *       off;
  unsigned int *        sz;
  double                rate;
  int                   flags;
  double *              lat;
  signed char *         verdict;
  fd_ed25519_hip_latency_result_t res;
  int                   err;
  char                  errmsg[ 256 ];   /* the worker's last_error (it is per thread) */
} tile_job_t;

static void *
tile_main( void * arg ) {
  tile_job_t * j = (tile_job_t *)arg;
  j->err = latency_run( j->device, j->slot_cnt, j->batch_sigs, j->payloads, j->off, j->sz, j->n, j->rate,
                       j->ring_depth, j->flags, j->lat, j->verdict, &j->res, -1 );
  if( j->err ) snprintf( j->errmsg, sizeof(j->errmsg), "%s", fd_ed25519_hip_last_error() );
  return NULL;
}

int
fd_ed25519_hip_latency_run_tiles( int device, unsigned tile_cnt, unsigned slot_cnt, unsigned long batch_sigs,
                                  unsigned char const * payloads, unsigned long const * payload_off,
                                  unsigned int const * payload_sz, unsigned long txn_cnt, double offered_txn_per_s,
                                  unsigned long ring_depth, int flags, double * lat_s, signed char * verdict,
                                  fd_ed25519_hip_latency_result_t * res ) {
  if( !tile_cnt || tile_cnt>64U || txn_cnt<tile_cnt || !lat_s || !verdict || !res ) return FD_ED25519_HIP_ERR_INVAL;
  tile_job_t job[ 64 ];
  pthread_t  th[ 64 ];
  memset( job, 0, sizeof(job) );
  int err = 0;
  for( unsigned k=0U; k<tile_cnt; k++ ) {
    tile_job_t * j = &job[k];
    j->n = (txn_cnt - k + tile_cnt - 1UL) / tile_cnt;   /* transactions k, k+K, k+2K, ... */
    j->off = (unsigned long *)malloc( j->n*sizeof(unsigned long) );
    j->sz  = (unsigned int  *)malloc( j->n*sizeof(unsigned int) );
    j->lat = (double *)malloc( j->n*sizeof(double) );
    j->verdict = (signed char *)malloc( j->n );
    if( !j->off || !j->sz || !j->lat || !j->verdict ) { err = FD_ED25519_HIP_ERR_NOMEM; break; }
    for( unsigned long i=0UL; i<j->n; i++ ) {
      j->off[i] = payload_off[ k + i*tile_cnt ];
      j->sz [i] = payload_sz [ k + i*tile_cnt ];
    }
    j->device = device; j->slot_cnt = slot_cnt; j->batch_sigs = batch_sigs; j->ring_depth = ring_depth;
    j->payloads = payloads; j->rate = offered_txn_per_s / (double)tile_cnt; j->flags = flags;
  }
  unsigned started = 0U;
  for( unsigned k=0U; !err && k<tile_cnt; k++ ) {
    if( pthread_create( &th[k], NULL, tile_main, &job[k] ) ) { err = FD_ED25519_HIP_ERR_NOMEM; break; }
    started++;
  }
  for( unsigned k=0U; k<started; k++ ) pthread_join( th[k], NULL );
  memset( res, 0, sizeof(*res) );
  res->offered_txn_per_s = offered_txn_per_s;
  for( unsigned k=0U; k<tile_cnt; k++ ) {
    tile_job_t * j = &job[k];
    if( !err && j->err ) { err = j->err; fd_ed25519_hip_private_set_error( j->errmsg ); }
    if( !err ) {
      for( unsigned long i=0UL; i<j->n; i++ ) {
        lat_s  [ k + i*tile_cnt ] = j->lat[i];
        verdict[ k + i*tile_cnt ] = j->verdict[i];
      }
      if( j->res.seconds>res->seconds ) res->seconds = j->res.seconds;
      res->txn_cnt       += j->res.txn_cnt;
      res->sig_cnt       += j->res.sig_cnt;
      res->batches       += j->res.batches;
      res->ring_overruns += j->res.ring_overruns;
    }
    free( j->off ); free( j->sz ); free( j->lat ); free( j->verdict );
  }
  if( !err && res->seconds>0.0 ) {
    res->achieved_txn_per_s = (double)res->txn_cnt / res->seconds;
    res->achieved_sig_per_s = (double)res->sig_cnt / res->seconds;
  }
  return err;
}

/* One dummy batch through every launch form a slot uses (a zero
   signature through the verify kernels, and -- GPU parse -- a one-byte
   payload through the device parser), on every slot: code objects load
   and first launches happen here, not under the first transactions. */
static int
vt_warm( fd_ed25519_hip_vtile_t * vt ) {
  fd_ed25519_hip_pipe_t * pipe = vt->pipe;
  pipe->warming = 1;
  for( unsigned k=0U; k<pipe->slot_cnt; k++ ) {
    fd_ed25519_hip_slot_t * s = fd_ed25519_hip_pipe_acquire( pipe );
    if( !s ) return FD_ED25519_HIP_ERR_INVAL;
    memset( s->sigs, 0, 64UL ); memset( s->pubs, 0, 32UL );
    s->msg_off[0] = 0UL; s->msg_sz[0] = 0U; s->txn_first[0] = 0U; s->txn_sig_cnt[0] = 1U;
    int err = fd_ed25519_hip_pipe_submit( pipe, s, 1UL, 0UL, 1UL );
    if( err ) return err;
    if( !fd_ed25519_hip_pipe_poll( pipe, 1 ) ) return pipe->err ? pipe->err : FD_ED25519_HIP_ERR_INVAL;
    fd_ed25519_hip_pipe_release( pipe, s );
    if( vt->gpu_parse ) {
      s = fd_ed25519_hip_pipe_acquire( pipe );
      if( !s ) return FD_ED25519_HIP_ERR_INVAL;
      s->msgs[0] = 0; s->msg_off[0] = 0UL; s->msg_sz[0] = 1U;
      err = fd_ed25519_hip_pipe_submit_txns( pipe, s, 1UL, 1UL );
      if( err ) return err;
      if( !fd_ed25519_hip_pipe_poll( pipe, 1 ) ) return pipe->err ? pipe->err : FD_ED25519_HIP_ERR_INVAL;
      fd_ed25519_hip_pipe_release( pipe, s );
    }
    if( vt->zero_copy ) {   /* and the DMA from the caller's page-locked memory, once per slot */
      s = fd_ed25519_hip_pipe_acquire( pipe );
      if( !s ) return FD_ED25519_HIP_ERR_INVAL;
      pipe_slot_t * ps = (pipe_slot_t *)s;
      ps->ext_src[0] = vt->zc_base; ps->ext_dev[0] = vt->zc_dev; ps->ext_len[0] = 1UL; ps->ext_counts = 1;
      s->msg_off[0] = 0UL; s->msg_sz[0] = 1U; s->txn_sig_cnt[0] = 0U;
      err = fd_ed25519_hip_pipe_submit_txns( pipe, s, 1UL, 1UL );
      if( err ) return err;
      if( !fd_ed25519_hip_pipe_poll( pipe, 1 ) ) return pipe->err ? pipe->err : FD_ED25519_HIP_ERR_INVAL;
      fd_ed25519_hip_pipe_release( pipe, s );
    }
  }
  pipe->seq = 0UL;   /* the stream's batches count from 0 */
  pipe->warming = 0;
  return FD_ED25519_HIP_OK;
}

/* ======================================================================
   vservice: the GPU process behind a sandboxed verify tile (shlink in,
   shlink out).

   Liveness and failure policy (the GPU side of fd_cnc's heartbeat,
   src/tango/cnc/fd_cnc.h:63-65,129-130, and of fd_topo_run's supervision,
   src/disco/topo/fd_topo_run.c:50-100): every pass of the loop, and every
   few polls while it waits for the GPU, ticks the heartbeat of `out` (the
   tile watches it and stops waiting when it goes stale,
   integration/fd_verify_hip.c) and watches the tile's heartbeat on `in`.
   What a tile causes -- it marked a link failed, overran its txn link, or
   its heartbeat stopped -- ends that link pair: nothing more is published
   on it, both links are marked failed with the code, its vtile (engines,
   device memory) is freed, and the service's other links are served on.
   What the device causes -- a batch the GPU failed or did not complete in
   time, a launch or allocation that failed -- ends every link: the failing
   link raises the service's stop flag and each sibling ends with
   FD_ED25519_HIP_SHLINK_FAIL_STOPPED.  The service never aborts the
   process mid-batch. */

/* an idle pass of a polling loop (FD_SPIN_PAUSE's role in the reference's
   tiles): a pause hint, so a link thread with nothing to do yields its
   core's pipeline to the sibling hyperthread */
static inline void
spin_pause( void ) {
#if defined(__x86_64__)
  __builtin_ia32_pause();
#endif
}

static long
now_ns( void ) {
  struct timespec ts;
  clock_gettime( CLOCK_MONOTONIC, &ts );
  return ts.tv_sec*1000000000L + ts.tv_nsec;
}

typedef struct {
  fd_ed25519_hip_shlink_t *        in;
  fd_ed25519_hip_shlink_t *        out;
  fd_ed25519_hip_shlink_watch_t    tile;       /* the tile's heartbeat on `in` */
  long                             tile_stale_ns;
  int volatile const *             ext_stop;   /* the caller's stop request */
  _Atomic int *                    dev_stop;   /* a sibling link saw the device fail */
  unsigned long                    beat;
  int                              hook_rc;    /* what the idle hook last ended a wait with ... */
  int                              hook_local; /* ... and whether that is the link's own end     */
} vsvc_link_t;

/* One liveness pass: ticks the service's heartbeat, then 0 (serve on) or
   the code the link ends with.  *local = 1 when the cause is the tile's
   or the caller's (the link alone ends), 0 when a sibling saw the device
   fail. */
static int
vsvc_check( vsvc_link_t * L, int * local ) {
  fd_ed25519_hip_shlink_heartbeat( L->out, L->beat++ );
  *local = 1;
  if( L->ext_stop && *L->ext_stop ) return FD_ED25519_HIP_SHLINK_FAIL_STOPPED;
  if( L->dev_stop && atomic_load_explicit( L->dev_stop, memory_order_acquire ) ) {
    *local = 0;
    return FD_ED25519_HIP_SHLINK_FAIL_STOPPED;
  }
  int ts = fd_ed25519_hip_shlink_status( L->in );
  if( !ts ) ts = fd_ed25519_hip_shlink_status( L->out );
  if( ts ) return ts;   /* the tile gave up on the link */
  if( fd_ed25519_hip_shlink_watch( &L->tile, L->in, now_ns(), L->tile_stale_ns )<0 )
    return FD_ED25519_HIP_SHLINK_FAIL_TILE_GONE;
  return 0;
}

/* the vtile's idle hook, for the rare wait inside a frag (a zero-copy
   payload out of ring order closes a batch and needs the next slot) */
static int
vsvc_idle( void * ctx ) {
  vsvc_link_t * L = (vsvc_link_t *)ctx;
  int local = 1;
  int rc = vsvc_check( L, &local );
  if( rc ) { L->hook_rc = rc; L->hook_local = local; }
  return rc;
}

/* 1 if the vtile takes one more frag of any shape without waiting for the
   GPU: the open batch has room for a transaction of 16 signatures and an
   MTU of bytes, or the next slot is free (completed batches are drained
   before this is asked) */
static int
vt_room( fd_ed25519_hip_vtile_t const * vt ) {
  if( vt->err ) return 0;
  fd_ed25519_hip_slot_t const * s = vt->open;
  if( s && s->sig_cnt+16UL<=s->sig_cap && s->txn_cnt+1UL<=s->txn_cap &&
      STAGE_ALIGN( s->msg_bytes ) + FD_ED25519_HIP_TXN_MTU + 64UL<=s->msg_cap ) return 1;
  fd_ed25519_hip_pipe_t const * pipe = vt->pipe;
  return pipe->slot[ pipe->next_acq % pipe->slot_cnt ].state==SLOT_FREE;
}

/* One link pair of the verify service.  A service thread serves one or
   more pairs, a pass over each in turn; a pass never waits for the GPU
   (frags stay in the txn link while the pair's slots are all in flight),
   so the pairs of a thread do not hold each other up. */
typedef struct {
  vsvc_link_t                       L;
  fd_ed25519_hip_vtile_t *          vt;
  unsigned char *                   buf;      /* a frag copied out of the shared dcache (copying modes) */
  void *                            reg;      /* zero-copy: the txn link's mapping, page-locked */
  fd_ed25519_hip_vservice_stats_t * stats;
  _Atomic int *                     stop;
  unsigned                          slot_cnt;
  int                               device;
  double                            t0, t_first, hang_s;
  unsigned long                     txns, pass;
  int                               eos, idle, live;
  char                              errmsg[ 256 ];   /* last_error of a device-wide end (it is per thread) */
#ifdef FD_ED25519_HIP_AB_SERVICE_PROFILE
  unsigned long long                pf_t[ 5 ], pf_idle, pf_pass, pf_cons;
#endif
} vsvc_t;

#ifdef FD_ED25519_HIP_AB_SERVICE_PROFILE
#define PF_MARK( i ) do { pf_n = __rdtsc(); S->pf_t[ i ] += pf_n - pf_c; pf_c = pf_n; } while(0)
#else
#define PF_MARK( i ) do {} while(0)
#endif

/* the pair ends with rc (0: EOS answered): both links marked failed with a
   failure code, the sibling pairs stopped when the cause is the device's
   (local = 0), the stats written, the vtile (engines, device memory) freed.

   A hung device (a batch past the hang bound, FD_ED25519_HIP_ERR_TIMEOUT)
   is different: freeing the vtile synchronises its streams, which never
   returns while the GPU is hung, and a sibling's streams may sit behind
   the hung queue too.  The stop word then says VSVC_STOP_HUNG, and every
   pair that ends under it leaves its vtile and its page-locked mapping as
   they are (host and device memory leak until the process exits, which
   the service does right away) so that the call returns and the links
   carry the code. */
#define VSVC_STOP_FAILED 1
#define VSVC_STOP_HUNG   2

static void
vsvc_end( vsvc_t * S, int rc, int local ) {
  if( rc ) {
    fd_ed25519_hip_shlink_fail( S->L.in, rc );
    fd_ed25519_hip_shlink_fail( S->L.out, rc );
    if( S->stop && !local ) {
      int want = rc==FD_ED25519_HIP_ERR_TIMEOUT ? VSVC_STOP_HUNG : VSVC_STOP_FAILED;
      int cur  = atomic_load_explicit( S->stop, memory_order_acquire );
      while( cur<want && !atomic_compare_exchange_weak_explicit( S->stop, &cur, want, memory_order_acq_rel,
                                                                 memory_order_acquire ) ) {}
    }
    if( !local ) snprintf( S->errmsg, sizeof(S->errmsg), "%s", fd_ed25519_hip_last_error() );
  }
  int hung = rc==FD_ED25519_HIP_ERR_TIMEOUT ||
             ( S->stop && atomic_load_explicit( S->stop, memory_order_acquire )==VSVC_STOP_HUNG );
  if( S->stats ) {
    S->stats->txn_cnt      = S->txns;
    S->stats->batches      = S->vt ? S->vt->pipe->seq : 0UL;
    S->stats->seconds      = now_s() - ( S->txns ? S->t_first : S->t0 );
    S->stats->device_bytes = S->vt ? fd_ed25519_hip_vtile_device_bytes( S->vt ) : 0UL;
    S->stats->shared_device_bytes = fd_ed25519_hip_shared_device_bytes( S->device );
    S->stats->end_code     = rc;
  }
#ifdef FD_ED25519_HIP_AB_SERVICE_PROFILE
  double d = (double)( S->txns + 1UL );
  fprintf( stderr, "vservice profile: %lu txns, %llu passes (%llu idle); cycles per txn: status %.0f publish %.0f "
           "poll %.0f consume+frag %.0f (of which consume %.0f) flush+pause %.0f; %llu batches: submit %.0f cycles each, "
           "round trip avg %.3f ms max %.3f ms; submit parts per batch: h2d %.0f (wait %.0f) launches %.0f d2h %.0f\n",
           S->txns, S->pf_pass, S->pf_idle, (double)S->pf_t[0]/d, (double)S->pf_t[1]/d, (double)S->pf_t[2]/d,
           (double)S->pf_t[3]/d, (double)S->pf_cons/d, (double)S->pf_t[4]/d, vt_submits,
           (double)vt_submit_cycles/(double)( vt_submits + 1ULL ), 1e3*vt_rtt_s/(double)( vt_rtt_n + 1ULL ),
           1e3*vt_rtt_max_s, (double)pf_sub_h2d/(double)( pf_sub_n + 1ULL ),
           (double)pf_sub_wait/(double)( pf_sub_n + 1ULL ), (double)pf_sub_launch/(double)( pf_sub_n + 1ULL ),
           (double)pf_sub_d2h/(double)( pf_sub_n + 1ULL ) );
#endif
  free( S->buf ); S->buf = NULL;
  if( hung ) {   /* nothing that waits on the device: left for the process exit */
    S->vt = NULL; S->reg = NULL; S->live = 0;
    if( S->stats ) S->stats->leaked_on_hang = 1U;
    return;
  }
  if( S->vt ) {
    S->vt->idle = NULL;   /* the delete below may wait for batches in flight */
    fd_ed25519_hip_vtile_delete( S->vt );
    S->vt = NULL;
  }
  if( S->reg ) { hipHostUnregister( S->reg ); S->reg = NULL; }   /* after the batches that read from it */
  S->live = 0;
}

/* builds the pair's vtile (and, zero-copy, page-locks the txn link) and
   runs every kernel once; 0, or the pair has ended with the code */
static int
vsvc_open( vsvc_t * S, int device, unsigned slot_cnt, unsigned long batch_sigs, int flags,
           fd_ed25519_hip_shlink_t * in, fd_ed25519_hip_shlink_t * out, fd_ed25519_hip_vservice_stats_t * stats,
           _Atomic int * stop, fd_ed25519_hip_vservice_opts_t const * opts ) {
  memset( S, 0, sizeof(*S) );
  S->L.in = in; S->L.out = out; S->L.dev_stop = stop; S->L.beat = 1UL;
  S->L.ext_stop      = opts ? opts->stop : NULL;
  S->L.tile_stale_ns = !opts || !opts->tile_stale_ns ? FD_ED25519_HIP_VSERVICE_TILE_STALE_NS : opts->tile_stale_ns;
  long hang_ns       = !opts || !opts->gpu_hang_ns ? FD_ED25519_HIP_VSERVICE_GPU_HANG_NS : opts->gpu_hang_ns;
  S->hang_s   = hang_ns>0L ? 1e-9*(double)hang_ns : 0.0;
  S->stats = stats; S->stop = stop; S->slot_cnt = slot_cnt; S->device = device;
  S->t0 = now_s(); S->idle = 1; S->live = 1;
  if( !in || !out ) { vsvc_end( S, FD_ED25519_HIP_ERR_INVAL, 0 ); return FD_ED25519_HIP_ERR_INVAL; }
  S->vt = fd_ed25519_hip_vtile_new( device, slot_cnt, batch_sigs, 16UL, 64UL, flags );
  if( !S->vt ) { vsvc_end( S, FD_ED25519_HIP_ERR_INVAL, 0 ); return FD_ED25519_HIP_ERR_INVAL; }
  fd_ed25519_hip_vtile_t * vt = S->vt;
  vt->trailer_only = 1;   /* the tile keeps its payloads: verdict frags carry the trailers */
  vt->idle     = vsvc_idle;
  vt->idle_ctx = &S->L;
  vt->hang_s   = S->hang_s;
  S->buf = (unsigned char *)malloc( FD_ED25519_HIP_SHLINK_MTU );
  if( !S->buf ) { vsvc_end( S, FD_ED25519_HIP_ERR_NOMEM, 0 ); return FD_ED25519_HIP_ERR_NOMEM; }
  if( flags & FD_ED25519_HIP_VSERVICE_ZERO_COPY ) {
    /* the txn link's mapping page-locked with the GPU: batches DMA their
       payloads from the rooms the tile wrote */
    unsigned long map_sz;
    void * m = fd_ed25519_hip_shlink_mapping( in, &map_sz );
    hipError_t he = hipHostRegister( m, map_sz, hipHostRegisterPortable | hipHostRegisterMapped );
    if( he!=hipSuccess ) { int rc = tile_fail( "hipHostRegister(txn link)", he ); vsvc_end( S, rc, 0 ); return rc; }
    S->reg = m;
    void * m_dev = NULL;
    he = hipHostGetDevicePointer( &m_dev, m, 0U );
    if( he!=hipSuccess ) { int rc = tile_fail( "hipHostGetDevicePointer(txn link)", he ); vsvc_end( S, rc, 0 ); return rc; }
    vt->zero_copy = 1;
    vt->gpu_parse = 1;
    vt->zc_base   = fd_ed25519_hip_shlink_dcache( in, &vt->zc_size );
    vt->zc_dev    = (unsigned char const *)m_dev + ( vt->zc_base - (unsigned char const *)m );
  }
  int we = vt_warm( vt );
  if( we ) { vsvc_end( S, we, 0 ); return we; }
  return 0;
}

/* the oldest batch in flight has been on the GPU longer than the bound */
static int
vsvc_hung( vsvc_t const * S ) {
  fd_ed25519_hip_pipe_t const * pipe = S->vt->pipe;
  if( S->hang_s<=0.0 || !pipe->in_flight ) return 0;
  pipe_slot_t const * o = &pipe->slot[ pipe->next_poll % pipe->slot_cnt ];
  return o->state==SLOT_BUSY && now_s() - o->pub.t_submit>S->hang_s;
}

/* One pass over a live pair: liveness, completed batches resolved and
   their verdicts published, then as many frags staged as the vtile takes
   without waiting.  Ends the pair (vsvc_end) on EOS or failure. */
static void
vsvc_pass( vsvc_t * S ) {
  fd_ed25519_hip_vtile_t * vt = S->vt;
  int rc, local = 1;
#ifdef FD_ED25519_HIP_AB_SERVICE_PROFILE
  unsigned long long pf_c = __rdtsc(), pf_n;
#endif
  /* the liveness pass (a clock read, the peer's header lines) runs every
     16th busy pass and on every idle one: microseconds apart either way */
  if( S->idle || !(++S->pass & 15UL) ) {
    if( (rc = vsvc_check( &S->L, &local )) ) { vsvc_end( S, rc, local ); return; }
    if( vsvc_hung( S ) ) {
      char msg[ 128 ];
      snprintf( msg, sizeof(msg), "vservice: batch %lu did not complete within %.1f s (GPU hang)",
                vt->pipe->seq - vt->pipe->in_flight, S->hang_s );
      fd_ed25519_hip_private_set_error( msg );
      vsvc_end( S, FD_ED25519_HIP_ERR_TIMEOUT, 0 );
      return;
    }
  }
  PF_MARK( 0 );
  /* completed batches resolve (in frag order); their verdicts go out as
     far as credits allow: the verdict byte, then (SUCCESS) the trailer of
     the frag the tile publishes (its fd_txn_t and payload_sz, from the
     vtile's arena: the tile has the payload) */
  while( vt_drain_one( vt, 0 ) ) {}
  PF_MARK( 2 );
  int published = 0;
  for( vrec_t const * r; (r = vt_head( vt )); ) {
    unsigned char * dst = fd_ed25519_hip_shlink_prepare( S->L.out );
    if( !dst ) break;
    unsigned long tsz = r->verdict==FD_ED25519_HIP_TXN_VERIFY_SUCCESS ? r->frag_sz : 0UL;
    dst[ 0 ] = (unsigned char)r->verdict;
    if( tsz ) memcpy( dst + 1, vt->oa + r->arena_off, tsz );
    if( (rc = fd_ed25519_hip_shlink_commit( S->L.out, 1UL + tsz, r->cookie, 0U )) ) { vsvc_end( S, rc, 0 ); return; }
    vt_pop( vt );
    published = 1;
  }
  PF_MARK( 1 );
  if( (rc = fd_ed25519_hip_vtile_error( vt )) ) {
    /* a wait the idle hook ended is the hook's cause; any other vtile error the device's */
    vsvc_end( S, rc, rc==S->L.hook_rc ? S->L.hook_local : 0 );
    return;
  }
  if( S->eos && !fd_ed25519_hip_vtile_pending( vt ) ) {
    /* every frag answered: the EOS frag when the verdict link has credit */
    int r = fd_ed25519_hip_shlink_publish( S->L.out, NULL, 0UL, 0UL, FD_ED25519_HIP_SHLINK_CTL_EOS );
    if( !r ) { vsvc_end( S, FD_ED25519_HIP_OK, 1 ); return; }
    if( r!=1 ) { vsvc_end( S, r, 0 ); return; }
    S->idle = 1;
    spin_pause();
    return;
  }
  /* after_frag for every frag that is ready and fits without a wait */
  int pulled = 0;
  while( !S->eos && vt->zero_copy && vt_room( vt ) ) {   /* in place: the payload stays in the link's room */
    unsigned long sz = 0UL, sig = 0UL;
    unsigned int ctl = 0U;
    int perr;
    unsigned char const * src = fd_ed25519_hip_shlink_peek( S->L.in, &sz, &sig, &ctl, &perr );
    if( !src ) {
      if( perr==1 ) break;
      vsvc_end( S, FD_ED25519_HIP_SHLINK_FAIL_PROTOCOL, 1 );   /* overrun, or a line out of bounds */
      return;
    }
    if( ctl & FD_ED25519_HIP_SHLINK_CTL_EOS ) { fd_ed25519_hip_shlink_advance( S->L.in ); S->eos = 1; break; }
    if( !S->txns ) S->t_first = now_s();
    int r = vt_frag_zc( vt, src, sz, sig );
    if( r<0 ) { vsvc_end( S, r, r==S->L.hook_rc ? S->L.hook_local : 0 ); return; }
    /* the credit goes back now: the room itself is reused only after its
       verdict (the tile's bound on unanswered frags) */
    if( fd_ed25519_hip_shlink_advance( S->L.in ) ) { vsvc_end( S, FD_ED25519_HIP_SHLINK_FAIL_PROTOCOL, 1 ); return; }
    S->txns++;
    pulled = 1;
  }
  while( !S->eos && !vt->zero_copy && vt_room( vt ) ) {
    unsigned long sz = 0UL, sig = 0UL;
    unsigned int ctl = 0U;
#ifdef FD_ED25519_HIP_AB_SERVICE_PROFILE
    unsigned long long c0 = __rdtsc();
#endif
    /* copied out of the shared dcache first: the tile is not trusted not
       to change it meanwhile */
    int r = fd_ed25519_hip_shlink_consume( S->L.in, S->buf, &sz, &sig, &ctl );
#ifdef FD_ED25519_HIP_AB_SERVICE_PROFILE
    S->pf_cons += __rdtsc() - c0;
#endif
    if( r==1 ) break;
    if( r ) { vsvc_end( S, FD_ED25519_HIP_SHLINK_FAIL_PROTOCOL, 1 ); return; }   /* overrun: the tile ignored credits */
    if( ctl & FD_ED25519_HIP_SHLINK_CTL_EOS ) { S->eos = 1; break; }
    if( !S->txns ) S->t_first = now_s();
    r = fd_ed25519_hip_vtile_frag( vt, S->buf, sz, sig );
    if( r<0 ) { vsvc_end( S, r, r==S->L.hook_rc ? S->L.hook_local : 0 ); return; }
    S->txns++;
    pulled = 1;
  }
  PF_MARK( 3 );
  /* `in` drained (or the vtile full): send the open batch if a slot can
     take it (all of it at the end) */
  int flushed = 0;
  if( !pulled && vt->open && vt->open->txn_cnt &&
      ( S->eos || S->slot_cnt==1U || partial_ok( fd_ed25519_hip_pipe_in_flight( vt->pipe ), S->slot_cnt ) ) ) {
    fd_ed25519_hip_vtile_flush( vt, S->eos );
    flushed = 1;
  }
  S->idle = !pulled && !published && !flushed;
#ifdef FD_ED25519_HIP_AB_SERVICE_PROFILE
  S->pf_idle += (unsigned long long)S->idle;
  S->pf_pass++;
#endif
  PF_MARK( 4 );
}
#undef PF_MARK

typedef struct {
  int                                    device, flags;
  int                                    cpu;      /* the CPU the thread runs on, or -1 */
  unsigned                               slot_cnt, k0, k1;   /* the thread serves link pairs [k0, k1) */
  unsigned long                          batch_sigs;
  fd_ed25519_hip_shlink_t * const *      in;
  fd_ed25519_hip_shlink_t * const *      out;
  vsvc_t *                               pair;      /* [link_cnt], this thread's [k0, k1) */
  fd_ed25519_hip_vservice_stats_t *      st;        /* [link_cnt] */
  _Atomic int *                          stop;
  fd_ed25519_hip_vservice_opts_t const * opts;
  _Atomic unsigned *                     ready;     /* link pairs that are ready to serve (or ended) */
} vservice_job_t;

static void *
vservice_main( void * arg ) {
  vservice_job_t * j = (vservice_job_t *)arg;
  if( j->cpu>=0 ) {   /* before anything allocates: first touch lands on the thread's own node */
    cpu_set_t set;
    CPU_ZERO( &set );
    CPU_SET( j->cpu, &set );
    if( pthread_setaffinity_np( pthread_self(), sizeof(set), &set ) ) {
      char msg[ 96 ];
      snprintf( msg, sizeof(msg), "vservice: cannot run a service thread on CPU %d", j->cpu );
      fd_ed25519_hip_private_set_error( msg );
      for( unsigned k=j->k0; k<j->k1; k++ ) {
        vsvc_t * S = &j->pair[ k ];
        memset( S, 0, sizeof(*S) );
        S->L.in = j->in[ k ]; S->L.out = j->out[ k ]; S->stats = &j->st[ k ]; S->stop = j->stop; S->device = j->device;
        S->t0 = now_s();
        vsvc_end( S, FD_ED25519_HIP_ERR_INVAL, 0 );
        atomic_fetch_add_explicit( j->ready, 1U, memory_order_release );
      }
      return NULL;
    }
  }
  for( unsigned k=j->k0; k<j->k1; k++ ) {
    vsvc_open( &j->pair[ k ], j->device, j->slot_cnt, j->batch_sigs, j->flags, j->in[ k ], j->out[ k ], &j->st[ k ],
               j->stop, j->opts );
    atomic_fetch_add_explicit( j->ready, 1U, memory_order_release );   /* ready (or ended): counted once */
  }
  for( int live=1; live; ) {
    live = 0;
    int busy = 0;
    for( unsigned k=j->k0; k<j->k1; k++ ) {
      vsvc_t * S = &j->pair[ k ];
      if( !S->live ) continue;
      vsvc_pass( S );
      live |= S->live;
      busy |= S->live && !S->idle;
    }
    if( !busy ) spin_pause();
  }
  return NULL;
}

/* link-local ends: the tile's (protocol, gone, its own status codes) and
   the caller's stop; everything else is the device's */
static int
vsvc_code_is_device( int rc ) {
  return rc && rc!=FD_ED25519_HIP_SHLINK_FAIL_PROTOCOL && rc!=FD_ED25519_HIP_SHLINK_FAIL_STOPPED &&
         rc!=FD_ED25519_HIP_SHLINK_FAIL_TILE_GONE;
}

int
fd_ed25519_hip_vservice_serve( int device, unsigned slot_cnt, unsigned long batch_sigs, int flags,
                               fd_ed25519_hip_shlink_t * const * in, fd_ed25519_hip_shlink_t * const * out,
                               unsigned link_cnt, fd_ed25519_hip_vservice_stats_t * stats,
                               fd_ed25519_hip_vservice_opts_t const * opts ) {
  if( !link_cnt || link_cnt>FD_ED25519_HIP_VSERVICE_LINK_MAX || !in || !out ) return FD_ED25519_HIP_ERR_INVAL;
  unsigned per = opts && opts->links_per_thread ? opts->links_per_thread : 1U;
  if( per>link_cnt ) per = link_cnt;
  unsigned thread_cnt = ( link_cnt + per - 1U ) / per;
  vservice_job_t *                  job  = (vservice_job_t *)calloc( thread_cnt, sizeof(vservice_job_t) );
  pthread_t *                       th   = (pthread_t *)calloc( thread_cnt, sizeof(pthread_t) );
  vsvc_t *                          pair = (vsvc_t *)calloc( link_cnt, sizeof(vsvc_t) );
  fd_ed25519_hip_vservice_stats_t * st   = (fd_ed25519_hip_vservice_stats_t *)calloc( link_cnt, sizeof(*st) );
  if( !job || !th || !pair || !st ) { free( job ); free( th ); free( pair ); free( st ); return FD_ED25519_HIP_ERR_NOMEM; }
  _Atomic int stop = 0;
  _Atomic unsigned ready = 0U;
  unsigned started = 0U;
  int rc = FD_ED25519_HIP_OK;
  for( unsigned t=0U; t<thread_cnt; t++ ) {
    vservice_job_t * j = &job[ t ];
    j->device = device; j->flags = flags; j->slot_cnt = slot_cnt; j->batch_sigs = batch_sigs;
    j->k0 = t*per; j->k1 = j->k0 + per<link_cnt ? j->k0 + per : link_cnt;
    j->cpu = opts && opts->link_cpu_cnt && opts->link_cpus ? opts->link_cpus[ t % opts->link_cpu_cnt ] : -1;
    j->in = in; j->out = out; j->pair = pair; j->st = st; j->stop = &stop; j->opts = opts; j->ready = &ready;
    if( pthread_create( &th[ t ], NULL, vservice_main, j ) ) {
      rc = FD_ED25519_HIP_ERR_NOMEM;
      atomic_store_explicit( &stop, 1, memory_order_release );
      for( unsigned m=j->k0; m<link_cnt; m++ ) {
        fd_ed25519_hip_shlink_fail( in[ m ], rc ); fd_ed25519_hip_shlink_fail( out[ m ], rc );
        st[ m ].end_code = rc;
      }
      break;
    }
    started++;
  }
  /* every link pair has built its engines and launched every kernel once */
  if( started==thread_cnt ) {
    while( atomic_load_explicit( &ready, memory_order_acquire )<link_cnt ) {
      struct timespec ts = { 0, 1000000L };
      nanosleep( &ts, NULL );
    }
    if( opts && opts->ready ) opts->ready( opts->ready_ctx );
  }
  for( unsigned t=0U; t<started; t++ ) pthread_join( th[ t ], NULL );
  /* the result: a device-wide failure's code first, else the first
     link-local end, else OK (every link ended with EOS) */
  int local_rc = FD_ED25519_HIP_OK;
  int msg_k = -1;
  unsigned served = started==thread_cnt ? link_cnt : started*per;
  for( unsigned k=0U; k<served; k++ ) {
    int r = st[ k ].end_code;
    if( vsvc_code_is_device( r ) ) { if( !vsvc_code_is_device( rc ) ) { rc = r; msg_k = (int)k; } }
    else if( r && !local_rc ) local_rc = r;
  }
  if( !rc ) rc = local_rc;
  /* the failing pair's message, for the caller's fd_ed25519_hip_last_error */
  if( msg_k>=0 && pair[ msg_k ].errmsg[0] ) fd_ed25519_hip_private_set_error( pair[ msg_k ].errmsg );
  if( stats ) for( unsigned k=0U; k<link_cnt; k++ ) stats[ k ] = st[ k ];
  free( job ); free( th ); free( pair ); free( st );
  return rc;
}

int
fd_ed25519_hip_vservice_run( int device, unsigned slot_cnt, unsigned long batch_sigs, int flags,
                             fd_ed25519_hip_shlink_t * in, fd_ed25519_hip_shlink_t * out,
                             fd_ed25519_hip_vservice_stats_t * stats ) {
  return fd_ed25519_hip_vservice_serve( device, slot_cnt, batch_sigs, flags, &in, &out, 1U, stats, NULL );
}

int
fd_ed25519_hip_vservice_run_links( int device, unsigned slot_cnt, unsigned long batch_sigs, int flags,
                                   fd_ed25519_hip_shlink_t * const * in, fd_ed25519_hip_shlink_t * const * out,
                                   unsigned link_cnt, fd_ed25519_hip_vservice_stats_t * stats ) {
  return fd_ed25519_hip_vservice_serve( device, slot_cnt, batch_sigs, flags, in, out, link_cnt, stats, NULL );
}

/* ======================================================================
   pool: one feeder thread per device, batches dealt round-robin (batch b
   to device b % N, the analogue of seq % verify_tile_count,
   src/app/fdctl/run/tiles/fd_verify.c:46).

   A batch reaches the device without its bytes being touched on the host
   when the caller's arrays are page-locked (fd_ed25519_hip_host_register,
   or hipHostMalloc'd): its messages go as one DMA of the byte range they
   span (the kernels index that range with the caller's own offsets, the
   device base pointer shifted by the range's start), msg_off / msg_sz /
   sigs / pubs as one DMA each, and the codes come back by DMA straight
   into out.  Pageable arrays, or messages scattered so widely that their
   span is far larger than their bytes, are packed into the slot's pinned
   staging block first.  Each slot has its own engine (stream and work
   arrays), so one batch's copies overlap another's kernels; the feeder
   thread runs on the CPUs of its GPU's NUMA node. */

typedef struct {
  fd_ed25519_hip_engine_t * eng;
  hipEvent_t                ev;
  hipEvent_t                ev_h2d;    /* this slot's last batch has crossed the link */
  unsigned char *           d_msgs;
  unsigned long *           d_off;
  unsigned int *            d_sz;
  unsigned char *           d_sigs;
  unsigned char *           d_pubs;
  signed char *             d_out;
  unsigned char *           h_stage;   /* pinned: [sigs | pubs | off | sz | msgs], staged batches only (lazy) */
  signed char *             h_out;     /* pinned codes, when out is pageable (lazy)                           */
  unsigned long             i0, i1;
  int                       busy;
} pool_slot_t;

#define POOL_DEV_MAX  64U
#define POOL_SLOT_MAX 8U

struct fd_ed25519_hip_pool {
  unsigned      device_cnt, slot_cnt;
  unsigned long batch_sigs, msg_cap;
  int           device[ POOL_DEV_MAX ];
  pool_slot_t   slot[ POOL_DEV_MAX ][ POOL_SLOT_MAX ];
};

typedef struct {
  fd_ed25519_hip_pool_t * pool;
  unsigned                rank;
  hipEvent_t              h2d_tail;   /* ev_h2d of the batch submitted last on this device (or NULL) */
  unsigned long           n;
  unsigned char const *   msgs;
  unsigned long const *   msg_off;
  unsigned int const *    msg_sz;
  unsigned char const *   sigs;
  unsigned char const *   pubs;
  signed char *           out;
  int                     direct_in, direct_out;   /* caller arrays page-locked */
  int                     err;
  char                    errmsg[ 256 ];   /* the feeder's last_error for err (last_error is per thread) */
  fd_ed25519_hip_pool_stats_t st;
} pool_job_t;

static int
host_locked( void const * p ) {
  if( !p ) return 0;
  hipPointerAttribute_t a;
  memset( &a, 0, sizeof(a) );
  if( hipPointerGetAttributes( &a, p )!=hipSuccess ) { (void)hipGetLastError(); return 0; }
  return a.type==hipMemoryTypeHost;
}

int
fd_ed25519_hip_host_register( void * ptr, unsigned long sz ) {
  if( !ptr || !sz ) return FD_ED25519_HIP_ERR_INVAL;
  TCHK( hipHostRegister( ptr, sz, hipHostRegisterPortable | hipHostRegisterMapped ), "hipHostRegister" );
  return FD_ED25519_HIP_OK;
}

int
fd_ed25519_hip_host_unregister( void * ptr ) {
  if( !ptr ) return FD_ED25519_HIP_ERR_INVAL;
  TCHK( hipHostUnregister( ptr ), "hipHostUnregister" );
  return FD_ED25519_HIP_OK;
}

void *
fd_ed25519_hip_host_alloc( unsigned long sz ) {
  void * p = NULL;
  hipError_t e = hipHostMalloc( &p, sz ? sz : 1UL, hipHostMallocPortable );
  if( e!=hipSuccess ) { tile_fail( "hipHostMalloc", e ); return NULL; }
  return p;
}

void
fd_ed25519_hip_host_free( void * ptr ) {
  if( ptr ) hipHostFree( ptr );
}

/* the calling thread onto the CPUs of the device's NUMA node (within its
   current affinity); no change when that cannot be read */
static void
pin_near_device( int device ) {
  char bdf[ 64 ];
  if( hipDeviceGetPCIBusId( bdf, (int)sizeof(bdf), device )!=hipSuccess ) return;
  for( char * c=bdf; *c; c++ ) if( *c>='A' && *c<='F' ) *c = (char)(*c - 'A' + 'a');
  char path[ 160 ];
  snprintf( path, sizeof(path), "/sys/bus/pci/devices/%s/local_cpulist", bdf );
  FILE * f = fopen( path, "r" );
  if( !f ) return;
  char list[ 1024 ];
  size_t len = fread( list, 1, sizeof(list)-1UL, f );
  fclose( f );
  list[ len ] = 0;
  cpu_set_t cur, want;
  if( pthread_getaffinity_np( pthread_self(), sizeof(cur), &cur ) ) return;
  CPU_ZERO( &want );
  for( char * t=list; *t; ) {
    char * e;
    long lo = strtol( t, &e, 10 ), hi = lo;
    if( e==t ) break;
    if( *e=='-' ) { t = e+1; hi = strtol( t, &e, 10 ); }
    for( long c=lo; c<=hi && c<CPU_SETSIZE; c++ ) if( c>=0 && CPU_ISSET( (int)c, &cur ) ) CPU_SET( (int)c, &want );
    if( *e!=',' ) break;
    t = e+1;
  }
  if( CPU_COUNT( &want ) ) pthread_setaffinity_np( pthread_self(), sizeof(want), &want );
}

/* a batch's message span [lo, hi) and its bytes */
static void
batch_span( pool_job_t const * j, unsigned long i0, unsigned long i1, unsigned long * lo, unsigned long * hi,
            unsigned long * bytes ) {
  unsigned long l = ~0UL, h = 0UL, b = 0UL;
  for( unsigned long i=i0; i<i1; i++ ) {
    unsigned long o = j->msg_off[i], e = o + j->msg_sz[i];
    l = o<l ? o : l;
    h = e>h ? e : h;
    b += j->msg_sz[i];
  }
  if( l>h ) l = h = 0UL;
  *lo = l; *hi = h; *bytes = b;
}

/* the span goes as it is when it fits and is not much larger than the
   bytes in it */
static int
span_direct( fd_ed25519_hip_pool_t const * pl, unsigned long span, unsigned long bytes ) {
  return span<=pl->msg_cap && span<=2UL*bytes + 65536UL;
}

static int
pool_slot_init( pool_slot_t * s, int device, unsigned long batch_sigs, unsigned long msg_cap ) {
  /* one stream per slot: the slots in flight overlap one another, a side
     stream per slot would only crowd the device's hardware queues */
  s->eng = fd_ed25519_hip_engine_new( device, batch_sigs, FD_ED25519_HIP_FLAG_ONE_STREAM );
  if( !s->eng ) return FD_ED25519_HIP_ERR_INVAL;
  unsigned long dsz = 112UL*batch_sigs + msg_cap + 64UL + 1024UL;
  unsigned char * d = NULL;
  TCHK( hipMalloc( (void **)&d, dsz ), "hipMalloc(pool slot)" );
  s->d_sigs = d;                                     d += 64UL*batch_sigs;
  s->d_pubs = d;                                     d += 32UL*batch_sigs;
  s->d_off  = (unsigned long *)d;                    d += 8UL*batch_sigs;
  s->d_sz   = (unsigned int *)d;                     d += 4UL*batch_sigs;
  s->d_out  = (signed char *)d;                      d += (batch_sigs + 255UL) & ~255UL;
  s->d_msgs = d;
  TCHK( hipEventCreateWithFlags( &s->ev, hipEventDisableTiming ), "hipEventCreate" );
  TCHK( hipEventCreateWithFlags( &s->ev_h2d, hipEventDisableTiming ), "hipEventCreate" );
  return FD_ED25519_HIP_OK;
}

static void
pool_slot_fini( pool_slot_t * s ) {
  if( s->eng ) fd_ed25519_hip_engine_sync( s->eng );
  hipFree( s->d_sigs );
  hipHostFree( s->h_stage ); hipHostFree( s->h_out );
  if( s->ev ) hipEventDestroy( s->ev );
  if( s->ev_h2d ) hipEventDestroy( s->ev_h2d );
  if( s->eng ) fd_ed25519_hip_engine_delete( s->eng );
  memset( s, 0, sizeof(*s) );
}

void
fd_ed25519_hip_pool_delete( fd_ed25519_hip_pool_t * pl ) {
  if( !pl ) return;
  for( unsigned r=0U; r<pl->device_cnt; r++ ) {
    hipSetDevice( pl->device[r] );
    for( unsigned k=0U; k<pl->slot_cnt; k++ ) pool_slot_fini( &pl->slot[r][k] );
  }
  free( pl );
}

fd_ed25519_hip_pool_t *
fd_ed25519_hip_pool_new( int const * devices, unsigned device_cnt, unsigned slot_cnt, unsigned long batch_sigs,
                         unsigned long msg_cap ) {
  if( !devices || !device_cnt || device_cnt>POOL_DEV_MAX || slot_cnt<1U || slot_cnt>POOL_SLOT_MAX || !batch_sigs ) {
    fd_ed25519_hip_private_set_error( "pool_new: 1..64 devices, 1..8 slots, batch_sigs > 0" );
    return NULL;
  }
  fd_ed25519_hip_pool_t * pl = (fd_ed25519_hip_pool_t *)calloc( 1, sizeof(*pl) );
  if( !pl ) return NULL;
  pl->device_cnt = device_cnt; pl->slot_cnt = slot_cnt; pl->batch_sigs = batch_sigs;
  pl->msg_cap = msg_cap ? msg_cap : 1UL;
  for( unsigned r=0U; r<device_cnt; r++ ) {
    pl->device[r] = devices[r];
    if( hipSetDevice( devices[r] )!=hipSuccess ) { tile_fail( "hipSetDevice", hipErrorInvalidDevice ); goto fail; }
    for( unsigned k=0U; k<slot_cnt; k++ )
      if( pool_slot_init( &pl->slot[r][k], devices[r], batch_sigs, pl->msg_cap ) ) goto fail;
  }
  return pl;
fail:
  fd_ed25519_hip_pool_delete( pl );
  return NULL;
}

static int
pool_enqueue( pool_job_t * j, pool_slot_t * s, unsigned long b ) {
  fd_ed25519_hip_pool_t * pl = j->pool;
  unsigned long i0 = b*pl->batch_sigs, i1 = i0+pl->batch_sigs < j->n ? i0+pl->batch_sigs : j->n, cnt = i1-i0;
  hipStream_t st = (hipStream_t)fd_ed25519_hip_engine_stream( s->eng );
  unsigned long lo, hi, bytes;
  batch_span( j, i0, i1, &lo, &hi, &bytes );
  unsigned char const * dmsgs;
#ifndef FD_ED25519_HIP_AB_POOL_PARALLEL_H2D
  /* One batch crosses the link at a time: this batch's copies start once
     the previous batch's are done (its kernels still overlap them).  Two
     batches copying at once split the link between two DMA streams and
     move fewer bytes in total than one (the host-fed rate fell to ~46M/s
     with 3 slots, 69M/s with 2, depending on where the slots' streams
     land on the device's hardware queues). */
  if( j->h2d_tail ) TCHK( hipStreamWaitEvent( st, j->h2d_tail, 0U ), "hipStreamWaitEvent(h2d)" );
#endif
  if( j->direct_in && span_direct( pl, hi-lo, bytes ) ) {
    if( hi>lo ) TCHK( hipMemcpyAsync( s->d_msgs, j->msgs + lo, hi-lo, hipMemcpyHostToDevice, st ), "H2D msgs" );
    TCHK( hipMemcpyAsync( s->d_off,  j->msg_off + i0, 8UL*cnt,  hipMemcpyHostToDevice, st ), "H2D off"  );
    TCHK( hipMemcpyAsync( s->d_sz,   j->msg_sz  + i0, 4UL*cnt,  hipMemcpyHostToDevice, st ), "H2D sz"   );
    TCHK( hipMemcpyAsync( s->d_sigs, j->sigs + 64UL*i0, 64UL*cnt, hipMemcpyHostToDevice, st ), "H2D sigs" );
    TCHK( hipMemcpyAsync( s->d_pubs, j->pubs + 32UL*i0, 32UL*cnt, hipMemcpyHostToDevice, st ), "H2D pubs" );
    j->st.direct_batches++;
    j->st.h2d_bytes += (hi-lo) + 108UL*cnt;
    dmsgs = s->d_msgs - lo;   /* msg_off[i] indexes the span from its start */
  } else {
    /* pack into pinned staging: [sigs | pubs | off | sz | msgs] */
    if( bytes>pl->msg_cap ) {
      fd_ed25519_hip_private_set_error( "pool: a batch's messages exceed the pool's msg_cap" );
      return FD_ED25519_HIP_ERR_INVAL;
    }
    if( !s->h_stage )
      TCHK( hipHostMalloc( (void **)&s->h_stage, 108UL*pl->batch_sigs + pl->msg_cap + 64UL, hipHostMallocDefault ),
            "hipHostMalloc(pool stage)" );
    unsigned char * h = s->h_stage;
    memcpy( h,               j->sigs + 64UL*i0, 64UL*cnt );
    memcpy( h + 64UL*cnt,    j->pubs + 32UL*i0, 32UL*cnt );
    unsigned long * off = (unsigned long *)(h + 96UL*cnt);
    unsigned int *  sz  = (unsigned int  *)(h + 104UL*cnt);
    unsigned char * m   = h + 108UL*cnt;
    unsigned long pos = 0UL;
    for( unsigned long i=i0; i<i1; i++ ) {
      unsigned long k = i-i0;
      if( j->msg_sz[i] ) memcpy( m + pos, j->msgs + j->msg_off[i], j->msg_sz[i] );
      off[k] = pos; sz[k] = j->msg_sz[i];
      pos += j->msg_sz[i];
    }
    TCHK( hipMemcpyAsync( s->d_sigs, h,            64UL*cnt, hipMemcpyHostToDevice, st ), "H2D sigs" );
    TCHK( hipMemcpyAsync( s->d_pubs, h + 64UL*cnt, 32UL*cnt, hipMemcpyHostToDevice, st ), "H2D pubs" );
    TCHK( hipMemcpyAsync( s->d_off,  off,          8UL*cnt,  hipMemcpyHostToDevice, st ), "H2D off"  );
    TCHK( hipMemcpyAsync( s->d_sz,   sz,           4UL*cnt,  hipMemcpyHostToDevice, st ), "H2D sz"   );
    if( pos ) TCHK( hipMemcpyAsync( s->d_msgs, m, pos, hipMemcpyHostToDevice, st ), "H2D msgs" );
    j->st.staged_batches++;
    j->st.h2d_bytes += pos + 108UL*cnt;
    dmsgs = s->d_msgs;
  }
  TCHK( hipEventRecord( s->ev_h2d, st ), "hipEventRecord(h2d)" );
  j->h2d_tail = s->ev_h2d;
#ifdef FD_ED25519_HIP_HOST_FAULT
  /* test build only (tests/test_gpu_pool_fault.py): the second batch's
     launch fails after its copies from the caller's arrays are enqueued */
  if( b==1UL ) {
    fd_ed25519_hip_private_set_error( "pool: injected launch failure (fault-injection build)" );
    return FD_ED25519_HIP_ERR_HIP - (int)hipErrorLaunchFailure;
  }
#endif
  int err = fd_ed25519_hip_verify_dev( s->eng, cnt, dmsgs, s->d_off, s->d_sz, s->d_sigs, s->d_pubs, s->d_out, st );
  if( err ) return err;
  if( !j->direct_out && !s->h_out )
    TCHK( hipHostMalloc( (void **)&s->h_out, pl->batch_sigs, hipHostMallocDefault ), "hipHostMalloc(pool out)" );
  signed char * dst = j->direct_out ? j->out + i0 : s->h_out;
  TCHK( hipMemcpyAsync( dst, s->d_out, cnt, hipMemcpyDeviceToHost, st ), "D2H codes" );
  TCHK( hipEventRecord( s->ev, st ), "hipEventRecord" );
  s->i0 = i0; s->i1 = i1; s->busy = 1;
  return FD_ED25519_HIP_OK;
}

/* A batch whose enqueue failed part way may have left copies from or into
   the caller's page-locked arrays on the slot's stream: they finish before
   the error is reported, so pool_run never returns while DMA may still
   touch memory the caller is free to release. */
static int
pool_submit( pool_job_t * j, pool_slot_t * s, unsigned long b ) {
  int err = pool_enqueue( j, s, b );
  if( err ) hipStreamSynchronize( (hipStream_t)fd_ed25519_hip_engine_stream( s->eng ) );
  return err;
}

static void *
pool_main( void * arg ) {
  pool_job_t * j = (pool_job_t *)arg;
  fd_ed25519_hip_pool_t * pl = j->pool;
  int dev = pl->device[ j->rank ];
  pin_near_device( dev );
  if( hipSetDevice( dev )!=hipSuccess ) {
    j->err = tile_fail( "hipSetDevice", hipErrorInvalidDevice );
    snprintf( j->errmsg, sizeof(j->errmsg), "%s", fd_ed25519_hip_last_error() );
    return NULL;
  }
  pool_slot_t * slot = pl->slot[ j->rank ];
  unsigned sc = pl->slot_cnt, ranks = pl->device_cnt;
  unsigned long nb = (j->n + pl->batch_sigs - 1UL) / pl->batch_sigs;
  unsigned long b_sub = j->rank, b_done = j->rank;
  unsigned next = 0U, oldest = 0U;
  while( b_done<nb ) {
    pool_slot_t * s = &slot[ next ];
    if( !j->err && b_sub<nb && !s->busy ) {
      int err = pool_submit( j, s, b_sub );
      if( err ) {   /* drain what is in flight */
        j->err = err;
        snprintf( j->errmsg, sizeof(j->errmsg), "%s", fd_ed25519_hip_last_error() );
        continue;
      }
      b_sub += ranks;
      next = (next+1U) % sc;
      continue;
    }
    pool_slot_t * d = &slot[ oldest ];
    if( !d->busy ) break;   /* an error stopped submission and everything drained */
    hipError_t e = hipEventSynchronize( d->ev );
    if( e!=hipSuccess && !j->err ) {
      j->err = tile_fail( "pool batch", e );
      snprintf( j->errmsg, sizeof(j->errmsg), "%s", fd_ed25519_hip_last_error() );
    }
    if( !j->direct_out && e==hipSuccess ) memcpy( j->out + d->i0, d->h_out, d->i1 - d->i0 );
    d->busy = 0;
    oldest = (oldest+1U) % sc;
    b_done += ranks;
  }
  return NULL;
}

int
fd_ed25519_hip_pool_run( fd_ed25519_hip_pool_t * pl, unsigned long n, unsigned char const * msgs,
                         unsigned long const * msg_off, unsigned int const * msg_sz, unsigned char const * sigs,
                         unsigned char const * pubs, signed char * out, double * seconds,
                         fd_ed25519_hip_pool_stats_t * stats ) {
  if( !pl || !out ) return FD_ED25519_HIP_ERR_INVAL;
  if( n && (!msg_off || !msg_sz || !sigs || !pubs || !msgs) ) return FD_ED25519_HIP_ERR_INVAL;
  pool_job_t job[ POOL_DEV_MAX ];
  pthread_t  th[ POOL_DEV_MAX ];
  int direct_in  = n && host_locked( msgs ) && host_locked( msg_off ) && host_locked( msg_sz ) &&
                   host_locked( sigs ) && host_locked( pubs );
  int direct_out = n && host_locked( out );
  double t0 = now_s();
  unsigned started = 0U;
  int err = 0;
  for( unsigned r=0U; r<pl->device_cnt; r++ ) {
    memset( &job[r], 0, sizeof(job[r]) );
    job[r].pool = pl; job[r].rank = r; job[r].n = n; job[r].msgs = msgs; job[r].msg_off = msg_off;
    job[r].msg_sz = msg_sz; job[r].sigs = sigs; job[r].pubs = pubs; job[r].out = out;
    job[r].direct_in = direct_in; job[r].direct_out = direct_out;
    if( pthread_create( &th[r], NULL, pool_main, &job[r] ) ) { err = FD_ED25519_HIP_ERR_NOMEM; break; }
    started++;
  }
  if( stats ) memset( stats, 0, sizeof(*stats) );
  for( unsigned r=0U; r<started; r++ ) {
    pthread_join( th[r], NULL );
    if( job[r].err && !err ) { err = job[r].err; fd_ed25519_hip_private_set_error( job[r].errmsg ); }
    if( stats ) {
      stats->direct_batches += job[r].st.direct_batches;
      stats->staged_batches += job[r].st.staged_batches;
      stats->h2d_bytes      += job[r].st.h2d_bytes;
    }
  }
  if( seconds ) *seconds = now_s() - t0;
  return err;
}

int
fd_ed25519_hip_pool_verify( int const * devices, unsigned device_cnt, unsigned slot_cnt, unsigned long batch_sigs,
                            unsigned long n, unsigned char const * msgs, unsigned long const * msg_off,
                            unsigned int const * msg_sz, unsigned char const * sigs, unsigned char const * pubs,
                            signed char * out, double * seconds ) {
  if( !batch_sigs ) return FD_ED25519_HIP_ERR_INVAL;
  /* capacity: the largest span of a batch */
  unsigned long cap = 1UL;
  pool_job_t tmp;
  memset( &tmp, 0, sizeof(tmp) );
  tmp.msg_off = msg_off; tmp.msg_sz = msg_sz;
  for( unsigned long i0=0UL; n && msg_off && msg_sz && i0<n; i0+=batch_sigs ) {
    unsigned long lo, hi, bytes;
    batch_span( &tmp, i0, i0+batch_sigs<n ? i0+batch_sigs : n, &lo, &hi, &bytes );
    unsigned long need = hi-lo<=2UL*bytes + 65536UL ? hi-lo : bytes;
    if( need>cap ) cap = need;
  }
  fd_ed25519_hip_pool_t * pl = fd_ed25519_hip_pool_new( devices, device_cnt, slot_cnt, batch_sigs, cap );
  if( !pl ) return FD_ED25519_HIP_ERR_INVAL;
  double t0 = now_s();
  int err = fd_ed25519_hip_pool_run( pl, n, msgs, msg_off, msg_sz, sigs, pubs, out, NULL, NULL );
  fd_ed25519_hip_pool_delete( pl );
  if( seconds ) *seconds = now_s() - t0;
  return err;
}

double
fd_ed25519_hip_h2d_gbps( int device, unsigned long bytes, unsigned reps ) {
  if( !bytes || !reps || hipSetDevice( device )!=hipSuccess ) return 0.0;
  void * h = NULL, * d = NULL;
  hipStream_t st = NULL;
  double r = 0.0;
  if( hipHostMalloc( &h, bytes, hipHostMallocDefault )==hipSuccess && hipMalloc( &d, bytes )==hipSuccess &&
      hipStreamCreateWithFlags( &st, hipStreamNonBlocking )==hipSuccess ) {
    memset( h, 0x5a, bytes );
    int ok = hipMemcpyAsync( d, h, bytes, hipMemcpyHostToDevice, st )==hipSuccess &&
             hipStreamSynchronize( st )==hipSuccess;   /* warm-up */
    double t0 = now_s();
    for( unsigned i=0U; ok && i<reps; i++ ) ok = hipMemcpyAsync( d, h, bytes, hipMemcpyHostToDevice, st )==hipSuccess;
    ok = ok && hipStreamSynchronize( st )==hipSuccess;
    double dt = now_s() - t0;
    if( ok && dt>0.0 ) r = (double)bytes * reps / dt * 1e-9;
  }
  if( st ) hipStreamDestroy( st );
  hipFree( d ); hipHostFree( h );
  return r;
}
