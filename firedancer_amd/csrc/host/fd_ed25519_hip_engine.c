/* fd_ed25519_hip_engine.c -- plain-C host runtime of libfd_ed25519_hip.

   Owns the device, stream and memory of an engine, batches host requests
   into pinned SoA staging buffers, and drives the HIP kernel shim
   (fd_ed25519_kernels.hip) through the C-ABI in fd_ed25519_hip_internal.h.
   Also provides the drop-in fd_ed25519_verify /
   fd_ed25519_verify_batch_single_msg / fd_ed25519_strerror symbols on a
   lazily created process-wide engine.

   HBM layout of an engine (sized once at creation, no per-call device
   allocation on the device-resident path):
     btab   129 x 36 int32            base-point table [0..128]B (LDS image, signing)
     btab16 32769 x 32 int32          base-point table [0..2^15]B (full-length verify, 4.2 MB)
     btabw  2 x 2^24 x 32 int32       [0..2^24)B, [0..2^24)[2^144]B (half-size verify, 2 x 2 GiB,
                                      shared by the engines of a device)
     atab   dsm waves x 163840 B      per-lane [1..8](-A), [1..8](-+R) tables
     work   max_chunk x 280 B         k, flags, half-size scalars, decoded A and R, lists per signature
     in/out staging for the host API  grown on demand */

#define _GNU_SOURCE
#include "../../../include/fd_ed25519_hip.h"
#include "../fd_ed25519_hip_internal.h"

#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define FD_ED25519_HIP_TIMING_MAX 256

_Static_assert( FD_ED25519_HIP_PHASE_CNT==FD_ED25519_PHASE_CNT, "public and internal phase counts differ" );

struct fd_ed25519_hip_engine {
  int          device;
  int          flags;
  hipStream_t  stream;
  int          cu_cnt;
  int          dsm_blocks_per_cu;
  uint32_t     dsm_grid;
  uint64_t     quad_max;   /* chunks of at most this many signatures run dsm4 */
  uint64_t     oct_max;    /* ... and of at most this many, dsm8            */
  uint64_t     r16_max;    /* ... and of at most this many, dsm16           */
  uint64_t     max_chunk;
  uint64_t     device_bytes;
  char         arch[ 64 ];
  int          pci[ 3 ];   /* domain, bus, device */

  int32_t *    d_btab;
  int32_t *    d_btab16;     /* [0..2^15]B, the verify kernels' wide B table  */
  int32_t *    d_btab8[2];   /* A/B build only (FD_ED25519_AB_LDS_BASE): the LDS-staged tables */
  int32_t *    btabw[2];    /* shared per device: [0..2^24)B, [0..2^24)[2^144]B */
  int32_t *    btabs[2][8]; /* shared per device: dsm16s<4>'s and <8>'s compact tables, when acquired */
  /* Pipeline lanes: the per-chunk scratch of a chunk in flight, and the
     streams its phases run on.  Lane 0 runs on the caller's stream (or the
     engine's); the chunks of a multi-chunk call alternate between lane 0
     and lane 1 (its own streams and scratch, made on the first such call),
     so one chunk's hash / scalar / decode run beside the previous chunk's
     dsm and fill the tail of that persistent kernel (its work items last
     ~1 ms, so its last ~0.46 ms per launch leaves SIMDs idle). */
  struct {
    void *      d_atab;      /* dsm lane tables (and the dsm4 quad tables)  */
    uint8_t *   d_work;      /* one allocation carved into the work arrays */
    uint32_t *  d_k;
    uint8_t *   d_sflag;
    uint8_t *   d_pflag;
    int32_t *   d_pts;
    uint32_t *  d_fix;       /* scalar -> dsm full-length list */
    uint32_t *  d_hs;        /* half-size scalars             */
    uint8_t *   d_hflag;
    uint32_t *  d_perm;      /* hash order (length-sorted) */
    uint32_t *  d_hist;      /* counting-sort scratch      */
    hipStream_t stream;      /* lane 1 only (lane 0: the call's stream)       */
    /* overlap: a large chunk's decode (A and R need neither the hash nor
       the scalars) runs on a side stream beside hash + scalar, dsm after */
    hipStream_t side;
    hipEvent_t  ev_dfork, ev_djoin;
  } lane[ 2 ];
  int          overlap;
  int          pipeline;     /* multi-chunk calls alternate lanes */
  hipEvent_t   ev_start, ev_end;   /* lane 1 after the call's prior work; the call's stream after lane 1 */

  /* host-API staging (pinned host + device mirrors), grown on demand */
  uint64_t     st_sig_cap;   /* signatures */
  uint64_t     st_msg_cap;   /* message bytes */
  uint64_t     st_txn_cap;   /* transactions */
  uint8_t *    h_msgs;  uint8_t *  d_msgs;
  uint64_t *   h_off;   uint64_t * d_off;
  uint32_t *   h_sz;    uint32_t * d_sz;
  uint8_t *    h_sigs;  uint8_t *  d_sigs;
  uint8_t *    h_pubs;  uint8_t *  d_pubs;
  int8_t *     h_out;   int8_t *   d_out;
  uint32_t *   h_tfirst; uint32_t * d_tfirst;
  uint32_t *   h_tcnt;  uint32_t * d_tcnt;
  int8_t *     h_tout;  int8_t *   d_tout;

  /* per-phase event timing (bench / profiling) */
  int          timing;
  int          tm_ev_init;
  int          tm_cnt;
  hipEvent_t   tm_ev[ FD_ED25519_HIP_TIMING_MAX ][ FD_ED25519_PHASE_CNT+1 ];
};

static __thread char fd_ed25519_hip_errbuf[ 256 ];

char const *
fd_ed25519_hip_last_error( void ) {
  return fd_ed25519_hip_errbuf;
}

/* for the other host files of the library (fd_ed25519_hip_tile.c) */
void
fd_ed25519_hip_private_set_error( char const * msg ) {
  snprintf( fd_ed25519_hip_errbuf, sizeof(fd_ed25519_hip_errbuf), "%s", msg );
}

static int
hip_fail( hipError_t err, char const * what ) {
  snprintf( fd_ed25519_hip_errbuf, sizeof(fd_ed25519_hip_errbuf), "%s: %s (%d)", what,
            hipGetErrorString( err ), (int)err );
  return FD_ED25519_HIP_ERR_HIP - (int)err;
}

#define HIPCHK( call, what ) do {                     \
    hipError_t _e = (call);                           \
    if( _e!=hipSuccess ) return hip_fail( _e, what ); \
  } while(0)

char const *
fd_ed25519_hip_strerror( int status ) {
  if( status==FD_ED25519_HIP_OK        ) return "ok";
  if( status==FD_ED25519_HIP_ERR_INVAL ) return "invalid argument";
  if( status==FD_ED25519_HIP_ERR_NOMEM ) return "out of memory";
  if( status<=FD_ED25519_HIP_ERR_HIP   ) return hipGetErrorString( (hipError_t)(FD_ED25519_HIP_ERR_HIP - status) );
  return "unknown";
}

/* The half-size form's base tables, [0..2^24)B and [0..2^24)[2^144]B
   (2 GiB each), are shared by every engine of a device: generated by the
   first engine (with a 640 MiB scratch freed right after), freed with the
   last.  The compact pair at radix 2^16 (8 MiB each,
   FD_ED25519_HIP_FLAG_COMPACT_TABLES) is shared the same way; kind 0 is
   the wide pair, kind 1 the compact one. */
#define FD_ED25519_HIP_MAX_DEV 64
static pthread_mutex_t btabw_lock = PTHREAD_MUTEX_INITIALIZER;
static struct { int refs; int32_t * tab[2]; } btabw[ 2 ][ FD_ED25519_HIP_MAX_DEV ];

static int
btab_kind_bits( int kind ) {
  return kind ? FD_ED25519_BTABC_BITS : FD_ED25519_BTABW_BITS;
}

static size_t
btabw_bytes( int kind ) {
  return sizeof(int32_t) * ((size_t)1 << btab_kind_bits( kind )) * FD_ED25519_BTAB16_STRIDE;
}

static int
btabw_acquire( int device, int kind, hipStream_t stream, int32_t * tab[2] ) {
  if( device<0 || device>=FD_ED25519_HIP_MAX_DEV ) {
    snprintf( fd_ed25519_hip_errbuf, sizeof(fd_ed25519_hip_errbuf), "device %d out of range", device );
    return FD_ED25519_HIP_ERR_INVAL;
  }
  pthread_mutex_lock( &btabw_lock );
  int rc = FD_ED25519_HIP_OK;
  int bits = btab_kind_bits( kind );
  if( !btabw[kind][device].refs ) {
    int32_t * t[2] = { NULL, NULL };
    int32_t * scratch = NULL;
    hipError_t he = hipMalloc( (void **)&t[0], btabw_bytes( kind ) );
    if( he==hipSuccess ) he = hipMalloc( (void **)&t[1], btabw_bytes( kind ) );
    if( he==hipSuccess ) he = hipMalloc( (void **)&scratch, sizeof(int32_t) * (((size_t)1 << bits) * 10 + 64) );
    if( he==hipSuccess ) he = (hipError_t)fd_ed25519_hip_launch_gen_btabw( t[0], 0, bits, scratch, stream );
    if( he==hipSuccess ) he = (hipError_t)fd_ed25519_hip_launch_gen_btabw( t[1], FD_ED25519_BTABW_SHIFT, bits, scratch, stream );
    if( he==hipSuccess ) he = hipStreamSynchronize( stream );
    hipFree( scratch );
    if( he!=hipSuccess ) {
      hipFree( t[0] ); hipFree( t[1] );
      rc = hip_fail( he, "base tables (btabw)" );
    } else {
      btabw[kind][device].tab[0] = t[0];
      btabw[kind][device].tab[1] = t[1];
    }
  }
  if( rc==FD_ED25519_HIP_OK ) {
    btabw[kind][device].refs++;
    tab[0] = btabw[kind][device].tab[0];
    tab[1] = btabw[kind][device].tab[1];
  }
  pthread_mutex_unlock( &btabw_lock );
  return rc;
}

/* dsm16s<S>'s compact tables at offsets 2^(CB q), q < S (8 MiB each; CB
   = 72 for S = 4, 32 for S = 8), shared per device like the pairs above,
   made with the drop-in engines (a pipe's on demand).  Set 0: S = 4, set
   1: S = 8. */
static struct { int refs; int32_t * tab[8]; } btabs[ 2 ][ FD_ED25519_HIP_MAX_DEV ];

static int split_set( int waves ) { return waves==8 ? 1 : 0; }
static int split_cb( int waves ) { return waves==8 ? 32 : 72; }

static int
btabs_acquire( int device, int waves, hipStream_t stream, int32_t * tab[8] ) {
  int set = split_set( waves );
  pthread_mutex_lock( &btabw_lock );
  int rc = FD_ED25519_HIP_OK;
  if( !btabs[set][device].refs ) {
    int32_t * t[8] = { NULL };
    int32_t * scratch = NULL;
    hipError_t he = hipSuccess;
    for( int q=0; q<waves && he==hipSuccess; q++ ) he = hipMalloc( (void **)&t[q], btabw_bytes( 1 ) );
    if( he==hipSuccess ) he = hipMalloc( (void **)&scratch, sizeof(int32_t) * (((size_t)1 << FD_ED25519_BTABC_BITS) * 10 + 64) );
    for( int q=0; q<waves && he==hipSuccess; q++ )
      he = (hipError_t)fd_ed25519_hip_launch_gen_btabw( t[q], split_cb( waves )*q, FD_ED25519_BTABC_BITS, scratch, stream );
    if( he==hipSuccess ) he = hipStreamSynchronize( stream );
    hipFree( scratch );
    if( he!=hipSuccess ) {
      for( int q=0; q<8; q++ ) hipFree( t[q] );
      rc = hip_fail( he, "base tables (dsm16s)" );
    } else {
      for( int q=0; q<8; q++ ) btabs[set][device].tab[q] = t[q];
    }
  }
  if( rc==FD_ED25519_HIP_OK ) {
    btabs[set][device].refs++;
    for( int q=0; q<8; q++ ) tab[q] = btabs[set][device].tab[q];
  }
  pthread_mutex_unlock( &btabw_lock );
  return rc;
}

static void
btabs_release( int device, int waves ) {
  int set = split_set( waves );
  pthread_mutex_lock( &btabw_lock );
  if( btabs[set][device].refs>0 && !--btabs[set][device].refs ) {
    for( int q=0; q<8; q++ ) { hipFree( btabs[set][device].tab[q] ); btabs[set][device].tab[q] = NULL; }
  }
  pthread_mutex_unlock( &btabw_lock );
}

unsigned long
fd_ed25519_hip_shared_device_bytes( int device ) {
  if( device<0 || device>=FD_ED25519_HIP_MAX_DEV ) return 0UL;
  pthread_mutex_lock( &btabw_lock );
  unsigned long b = 0UL;
  for( int kind=0; kind<2; kind++ ) if( btabw[kind][device].refs ) b += 2UL*btabw_bytes( kind );
  if( btabs[0][device].refs ) b += 4UL*btabw_bytes( 1 );
  if( btabs[1][device].refs ) b += 8UL*btabw_bytes( 1 );
  pthread_mutex_unlock( &btabw_lock );
  return b;
}

static void
btabw_release( int device, int kind ) {
  pthread_mutex_lock( &btabw_lock );
  if( btabw[kind][device].refs>0 && !--btabw[kind][device].refs ) {
    hipFree( btabw[kind][device].tab[0] );
    hipFree( btabw[kind][device].tab[1] );
    btabw[kind][device].tab[0] = btabw[kind][device].tab[1] = NULL;
  }
  pthread_mutex_unlock( &btabw_lock );
}

static int
engine_btab_kind( fd_ed25519_hip_engine_t const * e ) {
  return (e->flags & FD_ED25519_HIP_FLAG_COMPACT_TABLES) ? 1 : 0;
}

/* The device's stream set.  A process gets GPU_MAX_HW_QUEUES hardware
   queues per device (4 by default) and HIP binds each new stream to one of
   them; which one depends on every stream created before, so a feeder's
   slots could land on a shared queue or not depending on what else the
   process had made first (round 2: the host-fed pool at 47-57M/s or 70M/s
   by creation order).  Instead the library creates one stream per hardware
   queue per device, once, and every engine stream (its main stream, its
   second lane's, the decode side stream) is drawn from that set: the least
   used ones first, distinct within an engine.  Engines sharing a stream
   order their work together, which costs nothing while one of them is
   idle; concurrently busy engines get distinct streams as long as there
   are queues for them, which is the most concurrency the device gives the
   process anyway.  The set's size follows HIP's own GPU_MAX_HW_QUEUES
   (default 4, capped at 32); the streams live as long as the process. */
#define FD_ED25519_HIP_STREAM_SET_MAX 32
static pthread_mutex_t sset_lock = PTHREAD_MUTEX_INITIALIZER;
static struct {
  int         cnt;
  hipStream_t s[ FD_ED25519_HIP_STREAM_SET_MAX ];
  int         users[ FD_ED25519_HIP_STREAM_SET_MAX ];
} sset[ FD_ED25519_HIP_MAX_DEV ];

static int
stream_set_size( void ) {
  char const * q = getenv( "GPU_MAX_HW_QUEUES" );   /* the HIP runtime's knob, not the library's */
  long n = q ? strtol( q, NULL, 0 ) : 4L;
  if( n<1L ) n = 1L;
  if( n>FD_ED25519_HIP_STREAM_SET_MAX ) n = FD_ED25519_HIP_STREAM_SET_MAX;
  return (int)n;
}

/* a stream of the device's set, the least used one that is not in
   avoid[0..avoid_cnt) (if every stream is, the least used one) */
static int
stream_acquire( int device, hipStream_t const * avoid, int avoid_cnt, hipStream_t * out ) {
  if( device<0 || device>=FD_ED25519_HIP_MAX_DEV ) return FD_ED25519_HIP_ERR_INVAL;
#ifdef FD_ED25519_HIP_AB_FRESH_STREAMS
  /* A/B build only (tools/build_variant.sh): a new stream per request, as
     in round 2 */
  (void)avoid; (void)avoid_cnt;
  { hipError_t he = hipStreamCreateWithFlags( out, hipStreamNonBlocking );
    return he==hipSuccess ? FD_ED25519_HIP_OK : hip_fail( he, "stream" ); }
#endif
  pthread_mutex_lock( &sset_lock );
  int rc = FD_ED25519_HIP_OK;
  if( !sset[device].cnt ) {
    int n = stream_set_size();
#ifdef FD_ED25519_HIP_AB_SET_SKIP
    /* A/B build only: streams created (and never used) before the set */
    for( int i=0; i<FD_ED25519_HIP_AB_SET_SKIP; i++ ) { hipStream_t t; (void)hipStreamCreateWithFlags( &t, hipStreamNonBlocking ); }
#endif
    for( int i=0; i<n; i++ ) {
      hipError_t he = hipStreamCreateWithFlags( &sset[device].s[i], hipStreamNonBlocking );
      if( he!=hipSuccess ) {
        for( int j=0; j<i; j++ ) hipStreamDestroy( sset[device].s[j] );
        rc = hip_fail( he, "stream set" );
        break;
      }
      sset[device].users[i] = 0;
    }
    if( !rc ) sset[device].cnt = n;
  }
  if( !rc ) {
    int best = -1, best_avoided = -1;
    for( int i=0; i<sset[device].cnt; i++ ) {
      int avoided = 0;
      for( int j=0; j<avoid_cnt; j++ ) if( avoid[j]==sset[device].s[i] ) avoided = 1;
      if( avoided ) { if( best_avoided<0 || sset[device].users[i]<sset[device].users[best_avoided] ) best_avoided = i; }
      else if( best<0 || sset[device].users[i]<sset[device].users[best] ) best = i;
    }
    if( best<0 ) best = best_avoided;
    sset[device].users[best]++;
    *out = sset[device].s[best];
  }
  pthread_mutex_unlock( &sset_lock );
  return rc;
}

static void
stream_release( int device, hipStream_t st ) {
  if( !st || device<0 || device>=FD_ED25519_HIP_MAX_DEV ) return;
#ifdef FD_ED25519_HIP_AB_FRESH_STREAMS
  hipStreamDestroy( st );
  return;
#endif
  pthread_mutex_lock( &sset_lock );
  for( int i=0; i<sset[device].cnt; i++ )
    if( sset[device].s[i]==st && sset[device].users[i]>0 ) { sset[device].users[i]--; break; }
  pthread_mutex_unlock( &sset_lock );
}

static void
engine_free( fd_ed25519_hip_engine_t * e ) {
  if( !e ) return;
  hipSetDevice( e->device );
  /* all work of the engine's streams has drained before any buffer goes:
     a failed verify_dev may have left decode queued on the side stream */
  if( e->stream ) hipStreamSynchronize( e->stream );
  for( int l=0; l<2; l++ ) {
    if( e->lane[l].stream ) hipStreamSynchronize( e->lane[l].stream );
    if( e->lane[l].side   ) hipStreamSynchronize( e->lane[l].side );
  }
  hipFree( e->d_btab ); hipFree( e->d_btab16 ); hipFree( e->d_btab8[0] ); hipFree( e->d_btab8[1] );
  for( int l=0; l<2; l++ ) { hipFree( e->lane[l].d_atab ); hipFree( e->lane[l].d_work ); }
  if( e->btabw[0] ) btabw_release( e->device, engine_btab_kind( e ) );
  if( e->btabs[0][0] ) btabs_release( e->device, 4 );
  if( e->btabs[1][0] ) btabs_release( e->device, 8 );
  hipFree( e->d_msgs ); hipFree( e->d_off ); hipFree( e->d_sz ); hipFree( e->d_sigs ); hipFree( e->d_pubs );
  hipFree( e->d_out );  hipFree( e->d_tfirst ); hipFree( e->d_tcnt ); hipFree( e->d_tout );
  hipHostFree( e->h_msgs ); hipHostFree( e->h_off ); hipHostFree( e->h_sz ); hipHostFree( e->h_sigs );
  hipHostFree( e->h_pubs ); hipHostFree( e->h_out ); hipHostFree( e->h_tfirst ); hipHostFree( e->h_tcnt );
  hipHostFree( e->h_tout );
  if( e->tm_ev_init )
    for( int i=0; i<FD_ED25519_HIP_TIMING_MAX; i++ )
      for( int j=0; j<=FD_ED25519_PHASE_CNT; j++ ) hipEventDestroy( e->tm_ev[i][j] );
  for( int l=0; l<2; l++ ) {
    if( e->lane[l].side ) {
      hipEventDestroy( e->lane[l].ev_dfork ); hipEventDestroy( e->lane[l].ev_djoin );
      stream_release( e->device, e->lane[l].side );
    }
    stream_release( e->device, e->lane[l].stream );
  }
  if( e->lane[1].d_work ) { hipEventDestroy( e->ev_start ); hipEventDestroy( e->ev_end ); }
  stream_release( e->device, e->stream );
  free( e );
}

void
fd_ed25519_hip_engine_delete( fd_ed25519_hip_engine_t * engine ) {
  engine_free( engine );
}

/* a lane's dsm scratch: the one-lane kernel's tables for every wave of
   its grid, and room for the quad kernels' tables (4 x 864 B per
   signature, dsm4 / dsm8) for every chunk size that takes them */
static size_t
lane_atab_bytes( fd_ed25519_hip_engine_t const * e ) {
  size_t wide = (size_t)e->dsm_grid * (FD_ED25519_VERIFY_BLOCK / 64) * fd_ed25519_hip_atab_bytes_per_wave();
  uint64_t qn = e->max_chunk < FD_ED25519_HIP_QUAD_MAX_DEFAULT ? e->max_chunk : FD_ED25519_HIP_QUAD_MAX_DEFAULT;
  size_t quad = (size_t)qn * 4UL * FD_ED25519_QUAD_LANE_BYTES;
  return wide > quad ? wide : quad;
}

/* a lane's scratch (dsm lane tables + work arrays for max_chunk
   signatures); lane 1 also gets its stream and the join events.  All or
   nothing: the lane is usable once d_work is set, which happens last. */
static int
lane_alloc( fd_ed25519_hip_engine_t * e, int l ) {
  size_t atab_sz = lane_atab_bytes( e );
  size_t work_sz = (size_t)e->max_chunk * FD_ED25519_WORK_BYTES_PER_SIG + 1024;
  void * atab = NULL; uint8_t * work = NULL;
  hipStream_t st = NULL; hipEvent_t ev0 = NULL, ev1 = NULL;
  hipError_t he = hipMalloc( &atab, atab_sz );
  if( he==hipSuccess ) he = hipMalloc( (void **)&work, work_sz );
  int serr = FD_ED25519_HIP_OK;
  if( l ) {
    if( he==hipSuccess ) {
      hipStream_t avoid[3] = { e->stream, e->lane[0].side, NULL };
      serr = stream_acquire( e->device, avoid, 2, &st );
    }
    if( he==hipSuccess && !serr ) he = hipEventCreateWithFlags( &ev0, hipEventDisableTiming );
    if( he==hipSuccess && !serr ) he = hipEventCreateWithFlags( &ev1, hipEventDisableTiming );
  }
  if( he!=hipSuccess || serr ) {
    if( ev1 ) hipEventDestroy( ev1 );
    if( ev0 ) hipEventDestroy( ev0 );
    stream_release( e->device, st );
    hipFree( work ); hipFree( atab );
    return serr ? serr : hip_fail( he, "lane scratch" );
  }
  e->device_bytes += atab_sz + work_sz;
  uint64_t c = e->max_chunk;
  uint8_t * w = work;
  e->lane[l].d_k     = (uint32_t *)w; w += 8UL*4UL*c;
  e->lane[l].d_pts   = (int32_t  *)w; w += 2UL*20UL*4UL*c;
  e->lane[l].d_hs    = (uint32_t *)w; w += 19UL*4UL*c;
  e->lane[l].d_perm  = (uint32_t *)w; w += 4UL*c;
  e->lane[l].d_fix   = (uint32_t *)w; w += 4UL*c;
  e->lane[l].d_sflag = w;             w += c;
  e->lane[l].d_pflag = w;             w += 2UL*c;
  e->lane[l].d_hflag = w;             w += c;
  w = (uint8_t *)(((uintptr_t)w + 255UL) & ~(uintptr_t)255UL);
  e->lane[l].d_hist  = (uint32_t *)w; /* 2*SORT_BUCKETS words + fix count inside the 1024-byte slack */
  e->lane[l].d_atab  = atab;
  if( l ) { e->lane[l].stream = st; e->ev_start = ev0; e->ev_end = ev1; }
  e->lane[l].d_work  = work;
  return FD_ED25519_HIP_OK;
}

static int
engine_init( fd_ed25519_hip_engine_t * e, int device, uint64_t max_chunk, int flags ) {
  e->device    = device;
  e->flags     = flags;
  e->max_chunk = max_chunk ? max_chunk : (1UL<<20);
  HIPCHK( hipSetDevice( device ), "hipSetDevice" );
  hipDeviceProp_t prop;
  HIPCHK( hipGetDeviceProperties( &prop, device ), "hipGetDeviceProperties" );
  e->cu_cnt = prop.multiProcessorCount;
  snprintf( e->arch, sizeof(e->arch), "%.63s", prop.gcnArchName );
  e->pci[0] = prop.pciDomainID; e->pci[1] = prop.pciBusID; e->pci[2] = prop.pciDeviceID;
  if( strncmp( prop.gcnArchName, "gfx950", 6 ) ) {
    snprintf( fd_ed25519_hip_errbuf, sizeof(fd_ed25519_hip_errbuf),
              "device %d is %.63s; libfd_ed25519_hip is built for gfx950 only", device, prop.gcnArchName );
    return FD_ED25519_HIP_ERR_INVAL;
  }
  int serr = stream_acquire( device, NULL, 0, &e->stream );
  if( serr ) return serr;

  int bpc = 0;
  HIPCHK( (hipError_t)fd_ed25519_hip_verify_occupancy( &bpc ), "occupancy query" );
  if( bpc<1 ) bpc = 1;
  e->dsm_blocks_per_cu = bpc;
  e->dsm_grid = (uint32_t)(bpc * e->cu_cnt);
  /* the dsm launch never uses more blocks than a chunk needs (one wave of
     64 beyond it, fd_ed25519_hip_launch_phase): an engine of small chunks
     (a tile's or a pipe's slot) sizes its grid, and so its lane tables, to
     that -- ~14 MB instead of ~335 MB for a 4096-signature slot */
  uint64_t need = (e->max_chunk + 64UL + FD_ED25519_VERIFY_BLOCK - 1UL) / FD_ED25519_VERIFY_BLOCK;
  if( need < (uint64_t)e->dsm_grid ) e->dsm_grid = (uint32_t)need;

  size_t btab_sz = sizeof(int32_t) * FD_ED25519_BTAB_INTS;
  size_t btab16_sz = sizeof(int32_t) * (size_t)FD_ED25519_BTAB16_ENTRIES * FD_ED25519_BTAB16_STRIDE;
  size_t atab_sz = lane_atab_bytes( e );
  HIPCHK( hipMalloc( (void **)&e->d_btab, btab_sz ), "hipMalloc(btab)" );
  HIPCHK( hipMalloc( (void **)&e->d_btab16, btab16_sz ), "hipMalloc(btab16)" );
  e->device_bytes = btab_sz + btab16_sz;   /* + each lane's scratch; + the base tables shared per device */
  int lerr = lane_alloc( e, 0 );
  if( lerr ) return lerr;
  /* launch forms come from the engine flags only, never the environment */
  e->overlap  = !(flags & (FD_ED25519_HIP_FLAG_NO_OVERLAP  | FD_ED25519_HIP_FLAG_ONE_STREAM)) && FD_ED25519_HIP_OVERLAP_DEFAULT;
  e->pipeline = !(flags & (FD_ED25519_HIP_FLAG_NO_PIPELINE | FD_ED25519_HIP_FLAG_ONE_STREAM));
  /* dsm4 (a quad of lanes per signature) below the size where one lane
     per signature fills the chip; its lane tables live in the atab scratch */
  uint64_t quad_cap = atab_sz / (4UL * FD_ED25519_QUAD_LANE_BYTES);
  e->quad_max = FD_ED25519_HIP_QUAD_MAX_DEFAULT;
  e->oct_max  = FD_ED25519_HIP_OCT_MAX_DEFAULT;
  e->r16_max  = FD_ED25519_HIP_R16_MAX_DEFAULT;
  if( flags & FD_ED25519_HIP_FLAG_DSM_R16  ) { e->quad_max = ~0UL; e->oct_max = ~0UL; e->r16_max = ~0UL; }
  if( flags & FD_ED25519_HIP_FLAG_DSM_QUAD ) { e->quad_max = ~0UL; e->oct_max = 0UL; e->r16_max = 0UL; }
  if( flags & FD_ED25519_HIP_FLAG_DSM_OCT  ) { e->quad_max = ~0UL; e->oct_max = ~0UL; e->r16_max = 0UL; }
  if( flags & FD_ED25519_HIP_FLAG_DSM_WIDE ) { e->quad_max = 0UL; e->r16_max = 0UL; }
  if( e->quad_max > quad_cap ) e->quad_max = quad_cap;
  /* a throughput engine pipelines its multi-chunk calls: the second lane
     up front, so verify_dev never allocates (fd_ed25519_hip.h) */
  if( e->pipeline && e->max_chunk > FD_ED25519_HIP_QUAD_MAX_DEFAULT ) {
    lerr = lane_alloc( e, 1 );
    if( lerr ) return lerr;
  }

  int err = fd_ed25519_hip_launch_gen_btab( e->d_btab, e->stream );
  if( err ) return hip_fail( (hipError_t)err, "gen_btab launch" );
  err = fd_ed25519_hip_launch_gen_btab16( e->d_btab16, 0, e->stream );
  if( err ) return hip_fail( (hipError_t)err, "gen_btab16 launch" );
#ifdef FD_ED25519_AB_LDS_BASE
  for( int t=0; t<2; t++ ) {
    HIPCHK( hipMalloc( (void **)&e->d_btab8[t], sizeof(int32_t) * 256UL * FD_ED25519_BTAB16_STRIDE ), "hipMalloc(btab8)" );
    err = fd_ed25519_hip_launch_gen_btab8( e->d_btab8[t], t ? FD_ED25519_BTAB8_SHIFT : 0, e->stream );
    if( err ) return hip_fail( (hipError_t)err, "gen_btab8 launch" );
  }
#endif
  HIPCHK( hipStreamSynchronize( e->stream ), "gen_btab" );
  int32_t * tw[2] = { NULL, NULL };
  err = btabw_acquire( e->device, engine_btab_kind( e ), e->stream, tw );
  if( err ) return err;
  e->btabw[0] = tw[0];
  e->btabw[1] = tw[1];
  return FD_ED25519_HIP_OK;
}

fd_ed25519_hip_engine_t *
fd_ed25519_hip_engine_new( int device, unsigned long max_chunk, int flags ) {
  fd_ed25519_hip_engine_t * e = (fd_ed25519_hip_engine_t *)calloc( 1, sizeof(fd_ed25519_hip_engine_t) );
  if( !e ) { snprintf( fd_ed25519_hip_errbuf, sizeof(fd_ed25519_hip_errbuf), "calloc failed" ); return NULL; }
  if( engine_init( e, device, max_chunk, flags ) ) { engine_free( e ); return NULL; }
  return e;
}

int
fd_ed25519_hip_engine_set_forms( fd_ed25519_hip_engine_t * e, unsigned long quad_max, unsigned long oct_max ) {
  if( !e || oct_max>quad_max ) return FD_ED25519_HIP_ERR_INVAL;
  if( quad_max > lane_atab_bytes( e ) / (4UL * FD_ED25519_QUAD_LANE_BYTES) ) {
    snprintf( fd_ed25519_hip_errbuf, sizeof(fd_ed25519_hip_errbuf), "set_forms: quad_max above the lane tables' room" );
    return FD_ED25519_HIP_ERR_INVAL;
  }
  e->quad_max = quad_max;
  e->oct_max  = oct_max;
  if( e->r16_max > oct_max ) e->r16_max = oct_max;
  return FD_ED25519_HIP_OK;
}

int
fd_ed25519_hip_engine_set_r16_max( fd_ed25519_hip_engine_t * e, unsigned long n ) {
  if( !e || n>e->oct_max ) return FD_ED25519_HIP_ERR_INVAL;
  e->r16_max = n;
  return FD_ED25519_HIP_OK;
}

int
fd_ed25519_hip_engine_info( fd_ed25519_hip_engine_t const * e, fd_ed25519_hip_info_t * info ) {
  if( !e || !info ) return FD_ED25519_HIP_ERR_INVAL;
  memset( info, 0, sizeof(*info) );
  info->device            = e->device;
  info->cu_cnt            = e->cu_cnt;
  info->dsm_blocks_per_cu = e->dsm_blocks_per_cu;
  info->dsm_grid          = e->dsm_grid;
  info->max_chunk         = e->max_chunk;
  info->device_bytes      = e->device_bytes;
  info->flags             = e->flags;
  memcpy( info->arch, e->arch, sizeof(info->arch) );
  info->pci_domain        = e->pci[0];
  info->pci_bus           = e->pci[1];
  info->pci_device        = e->pci[2];
  return FD_ED25519_HIP_OK;
}

void *
fd_ed25519_hip_engine_stream( fd_ed25519_hip_engine_t * e ) {
  return e ? (void *)e->stream : NULL;
}

/* longest |d| the scalar phase may return (fd25519_half.h) */
static int
engine_half_dbits( fd_ed25519_hip_engine_t const * e ) {
  return (e->flags & FD_ED25519_HIP_FLAG_HALF_STRICT) ? 131 : 151;
}

int
fd_ed25519_hip_diag_half_scalars( fd_ed25519_hip_engine_t * e, unsigned int const * k, unsigned long n,
                                  unsigned int * out ) {
  if( !e || (n && (!k || !out)) ) return FD_ED25519_HIP_ERR_INVAL;
  if( !n ) return FD_ED25519_HIP_OK;
  HIPCHK( hipSetDevice( e->device ), "hipSetDevice" );
  uint32_t * d_k = NULL, * d_out = NULL;
  hipError_t he = hipMalloc( (void **)&d_k, 32UL * n );
  if( he==hipSuccess ) he = hipMalloc( (void **)&d_out, 48UL * n );
  if( he==hipSuccess ) he = hipMemcpyAsync( d_k, k, 32UL * n, hipMemcpyHostToDevice, e->stream );
  if( he==hipSuccess ) he = (hipError_t)fd_ed25519_hip_launch_diag_half( d_k, d_out, n, engine_half_dbits( e ), e->stream );
  if( he==hipSuccess ) he = hipMemcpyAsync( out, d_out, 48UL * n, hipMemcpyDeviceToHost, e->stream );
  if( he==hipSuccess ) he = hipStreamSynchronize( e->stream );
  hipFree( d_k ); hipFree( d_out );
  if( he!=hipSuccess ) return hip_fail( he, "diag_half_scalars" );
  return FD_ED25519_HIP_OK;
}

int
fd_ed25519_hip_engine_sync( fd_ed25519_hip_engine_t * e ) {
  if( !e ) return FD_ED25519_HIP_ERR_INVAL;
  HIPCHK( hipStreamSynchronize( e->stream ), "hipStreamSynchronize" );
  return FD_ED25519_HIP_OK;
}

/* one chunk [base,base+cnt) through the phases on lane l's scratch, on
   stream st (the call's stream for lane 0, lane 1's own stream otherwise) */
static int
verify_chunk( fd_ed25519_hip_engine_t * e, fd_ed25519_verify_params_t * p, int l,
              uint64_t base, uint64_t cnt, hipStream_t st ) {
  p->k = e->lane[l].d_k; p->sflag = e->lane[l].d_sflag; p->pflag = e->lane[l].d_pflag; p->pts = e->lane[l].d_pts;
  p->fix_list = e->lane[l].d_fix; p->fix_cnt = e->lane[l].d_hist + 2*FD_ED25519_SORT_BUCKETS;
  p->work_ctr = p->fix_cnt + 1; p->hs = e->lane[l].d_hs; p->hflag = e->lane[l].d_hflag;
  p->hist = e->lane[l].d_hist; p->atab = e->lane[l].d_atab;
  p->base  = base;
  p->n     = cnt;
  p->small = p->n > e->quad_max ? 0 : p->n <= e->r16_max ? 3 : (p->n <= e->oct_max ? 2 : 1);
  /* always true when small==3: quad_max <= the quad tables' room, which is
     below one 2.5 KB atab slot per signature; kept as the kernel's bound */
  p->full_in_prep = FD_ED25519_FULL_IN_PREP && p->small==3 && p->n <= lane_atab_bytes( e ) / (fd_ed25519_hip_atab_bytes_per_wave() / 64UL);
  p->perm  = ( p->small || p->digests ) ? NULL : e->lane[l].d_perm;   /* digests: no hash lengths to sort by */
  if( e->timing && e->tm_cnt<FD_ED25519_HIP_TIMING_MAX ) {
    /* events bracket each phase kernel on the stream it runs on */
    hipEvent_t * ev = e->tm_ev[ e->tm_cnt++ ];
    HIPCHK( hipEventRecord( ev[0], st ), "hipEventRecord" );
    for( int ph=0; ph<FD_ED25519_PHASE_CNT; ph++ ) {
      int err = fd_ed25519_hip_launch_phase( p, ph, e->dsm_grid, st );
      if( err ) return hip_fail( (hipError_t)err, "verify launch" );
      HIPCHK( hipEventRecord( ev[ph+1], st ), "hipEventRecord" );
    }
  } else if( e->overlap && !p->small ) {
    if( !e->lane[l].side ) {
      /* created on the first large chunk only: an engine that only sees
         small batches (a tile slot) keeps to one stream, since the
         device's few hardware queues are shared by every stream of the
         process and extra streams serialise the slots */
      hipStream_t avoid[2] = { e->stream, e->lane[1].stream };
      int serr = stream_acquire( e->device, avoid, 2, &e->lane[l].side );
      if( serr ) return serr;
      HIPCHK( hipEventCreateWithFlags( &e->lane[l].ev_dfork, hipEventDisableTiming ), "hipEventCreate" );
      HIPCHK( hipEventCreateWithFlags( &e->lane[l].ev_djoin, hipEventDisableTiming ), "hipEventCreate" );
    }
    HIPCHK( hipEventRecord( e->lane[l].ev_dfork, st ), "hipEventRecord" );
    HIPCHK( hipStreamWaitEvent( e->lane[l].side, e->lane[l].ev_dfork, 0 ), "hipStreamWaitEvent" );
    int err = fd_ed25519_hip_launch_phase( p, FD_ED25519_PHASE_DECODE, e->dsm_grid, e->lane[l].side );
    if( err ) return hip_fail( (hipError_t)err, "verify launch" );
    HIPCHK( hipEventRecord( e->lane[l].ev_djoin, e->lane[l].side ), "hipEventRecord" );
    err = fd_ed25519_hip_launch_phase( p, FD_ED25519_PHASE_HASH, e->dsm_grid, st );
    if( !err ) err = fd_ed25519_hip_launch_phase( p, FD_ED25519_PHASE_SCALAR, e->dsm_grid, st );
    /* dsm (and the lane's next chunk, which reuses the work arrays) after
       decode, even when a launch above failed */
    hipError_t we = hipStreamWaitEvent( st, e->lane[l].ev_djoin, 0 );
    if( err ) return hip_fail( (hipError_t)err, "verify launch" );
    HIPCHK( we, "hipStreamWaitEvent" );
    err = fd_ed25519_hip_launch_phase( p, FD_ED25519_PHASE_DSM, e->dsm_grid, st );
    if( err ) return hip_fail( (hipError_t)err, "verify launch" );
  } else {
    int err = fd_ed25519_hip_launch_verify( p, e->dsm_grid, st );
    if( err ) return hip_fail( (hipError_t)err, "verify launch" );
  }
  return FD_ED25519_HIP_OK;
}

/* the engine-wide part of a launch's parameters: capacity, base tables,
   code flavour, half-size bound */
static void
params_tables( fd_ed25519_hip_engine_t * e, fd_ed25519_verify_params_t * p ) {
  p->cap = e->max_chunk;
  p->btab = e->d_btab; p->btab16 = e->d_btab16; p->btab_lo = e->btabw[0]; p->btab_hi = e->btabw[1];
  p->btab8_lo = e->d_btab8[0]; p->btab8_hi = e->d_btab8[1];
  p->bw_bits = engine_btab_kind( e ) ? FD_ED25519_BTABC_BITS : FD_ED25519_BTABW_BITS;
  p->codes_portable = (e->flags & FD_ED25519_HIP_FLAG_CODES_PORTABLE) ? 1 : 0;
  p->half_dbits     = engine_half_dbits( e );
}

/* verify_dev and verify_digests_dev: messages hashed on the device, or
   the caller's digests of R||A||M (digests != NULL, msgs unused) */
static int
verify_common( fd_ed25519_hip_engine_t * e, unsigned long n,
               unsigned char const * msgs, unsigned long const * msg_off, unsigned int const * msg_sz,
               unsigned char const * digests, unsigned char const * sigs, unsigned char const * pubs,
               signed char * out, void * stream ) {
  if( !e ) return FD_ED25519_HIP_ERR_INVAL;
  if( !n ) return FD_ED25519_HIP_OK;
  if( ( !digests && ( !msg_off || !msg_sz ) ) || !sigs || !pubs || !out ) return FD_ED25519_HIP_ERR_INVAL;
  if( ((uintptr_t)sigs & 15UL) || ((uintptr_t)pubs & 15UL) || ((uintptr_t)digests & 15UL) ) {
    snprintf( fd_ed25519_hip_errbuf, sizeof(fd_ed25519_hip_errbuf), "sigs/pubs/digests must be 16-byte aligned" );
    return FD_ED25519_HIP_ERR_INVAL;
  }
  hipStream_t st = stream ? (hipStream_t)stream : e->stream;
  HIPCHK( hipSetDevice( e->device ), "hipSetDevice" );
  fd_ed25519_verify_params_t p;
  memset( &p, 0, sizeof(p) );
  p.msgs = msgs; p.msg_off = (uint64_t const *)msg_off; p.msg_sz = msg_sz; p.digests = digests;
  p.sigs = sigs; p.pubs = pubs; p.out = (int8_t *)out;
  params_tables( e, &p );
  uint64_t chunk = e->max_chunk;
  /* a multi-chunk call alternates its chunks between the two lanes; lane 1
     starts after the work already queued on the call's stream and the
     call's stream waits for lane 1 before it returns, so the call stays
     one ordered unit of work on the caller's stream */
  int two = e->pipeline && !e->timing && n > chunk;
  if( two && !e->lane[1].d_work ) {
    int err = lane_alloc( e, 1 );
    if( err ) return err;
  }
  if( two ) {
    HIPCHK( hipEventRecord( e->ev_start, st ), "hipEventRecord" );
    HIPCHK( hipStreamWaitEvent( e->lane[1].stream, e->ev_start, 0 ), "hipStreamWaitEvent" );
  }
  int err = FD_ED25519_HIP_OK;
  uint64_t c = 0UL;
  for( uint64_t base=0UL; base<n && !err; base+=chunk, c++ ) {
    int l = two ? (int)(c & 1UL) : 0;
    err = verify_chunk( e, &p, l, base, (n-base) < chunk ? (n-base) : chunk, l ? e->lane[1].stream : st );
  }
  if( two ) {
    /* joined even when a launch failed, so the caller's stream never runs
       ahead of work still queued on lane 1 */
    hipError_t re = hipEventRecord( e->ev_end, e->lane[1].stream );
    if( re==hipSuccess ) re = hipStreamWaitEvent( st, e->ev_end, 0 );
    if( re!=hipSuccess ) {
      hipStreamSynchronize( e->lane[1].stream );
      if( !err ) return hip_fail( re, "lane join" );
    }
  }
  return err;
}

int
fd_ed25519_hip_verify_dev( fd_ed25519_hip_engine_t * e,
                           unsigned long n,
                           unsigned char const * msgs, unsigned long const * msg_off, unsigned int const * msg_sz,
                           unsigned char const * sigs, unsigned char const * pubs, signed char * out,
                           void * stream ) {
  return verify_common( e, n, msgs, msg_off, msg_sz, NULL, sigs, pubs, out, stream );
}

/* The drop-in's host-scalar launches (dropin_run, a few signatures): the
   decompressions first (prep16's decode blocks only), and the group
   equation (dsm16) once the calling thread has written each signature's
   scalars (fd_ed25519_hip_private_hsrec) into page-locked memory the device
   reads in place -- sflag [cap], hflag [cap] and hs [19][cap], the work
   arrays' layout.  The caller computes while the decompressions run. */
static int
hs_params( fd_ed25519_hip_engine_t * e, fd_ed25519_verify_params_t * p, unsigned long n, unsigned char const * sigs,
           unsigned char const * pubs, signed char * out ) {
  if( !e || !n || n>e->r16_max || n>e->max_chunk || !sigs || !pubs || !out ||
      ((uintptr_t)sigs & 15UL) || ((uintptr_t)pubs & 15UL) ) return FD_ED25519_HIP_ERR_INVAL;
  memset( p, 0, sizeof(*p) );
  p->sigs = sigs; p->pubs = pubs; p->out = (int8_t *)out;
  params_tables( e, p );
  p->k = e->lane[0].d_k; p->sflag = e->lane[0].d_sflag; p->pflag = e->lane[0].d_pflag; p->pts = e->lane[0].d_pts;
  p->fix_list = e->lane[0].d_fix; p->fix_cnt = e->lane[0].d_hist + 2*FD_ED25519_SORT_BUCKETS;
  p->work_ctr = p->fix_cnt + 1; p->hs = e->lane[0].d_hs; p->hflag = e->lane[0].d_hflag;
  p->hist = e->lane[0].d_hist; p->atab = e->lane[0].d_atab;
  p->n = n; p->small = 3; p->hs_host = 1;
  return FD_ED25519_HIP_OK;
}

int
fd_ed25519_hip_private_half_dbits( fd_ed25519_hip_engine_t const * e ) {
  return engine_half_dbits( e );
}

int
fd_ed25519_hip_private_codes_portable( fd_ed25519_hip_engine_t const * e ) {
  return (e->flags & FD_ED25519_HIP_FLAG_CODES_PORTABLE) ? 1 : 0;
}

int
fd_ed25519_hip_private_hs_decode( fd_ed25519_hip_engine_t * e, unsigned long n, unsigned char const * sigs,
                                  unsigned char const * pubs, signed char * out, void * stream ) {
  fd_ed25519_verify_params_t p;
  int err = hs_params( e, &p, n, sigs, pubs, out );
  if( err ) return err;
  HIPCHK( hipSetDevice( e->device ), "hipSetDevice" );
  err = fd_ed25519_hip_launch_phase( &p, FD_ED25519_PHASE_HASH, e->dsm_grid, stream ? (hipStream_t)stream : e->stream );
  if( err ) return hip_fail( (hipError_t)err, "verify launch" );
  return FD_ED25519_HIP_OK;
}

int
fd_ed25519_hip_private_hs_dsm( fd_ed25519_hip_engine_t * e, unsigned long n, unsigned char const * sigs,
                               unsigned char const * pubs, signed char * out, unsigned char const * sflag,
                               unsigned char const * hflag, unsigned int const * hs, int const * pts,
                               unsigned char const * pflag, unsigned int const * go, void * stream ) {
  fd_ed25519_verify_params_t p;
  int err = hs_params( e, &p, n, sigs, pubs, out );
  if( err ) return err;
  if( !sflag || !hflag || !hs || !pts!=!pflag ) return FD_ED25519_HIP_ERR_INVAL;
  p.sflag = (uint8_t *)sflag; p.hflag = (uint8_t *)hflag; p.hs = (uint32_t *)hs;
  if( pts ) {   /* every array the caller's: its small stride */
    if( n>FD_ED25519_HS_STRIDE ) return FD_ED25519_HIP_ERR_INVAL;
    p.pts = (int32_t *)pts; p.pflag = (uint8_t *)pflag; p.cap = FD_ED25519_HS_STRIDE;
  }
  p.go = (uint32_t const *)go;
  err = fd_ed25519_hip_launch_phase( &p, FD_ED25519_PHASE_DSM, e->dsm_grid, stream ? (hipStream_t)stream : e->stream );
  if( err ) return hip_fail( (hipError_t)err, "verify launch" );
  return FD_ED25519_HIP_OK;
}

int
fd_ed25519_hip_private_hs_dsms( fd_ed25519_hip_engine_t * e, int waves, unsigned long n, unsigned char const * sigs,
                                unsigned char const * pubs, signed char * out, unsigned char const * sflag,
                                unsigned char const * hflag, unsigned int const * hq, int const * pts,
                                unsigned char const * pflag, unsigned int const * go, void * stream ) {
  fd_ed25519_verify_params_t p;
  int err = hs_params( e, &p, n, sigs, pubs, out );
  if( err ) return err;
  if( (waves!=4 && waves!=8) || !sflag || !hflag || !hq || !pts || !pflag || !e->btabs[ split_set( waves ) ][0] )
    return FD_ED25519_HIP_ERR_INVAL;
  if( n>FD_ED25519_HS_STRIDE ) return FD_ED25519_HIP_ERR_INVAL;
  p.sflag = (uint8_t *)sflag; p.hflag = (uint8_t *)hflag; p.hs = (uint32_t *)hq;
  p.pts = (int32_t *)pts; p.pflag = (uint8_t *)pflag; p.cap = FD_ED25519_HS_STRIDE;   /* every array the caller's */
  p.go = (uint32_t const *)go;
  for( int q=0; q<8; q++ ) p.btabq[q] = e->btabs[ split_set( waves ) ][q];
  err = fd_ed25519_hip_launch_dsm16s( &p, waves, stream ? (hipStream_t)stream : e->stream );
  if( err ) return hip_fail( (hipError_t)err, "verify launch" );
  return FD_ED25519_HIP_OK;
}

/* dsm16s<waves>'s tables for engine e (with the lane-split form), made on
   first use per device: the drop-in engines take them at creation, a
   pipe's engines only when a split form is asked for.  1: available. */
int
fd_ed25519_hip_private_want_dsms( fd_ed25519_hip_engine_t * e, int waves ) {
  if( !e || !e->r16_max || (waves!=4 && waves!=8) ) return 0;
  int set = split_set( waves );
  if( !e->btabs[set][0] && hipSetDevice( e->device )==hipSuccess ) {
    int32_t * t[8] = { NULL };
    if( !btabs_acquire( e->device, waves, e->stream, t ) ) for( int q=0; q<8; q++ ) e->btabs[set][q] = t[q];
  }
  return e->btabs[set][0] ? 1 : 0;
}

int
fd_ed25519_hip_verify_digests_dev( fd_ed25519_hip_engine_t * e, unsigned long n, unsigned char const * digests,
                                   unsigned char const * sigs, unsigned char const * pubs, signed char * out,
                                   void * stream ) {
  if( !digests ) return FD_ED25519_HIP_ERR_INVAL;
  return verify_common( e, n, NULL, NULL, NULL, digests, sigs, pubs, out, stream );
}

int
fd_ed25519_hip_engine_timing( fd_ed25519_hip_engine_t * e, int enable ) {
  if( !e ) return FD_ED25519_HIP_ERR_INVAL;
  HIPCHK( hipSetDevice( e->device ), "hipSetDevice" );
  if( enable && !e->tm_ev_init ) {
    for( int i=0; i<FD_ED25519_HIP_TIMING_MAX; i++ )
      for( int j=0; j<=FD_ED25519_PHASE_CNT; j++ )
        HIPCHK( hipEventCreate( &e->tm_ev[i][j] ), "hipEventCreate" );
    e->tm_ev_init = 1;
  }
  e->timing = enable;
  e->tm_cnt = 0;
  return FD_ED25519_HIP_OK;
}

int
fd_ed25519_hip_engine_timing_read( fd_ed25519_hip_engine_t * e, double * phase_ms, unsigned long * launches ) {
  if( !e || !phase_ms ) return FD_ED25519_HIP_ERR_INVAL;
  HIPCHK( hipSetDevice( e->device ), "hipSetDevice" );
  for( int ph=0; ph<FD_ED25519_PHASE_CNT; ph++ ) phase_ms[ph] = 0.0;
  for( int i=0; i<e->tm_cnt; i++ ) {
    HIPCHK( hipEventSynchronize( e->tm_ev[i][FD_ED25519_PHASE_CNT] ), "hipEventSynchronize" );
    for( int ph=0; ph<FD_ED25519_PHASE_CNT; ph++ ) {
      float ms = 0.f;
      HIPCHK( hipEventElapsedTime( &ms, e->tm_ev[i][ph], e->tm_ev[i][ph+1] ), "hipEventElapsedTime" );
      phase_ms[ph] += (double)ms;
    }
  }
  if( launches ) *launches = (unsigned long)e->tm_cnt;
  e->tm_cnt = 0;
  return FD_ED25519_HIP_OK;
}

/* ---- base-table self-check ------------------------------------------ */

#if FD_ED25519_BTABW_BITS != FD_ED25519_HIP_BASE_TABLE_BITS || FD_ED25519_BTABW_SHIFT != FD_ED25519_HIP_BASE_TABLE_SHIFT
#error "base table geometry differs from the public header's"
#endif

int
fd_ed25519_hip_engine_check_base_tables( fd_ed25519_hip_engine_t * e, unsigned long bad[3] ) {
  if( !e || !bad || !e->btabw[0] || !e->btabw[1] || !e->d_btab16 ) return FD_ED25519_HIP_ERR_INVAL;
  HIPCHK( hipSetDevice( e->device ), "hipSetDevice" );
  uint32_t * d_bad = NULL;
  HIPCHK( hipMalloc( (void **)&d_bad, 3*sizeof(uint32_t) ), "hipMalloc" );
  uint32_t h_bad[3] = { 0U, 0U, 0U };
  int32_t const * tab[3] = { e->btabw[0], e->btabw[1], e->d_btab16 };
  int             ent    = 1 << btab_kind_bits( engine_btab_kind( e ) );
  int             cnt[3] = { ent, ent, FD_ED25519_BTAB16_ENTRIES };
  hipError_t he = hipMemsetAsync( d_bad, 0, 3*sizeof(uint32_t), e->stream );
  for( int t=0; t<3 && he==hipSuccess; t++ )
    he = (hipError_t)fd_ed25519_hip_launch_check_btabw( tab[t], cnt[t], d_bad + t, e->stream );
  if( he==hipSuccess ) he = hipMemcpyAsync( h_bad, d_bad, sizeof(h_bad), hipMemcpyDeviceToHost, e->stream );
  if( he==hipSuccess ) he = hipStreamSynchronize( e->stream );
  hipFree( d_bad );
  if( he!=hipSuccess ) return hip_fail( he, "check_base_tables" );
  for( int t=0; t<3; t++ ) bad[t] = h_bad[t];
  return FD_ED25519_HIP_OK;
}

int
fd_ed25519_hip_engine_base_entry( fd_ed25519_hip_engine_t * e, int which, unsigned long index, int out[30] ) {
  if( !e || !out || which<0 || which>1 || index>=(1UL << btab_kind_bits( engine_btab_kind( e ) )) || !e->btabw[which] )
    return FD_ED25519_HIP_ERR_INVAL;
  HIPCHK( hipSetDevice( e->device ), "hipSetDevice" );
  HIPCHK( hipMemcpyAsync( out, e->btabw[which] + index*FD_ED25519_BTAB16_STRIDE, 30*sizeof(int32_t),
                          hipMemcpyDeviceToHost, e->stream ), "hipMemcpy" );
  HIPCHK( hipStreamSynchronize( e->stream ), "hipStreamSynchronize" );
  return FD_ED25519_HIP_OK;
}

/* ---- device memory helpers (the engine's HIP runtime) ---------------- */

void *
fd_ed25519_hip_dev_alloc( fd_ed25519_hip_engine_t * e, unsigned long bytes ) {
  if( !e ) return NULL;
  if( hipSetDevice( e->device )!=hipSuccess ) return NULL;
  void * p = NULL;
  hipError_t err = hipMalloc( &p, bytes ? bytes : 1UL );
  if( err!=hipSuccess ) { hip_fail( err, "hipMalloc" ); return NULL; }
  return p;
}

int
fd_ed25519_hip_dev_free( fd_ed25519_hip_engine_t * e, void * p ) {
  if( !e ) return FD_ED25519_HIP_ERR_INVAL;
  HIPCHK( hipSetDevice( e->device ), "hipSetDevice" );
  HIPCHK( hipFree( p ), "hipFree" );
  return FD_ED25519_HIP_OK;
}

int
fd_ed25519_hip_memcpy( fd_ed25519_hip_engine_t * e, void * dst, void const * src, unsigned long bytes, int dir ) {
  if( !e ) return FD_ED25519_HIP_ERR_INVAL;
  HIPCHK( hipSetDevice( e->device ), "hipSetDevice" );
  hipMemcpyKind k = dir==FD_ED25519_HIP_H2D ? hipMemcpyHostToDevice
                  : dir==FD_ED25519_HIP_D2H ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
  HIPCHK( hipMemcpyAsync( dst, src, bytes, k, e->stream ), "hipMemcpyAsync" );
  HIPCHK( hipStreamSynchronize( e->stream ), "hipStreamSynchronize" );
  return FD_ED25519_HIP_OK;
}

int
fd_ed25519_hip_device_clock_mhz( fd_ed25519_hip_engine_t * e ) {
  if( !e ) return 0;
  hipDeviceProp_t prop;
  if( hipGetDeviceProperties( &prop, e->device )!=hipSuccess ) return 0;
  return prop.clockRate / 1000;
}

int
fd_ed25519_hip_device_count( void ) {
  int n = 0;
  if( hipGetDeviceCount( &n )!=hipSuccess ) return 0;
  return n;
}

int
fd_ed25519_hip_txn_combine_dev( fd_ed25519_hip_engine_t * e, unsigned long ntxn,
                                signed char const * sig_codes, unsigned int const * txn_first,
                                unsigned int const * txn_cnt, signed char * txn_out, void * stream ) {
  if( !e ) return FD_ED25519_HIP_ERR_INVAL;
  if( !ntxn ) return FD_ED25519_HIP_OK;
  hipStream_t st = stream ? (hipStream_t)stream : e->stream;
  HIPCHK( hipSetDevice( e->device ), "hipSetDevice" );
  int err = fd_ed25519_hip_launch_txn_combine( (int8_t const *)sig_codes, txn_first, txn_cnt,
                                               (int8_t *)txn_out, ntxn, st );
  if( err ) return hip_fail( (hipError_t)err, "txn_combine launch" );
  return FD_ED25519_HIP_OK;
}

int
fd_ed25519_hip_sign_dev( fd_ed25519_hip_engine_t * e, unsigned long n,
                         unsigned char const * msgs, unsigned long const * msg_off, unsigned int const * msg_sz,
                         unsigned char const * privs, unsigned char * sigs, unsigned char * pubs, void * stream ) {
  if( !e || (!privs && n) ) return FD_ED25519_HIP_ERR_INVAL;
  if( !n ) return FD_ED25519_HIP_OK;
  if( ((uintptr_t)sigs & 15UL) || ((uintptr_t)pubs & 15UL) || ((uintptr_t)privs & 15UL) ) return FD_ED25519_HIP_ERR_INVAL;
  HIPCHK( hipSetDevice( e->device ), "hipSetDevice" );
  fd_ed25519_sign_params_t p;
  memset( &p, 0, sizeof(p) );
  p.msgs = msgs; p.msg_off = (uint64_t const *)msg_off; p.msg_sz = msg_sz; p.privs = privs;
  p.sigs = sigs; p.pubs = pubs; p.n = n; p.btab = e->d_btab;
  int err = fd_ed25519_hip_launch_sign( &p, stream ? stream : (void *)e->stream );
  if( err ) return hip_fail( (hipError_t)err, "sign launch" );
  return FD_ED25519_HIP_OK;
}

int
fd_ed25519_hip_gen_dev( fd_ed25519_hip_engine_t * e, unsigned long n, unsigned long seed, unsigned long index_base,
                        unsigned char * msgs, unsigned long msg_bytes, unsigned long const * msg_off,
                        unsigned int const * msg_sz, unsigned char * sigs, unsigned char * pubs, void * stream ) {
  if( !e ) return FD_ED25519_HIP_ERR_INVAL;
  if( ((uintptr_t)sigs & 15UL) || ((uintptr_t)pubs & 15UL) ) return FD_ED25519_HIP_ERR_INVAL;
  HIPCHK( hipSetDevice( e->device ), "hipSetDevice" );
  void * st = stream ? stream : (void *)e->stream;
  int err = fd_ed25519_hip_launch_fill_random( msgs, msg_bytes, seed, st );
  if( err ) return hip_fail( (hipError_t)err, "fill launch" );
  fd_ed25519_sign_params_t p;
  memset( &p, 0, sizeof(p) );
  p.msgs = msgs; p.msg_off = (uint64_t const *)msg_off; p.msg_sz = msg_sz; p.privs = NULL;
  p.sigs = sigs; p.pubs = pubs; p.n = n; p.seed = seed; p.index_base = index_base; p.btab = e->d_btab;
  if( (err = fd_ed25519_hip_launch_sign( &p, st )) ) return hip_fail( (hipError_t)err, "sign launch" );
  return FD_ED25519_HIP_OK;
}

int
fd_ed25519_hip_corrupt_dev( fd_ed25519_hip_engine_t * e, unsigned long n, unsigned long seed,
                            unsigned long index_base, unsigned int ppm, unsigned char * msgs,
                            unsigned long const * msg_off, unsigned int const * msg_sz, unsigned char * sigs,
                            unsigned char * pubs, signed char * expect, unsigned char * cls, void * stream ) {
  if( !e ) return FD_ED25519_HIP_ERR_INVAL;
  if( ((uintptr_t)sigs & 15UL) || ((uintptr_t)pubs & 15UL) ) return FD_ED25519_HIP_ERR_INVAL;
  HIPCHK( hipSetDevice( e->device ), "hipSetDevice" );
  fd_ed25519_corrupt_params_t p;
  memset( &p, 0, sizeof(p) );
  p.msgs = msgs; p.msg_off = (uint64_t const *)msg_off; p.msg_sz = msg_sz; p.sigs = sigs; p.pubs = pubs;
  p.n = n; p.seed = seed; p.index_base = index_base; p.ppm = ppm; p.expect = (int8_t *)expect; p.cls = cls;
  int err = fd_ed25519_hip_launch_corrupt( &p, stream ? stream : (void *)e->stream );
  if( err ) return hip_fail( (hipError_t)err, "corrupt launch" );
  return FD_ED25519_HIP_OK;
}

/* ---- host staging ------------------------------------------------------ */

static int
grow_pair( void ** h, void ** d, uint64_t * cap, uint64_t need, uint64_t elem ) {
  if( need<=*cap ) return FD_ED25519_HIP_OK;
  uint64_t ncap = *cap ? *cap : 1024UL;
  while( ncap<need ) ncap *= 2UL;
  hipHostFree( *h ); hipFree( *d ); *h = NULL; *d = NULL; *cap = 0UL;
  HIPCHK( hipHostMalloc( h, ncap*elem + 64UL, hipHostMallocDefault ), "hipHostMalloc" );
  HIPCHK( hipMalloc( d, ncap*elem + 64UL ), "hipMalloc" );
  *cap = ncap;
  return FD_ED25519_HIP_OK;
}

static int
stage_sigs( fd_ed25519_hip_engine_t * e, uint64_t n ) {
  if( n<=e->st_sig_cap ) return FD_ED25519_HIP_OK;
  uint64_t c0 = e->st_sig_cap, c = 0;
  int err;
  c = c0; if( (err = grow_pair( (void **)&e->h_off,  (void **)&e->d_off,  &c, n, 8UL  )) ) return err;
  c = c0; if( (err = grow_pair( (void **)&e->h_sz,   (void **)&e->d_sz,   &c, n, 4UL  )) ) return err;
  c = c0; if( (err = grow_pair( (void **)&e->h_sigs, (void **)&e->d_sigs, &c, n, 64UL )) ) return err;
  c = c0; if( (err = grow_pair( (void **)&e->h_pubs, (void **)&e->d_pubs, &c, n, 32UL )) ) return err;
  c = c0; if( (err = grow_pair( (void **)&e->h_out,  (void **)&e->d_out,  &c, n, 1UL  )) ) return err;
  e->st_sig_cap = c;
  return FD_ED25519_HIP_OK;
}

static int
stage_msgs( fd_ed25519_hip_engine_t * e, uint64_t bytes ) {
  return grow_pair( (void **)&e->h_msgs, (void **)&e->d_msgs, &e->st_msg_cap, bytes ? bytes : 1UL, 1UL );
}

static int
stage_txns( fd_ed25519_hip_engine_t * e, uint64_t ntxn ) {
  if( ntxn<=e->st_txn_cap ) return FD_ED25519_HIP_OK;
  uint64_t c0 = e->st_txn_cap, c = 0;
  int err;
  c = c0; if( (err = grow_pair( (void **)&e->h_tfirst, (void **)&e->d_tfirst, &c, ntxn, 4UL )) ) return err;
  c = c0; if( (err = grow_pair( (void **)&e->h_tcnt,   (void **)&e->d_tcnt,   &c, ntxn, 4UL )) ) return err;
  c = c0; if( (err = grow_pair( (void **)&e->h_tout,   (void **)&e->d_tout,   &c, ntxn, 1UL )) ) return err;
  e->st_txn_cap = c;
  return FD_ED25519_HIP_OK;
}

static int
upload_and_verify( fd_ed25519_hip_engine_t * e, uint64_t n, uint64_t msg_bytes ) {
  hipStream_t st = e->stream;
  HIPCHK( hipMemcpyAsync( e->d_msgs, e->h_msgs, msg_bytes ? msg_bytes : 1UL, hipMemcpyHostToDevice, st ), "H2D msgs" );
  HIPCHK( hipMemcpyAsync( e->d_off,  e->h_off,  8UL*n,  hipMemcpyHostToDevice, st ), "H2D off" );
  HIPCHK( hipMemcpyAsync( e->d_sz,   e->h_sz,   4UL*n,  hipMemcpyHostToDevice, st ), "H2D sz" );
  HIPCHK( hipMemcpyAsync( e->d_sigs, e->h_sigs, 64UL*n, hipMemcpyHostToDevice, st ), "H2D sigs" );
  HIPCHK( hipMemcpyAsync( e->d_pubs, e->h_pubs, 32UL*n, hipMemcpyHostToDevice, st ), "H2D pubs" );
  return fd_ed25519_hip_verify_dev( e, n, e->d_msgs, (unsigned long const *)e->d_off, e->d_sz, e->d_sigs,
                                    e->d_pubs, (signed char *)e->d_out, st );
}

int
fd_ed25519_hip_verify_host( fd_ed25519_hip_engine_t * e, unsigned long n,
                            unsigned char const * msgs, unsigned long const * msg_off, unsigned int const * msg_sz,
                            unsigned char const * sigs, unsigned char const * pubs, signed char * out ) {
  if( !e ) return FD_ED25519_HIP_ERR_INVAL;
  if( !n ) return FD_ED25519_HIP_OK;
  if( !msg_off || !msg_sz || !sigs || !pubs || !out ) return FD_ED25519_HIP_ERR_INVAL;
  HIPCHK( hipSetDevice( e->device ), "hipSetDevice" );
  int err;
  if( (err = stage_sigs( e, n )) ) return err;
  uint64_t bytes = 0UL;
  for( uint64_t i=0UL; i<n; i++ ) bytes += msg_sz[i];
  if( (err = stage_msgs( e, bytes )) ) return err;
  /* pack messages contiguously (pinned), rewrite offsets */
  uint64_t pos = 0UL;
  for( uint64_t i=0UL; i<n; i++ ) {
    if( msg_sz[i] ) memcpy( e->h_msgs + pos, msgs + msg_off[i], msg_sz[i] );
    e->h_off[i] = pos;
    e->h_sz [i] = msg_sz[i];
    pos += msg_sz[i];
  }
  memcpy( e->h_sigs, sigs, 64UL*n );
  memcpy( e->h_pubs, pubs, 32UL*n );
  if( (err = upload_and_verify( e, n, bytes )) ) return err;
  HIPCHK( hipMemcpyAsync( e->h_out, e->d_out, n, hipMemcpyDeviceToHost, e->stream ), "D2H out" );
  HIPCHK( hipStreamSynchronize( e->stream ), "verify" );
  memcpy( out, e->h_out, n );
  return FD_ED25519_HIP_OK;
}

int
fd_ed25519_hip_verify_txns_host( fd_ed25519_hip_engine_t * e, unsigned long ntxn,
                                 unsigned char const * msgs, unsigned long const * txn_msg_off,
                                 unsigned int const * txn_msg_sz, unsigned int const * txn_first,
                                 unsigned int const * txn_cnt, unsigned char const * sigs,
                                 unsigned char const * pubs, signed char * out_txn, signed char * out_sig ) {
  if( !e ) return FD_ED25519_HIP_ERR_INVAL;
  if( !ntxn ) return FD_ED25519_HIP_OK;
  if( !txn_msg_off || !txn_msg_sz || !txn_first || !txn_cnt || !out_txn ) return FD_ED25519_HIP_ERR_INVAL;
  HIPCHK( hipSetDevice( e->device ), "hipSetDevice" );
  /* signatures actually verified: those of transactions with 1..16 signers
     (others are ERR_SIG without reading their inputs, as the reference) */
  uint64_t n = 0UL, bytes = 0UL;
  for( uint64_t t=0UL; t<ntxn; t++ ) {
    if( txn_cnt[t]>=1U && txn_cnt[t]<=16U ) n += txn_cnt[t];
    bytes += txn_msg_sz[t];
  }
  int err;
  if( (err = stage_sigs( e, n ? n : 1UL )) ) return err;
  if( (err = stage_msgs( e, bytes )) ) return err;
  if( (err = stage_txns( e, ntxn )) ) return err;
  uint64_t pos = 0UL, k = 0UL;
  for( uint64_t t=0UL; t<ntxn; t++ ) {
    uint64_t moff = pos;
    if( txn_msg_sz[t] ) memcpy( e->h_msgs + pos, msgs + txn_msg_off[t], txn_msg_sz[t] );
    pos += txn_msg_sz[t];
    uint32_t cnt = txn_cnt[t];
    e->h_tfirst[t] = (uint32_t)k;
    e->h_tcnt  [t] = cnt;
    if( cnt<1U || cnt>16U ) continue;
    for( uint32_t j=0U; j<cnt; j++, k++ ) {
      uint64_t s = (uint64_t)txn_first[t] + j;
      e->h_off[k] = moff;
      e->h_sz [k] = txn_msg_sz[t];
      memcpy( e->h_sigs + 64UL*k, sigs + 64UL*s, 64UL );
      memcpy( e->h_pubs + 32UL*k, pubs + 32UL*s, 32UL );
    }
  }
  if( n && (err = upload_and_verify( e, n, bytes )) ) return err;
  HIPCHK( hipMemcpyAsync( e->d_tfirst, e->h_tfirst, 4UL*ntxn, hipMemcpyHostToDevice, e->stream ), "H2D tfirst" );
  HIPCHK( hipMemcpyAsync( e->d_tcnt,   e->h_tcnt,   4UL*ntxn, hipMemcpyHostToDevice, e->stream ), "H2D tcnt" );
  if( (err = fd_ed25519_hip_txn_combine_dev( e, ntxn, (signed char const *)e->d_out, e->d_tfirst, e->d_tcnt,
                                             (signed char *)e->d_tout, e->stream )) ) return err;
  HIPCHK( hipMemcpyAsync( e->h_tout, e->d_tout, ntxn, hipMemcpyDeviceToHost, e->stream ), "D2H tout" );
  if( out_sig && n ) HIPCHK( hipMemcpyAsync( e->h_out, e->d_out, n, hipMemcpyDeviceToHost, e->stream ), "D2H out" );
  HIPCHK( hipStreamSynchronize( e->stream ), "verify_txns" );
  memcpy( out_txn, e->h_tout, ntxn );
  if( out_sig ) {
    /* scatter per-signature codes back to the caller's indexing */
    for( uint64_t t=0UL; t<ntxn; t++ ) {
      uint32_t cnt = txn_cnt[t];
      for( uint32_t j=0U; j<cnt; j++ )
        out_sig[ txn_first[t] + j ] = (cnt>=1U && cnt<=16U) ? e->h_out[ e->h_tfirst[t] + j ] : (signed char)FD_ED25519_ERR_SIG;
    }
  }
  return FD_ED25519_HIP_OK;
}

/* ---- drop-in API -------------------------------------------------------

   fd_ed25519_verify / fd_ed25519_verify_batch_single_msg for any number of
   calling threads (the reference's are reentrant and keep no global state,
   src/ballet/ed25519/fd_ed25519.h:86-94).  Concurrent calls are coalesced
   by flat combining: each call queues a request; a caller that finds one
   of the process's DROPIN_ENGINES drop-in engines idle takes every queued
   request (its own and the others', up to DROPIN_BATCH_MAX) into one
   launch -- each request one transaction of 1..16 signatures over its
   message, with batch_single_msg's combine -- and hands every caller its
   code; the others wait on a condition variable.  One caller alone pays
   one GPU round trip as before; N concurrent callers share a round trip,
   and four engines keep batches filling while others are on the GPU, so
   calls per second grow with the caller count instead of serialising on
   one lock.  The engines use the compact base tables
   (FD_ED25519_HIP_FLAG_COMPACT_TABLES: 2 x 8 MiB instead of 2 x 2 GiB) and
   small chunks, so a process that only uses the drop-ins holds well under
   600 MB of device memory. */

#define DROPIN_ENGINES   4
#define DROPIN_BATCH_MAX 4096UL
#define DROPIN_CHUNK     16384UL
#define DROPIN_PENDING 0x55   /* a direct launch's codes before the kernels write them */
#ifndef DROPIN_DIRECT_MAX
#define DROPIN_DIRECT_MAX 64UL   /* launches of at most this many signatures read the pinned block in place */
#endif
/* ... and of at most this many input bytes: the hash kernels read a direct
   launch's messages word by word over the link from uncached coherent
   pinned memory, which pays for a few hundred bytes but not for a
   multi-MB message (one bulk pull into HBM first is faster there). */
#ifndef DROPIN_DIRECT_MAX_BYTES
#define DROPIN_DIRECT_MAX_BYTES 65536UL
#endif

typedef struct dropin_req {
  unsigned char const * msg;
  unsigned long         msg_sz;
  unsigned char const * sigs;
  unsigned char const * pubs;
  unsigned int          cnt;      /* signatures, 1..16                     */
  int                   single;   /* fd_ed25519_verify: the signature's code */
  int                   hashed;   /* dig holds SHA-512(R_j||A_j||M): the message stays on the host */
  int                   result;
  int                   done;
  struct dropin_req *   next;
  unsigned char         dig[ 16 ][ 64 ];
} dropin_req_t;

/* Messages of at least this many bytes are hashed on the host by the
   calling thread (fd_ed25519_hip_private_challenge) and verified from their
   digests: the device path's message sizes are 32-bit, and the reference
   takes any ulong size (src/ballet/ed25519/fd_ed25519.h:96-101).  A test
   hook moves the limit down (fd_ed25519_hip_dropin_set_host_hash_min). */
static unsigned long dropin_host_hash_min = 1UL<<32;

/* clamped to 4 GiB: a limit above that would leave messages the device's
   32-bit sizes cannot carry on the device path */
void
fd_ed25519_hip_dropin_set_host_hash_min( unsigned long bytes ) {
  dropin_host_hash_min = ( bytes && bytes<(1UL<<32) ) ? bytes : 1UL<<32;
}

void fd_ed25519_hip_private_challenge( unsigned char const sig[ 64 ], unsigned char const pub[ 32 ],
                                       unsigned char const * msg, unsigned long msg_sz, unsigned char out[ 64 ] );

/* Direct launches of at most this many signatures take their scalars from
   the calling thread (host/fd_ed25519_hip_hsrec.cc, ~8 us each) while the
   device decompresses A and R, instead of prep16's hash -> search chain of
   one lane; more would cost the caller more than the chain.  Test hook:
   fd_ed25519_hip_dropin_set_host_scalars (0 turns the mode off). */
#ifndef DROPIN_HS_MAX
#define DROPIN_HS_MAX 4UL
#endif
static unsigned long dropin_hs_max = DROPIN_HS_MAX;
#define FD_HALF_DBITS_HOST_MAX 151   /* fd25519_half.h FD_HALF_DBITS_MAX */

void
fd_ed25519_hip_dropin_set_host_scalars( unsigned long max_sigs ) {
  dropin_hs_max = max_sigs>DROPIN_DIRECT_MAX ? DROPIN_DIRECT_MAX : max_sigs;
}

/* Test hook: the host search's bound on |d| (0: the engine's, 151).  No
   random k without a pair at 151 bits turned up in 40M trials, so tests
   reach the launch's fallback (the device path from the digests, at the
   engine's bound) with k that have no pair at 131 bits
   (tests/golden/halfsize.npz). */
static int dropin_hs_dbits;

void
fd_ed25519_hip_dropin_set_host_scalars_dbits( int dbits ) {
  dropin_hs_dbits = dbits>0 && dbits<=FD_HALF_DBITS_HOST_MAX ? dbits : 0;
}

/* Launches of at most this many host-scalar signatures also decompress A
   and R on the calling thread (host/fd_ed25519_hip_hsdec.cc; both points
   of a signature side by side, ~9 us a signature on one core) and launch
   dsm16 alone: the host's scalars plus decompressions then cost less than
   the decode blocks' ~44 us they replace.  At four signatures (~70 us of
   host work) they would not.  Test hook: fd_ed25519_hip_dropin_set_host_decode. */
#ifndef DROPIN_HD_MAX
#define DROPIN_HD_MAX 2UL
#endif
#define DROPIN_HD_CAP 4UL   /* the hook's bound: the host arrays below */
static unsigned long dropin_hd_max = DROPIN_HD_MAX;

/* host-decoded drop-in launches take the split form of this many waves
   (dsm16s: 4 or 8, the host doubling A and R and splitting the scalars;
   2: dsm16) when the engine holds its tables: p50 82.3 / 68.8 / 76.2 us
   with 2 / 4 / 8 for one caller, back to back on one box -- eight waves
   halve the chain again but pay more host doublings, eight table builds
   and three rounds of additions (profiles/r6_dropin_split_waves.json);
   test / A-B hook fd_ed25519_hip_dropin_set_split_waves */
#ifndef DROPIN_SPLIT_WAVES
#define DROPIN_SPLIT_WAVES 4
#endif
static int dropin_split = DROPIN_SPLIT_WAVES;

void
fd_ed25519_hip_dropin_set_split_waves( int waves ) {
  dropin_split = waves==4 || waves==8 ? waves : 2;
}

void
fd_ed25519_hip_dropin_set_host_decode( unsigned long max_sigs ) {
  dropin_hd_max = max_sigs>DROPIN_HD_CAP ? DROPIN_HD_CAP : max_sigs;
}

static pthread_once_t  dropin_once = PTHREAD_ONCE_INIT;
static pthread_mutex_t dropin_lock = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t  dropin_cv   = PTHREAD_COND_INITIALIZER;
static struct {
  fd_ed25519_hip_engine_t * eng[ DROPIN_ENGINES ];
  int                       busy[ DROPIN_ENGINES ];
  unsigned char *           h_blk[ DROPIN_ENGINES ];   /* pinned, coherent: one launch's inputs, then its codes */
  unsigned char *           h_dev[ DROPIN_ENGINES ];   /* h_blk as the device sees it */
  unsigned char *           d_blk[ DROPIN_ENGINES ];
  uint64_t                  blk_cap[ DROPIN_ENGINES ];
  int                       direct_pending[ DROPIN_ENGINES ];   /* last launch returned before its stream ended */
  dropin_req_t *            head;
  dropin_req_t *            tail;
  unsigned long             launches, requests;   /* for fd_ed25519_hip_dropin_stats */
  int                       device, flags;        /* what the engines are made with */
  /* failure policy (fd_ed25519_hip_dropin_set_on_lost), under dropin_lock */
  int                       on_lost;
  int                       lost;                 /* 0, or the code that lost the device */
  unsigned long             recoveries;
} dq;

/* the message, then abort(): the ABORT policy's end */
static void
dropin_fatal( int err, char const * what ) {
  fprintf( stderr, "libfd_ed25519_hip: FATAL: %s: %s (%d): %s; the device is lost to the drop-ins (policy: abort)\n",
           what, fd_ed25519_hip_strerror( err ), err, fd_ed25519_hip_last_error() );
  abort();
}

/* engine k anew (its staging block too): any previous one is deleted
   first.  0 or the creation's error code (dq.eng[k] then NULL). */
static int
dropin_engine_make( int k ) {
  if( dq.eng[k] ) { fd_ed25519_hip_engine_delete( dq.eng[k] ); dq.eng[k] = NULL; }
  hipHostFree( dq.h_blk[k] ); hipFree( dq.d_blk[k] );
  dq.h_blk[k] = NULL; dq.h_dev[k] = NULL; dq.d_blk[k] = NULL; dq.blk_cap[k] = 0UL;
  dq.direct_pending[k] = 0;
  dq.eng[k] = fd_ed25519_hip_engine_new( dq.device, DROPIN_CHUNK, dq.flags );
  if( dq.eng[k] && dropin_split>2 ) fd_ed25519_hip_private_want_dsms( dq.eng[k], dropin_split );   /* without: dsm16 */
  return dq.eng[k] ? FD_ED25519_HIP_OK : FD_ED25519_HIP_ERR_INVAL;
}

/* every engine, each with one more attempt if its first creation fails */
static int
dropin_engines_make( void ) {
  for( int k=0; k<DROPIN_ENGINES; k++ ) {
    int err = dropin_engine_make( k );
    if( err ) err = dropin_engine_make( k );
    if( err ) return err;
  }
  return FD_ED25519_HIP_OK;
}

static void
dropin_init( void ) {
  char const * dev_s   = getenv( "FD_ED25519_HIP_DEVICE" );
  char const * codes_s = getenv( "FD_ED25519_HIP_CODES" );
  dq.device = dev_s ? atoi( dev_s ) : 0;
  dq.flags  = FD_ED25519_HIP_FLAG_COMPACT_TABLES | FD_ED25519_HIP_FLAG_ONE_STREAM |
              ((codes_s && !strcmp( codes_s, "portable" )) ? FD_ED25519_HIP_FLAG_CODES_PORTABLE : 0);
  int err = dropin_engines_make();
  if( err ) {
    pthread_mutex_lock( &dropin_lock );
    dq.lost = err;
    int abort_now = dq.on_lost==FD_ED25519_HIP_DROPIN_ON_LOST_ABORT;
    pthread_mutex_unlock( &dropin_lock );
    if( abort_now ) dropin_fatal( err, "cannot create the drop-in GPU engines" );
    fprintf( stderr, "libfd_ed25519_hip: cannot create the drop-in GPU engines: %s; every drop-in call returns "
                     "FD_ED25519_ERR_SIG (policy: reject) until fd_ed25519_hip_dropin_reset\n",
             fd_ed25519_hip_last_error() );
  }
}

int
fd_ed25519_hip_dropin_set_on_lost( int policy ) {
  if( policy!=FD_ED25519_HIP_DROPIN_ON_LOST_ABORT && policy!=FD_ED25519_HIP_DROPIN_ON_LOST_REJECT )
    return FD_ED25519_HIP_ERR_INVAL;
  pthread_mutex_lock( &dropin_lock );
  int prev = dq.on_lost;
  dq.on_lost = policy;
  pthread_mutex_unlock( &dropin_lock );
  return prev;
}

int
fd_ed25519_hip_dropin_status( unsigned long * recoveries ) {
  pthread_mutex_lock( &dropin_lock );
  int lost = dq.lost;
  if( recoveries ) *recoveries = dq.recoveries;
  pthread_mutex_unlock( &dropin_lock );
  return lost;
}

/* One combined launch of the requests in list (n of them) on drop-in
   engine k.  A drop-in call is latency-bound (a handful of signatures per
   GPU round trip), so the launch moves one pinned block each way instead
   of an array per field: in, [off | sz | tfirst | tcnt | sigs | pubs |
   msgs] (sigs and pubs 16-byte aligned, 16 readable bytes past the last
   message for the SHA-512 loader); out, [codes | per-transaction codes].
   The per-transaction combine (batch_single_msg's priority rule) runs only
   when a request has more than one signature; a lone signature's code is
   its request's result. */
#define DROPIN_ALIGN16( x ) (((x) + 15UL) & ~15UL)

#ifdef FD_ED25519_HIP_HOST_FAULT
/* test build only (tests/test_gpu_dropin_fault.py): with
   $FD_ED25519_HIP_FAULT_DROPIN = "a:b", drop-in launches a .. a+b-1 (counted
   from 1 over the process, retries included) fail as a launch failure
   would, after their inputs are staged */
static int
dropin_fault( void ) {
  static unsigned long cnt;
  char const * f = getenv( "FD_ED25519_HIP_FAULT_DROPIN" );
  unsigned long i = __atomic_add_fetch( &cnt, 1UL, __ATOMIC_RELAXED );
  if( !f || !*f ) return 0;
  char * e;
  unsigned long a = strtoul( f, &e, 10 ), b = *e==':' ? strtoul( e+1, NULL, 10 ) : 1UL;
  return i>=a && i<a+b;
}
#endif

static int
dropin_run( int k, dropin_req_t * list, unsigned long n ) {
  fd_ed25519_hip_engine_t * e = dq.eng[k];
  if( !e ) {
    snprintf( fd_ed25519_hip_errbuf, sizeof(fd_ed25519_hip_errbuf), "drop-in engine %d was not created", k );
    return FD_ED25519_HIP_ERR_INVAL;
  }
  HIPCHK( hipSetDevice( e->device ), "hipSetDevice" );
  /* A direct launch returned when its codes landed, before its stream's
     completion signal (below): an error raised after that (a wave faulting
     on its way out) surfaces here, before this launch restages the block.
     It is reported as the earlier launch's, and this launch then runs on a
     re-created engine (dropin_retry). */
  if( dq.direct_pending[k] ) {
    dq.direct_pending[k] = 0;
    hipError_t q = hipStreamQuery( e->stream );
    if( q!=hipSuccess && q!=hipErrorNotReady ) {
      snprintf( fd_ed25519_hip_errbuf, sizeof(fd_ed25519_hip_errbuf),
                "drop-in: engine %d's previous direct launch ended with %s after its codes landed", k,
                hipGetErrorString( q ) );
      return FD_ED25519_HIP_ERR_HIP - (int)q;
    }
  }
  /* signatures of requests hashed on the host go after the others: the
     device hashes [0, nsig_m), takes digests for [nsig_m, nsig) */
  uint64_t nsig = 0UL, nsig_h = 0UL, bytes = 0UL;
  int multi = 0;
  for( dropin_req_t * r=list; r; r=r->next ) {
    nsig += r->cnt; multi |= r->cnt>1U;
    if( r->hashed ) nsig_h += r->cnt; else bytes += r->msg_sz;
  }
  uint64_t nsig_m = nsig - nsig_h;
  /* host scalars (a launch of a few signatures -- fd_ed25519_verify calls,
     or batch_single_msg transactions of a few signatures, whose codes are
     then combined on the host -- any message size below the host-hash
     limit): the calling thread hashes and finds
     the scalars, the device reads sflag / hflag [cap] and hs [19][cap] in
     the block (the work arrays' stride, the first nsig of each row
     written) and never the messages, which are not staged; a signature
     without a half-size pair (~1e-6) takes the device path from its
     digest (room for nsig digests) */
  int hsmode = nsig<=dropin_hs_max && !nsig_h;
  int hdmode = hsmode && nsig<=dropin_hd_max;
  uint64_t ndig   = hsmode ? nsig : nsig_h;
  uint64_t o_off  = 0UL;
  uint64_t o_sz   = DROPIN_ALIGN16( o_off  + 8UL*nsig );
  uint64_t o_tf   = DROPIN_ALIGN16( o_sz   + 4UL*nsig );
  uint64_t o_tc   = DROPIN_ALIGN16( o_tf   + 4UL*n );
  uint64_t o_sig  = DROPIN_ALIGN16( o_tc   + 4UL*n );
  uint64_t o_pub  = DROPIN_ALIGN16( o_sig  + 64UL*nsig );
  uint64_t o_dig  = DROPIN_ALIGN16( o_pub  + 32UL*nsig );
  uint64_t o_msg  = DROPIN_ALIGN16( o_dig  + 64UL*ndig );
  uint64_t in_sz  = o_msg + ( hsmode ? 0UL : bytes );
  uint64_t o_out  = DROPIN_ALIGN16( in_sz + 16UL );
  uint64_t o_tout = o_out + nsig;
  uint64_t need   = o_tout + n + 16UL;
  /* the host arrays' stride: the work arrays' when the device decodes
     (its pts / pflag), a small one when every array is the caller's */
  uint64_t cap_hs = hdmode ? FD_ED25519_HS_STRIDE : e->max_chunk;
  uint64_t o_hsf = DROPIN_ALIGN16( need ), o_hhf = DROPIN_ALIGN16( o_hsf + cap_hs ), o_hs = DROPIN_ALIGN16( o_hhf + cap_hs );
  /* hs: 19 rows (dsm16) or 24 (dsm16s's split scalars); pts: A, R and,
     for dsm16s, the doubled points (up to 8 rows of 40 limbs: dsm16s reads
     rows of 40, dsm16 of 20) */
  int split = hdmode && dropin_split>2 && fd_ed25519_hip_private_want_dsms( e, dropin_split ) ? dropin_split : 0;
  uint64_t o_pts = DROPIN_ALIGN16( o_hs + 24UL*4UL*cap_hs ), o_pfl = DROPIN_ALIGN16( o_pts + 8UL*40UL*4UL*cap_hs );
  uint64_t o_go  = DROPIN_ALIGN16( o_pfl + 2UL*cap_hs );
  if( hsmode ) need = hdmode ? o_go + 16UL : o_hs + 19UL*4UL*cap_hs;
  if( need>dq.blk_cap[k] ) {
    uint64_t cap = dq.blk_cap[k] ? dq.blk_cap[k] : (1UL<<20);
    while( cap<need ) cap *= 2UL;
    hipStreamSynchronize( e->stream );   /* a direct launch may still be ending (see below) */
    hipHostFree( dq.h_blk[k] ); hipFree( dq.d_blk[k] );
    dq.h_blk[k] = NULL; dq.h_dev[k] = NULL; dq.d_blk[k] = NULL; dq.blk_cap[k] = 0UL;
    HIPCHK( hipHostMalloc( (void **)&dq.h_blk[k], cap, hipHostMallocCoherent ), "hipHostMalloc(drop-in)" );
    HIPCHK( hipHostGetDevicePointer( (void **)&dq.h_dev[k], dq.h_blk[k], 0U ), "hipHostGetDevicePointer(drop-in)" );
    HIPCHK( hipMalloc( (void **)&dq.d_blk[k], cap ), "hipMalloc(drop-in)" );
    dq.blk_cap[k] = cap;
  }
  unsigned char * h = dq.h_blk[k];
  unsigned char * d = dq.d_blk[k];
  unsigned long * off = (unsigned long *)(h + o_off);
  unsigned int *  sz  = (unsigned int  *)(h + o_sz);
  uint32_t *      tf  = (uint32_t      *)(h + o_tf);
  uint32_t *      tc  = (uint32_t      *)(h + o_tc);
  uint64_t pos = 0UL, j = 0UL, jh = nsig_m, t = 0UL;
  for( dropin_req_t * r=list; r; r=r->next, t++ ) {
    uint64_t s0 = r->hashed ? jh : j;
    tf[t] = (uint32_t)s0;
    tc[t] = r->cnt;
    memcpy( h + o_sig + 64UL*s0, r->sigs, 64UL*r->cnt );
    memcpy( h + o_pub + 32UL*s0, r->pubs, 32UL*r->cnt );
    if( r->hashed ) {
      memcpy( h + o_dig + 64UL*(s0 - nsig_m), r->dig, 64UL*r->cnt );
      for( uint32_t i=0U; i<r->cnt; i++ ) { off[s0+i] = 0UL; sz[s0+i] = 0U; }
      jh += r->cnt;
    } else if( hsmode ) {   /* the device never reads the message */
      for( uint32_t i=0U; i<r->cnt; i++ ) { off[s0+i] = 0UL; sz[s0+i] = 0U; }
      j += r->cnt;
    } else {
      if( r->msg_sz ) memcpy( h + o_msg + pos, r->msg, r->msg_sz );
      for( uint32_t i=0U; i<r->cnt; i++ ) { off[s0+i] = pos; sz[s0+i] = (unsigned int)r->msg_sz; }
      pos += r->msg_sz;
      j += r->cnt;
    }
  }
  hipStream_t st = e->stream;
#ifdef FD_ED25519_HIP_HOST_FAULT
  if( dropin_fault() ) {
    snprintf( fd_ed25519_hip_errbuf, sizeof(fd_ed25519_hip_errbuf),
              "drop-in: injected launch failure (fault-injection build)" );
    return FD_ED25519_HIP_ERR_HIP - (int)hipErrorLaunchFailure;
  }
#endif
  /* A launch of a few signatures (one caller alone, the latency case) has
     the kernels read its inputs and write its codes through the pinned
     block's device-visible address: no copy launches, two kernels fewer on
     the call's path (the hash's first loads wait on the link instead, a
     few hundred bytes).  A larger combined launch moves the block by
     device launches (fd_ed25519_hip_launch_pull), not copy-engine calls:
     several drop-in engines submit from their callers' threads at once
     (DESIGN.md 3c), and one bulk read beats every lane reading over the
     link. */
  int direct = hsmode || ( nsig<=DROPIN_DIRECT_MAX && !multi && in_sz<=DROPIN_DIRECT_MAX_BYTES );
  unsigned char * src = direct ? dq.h_dev[k] : d;
  if( direct ) memset( h + o_out, DROPIN_PENDING, nsig );   /* no code is this value */
  fd_ed25519_pull_params_t pp;
  memset( &pp, 0, sizeof(pp) );
  if( !direct ) {
    pp.src[0] = dq.h_dev[k]; pp.dst[0] = d; pp.n[0] = in_sz ? in_sz : 1UL; pp.cnt = 1U;
    HIPCHK( (hipError_t)fd_ed25519_hip_launch_pull( &pp, st ), "H2D drop-in" );
  }
  int err = FD_ED25519_HIP_OK, hsdone = 0;
  if( direct && hsmode ) {
    /* the device's decompressions now and the group equation after the
       scalars this thread computes meanwhile -- or, for the fewest
       signatures, the group equation launched first, waiting, and this
       thread's scalars and decompressions while it is dispatched (a
       signature without a half-size pair, ~1e-6, sends the launch down the
       device's own path instead) */
    volatile uint32_t * go = (volatile uint32_t *)(h + o_go);
    if( !hdmode ) {
      err = fd_ed25519_hip_private_hs_decode( e, nsig, src + o_sig, src + o_pub, (signed char *)(src + o_out), st );
      if( err ) { hipStreamSynchronize( st ); return err; }
    } else {
      /* dsm16 goes first and waits on the go word (params.go), so its
         dispatch overlaps this thread's scalars and decompressions; from
         here every path stores RUN or CANCEL */
      *go = 0U;
      if( split )
        err = fd_ed25519_hip_private_hs_dsms( e, split, nsig, src + o_sig, src + o_pub, (signed char *)(src + o_out),
                                              src + o_hsf, src + o_hhf, (unsigned int const *)(src + o_hs),
                                              (int const *)(src + o_pts), src + o_pfl,
                                              (unsigned int const *)(src + o_go), st );
      else
        err = fd_ed25519_hip_private_hs_dsm( e, nsig, src + o_sig, src + o_pub, (signed char *)(src + o_out),
                                             src + o_hsf, src + o_hhf, (unsigned int const *)(src + o_hs),
                                             (int const *)(src + o_pts), src + o_pfl,
                                             (unsigned int const *)(src + o_go), st );
      if( err ) { hipStreamSynchronize( st ); return err; }
    }
    uint8_t *  hsf = (uint8_t *)(h + o_hsf);
    uint8_t *  hhf = (uint8_t *)(h + o_hhf);
    uint32_t * hs  = (uint32_t *)(h + o_hs);
    int all = 1;
    int dbits = dropin_hs_dbits ? dropin_hs_dbits : engine_half_dbits( e );
    t = 0UL;
    for( dropin_req_t * r=list; r && all; r=r->next, t++ ) {
      for( uint32_t i=0U; i<r->cnt && all; i++ ) {   /* a batch_single_msg request: its signatures over one message */
        uint32_t rec[ 32 ];
        all = fd_ed25519_hip_private_hsrec( r->sigs + 64UL*i, r->pubs + 32UL*i, r->msg, r->msg_sz, dbits, rec );
        if( !all ) break;
        uint64_t j = tf[ t ] + i;
        if( split ) fd_ed25519_hip_private_hssplit( rec, split, hs, cap_hs, j );
        else for( int w=0; w<19; w++ ) hs[ (uint64_t)w*cap_hs + j ] = rec[ 8 + w ];
        hsf[ j ] = (uint8_t)rec[ 27 ];
        hhf[ j ] = (uint8_t)rec[ 28 ];
      }
    }
    if( all && hdmode ) {   /* A and R of each signature, side by side (and doubled, for dsm16s) */
      unsigned char const * enc[ 2UL*DROPIN_HD_CAP ];
      int32_t       pt[ 2UL*DROPIN_HD_CAP ][ 20 ], ptx[ 2UL*DROPIN_HD_CAP*3UL ][ 40 ];
      unsigned char fl[ 2UL*DROPIN_HD_CAP ];
      int nx = split ? split/2 - 1 : 0, step = split==4 ? 66 : 33;
      /* signature j (the requests' signatures in order) at enc[2j], enc[2j+1] */
      t = 0UL;
      for( dropin_req_t * r=list; r; r=r->next, t++ )
        for( uint32_t i=0U; i<r->cnt; i++ ) {
          enc[ 2UL*( tf[ t ] + i ) ] = r->pubs + 32UL*i; enc[ 2UL*( tf[ t ] + i ) + 1UL ] = r->sigs + 64UL*i;
        }
      fd_ed25519_hip_private_hsdec3_n( enc, 2UL*nsig, !(e->flags & FD_ED25519_HIP_FLAG_CODES_PORTABLE), &pt[0][0],
                                       split ? &ptx[0][0] : NULL, nx, step, fl );
      int32_t * pts = (int32_t *)(h + o_pts);
      uint8_t * pfl = (uint8_t *)(h + o_pfl);
      uint64_t rs = split ? 40UL : 20UL;   /* the row stride in limbs: dsm16s's, dsm16's */
      for( uint64_t j=0UL; j<nsig; j++ ) {
        for( uint64_t side=0UL; side<2UL; side++ ) {   /* rows 2i + side: A, R, A_1, R_1, .. */
          uint64_t pi = 2UL*j + side;
          for( uint64_t l=0UL; l<20UL; l++ ) pts[ ( side*rs + l )*cap_hs + j ] = pt[ pi ][ l ];
          for( int m=1; m<=nx; m++ )
            for( uint64_t l=0UL; l<40UL; l++ )
              pts[ ( ( 2UL*(uint64_t)m + side )*40UL + l )*cap_hs + j ] = ptx[ pi*(uint64_t)nx + (uint64_t)(m-1) ][ l ];
          pfl[ side*cap_hs + j ] = fl[ pi ];
        }
      }
    }
    if( hdmode ) __atomic_store_n( go, all ? FD_ED25519_GO_RUN : FD_ED25519_GO_CANCEL, __ATOMIC_RELEASE );
    if( all && !hdmode ) {
      err = fd_ed25519_hip_private_hs_dsm( e, nsig, src + o_sig, src + o_pub, (signed char *)(src + o_out),
                                           src + o_hsf, src + o_hhf, (unsigned int const *)(src + o_hs), NULL, NULL,
                                           NULL, st );
    } else if( !all ) {   /* the device path from the digests (the messages were not staged) */
      t = 0UL;
      for( dropin_req_t * r=list; r; r=r->next, t++ )
        for( uint32_t i=0U; i<r->cnt; i++ )
          fd_ed25519_hip_private_challenge( r->sigs + 64UL*i, r->pubs + 32UL*i, r->msg, r->msg_sz,
                                            h + o_dig + 64UL*( tf[ t ] + i ) );
      err = fd_ed25519_hip_verify_digests_dev( e, nsig, src + o_dig, src + o_sig, src + o_pub,
                                               (signed char *)(src + o_out), st );
    }
    if( err ) { hipStreamSynchronize( st ); return err; }
    hsdone = 1;
  }
  if( !hsdone )
    err = fd_ed25519_hip_verify_dev( e, nsig_m, src + o_msg, (unsigned long const *)(src + o_off),
                                     (unsigned int const *)(src + o_sz), src + o_sig, src + o_pub,
                                     (signed char *)(src + o_out), st );
  if( !err && nsig_h )
    err = fd_ed25519_hip_verify_digests_dev( e, nsig_h, src + o_dig, src + o_sig + 64UL*nsig_m,
                                             src + o_pub + 32UL*nsig_m, (signed char *)(src + o_out + nsig_m), st );
  if( err ) { hipStreamSynchronize( st ); return err; }
  if( multi && !direct ) {   /* (a direct multi-signature launch is a host-scalar one: combined below) */
    err = fd_ed25519_hip_txn_combine_dev( e, n, (signed char const *)(d + o_out), (uint32_t const *)(d + o_tf),
                                          (uint32_t const *)(d + o_tc), (signed char *)(d + o_tout), st );
    if( err ) { hipStreamSynchronize( st ); return err; }
  }
  if( !direct ) {
    pp.src[0] = d + o_out; pp.dst[0] = dq.h_dev[k] + o_out; pp.n[0] = multi ? nsig + n : nsig;
    HIPCHK( (hipError_t)fd_ed25519_hip_launch_pull( &pp, st ), "D2H drop-in" );
  }
  if( direct ) {
    /* The codes land in the pinned block as the kernels write them: the
       call returns when all are there, without waiting for the stream's
       completion signal (the kernels read nothing of this block after
       writing a code, and the engine's next launch is ordered behind
       them on its stream).  The stream is queried every 64 polls, so a
       failed launch still ends the wait with its error. */
    volatile signed char const * c = (volatile signed char const *)(h + o_out);
    for( unsigned long spin=1UL;; spin++ ) {
      unsigned long i = 0UL;
      while( i<nsig && c[ i ]!=(signed char)DROPIN_PENDING ) i++;
      if( i==nsig ) break;
      if( !(spin & 63UL) ) {
        hipError_t q = hipStreamQuery( st );
        if( q==hipErrorNotReady ) continue;
        HIPCHK( q, "drop-in verify" );
        /* the stream is done: every code must be there */
        for( i=0UL; i<nsig && c[ i ]!=(signed char)DROPIN_PENDING; i++ ) ;
        if( i<nsig ) {
          snprintf( fd_ed25519_hip_errbuf, sizeof(fd_ed25519_hip_errbuf), "drop-in: a launch ended without a code" );
          return FD_ED25519_HIP_ERR_HIP - (int)hipErrorLaunchFailure;
        }
        break;
      }
      __builtin_ia32_pause();
    }
    dq.direct_pending[k] = 1;
  } else {
    HIPCHK( hipStreamSynchronize( st ), "drop-in verify" );
  }
  signed char const * codes = (signed char const *)(h + o_out);
  signed char const * tcode = (signed char const *)(h + o_tout);
  if( multi && direct ) {
    /* batch_single_msg's rule per request (fd_ed25519_user.c:231-309, the
       device's fd_ed25519_txn_combine_kernel): the first error other than
       ERR_MSG in signature order, else ERR_MSG if any signature had it,
       else SUCCESS (1..16 signatures: the guard ran before submit) */
    t = 0UL;
    for( dropin_req_t * r=list; r; r=r->next, t++ ) {
      int code = FD_ED25519_SUCCESS, msg_fail = 0;
      for( uint32_t i=0U; i<r->cnt; i++ ) {
        int c = codes[ tf[ t ] + i ];
        if( c==FD_ED25519_ERR_MSG ) msg_fail = 1;
        else if( c!=FD_ED25519_SUCCESS ) { code = c; break; }
      }
      if( code==FD_ED25519_SUCCESS && msg_fail ) code = FD_ED25519_ERR_MSG;
      ((signed char *)(h + o_tout))[ t ] = (signed char)code;
    }
  }
  t = 0UL;
  for( dropin_req_t * r=list; r; r=r->next, t++ )
    r->result = (r->single || !multi) ? (int)codes[ tf[t] ] : (int)tcode[t];
  return FD_ED25519_HIP_OK;
}

/* a failed launch on engine k: the engine is made anew and the launch run
   once more (outside the lock, engine k is this thread's while busy) */
static int
dropin_retry( int k, dropin_req_t * list, unsigned long n, int err ) {
  fprintf( stderr, "libfd_ed25519_hip: drop-in launch failed: %s (%d): %s; re-creating engine %d and retrying once\n",
           fd_ed25519_hip_strerror( err ), err, fd_ed25519_hip_last_error(), k );
  int e2 = dropin_engine_make( k );
  if( !e2 ) e2 = dropin_run( k, list, n );
  return e2;
}

/* the device is lost (under dropin_lock): the ABORT policy ends here; the
   REJECT one fails every queued request closed */
static void
dropin_lose( int err ) {
  if( !dq.lost ) dq.lost = err;
  if( dq.on_lost==FD_ED25519_HIP_DROPIN_ON_LOST_ABORT ) dropin_fatal( err, "GPU verify failed twice (after a retry)" );
  for( dropin_req_t * q=dq.head; q; ) { dropin_req_t * nx = q->next; q->result = FD_ED25519_ERR_SIG; q->done = 1; q = nx; }
  dq.head = dq.tail = NULL;
}

static int
dropin_submit( dropin_req_t * r ) {
  pthread_once( &dropin_once, dropin_init );
  r->done = 0; r->next = NULL;
  pthread_mutex_lock( &dropin_lock );
  if( dq.lost ) {   /* fail closed (REJECT; ABORT never gets here) */
    pthread_mutex_unlock( &dropin_lock );
    return FD_ED25519_ERR_SIG;
  }
  if( dq.tail ) dq.tail->next = r; else dq.head = r;
  dq.tail = r;
  while( !r->done ) {
    int k = -1;
    for( int i=0; i<DROPIN_ENGINES; i++ ) if( !dq.busy[i] ) { k = i; break; }
    if( k<0 || !dq.head ) { pthread_cond_wait( &dropin_cv, &dropin_lock ); continue; }
    /* combine: take up to DROPIN_BATCH_MAX queued requests onto engine k */
    dropin_req_t * list = dq.head, * last = dq.head;
    unsigned long n = 1UL;
    while( last->next && n<DROPIN_BATCH_MAX ) { last = last->next; n++; }
    dq.head = last->next;
    if( !dq.head ) dq.tail = NULL;
    last->next = NULL;
    dq.busy[k] = 1;
    dq.launches++; dq.requests += n;
    pthread_mutex_unlock( &dropin_lock );
    int err = dropin_run( k, list, n ), retried = 0;
    if( err ) { err = dropin_retry( k, list, n, err ); retried = 1; }
    pthread_mutex_lock( &dropin_lock );
    if( err ) {
      for( dropin_req_t * q=list; q; q=q->next ) q->result = FD_ED25519_ERR_SIG;
      dropin_lose( err );
    } else if( retried ) {
      dq.recoveries++;
    }
    for( dropin_req_t * q=list; q; ) { dropin_req_t * nx = q->next; q->done = 1; q = nx; }
    dq.busy[k] = 0;
    pthread_cond_broadcast( &dropin_cv );
  }
  pthread_mutex_unlock( &dropin_lock );
  return r->result;
}

void
fd_ed25519_hip_dropin_stats( unsigned long * launches, unsigned long * requests ) {
  pthread_mutex_lock( &dropin_lock );
  if( launches ) *launches = dq.launches;
  if( requests ) *requests = dq.requests;
  pthread_mutex_unlock( &dropin_lock );
}

unsigned long
fd_ed25519_hip_dropin_device_bytes( void ) {
  pthread_once( &dropin_once, dropin_init );
  unsigned long b = 0UL;
  for( int k=0; k<DROPIN_ENGINES; k++ ) if( dq.eng[k] ) b += dq.eng[k]->device_bytes + dq.blk_cap[k];
  return b + fd_ed25519_hip_shared_device_bytes( dq.device );
}

int
fd_ed25519_hip_dropin_reset( void ) {
  pthread_once( &dropin_once, dropin_init );
  pthread_mutex_lock( &dropin_lock );
  /* every engine idle, then held: no launch starts while they are re-made */
  for( ;; ) {
    int any = 0;
    for( int k=0; k<DROPIN_ENGINES; k++ ) any |= dq.busy[k];
    if( !any ) break;
    pthread_cond_wait( &dropin_cv, &dropin_lock );
  }
  for( int k=0; k<DROPIN_ENGINES; k++ ) dq.busy[k] = 1;
  pthread_mutex_unlock( &dropin_lock );
  int err = dropin_engines_make();
  pthread_mutex_lock( &dropin_lock );
  if( !err ) dq.lost = 0;
  else if( !dq.lost ) dq.lost = err;
  for( int k=0; k<DROPIN_ENGINES; k++ ) dq.busy[k] = 0;
  pthread_cond_broadcast( &dropin_cv );
  pthread_mutex_unlock( &dropin_lock );
  return err;
}

/* The device path carries message sizes as 32-bit values; the reference
   takes any ulong size.  A message of dropin_host_hash_min bytes or more
   (4 GiB: the first size the device cannot carry) is hashed here, in the
   calling thread, with the library's own SHA-512 (one digest of R_j||A_j||M
   per signature), before the request is queued; everything after the hash
   -- the reduction mod L, decompression, the group equation, the batch
   priority rule -- runs on the GPU as for any other request.  The message
   is never truncated. */
static void
dropin_prepare( dropin_req_t * r ) {
  /* the second test is the guard whatever the limit says: a size the
     device path would truncate is never sent there */
  r->hashed = r->msg_sz>=dropin_host_hash_min || r->msg_sz>(unsigned long)UINT32_MAX;
  if( !r->hashed ) return;
  for( unsigned int j=0U; j<r->cnt; j++ )
    fd_ed25519_hip_private_challenge( r->sigs + 64UL*j, r->pubs + 32UL*j, r->msg, r->msg_sz, r->dig[ j ] );
}

int
fd_ed25519_verify( unsigned char const msg[], unsigned long msg_sz, unsigned char const sig[ 64 ],
                   unsigned char const public_key[ 32 ], fd_sha512_t * sha ) {
  (void)sha;
  dropin_req_t r;
  r.msg = msg; r.msg_sz = msg_sz; r.sigs = sig; r.pubs = public_key; r.cnt = 1U; r.single = 1;
  dropin_prepare( &r );
  return dropin_submit( &r );
}

int
fd_ed25519_verify_batch_single_msg( unsigned char const msg[], unsigned long const msg_sz,
                                    unsigned char const signatures[ 64 ], unsigned char const pubkeys[ 32 ],
                                    fd_sha512_t * shas[ 1 ], unsigned char const batch_sz ) {
  (void)shas;
  if( batch_sz==0 || batch_sz>16 ) return FD_ED25519_ERR_SIG;
  dropin_req_t r;
  r.msg = msg; r.msg_sz = msg_sz; r.sigs = signatures; r.pubs = pubkeys; r.cnt = batch_sz;
  r.single = 0;
  dropin_prepare( &r );
  return dropin_submit( &r );
}

char const *
fd_ed25519_strerror( int err ) {
  switch( err ) {
  case FD_ED25519_SUCCESS:    return "success";
  case FD_ED25519_ERR_SIG:    return "bad signature";
  case FD_ED25519_ERR_PUBKEY: return "bad public key";
  case FD_ED25519_ERR_MSG:    return "bad message";
  default: break;
  }
  return "unknown";
}
