/* fd_ed25519_hip_shlink.c -- a tango-style link in POSIX shared memory,
   so that the verify tile (inside its write/fsync-only sandbox,
   src/app/fdctl/run/tiles/verify.seccomppolicy) and a GPU process outside
   it exchange frags with memory operations only.

   One shm object per direction holds the header, an mcache of
   fd_frag_meta_t-shaped lines (src/tango/fd_tango_base.h:123-203: seq,
   sig, chunk, sz, ctl, tsorig, tspub) and a dcache of 64-byte chunks.
   Single producer, single consumer.  The producer invalidates a line
   (seq - 1), writes the payload and the metadata, then publishes seq with
   release order; the consumer reads seq with acquire order, copies, and
   re-reads seq to detect an overrun.  Flow control is credit based: the
   consumer publishes how many frags it has taken, and the producer never
   runs more than depth frags ahead (the reference's fctl / fseq pair,
   reduced to one counter).  Both sides touch that counter lazily, as
   fd_fctl does (src/tango/fctl/fd_fctl.h: credits are refilled only when
   the cached ones run out, the consumer's fseq is published periodically):
   the producer re-reads it only when the credits it last saw are spent,
   and the consumer publishes it every depth/16 frags and whenever it finds
   the link empty, so the counter's cache line does not move between the
   two cores on every frag.

   Liveness (fd_cnc's heartbeat / signal pair, src/tango/cnc/fd_cnc.h:63-65,
   129-130, reduced to two words): each producer ticks a heartbeat word in
   the header of the link it produces, and either side can mark the link
   failed with a nonzero status.  A peer that sees the heartbeat stop
   advancing for longer than its bound, or a failed status, knows the other
   process is gone or gave up, instead of waiting on credits or frags that
   will never come.

   Zero-copy forms: prepare / commit let a producer write a payload straight
   into the dcache (the verify tile's during_frag copies an incoming frag
   there), peek / advance let a consumer read a frag in place.

   The two sides need not trust each other (the tile may be compromised):
   the geometry (depth, chunk count, MTU) is validated once at create /
   join and kept in the process-local handle; later writes to the shared
   header are never read again, and every frag a consumer takes is bounds
   checked against the local geometry before its payload is copied (the
   reference tile's own check, src/app/fdctl/run/tiles/fd_verify.c:67).

   Versioning and restarts: the header carries the frag protocol both
   sides speak (FD_ED25519_HIP_SHLINK_PROTO); join refuses a link of
   another protocol (errno EPROTO), so a tile and a service built from
   different revisions of the verdict protocol never exchange frags.  The
   creator holds an exclusive flock on the link's object for the link's
   lifetime (the kernel drops it when the creator exits, however it
   exits): create reclaims a same-name link whose lock it can take (a
   service that was killed leaves its links behind) instead of failing,
   and still refuses one whose creator holds the lock.  The lock lives on
   the object, not on a pid, so it means the same in every PID namespace
   that maps /dev/shm; the reclaimer holds it while it unlinks, and only
   unlinks the object it inspected (same inode), so two creators racing
   for one stale name cannot remove each other's new link.  The creator's
   pid is still recorded (diagnostics).

   No HIP: this file is also linked into the standalone sandboxed producer
   (tools/shlink_producer.c). */
#define _GNU_SOURCE
#include "../../../include/fd_ed25519_hip_tile.h"

#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/file.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#define SHLINK_MAGIC 0xfd25519517a4c0dfUL   /* ...c0de before the protocol word (ABI <= 4) */
#define SHLINK_CHUNK 64UL

typedef struct {
  _Atomic uint64_t seq;
  uint64_t         sig;
  uint32_t         chunk;
  uint16_t         sz;
  uint16_t         ctl;
  uint32_t         tsorig;
  uint32_t         tspub;
} shlink_meta_t;

typedef struct {
  uint64_t         magic;
  uint64_t         depth;       /* mcache lines, power of 2 */
  uint64_t         chunk_cnt;   /* dcache chunks */
  uint64_t         mtu;
  _Atomic uint64_t heartbeat;   /* producer's liveness tick (0: not started) */
  _Atomic uint64_t status;      /* 0, or a failure code either side wrote     */
  uint64_t         proto;       /* FD_ED25519_HIP_SHLINK_PROTO of the creator  */
  uint64_t         creator;     /* pid of the creating process                 */
  _Atomic uint64_t consumed;    /* consumer -> producer credits (own line) */
  uint64_t         pad1[7];
} shlink_hdr_t;

struct fd_ed25519_hip_shlink {
  shlink_hdr_t *  hdr;
  shlink_meta_t * mcache;
  unsigned char * dcache;
  size_t          map_sz;
  char            name[ 128 ];
  int             lock_fd;    /* creator: the object's fd holding its flock (-1: a joined link) */
  /* process-local cursor: the next seq to publish (producer) or take
     (consumer), and the producer's next dcache chunk */
  uint64_t        seq;
  uint64_t        chunk;
  int             prepared;   /* producer: prepare() found a credit for seq */
  uint64_t        cr_seen;    /* producer: the consumer's count when last read */
  uint64_t        cr_pub;     /* consumer: the count last published          */
  uint64_t        cr_batch;   /* consumer: publish at least every cr_batch frags */
  /* process-local geometry, validated at create / join */
  uint64_t        depth;
  uint64_t        chunk_cnt;
  uint64_t        mtu;
};

static uint64_t
shlink_mtu_chunks( void ) {
  return (FD_ED25519_HIP_SHLINK_MTU + SHLINK_CHUNK - 1UL) / SHLINK_CHUNK;
}

static size_t
shlink_footprint( uint64_t depth, uint64_t chunk_cnt ) {
  return sizeof(shlink_hdr_t) + depth * sizeof(shlink_meta_t) + chunk_cnt * SHLINK_CHUNK;
}

static fd_ed25519_hip_shlink_t *
shlink_map( char const * name, int fd, size_t sz ) {
  /* MAP_POPULATE: every page of the link is allocated (creator) and
     mapped (either side) here, not by a first touch inside the stream --
     a fault per 4 KiB of dcache as the first frags pass held both sides
     for microseconds at a time */
  void * m = mmap( NULL, sz, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd, 0 );
  close( fd );
  if( m==MAP_FAILED ) return NULL;
  fd_ed25519_hip_shlink_t * l = (fd_ed25519_hip_shlink_t *)calloc( 1, sizeof(*l) );
  if( !l ) { munmap( m, sz ); return NULL; }
  l->hdr    = (shlink_hdr_t *)m;
  l->mcache = (shlink_meta_t *)( (unsigned char *)m + sizeof(shlink_hdr_t) );
  l->map_sz = sz;
  snprintf( l->name, sizeof(l->name), "%s", name );
  l->lock_fd = -1;
  return l;
}

/* Removes `name` if it is a link of this layout left behind by a creator
   that has exited: its flock can be taken.  The lock is held across the
   unlink, and the name is removed only while it still refers to the
   object inspected (same device and inode).  1 if removed. */
static int
shlink_reclaim( char const * name ) {
  int fd = shm_open( name, O_RDONLY, 0 );
  if( fd<0 ) return 0;
  int removed = 0;
  struct stat st;
  if( !flock( fd, LOCK_EX | LOCK_NB ) && !fstat( fd, &st ) && (size_t)st.st_size>=sizeof(shlink_hdr_t) ) {
    void * m = mmap( NULL, sizeof(shlink_hdr_t), PROT_READ, MAP_SHARED, fd, 0 );
    if( m!=MAP_FAILED ) {
      shlink_hdr_t const * h = (shlink_hdr_t const *)m;
      int ours = h->magic==SHLINK_MAGIC;   /* a half-made object is its creator's, locked */
      /* A creator of protocol 5 held no flock: for its links the free lock
         says nothing, and only a creator pid that no longer exists does. */
      if( ours && h->proto<FD_ED25519_HIP_SHLINK_PROTO &&
          ( !h->creator || !kill( (pid_t)h->creator, 0 ) || errno!=ESRCH ) ) ours = 0;
      munmap( m, sizeof(shlink_hdr_t) );
      char path[ 160 ];
      struct stat now;
      snprintf( path, sizeof(path), "/dev/shm/%s", name[0]=='/' ? name + 1 : name );
      if( ours && !stat( path, &now ) && now.st_ino==st.st_ino && now.st_dev==st.st_dev && !shm_unlink( name ) )
        removed = 1;
    }
  }
  close( fd );   /* drops the lock */
  return removed;
}

fd_ed25519_hip_shlink_t *
fd_ed25519_hip_shlink_create( char const * name, unsigned long depth ) {
  if( !name || !depth || (depth & (depth-1UL)) || strlen( name )>=120 ) { errno = EINVAL; return NULL; }
  uint64_t chunk_cnt  = (depth + 2UL) * shlink_mtu_chunks();
  size_t   sz         = shlink_footprint( depth, chunk_cnt );
  int fd = shm_open( name, O_RDWR | O_CREAT | O_EXCL, 0600 );
  if( fd<0 && errno==EEXIST ) {
    /* a previous creator's link: reclaimed (a peer that still maps it keeps
       the old object, whose heartbeat has stopped); a live creator's stays */
    if( shlink_reclaim( name ) ) fd = shm_open( name, O_RDWR | O_CREAT | O_EXCL, 0600 );
    else                         errno = EEXIST;
  }
  if( fd<0 ) return NULL;   /* errno EEXIST: a live process's link of that name */
  /* the creator's lock, before the object has a size or a magic: a
     reclaimer that got in first sees no magic and lets go (blocking here
     only for that moment) */
  int lk;
  do lk = flock( fd, LOCK_EX ); while( lk && errno==EINTR );
  int mfd = lk ? -1 : dup( fd );
  if( lk || mfd<0 || ftruncate( fd, (off_t)sz ) ) {
    int e = errno;
    if( mfd>=0 ) close( mfd );
    close( fd ); shm_unlink( name ); errno = e; return NULL;
  }
  fd_ed25519_hip_shlink_t * l = shlink_map( name, mfd, sz );
  if( !l ) { close( fd ); shm_unlink( name ); return NULL; }
  l->lock_fd = fd;
  l->dcache = (unsigned char *)l->mcache + depth * sizeof(shlink_meta_t);
  for( uint64_t k=0UL; k<depth; k++ ) {
    atomic_store_explicit( &l->mcache[ k ].seq, k - depth, memory_order_relaxed );
  }
  l->hdr->depth     = l->depth     = depth;
  l->hdr->chunk_cnt = l->chunk_cnt = chunk_cnt;
  l->cr_batch       = depth>=16UL ? depth/16UL : 1UL;
  l->hdr->mtu       = l->mtu       = FD_ED25519_HIP_SHLINK_MTU;
  l->hdr->proto     = FD_ED25519_HIP_SHLINK_PROTO;
  l->hdr->creator   = (uint64_t)getpid();
  atomic_store_explicit( &l->hdr->consumed, 0UL, memory_order_relaxed );
  atomic_store_explicit( &l->hdr->heartbeat, 0UL, memory_order_relaxed );
  atomic_store_explicit( &l->hdr->status, 0UL, memory_order_relaxed );
  atomic_thread_fence( memory_order_release );
  l->hdr->magic = SHLINK_MAGIC;
  return l;
}

fd_ed25519_hip_shlink_t *
fd_ed25519_hip_shlink_join( char const * name ) {
  if( !name ) { errno = EINVAL; return NULL; }
  int fd = shm_open( name, O_RDWR, 0600 );
  if( fd<0 ) return NULL;   /* errno ENOENT: no such link (no service) */
  struct stat st;
  if( fstat( fd, &st ) || (size_t)st.st_size<sizeof(shlink_hdr_t) ) { close( fd ); errno = EINVAL; return NULL; }
  fd_ed25519_hip_shlink_t * l = shlink_map( name, fd, (size_t)st.st_size );
  if( !l ) return NULL;
  /* one snapshot of the geometry, checked against what create makes */
  uint64_t magic     = l->hdr->magic;
  atomic_thread_fence( memory_order_acquire );
  uint64_t depth     = l->hdr->depth;
  uint64_t chunk_cnt = l->hdr->chunk_cnt;
  uint64_t mtu       = l->hdr->mtu;
  uint64_t proto     = l->hdr->proto;
  if( magic!=SHLINK_MAGIC || proto!=FD_ED25519_HIP_SHLINK_PROTO ) {
    /* another layout or frag protocol (an earlier magic is a link of ABI <= 4) */
    munmap( l->hdr, l->map_sz ); free( l ); errno = EPROTO; return NULL;
  }
  if( !depth || (depth & (depth-1UL)) || depth>(1UL<<30) ||
      mtu!=FD_ED25519_HIP_SHLINK_MTU || chunk_cnt!=(depth + 2UL) * shlink_mtu_chunks() ||
      shlink_footprint( depth, chunk_cnt )!=l->map_sz ) {
    munmap( l->hdr, l->map_sz ); free( l ); errno = EINVAL; return NULL;
  }
  l->depth = depth; l->chunk_cnt = chunk_cnt; l->mtu = mtu;
  l->cr_batch = depth>=16UL ? depth/16UL : 1UL;
  l->dcache = (unsigned char *)l->mcache + depth * sizeof(shlink_meta_t);
  return l;
}

void
fd_ed25519_hip_shlink_leave( fd_ed25519_hip_shlink_t * l, int unlink ) {
  if( !l ) return;
  if( unlink ) shm_unlink( l->name );
  munmap( l->hdr, l->map_sz );
  if( l->lock_fd>=0 ) close( l->lock_fd );   /* the creator's lock goes last */
  free( l );
}

unsigned long
fd_ed25519_hip_shlink_depth( fd_ed25519_hip_shlink_t const * l ) {
  return l ? l->depth : 0UL;
}

unsigned char const *
fd_ed25519_hip_shlink_dcache( fd_ed25519_hip_shlink_t const * l, unsigned long * sz ) {
  if( sz ) *sz = l->chunk_cnt*SHLINK_CHUNK;
  return l->dcache;
}

void *
fd_ed25519_hip_shlink_mapping( fd_ed25519_hip_shlink_t const * l, unsigned long * sz ) {
  if( sz ) *sz = l->map_sz;
  return l->hdr;
}

/* The payload room of the next frag if the consumer has returned a credit
   for it, else NULL.  The room is MTU bytes inside this side's dcache; it
   is reused for a later frag only after depth+1 more frags, so it is never
   a region the consumer may still be reading. */
unsigned char *
fd_ed25519_hip_shlink_prepare( fd_ed25519_hip_shlink_t * l ) {
  /* a bogus credit count from the consumer only lets the producer overrun
     that consumer: every write stays inside the local geometry.  The count
     is re-read only when the credits last seen are spent. */
  if( l->seq - l->cr_seen>=l->depth ) {
    l->cr_seen = atomic_load_explicit( &l->hdr->consumed, memory_order_acquire );
    if( l->seq - l->cr_seen>=l->depth ) return NULL;
  }
  uint64_t mtu_chunks = (l->mtu + SHLINK_CHUNK - 1UL) / SHLINK_CHUNK;
  if( l->chunk + mtu_chunks>l->chunk_cnt ) l->chunk = 0UL;   /* compact wrap */
  l->prepared = 1;
  return l->dcache + l->chunk*SHLINK_CHUNK;
}

int
fd_ed25519_hip_shlink_commit( fd_ed25519_hip_shlink_t * l, unsigned long sz, unsigned long sig, unsigned int ctl ) {
  if( !l->prepared || sz>l->mtu ) return FD_ED25519_HIP_ERR_INVAL;
  uint64_t seq = l->seq;
  shlink_meta_t * m = &l->mcache[ seq & (l->depth-1UL) ];
  /* the payload is already in place: invalidate the line, then write the
     metadata and publish seq (fd_mcache_publish's order) */
  atomic_store_explicit( &m->seq, seq-1UL, memory_order_relaxed );
  atomic_thread_fence( memory_order_release );
  m->sig    = sig;
  m->chunk  = (uint32_t)l->chunk;
  m->sz     = (uint16_t)sz;
  m->ctl    = (uint16_t)ctl;
  m->tsorig = 0U;
  m->tspub  = 0U;
  atomic_store_explicit( &m->seq, seq, memory_order_release );
  l->chunk   += (sz + SHLINK_CHUNK - 1UL) / SHLINK_CHUNK;
  l->seq      = seq + 1UL;
  l->prepared = 0;
  return 0;
}

int
fd_ed25519_hip_shlink_publish( fd_ed25519_hip_shlink_t * l, unsigned char const * payload, unsigned long sz,
                               unsigned long sig, unsigned int ctl ) {
  if( sz>l->mtu ) return FD_ED25519_HIP_ERR_INVAL;
  unsigned char * dst = fd_ed25519_hip_shlink_prepare( l );
  if( !dst ) return 1;   /* no credit */
  if( sz ) memcpy( dst, payload, sz );
  return fd_ed25519_hip_shlink_commit( l, sz, sig, ctl );
}

/* The next frag in place: its payload address inside this side's dcache
   (bounds checked against the local geometry, fd_verify.c:67), or NULL
   with *err = 1 (none published yet) or -1 (overrun, or a line pointing
   outside the dcache).  The bytes may be overwritten by a producer that
   ignores credits; advance() tells whether they were. */
unsigned char const *
fd_ed25519_hip_shlink_peek( fd_ed25519_hip_shlink_t * l, unsigned long * sz, unsigned long * sig, unsigned int * ctl,
                            int * err ) {
  uint64_t seq = l->seq;
  shlink_meta_t * m = &l->mcache[ seq & (l->depth-1UL) ];
  uint64_t s0 = atomic_load_explicit( &m->seq, memory_order_acquire );
  if( (int64_t)(s0 - seq)<0 ) {                               /* not yet published: */
    if( l->cr_pub!=seq ) {                                    /* the credits taken so far go back */
      l->cr_pub = seq;
      atomic_store_explicit( &l->hdr->consumed, seq, memory_order_release );
    }
    *err = 1;
    return NULL;
  }
  if( s0!=seq ) { *err = -1; return NULL; }                   /* overrun */
  unsigned long n     = m->sz;
  unsigned long sg    = m->sig;
  unsigned int  c     = m->ctl;
  unsigned long chunk = m->chunk;
  if( n>l->mtu || chunk>=l->chunk_cnt || chunk*SHLINK_CHUNK + n>l->chunk_cnt*SHLINK_CHUNK ) { *err = -1; return NULL; }
  *sz = n; *sig = sg; *ctl = c; *err = 0;
  return l->dcache + chunk*SHLINK_CHUNK;
}

/* Done with the peeked frag: 0 if it was intact while it was read, -1 if
   the producer overran it meanwhile.  Either way the credit goes back. */
int
fd_ed25519_hip_shlink_advance( fd_ed25519_hip_shlink_t * l ) {
  uint64_t seq = l->seq;
  shlink_meta_t * m = &l->mcache[ seq & (l->depth-1UL) ];
  atomic_thread_fence( memory_order_acquire );
  int ok = atomic_load_explicit( &m->seq, memory_order_relaxed )==seq;
  l->seq = seq + 1UL;
  if( l->seq - l->cr_pub>=l->cr_batch ) {
    l->cr_pub = l->seq;
    atomic_store_explicit( &l->hdr->consumed, l->seq, memory_order_release );
  }
  return ok ? 0 : -1;
}

int
fd_ed25519_hip_shlink_consume( fd_ed25519_hip_shlink_t * l, unsigned char * payload, unsigned long * sz,
                               unsigned long * sig, unsigned int * ctl ) {
  unsigned long n = 0UL, sg = 0UL;
  unsigned int c = 0U;
  int err;
  unsigned char const * src = fd_ed25519_hip_shlink_peek( l, &n, &sg, &c, &err );
  if( !src ) return err;
  if( n ) memcpy( payload, src, n );
  /* a frag overwritten during the copy is an overrun (never happens when
     the producer honours credits) */
  atomic_thread_fence( memory_order_acquire );
  shlink_meta_t * m = &l->mcache[ l->seq & (l->depth-1UL) ];
  if( atomic_load_explicit( &m->seq, memory_order_relaxed )!=l->seq ) return -1;
  *sz = n; *sig = sg; *ctl = c;
  fd_ed25519_hip_shlink_advance( l );
  return 0;
}

void
fd_ed25519_hip_shlink_heartbeat( fd_ed25519_hip_shlink_t * l, unsigned long now ) {
  atomic_store_explicit( &l->hdr->heartbeat, now, memory_order_release );
}

unsigned long
fd_ed25519_hip_shlink_heartbeat_query( fd_ed25519_hip_shlink_t const * l ) {
  return atomic_load_explicit( &l->hdr->heartbeat, memory_order_acquire );
}

int
fd_ed25519_hip_shlink_watch( fd_ed25519_hip_shlink_watch_t * w, fd_ed25519_hip_shlink_t const * l, long now_ns,
                             long stale_ns ) {
  unsigned long hb = fd_ed25519_hip_shlink_heartbeat_query( l );
  if( !w->seen || hb!=w->last ) { w->last = hb; w->t_ns = now_ns; w->seen = 1; }
  if( !hb ) return 1;     /* the producer has not ticked yet */
  return ( stale_ns>0L && now_ns - w->t_ns>stale_ns ) ? -1 : 0;
}

void
fd_ed25519_hip_shlink_fail( fd_ed25519_hip_shlink_t * l, int code ) {
  atomic_store_explicit( &l->hdr->status, (uint64_t)(int64_t)(code ? code : -1), memory_order_release );
}

int
fd_ed25519_hip_shlink_status( fd_ed25519_hip_shlink_t const * l ) {
  return (int)(int64_t)atomic_load_explicit( &l->hdr->status, memory_order_acquire );
}
