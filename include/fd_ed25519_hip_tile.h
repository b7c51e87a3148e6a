#ifndef HEADER_fd_ed25519_hip_tile_h
#define HEADER_fd_ed25519_hip_tile_h

/* libfd_ed25519_hip, part 2: the host runtime that feeds the GPU from the
   verify tile's side of Firedancer (SURVEY.md §8(b) "Needed extension for
   GPU throughput", §8(e), §8(f) rows 1-2).  Plain C over the engine of
   fd_ed25519_hip.h; every entry point is a C-ABI function of
   libfd_ed25519_hip.so.

     pipe    asynchronous submit / poll of pinned SoA batches, several in
             flight per GPU (H2D, kernels and D2H of one batch overlap the
             next batch's packing)
     txn     fd_txn_parse restated for the fields the verify tile uses
             (src/ballet/txn/fd_txn_parse.c:6-244), and the verify tile's
             tcache dedup (src/tango/tcache/fd_tcache.h:259-404)
     vtile   the verify tile's per-transaction logic, fd_txn_verify
             (src/app/fdctl/run/tiles/fd_verify.h:43-88), batched: frags
             are parsed and staged as they arrive, verified a batch at a
             time, and their verdicts released in arrival order with the
             reference's dedup semantics
     ring    a tango-style mcache / dcache (src/tango/fd_tango_base.h:123-203)
             between a producer thread and the vtile, for the latency mode
     pool    one host feeder thread and pipe per GPU, batches dealt
             round-robin (the analogue of seq % verify_tile_count,
             src/app/fdctl/run/tiles/fd_verify.c:36-47)
     shlink  the same mcache / dcache in POSIX shared memory, between
             processes, and the GPU-side verify service behind it: the
             verify tile keeps its write/fsync-only sandbox
             (src/app/fdctl/run/tiles/verify.seccomppolicy) and talks to
             the GPU process with memory operations only */

#include "fd_ed25519_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- pipe ------------------------------------------------------------- */

typedef struct fd_ed25519_hip_pipe fd_ed25519_hip_pipe_t;

/* One batch of a pipe.  Between acquire and submit the caller fills the
   pinned host arrays in place (no extra copy): signature i is sigs[64 i..]
   by pubs[32 i..] over msgs[msg_off[i] .. + msg_sz[i]).  Optionally, with
   txn_cnt > 0 at submit, transactions group consecutive signatures:
   transaction t owns [txn_first[t], txn_first[t] + txn_sig_cnt[t]) and
   gets fd_ed25519_verify_batch_single_msg's code in txn_out[t] (a count of
   0 or > 16 gives ERR_SIG, such transactions stage no signatures).  After
   poll returns the slot, sig_out / txn_out hold the codes, and after a
   raw-transaction submit txn_trailer[64 t ..] the first 64 bytes of
   transaction t's fd_txn_t as the device parsed it (complete when its
   footprint, FD_ED25519_HIP_TXN_FOOTPRINT, is at most 64 bytes). */
typedef struct {
  unsigned char *  msgs;
  unsigned long *  msg_off;
  unsigned int *   msg_sz;
  unsigned char *  sigs;
  unsigned char *  pubs;
  unsigned int *   txn_first;
  unsigned int *   txn_sig_cnt;
  signed char *    sig_out;
  signed char *    txn_out;
  unsigned char *  txn_trailer;
  unsigned long    sig_cap;
  unsigned long    msg_cap;
  unsigned long    txn_cap;
  /* set by submit */
  unsigned long    sig_cnt;
  unsigned long    msg_bytes;
  unsigned long    txn_cnt;
  unsigned long    seq;        /* submission number, 0, 1, 2, ...         */
  double           t_submit;   /* CLOCK_MONOTONIC seconds at submit        */
  double           t_done;     /* ... when poll saw the batch complete     */
  unsigned long    user;       /* caller cookie, untouched                 */
} fd_ed25519_hip_slot_t;

/* slot_cnt batches (1..8) of up to sig_cap signatures, msg_cap message
   bytes and txn_cap transactions each, on HIP device `device`; each slot
   owns an engine (its own stream and work arrays), so the batches in
   flight run concurrently.  NULL on failure (fd_ed25519_hip_last_error). */
fd_ed25519_hip_pipe_t *
fd_ed25519_hip_pipe_new( int device, unsigned slot_cnt, unsigned long sig_cap, unsigned long msg_cap,
                         unsigned long txn_cap, int flags );

void
fd_ed25519_hip_pipe_delete( fd_ed25519_hip_pipe_t * pipe );

/* The next slot in ring order if it is free, else NULL. */
fd_ed25519_hip_slot_t *
fd_ed25519_hip_pipe_acquire( fd_ed25519_hip_pipe_t * pipe );

/* Enqueues H2D, verification (and the per-transaction combine if
   txn_cnt>0) and D2H of an acquired slot; returns immediately.
   FD_ED25519_HIP_ERR_INVAL, with nothing enqueued, if a count exceeds its
   capacity, a signature's message range [msg_off, msg_off+msg_sz) is not
   within the msg_bytes staged, or a transaction's signature range
   [txn_first, txn_first+txn_sig_cnt) (counts 1..16) is not within the
   sig_cnt staged (the kernels would read out of bounds). */
int
fd_ed25519_hip_pipe_submit( fd_ed25519_hip_pipe_t * pipe, fd_ed25519_hip_slot_t * slot,
                            unsigned long sig_cnt, unsigned long msg_bytes, unsigned long txn_cnt );

/* Raw transactions: the caller copies txn_cnt
   payloads (the TPU wire format fd_txn_parse reads) into msgs, with
   msg_off[t] / msg_sz[t] per transaction.  The device parses them
   (fd_txn_parse's exact acceptance), gathers signatures and signer keys,
   verifies, and writes txn_out[t]: fd_ed25519_verify_batch_single_msg's
   code, or FD_ED25519_HIP_TXN_CODE_PARSE_FAILED.  txn_first / txn_sig_cnt
   are filled by the pipe (from payload byte 0, the signature count).  The
   signature slots (counts of 1..16) must fit sig_cap, payloads msg_cap
   (the buffer is readable 64 bytes past the end, as the kernels need);
   a payload range outside the payload_bytes staged is
   FD_ED25519_HIP_ERR_INVAL, nothing enqueued. */
#define FD_ED25519_HIP_TXN_CODE_PARSE_FAILED (-4)

int
fd_ed25519_hip_pipe_submit_txns( fd_ed25519_hip_pipe_t * pipe, fd_ed25519_hip_slot_t * slot,
                                 unsigned long txn_cnt, unsigned long payload_bytes );

/* The oldest submitted slot once its results are on the host (wait != 0:
   block until it is), else NULL.  Slots come back in submission order. */
fd_ed25519_hip_slot_t *
fd_ed25519_hip_pipe_poll( fd_ed25519_hip_pipe_t * pipe, int wait );

/* Returns a polled slot to the free ring. */
void
fd_ed25519_hip_pipe_release( fd_ed25519_hip_pipe_t * pipe, fd_ed25519_hip_slot_t * slot );

unsigned
fd_ed25519_hip_pipe_in_flight( fd_ed25519_hip_pipe_t const * pipe );

/* 0, or the sticky error of a batch that failed on the GPU
   (FD_ED25519_HIP_ERR_HIP - hipError_t): poll then returns NULL for that
   batch and every later one, and the pipe must be deleted. */
int
fd_ed25519_hip_pipe_error( fd_ed25519_hip_pipe_t const * pipe );

/* Device memory the pipe holds: its slots' engines (lane tables sized to
   the batch, work arrays, the full-length table) and staging mirrors; the
   base tables shared by the process are fd_ed25519_hip_shared_device_bytes. */
unsigned long
fd_ed25519_hip_pipe_device_bytes( fd_ed25519_hip_pipe_t const * pipe );

/* Batches of at most max_sigs signatures (a tile at a low load: one or two
   transactions each; default 4, 0: none) take each signature's scalars --
   k = SHA-512(R||A||M) mod L, S < L, the half-size pair -- from the
   submitting thread while the GPU decompresses A and R, are read by the
   kernels from the staging block in place, write their codes straight into
   the page-locked output, and have their transactions' codes combined on
   the host at poll: two kernel launches instead of five.  Process-wide;
   raw (GPU-parse) and zero-copy batches keep the device path. */
void
fd_ed25519_hip_pipe_set_host_scalars( unsigned long max_sigs );

/* ... and batches of at most `max_sigs` signatures also decompress A and R
   on the submitting thread, so that one launch (the group equation) is
   left (0: never; default 4; at most 4 and at most the host scalars'
   bound). */
void
fd_ed25519_hip_pipe_set_host_decode( unsigned long max_sigs );

/* ... and those batches split over 4 or 8 waves
   (fd_ed25519_hip_dropin_set_split_waves's forms) or dsm16's two (2, the
   default: the extra host work sits on the tile's own thread, where it
   costs more than the shorter chain saves). */
void
fd_ed25519_hip_pipe_set_split_waves( int waves );

/* ---- txn -------------------------------------------------------------- */

/* The fields of fd_txn_t (src/ballet/txn/fd_txn.h) the verify tile reads. */
typedef struct {
  unsigned char  transaction_version;   /* 0xFF legacy, 0x00 v0 */
  unsigned char  signature_cnt;
  unsigned short signature_off;
  unsigned short message_off;
  unsigned char  readonly_signed_cnt;
  unsigned char  readonly_unsigned_cnt;
  unsigned short acct_addr_cnt;
  unsigned short acct_addr_off;
  unsigned short recent_blockhash_off;
  unsigned short instr_cnt;
  unsigned char  addr_table_lookup_cnt;
  unsigned char  addr_table_adtl_writable_cnt;
  unsigned char  addr_table_adtl_cnt;
} fd_ed25519_hip_txn_t;

#define FD_ED25519_HIP_TXN_MTU (1232UL)
#define FD_ED25519_HIP_TXN_MAX_SZ (852UL)                 /* FD_TXN_MAX_SZ, src/ballet/txn/fd_txn.h */
/* the verify tile's output frag: payload, pad, fd_txn_t, payload_sz
   (FD_TPU_DCACHE_MTU, src/disco/fd_disco_base.h:41) */
#define FD_ED25519_HIP_TPU_DCACHE_MTU (FD_ED25519_HIP_TXN_MTU + FD_ED25519_HIP_TXN_MAX_SZ + 2UL)
/* fd_txn_footprint: 20-byte header, 10 bytes per instruction, 8 per
   address table lookup */
#define FD_ED25519_HIP_TXN_FOOTPRINT( instr_cnt, lut_cnt ) (20UL + 10UL*(instr_cnt) + 8UL*(lut_cnt))

/* Accepts exactly the payloads fd_txn_parse(payload, sz, out, NULL)
   accepts (fd_txn_parse_core with allow_zero_signatures=0 and no trailing
   bytes), returning 1 and the fields, else 0. */
int
fd_ed25519_hip_txn_parse( unsigned char const * payload, unsigned long payload_sz, fd_ed25519_hip_txn_t * out );

/* fd_txn_parse itself: writes the reference's fd_txn_t (src/ballet/txn/
   fd_txn.h: header, instr[], address table lookups) byte for byte into
   out_txn (FD_ED25519_HIP_TXN_MAX_SZ bytes) and returns its footprint,
   or 0 if the payload is rejected. */
unsigned long
fd_ed25519_hip_txn_parse_full( unsigned char const * payload, unsigned long payload_sz, void * out_txn );

/* after_frag's transformation of a frag (src/app/fdctl/run/tiles/
   fd_verify.c:102-133): out (FD_ED25519_HIP_TPU_DCACHE_MTU bytes) receives
   the payload, a zero pad byte to 2-byte alignment, the fd_txn_t and the
   payload size as a little-endian u16; returns that frag's size (new_sz),
   or 0 if fd_txn_parse rejects the payload (after_frag's filter). */
unsigned long
fd_ed25519_hip_txn_frag( unsigned char const * payload, unsigned long payload_sz, unsigned char * out );

/* tcache: the verify tile's HA dedup cache of the last `depth` tags
   (map_cnt a power of two >= depth+2; the tile uses 16 / 64). */
typedef struct fd_ed25519_hip_tcache fd_ed25519_hip_tcache_t;

fd_ed25519_hip_tcache_t *
fd_ed25519_hip_tcache_new( unsigned long depth, unsigned long map_cnt );

void
fd_ed25519_hip_tcache_delete( fd_ed25519_hip_tcache_t * tc );

/* 1 if tag is present (FD_TCACHE_QUERY) */
int
fd_ed25519_hip_tcache_query( fd_ed25519_hip_tcache_t const * tc, unsigned long tag );

/* FD_TCACHE_INSERT: 1 if tag was already present (nothing changes), else
   inserts it, evicting the oldest of depth tags, and returns 0 */
int
fd_ed25519_hip_tcache_insert( fd_ed25519_hip_tcache_t * tc, unsigned long tag );

/* ---- vtile ------------------------------------------------------------ */

/* Verdicts of fd_txn_verify (src/app/fdctl/run/tiles/fd_verify.h:9-11),
   plus the filters after_frag applies before it. */
#define FD_ED25519_HIP_TXN_VERIFY_SUCCESS (0)
#define FD_ED25519_HIP_TXN_VERIFY_FAILED  (-1)
#define FD_ED25519_HIP_TXN_VERIFY_DEDUP   (-2)
#define FD_ED25519_HIP_TXN_PARSE_FAILED   (-3)  /* after_frag: fd_txn_parse failed -> filtered */

typedef struct fd_ed25519_hip_vtile fd_ed25519_hip_vtile_t;

/* A verify tile's batched core on `device`: batches of up to batch_sigs
   signatures (at least 16, the most a transaction stages: smaller values
   are raised to 16; 0 = 4096), slot_cnt in flight, tcache of tcache_depth / tcache_map_cnt
   (the reference: 16 / 64, fd_verify.h:6-7).  flags: the engine flags
   (FD_ED25519_HIP_FLAG_CODES_PORTABLE) and FD_ED25519_HIP_VTILE_GPU_PARSE:
   payloads go to the device as they are and fd_txn_parse runs there
   (fd_ed25519_hip_pipe_submit_txns); the verdicts are the same. */
#define FD_ED25519_HIP_VTILE_GPU_PARSE (2)

fd_ed25519_hip_vtile_t *
fd_ed25519_hip_vtile_new( int device, unsigned slot_cnt, unsigned long batch_sigs, unsigned long tcache_depth,
                          unsigned long tcache_map_cnt, int flags );

void
fd_ed25519_hip_vtile_delete( fd_ed25519_hip_vtile_t * vt );

/* after_frag for one transaction payload: parse and stage it (copying the
   payload into the open batch).  `cookie` comes back with its verdict.
   Returns 1 if staged, 0 if it was answered immediately (parse failure:
   the verdict is queued for the next vtile_poll in order), or the vtile's
   sticky error (negative, see vtile_error; nothing staged).  May submit the
   open batch when it is full; blocks only if every slot is in flight. */
int
fd_ed25519_hip_vtile_frag( fd_ed25519_hip_vtile_t * vt, unsigned char const * payload, unsigned long payload_sz,
                           unsigned long cookie );

/* Submits the open batch if it holds any transaction and a slot is free
   (wait != 0: waits for one).  Returns 1 if a batch was submitted. */
int
fd_ed25519_hip_vtile_flush( fd_ed25519_hip_vtile_t * vt, int wait );

/* Completed verdicts, in frag order: up to max entries of (cookie,
   verdict, dedup tag = first 8 signature bytes).  wait != 0 blocks for
   the oldest batch in flight.  Returns the number written. */
unsigned long
fd_ed25519_hip_vtile_poll( fd_ed25519_hip_vtile_t * vt, int wait, unsigned long max, unsigned long * cookie,
                           signed char * verdict, unsigned long * tag );

/* The same, with the frags the tile publishes: for each verdict also
   frag_off[k] / frag_sz[k], the frag after_frag publishes for a SUCCESS
   transaction (fd_ed25519_hip_txn_frag's layout: payload, pad, fd_txn_t,
   payload_sz; publish sig = tag) copied into frag_buf at frag_off[k]
   (64-byte aligned, like the reference's compact dcache chunks), and
   frag_sz[k] = 0 for filtered transactions.  Stops early, before a frag
   that would not fit in frag_buf_sz bytes. */
unsigned long
fd_ed25519_hip_vtile_poll_frags( fd_ed25519_hip_vtile_t * vt, int wait, unsigned long max, unsigned long * cookie,
                                 signed char * verdict, unsigned long * tag, unsigned long * frag_off,
                                 unsigned long * frag_sz, unsigned char * frag_buf, unsigned long frag_buf_sz );

/* Transactions staged or in flight whose verdicts have not been polled. */
unsigned long
fd_ed25519_hip_vtile_pending( fd_ed25519_hip_vtile_t const * vt );

/* 0, or the vtile's sticky failure: a batch failed on the GPU or could not
   be launched (FD_ED25519_HIP_ERR_HIP - hipError_t, or an engine status),
   or a host allocation failed (FD_ED25519_HIP_ERR_NOMEM).  The library never
   aborts the process for these: the transactions in flight have no
   verdicts, vtile_frag refuses new ones, and the caller stops (the verify
   service marks its links failed, fd_ed25519_hip_vservice_run). */
int
fd_ed25519_hip_vtile_error( fd_ed25519_hip_vtile_t const * vt );

/* Device memory the vtile holds (its pipe's, above). */
unsigned long
fd_ed25519_hip_vtile_device_bytes( fd_ed25519_hip_vtile_t const * vt );

/* ---- ring + latency mode ------------------------------------------- */

/* Latency mode: a producer thread publishes the txn
   payloads into a tango-style mcache/dcache ring at a fixed offered rate
   (txns/s; 0 = as fast as possible) with a publish timestamp; the vtile
   thread pulls frags, stages them, submits a batch once it holds
   batch_sigs signatures or the ring is drained and a slot is free, and
   timestamps each verdict when the batch completes.  lat_s[i] is txn i's
   publish -> verdict latency in seconds; verdict[i] its verdict.  flags as
   for fd_ed25519_hip_vtile_new. */
typedef struct {
  double        offered_txn_per_s;
  double        achieved_txn_per_s;
  double        achieved_sig_per_s;
  double        seconds;
  unsigned long txn_cnt;
  unsigned long sig_cnt;
  unsigned long batches;
  unsigned long ring_overruns;     /* frags the consumer lost (must be 0) */
} fd_ed25519_hip_latency_result_t;

int
fd_ed25519_hip_latency_run( int device, unsigned slot_cnt, unsigned long batch_sigs,
                            unsigned char const * payloads, unsigned long const * payload_off,
                            unsigned int const * payload_sz, unsigned long txn_cnt, double offered_txn_per_s,
                            unsigned long ring_depth, int flags, double * lat_s, signed char * verdict,
                            fd_ed25519_hip_latency_result_t * res );

/* Pins fd_ed25519_hip_latency_run's producer thread to producer_cpu and
   its tile (the calling thread, for the run; its affinity restored after)
   to tile_cpu, as fdctl pins each tile to a core of its own; -1 leaves a
   thread unpinned (the default).  Both on one CPU is refused
   (FD_ED25519_HIP_ERR_INVAL).  Threads that float can land on the two SMT
   siblings of one core, or share a core with other work, and the tile's
   per-frag rate then varies run to run. */
int
fd_ed25519_hip_latency_set_cpus( int producer_cpu, int tile_cpu );

/* Several verify tiles on one GPU (the reference runs
   verify_tile_count of them, src/app/fdctl/config/default.toml:535, frag
   seq going to tile seq % count, src/app/fdctl/run/tiles/fd_verify.c:46):
   tile_cnt threads, each with its own ring, producer, tcache and pipe
   (slot_cnt batches in flight), transaction i to tile i % tile_cnt, all at
   the offered rate in total.  lat_s / verdict are by transaction index;
   res sums the tiles (seconds: the longest tile). */
int
fd_ed25519_hip_latency_run_tiles( int device, unsigned tile_cnt, unsigned slot_cnt, unsigned long batch_sigs,
                                  unsigned char const * payloads, unsigned long const * payload_off,
                                  unsigned int const * payload_sz, unsigned long txn_cnt, double offered_txn_per_s,
                                  unsigned long ring_depth, int flags, double * lat_s, signed char * verdict,
                                  fd_ed25519_hip_latency_result_t * res );

/* ---- shlink + verify service (GPU process outside the sandbox) -------- */

/* A single-producer single-consumer tango-style link in a POSIX shm object
   `name` (e.g. "/fd_verify_in"): an mcache of depth (power of 2)
   fd_frag_meta_t-shaped lines and a dcache of 64-byte chunks for payloads
   of up to FD_ED25519_HIP_SHLINK_MTU bytes, with credit-based flow control.
   create makes the object, join maps an existing one; each process keeps
   its own cursor, so one handle per side.  After the mapping, publish /
   consume are memory operations only (they may run under seccomp strict
   mode).

   create fails (NULL, errno EEXIST) if a live process's link of that name
   exists; a link left behind by a creator that has exited (a killed
   service) is removed and made anew.  join fails with errno ENOENT (no
   such link), EPROTO (a link of another frag protocol or layout: the two
   sides were built from different revisions of this header) or EINVAL
   (bad geometry). */
typedef struct fd_ed25519_hip_shlink fd_ed25519_hip_shlink_t;

/* The verdict frag protocol and link layout a link speaks, recorded in its
   header by create and checked by join (1-4: earlier layouts without the
   word; 5: trailer-only SUCCESS verdicts, below, and the creator's pid;
   6: the creator holds a flock on the object for its lifetime, and a link
   whose lock can be taken is reclaimable -- a protocol-5 link only when
   its creator pid is gone, since its creator held no lock). */
#define FD_ED25519_HIP_SHLINK_PROTO (6UL)

/* the largest frag either direction carries (a verdict frag is smaller
   than this: 1 verdict byte + at most FD_ED25519_HIP_TXN_MAX_SZ + 2) */
#define FD_ED25519_HIP_SHLINK_MTU (1UL + FD_ED25519_HIP_TPU_DCACHE_MTU)

/* The verdict frag protocol (service -> tile).  One frag per transaction,
   in the tile's frag order, sig = the tile's cookie: byte 0 the verdict
   (FD_ED25519_HIP_TXN_VERIFY_* / FD_ED25519_HIP_TXN_PARSE_FAILED), then,
   for SUCCESS only, the published frag's trailer: the bytes that follow
   the payload and its 2-byte alignment pad in the frag after_frag
   publishes (src/app/fdctl/run/tiles/fd_verify.c:102-133), i.e. the
   fd_txn_t and the u16 payload_sz.  The tile still holds the payload (it
   wrote it into the txn link), so only the trailer crosses back and the
   tile assembles payload | pad | trailer in its out dcache.
   fd_ed25519_hip_frag_assemble does that into dst (room for
   FD_ED25519_HIP_TPU_DCACHE_MTU bytes) and returns the frag's size, or 0
   if the trailer does not belong to a payload of payload_sz bytes (too
   short or too long, or its payload_sz differs): a protocol error.  The
   pad byte is written as 0. */
static inline unsigned long
fd_ed25519_hip_frag_assemble( unsigned char * dst, unsigned char const * payload, unsigned long payload_sz,
                              unsigned char const * trailer, unsigned long trailer_sz ) {
  if( payload_sz>FD_ED25519_HIP_TXN_MTU || trailer_sz<2UL || trailer_sz>FD_ED25519_HIP_TXN_MAX_SZ + 2UL ) return 0UL;
  if( ( (unsigned long)trailer[ trailer_sz-2UL ] | ( (unsigned long)trailer[ trailer_sz-1UL ]<<8 ) )!=payload_sz ) return 0UL;
  unsigned long toff = ( payload_sz + 1UL ) & ~1UL;
  __builtin_memcpy( dst, payload, payload_sz );
  if( toff>payload_sz ) dst[ payload_sz ] = 0;
  __builtin_memcpy( dst + toff, trailer, trailer_sz );
  return toff + trailer_sz;
}

fd_ed25519_hip_shlink_t *
fd_ed25519_hip_shlink_create( char const * name, unsigned long depth );

fd_ed25519_hip_shlink_t *
fd_ed25519_hip_shlink_join( char const * name );

/* Unmaps (and with unlink != 0 removes the name). */
void
fd_ed25519_hip_shlink_leave( fd_ed25519_hip_shlink_t * link, int unlink );

unsigned long
fd_ed25519_hip_shlink_depth( fd_ed25519_hip_shlink_t const * link );

/* The link's dcache (payload rooms, *sz bytes) and its whole mapping (for
   page-locking it with the GPU: the zero-copy service DMAs payloads from
   the rooms, FD_ED25519_HIP_VSERVICE_ZERO_COPY). */
unsigned char const *
fd_ed25519_hip_shlink_dcache( fd_ed25519_hip_shlink_t const * link, unsigned long * sz );

void *
fd_ed25519_hip_shlink_mapping( fd_ed25519_hip_shlink_t const * link, unsigned long * sz );

/* Producer: publishes one frag (payload of sz bytes, sig, ctl).  Returns
   0, 1 if the consumer has not returned a credit yet (retry), or an
   error status. */
int
fd_ed25519_hip_shlink_publish( fd_ed25519_hip_shlink_t * link, unsigned char const * payload, unsigned long sz,
                               unsigned long sig, unsigned int ctl );

/* Consumer: takes the next frag into payload (FD_ED25519_HIP_SHLINK_MTU
   bytes of room).  Returns 0, 1 if none is published yet, -1 if the
   producer overran the consumer. */
int
fd_ed25519_hip_shlink_consume( fd_ed25519_hip_shlink_t * link, unsigned char * payload, unsigned long * sz,
                               unsigned long * sig, unsigned int * ctl );

/* Zero-copy producer: prepare returns the room (MTU bytes, inside the
   dcache) for the next frag's payload if the consumer has returned a
   credit for it, else NULL; the caller writes the payload there and
   commit publishes it (FD_ED25519_HIP_ERR_INVAL without a successful
   prepare, or sz above the MTU).  prepare may be repeated before commit
   (it returns the same room). */
unsigned char *
fd_ed25519_hip_shlink_prepare( fd_ed25519_hip_shlink_t * link );

int
fd_ed25519_hip_shlink_commit( fd_ed25519_hip_shlink_t * link, unsigned long sz, unsigned long sig, unsigned int ctl );

/* Zero-copy consumer: peek returns the next frag's payload in place
   (bounds checked against this side's geometry) and its size, sig and ctl,
   or NULL with *err = 1 (nothing published yet) or -1 (overrun / a line
   pointing outside the dcache); advance then returns its credit and
   reports 0 if the bytes were intact while they were read, -1 if the
   producer overran them meanwhile. */
unsigned char const *
fd_ed25519_hip_shlink_peek( fd_ed25519_hip_shlink_t * link, unsigned long * sz, unsigned long * sig,
                            unsigned int * ctl, int * err );

int
fd_ed25519_hip_shlink_advance( fd_ed25519_hip_shlink_t * link );

/* Liveness (fd_cnc's heartbeat and signal, src/tango/cnc/fd_cnc.h:63-65,
   129-130): the producer of a link ticks its heartbeat word (any value that
   changes while it is alive; 0 means not started), either side may mark
   the link failed with a nonzero code (FD_ED25519_HIP_ERR_* or
   FD_ED25519_HIP_SHLINK_FAIL_*), status returns it (0: healthy).  A
   consumer that sees the heartbeat unchanged for longer than its bound, or
   a nonzero status, stops waiting on the link. */
#define FD_ED25519_HIP_SHLINK_FAIL_PROTOCOL (-100)   /* the peer broke the frag protocol */
#define FD_ED25519_HIP_SHLINK_FAIL_STOPPED  (-101)   /* the service was told to stop      */
#define FD_ED25519_HIP_SHLINK_FAIL_TILE_GONE (-102)  /* the tile's heartbeat stopped: the service ended the link */

void
fd_ed25519_hip_shlink_heartbeat( fd_ed25519_hip_shlink_t * link, unsigned long now );

unsigned long
fd_ed25519_hip_shlink_heartbeat_query( fd_ed25519_hip_shlink_t const * link );

void
fd_ed25519_hip_shlink_fail( fd_ed25519_hip_shlink_t * link, int code );

int
fd_ed25519_hip_shlink_status( fd_ed25519_hip_shlink_t const * link );

/* A consumer's view of its producer's heartbeat (zero-initialised):
   watch returns 1 while the producer has never ticked (0), 0 while its
   heartbeat changes, -1 once it has not changed for more than stale_ns
   (<= 0: never stale); now_ns any monotonic clock. */
typedef struct {
  unsigned long last;
  long          t_ns;
  int           seen;
} fd_ed25519_hip_shlink_watch_t;

int
fd_ed25519_hip_shlink_watch( fd_ed25519_hip_shlink_watch_t * w, fd_ed25519_hip_shlink_t const * link, long now_ns,
                             long stale_ns );

/* ctl bit of the last frag of a stream, both directions */
#define FD_ED25519_HIP_SHLINK_CTL_EOS (1U)

typedef struct {
  unsigned long txn_cnt;
  unsigned long batches;
  double        seconds;        /* from the first frag consumed to the end of the stream */
  unsigned long device_bytes;   /* the link pair's own device memory (its vtile's) */
  unsigned long shared_device_bytes;   /* the process's base tables on the device, shared by every pair */
  int           end_code;       /* how the link pair ended: 0 (EOS) or its failure code */
  unsigned      leaked_on_hang; /* 1: the pair ended under a GPU hang (FD_ED25519_HIP_ERR_TIMEOUT) and left its
                                   engines and device memory unfreed -- freeing them waits on the hung device --
                                   for the process exit to reclaim (the service exits at once) */
} fd_ed25519_hip_vservice_stats_t;

/* The GPU side of a sandboxed verify tile: consumes transaction payload
   frags from `in` (sig = the tile's cookie), runs them through a vtile
   (slot_cnt, batch_sigs, flags as for fd_ed25519_hip_vtile_new) and
   publishes one frag per transaction to `out` in frag order: sig = cookie,
   the verdict (FD_ED25519_HIP_TXN_VERIFY_* / FD_ED25519_HIP_TXN_PARSE_FAILED)
   as byte 0, and for SUCCESS the trailer of the frag the verify tile
   publishes to dedup after it (fd_ed25519_hip_frag_assemble above; the
   frag as fd_ed25519_hip_txn_frag lays it out).  A frag with ctl EOS ends the stream:
   the service answers everything before it, publishes an EOS frag and
   returns.  A batch is submitted when full, or when `in` is drained and a
   slot is free. */
int
fd_ed25519_hip_vservice_run( int device, unsigned slot_cnt, unsigned long batch_sigs, int flags,
                             fd_ed25519_hip_shlink_t * in, fd_ed25519_hip_shlink_t * out,
                             fd_ed25519_hip_vservice_stats_t * stats );

/* One service process for several verify tiles of a GPU (the reference
   runs verify_tile_count tiles, src/app/fdctl/config/default.toml:535):
   link_cnt (1..FD_ED25519_HIP_VSERVICE_LINK_MAX) link pairs, each served as
   by vservice_run with its own vtile (engines,
   streams, tcache), all sharing the device's base tables -- one copy of the
   4 GiB per GPU instead of one per tile process; a thread per pair, or
   several pairs per thread (fd_ed25519_hip_vservice_serve's
   links_per_thread).  Returns when every link
   pair has ended (EOS), or on the first failure, which stops the others
   (their links marked FD_ED25519_HIP_SHLINK_FAIL_STOPPED); stats[k] per
   pair (optional).

   Liveness and failure policy, both entry points: the service ticks the
   heartbeat of each `out` link on every idle pass of its loop and every
   16th busy one (microseconds apart either way); on a GPU or
   launch failure, an allocation failure, a tile that overran its own link
   or marked a link failed, it stops publishing, marks both links failed
   with the code and returns it (it never aborts the process). */
#define FD_ED25519_HIP_VSERVICE_LINK_MAX (64U)

/* Service flag (with the vtile flags): zero-copy GPU parse.  The service
   does not copy payloads out of the txn link: its dcache is page-locked
   with the GPU, the service reads only each frag's signature count and
   dedup tag in place, and each batch's payloads are DMA'd from the link's
   rooms as they lie (one or two spans) to the device, which parses them
   (FD_ED25519_HIP_VTILE_GPU_PARSE's parser) and returns the fd_txn_t
   trailers.  Safe because the tile reuses a room only after its frag is
   answered (integration/fd_verify_hip.c), and the device parser takes any
   bytes: a tile that rewrites its own payloads can only change its own
   verdicts.  Same verdicts and frags as the other modes. */
#define FD_ED25519_HIP_VSERVICE_ZERO_COPY (4)

int
fd_ed25519_hip_vservice_run_links( int device, unsigned slot_cnt, unsigned long batch_sigs, int flags,
                                   fd_ed25519_hip_shlink_t * const * in, fd_ed25519_hip_shlink_t * const * out,
                                   unsigned link_cnt, fd_ed25519_hip_vservice_stats_t * stats );

/* run_links with a lifecycle (fd_topo_run.c's supervision of tiles,
   src/disco/topo/fd_topo_run.c:50-100, and fd_cnc's heartbeat,
   src/tango/cnc/fd_cnc.h:63-65,129-130, on the service's side):

     stop          while *stop is nonzero every link ends (marked
                   FD_ED25519_HIP_SHLINK_FAIL_STOPPED): the caller's signal
                   handler or parent watch sets it (NULL: never)
     tile_stale_ns a link whose tile has ticked its txn-link heartbeat and
                   then not changed it for this long is ended (both links
                   marked FD_ED25519_HIP_SHLINK_FAIL_TILE_GONE, its engines
                   and device memory freed) while the other links are served
                   on (0: FD_ED25519_HIP_VSERVICE_TILE_STALE_NS, < 0: never)
     gpu_hang_ns   a batch that has not completed after this long is a hung
                   GPU: every link fails with FD_ED25519_HIP_ERR_TIMEOUT
                   (0: FD_ED25519_HIP_VSERVICE_GPU_HANG_NS)

   Failure domains: what a tile causes (its links marked failed by the
   tile, an overrun, a stale heartbeat) ends that tile's link pair only; a
   GPU, launch or allocation failure ends every link (the device is not
   trusted for anyone).  While the service waits for the GPU it keeps
   ticking its heartbeats and watching its links, so a slow GPU is never
   mistaken for a dead service.  Returns FD_ED25519_HIP_OK when every link
   ended with its tile's EOS, the device-wide failure's code if there was
   one, else FD_ED25519_HIP_SHLINK_FAIL_TILE_GONE (or _PROTOCOL / _STOPPED:
   the first link-local end); stats[k].end_code says how each link ended. */
#define FD_ED25519_HIP_VSERVICE_TILE_STALE_NS (5L*1000L*1000L*1000L)
#define FD_ED25519_HIP_VSERVICE_GPU_HANG_NS   (30L*1000L*1000L*1000L)

typedef struct {
  int volatile const * stop;
  long                 tile_stale_ns;
  long                 gpu_hang_ns;
  /* called once, from the calling thread, when every link pair is ready
     to serve (engines and base tables built, every kernel launched once
     on a dummy batch): the service announces itself there, so no tile's
     first frags wait for the device's set-up (NULL: none) */
  void              (* ready)( void * ctx );
  void *               ready_ctx;
  /* link pairs one service thread serves (0: 1, a thread per tile).  A
     thread passes over its pairs in turn and never waits for the GPU on
     one pair while another has frags, so several tiles per thread cost
     the service fewer cores where its threads would otherwise spin idle
     (ABI 6) */
  unsigned             links_per_thread;
  /* CPUs for the service threads (fdctl pins each tile to a core): thread
     t runs on link_cpus[t % link_cpu_cnt] (0 entries: the process's
     affinity, as before).  A CPU outside the process's affinity fails the
     thread's pairs with FD_ED25519_HIP_ERR_INVAL.  (ABI 7) */
  int const *          link_cpus;
  unsigned             link_cpu_cnt;
} fd_ed25519_hip_vservice_opts_t;

int
fd_ed25519_hip_vservice_serve( int device, unsigned slot_cnt, unsigned long batch_sigs, int flags,
                               fd_ed25519_hip_shlink_t * const * in, fd_ed25519_hip_shlink_t * const * out,
                               unsigned link_cnt, fd_ed25519_hip_vservice_stats_t * stats,
                               fd_ed25519_hip_vservice_opts_t const * opts );

/* ---- pool ------------------------------------------------------------- */

/* Verifies n signatures (host SoA as in fd_ed25519_hip_verify_host) on
   device_cnt GPUs: batches of batch_sigs signatures are dealt round-robin,
   batch b to device devices[b % device_cnt] (the reference's
   seq % verify_tile_count, src/app/fdctl/run/tiles/fd_verify.c:46); one
   host thread per device, on the CPUs of that GPU's NUMA node, keeps
   slot_cnt (1..8) batches in flight and writes the codes into out.

   When msgs, msg_off, msg_sz, sigs and pubs are page-locked
   (fd_ed25519_hip_host_register or hipHostMalloc), a batch is DMA'd from
   them as it is (its messages as the one byte range they span) and the
   host never copies a byte; when out is page-locked too, the codes are
   DMA'd into it.  Otherwise batches are packed into pinned staging first.
   Returns 0 or an engine status; *seconds (optional) is the wall time of
   the whole call. */
int
fd_ed25519_hip_pool_verify( int const * devices, unsigned device_cnt, unsigned slot_cnt, unsigned long batch_sigs,
                            unsigned long n, unsigned char const * msgs, unsigned long const * msg_off,
                            unsigned int const * msg_sz, unsigned char const * sigs, unsigned char const * pubs,
                            signed char * out, double * seconds );

typedef struct {
  unsigned long direct_batches;   /* DMA'd from the caller's page-locked arrays */
  unsigned long staged_batches;   /* packed into pinned staging first          */
  unsigned long h2d_bytes;        /* bytes moved host -> device                */
} fd_ed25519_hip_pool_stats_t;

/* The same pool as a long-lived object (a deployment's feeder: engines,
   streams and device buffers are set up once): slot_cnt (1..8) batches of
   batch_sigs signatures in flight per device, msg_cap bytes of messages
   per batch (the span a batch's messages cover when DMA'd in place, or
   their bytes when packed).  pool_run verifies one SoA set as
   fd_ed25519_hip_pool_verify does; stats (optional) reports the
   transfers. */
typedef struct fd_ed25519_hip_pool fd_ed25519_hip_pool_t;

fd_ed25519_hip_pool_t *
fd_ed25519_hip_pool_new( int const * devices, unsigned device_cnt, unsigned slot_cnt, unsigned long batch_sigs,
                         unsigned long msg_cap );

int
fd_ed25519_hip_pool_run( fd_ed25519_hip_pool_t * pool, unsigned long n, unsigned char const * msgs,
                         unsigned long const * msg_off, unsigned int const * msg_sz, unsigned char const * sigs,
                         unsigned char const * pubs, signed char * out, double * seconds,
                         fd_ed25519_hip_pool_stats_t * stats );

void
fd_ed25519_hip_pool_delete( fd_ed25519_hip_pool_t * pool );

/* Page-locks [ptr, ptr+sz) of the caller's memory for every device
   (hipHostRegister, portable + mapped) so the pool and the pipe DMA
   directly from it; unregister with the same ptr. */
int
fd_ed25519_hip_host_register( void * ptr, unsigned long sz );

int
fd_ed25519_hip_host_unregister( void * ptr );

/* Page-locked host memory from the HIP driver (hipHostMalloc, portable),
   for host-fed streams that need no registration; NULL on failure. */
void *
fd_ed25519_hip_host_alloc( unsigned long sz );

void
fd_ed25519_hip_host_free( void * ptr );

/* Host -> device copy bandwidth of `device` in GB/s: reps copies of bytes
   from a pinned buffer (the PCIe bound of a host-fed batch). */
double
fd_ed25519_hip_h2d_gbps( int device, unsigned long bytes, unsigned reps );

#ifdef __cplusplus
}
#endif
#endif
