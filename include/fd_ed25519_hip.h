#ifndef HEADER_fd_ed25519_hip_h
#define HEADER_fd_ed25519_hip_h

/* libfd_ed25519_hip -- MI355X (gfx950) ed25519 signature verification for
   Firedancer, as a C-ABI shared library.

   Part 1 is a drop-in for the reference's verify API
   (tigarcia/firedancer src/ballet/ed25519/fd_ed25519.h:96-138): the same
   symbols, prototypes, argument meaning and return codes, so a binary that
   links libfd_ed25519_hip ahead of libfd_ballet.a resolves them here.

   Part 2 is the batch engine the drop-ins sit on.  A synchronous per-call
   API cannot feed a GPU; callers that batch (the verify
   tile, bench.py) use the SoA entry points below, either with host buffers
   (staged through pinned memory) or with device-resident buffers (enqueued
   asynchronously on a HIP stream).

   Verdicts and error codes are bit-identical to fd_ed25519_verify of the
   reference's AVX-512 backend (the production build); an engine created with
   FD_ED25519_HIP_FLAG_CODES_PORTABLE reproduces the portable backend's codes
   instead (they differ only in the code returned for an undecodable public
   key). */

#ifdef __cplusplus
extern "C" {
#endif

/* Reference codes, src/ballet/ed25519/fd_ed25519.h:11-14 */
#define FD_ED25519_SUCCESS    ( 0)
#define FD_ED25519_ERR_SIG    (-1)
#define FD_ED25519_ERR_PUBKEY (-2)
#define FD_ED25519_ERR_MSG    (-3)

/* The reference's sha512 calculator (src/ballet/sha512/fd_sha512.h:15-16,
   56-77: 256 bytes, 128-byte aligned) is opaque here: the drop-ins accept
   the caller's handle and do not touch it (the hash runs on the GPU). */
#ifndef FD_SHA512_ALIGN
typedef struct fd_sha512_private fd_sha512_t;
#endif

/* ---- Part 1: drop-in verify API ------------------------------------- */

/* Replaces fd_ed25519_verify (src/ballet/ed25519/fd_ed25519.h:96-101,
   implementation src/ballet/ed25519/fd_ed25519_user.c:134-229).  msg may be
   NULL if msg_sz==0.  Returns FD_ED25519_SUCCESS or FD_ED25519_ERR_*.
   Synchronous; runs on the process-wide default engine (device from
   $FD_ED25519_HIP_DEVICE, default 0; codes from $FD_ED25519_HIP_CODES =
   "avx512" (default) | "portable").  A failed launch is retried once on a
   re-created engine; a device that fails again is lost, and the process's
   policy decides (fd_ed25519_hip_dropin_set_on_lost below: abort with a
   message, the default, or fail closed); this path never falls back to
   the CPU.  Any
   msg_sz is accepted, as by the reference (4 GiB and more: the message is
   hashed on the host, fd_ed25519_hip_dropin_set_host_hash_min). */
int
fd_ed25519_verify( unsigned char const   msg[],
                   unsigned long         msg_sz,
                   unsigned char const   sig[ 64 ],
                   unsigned char const   public_key[ 32 ],
                   fd_sha512_t *         sha );

/* Replaces fd_ed25519_verify_batch_single_msg (src/ballet/ed25519/fd_ed25519.h:124-130,
   implementation src/ballet/ed25519/fd_ed25519_user.c:231-309), with the
   reference's parameter spellings (array bounds included, so the two
   headers compile together: tests/test_abi.py): batch_sz
   signatures (64 B each, contiguous) by batch_sz public keys (32 B each,
   contiguous) over one message.  batch_sz==0 or >16 -> FD_ED25519_ERR_SIG.
   Otherwise the first phase-1 error (bad S, undecodable or small-order key
   or R) in signature order wins, then FD_ED25519_ERR_MSG if any equation
   fails. */
int
fd_ed25519_verify_batch_single_msg( unsigned char const   msg[],
                                    unsigned long const   msg_sz,
                                    unsigned char const   signatures[ 64 ], /* 64 * batch_sz */
                                    unsigned char const   pubkeys[ 32 ],    /* 32 * batch_sz */
                                    fd_sha512_t *         shas[ 1 ],        /* batch_sz      */
                                    unsigned char const   batch_sz );

/* Replaces fd_ed25519_strerror (src/ballet/ed25519/fd_ed25519_user.c:311-321). */
char const *
fd_ed25519_strerror( int err );

/* The drop-ins above serve any number of calling threads: concurrent calls
   are coalesced into shared launches on the process's four drop-in engines
   (compact tables, 16K-signature chunks).  dropin_stats reports the
   launches made and the calls they carried; dropin_device_bytes the device
   memory the drop-ins hold (their engines plus the compact tables; it
   creates them if no call has yet). */
void
fd_ed25519_hip_dropin_stats( unsigned long * launches, unsigned long * requests );

/* A message of 4 GiB or more does not fit the device path's 32-bit message
   sizes: the drop-ins hash it (R_j || A_j || M per signature) on the
   calling thread with the library's SHA-512 and verify the rest on the GPU
   from the digests (fd_ed25519_hip_verify_digests_dev); no message is ever
   truncated or refused.  Test hook: messages of at least `bytes` bytes take
   that path (0 restores 4 GiB). */
void
fd_ed25519_hip_dropin_set_host_hash_min( unsigned long bytes );

/* A direct drop-in launch (one caller alone, at most a few signatures)
   computes each signature's scalars -- k = SHA-512(R||A||M) mod L, S < L,
   the half-size pair -- on the calling thread while the GPU decompresses A
   and R, instead of in one GPU lane before them (the latency path's
   longest chain).  Test hook: launches of at most `max_sigs` signatures
   take that path (0: never; the default is 4). */
void
fd_ed25519_hip_dropin_set_host_scalars( unsigned long max_sigs );

/* Test hook: the bound on |d| the calling thread's search uses (0 restores
   the engine's, 151).  A signature whose k has no pair within it sends the
   launch down the device path from its digest, whose own search runs at
   the engine's bound -- the fallback a test reaches with k that have no
   pair at 131 bits. */
void
fd_ed25519_hip_dropin_set_host_scalars_dbits( int dbits );

/* The fewest-signature host-scalar launches also decompress A and R on the
   calling thread (a few us a point on one core, against ~44 us for the
   GPU's decode blocks, whose one 16-lane row per point is a chain of ~265
   dependent field operations) and launch only the group equation, which
   reads the points in place.  Test hook: launches of at most `max_sigs`
   signatures take that path (0: never; the default is 2; at most the host
   scalars' bound). */
void
fd_ed25519_hip_dropin_set_host_decode( unsigned long max_sigs );

/* Host-decoded drop-in launches run the group equation split over
   `waves` waves (4 or 8; 2: dsm16's two) -- the calling thread also
   doubles A and R every 66 (4) or 33 (8) bits and splits the half-size
   scalars there and s' into 72- or 32-bit chunks, so each wave's chain is
   ~17 or ~9 windows instead of 33 -- from compact base tables at offsets
   2^(72 q) or 2^(32 q) (32 or 64 MiB per device, the default's made with
   the drop-in engines).  Test / A-B hook, process-wide (default 4: eight measured
   slower). */
void
fd_ed25519_hip_dropin_set_split_waves( int waves );

unsigned long
fd_ed25519_hip_dropin_device_bytes( void );

/* Failure policy of the drop-ins.  The reference's verify cannot fail: it
   returns only the codes above (src/ballet/ed25519/fd_ed25519_user.c:
   134-229), and its tile stops the process only on input it cannot trust
   (FD_LOG_ERR, src/app/fdctl/run/tiles/fd_verify.c:67-68).  Here the GPU
   can fail.  When a drop-in launch fails (a kernel launch, a copy, the
   completion wait) -- or a drop-in engine cannot be created -- the failing
   engine is deleted, created anew and the same launch run once more: a
   transient failure costs the callers of that launch one retry and shows
   only in fd_ed25519_hip_dropin_status's recovery count.  If the retry
   fails as well, the device is lost to the drop-ins and the policy set
   here decides:

     FD_ED25519_HIP_DROPIN_ON_LOST_ABORT (the default): a message on stderr
       naming the failure, then abort() -- fail-stop, as a tile that cannot
       do its work stops the validator;
     FD_ED25519_HIP_DROPIN_ON_LOST_REJECT: fail closed -- the calls of the
       failed launch, the calls queued behind it and every later call return
       FD_ED25519_ERR_SIG without touching the device, so no signature is
       ever accepted unverified; fd_ed25519_hip_dropin_status reports the
       loss, and the caller alerts, restarts the process or calls
       fd_ed25519_hip_dropin_reset.

   There is no CPU fallback in either case: the library has one verify
   implementation, the GPU's.

   set_on_lost returns the previous policy (FD_ED25519_HIP_ERR_INVAL for an
   unknown one, nothing changed).  dropin_status returns 0 while the
   drop-ins are usable, else the error code that lost the device (an
   FD_ED25519_HIP_ERR_* code; fd_ed25519_hip_last_error in the thread that
   lost it has the message), and the count of launches that succeeded on a
   re-created engine in *recoveries (optional).  dropin_reset waits for the
   launches in flight, deletes and re-creates every drop-in engine and, if
   that succeeds, makes the drop-ins usable again: 0, or the creation's
   error code (still lost).

   What a retry or a reset can recover: a failure that leaves the HIP
   context usable (an allocation or a launch refused, a queue that could
   not be made, an error the library raised itself).  A device fault inside
   a kernel (an illegal address, a memory violation, a hardware exception)
   is sticky on ROCm: the process's context stays failed, so the retry
   fails too, the device is lost, and dropin_reset keeps returning the
   context's error code.  Only a process restart recovers from that, and a
   caller that sees dropin_reset fail should restart the process (the
   ABORT policy's default does exactly that, by ending it). */
#define FD_ED25519_HIP_DROPIN_ON_LOST_ABORT  (0)
#define FD_ED25519_HIP_DROPIN_ON_LOST_REJECT (1)

int
fd_ed25519_hip_dropin_set_on_lost( int policy );

int
fd_ed25519_hip_dropin_status( unsigned long * recoveries );

int
fd_ed25519_hip_dropin_reset( void );

/* ---- Part 2: batch engine -------------------------------------------- */

typedef struct fd_ed25519_hip_engine fd_ed25519_hip_engine_t;

/* ABI version of the two headers (include/fd_ed25519_hip.h and
   include/fd_ed25519_hip_tile.h): bumped whenever a flag's meaning, a
   struct layout or a prototype changes (3: round 3 -- engine flags 64..256,
   vservice stats' device bytes, shlink liveness words; 4: a SUCCESS verdict
   frag carries the published frag's trailer only, the tile keeps the
   payload; 5: shlink protocol word and creator, vservice lifecycle and
   end codes; 6: vservice links_per_thread; 7: vservice link_cpus; 8:
   vservice stats' leaked_on_hang, the drop-ins' device-lost state, the
   dsm16 form and its flag; 9: shlink protocol 6, flock-owned links).  A
   consumer checks
   the library it loaded against the header it was built with:
   fd_ed25519_hip_abi_check( FD_ED25519_HIP_ABI_VERSION,
   sizeof(fd_ed25519_hip_slot_t), sizeof(fd_ed25519_hip_info_t),
   sizeof(fd_ed25519_hip_vservice_stats_t) ) returns 0 when they agree,
   FD_ED25519_HIP_ERR_INVAL (with fd_ed25519_hip_last_error) when not. */
#define FD_ED25519_HIP_ABI_VERSION (10U)

unsigned
fd_ed25519_hip_abi_version( void );

int
fd_ed25519_hip_abi_check( unsigned version, unsigned long slot_sz, unsigned long info_sz,
                          unsigned long vservice_stats_sz );

/* Engine API status codes (not verdicts). */
#define FD_ED25519_HIP_OK          (0)
#define FD_ED25519_HIP_ERR_INVAL   (-22)   /* bad argument / misaligned device buffer */
#define FD_ED25519_HIP_ERR_NOMEM   (-12)   /* host or device allocation failed        */
#define FD_ED25519_HIP_ERR_TIMEOUT (-110)  /* the GPU did not complete a batch in time  */
#define FD_ED25519_HIP_ERR_HIP     (-1000) /* HIP runtime error: -1000 - hipError_t    */

#define FD_ED25519_HIP_FLAG_CODES_PORTABLE (1)  /* portable-backend error codes */
/* Half-size scalars with |d| < 2^131 only (the strict form): signatures
   whose k has no such pair take the full-length multiplication.  Default:
   |d| up to 2^151 with a few more windows, the full-length form only for
   ~1e-6 of random k.  Same verdicts either way; for tests and A/B. */
#define FD_ED25519_HIP_FLAG_HALF_STRICT    (2)
/* The dsm phase runs one signature per lane (throughput) or, for chunks of
   at most FD_ED25519_HIP_QUAD_MAX_DEFAULT signatures,
   one per quad of lanes (latency: each group operation in one
   multiplication's time), and for at most FD_ED25519_HIP_OCT_MAX_DEFAULT
   one per two quads (the two halves of the multi-scalar sum in parallel)
   (fd_ed25519_hip_engine_set_forms moves both thresholds).  These force
   one form (tests / A-B). */
#define FD_ED25519_HIP_FLAG_DSM_QUAD       (4)
#define FD_ED25519_HIP_FLAG_DSM_WIDE       (8)
#define FD_ED25519_HIP_FLAG_DSM_OCT        (16)
/* The engine keeps to its one stream (no side stream for the decode
   overlap): for engines whose batches overlap one another already (the
   pool's and the pipe's slots), where extra streams only crowd the
   device's few hardware queues. */
#define FD_ED25519_HIP_FLAG_ONE_STREAM     (32)
/* A large chunk's phases in sequence on the call's stream (no decode side
   stream, below), and a call of several chunks on one set of work arrays
   (no second lane, fd_ed25519_hip_verify_dev): same verdicts; A/B and
   tests.  FLAG_ONE_STREAM implies both.  The library reads no environment
   variable for its launch forms. */
#define FD_ED25519_HIP_FLAG_NO_OVERLAP     (64)
#define FD_ED25519_HIP_FLAG_NO_PIPELINE    (128)
/* The half-size form's two base tables at radix 2^16 ([0..2^16)B and
   [0..2^16)[2^144]B, 8 MiB each, shared by the process's compact engines
   of a device) instead of radix 2^24 (2 GiB each): 9 + 7 instead of 6 + 5
   mixed additions per signature, same verdicts.  For processes that verify
   little and should not hold 4 GiB of device memory; the drop-ins use it. */
#define FD_ED25519_HIP_FLAG_COMPACT_TABLES (256)
/* dsm16 at every chunk size (tests / A-B): the field arithmetic itself
   spread over 16 lanes, two waves per signature (fd25519_r16.h), the
   default for chunks of at most FD_ED25519_HIP_R16_MAX_DEFAULT signatures,
   where a batch's latency is one signature's chain of group operations
   (fd_ed25519_hip_engine_set_r16_max moves the threshold).  FLAG_DSM_QUAD,
   _OCT and _WIDE exclude it. */
#define FD_ED25519_HIP_FLAG_DSM_R16        (512)
#define FD_ED25519_HIP_QUAD_MAX_DEFAULT    (32768UL)
#define FD_ED25519_HIP_OCT_MAX_DEFAULT     (8192UL)
#define FD_ED25519_HIP_R16_MAX_DEFAULT     (512UL)
/* Overlap: a large chunk's decode phase (A and R need neither the hash nor
   the scalars) runs on a side stream beside its hash and scalar phases, dsm
   after both: +1% at 1M, measured.  Per-phase timing runs the phases in
   sequence.  (FD_ED25519_HIP_FLAG_NO_OVERLAP turns it off.) */
#define FD_ED25519_HIP_OVERLAP_DEFAULT     (1)

/* Creates an engine on HIP device `device`.  max_chunk is the number of
   signatures processed per kernel sequence (0 = default 1<<20); larger
   batches are processed in chunks.  Returns NULL on failure (reason via
   fd_ed25519_hip_last_error()). */
fd_ed25519_hip_engine_t *
fd_ed25519_hip_engine_new( int device, unsigned long max_chunk, int flags );

void
fd_ed25519_hip_engine_delete( fd_ed25519_hip_engine_t * engine );

/* Device memory this process shares between all its engines on `device`:
   the half-size form's two base tables while any engine holds them (2 x 2
   GiB; 2 x 8 MiB for FD_ED25519_HIP_FLAG_COMPACT_TABLES engines), else 0.  An engine's own memory is fd_ed25519_hip_engine_info's
   device_bytes. */
unsigned long
fd_ed25519_hip_shared_device_bytes( int device );

/* Moves the chunk sizes at which the engine switches from one quad of lanes
   per signature (chunks of at most quad_max) and two quads (at most
   oct_max) to one lane per signature.  FD_ED25519_HIP_ERR_INVAL if
   oct_max > quad_max or quad_max exceeds what the engine's lane tables
   hold.  For tests and tuning; the defaults are the measured crossovers. */
int
fd_ed25519_hip_engine_set_forms( fd_ed25519_hip_engine_t * engine, unsigned long quad_max, unsigned long oct_max );

/* Chunks of at most n signatures run dsm16 (0: never); n <= the oct
   threshold.  FD_ED25519_HIP_ERR_INVAL otherwise. */
int
fd_ed25519_hip_engine_set_r16_max( fd_ed25519_hip_engine_t * engine, unsigned long n );

typedef struct {
  int           device;
  int           cu_cnt;
  int           dsm_blocks_per_cu;
  unsigned      dsm_grid;
  unsigned long max_chunk;
  unsigned long device_bytes;   /* device memory held by the engine */
  int           flags;
  char          arch[ 64 ];
  int           pci_domain;     /* the device's PCI address (tells ranks' devices apart) */
  int           pci_bus;
  int           pci_device;
} fd_ed25519_hip_info_t;

int
fd_ed25519_hip_engine_info( fd_ed25519_hip_engine_t const * engine, fd_ed25519_hip_info_t * info );

/* The engine's HIP stream (a hipStream_t).  Engine streams are drawn from
   one per-device set of GPU_MAX_HW_QUEUES streams that the library creates
   once and every engine of the process shares (at most 32; 4 by default),
   so this stream may also carry other engines' work: waiting on it
   (hipStreamSynchronize, fd_ed25519_hip_engine_sync, events recorded on
   it) waits for theirs too.  Order your own work with events recorded
   right after it, not with whole-stream waits, when other engines run. */
void *
fd_ed25519_hip_engine_stream( fd_ed25519_hip_engine_t * engine );

/* Device-resident batch: every pointer is a device pointer.  Signature i
   is sigs[64 i .. 64 i + 64) = R || S over message msgs[msg_off[i] ..
   msg_off[i] + msg_sz[i]) by public key pubs[32 i .. 32 i + 32); out[i]
   receives its code.  sigs and pubs must be 16-byte aligned; messages may
   start at any byte, and the message buffer must stay readable at least 16
   bytes past the end of the last message (the SHA-512 loader reads aligned
   16-byte granules, up to 15 bytes beyond a message's last byte; the same
   holds for fd_ed25519_hip_sign_dev / _gen_dev).  Enqueued on `stream` (NULL = the engine's stream) and
   returns immediately; the engine's work arrays are reused by the next
   call, so calls on one engine must be ordered on one stream.  A call of
   more than max_chunk signatures alternates its chunks between two sets of
   work arrays on two streams (the second set, max_chunk x 280 B plus the
   dsm lane tables, allocated on the first such call), so a chunk's hash,
   scalar and decode phases fill the tail of the previous chunk's dsm; the
   call still completes in order on `stream` (FD_ED25519_HIP_FLAG_NO_PIPELINE
   or FD_ED25519_HIP_FLAG_ONE_STREAM keeps one set, per-phase timing too).
   An engine whose max_chunk exceeds FD_ED25519_HIP_QUAD_MAX_DEFAULT and that
   may pipeline allocates the second set with the first, in engine_new, so
   no call allocates device memory or fails for lack of it; a smaller
   engine allocates it on its first multi-chunk call (one hipMalloc, which
   may synchronise the device once). */
int
fd_ed25519_hip_verify_dev( fd_ed25519_hip_engine_t * engine,
                           unsigned long             n,
                           unsigned char const *     msgs,
                           unsigned long const *     msg_off,
                           unsigned int const *      msg_sz,
                           unsigned char const *     sigs,
                           unsigned char const *     pubs,
                           signed char *             out,
                           void *                    stream );

/* The same verification from the caller's digests: signature i's
   challenge k = SHA-512(R || A || M) mod L is reduced from digests[64 i ..
   64 i + 64) (the SHA-512 of R || A || M, computed by the caller; 16-byte
   aligned device memory), everything else as fd_ed25519_hip_verify_dev.
   For messages the device path's 32-bit sizes cannot carry (the drop-ins
   use it for messages of 4 GiB and more, hashing them on the host). */
int
fd_ed25519_hip_verify_digests_dev( fd_ed25519_hip_engine_t * engine,
                                   unsigned long             n,
                                   unsigned char const *     digests,
                                   unsigned char const *     sigs,
                                   unsigned char const *     pubs,
                                   signed char *             out,
                                   void *                    stream );

/* SHA-512 on the host (FIPS 180-4; the library's own, used for the
   drop-ins' large messages). */
void
fd_ed25519_hip_sha512( void const * data, unsigned long sz, unsigned char out[ 64 ] );

/* Per-transaction combine on the device (fd_ed25519_verify_batch_single_msg
   priority), for transactions whose signatures were verified with
   fd_ed25519_hip_verify_dev: txn t owns signatures [txn_first[t],
   txn_first[t] + txn_cnt[t]). */
int
fd_ed25519_hip_txn_combine_dev( fd_ed25519_hip_engine_t * engine,
                                unsigned long             ntxn,
                                signed char const *       sig_codes,
                                unsigned int const *      txn_first,
                                unsigned int const *      txn_cnt,
                                signed char *             txn_out,
                                void *                    stream );

/* Host-buffer batch, synchronous: messages are packed into pinned staging
   memory (any offsets / aliasing allowed), copied, verified, and the codes
   copied back to out[0..n). */
int
fd_ed25519_hip_verify_host( fd_ed25519_hip_engine_t * engine,
                            unsigned long             n,
                            unsigned char const *     msgs,
                            unsigned long const *     msg_off,
                            unsigned int const *      msg_sz,
                            unsigned char const *     sigs,
                            unsigned char const *     pubs,
                            signed char *             out );

/* Host-buffer transactions (fd_ed25519_verify_batch_single_msg semantics
   for each): txn t has message msgs[txn_msg_off[t] .. + txn_msg_sz[t]) and
   signatures/keys [txn_first[t], txn_first[t] + txn_cnt[t]) of sigs/pubs.
   out_txn[t] receives the transaction's code; out_sig (optional, may be
   NULL) the per-signature codes. */
int
fd_ed25519_hip_verify_txns_host( fd_ed25519_hip_engine_t * engine,
                                 unsigned long             ntxn,
                                 unsigned char const *     msgs,
                                 unsigned long const *     txn_msg_off,
                                 unsigned int const *      txn_msg_sz,
                                 unsigned int const *      txn_first,
                                 unsigned int const *      txn_cnt,
                                 unsigned char const *     sigs,
                                 unsigned char const *     pubs,
                                 signed char *             out_txn,
                                 signed char *             out_sig );

/* ---- Part 3: batched signing and the synthetic workload generator ------ */

/* Batched fd_ed25519_public_from_private + fd_ed25519_sign on the device
   (src/ballet/ed25519/fd_ed25519_user.c:4-132): for each i, pubs[32 i..]
   and sigs[64 i..] receive the public key of privs[32 i..] and its
   signature of msgs[msg_off[i] .. + msg_sz[i]).  Device pointers; privs,
   sigs and pubs 16-byte aligned.  Async on `stream` (NULL = engine). */
int
fd_ed25519_hip_sign_dev( fd_ed25519_hip_engine_t * engine,
                         unsigned long             n,
                         unsigned char const *     msgs,
                         unsigned long const *     msg_off,
                         unsigned int const *      msg_sz,
                         unsigned char const *     privs,
                         unsigned char *           sigs,
                         unsigned char *           pubs,
                         void *                    stream );

/* Deterministic synthetic workload (bench.py): fills
   msgs[0..msg_bytes) with bytes derived from `seed`, derives the private
   key of signature g = index_base + i from (seed, g) and writes its public
   key and signature of message i.  Same (seed, g) -> same bytes on any GPU
   (firedancer_amd/workload.py recomputes them on the host). */
int
fd_ed25519_hip_gen_dev( fd_ed25519_hip_engine_t * engine,
                        unsigned long             n,
                        unsigned long             seed,
                        unsigned long             index_base,
                        unsigned char *           msgs,
                        unsigned long             msg_bytes,
                        unsigned long const *     msg_off,
                        unsigned int const *      msg_sz,
                        unsigned char *           sigs,
                        unsigned char *           pubs,
                        void *                    stream );

/* Corrupts about ppm/10^6 of the signatures in place with the invalid
   classes of SURVEY.md §8(d) C2 (bad S, small-order A/R, undecodable A/R,
   non-canonical A, flipped message bit); expect[i] (optional) receives the
   code the reference's AVX-512 build returns, cls[i] (optional) the class. */
int
fd_ed25519_hip_corrupt_dev( fd_ed25519_hip_engine_t * engine,
                            unsigned long             n,
                            unsigned long             seed,
                            unsigned long             index_base,
                            unsigned int              ppm,
                            unsigned char *           msgs,
                            unsigned long const *     msg_off,
                            unsigned int const *      msg_sz,
                            unsigned char *           sigs,
                            unsigned char *           pubs,
                            signed char *             expect,
                            unsigned char *           cls,
                            void *                    stream );

/* ---- Part 4: measurement and device-memory helpers ------------------ */

/* Phase timing: while enabled, fd_ed25519_hip_verify_dev brackets each of
   its phases (0 hash, 1 scalar, 2 decode, 3 dsm) with HIP events on the stream
   they run on (up to 256 chunk launches); _timing_read waits for them and
   returns the summed milliseconds per phase and the number of chunk
   launches, then resets.  Enabling resets too. */
#define FD_ED25519_HIP_PHASE_CNT (4)

int
fd_ed25519_hip_engine_timing( fd_ed25519_hip_engine_t * engine, int enable );

int
fd_ed25519_hip_engine_timing_read( fd_ed25519_hip_engine_t * engine,
                                   double * phase_ms /* [FD_ED25519_HIP_PHASE_CNT] */, unsigned long * launches );

/* The half-size form's base tables (generated on the device, shared by the
   engines of a device): table 0 holds [e]B, table 1 [e][2^SHIFT]B, for
   0 <= e < 2^BITS, as (y+x, y-x, 2dxy) in ten radix-2^25.5 limbs each.
   check_base_tables counts, per table (bad[2]: the full-length form's
   [0..2^15]B table), the entries e with entry e+1 != entry e + entry 1 (or
   entry 0 not the identity); together with a few
   entries compared against an independent [s]B (base_entry), a zero count
   proves the whole table.  base_entry copies entry `index` of table
   `which` (30 int32) to the host.  An engine with
   FD_ED25519_HIP_FLAG_COMPACT_TABLES has the 2^FD_ED25519_HIP_COMPACT_TABLE_BITS-entry
   pair instead. */
#define FD_ED25519_HIP_BASE_TABLE_BITS  24
#define FD_ED25519_HIP_COMPACT_TABLE_BITS 16
#define FD_ED25519_HIP_BASE_TABLE_SHIFT 144

int
fd_ed25519_hip_engine_check_base_tables( fd_ed25519_hip_engine_t * engine, unsigned long bad[3] );

int
fd_ed25519_hip_engine_base_entry( fd_ed25519_hip_engine_t * engine, int which, unsigned long index, int out[30] );

/* Device memory from the engine's HIP runtime (so callers need not link a
   second runtime).  memcpy is synchronous on the engine's stream. */
#define FD_ED25519_HIP_H2D (0)
#define FD_ED25519_HIP_D2H (1)
#define FD_ED25519_HIP_D2D (2)

void *
fd_ed25519_hip_dev_alloc( fd_ed25519_hip_engine_t * engine, unsigned long bytes );

int
fd_ed25519_hip_dev_free( fd_ed25519_hip_engine_t * engine, void * ptr );

int
fd_ed25519_hip_memcpy( fd_ed25519_hip_engine_t * engine, void * dst, void const * src, unsigned long bytes, int dir );

/* Number of visible HIP devices (0 if none / no driver). */
int
fd_ed25519_hip_device_count( void );

/* Peak shader clock of the engine's device in MHz (hipDeviceProp clockRate). */
int
fd_ed25519_hip_device_clock_mhz( fd_ed25519_hip_engine_t * engine );

/* Waits for all work enqueued on the engine's stream -- which other
   engines of the device may share (fd_ed25519_hip_engine_stream). */
int
fd_ed25519_hip_engine_sync( fd_ed25519_hip_engine_t * engine );

/* Diagnostic: the verify kernels' half-size scalar search
   (csrc/fd25519_half.h) run on the device for n scalars k (8 little-endian
   32-bit words each, k < L), host buffers in and out.  out[12*i]: 1 if a
   pair was found, out[12*i+1]: d < 0, out[12*i+2..6]: c, out[12*i+7..11]:
   |d| (5 words each).  Synchronous.  For tests: the device search must
   agree with the host build of the same header. */
int
fd_ed25519_hip_diag_half_scalars( fd_ed25519_hip_engine_t * engine,
                                  unsigned int const *      k,
                                  unsigned long             n,
                                  unsigned int *            out );

/* Human-readable form of an engine status code / of the last failure. */
char const *
fd_ed25519_hip_strerror( int status );

char const *
fd_ed25519_hip_last_error( void );

#ifdef __cplusplus
}
#endif

#endif /* HEADER_fd_ed25519_hip_h */
