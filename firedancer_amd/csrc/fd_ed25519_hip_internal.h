/* fd_ed25519_hip_internal.h -- contract between the plain-C host runtime
   (host/fd_ed25519_hip_engine.c) and the HIP kernel shim
   (fd_ed25519_kernels.hip).  Only plain pointers and sizes cross it. */
#ifndef FD_ED25519_HIP_INTERNAL_H
#define FD_ED25519_HIP_INTERNAL_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Base-point table: [0..128] B in affine precomputed form (y+x, y-x, 2dxy),
   36 int32 per entry (30 used), kept in LDS by the verify kernel. */
#define FD_ED25519_BTAB_ENTRIES   129
#define FD_ED25519_BTAB_STRIDE    36
#define FD_ED25519_BTAB_INTS      (FD_ED25519_BTAB_ENTRIES * FD_ED25519_BTAB_STRIDE)

/* Wide base-point tables of the verify kernels, 128-byte entries
   (y+x, y-x, 2dxy, pad), read from HBM / L2 / MALL with each entry loaded
   ahead of its use:
     btab16   [0..2^15]B, signed radix-2^16 digits of S (full-length form), 4.2 MB
     btab_lo  [0..2^24)B, unsigned radix-2^24 digits of s_lo (half-size form), 2 GiB
     btab_hi  [0..2^24)[2^144]B, digits of s_hi, 2 GiB
   The two wide tables are shared by all engines of a device (4 GiB of the
   288 GB: s' = s_lo + 2^144 s_hi costs 6 + 5 mixed additions, against
   7 + 7 at radix 2^20 with 2 x 128 MB; the random 128-byte reads, 11 per
   signature, are prefetched a window ahead). */
#define FD_ED25519_BTAB16_ENTRIES ((1 << 15) + 1)
#define FD_ED25519_BTAB16_STRIDE  32
#define FD_ED25519_BTABW_BITS     24
#define FD_ED25519_BTABW_ENTRIES  (1 << FD_ED25519_BTABW_BITS)
#define FD_ED25519_BTABW_SHIFT    144   /* s_lo: 6 digits (bits 0..143), s_hi: 5 digits (109 bits) */
/* The compact tables (FD_ED25519_HIP_FLAG_COMPACT_TABLES): the same two
   tables at radix 2^16, [0..2^16)B and [0..2^16)[2^144]B, 8 MiB each,
   9 + 7 mixed additions per signature -- for processes that verify little
   (the drop-in's engines) and should not hold 4 GiB. */
#define FD_ED25519_BTABC_BITS     16
#define FD_ED25519_BTABC_ENTRIES  (1 << FD_ED25519_BTABC_BITS)

/* Per-lane tables [1..8](-A) and [1..8](-+R) in cached form, in HBM: 2 x 8
   entries x 40 int32 per lane, laid out [wave][lane][entry][quad] (int4
   granules, lane stride 160 int4): a lookup
   reads 160 contiguous bytes of the lane's own table, so every fetched line
   is fully used (the [entry][quad][lane] layout fetched ~2.4x the table
   bytes from HBM because lanes pick different entries).  A zero digit reads
   one identity entry shared by all lanes (L2-resident) instead of a
   per-lane copy: 1/9 less table written, dsm -1.2%
   (profiles/r2_ab_atab_ident.txt).  The full-length form keeps [0..8] at
   tabA, 9 entries, extending into the (then unused) tabR half. */
#define FD_ED25519_ATAB_STRIDE 8UL
#define FD_ED25519_ATAB_BYTES_PER_WAVE (2UL * FD_ED25519_ATAB_STRIDE * 10UL * 64UL * 16UL)  /* -A and -+R tables */

#define FD_ED25519_VERIFY_BLOCK 256
#define FD_ED25519_QUAD_LANE_BYTES 864UL   /* dsm4 lane tables: 2 x 9 entries x 48 B */
/* Occupancy targets (waves per SIMD) of the phase kernels; each caps the
   kernel's register allocation (512 / waves VGPRs). */
#ifndef FD_ED25519_DSM_WAVES_PER_SIMD
#define FD_ED25519_DSM_WAVES_PER_SIMD 2
#endif
#ifndef FD_ED25519_HASH_WAVES_PER_SIMD
#define FD_ED25519_HASH_WAVES_PER_SIMD 2  /* measured: 2 (200 VGPR, no spill) beats 3 (spills) */
#endif
#ifndef FD_ED25519_SCALAR_WAVES_PER_SIMD
#define FD_ED25519_SCALAR_WAVES_PER_SIMD 4
#endif
#ifndef FD_ED25519_DECODE_WAVES_PER_SIMD
#define FD_ED25519_DECODE_WAVES_PER_SIMD 4  /* 128 VGPR: spills 292 B/lane outside the squaring loops; 1.87 -> 1.85 ms (profiles/r2_ab_decode_waves.txt) */
#endif
#define FD_ED25519_SORT_BUCKETS 64

/* Work arrays handed between the phase kernels, per signature of a chunk
   (SoA, [field][cap] so every access is one coalesced dword per lane):
     k        [8][cap]   u32  k = SHA-512(R||A||M) mod L
     sflag    [cap]      u8   S < L
     pflag    [2][cap]   u8   A, R: bit0 decode failure, bit1 small order
     pts      [2][20][cap] i32 A, R: x (10 limbs), y (10 limbs), radix 2^25.5
     hs       [19][cap]  u32  half-size scalars: c, |d|, s_lo (5 words), s_hi (4)
     hflag    [cap]      u8   bit0 d < 0, bit1 no verified half-size pair (full-length form)
     perm     [cap]      u32  hash order (length-sorted)
     fix_list [cap]      u32  signatures for the full-length form (scalar -> dsm)
   FD_ED25519_WORK_BYTES_PER_SIG bytes per signature of capacity. */
#define FD_ED25519_WORK_BYTES_PER_SIG (8UL * 4UL + 1UL + 2UL + 2UL * 20UL * 4UL + 19UL * 4UL + 1UL + 4UL + 4UL)

typedef struct {
  /* inputs (signature i = base + j for chunk-local j in [0,n)) */
  uint8_t const *  msgs;     /* message bytes (any alignment)                 */
  uint64_t const * msg_off;  /* [N] byte offset of message i in msgs          */
  uint32_t const * msg_sz;   /* [N] message size                              */
  uint8_t const *  sigs;     /* [N][64] R||S, 16-byte aligned                  */
  uint8_t const *  pubs;     /* [N][32] A, 16-byte aligned                     */
  uint8_t const *  digests;  /* [N][64] SHA-512(R||A||M) computed by the caller,
                                16-byte aligned (msgs unused); NULL: hashed here */
  int8_t *         out;      /* [N] FD_ED25519_SUCCESS / ERR_* codes           */
  uint64_t         base;
  uint64_t         n;        /* chunk size, <= cap                             */
  /* work arrays */
  uint32_t *       k;
  uint8_t *        sflag;
  uint8_t *        pflag;
  int32_t *        pts;
  uint32_t *       hs;
  uint8_t *        hflag;
  uint32_t *       fix_list;
  uint32_t *       fix_cnt;  /* 1 word: entries of fix_list                   */
  uint32_t *       work_ctr; /* 1 word: dsm items handed out (fix_cnt + 1)      */
  uint32_t *       perm;     /* [cap] hash order (length-sorted), NULL: identity */
  uint32_t *       hist;     /* [2*SORT_BUCKETS] counting-sort scratch          */
  uint64_t         cap;
  int32_t const *  btab;     /* device base-point table (FD_ED25519_BTAB_INTS) */
  int32_t const *  btab16;   /* [0..2^15]B,          [FD_ED25519_BTAB16_ENTRIES][32] */
  int32_t const *  btab_lo;  /* [0..2^24)B,          [FD_ED25519_BTABW_ENTRIES][32] */
  int32_t const *  btab_hi;  /* [0..2^24)[2^144]B,   same layout                     */
  void *           atab;     /* device scratch, waves * ATAB_BYTES_PER_WAVE    */
  int              codes_portable; /* 0: AVX-512 backend codes, 1: portable  */
  int              half_dbits;     /* longest |d| of the half-size form (fd25519_half.h) */
  int              small;          /* small chunk: fused prep kernel, no sort, dsm4 (1: a
                                      quad of lanes per signature), dsm8 (2: two quads)
                                      or dsm16 (3: two waves, prep16 before it); the
                                      full-length items by a scan of hflag (1, 2)    */
  int              full_in_prep;   /* small == 3 and atab holds a lane per signature:
                                      prep16's hash waves run the full-length items
                                      (atab slot j) and no scan follows dsm16          */
  int              bw_bits;        /* radix of btab_lo / btab_hi: FD_ED25519_BTABW_BITS or
                                      FD_ED25519_BTABC_BITS (compact)                 */
  int              hs_host;        /* small == 3 only: the scalars came from the calling
                                      thread (host/fd_ed25519_hip_hsrec.cc): prep16 runs
                                      its decode blocks only, and dsm16's sflag / hs /
                                      hflag point at the caller's page-locked block (the
                                      same [field][cap] layout); never a full-length item */
  int32_t const *  btabq[8];       /* dsm16s<S>: compact [0..2^16)[2^(CB q)]B, q < S (shared per device) */
  uint32_t const * go;             /* dsm16 with host scalars and points: NULL, or a
                                      page-locked word the kernel waits on before it
                                      reads anything else -- the launch goes ahead of
                                      the host's work, so its dispatch overlaps it.
                                      FD_ED25519_GO_RUN: proceed; FD_ED25519_GO_CANCEL:
                                      exit writing nothing (the launch takes another
                                      path); unset after FD_ED25519_GO_SPIN_MAX polls
                                      (>= 0.1 s): exit writing nothing, which the host
                                      reports as a launch that ended without a code */
  /* A/B build only (-DFD_ED25519_AB_LDS_BASE=1): the base
     tables staged in LDS instead, [0..256)B and [0..256)[2^136]B, 32 KiB
     each, radix-2^8 unsigned digits of s' split at 2^136 */
  int32_t const *  btab8_lo;
  int32_t const *  btab8_hi;
} fd_ed25519_verify_params_t;

/* host-decoded launches (params.pts in host memory): every host array's
   stride (params.cap), the launch's signatures being at most this many */
#define FD_ED25519_HS_STRIDE   8UL
#define FD_ED25519_GO_RUN      1U
#define FD_ED25519_GO_CANCEL   2U
#define FD_ED25519_GO_SPIN_MAX 200000U

/* 0: prep16 leaves the full-length items to a flag scan after dsm16 (A/B
   build) */
#ifndef FD_ED25519_FULL_IN_PREP
#define FD_ED25519_FULL_IN_PREP 1
#endif

#define FD_ED25519_BTAB8_SHIFT 136   /* A/B LDS tables: s' = lo (17 digits) + 2^136 hi (15 digits) */

/* All launchers are asynchronous on `stream` (a hipStream_t) and return a
   hipError_t value (0 on success). */
int fd_ed25519_hip_launch_gen_btab( int32_t * d_btab, void * stream );
int fd_ed25519_hip_launch_gen_btab16( int32_t * d_btab16, int base_doublings, void * stream );
/* [0..256)[2^base_doublings]B, 128-byte entries (the LDS A/B's tables) */
int fd_ed25519_hip_launch_gen_btab8( int32_t * d_tab, int base_doublings, void * stream );
/* [0..2^bits)[2^base_doublings]B into d_tab (bits FD_ED25519_BTABW_BITS or
   FD_ED25519_BTABC_BITS); d_scratch holds 2^bits*10 + 40 int32 */
int fd_ed25519_hip_launch_gen_btabw( int32_t * d_tab, int base_doublings, int bits, int32_t * d_scratch, void * stream );
/* counts into *d_bad the entries e < entries-1 of a 32-int-stride base
   table with entry e+1 != entry e + entry 1 (and entry 0 not the identity) */
int fd_ed25519_hip_launch_check_btabw( int32_t const * d_tab, int entries, uint32_t * d_bad, void * stream );
/* Enqueues hash, decode and dsm for one chunk; `grid` caps the persistent
   dsm grid (its atab scratch must hold grid*VERIFY_BLOCK/64 waves). */
int fd_ed25519_hip_launch_verify( fd_ed25519_verify_params_t const * p, uint32_t grid, void * stream );

/* The same, one phase at a time (so the host can bracket each with events). */
#define FD_ED25519_PHASE_HASH   0
#define FD_ED25519_PHASE_SCALAR 1
#define FD_ED25519_PHASE_DECODE 2
#define FD_ED25519_PHASE_DSM    3
#define FD_ED25519_PHASE_CNT    4
int fd_ed25519_hip_launch_phase( fd_ed25519_verify_params_t const * p, int phase, uint32_t grid, void * stream );
/* dsm16s (fd_ed25519_kernels.hip): the four- or eight-wave form for
   launches whose points and split scalars all came from the host */
int fd_ed25519_hip_launch_dsm16s( fd_ed25519_verify_params_t const * p, int waves, void * stream );

/* Host scalars (host/fd_ed25519_hip_hsrec.cc, host/fd_ed25519_hip_engine.c):
   a launch of a few signatures whose k, S < L and half-size pair the
   calling thread computes while the device decompresses A and R.
   hsrec: 1 and the 32-word record (k[8], hs[19], sflag, hflag), or 0 when
   k has no half-size pair within dbits (the launch then takes the device's
   own path).  hs_decode: prep16's decode blocks; hs_dsm: dsm16 with
   sflag [cap], hflag [cap], hs [19][cap] read in place (cap = the engine's
   max_chunk).  The engine's dsm16 form must take n (n <= its r16 bound).
   Host decompressions (host/fd_ed25519_hip_hsdec.cc) for the fewest
   signatures: hsdec_n writes each point's 20 limbs and flags as the decode
   blocks would, and hs_dsm then reads pts [2][20][cap] and pflag [2][cap]
   in place too (pts NULL: the decode blocks' arrays on the device).  go:
   NULL, or the page-locked word dsm16 waits on (params.go): the caller
   launches first, writes the block, then stores FD_ED25519_GO_RUN (or
   FD_ED25519_GO_CANCEL) -- on every path, or the kernel spins to its bound. */
#ifdef __cplusplus
extern "C" {
#endif
struct fd_ed25519_hip_engine;
int fd_ed25519_hip_private_hsrec( unsigned char const sig[ 64 ], unsigned char const pub[ 32 ],
                                  unsigned char const * msg, unsigned long msg_sz, int dbits, uint32_t rec[ 32 ] );
int fd_ed25519_hip_private_half_dbits( struct fd_ed25519_hip_engine const * e );
int fd_ed25519_hip_private_codes_portable( struct fd_ed25519_hip_engine const * e );
int fd_ed25519_hip_private_hs_decode( struct fd_ed25519_hip_engine * e, unsigned long n, unsigned char const * sigs,
                                      unsigned char const * pubs, signed char * out, void * stream );
int fd_ed25519_hip_private_hs_dsm( struct fd_ed25519_hip_engine * e, unsigned long n, unsigned char const * sigs,
                                   unsigned char const * pubs, signed char * out, unsigned char const * sflag,
                                   unsigned char const * hflag, unsigned int const * hs, int const * pts,
                                   unsigned char const * pflag, unsigned int const * go, void * stream );
void fd_ed25519_hip_private_hsdec_n( unsigned char const * const * enc, unsigned long n, int avx_rule, int32_t * pt,
                                     unsigned char * flags );
/* The split forms (dsm16s<S>, S = 4 or 8 waves) for host-decoded
   launches: hssplit turns one signature's record into the split scalars
   and s' chunks (hq: 24 rows of stride cap, layout at the function), and
   hsdec3_n also returns each point doubled step, 2 step, .. nx step times
   (S = 4: nx 1, step 66; S = 8: nx 3, step 33) in extended coordinates
   (40 limbs) for pts rows 2i + side of 40 limbs (row 0 A, 1 R -- affine,
   the first 20 -- 2 A_1, 3 R_1, ..); hs_dsms launches dsm16s<waves> on them
   once want_dsms has made (or found) the engine's tables for that form. */
void fd_ed25519_hip_private_hssplit( uint32_t const rec[ 32 ], int waves, uint32_t * hq, unsigned long cap,
                                     unsigned long j );
void fd_ed25519_hip_private_hsdec3_n( unsigned char const * const * enc, unsigned long n, int avx_rule, int32_t * pt,
                                      int32_t * ptx, int nx, int step, unsigned char * flags );
int fd_ed25519_hip_private_hs_dsms( struct fd_ed25519_hip_engine * e, int waves, unsigned long n,
                                    unsigned char const * sigs, unsigned char const * pubs, signed char * out,
                                    unsigned char const * sflag, unsigned char const * hflag, unsigned int const * hq,
                                    int const * pts, unsigned char const * pflag, unsigned int const * go,
                                    void * stream );
int fd_ed25519_hip_private_want_dsms( struct fd_ed25519_hip_engine * e, int waves );
#ifdef __cplusplus
}
#endif
int fd_ed25519_hip_verify_occupancy( int * blocks_per_cu );
/* lane-table bytes per dsm wave as compiled into the kernels (the host
   sizes the atab scratch from this, never from its own copy of the macro) */
unsigned long fd_ed25519_hip_atab_bytes_per_wave( void );

/* Per-transaction combine with fd_ed25519_verify_batch_single_msg's
   priority (src/ballet/ed25519/fd_ed25519_user.c:231-309): the first
   phase-1 error (ERR_SIG/ERR_PUBKEY) in signature order wins, else ERR_MSG
   if any equation fails, else SUCCESS; cnt==0 or cnt>16 -> ERR_SIG. */
int fd_ed25519_hip_launch_txn_combine( int8_t const * d_sig_codes, uint32_t const * d_txn_first,
                                       uint32_t const * d_txn_cnt, int8_t * d_txn_out, uint64_t ntxn,
                                       void * stream );

/* diagnostic: fd_half_scalars on the device, 12 words out per k (see
   fd_ed25519_hip_diag_half_scalars) */
int fd_ed25519_hip_launch_diag_half( uint32_t const * d_k, uint32_t * d_out, uint64_t n, int dbits, void * stream );

/* ---- raw transactions (fd_ed25519_txn.hip) ---- */

/* per-transaction code for a payload fd_txn_parse rejects (never an
   ed25519 code) */
#define FD_ED25519_TXN_PARSE_FAILED_CODE (-4)

typedef struct {
  uint8_t const *  payloads;   /* payload bytes, readable 16 B past each   */
  uint64_t const * pay_off;    /* [ntxn]                                   */
  uint32_t const * pay_sz;     /* [ntxn]                                   */
  uint32_t const * txn_first;  /* [ntxn] first signature slot               */
  uint32_t const * txn_cnt;    /* [ntxn] payload byte 0 (slots: 1..16 -> cnt, else 0) */
  uint64_t         ntxn;
  uint8_t *        sigs;       /* [slots][64] out, 16-B aligned            */
  uint8_t *        pubs;       /* [slots][32] out                          */
  uint64_t *       msg_off;    /* [slots] out: into payloads                */
  uint32_t *       msg_sz;     /* [slots] out                               */
  uint8_t *        parse_ok;   /* [ntxn] out                                */
  uint8_t *        trailer;    /* [ntxn][64] out (optional): fd_txn_t bytes  */
} fd_ed25519_txn_stage_params_t;

int fd_ed25519_hip_launch_txn_stage( fd_ed25519_txn_stage_params_t const * p, void * stream );

/* H2D without the copy engines: one launch in which the device reads up to
   FD_ED25519_PULL_SPAN_MAX spans of page-locked host memory (device-visible
   addresses, 16-byte aligned) and writes them to device memory (16-byte
   aligned), exactly n bytes each.  A launch is asynchronous; a
   hipMemcpyAsync H2D issued by a thread whose stream shares the device with
   busy compute streams can hold the calling thread for the copy's
   duration (measured in the verify service: tools/ubench/h2d_call_probe.hip,
   DESIGN.md 3c). */
#define FD_ED25519_PULL_SPAN_MAX 8
typedef struct {
  uint8_t const * src[ FD_ED25519_PULL_SPAN_MAX ];
  uint8_t *       dst[ FD_ED25519_PULL_SPAN_MAX ];
  uint64_t        n  [ FD_ED25519_PULL_SPAN_MAX ];
  uint32_t        cnt;
} fd_ed25519_pull_params_t;

int fd_ed25519_hip_launch_pull( fd_ed25519_pull_params_t const * p, void * stream );

/* fault-injection build only (-DFD_ED25519_HALF_FAULT=1): one wave that
   sleeps for ms milliseconds (at most 10 s) of the device's wall clock */
int fd_ed25519_hip_launch_stall( unsigned ms, void * stream );
int fd_ed25519_hip_launch_txn_finish( int8_t const * d_sig_codes, uint32_t const * d_txn_first,
                                      uint32_t const * d_txn_cnt, uint8_t const * d_parse_ok, int8_t * d_txn_out,
                                      uint64_t ntxn, void * stream );

/* ---- generator (fd_ed25519_gen.hip) ---- */

typedef struct {
  uint8_t const *  msgs;
  uint64_t const * msg_off;
  uint32_t const * msg_sz;
  uint8_t const *  privs;      /* [n][32], 16-byte aligned; NULL: derive from (seed, index_base+i) */
  uint8_t *        sigs;       /* [n][64] out */
  uint8_t *        pubs;       /* [n][32] out */
  uint64_t         n;
  uint64_t         seed;
  uint64_t         index_base;
  int32_t const *  btab;
} fd_ed25519_sign_params_t;

typedef struct {
  uint8_t *        msgs;
  uint64_t const * msg_off;
  uint32_t const * msg_sz;
  uint8_t *        sigs;
  uint8_t *        pubs;
  uint64_t         n;
  uint64_t         seed;
  uint64_t         index_base;
  uint32_t         ppm;        /* corrupted fraction, parts per million */
  int8_t *         expect;     /* [n] out (optional): reference AVX-512 code */
  uint8_t *        cls;        /* [n] out (optional): class 0..7 */
} fd_ed25519_corrupt_params_t;

int fd_ed25519_hip_launch_fill_random( uint8_t * d, uint64_t nbytes, uint64_t seed, void * stream );
int fd_ed25519_hip_launch_sign( fd_ed25519_sign_params_t const * p, void * stream );
int fd_ed25519_hip_launch_corrupt( fd_ed25519_corrupt_params_t const * p, void * stream );

#ifdef __cplusplus
}
#endif
#endif
