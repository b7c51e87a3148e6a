/* fd_verify_hip_service -- the GPU process behind sandboxed verify tiles.

   The verify tile runs under a write/fsync-only seccomp policy
   (src/app/fdctl/run/tiles/verify.seccomppolicy) and cannot drive a GPU;
   its accelerated form (integration/fd_verify_hip.c) hands transaction
   payloads to this process over two shared-memory links per tile and
   publishes the verdict frags that come back.  One service process serves
   every verify tile of one GPU, so the device's 4 GiB of base tables exist
   once per GPU, not once per tile (fd_ed25519_hip_vservice_run_links).

     fd_verify_hip_service --prefix NAME --tiles K [--gpu G] [--depth D]
                           [--slots S] [--batch B] [--gpu-parse] [--codes portable|avx512]

   creates, for k in [0,K), the links NAME<k>_txn (tile -> service) and
   NAME<k>_vd (service -> tile), each of D lines (default 16384), prints
   "ready K" on stdout once they exist, and serves them until every tile
   has sent its end-of-stream frag (a validator's tiles never do).  Exit
   status: 0 after a clean end; 1 on bad arguments or if a link cannot be
   created (a stale one of the same name exists: a previous service was
   killed; remove /dev/shm/NAME*); 2 when the service failed -- a GPU or
   launch failure, or a tile broke the protocol -- after marking every link
   failed, so each tile stops waiting (its heartbeat check) instead of
   blocking.  The links are removed on every exit path.

   Each link pair runs slot_cnt engines with one stream each: a process
   gets GPU_MAX_HW_QUEUES hardware queues (4 by default), so a service for
   several tiles should be started with that raised to about K x S (at most
   the device's limit), as tools/ and tests/ do. */
#define _GNU_SOURCE
#include "../../../include/fd_ed25519_hip_tile.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static void
usage( char const * argv0 ) {
  fprintf( stderr, "usage: %s --prefix NAME --tiles K [--gpu G] [--depth D] [--slots S] [--batch B] "
                   "[--gpu-parse] [--codes portable|avx512]\n", argv0 );
}

int
main( int argc, char ** argv ) {
  char const *  prefix = NULL;
  unsigned      tiles  = 0U, slots = 3U;
  int           gpu    = 0, flags = 0;
  unsigned long depth  = 16384UL, batch = 4096UL;
  for( int i=1; i<argc; i++ ) {
    char const * a = argv[ i ];
    char const * v = i+1<argc ? argv[ i+1 ] : NULL;
    if(      !strcmp( a, "--prefix" ) && v ) { prefix = v; i++; }
    else if( !strcmp( a, "--tiles"  ) && v ) { tiles = (unsigned)strtoul( v, NULL, 0 ); i++; }
    else if( !strcmp( a, "--gpu"    ) && v ) { gpu = (int)strtol( v, NULL, 0 ); i++; }
    else if( !strcmp( a, "--depth"  ) && v ) { depth = strtoul( v, NULL, 0 ); i++; }
    else if( !strcmp( a, "--slots"  ) && v ) { slots = (unsigned)strtoul( v, NULL, 0 ); i++; }
    else if( !strcmp( a, "--batch"  ) && v ) { batch = strtoul( v, NULL, 0 ); i++; }
    else if( !strcmp( a, "--gpu-parse" ) )   { flags |= FD_ED25519_HIP_VTILE_GPU_PARSE; }
    else if( !strcmp( a, "--codes" ) && v ) {
      if(      !strcmp( v, "portable" ) ) flags |= FD_ED25519_HIP_FLAG_CODES_PORTABLE;
      else if( strcmp( v, "avx512" ) ) { usage( argv[0] ); return 1; }
      i++;
    }
    else { usage( argv[0] ); return 1; }
  }
  if( !prefix || !tiles || tiles>FD_ED25519_HIP_VSERVICE_LINK_MAX || strlen( prefix )>96 ) { usage( argv[0] ); return 1; }

  fd_ed25519_hip_shlink_t * in [ FD_ED25519_HIP_VSERVICE_LINK_MAX ];
  fd_ed25519_hip_shlink_t * out[ FD_ED25519_HIP_VSERVICE_LINK_MAX ];
  memset( in, 0, sizeof(in) ); memset( out, 0, sizeof(out) );
  int rc = 0;
  for( unsigned k=0U; k<tiles; k++ ) {
    char name[ 128 ];
    snprintf( name, sizeof(name), "%s%u_txn", prefix, k );
    in[ k ] = fd_ed25519_hip_shlink_create( name, depth );
    snprintf( name, sizeof(name), "%s%u_vd", prefix, k );
    out[ k ] = fd_ed25519_hip_shlink_create( name, depth );
    if( !in[ k ] || !out[ k ] ) {
      fprintf( stderr, "fd_verify_hip_service: cannot create the links of tile %u (%s*: stale from a killed service?)\n",
               k, prefix );
      rc = 1;
      break;
    }
  }
  if( !rc ) {
    printf( "ready %u\n", tiles );
    fflush( stdout );
    fd_ed25519_hip_vservice_stats_t st[ FD_ED25519_HIP_VSERVICE_LINK_MAX ];
    memset( st, 0, sizeof(st) );
    int err = fd_ed25519_hip_vservice_run_links( gpu, slots, batch, flags, in, out, tiles, st );
    /* one JSON line for tools and tests: per-tile device memory and the
       base tables this one process holds for all of them */
    unsigned long shared = 0UL;
    for( unsigned k=0U; k<tiles; k++ ) if( st[ k ].shared_device_bytes>shared ) shared = st[ k ].shared_device_bytes;
    printf( "{\"tiles\": %u, \"shared_device_bytes\": %lu, \"tile_device_bytes\": [", tiles, shared );
    for( unsigned k=0U; k<tiles; k++ ) printf( "%s%lu", k ? ", " : "", st[ k ].device_bytes );
    printf( "], \"txns\": [" );
    for( unsigned k=0U; k<tiles; k++ ) printf( "%s%lu", k ? ", " : "", st[ k ].txn_cnt );
    printf( "], \"rc\": %d}\n", err );
    fflush( stdout );
    if( err ) {
      fprintf( stderr, "fd_verify_hip_service: FAILED: %s (%d): %s; every link is marked failed\n",
               fd_ed25519_hip_strerror( err ), err, fd_ed25519_hip_last_error() );
      rc = 2;
    } else {
      for( unsigned k=0U; k<tiles; k++ )
        fprintf( stderr, "fd_verify_hip_service: tile %u: %lu txns in %lu batches, %.3f s, %lu device bytes\n", k,
                 st[ k ].txn_cnt, st[ k ].batches, st[ k ].seconds, st[ k ].device_bytes );
    }
  }
  for( unsigned k=0U; k<tiles; k++ ) {
    fd_ed25519_hip_shlink_leave( in [ k ], 1 );
    fd_ed25519_hip_shlink_leave( out[ k ], 1 );
  }
  return rc;
}
