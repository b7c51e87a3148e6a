/* ref_dropin_ed25519.c -- TEST INFRASTRUCTURE ONLY (oracle/Makefile
   ref-dropin): the reference's own verify tests, compiled from its sources
   (src/ballet/ed25519/test_ed25519.c:1013-1082: test_wycheproofs,
   test_cctv, test_cctv_batch), linked so that fd_ed25519_verify and
   fd_ed25519_verify_batch_single_msg resolve to libfd_ed25519_hip.so (the
   reference's own definitions are made local to their object by objcopy)
   while everything else they use (sign, public_from_private, sha512, the
   wycheproof / cctv tables, fd_log) is the reference's.  Exit 0 means the
   reference's tests passed against the GPU drop-ins.

   test_ed25519.c's main also runs the field / scalar unit tests and a
   verify benchmark of ~300K synchronous single calls; this driver runs only
   the three verify suites, the ones that exercise the drop-ins. */
#define main fdref_test_ed25519_unused_main
#include "ballet/ed25519/test_ed25519.c"
#undef main

int
main( int     argc,
      char ** argv ) {
  fd_log_private_boot( &argc, &argv );
  fd_rng_t _rng[1]; fd_rng_t * rng = fd_rng_join( fd_rng_new( _rng, 0U, 0UL ) );
  fd_sha512_t _sha[1]; fd_sha512_t * sha = fd_sha512_join( fd_sha512_new( _sha ) );
  test_wycheproofs( sha );
  test_cctv       ( sha );
  test_cctv_batch ( rng, sha );
  fd_sha512_delete( fd_sha512_leave( sha ) );
  fd_rng_delete( fd_rng_leave( rng ) );
  FD_LOG_NOTICE(( "pass" ));
  fd_log_private_halt();
  return 0;
}
