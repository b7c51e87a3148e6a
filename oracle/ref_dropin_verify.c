/* ref_dropin_verify.c -- TEST INFRASTRUCTURE ONLY (oracle/Makefile
   ref-dropin): the reference verify tile's own unit test
   (src/app/fdctl/run/tiles/test_verify.c: fd_txn_verify over its fixture
   transactions, success / failure / dedup, src/app/fdctl/run/tiles/
   test_verify.c:162-261) compiled from the reference's sources, with
   fd_ed25519_verify_batch_single_msg resolving to libfd_ed25519_hip.so
   (the reference's definition made local by objcopy).  Exit 0: the tile's
   verdicts are the reference's with the GPU drop-in underneath. */
#define main fdref_test_verify_unused_main
#include "app/fdctl/run/tiles/test_verify.c"
#undef main

int
main( int     argc,
      char ** argv ) {
  fd_log_private_boot( &argc, &argv );
  test_verify_success();
  test_verify_invalid_sigs_success();
  test_verify_invalid_dedup_success();
  FD_LOG_NOTICE(( "pass" ));
  fd_log_private_halt();
  return 0;
}
