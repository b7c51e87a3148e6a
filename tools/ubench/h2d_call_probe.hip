/* h2d_call_probe -- what a verify-service batch submit costs the host
   thread (run on the box): the time inside hipMemcpyAsync H2D calls for
   the sizes a batch moves, from hipHostMalloc'd memory, from malloc'd
   memory registered with hipHostRegister, and from a registered shared
   mapping (the zero-copy service's txn link), then the transfer's own
   rate; an empty kernel launch and an event record / query; and the same
   copy calls from 1, 4 and 8 threads at once (the service's link threads),
   each on its own stream.  One JSON object per line.

     hipcc --offload-arch=gfx950 -O2 -o h2d_call_probe tools/ubench/h2d_call_probe.hip -lpthread
     ./h2d_call_probe */
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

#define CK( x ) do { hipError_t e_ = (x); if( e_!=hipSuccess ) { fprintf( stderr, "%s: %s\n", #x, hipGetErrorString( e_ ) ); exit( 1 ); } } while(0)

static double
now( void ) {
  struct timespec t;
  clock_gettime( CLOCK_MONOTONIC, &t );
  return (double)t.tv_sec + 1e-9*(double)t.tv_nsec;
}

__global__ void empty_kernel( int * p ) { if( p && blockIdx.x==0 && threadIdx.x<64 ) p[threadIdx.x] = (int)threadIdx.x; }

static void
copy_calls( char const * kind, unsigned char * src, void * dst, size_t sz, hipStream_t st, int reps ) {
  CK( hipMemcpyAsync( dst, src, sz, hipMemcpyHostToDevice, st ) );   /* first use outside the timing */
  CK( hipStreamSynchronize( st ) );
  double call = 0.0;
  double t0 = now();
  for( int r=0; r<reps; r++ ) {
    double c0 = now();
    CK( hipMemcpyAsync( dst, src, sz, hipMemcpyHostToDevice, st ) );
    call += now() - c0;
  }
  CK( hipStreamSynchronize( st ) );
  double tot = now() - t0;
  printf( "{\"probe\": \"h2d\", \"src\": \"%s\", \"bytes\": %zu, \"call_us\": %.2f, \"per_copy_us\": %.2f, \"GBps\": %.2f}\n",
          kind, sz, 1e6*call/reps, 1e6*tot/reps, (double)sz*reps/tot/1e9 );
  fflush( stdout );
}

typedef struct {
  unsigned char * src;
  void *          dst;
  size_t          sz;
  int             reps;
  int             kernels;   /* a launch after each copy */
  double          call_us;
  double          launch_us;
} th_arg_t;

static void *
th_main( void * a ) {
  th_arg_t * t = (th_arg_t *)a;
  hipStream_t st;
  CK( hipStreamCreateWithFlags( &st, hipStreamNonBlocking ) );
  CK( hipMemcpyAsync( t->dst, t->src, t->sz, hipMemcpyHostToDevice, st ) );
  CK( hipStreamSynchronize( st ) );
  double call = 0.0, launch = 0.0;
  for( int r=0; r<t->reps; r++ ) {
    double c0 = now();
    CK( hipMemcpyAsync( t->dst, t->src, t->sz, hipMemcpyHostToDevice, st ) );
    double c1 = now();
    if( t->kernels ) hipLaunchKernelGGL( empty_kernel, dim3( 16 ), dim3( 256 ), 0, st, (int *)NULL );
    double c2 = now();
    call += c1 - c0; launch += c2 - c1;
    if( !(r & 7) ) CK( hipStreamSynchronize( st ) );
  }
  CK( hipStreamSynchronize( st ) );
  t->call_us = 1e6*call/t->reps; t->launch_us = 1e6*launch/t->reps;
  CK( hipStreamDestroy( st ) );
  return NULL;
}

int
main( void ) {
  CK( hipSetDevice( 0 ) );
  size_t cap = 8UL << 20;
  void * d;
  CK( hipMalloc( &d, 8 * cap ) );
  hipStream_t st;
  CK( hipStreamCreateWithFlags( &st, hipStreamNonBlocking ) );

  unsigned char * hm;
  CK( hipHostMalloc( (void **)&hm, cap, hipHostMallocDefault ) );
  memset( hm, 1, cap );
  unsigned char * rm = (unsigned char *)aligned_alloc( 4096, cap );
  memset( rm, 2, cap );
  CK( hipHostRegister( rm, cap, hipHostRegisterPortable ) );
  char name[ 64 ];
  snprintf( name, sizeof(name), "/h2d_probe_%d", (int)getpid() );
  int fd = shm_open( name, O_RDWR | O_CREAT | O_EXCL, 0600 );
  if( fd<0 || ftruncate( fd, (off_t)cap ) ) { perror( "shm" ); return 1; }
  unsigned char * sm = (unsigned char *)mmap( NULL, cap, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0 );
  close( fd );
  shm_unlink( name );
  if( sm==MAP_FAILED ) { perror( "mmap" ); return 1; }
  memset( sm, 3, cap );
  CK( hipHostRegister( sm, cap, hipHostRegisterPortable ) );

  size_t sizes[] = { 16UL << 10, 64UL << 10, 256UL << 10, 1UL << 20, 2UL << 20, 4UL << 20 };
  for( unsigned i=0; i<sizeof(sizes)/sizeof(sizes[0]); i++ ) {
    copy_calls( "hipHostMalloc", hm, d, sizes[i], st, 64 );
    copy_calls( "malloc+hipHostRegister", rm, d, sizes[i], st, 64 );
    copy_calls( "shm+hipHostRegister", sm, d, sizes[i], st, 64 );
    copy_calls( "shm+hipHostRegister+4KiB", sm + 4096, d, sizes[i] - 4096, st, 64 );
  }

  /* a launch and an event on a stream */
  hipEvent_t ev;
  CK( hipEventCreateWithFlags( &ev, hipEventDisableTiming ) );
  hipLaunchKernelGGL( empty_kernel, dim3( 16 ), dim3( 256 ), 0, st, (int *)NULL );
  CK( hipStreamSynchronize( st ) );
  double la = 0.0, er = 0.0, eq = 0.0;
  for( int r=0; r<256; r++ ) {
    double c0 = now();
    hipLaunchKernelGGL( empty_kernel, dim3( 16 ), dim3( 256 ), 0, st, (int *)NULL );
    double c1 = now();
    CK( hipEventRecord( ev, st ) );
    double c2 = now();
    (void)hipEventQuery( ev );
    double c3 = now();
    la += c1 - c0; er += c2 - c1; eq += c3 - c2;
  }
  CK( hipStreamSynchronize( st ) );
  printf( "{\"probe\": \"calls\", \"launch_us\": %.2f, \"event_record_us\": %.2f, \"event_query_us\": %.2f}\n",
          1e6*la/256, 1e6*er/256, 1e6*eq/256 );
  fflush( stdout );

  /* several threads submitting at once (1 MiB copies + a launch each) */
  int counts[] = { 1, 4, 8, 1, 8 };
  for( unsigned c=0; c<5; c++ ) {
    int n = counts[c], kernels = c<3;
    pthread_t th[ 8 ];
    th_arg_t ta[ 8 ];
    unsigned char * srcs[ 8 ];
    for( int k=0; k<n; k++ ) {
      CK( hipHostMalloc( (void **)&srcs[k], 1UL << 20, hipHostMallocDefault ) );
      memset( srcs[k], k, 1UL << 20 );
      ta[k].src = srcs[k]; ta[k].dst = (unsigned char *)d + (size_t)k * cap; ta[k].sz = 1UL << 20; ta[k].reps = 256; ta[k].kernels = kernels;
      pthread_create( &th[k], NULL, th_main, &ta[k] );
    }
    double call = 0.0, launch = 0.0;
    for( int k=0; k<n; k++ ) { pthread_join( th[k], NULL ); call += ta[k].call_us; launch += ta[k].launch_us; }
    printf( "{\"probe\": \"threads\", \"threads\": %d, \"kernel_after_each_copy\": %d, \"h2d_1MiB_call_us\": %.2f, "
            "\"launch_us\": %.2f, \"HSA_ENABLE_SDMA\": \"%s\"}\n", n, kernels, call/n, launch/n,
            getenv( "HSA_ENABLE_SDMA" ) ? getenv( "HSA_ENABLE_SDMA" ) : "" );
    fflush( stdout );
    for( int k=0; k<n; k++ ) CK( hipHostFree( srcs[k] ) );
  }
  /* submit patterns of one batch (1 thread): which call blocks the host */
  {
    hipStream_t s1, s2;
    CK( hipStreamCreateWithFlags( &s1, hipStreamNonBlocking ) );
    CK( hipStreamCreateWithFlags( &s2, hipStreamNonBlocking ) );
    hipEvent_t e1, e2;
    CK( hipEventCreateWithFlags( &e1, hipEventDisableTiming ) );
    CK( hipEventCreateWithFlags( &e2, hipEventDisableTiming ) );
    size_t in = 1UL << 20, out = 16UL << 10;
    for( int pat=0; pat<5; pat++ ) {
      double t_h2d = 0.0, t_k = 0.0, t_d2h = 0.0;
      int reps = 128;
      for( int r=0; r<reps; r++ ) {
        double c0 = now(), c1, c2, c3;
        if( pat==0 ) {          /* one stream: H2D, kernel, D2H (the pipe today) */
          CK( hipMemcpyAsync( d, hm, in, hipMemcpyHostToDevice, s1 ) ); c1 = now();
          hipLaunchKernelGGL( empty_kernel, dim3( 64 ), dim3( 256 ), 0, s1, (int *)NULL ); c2 = now();
          CK( hipMemcpyAsync( hm + in, d, out, hipMemcpyDeviceToHost, s1 ) ); c3 = now();
        } else if( pat==1 ) {   /* copies on s2, kernel on s1, joined by events */
          CK( hipMemcpyAsync( d, hm, in, hipMemcpyHostToDevice, s2 ) );
          CK( hipEventRecord( e1, s2 ) ); c1 = now();
          CK( hipStreamWaitEvent( s1, e1, 0 ) );
          hipLaunchKernelGGL( empty_kernel, dim3( 64 ), dim3( 256 ), 0, s1, (int *)NULL );
          CK( hipEventRecord( e2, s1 ) ); c2 = now();
          CK( hipStreamWaitEvent( s2, e2, 0 ) );
          CK( hipMemcpyAsync( hm + in, d, out, hipMemcpyDeviceToHost, s2 ) ); c3 = now();
        } else if( pat==2 ) {   /* H2D on s2, kernel on s1, no D2H (the kernel writes host memory) */
          CK( hipMemcpyAsync( d, hm, in, hipMemcpyHostToDevice, s2 ) );
          CK( hipEventRecord( e1, s2 ) ); c1 = now();
          CK( hipStreamWaitEvent( s1, e1, 0 ) );
          hipLaunchKernelGGL( empty_kernel, dim3( 64 ), dim3( 256 ), 0, s1, (int *)(hm + in) );
          CK( hipEventRecord( e2, s1 ) ); c2 = now(); c3 = c2;
        } else if( pat==3 ) {   /* one stream: H2D, kernel (no D2H) */
          CK( hipMemcpyAsync( d, hm, in, hipMemcpyHostToDevice, s1 ) ); c1 = now();
          hipLaunchKernelGGL( empty_kernel, dim3( 64 ), dim3( 256 ), 0, s1, (int *)(hm + in) ); c2 = now(); c3 = c2;
        } else {                /* one stream: kernel, D2H only */
          c1 = c0;
          hipLaunchKernelGGL( empty_kernel, dim3( 64 ), dim3( 256 ), 0, s1, (int *)NULL ); c2 = now();
          CK( hipMemcpyAsync( hm + in, d, out, hipMemcpyDeviceToHost, s1 ) ); c3 = now();
        }
        t_h2d += c1 - c0; t_k += c2 - c1; t_d2h += c3 - c2;
        if( (r & 3)==3 ) { CK( hipStreamSynchronize( s1 ) ); CK( hipStreamSynchronize( s2 ) ); }
      }
      CK( hipStreamSynchronize( s1 ) ); CK( hipStreamSynchronize( s2 ) );
      printf( "{\"probe\": \"pattern\", \"pattern\": %d, \"h2d_call_us\": %.2f, \"kernel_call_us\": %.2f, "
              "\"d2h_call_us\": %.2f, \"HSA_ENABLE_SDMA\": \"%s\"}\n", pat, 1e6*t_h2d/reps, 1e6*t_k/reps,
              1e6*t_d2h/reps, getenv( "HSA_ENABLE_SDMA" ) ? getenv( "HSA_ENABLE_SDMA" ) : "" );
      fflush( stdout );
    }
  }
  CK( hipHostUnregister( sm ) );
  CK( hipHostUnregister( rm ) );
  CK( hipHostFree( hm ) );
  CK( hipFree( d ) );
  return 0;
}
