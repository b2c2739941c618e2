// Does a cross-stream wait delay a kernel while another stream runs a chain of
// small dependent kernels?  (Batch pipeline study)  Stream A runs
// "big" kernels back to back (every CU busy ~1 ms); stream B runs, after each
// big kernel, a chain of N tiny kernels (~20 us each); before each big kernel
// stream A waits on an event of stream C that completed long ago (variant 1),
// or on nothing (variant 0).  Prints the idle gap between consecutive big kernels.
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/queue_gate.hip -o queue_gate
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                        \
  do {                                                               \
    hipError_t e_ = (x);                                             \
    if (e_ != hipSuccess) {                                          \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
      return 1;                                                      \
    }                                                                \
  } while (0)

__global__ void k_spin(long long cycles, int *sink) {
  const long long t0 = clock64();
  while (clock64() - t0 < cycles) {
  }
  if (threadIdx.x == 0 && blockIdx.x == 0x7fffffff) *sink = 1;
}

int main(int argc, char **argv) {
  const int NT = argc > 1 ? atoi(argv[1]) : 40;  // tiny kernels per big kernel
  int *sink;
  CK(hipMalloc(&sink, 4));
  hipStream_t A, B, C;
  int lo, hi;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
  CK(hipStreamCreateWithPriority(&C, hipStreamNonBlocking, hi));
  // clock64 runs at the shader clock: calibrate ~1 us
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, A));
  hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, A, 1000000LL, sink);
  CK(hipEventRecord(e1, A));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double cyc_per_us = 1e6 / (ms * 1e3);
  printf("clock64: %.0f cycles/us\n", cyc_per_us);
  const int K = 12;
  for (int variant = 0; variant < 3; ++variant) {
    std::vector<hipEvent_t> bs(K), be(K), ea(K), ec(K), eb(K);
    for (int k = 0; k < K; ++k) {
      CK(hipEventCreate(&bs[k]));
      CK(hipEventCreate(&be[k]));
      CK(hipEventCreateWithFlags(&ea[k], hipEventDisableTiming));
      CK(hipEventCreateWithFlags(&ec[k], hipEventDisableTiming));
      CK(hipEventCreateWithFlags(&eb[k], hipEventDisableTiming));
    }
    CK(hipDeviceSynchronize());
    for (int k = 0; k < K; ++k) {
      if (variant >= 1) {  // an already-finished dependency from stream C
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, C, (long long)(5 * cyc_per_us), sink);
        CK(hipEventRecord(ec[k], C));
        CK(hipStreamWaitEvent(A, ec[k], 0));
      }
      if (variant == 2 && k >= 1) CK(hipStreamWaitEvent(A, eb[k - 1], 0));  // first tiny kernel of the previous chain
      CK(hipEventRecord(bs[k], A));
      hipLaunchKernelGGL(k_spin, dim3(256 * 12), dim3(256), 0, A, (long long)(1000 * cyc_per_us), sink);  // ~1 ms
      CK(hipEventRecord(be[k], A));
      CK(hipEventRecord(ea[k], A));
      CK(hipStreamWaitEvent(B, ea[k], 0));
      for (int t = 0; t < NT; ++t) {
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, B, (long long)(18 * cyc_per_us), sink);
        if (t == 0) CK(hipEventRecord(eb[k], B));
      }
    }
    CK(hipDeviceSynchronize());
    double gap = 0, big = 0;
    for (int k = 1; k < K; ++k) {
      float g, b;
      CK(hipEventElapsedTime(&g, be[k - 1], bs[k]));
      CK(hipEventElapsedTime(&b, bs[k], be[k]));
      gap += g, big += b;
    }
    printf("variant %d (%s), %d tiny kernels per big: big %.3f ms, gap between bigs %.1f us (mean of %d)\n",
           variant, variant == 0 ? "no cross-stream wait" : variant == 1 ? "wait on finished stream-C event" : "+ wait on the first kernel of the previous B chain",
           NT, big / (K - 1), gap / (K - 1) * 1e3, K - 1);
  }
  return 0;
}
