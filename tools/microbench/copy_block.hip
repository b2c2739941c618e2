// Host-side cost of hipMemcpyAsync H2D enqueues in the batch's copy pattern.
// The bench's H2D headline sometimes lost ~7 ms because ONE hipMemcpyAsync call
// (the second of a batch) blocked the host thread that enqueues the whole
// pipeline (rocprofv3 HIP API trace, profiles/r05_h2d_block.txt).  This probe
// repeats the pattern -- a kernel on stream A, an event on A, the copy stream
// waiting on it, then K 32-MiB copies from page-locked memory on the copy
// stream -- with an idle gap before each round, and prints the longest enqueue
// per round and which call it was.
//   usage: copy_block [rounds] [K] [gap_ms] [mode] [MiB per copy]
//   mode 0: copy stream waits on A's event first (the batch's pattern)
//   mode 1: no cross-stream wait
//   mode 2: copies issued by a second host thread (the main thread only waits)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__global__ void k_spin(unsigned *p, int n) {
  unsigned v = threadIdx.x;
  for (int i = 0; i < n; ++i) v = v * 1664525u + 1013904223u;
  if (v == 0x12345678u) p[threadIdx.x] = v;
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 30;
  const int K = argc > 2 ? atoi(argv[2]) : 20;
  const double gap = argc > 3 ? atof(argv[3]) : 10.0;
  const int mode = argc > 4 ? atoi(argv[4]) : 0;
  const size_t S = (size_t)(argc > 5 ? atoi(argv[5]) : 32) << 20;
  long calls = 0;
  void *host = nullptr, *dev = nullptr;
  unsigned *scratch = nullptr;
  CK(hipHostMalloc(&host, S * K, hipHostMallocDefault));
  memset(host, 1, S * K);
  CK(hipMalloc(&dev, S * K));
  CK(hipMalloc(&scratch, 4096));
  hipStream_t a, c;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&c, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  int slow = 0;
  for (int r = 0; r < rounds; ++r) {
    std::this_thread::sleep_for(std::chrono::microseconds((long)(gap * 1000)));
    const double t0 = now_ms();
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, a, scratch, 1000);
    CK(hipEventRecord(ev, a));
    std::vector<double> dt(K);
    auto issue = [&] {
      if (mode == 0) CK(hipStreamWaitEvent(c, ev, 0));
      for (int k = 0; k < K; ++k) {
        const double t = now_ms();
        CK(hipMemcpyAsync((char *)dev + k * S, (char *)host + k * S, S, hipMemcpyHostToDevice, c));
        dt[k] = now_ms() - t;
        if (dt[k] > 1.0) printf("  blocked: call %ld (round %d, #%d) %.3f ms\n", calls, r, k, dt[k]);
        ++calls;
      }
    };
    if (mode == 2) {
      std::thread th(issue);
      th.join();
    } else {
      issue();
    }
    const double t_issue = now_ms() - t0;
    CK(hipStreamSynchronize(c));
    CK(hipStreamSynchronize(a));
    const double t_all = now_ms() - t0;
    int arg = 0;
    for (int k = 1; k < K; ++k)
      if (dt[k] > dt[arg]) arg = k;
    slow += dt[arg] > 1.0;
    printf("round %2d issue %7.3f ms  total %7.3f ms  longest call #%d %7.3f ms\n", r, t_issue, t_all, arg, dt[arg]);
  }
  printf("mode %d gap %.1f ms: %d of %d rounds had a call > 1 ms\n", mode, gap, slow, rounds);
  return 0;
}
