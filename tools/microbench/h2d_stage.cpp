// h2d_stage.cpp -- host -> HBM upload rates for the blst drop-in's inputs
// (caller-owned pageable memory): 128 MiB = the points + scalars of a G1
// n = 2^20 blst_p1s_mult_pippenger call.
//   pageable   : one hipMemcpy from pageable memory (HIP stages internally)
//   pinned     : one hipMemcpyAsync from page-locked memory (the DMA ceiling)
//   memcpy Tn  : host memcpy pageable -> pinned with n threads (no DMA)
//   staged Tn  : chunked pipeline: n threads fill a pinned chunk, DMA it while
//                the next chunk fills (chunk size / slot count as printed)
// build: hipcc -O2 -std=c++17 --offload-arch=gfx950 h2d_stage.cpp -o h2d_stage -lpthread
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <chrono>
#include <thread>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void par_copy(uint8_t *dst, const uint8_t *src, size_t bytes, int nt) {
  if (nt <= 1) {
    memcpy(dst, src, bytes);
    return;
  }
  std::vector<std::thread> th;
  size_t per = (bytes / nt + 4095) & ~(size_t)4095;
  for (int t = 0; t < nt; ++t) {
    size_t a = std::min(bytes, t * per), b = std::min(bytes, a + per);
    if (a < b) th.emplace_back([=] { memcpy(dst + a, src + a, b - a); });
  }
  for (auto &x : th) x.join();
}

int main() {
  const size_t bytes = 128ull << 20;
  std::vector<uint8_t> src(bytes);
  for (size_t i = 0; i < bytes; ++i) src[i] = (uint8_t)(i * 131 + 7);
  void *dev, *pin;
  CK(hipMalloc(&dev, bytes));
  CK(hipHostMalloc(&pin, bytes, 0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  auto best = [&](auto fn) {
    double b = 1e9;
    for (int r = 0; r < 5; ++r) {
      CK(hipDeviceSynchronize());
      double t = now();
      fn();
      CK(hipDeviceSynchronize());
      b = std::min(b, now() - t);
    }
    return b;
  };
  double t = best([&] { CK(hipMemcpy(dev, src.data(), bytes, hipMemcpyHostToDevice)); });
  printf("pageable hipMemcpy     %7.3f ms  %6.1f GB/s\n", t * 1e3, bytes / t / 1e9);
  t = best([&] { CK(hipMemcpyAsync(dev, pin, bytes, hipMemcpyHostToDevice, s)); });
  printf("pinned hipMemcpyAsync  %7.3f ms  %6.1f GB/s\n", t * 1e3, bytes / t / 1e9);
  for (int nt : {1, 2, 4, 8, 16}) {
    t = best([&] { par_copy((uint8_t *)pin, src.data(), bytes, nt); });
    printf("memcpy -> pinned T%-2d   %7.3f ms  %6.1f GB/s\n", nt, t * 1e3, bytes / t / 1e9);
  }
  for (size_t chunk : {(size_t)4 << 20, (size_t)8 << 20, (size_t)16 << 20}) {
    const int slots = 4;
    std::vector<hipEvent_t> ev(slots);
    for (auto &e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (int nt : {4, 8, 16}) {
      t = best([&] {
        size_t k = 0;
        for (size_t off = 0; off < bytes; off += chunk, ++k) {
          int sl = (int)(k % slots);
          if (k >= (size_t)slots) CK(hipEventSynchronize(ev[sl]));
          size_t len = std::min(chunk, bytes - off);
          uint8_t *p = (uint8_t *)pin + sl * chunk;
          par_copy(p, src.data() + off, len, nt);
          CK(hipMemcpyAsync((uint8_t *)dev + off, p, len, hipMemcpyHostToDevice, s));
          CK(hipEventRecord(ev[sl], s));
        }
      });
      printf("staged %2zu MiB x%d T%-2d  %7.3f ms  %6.1f GB/s\n", chunk >> 20, slots, nt, t * 1e3, bytes / t / 1e9);
    }
    for (auto &e : ev) CK(hipEventDestroy(e));
  }
  std::vector<uint8_t> back(bytes);
  CK(hipMemcpy(back.data(), dev, bytes, hipMemcpyDeviceToHost));
  printf("check %s\n", memcmp(back.data(), src.data(), bytes) ? "FAIL" : "ok");
  printf("hw threads %u\n", std::thread::hardware_concurrency());
  return 0;
}
