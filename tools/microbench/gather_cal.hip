// Calibration of rocprofv3 FETCH_SIZE for the bucket accumulation's access
// pattern (MI355X_MICROARCH.md, HBM section: "other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern").
//
// k_gather: every lane reads ONE random 128-B row of a 4-GiB table as seven
// 16-B loads (112 B: the internal affine row of k_accumulate, kernels.hpp),
// like the accumulation's table gathers; 12.58 M lanes (the CHES 2^20 entry
// count).  k_stream: a coalesced 16-B/lane streaming read of 1 GiB (the
// guide's x2 case).  Known byte counts are printed; run each under
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace ... -- ./gather_cal
// and divide FETCH_SIZE*1024 by them (tools/pmc_traffic.py applies the result).
//
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/gather_cal.hip -o gather_cal
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                  \
      return 1;                                                               \
    }                                                                         \
  } while (0)

__global__ __launch_bounds__(256) void k_gather(const uint4 *__restrict__ table, const uint32_t *__restrict__ idx,
                                                uint32_t *__restrict__ out, size_t n) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4 *row = table + (size_t)idx[i] * 8;  // 128-B rows
  uint32_t x = 0;
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    uint4 v = row[k];
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  out[i] = x;
}

__global__ __launch_bounds__(256) void k_stream(const uint4 *__restrict__ a, uint32_t *__restrict__ out, size_t n) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint4 v = a[i];
  if ((v.x ^ v.y ^ v.z ^ v.w) == 0x12345678u) out[0] = 1;  // keeps the load, ~never stores
}

int main() {
  const size_t rows = (size_t)1 << 25;            // 32 M rows x 128 B = 4 GiB
  const size_t n = (size_t)12582912;              // CHES 2^20 entries (n h)
  const size_t sn = ((size_t)1 << 30) / 16;       // 1 GiB streamed
  uint4 *table;
  uint32_t *idx, *out;
  CK(hipMalloc(&table, rows * 128));
  CK(hipMemset(table, 0x5a, rows * 128));
  std::vector<uint32_t> h(n);
  uint64_t s = 0x9e3779b97f4a7c15ull;
  for (size_t i = 0; i < n; ++i) {
    s ^= s << 13, s ^= s >> 7, s ^= s << 17;
    h[i] = (uint32_t)(s % rows);
  }
  CK(hipMalloc(&idx, n * 4));
  CK(hipMalloc(&out, n * 4));
  CK(hipMemcpy(idx, h.data(), n * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_gather, dim3((n + 255) / 256), dim3(256), 0, 0, table, idx, out, n);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("k_gather: %zu rows x 112 B = %zu B read (%zu B of 128-B lines) + %zu B idx + %zu B out written, %.3f ms, %.0f GB/s\n",
           n, n * 112, n * 128, n * 4, n * 4, ms, (n * 112.0 + n * 8.0) / ms / 1e6);
  }
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_stream, dim3((sn + 255) / 256), dim3(256), 0, 0, table, out, sn);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("k_stream: %zu B read, %.3f ms, %.0f GB/s\n", sn * 16, ms, sn * 16.0 / ms / 1e6);
  }
  CK(hipFree(table));
  CK(hipFree(idx));
  CK(hipFree(out));
  return 0;
}
