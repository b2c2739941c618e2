// Instruction-throughput microbenchmark for gfx950 integer/fp64 ops used by
// Fp381 Montgomery arithmetic.  Each lane runs 8 independent dependency
// chains of one instruction; the grid fills the chip.  Prints ops/s per
// instruction (ops = lane-instructions).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 256
#define CH 8

template <int KIND>
__global__ __launch_bounds__(256) void k_rate(uint32_t *out, uint32_t seed) {
  uint32_t t = threadIdx.x + blockIdx.x * blockDim.x;
  uint64_t acc[CH];
  uint32_t a[CH];
  double d[CH];
#pragma unroll
  for (int k = 0; k < CH; ++k) { acc[k] = t * 0x9e3779b9u + k + seed; a[k] = (t ^ (k * 0x85ebca6bu)) | 1; d[k] = (double)(t + k); }
  uint32_t b = seed | 3;
  double db = 1.0000001;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      if constexpr (KIND == 0) {  // v_mad_u64_u32
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[k]) : "v"(a[k]), "v"(b) : "vcc");
      } else if constexpr (KIND == 1) {  // v_mul_lo_u32
        uint32_t x = (uint32_t)acc[k];
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(a[k]));
        acc[k] = x;
      } else if constexpr (KIND == 2) {  // v_mul_hi_u32
        uint32_t x = (uint32_t)acc[k];
        asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(a[k]));
        acc[k] = x;
      } else if constexpr (KIND == 3) {  // v_add_co_u32 / v_addc_co_u32 pair (2 ops)
        uint32_t lo = (uint32_t)acc[k], hi = (uint32_t)(acc[k] >> 32);
        asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %2, vcc" : "+v"(lo), "+v"(hi) : "v"(a[k]) : "vcc");
        acc[k] = ((uint64_t)hi << 32) | lo;
      } else if constexpr (KIND == 4) {  // v_fma_f64
        asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d[k]) : "v"(db));
      } else if constexpr (KIND == 5) {  // v_mad_u32_u24
        uint32_t x = (uint32_t)acc[k];
        asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(x) : "v"(a[k]));
        acc[k] = x;
      } else if constexpr (KIND == 6) {  // v_add3_u32
        uint32_t x = (uint32_t)acc[k];
        asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(x) : "v"(a[k]));
        acc[k] = x;
      } else if constexpr (KIND == 7) {  // v_mul_hi_u32_u24
        uint32_t x = (uint32_t)acc[k];
        asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(x) : "v"(a[k]));
        acc[k] = x;
      } else if constexpr (KIND == 8) {  // v_add_co_u32 alone (carry to vcc)
        uint32_t x = (uint32_t)acc[k];
        asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(x) : "v"(a[k]) : "vcc");
        acc[k] = x;
      } else if constexpr (KIND == 9) {  // v_mad_u64_u32 with SGPR-pair carry out (not vcc)
        asm volatile("v_mad_u64_u32 %0, s[20:21], %1, %2, %0" : "+v"(acc[k]) : "v"(a[k]), "v"(b) : "s20", "s21");
      } else if constexpr (KIND == 10) {  // v_lshl_add_u64 (gfx94x+)
        asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(acc[k]) : "v"((uint64_t)a[k]));
      } else if constexpr (KIND == 11) {  // v_add_u32 (plain)
        uint32_t x = (uint32_t)acc[k];
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(a[k]));
        acc[k] = x;
      } else if constexpr (KIND == 12) {  // v_lshrrev_b64 (the FIPS column carry shift)
        asm volatile("v_lshrrev_b64 %0, 28, %0" : "+v"(acc[k]));
      } else if constexpr (KIND == 13) {  // v_and_b32
        uint32_t x = (uint32_t)acc[k];
        asm volatile("v_and_b32 %0, %0, %1" : "+v"(x) : "v"(a[k]));
        acc[k] = x;
      } else if constexpr (KIND == 14) {  // v_alignbit_b32 (one half of a 64-bit shift)
        uint32_t x = (uint32_t)acc[k];
        asm volatile("v_alignbit_b32 %0, %1, %0, 28" : "+v"(x) : "v"(a[k]));
        acc[k] = x;
      } else if constexpr (KIND == 15) {  // v_mad_u64_u32 with a zero addend (a 32x32->64 multiply)
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(acc[k]) : "v"((uint32_t)acc[k]), "v"(b) : "vcc");
      }
    }
  }
  uint64_t s = 0; double ds = 0;
#pragma unroll
  for (int k = 0; k < CH; ++k) { s += acc[k]; ds += d[k]; }
  if (s == 0x123456789ull && ds == 1.2345) out[t] = 1;
}

static const char *names[] = {"v_mad_u64_u32(vcc)", "v_mul_lo_u32", "v_mul_hi_u32", "v_add_co+v_addc_co (pair)", "v_fma_f64",
                              "v_mad_u32_u24", "v_add3_u32", "v_mul_hi_u32_u24", "v_add_co_u32", "v_mad_u64_u32(sgpr)", "v_lshl_add_u64", "v_add_u32",
                              "v_lshrrev_b64", "v_and_b32", "v_alignbit_b32", "v_mad_u64_u32(x,y,0)"};

template <int K>
void run(uint32_t *d_out, int blocks) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k_rate<K>, dim3(blocks), dim3(256), 0, 0, d_out, 7u);
  hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_rate<K>, dim3(blocks), dim3(256), 0, 0, d_out, 7u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  double ops = (double)blocks * 256 * ITERS * CH;
  printf("%-28s %8.3f ms  %8.2f T lane-ops/s  (%.3f lane-ops/clk/CU @2.4GHz)\n", names[K], best, ops / best / 1e9,
         ops / (best * 1e-3) / 2.4e9 / 256);
}

int main() {
  uint32_t *d_out; int blocks = 256 * 32;
  hipMalloc(&d_out, (size_t)blocks * 256 * 4);
  run<0>(d_out, blocks); run<9>(d_out, blocks); run<1>(d_out, blocks); run<2>(d_out, blocks); run<3>(d_out, blocks);
  run<4>(d_out, blocks); run<5>(d_out, blocks); run<6>(d_out, blocks); run<7>(d_out, blocks); run<8>(d_out, blocks);
  run<10>(d_out, blocks); run<11>(d_out, blocks); run<12>(d_out, blocks); run<13>(d_out, blocks);
  run<14>(d_out, blocks); run<15>(d_out, blocks);
  hipFree(d_out);
  return 0;
}
