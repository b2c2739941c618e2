// bucket_sort.hpp -- two-level counting sort of MSM entries by bucket (gfx950).
//
// Input: one (key, val) per entry, key = bucket id < NB (or KEY_NONE = skip),
// val = payload (point/table slot | sign << 31).  Output: vals grouped by
// bucket, per-bucket counts and offsets, and a schedule key per bucket.
// All counting is in LDS; global memory only sees streaming reads and writes
// that are contiguous per (tile, coarse bin) or within one coarse bin:
//
//   k_bs_hist     per tile of TILE entries: LDS histogram over coarse bins
//                 (bucket >> FB_BITS) -> ghist[bin * ntiles + tile]
//   (hipcub)      exclusive scan of ghist (bin-major) -> gbase
//   k_bs_coarse   per tile: LDS rank within (tile, bin) -> coarse-sorted keys/vals
//   k_bs_fine     one workgroup per coarse bin: LDS histogram over its 2^FB_BITS
//                 buckets, scan, counts/offsets out, scatter vals in bucket order
//
// Replaces the random-address global atomicAdd ranks of the first engine
// (~20 G atomics/s chip-wide, MI355X_MICROARCH.md "64 lanes in 64 different rows").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace msm {

constexpr int BS_TILE = 8192;      // entries per tile (256 threads x 32)
constexpr int BS_FB_BITS = 10;     // fine buckets per coarse bin = 1024
constexpr int BS_MAX_CB = 8192;    // coarse bins held in LDS (32 KiB): NB <= 2^23
constexpr uint32_t BS_NONE = 0xffffffffu;

static __global__ void __launch_bounds__(256)
    k_bs_hist(const uint32_t *__restrict__ keys, size_t ne, int ncb, int ntiles, uint32_t *__restrict__ ghist) {
  __shared__ uint32_t h[BS_MAX_CB];
  for (int b = threadIdx.x; b < ncb; b += blockDim.x) h[b] = 0;
  __syncthreads();
  const size_t t0 = (size_t)blockIdx.x * BS_TILE;
  const size_t t1 = t0 + BS_TILE < ne ? t0 + BS_TILE : ne;
  for (size_t e = t0 + threadIdx.x; e < t1; e += blockDim.x) {
    uint32_t k = keys[e];
    if (k != BS_NONE) atomicAdd(&h[k >> BS_FB_BITS], 1u);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < ncb; b += blockDim.x) ghist[(size_t)b * ntiles + blockIdx.x] = h[b];
}

static __global__ void __launch_bounds__(256)
    k_bs_coarse(const uint32_t *__restrict__ keys, const uint32_t *__restrict__ vals, size_t ne, int ncb, int ntiles,
                const uint32_t *__restrict__ gbase, uint32_t *__restrict__ okeys, uint32_t *__restrict__ ovals) {
  __shared__ uint32_t cur[BS_MAX_CB];
  for (int b = threadIdx.x; b < ncb; b += blockDim.x) cur[b] = gbase[(size_t)b * ntiles + blockIdx.x];
  __syncthreads();
  const size_t t0 = (size_t)blockIdx.x * BS_TILE;
  const size_t t1 = t0 + BS_TILE < ne ? t0 + BS_TILE : ne;
  for (size_t e = t0 + threadIdx.x; e < t1; e += blockDim.x) {
    uint32_t k = keys[e];
    if (k == BS_NONE) continue;
    uint32_t pos = atomicAdd(&cur[k >> BS_FB_BITS], 1u);
    okeys[pos] = k;
    ovals[pos] = vals[e];
  }
}

// bin b covers buckets [b << FB_BITS, (b+1) << FB_BITS) and coarse-sorted
// entries [gbase[b * ntiles], end_b) where end_b = gbase[(b+1) * ntiles] or total.
// sched_key[bucket] = min(count, 255) (the accumulation schedule sorts by it).
static __global__ void __launch_bounds__(512)
    k_bs_fine(const uint32_t *__restrict__ okeys, const uint32_t *__restrict__ ovals, int ncb, int ntiles,
              const uint32_t *__restrict__ gbase, const uint32_t *__restrict__ total, uint32_t nb,
              uint32_t *__restrict__ sorted, uint32_t *__restrict__ counts, uint32_t *__restrict__ offsets,
              uint32_t *__restrict__ sched_key) {
  constexpr int FB = 1 << BS_FB_BITS;
  __shared__ uint32_t cnt[FB];
  __shared__ uint32_t off[FB];
  const int b = blockIdx.x;
  const uint32_t lo = gbase[(size_t)b * ntiles];
  const uint32_t hi = b + 1 < ncb ? gbase[(size_t)(b + 1) * ntiles] : *total;
  for (int f = threadIdx.x; f < FB; f += blockDim.x) cnt[f] = 0;
  __syncthreads();
  for (uint32_t e = lo + threadIdx.x; e < hi; e += blockDim.x) atomicAdd(&cnt[okeys[e] & (FB - 1)], 1u);
  __syncthreads();
  // exclusive scan of cnt[0..FB) by one wave (FB = 1024 = 16 per lane)
  if (threadIdx.x < 64) {
    const int l = threadIdx.x;
    uint32_t loc[FB / 64], s = 0;
#pragma unroll
    for (int k = 0; k < FB / 64; ++k) {
      loc[k] = s;
      s += cnt[l * (FB / 64) + k];
    }
    uint32_t incl = s;  // wave-inclusive scan of the per-lane totals
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      uint32_t v = __shfl_up(incl, d, 64);
      if (l >= d) incl += v;
    }
    uint32_t base = incl - s;
#pragma unroll
    for (int k = 0; k < FB / 64; ++k) off[l * (FB / 64) + k] = base + loc[k];
  }
  __syncthreads();
  for (int f = threadIdx.x; f < FB; f += blockDim.x) {
    uint32_t bucket = ((uint32_t)b << BS_FB_BITS) + f;
    if (bucket < nb) {
      uint32_t c = cnt[f];
      counts[bucket] = c;
      offsets[bucket] = lo + off[f];
      sched_key[bucket] = c < 255u ? c : 255u;
    }
  }
  __syncthreads();
  for (uint32_t e = lo + threadIdx.x; e < hi; e += blockDim.x) {
    uint32_t k = okeys[e];
    uint32_t pos = atomicAdd(&off[k & (FB - 1)], 1u);
    sorted[lo + pos] = ovals[e];
  }
}

// total number of valid entries = inclusive end of the last (bin, tile) slot
static __global__ void k_bs_total(const uint32_t *__restrict__ gbase, const uint32_t *__restrict__ ghist, size_t nslots,
                           uint32_t *__restrict__ total) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *total = gbase[nslots - 1] + ghist[nslots - 1];
}

}  // namespace msm
