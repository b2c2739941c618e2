// bucket_sort.hpp -- two-level counting sort of MSM entries by bucket (gfx950).
//
// Input: one (key, val) per entry, key = bucket id < NB (or KEY_NONE = skip),
// val = payload (point/table slot | sign << 31).  Output: vals grouped by
// bucket and per-bucket counts and offsets.  All counting is in LDS; global
// memory only sees streaming reads and writes that are contiguous per
// (tile, coarse bin) or confined to one coarse bin's range:
//
//   k_bs_hist     per tile of TILE entries: LDS histogram over coarse bins
//                 (bucket >> fb_bits) -> ghist[bin * ntiles + tile]
//   (hipcub)      exclusive scan of ghist (bin-major) -> gbase
//   k_bs_coarse   per tile: LDS rank within (tile, bin) -> coarse-sorted keys/vals
//   k_bs_fine     one workgroup (1024 or 256 threads) per coarse bin: LDS histogram over
//                 its 2^fb_bits buckets, block scan, counts/offsets out, vals
//                 placed in bucket order in LDS windows and streamed out; also
//                 the accumulation schedule's class histogram
//   k_sched_scatter  bucket ids ordered by entry count (the schedule)
//
// Seven launches per sort including the digit kernel that feeds it (hist,
// two hipcub scan kernels, coarse, fine, scatter): every launch that runs
// beside a batch accumulation costs it ~10-20 us, so the total,
// the counter clears and the class scan ride in the kernels above instead of
// launches of their own.  Several independent sets (the MSMs of a batch front
// group, Ches::run_batch) sort in the same seven launches: blockIdx.y is the
// set, each set has its own ne input entries (keys + set ne), its own slots
// of the histogram (set-major, so ONE exclusive scan yields global offsets and
// the sets' outputs land consecutively in okeys / sorted), its own nb counts /
// offsets / order entries (offsets are global positions in `sorted`) and its
// own 512 class counters.
//
// fb_bits is chosen per problem so that there are ~256 coarse bins: few enough
// that a tile's writes to one bin form runs of tens of entries (the L2 merges
// them), many enough to fill the chip in k_bs_fine.  Replaces the random-
// address global atomicAdd ranks of the first engine (~20 G atomics/s
// chip-wide, MI355X_MICROARCH.md "64 lanes in 64 different rows").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace msm {

constexpr int BS_TILE = 4096;         // entries per tile (256 threads x 16; staged in 32 KiB of LDS)
constexpr int BS_MAX_FB_BITS = 12;    // fine buckets per coarse bin <= 4096 (2 x 16 KiB LDS)
constexpr int BS_MAX_CB = 8192;       // coarse bins held in LDS (32 KiB)
constexpr uint32_t BS_NONE = 0xffffffffu;
// accumulation schedule classes (see k_sched_scatter): class = 255 - min(count, 255)
constexpr int SCHED_PER_THREAD = 16;
constexpr int SCHED_PER_BLOCK = 256 * SCHED_PER_THREAD;
__device__ __forceinline__ uint32_t sched_class(uint32_t c) { return 255u - (c < 255u ? c : 255u); }

// Block 0 also clears the schedule's class counters (SCHED_WORDS words), which
// k_bs_fine and k_sched_scatter of this same sort use later in stream order.
static __global__ void __launch_bounds__(256)
    k_bs_hist(const uint32_t *__restrict__ keys, size_t ne, int fb_bits, int ncb, int ntiles,
              uint32_t *__restrict__ ghist, uint32_t *__restrict__ classes) {
  __shared__ uint32_t h[BS_MAX_CB];
  keys += (size_t)blockIdx.y * ne;
  ghist += (size_t)blockIdx.y * ncb * ntiles;
  if (blockIdx.x == 0)
    for (int c = threadIdx.x; c < 512; c += blockDim.x) classes[(size_t)blockIdx.y * 512 + c] = 0;
  for (int b = threadIdx.x; b < ncb; b += blockDim.x) h[b] = 0;
  __syncthreads();
  const size_t t0 = (size_t)blockIdx.x * BS_TILE;
  uint32_t kk[BS_TILE / 256];  // all of this thread's keys in flight at once
#pragma unroll
  for (int r = 0; r < BS_TILE / 256; ++r) {
    size_t e = t0 + threadIdx.x + (size_t)r * 256;
    kk[r] = e < ne ? keys[e] : BS_NONE;
  }
#pragma unroll
  for (int r = 0; r < BS_TILE / 256; ++r)
    if (kk[r] != BS_NONE) atomicAdd(&h[kk[r] >> fb_bits], 1u);
  __syncthreads();
  for (int b = threadIdx.x; b < ncb; b += blockDim.x) ghist[(size_t)b * ntiles + blockIdx.x] = h[b];
}

// exclusive scan of a[0..n) in LDS by a 256-thread block (n <= 256 * 32);
// returns the total.  wsum: 4 words of LDS scratch.
__device__ __forceinline__ uint32_t block_exclusive_scan_256(uint32_t *a, int n, uint32_t *wsum) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int per = (n + 255) / 256, lo = t * per, hi = min(n, lo + per);
  uint32_t s = 0;
  for (int i = lo; i < hi; ++i) s += a[i];
  uint32_t incl = s;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t v = __shfl_up(incl, d, 64);
    if (lane >= d) incl += v;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  uint32_t before = 0, total = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    before += w < wave ? wsum[w] : 0u;
    total += wsum[w];
  }
  uint32_t run = before + incl - s;
  for (int i = lo; i < hi; ++i) {
    uint32_t x = a[i];
    a[i] = run;
    run += x;
  }
  __syncthreads();
  return total;
}

// Per tile: rank the entries by coarse bin in LDS, stage the tile bin-sorted in
// LDS, then stream it out so that consecutive lanes write consecutive addresses
// of a bin's run (coalesced), instead of 64 lanes writing 64 different bins.
// Dynamic LDS: 2 ncb + 2 BS_TILE words.
static __global__ void __launch_bounds__(256)
    k_bs_coarse(const uint32_t *__restrict__ keys, const uint32_t *__restrict__ vals, size_t ne, int fb_bits,
                int ncb, int ntiles, const uint32_t *__restrict__ gbase, uint32_t *__restrict__ okeys,
                uint32_t *__restrict__ ovals) {
  extern __shared__ uint32_t sm[];
  __shared__ uint32_t wsum[4];
  uint32_t *loff = sm, *gb = sm + ncb, *sk = sm + 2 * ncb, *sv = sk + BS_TILE;
  keys += (size_t)blockIdx.y * ne;
  vals += (size_t)blockIdx.y * ne;
  gbase += (size_t)blockIdx.y * ncb * ntiles;
  for (int b = threadIdx.x; b < ncb; b += blockDim.x) {
    loff[b] = 0;
    gb[b] = gbase[(size_t)b * ntiles + blockIdx.x];
  }
  __syncthreads();
  const size_t t0 = (size_t)blockIdx.x * BS_TILE;
  constexpr int R = BS_TILE / 256;
  uint32_t kk[R], vv[R], rk[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    size_t e = t0 + threadIdx.x + (size_t)r * 256;
    kk[r] = e < ne ? keys[e] : BS_NONE;
    vv[r] = e < ne ? vals[e] : 0u;
  }
#pragma unroll
  for (int r = 0; r < R; ++r) rk[r] = kk[r] != BS_NONE ? atomicAdd(&loff[kk[r] >> fb_bits], 1u) : 0u;
  __syncthreads();
  const uint32_t total = block_exclusive_scan_256(loff, ncb, wsum);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (kk[r] == BS_NONE) continue;
    const uint32_t pos = loff[kk[r] >> fb_bits] + rk[r];
    sk[pos] = kk[r];
    sv[pos] = vv[r];
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < total; i += 256) {
    const uint32_t k = sk[i], b = k >> fb_bits;
    const uint32_t g = gb[b] + (i - loff[b]);
    okeys[g] = k;
    ovals[g] = sv[i];
  }
}

// exclusive scan of a[0..n) in LDS by a BT-thread block (n <= 4096, so at most
// 4096 / BT consecutive elements per thread); wsum: BT / 64 words of LDS
template <int BT>
__device__ __forceinline__ void block_exclusive_scan_4096(uint32_t *a, int n, uint32_t *wsum) {
  constexpr int PER = 4096 / BT, NW = BT / 64;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int per = (n + BT - 1) / BT;
  uint32_t loc[PER], s = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    int i = t * per + k;
    loc[k] = s;
    if (k < per && i < n) s += a[i];
  }
  uint32_t incl = s;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t v = __shfl_up(incl, d, 64);
    if (lane >= d) incl += v;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  if (t == 0) {
    uint32_t run = 0;
    for (int w = 0; w < NW; ++w) {
      uint32_t x = wsum[w];
      wsum[w] = run;
      run += x;
    }
  }
  __syncthreads();
  const uint32_t base = wsum[wave] + incl - s;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    int i = t * per + k;
    if (k < per && i < n) a[i] = base + loc[k];
  }
  __syncthreads();
}

// bin b covers buckets [b << fb_bits, (b+1) << fb_bits) and coarse-sorted
// entries [gbase[b * ntiles], end_b) where end_b = gbase[(b+1) * ntiles] or total.
//
// The bin's output range (~50k entries) is written through an LDS staging
// buffer in windows of <= BS_FINE_CAP entries: window k holds the fine buckets
// whose exclusive offset lies in [k C, (k+1) C), C = BS_FINE_STEP.  Each
// window re-reads the bin's keys (L2/MALL-resident), places its entries in LDS
// and streams the window out with consecutive lanes on consecutive addresses.
// Scattering 4-B values straight to global memory left every 128-B line
// partially written several times over (0.24 ms at 2^20 CHES vs 0.07 staged).
// An entry past the window's LDS capacity (one bucket heavier than the slack)
// is written directly; a bin needing more than BS_FINE_MAXW windows
// (degenerate inputs) is scattered directly as a whole.
constexpr int BS_FINE_CAP = 30 * 1024;                        // staged entries (120 KiB)
constexpr int BS_FINE_STEP = BS_FINE_CAP - BS_FINE_CAP / 8;   // window stride, leaves slack
constexpr int BS_FINE_MAXW = 8;

//
// BT = threads per workgroup: 1024 (the default everywhere).  256 (one wave
// per SIMD, 56 VGPRs) fits beside three k_accumulate waves per SIMD, so a batch
// front dispatched under an accumulation need not wait for a CU to drain; it
// measured slower in the batch (Ches::run_jobs, MSM_FINE_BT).
template <int BT>
static __global__ void __launch_bounds__(BT)
    k_bs_fine(const uint32_t *__restrict__ okeys, const uint32_t *__restrict__ ovals, int fb_bits, int ncb,
              int ntiles, const uint32_t *__restrict__ gbase, const uint32_t *__restrict__ ghist, uint32_t nb,
              uint32_t *__restrict__ sorted, uint32_t *__restrict__ counts, uint32_t *__restrict__ offsets,
              uint32_t *__restrict__ class_total, int nsets) {
  __shared__ uint32_t off[1 << BS_MAX_FB_BITS];
  __shared__ uint8_t win[1 << BS_MAX_FB_BITS];
  __shared__ uint32_t stage[BS_FINE_CAP];
  __shared__ uint32_t wsum[BT / 64];
  __shared__ uint32_t wb[BS_FINE_MAXW + 1];
  __shared__ uint32_t cls[256];
  const int FB = 1 << fb_bits;
  const uint32_t fmask = (uint32_t)FB - 1u;
  const int b = blockIdx.x, set = blockIdx.y;
  const size_t per = (size_t)ncb * ntiles, s0 = (size_t)set * per;
  const size_t last = (size_t)nsets * per - 1;  // the last (set, bin, tile) slot ends the valid entries
  const uint32_t lo = gbase[s0 + (size_t)b * ntiles];
  const uint32_t hi = b + 1 < ncb ? gbase[s0 + (size_t)(b + 1) * ntiles]
                                  : (set + 1 < nsets ? gbase[s0 + per] : gbase[last] + ghist[last]);
  counts += (size_t)set * nb;
  offsets += (size_t)set * nb;
  class_total += (size_t)set * 512;
  const uint32_t nbin = hi - lo;
  for (int f = threadIdx.x; f < FB; f += blockDim.x) off[f] = 0;
  for (int c = threadIdx.x; c < 256; c += BT) cls[c] = 0;
  if (threadIdx.x <= BS_FINE_MAXW) wb[threadIdx.x] = nbin;
  __syncthreads();
  constexpr int U = 16, UW = 12;  // loads in flight per thread (histogram / window passes)
  for (uint32_t e0 = lo; e0 < hi; e0 += U * BT) {
    uint32_t kk[U];
#pragma unroll
    for (int r = 0; r < U; ++r) {
      uint32_t e = e0 + threadIdx.x + r * BT;
      kk[r] = e < hi ? okeys[e] : BS_NONE;
    }
#pragma unroll
    for (int r = 0; r < U; ++r)
      if (kk[r] != BS_NONE) atomicAdd(&off[kk[r] & fmask], 1u);
  }
  __syncthreads();
  for (int f = threadIdx.x; f < FB; f += blockDim.x) {
    uint32_t bucket = ((uint32_t)b << fb_bits) + f;
    if (bucket < nb) {
      counts[bucket] = off[f];
      atomicAdd(&cls[sched_class(off[f])], 1u);  // the schedule's class histogram (was k_sched_hist)
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 256; c += BT)
    if (cls[c]) atomicAdd(&class_total[c], cls[c]);
  block_exclusive_scan_4096<BT>(off, FB, wsum);
  const uint32_t nwin = (nbin + BS_FINE_STEP - 1) / BS_FINE_STEP;
  const bool staged = nwin <= (uint32_t)BS_FINE_MAXW;
  for (int f = threadIdx.x; f < FB; f += blockDim.x) {
    uint32_t bucket = ((uint32_t)b << fb_bits) + f;
    if (bucket < nb) offsets[bucket] = lo + off[f];
    if (staged) {
      uint32_t w = off[f] / BS_FINE_STEP;
      win[f] = (uint8_t)w;
      atomicMin(&wb[w], off[f]);  // window base = smallest offset in it
    }
  }
  __syncthreads();
  if (!staged) {
    for (uint32_t e0 = lo; e0 < hi; e0 += U * BT) {
      uint32_t kk[U], vv[U];
#pragma unroll
      for (int r = 0; r < U; ++r) {
        uint32_t e = e0 + threadIdx.x + r * BT;
        kk[r] = e < hi ? okeys[e] : BS_NONE;
        vv[r] = e < hi ? ovals[e] : 0u;
      }
#pragma unroll
      for (int r = 0; r < U; ++r) {
        if (kk[r] == BS_NONE) continue;
        uint32_t pos = atomicAdd(&off[kk[r] & fmask], 1u);
        sorted[lo + pos] = vv[r];
      }
    }
    return;
  }
  for (uint32_t k = 0; k < nwin; ++k) {
    const uint32_t base = wb[k];
    if (base == nbin) continue;  // empty window (a heavy bucket spans it)
    uint32_t end = nbin;
    for (uint32_t j = k + 1; j < nwin; ++j)
      if (wb[j] < end) end = wb[j];
    for (uint32_t e0 = lo; e0 < hi; e0 += UW * BT) {
      // keys and vals in one round trip (a dependent vals load per key would
      // double the latency-bound passes); vals of other windows are re-read
      uint32_t kk[UW], vv[UW];
#pragma unroll
      for (int r = 0; r < UW; ++r) {
        uint32_t e = e0 + threadIdx.x + r * BT;
        kk[r] = e < hi ? okeys[e] : BS_NONE;
        vv[r] = e < hi ? ovals[e] : 0u;
      }
#pragma unroll
      for (int r = 0; r < UW; ++r) {
        if (kk[r] == BS_NONE || win[kk[r] & fmask] != k) continue;
        uint32_t li = atomicAdd(&off[kk[r] & fmask], 1u) - base;
        if (li < (uint32_t)BS_FINE_CAP)
          stage[li] = vv[r];
        else
          sorted[lo + base + li] = vv[r];
      }
    }
    __syncthreads();
    const uint32_t nst = min(end - base, (uint32_t)BS_FINE_CAP);
    for (uint32_t i = threadIdx.x; i < nst; i += BT) sorted[lo + base + i] = stage[i];
    __syncthreads();
  }
}

// ---- accumulation schedule: bucket ids ordered by entry count, descending ----
// class = 255 - min(count, 255).  k_bs_fine accumulates the per-class totals
// (an LDS histogram per coarse bin, one global atomic per non-empty class and
// bin).  k_sched_scatter: every workgroup scans the 256 class totals in LDS
// (exclusive class bases), reserves its per-class ranges with one global
// atomic per class on the cursors class_total[256 + c], and writes its bucket
// ids.  The order inside a class is arbitrary.  A block covers 4096 buckets so
// that the ~20 busy class cursors see a few hundred atomics, not one per 256
// buckets (a single address saturates at ~88 atomics/us, MI355X_MICROARCH.md).
// The bucket's count and payload offset are written beside its id in schedule
// order (scnt / soff), so the accumulation reads them coalesced by lane instead
// of two random 4-B loads (two 64-B lines) per bucket.
static __global__ void __launch_bounds__(256, 6)  // <= 80 VGPRs: fits beside three k_accumulate waves per SIMD
    k_sched_scatter(const uint32_t *__restrict__ counts, const uint32_t *__restrict__ offsets, uint32_t nb,
                    uint32_t *__restrict__ class_total, uint32_t *__restrict__ order, uint32_t *__restrict__ scnt,
                    uint32_t *__restrict__ soff) {
  __shared__ uint32_t h[256];
  __shared__ uint32_t base[256];
  __shared__ uint32_t wsum[4];
  counts += (size_t)blockIdx.y * nb;
  offsets += (size_t)blockIdx.y * nb;
  order += (size_t)blockIdx.y * nb;
  scnt += (size_t)blockIdx.y * nb;
  soff += (size_t)blockIdx.y * nb;
  class_total += (size_t)blockIdx.y * 512;
  const uint32_t t = threadIdx.x, b0 = blockIdx.x * SCHED_PER_BLOCK, lane = t & 63, wave = t >> 6;
  h[t] = 0;
  // exclusive scan of the class totals: one value per thread, wave scans + 4 wave sums
  const uint32_t v = class_total[t];
  uint32_t incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t u = __shfl_up(incl, d, 64);
    if (lane >= (uint32_t)d) incl += u;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  uint32_t cbase = incl - v;
  for (uint32_t w = 0; w < wave; ++w) cbase += wsum[w];
  uint32_t rank[SCHED_PER_THREAD], cnt[SCHED_PER_THREAD];  // (the class is recomputed from the count)
#pragma unroll
  for (int r = 0; r < SCHED_PER_THREAD; ++r) {
    const uint32_t b = b0 + r * 256 + t;
    cnt[r] = b < nb ? counts[b] : 0u;
    rank[r] = b < nb ? atomicAdd(&h[sched_class(cnt[r])], 1u) : 0u;
  }
  __syncthreads();
  if (h[t]) base[t] = cbase + atomicAdd(&class_total[256 + t], h[t]);
  __syncthreads();
#pragma unroll
  for (int r = 0; r < SCHED_PER_THREAD; ++r) {
    const uint32_t b = b0 + r * 256 + t;
    if (b < nb) {
      const uint32_t pos = base[sched_class(cnt[r])] + rank[r];
      order[pos] = b;
      scnt[pos] = cnt[r];
      soff[pos] = offsets[b];
    }
  }
}

// Interleaved payload.  The 64 lanes of an accumulation wave walk 64 buckets
// of nearly equal count (the schedule above); with the payload in bucket order
// step k of the wave reads 64 scattered 4-B entries -- 64 line fetches, the
// lines evicted (by the point loads) before step k + 1.  Wave group w of 64
// schedule positions instead gets a block of head(w) rows of 64 entries, head
// = the count at its first position (the largest: the schedule is sorted by
// exact count below 255); row k holds entry k of each of its buckets, so step
// k is one coalesced 256-B read.  Groups that start inside class 0 (counts >=
// 255, not sorted) keep the bucket-ordered payload (wbase = ~0).  The blocks
// need no scan: the count at a position follows from the class totals, so
// group w's first row is sum over the earlier interleaved groups of their
// heads, computed per class from the totals in LDS.  Size: head(w) <= the
// smallest count of group w - 1, so the rows of all groups but the first fit
// in the entries of their predecessors: <= ne + 64 * 255 per set.
constexpr size_t BS_IPAY_SLACK = 64 * 256;
static __global__ void __launch_bounds__(256)
    k_interleave(const uint32_t *__restrict__ scnt, const uint32_t *__restrict__ soff, uint32_t nb, uint32_t nw,
                 const uint32_t *__restrict__ class_total, const uint32_t *__restrict__ sorted,
                 uint32_t *__restrict__ ipay, size_t ipay_stride, uint32_t *__restrict__ wbase) {
  __shared__ uint32_t ct[256], hs[256], wsum[4];
  const size_t set = blockIdx.y;
  const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const uint32_t tot = class_total[set * 512 + t];
  // exclusive scan of the class totals (class order = position order)
  uint32_t incl = tot;
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t u = __shfl_up(incl, d, 64);
    if (lane >= (uint32_t)d) incl += u;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  uint32_t c0 = incl - tot;
  for (uint32_t w = 0; w < wave; ++w) c0 += wsum[w];
  ct[t] = c0;
  __syncthreads();
  const uint32_t t0r = (ct[1] + 63) & ~63u;  // first interleaved position (class 0 = ct[0] .. ct[1])
  // heads of class t: multiples of 64 in [max(ct, t0r), ct + tot), each a row block of 255 - t rows
  const uint32_t lo = max(c0, t0r), hi = c0 + tot;
  const uint32_t contrib = (t > 0 && lo < hi) ? (255u - t) * (((hi + 63) >> 6) - ((lo + 63) >> 6)) : 0u;
  __syncthreads();
  incl = contrib;
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t u = __shfl_up(incl, d, 64);
    if (lane >= (uint32_t)d) incl += u;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  uint32_t h0 = incl - contrib;
  for (uint32_t w = 0; w < wave; ++w) h0 += wsum[w];
  hs[t] = h0;
  __syncthreads();
  const uint32_t p = blockIdx.x * 256 + t;
  const uint32_t g = p >> 6, head = g << 6;
  uint32_t base = ~0u;
  if (head >= t0r && head < nb) {
    // class of the head position: the last c with ct[c] <= head (empty classes
    // share ct with their successor, so the last such c is non-empty)
    uint32_t c = 0;
    for (uint32_t step = 128; step; step >>= 1)
      if (ct[c + step] <= head) c += step;
    const uint32_t first = max(ct[c], t0r);
    base = hs[c] + (255u - c) * ((head >> 6) - ((first + 63) >> 6));
  }
  if (lane == 0 && g < nw) wbase[set * nw + g] = base;
  if (base == ~0u || p >= nb) return;
  const uint32_t n = scnt[set * nb + p], o = soff[set * nb + p];
  uint32_t *dst = ipay + set * ipay_stride + (size_t)base * 64 + lane;
  const uint32_t *src = sorted + o;
  uint32_t k = 0;
  for (; k + 4 <= n; k += 4) {  // four loads in flight per lane
    const uint32_t a = src[k], b = src[k + 1], c = src[k + 2], d = src[k + 3];
    dst[(size_t)k * 64] = a;
    dst[(size_t)(k + 1) * 64] = b;
    dst[(size_t)(k + 2) * 64] = c;
    dst[(size_t)(k + 3) * 64] = d;
  }
  for (; k < n; ++k) dst[(size_t)k * 64] = src[k];
}

}  // namespace msm
