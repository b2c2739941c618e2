// compat.hip -- the blst-level CHES / BGMW95 tile entry points of the
// reference (bindings/blst.h:255-357, src/multi_scalar.c:421-547, 609-790) on
// the GPU, for callers that drive the CHES loops themselves (ref main_p1.cpp
// :233-236, :279-282, :384) instead of using the device-resident contexts.
//
// Each tile call is one "entry MSM": host arrays of (point, bucket, sign)
// entries -> device: points converted once, BucketSort by bucket,
// k_accumulate (one lane per bucket), optional export of the bucket sums back
// into the caller's blst_p*xyzz buckets[] (the reference leaves them filled),
// WeightedReducer for sum_b w_b S_b.  Reference weights: bucket_set_ascend[idx]
// (d_CHES), the bucket value itself (noindexhash, BGMW95).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>

#include "ches_kernels.hpp"
#include "engine.hpp"
#include "heavy.hpp"
#include "hoststage.hpp"
#include "pair_kernels.hpp"
#include "pool.hpp"
#include "table_registry.hpp"

#ifndef MSM_GROUP
#error "define MSM_GROUP (1 or 2)"
#endif

namespace msm {

// page-locked host staging of the pointer-array tiles (entry_msm_ptrs)
struct PinnedBuf {
  void *p = nullptr;
  size_t bytes = 0;
  PinnedBuf() = default;
  PinnedBuf(const PinnedBuf &) = delete;
  PinnedBuf &operator=(const PinnedBuf &) = delete;
  ~PinnedBuf() {
    if (p) (void)hipHostFree(p);
  }
  void ensure(size_t b) {  // callers synchronise the stream that reads it first
    if (b <= bytes) return;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    bytes = 0;
    MSM_HIP_CHECK(hipHostMalloc(&p, b, hipHostMallocDefault));
    bytes = b;
  }
  template <class T>
  T *as() const {
    return reinterpret_cast<T *>(p);
  }
};

template <int G>
struct EntryMsmState {
  DevBuf pts, keys, vals, sorted, counts, offsets, order, buckets, xfer, bx;
  BucketSort sort;
  WeightedReducer<G> red;
  std::vector<uint32_t> planned;  // weights the reducer plan was built for
  PinnedBuf hkv, hring, hbx;      // pinned: keys + vals, the point-row ring, exported buckets
  HeavyScratch heavy;             // heavy buckets split over several lanes (heavy.hpp)
  hipEvent_t ring_ev[4] = {};
  hipStream_t up = nullptr;  // row uploads: beside the sort on the lease's stream
  hipEvent_t up_ev = nullptr;
  ~EntryMsmState() {
    for (hipEvent_t &e : ring_ev)
      if (e) (void)hipEventDestroy(e);
    if (up_ev) (void)hipEventDestroy(up_ev);
    if (up) (void)hipStreamDestroy(up);
  }
  size_t device_bytes() const {  // device buffers + pinned staging (the pool's idle budget counts both)
    size_t b = hkv.bytes + hring.bytes + hbx.bytes;
    for (const DevBuf *d : {&pts, &keys, &vals, &sorted, &counts, &offsets, &order, &buckets, &xfer, &bx}) b += d->bytes;
    return b + sort.device_bytes() + red.device_bytes() + heavy.device_bytes();
  }
};

// pooled per device (pool.hpp): concurrent tile calls each lease their own state
template <int G>
static std::unique_ptr<typename EnginePool<EntryMsmState<G>>::Lease> entry_state() {
  int dev = 0;
  MSM_HIP_CHECK(hipGetDevice(&dev));
  return EnginePool<EntryMsmState<G>>::get().lease(dev, 0, [] { return std::make_unique<EntryMsmState<G>>(); });
}

template <int G>
static void plan_if_changed(EntryMsmState<G> &S, const uint32_t *w, size_t nb) {
  if (S.planned.size() == nb && std::equal(w, w + nb, S.planned.begin())) return;
  S.planned.assign(w, w + nb);
  S.red.plan(S.planned);
}

// MSM_TILE_TIMING=1: host-side phase times of each pointer-array tile call on
// stderr (study knob for the per-call fixed cost)
struct TileClock {
  bool on;
  std::chrono::steady_clock::time_point t0, t;
  std::string line;
  TileClock() {
    static const bool env = [] {
      const char *e = getenv("MSM_TILE_TIMING");
      return e && atoi(e) != 0;
    }();
    on = env;
    t0 = t = std::chrono::steady_clock::now();
  }
  void lap(const char *what) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    char b[64];
    snprintf(b, sizeof b, " %s=%.3f", what, std::chrono::duration<double, std::milli>(n - t).count());
    line += b;
    t = n;
  }
  ~TileClock() {
    if (on)
      fprintf(stderr, "[tile] total=%.3f ms:%s\n",
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(), line.c_str());
  }
};

template <int G, class PT>
static void entry_msm_back(EntryMsmState<G> &S, hipStream_t s, const PT *pts, void *ret, size_t ne, size_t nb,
                           const uint32_t *weights, void *buckets_out, bool pinned_export, TileClock *clk = nullptr,
                           bool presorted = false);

// bucket sort of the entries in S.keys / S.vals (counts, offsets, schedule)
template <int G>
static void entry_sort(EntryMsmState<G> &S, hipStream_t s, size_t ne, size_t nb) {
  S.counts.ensure(nb * 4);
  S.offsets.ensure(nb * 4);
  S.order.ensure(nb * 4);
  S.sort.run(s, S.keys.template as<uint32_t>(), S.vals.template as<uint32_t>(), ne, (uint32_t)nb,
             S.sorted.template as<uint32_t>(), S.counts.template as<uint32_t>(), S.offsets.template as<uint32_t>(),
             S.order.template as<uint32_t>());
}

template <int G>
void entry_msm(void *ret, const void *pts_blst, size_t npts, const uint32_t *keys, const uint32_t *vals, size_t ne,
               size_t nb, const uint32_t *weights, void *buckets_out) {
  typedef typename FieldOf<G>::F F;
  typedef typename HostField<G>::F HF;
  hfp::Jac<HF> out;
  std::memset(&out, 0, sizeof out);
  if (nb == 0) {
    std::memcpy(ret, &out, sizeof out);
    return;
  }
  auto lease = entry_state<G>();
  EntryMsmState<G> &S = **lease;
  hipStream_t s = lease->stream();
  if (ne >= (1ull << 31) || npts >= (1ull << 31)) throw std::runtime_error("entry MSM too large");
  S.xfer.ensure(std::max<size_t>(npts * 96 * G, 16));
  S.pts.ensure(std::max<size_t>(npts, 1) * sizeof(Aff<F>));
  if (npts) {
    MSM_HIP_CHECK(hipMemcpyAsync(S.xfer.p, pts_blst, npts * 96 * G, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_convert_points<G>, dim3(nblk(npts, 256)), dim3(256), 0, s, S.xfer.template as<uint64_t>(),
                       S.pts.template as<Aff<F>>(), npts);
    MSM_HIP_CHECK(hipGetLastError());
  }
  S.keys.ensure(std::max<size_t>(ne, 1) * 4);
  S.vals.ensure(std::max<size_t>(ne, 1) * 4);
  S.sorted.ensure(std::max<size_t>(ne, 1) * 4 + 64);  // + the accumulation's payload window
  if (ne) {
    MSM_HIP_CHECK(hipMemcpyAsync(S.keys.p, keys, ne * 4, hipMemcpyHostToDevice, s));
    MSM_HIP_CHECK(hipMemcpyAsync(S.vals.p, vals, ne * 4, hipMemcpyHostToDevice, s));
  }
  entry_msm_back<G>(S, s, S.pts.template as<Aff<F>>(), ret, ne, nb, weights, buckets_out, false);
}

// sort + accumulate + (bucket export) + weighted reduction of the entries in
// S.keys / S.vals over the point rows pts (S.pts, or a registered table)
template <int G, class PT>
static void entry_msm_back(EntryMsmState<G> &S, hipStream_t s, const PT *pts, void *ret, size_t ne, size_t nb,
                           const uint32_t *weights, void *buckets_out, bool pinned_export, TileClock *clk,
                           bool presorted) {
  typedef typename FieldOf<G>::F F;
  typedef typename HostField<G>::F HF;
  hfp::Jac<HF> out;
  S.buckets.ensure(nb * sizeof(Xyzz<F>));
  if (!presorted) entry_sort(S, s, ne, nb);
  // the caller's entries as they come: the CHES top digit's few buckets hold
  // n entries between them, so heavy buckets are split over several lanes
  launch_accumulate_heavy<G>(s, S.sort.sched(S.order.template as<uint32_t>(), S.sorted.template as<uint32_t>(), 0, nb),
                             pts, S.buckets.template as<Xyzz<F>>(), nb, S.heavy);
  MSM_HIP_CHECK(hipGetLastError());
  plan_if_changed(S, weights, nb);
  S.red.launch(s, S.buckets.p);
  if (buckets_out) {
    S.bx.ensure(nb * 192 * G);
    hipLaunchKernelGGL(k_export_xyzz<G>, dim3(nblk(nb, 256)), dim3(256), 0, s, S.buckets.template as<Xyzz<F>>(),
                       S.bx.template as<uint64_t>(), nb);
    MSM_HIP_CHECK(hipGetLastError());
    if (pinned_export) {  // DMA into page-locked memory, then a parallel copy into the caller's buckets
      S.hbx.ensure(nb * 192 * G);
      MSM_HIP_CHECK(hipMemcpyAsync(S.hbx.p, S.bx.p, nb * 192 * G, hipMemcpyDeviceToHost, s));
    } else {
      MSM_HIP_CHECK(hipMemcpyAsync(buckets_out, S.bx.p, nb * 192 * G, hipMemcpyDeviceToHost, s));
    }
  }
  if (clk) clk->lap("enqueue");
  out = S.red.read(s);
  if (clk) clk->lap("gpu");
  if (buckets_out && pinned_export) parallel_memcpy(buckets_out, S.hbx.p, nb * 192 * G);
  if (clk) clk->lap("export");
  std::memcpy(ret, &out, sizeof out);
}

template <int G>
void entry_msm_ptrs(void *ret, const void *const *points, size_t ne, EntryFill fill, void *fill_ctx, size_t nb,
                    const uint32_t *weights, void *buckets_out) {
  typedef typename FieldOf<G>::F F;
  typedef typename HostField<G>::F HF;
  if (nb == 0 || ne == 0) {
    hfp::Jac<HF> out;
    std::memset(&out, 0, sizeof out);
    if (ne == 0 && nb && buckets_out) std::memset(buckets_out, 0, nb * 192 * G);
    std::memcpy(ret, &out, sizeof out);
    return;
  }
  if (ne >= (1ull << 31)) throw std::runtime_error("entry MSM too large");
  TileClock clk;
  auto lease = entry_state<G>();
  EntryMsmState<G> &S = **lease;
  hipStream_t s = lease->stream();
  MSM_HIP_CHECK(hipStreamSynchronize(s));  // the pinned buffers are free (no DMA of an earlier call pending)
  clk.lap("lease");
  const size_t psz = 96 * G;
  // keys / vals: filled in parallel straight into pinned memory, one DMA each
  S.hkv.ensure(ne * 8);
  uint32_t *hk = S.hkv.template as<uint32_t>(), *hv = hk + ne;
  const size_t piece = std::max<size_t>((size_t)1 << 16, (ne + 63) / 64);
  WorkerPool::get().parallel_for((ne + piece - 1) / piece, [&](size_t c) {
    const size_t t0 = c * piece, t1 = std::min(ne, t0 + piece);
    fill(fill_ctx, t0, t1, hk + t0, hv + t0);
  });
  clk.lap("fill");
  // a registered table holding every pointed-to row: vals become row indices
  // (sign bit kept) and no row is gathered (table_registry.hpp)
  int dev = 0;
  MSM_HIP_CHECK(hipGetDevice(&dev));
  std::shared_ptr<HostTable> tab = TableRegistry::get().find(G, dev, points[0]);
  if (tab) tab = fresh<G>(tab, 0, tab->nrows - 1);  // rows edited since registration: re-uploaded
  if (tab) {
    std::atomic<bool> outside{false};
    const uint8_t *base = tab->base;
    const size_t span = tab->nrows * psz;
    WorkerPool::get().parallel_for((ne + piece - 1) / piece, [&](size_t c) {
      const size_t t0 = c * piece, t1 = std::min(ne, t0 + piece);
      for (size_t t = t0; t < t1; ++t) {
        const size_t off = (size_t)(static_cast<const uint8_t *>(points[t]) - base);
        if (off >= span || off % psz) {
          outside.store(true, std::memory_order_relaxed);
          return;
        }
        hv[t] = (uint32_t)(off / psz) | (hv[t] & 0x80000000u);
      }
    });
    if (outside.load()) {  // back to entry indices (vals were t | sign) and the gather
      WorkerPool::get().parallel_for((ne + piece - 1) / piece, [&](size_t c) {
        const size_t t0 = c * piece, t1 = std::min(ne, t0 + piece);
        for (size_t t = t0; t < t1; ++t) hv[t] = (uint32_t)t | (hv[t] & 0x80000000u);
      });
      tab.reset();
    }
  }
  S.keys.ensure(ne * 4);
  S.vals.ensure(ne * 4);
  S.sorted.ensure(ne * 4 + 64);  // + the accumulation's payload window
  MSM_HIP_CHECK(hipMemcpyAsync(S.keys.p, hk, ne * 4, hipMemcpyHostToDevice, s));
  MSM_HIP_CHECK(hipMemcpyAsync(S.vals.p, hv, ne * 4, hipMemcpyHostToDevice, s));
  clk.lap("rows");
  if (tab) {
    entry_msm_back<G>(S, s, tab->rows.template as<AffP<F>>(), ret, ne, nb, weights, buckets_out, true, &clk);
    return;
  }
  // the sort needs only keys / vals: it runs on the GPU while the host gathers
  entry_sort(S, s, ne, nb);
  // point rows: gathered chunk by chunk into a 4-slot pinned ring (the host
  // gather of chunk c + 1 overlaps the DMA of chunk c), uploaded and converted
  // on a second stream (not queued behind the sort), which the accumulation
  // waits for.  4 slots of at most 32 MiB: the ring is 128 MiB of page-locked
  // memory whatever ne (ne / 16 rows per slot kept ~300 MB / 600 MB pinned per
  // pooled state for a 2^20 G1 / G2 tile); smaller slots made the
  // host wait for the DMA more often (8 MiB: 2^16 tile 5.77 vs 5.46 ms, 2^20
  // 53 vs 50 ms; profiles/r05_tile_timing.txt).  The upload stream needs no
  // wait on the lease's stream: the lease synchronised it above, and a copy
  // enqueued behind a cross-stream wait can block the host
  // (profiles/r05_h2d_block.txt).
  constexpr int kSlots = 4;
  if (!S.up) {
    MSM_HIP_CHECK(hipStreamCreateWithFlags(&S.up, hipStreamNonBlocking));
    MSM_HIP_CHECK(hipEventCreateWithFlags(&S.up_ev, hipEventDisableTiming));
  }
  static const size_t kRingSlotBytes = [] {  // A/B knob MSM_RING_SLOT_MIB
    const char *e = getenv("MSM_RING_SLOT_MIB");
    return (size_t)(e ? std::max(1, std::min(64, atoi(e))) : 32) << 20;
  }();
  static const size_t kGatherAhead = [] {  // A/B knob MSM_GATHER_AHEAD (rows; 0: no prefetch)
    const char *e = getenv("MSM_GATHER_AHEAD");
    return (size_t)(e ? std::max(0, std::min(256, atoi(e))) : 16);
  }();
  const size_t chunk = std::min(ne, (kRingSlotBytes) / psz);
  S.hring.ensure(chunk * psz * kSlots);
  for (hipEvent_t &e : S.ring_ev)
    if (!e) MSM_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  S.xfer.ensure(ne * psz);
  S.pts.ensure(ne * sizeof(Aff<F>));
  bool used[kSlots] = {};
  for (size_t c0 = 0, k = 0; c0 < ne; c0 += chunk, k = (k + 1) % kSlots) {
    const size_t cnt = std::min(chunk, ne - c0);
    if (used[k]) MSM_HIP_CHECK(hipEventSynchronize(S.ring_ev[k]));
    uint8_t *slot = S.hring.template as<uint8_t>() + k * chunk * psz;
    const size_t sub = std::max<size_t>(4096, (cnt + 15) / 16);
    WorkerPool::get().parallel_for((cnt + sub - 1) / sub, [&](size_t j) {
      const size_t a = j * sub, b = std::min(cnt, a + sub);
      // random row reads: prefetch kGatherAhead rows ahead (both 64-B lines of
      // a G1 row) to keep more DRAM misses in flight per thread
      for (size_t t = a; t < b; ++t) {
        if (kGatherAhead && t + kGatherAhead < b) {
          const char *q = static_cast<const char *>(points[c0 + t + kGatherAhead]);
          for (size_t l = 0; l < psz; l += 64) __builtin_prefetch(q + l);
        }
        std::memcpy(slot + t * psz, points[c0 + t], psz);
      }
    });
    MSM_HIP_CHECK(hipMemcpyAsync(S.xfer.template as<uint8_t>() + c0 * psz, slot, cnt * psz, hipMemcpyHostToDevice, S.up));
    MSM_HIP_CHECK(hipEventRecord(S.ring_ev[k], S.up));
    used[k] = true;
    // convert this chunk while the next one is gathered and copied
    hipLaunchKernelGGL(k_convert_points<G>, dim3(nblk(cnt, 256)), dim3(256), 0, S.up,
                       S.xfer.template as<uint64_t>() + c0 * (psz / 8), S.pts.template as<Aff<F>>() + c0, cnt);
    MSM_HIP_CHECK(hipGetLastError());
  }
  MSM_HIP_CHECK(hipEventRecord(S.up_ev, S.up));
  MSM_HIP_CHECK(hipStreamWaitEvent(s, S.up_ev, 0));
  clk.lap("gather");
  entry_msm_back<G>(S, s, S.pts.template as<Aff<F>>(), ret, ne, nb, weights, buckets_out, true, &clk, true);
}

template <int G>
void register_host_table(const void *rows, size_t nrows) {
  typedef typename FieldOf<G>::F F;
  if (!rows || !nrows) throw std::runtime_error("empty table");
  if (nrows >= (1ull << 31)) throw std::runtime_error("registered table exceeds 31-bit row indices");
  auto t = std::make_shared<HostTable>();
  MSM_HIP_CHECK(hipGetDevice(&t->device));
  t->group = G;
  t->base = static_cast<const uint8_t *>(rows);
  t->nrows = nrows;
  t->row_bytes = sizeof(AffP<F>);
  t->take_samples();  // before the upload: a concurrent edit then shows as stale next call
  t->rows.ensure(nrows * sizeof(AffP<F>));
  const size_t psz = 96 * G, chunk = std::min<size_t>(nrows, ((size_t)64 << 20) / psz);
  hipStream_t s;
  MSM_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  try {
    DevBuf stage;
    stage.ensure(chunk * psz);
    for (size_t r0 = 0; r0 < nrows; r0 += chunk) {  // pageable caller rows, 64-MiB pieces
      const size_t cnt = std::min(chunk, nrows - r0);
      MSM_HIP_CHECK(hipMemcpyAsync(stage.p, t->base + r0 * psz, cnt * psz, hipMemcpyHostToDevice, s));
      hipLaunchKernelGGL((k_convert_points<G, AffP<F>>), dim3(nblk(cnt, 256)), dim3(256), 0, s,
                         stage.template as<uint64_t>(), t->rows.template as<AffP<F>>() + r0, cnt);
      MSM_HIP_CHECK(hipGetLastError());
      MSM_HIP_CHECK(hipStreamSynchronize(s));  // the stage is reused
    }
  } catch (...) {
    (void)hipStreamDestroy(s);
    throw;
  }
  MSM_HIP_CHECK(hipStreamDestroy(s));
  TableRegistry::get().add(std::move(t));
}

// sum_i w_i buckets[i] for caller-filled blst xyzz buckets
template <int G>
void weighted_bucket_sum(void *ret, const void *buckets_blst, size_t nb, const uint32_t *weights) {
  typedef typename FieldOf<G>::F F;
  typedef typename HostField<G>::F HF;
  hfp::Jac<HF> out;
  std::memset(&out, 0, sizeof out);
  if (nb == 0) {
    std::memcpy(ret, &out, sizeof out);
    return;
  }
  auto lease = entry_state<G>();
  EntryMsmState<G> &S = **lease;
  hipStream_t s = lease->stream();
  S.xfer.ensure(nb * 192 * G);
  S.buckets.ensure(nb * sizeof(Xyzz<F>));
  MSM_HIP_CHECK(hipMemcpyAsync(S.xfer.p, buckets_blst, nb * 192 * G, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_import_xyzz<G>, dim3(nblk(nb, 256)), dim3(256), 0, s, S.xfer.template as<uint64_t>(),
                     S.buckets.template as<Xyzz<F>>(), nb);
  MSM_HIP_CHECK(hipGetLastError());
  plan_if_changed(S, weights, nb);
  S.red.launch(s, S.buckets.p);
  out = S.red.read(s);
  std::memcpy(ret, &out, sizeof out);
}

template void entry_msm<MSM_GROUP>(void *, const void *, size_t, const uint32_t *, const uint32_t *, size_t, size_t,
                                   const uint32_t *, void *);
template void weighted_bucket_sum<MSM_GROUP>(void *, const void *, size_t, const uint32_t *);
template void entry_msm_ptrs<MSM_GROUP>(void *, const void *const *, size_t, EntryFill, void *, size_t,
                                        const uint32_t *, void *);
template void register_host_table<MSM_GROUP>(const void *, size_t);

}  // namespace msm
