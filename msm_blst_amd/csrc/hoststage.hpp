// hoststage.hpp -- uploads from caller-owned pageable host memory.
//
// The blst entry points receive points and scalars in the caller's memory
// (ref multi_scalar.c:581-607), usually fresh pageable buffers.  HIP's own
// pageable copy path pins user pages on the fly: measured on MI355X it is as
// fast as a pinned copy for a buffer it has seen before (56 GB/s for 128 MiB),
// but 10-37 ms per 2^20-point call with fresh buffers, growing call by call
// (tools/dropin_timing.py).  HostStager instead streams the bytes through a
// small pinned ring: the host copy of chunk c + 1 (split over a persistent
// worker pool) overlaps the DMA of chunk c, so the upload runs at the DMA rate
// (tools/microbench/h2d_stage.cpp: 16 MiB x 4 slots, 4-8 threads ~49 GB/s).
#pragma once
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "engine.hpp"
#include "workers.hpp"  // WorkerPool

namespace msm {

// memcpy of `bytes` split over the worker pool (1-MiB pieces or more)
inline void parallel_memcpy(void *dst, const void *src, size_t bytes) {
  const size_t piece = std::max<size_t>((size_t)1 << 20, (bytes + 7) / 8);
  const size_t n = (bytes + piece - 1) / piece;
  WorkerPool::get().parallel_for(n, [&](size_t i) {
    const size_t a = i * piece, b = std::min(bytes, a + piece);
    memcpy(static_cast<uint8_t *>(dst) + a, static_cast<const uint8_t *>(src) + a, b - a);
  });
}

// true if p is page-locked / registered host memory (a direct DMA source)
inline bool host_pinned(const void *p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // unregistered pageable memory reports an error: clear it
    return false;
  }
  return a.type == hipMemoryTypeHost || a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

// Pinned ring for host -> device uploads; one per engine (engines are leased by
// one thread at a time, pool.hpp).  The ring is sized for the uploads it has
// seen -- kSlots slots of min(kChunk, bytes / kSlots rounded up to 1 MiB) --
// and grows (after its pending DMAs finish) only when a larger upload arrives,
// so an engine serving small calls (a Go tile, a 2^12-point MSM) holds a few
// MiB of page-locked memory, not 64.  Uploads below kDirect bytes skip the ring
// (HIP's own staged pageable copy).
class HostStager {
 public:
  static constexpr size_t kChunk = (size_t)16 << 20;
  static constexpr size_t kMinSlot = (size_t)1 << 20;
  static constexpr size_t kDirect = (size_t)1 << 20;
  static constexpr int kSlots = 4;
  HostStager() = default;
  HostStager(const HostStager &) = delete;
  HostStager &operator=(const HostStager &) = delete;
  ~HostStager() { release(); }
  size_t pinned_bytes() const { return ring_ ? slot_ * kSlots : 0; }

  // dst (device) <- src (host), enqueued on s; returns when every chunk is
  // enqueued and src is no longer read.  Pinned sources go straight to the DMA.
  void upload(void *dst, const void *src, size_t bytes, hipStream_t s) {
    if (!bytes) return;
    if (bytes < kDirect || host_pinned(src)) {
      MSM_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
      return;
    }
    const size_t want = std::min(kChunk, std::max(kMinSlot, ((bytes + kSlots - 1) / kSlots + kMinSlot - 1) &
                                                                ~(kMinSlot - 1)));
    if (!ring_ || want > slot_) {
      release();
      MSM_HIP_CHECK(hipHostMalloc(&ring_, want * kSlots, hipHostMallocDefault));
      slot_ = want;
      for (int k = 0; k < kSlots; ++k) MSM_HIP_CHECK(hipEventCreateWithFlags(&ev_[k], hipEventDisableTiming));
    }
    for (size_t off = 0; off < bytes; off += slot_) {
      const int k = next_;
      next_ = (next_ + 1) % kSlots;
      if (used_[k]) MSM_HIP_CHECK(hipEventSynchronize(ev_[k]));  // the slot's previous DMA is done
      const size_t len = std::min(slot_, bytes - off);
      uint8_t *slot = static_cast<uint8_t *>(ring_) + (size_t)k * slot_;
      parallel_memcpy(slot, static_cast<const uint8_t *>(src) + off, len);
      MSM_HIP_CHECK(hipMemcpyAsync(static_cast<uint8_t *>(dst) + off, slot, len, hipMemcpyHostToDevice, s));
      MSM_HIP_CHECK(hipEventRecord(ev_[k], s));
      used_[k] = true;
    }
  }

 private:
  void *ring_ = nullptr;
  size_t slot_ = 0;
  hipEvent_t ev_[kSlots] = {};
  bool used_[kSlots] = {};
  int next_ = 0;
  void release() noexcept {  // waits for the ring's pending DMAs
    for (int k = 0; k < kSlots; ++k) {
      if (ev_[k]) {
        if (used_[k]) (void)hipEventSynchronize(ev_[k]);
        (void)hipEventDestroy(ev_[k]);
      }
      ev_[k] = nullptr;
      used_[k] = false;
    }
    if (ring_) (void)hipHostFree(ring_);
    ring_ = nullptr;
    slot_ = 0;
    next_ = 0;
  }
};

}  // namespace msm
