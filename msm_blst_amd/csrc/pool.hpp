// pool.hpp -- engines behind the stateless blst-named entry points.
//
// blst's MSM calls carry no context (ref multi_scalar.c:581-607: the caller
// owns a scratch buffer and nothing else), yet the GPU path needs device
// buffers sized for n.  Engines are therefore kept in a process-wide pool per
// (device, parameter) key: a call leases one (creating it when every pooled
// engine is in use by another thread -- concurrent tile calls from the Go
// binding's worker threads, blst.go:2105-2167, each get their own), runs on the
// engine's own non-blocking stream, and returns it.  Device memory is bounded
// by the peak number of concurrent calls, not by the number of threads that
// ever called (a thread-local cache pinned one engine per OS thread of a Go
// pool); idle engines beyond a byte budget per device are freed when they are
// returned, and msm_release_engine_cache() frees every idle engine.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <exception>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <utility>
#include <vector>

#include "engine.hpp"

namespace msm {

struct PoolStats {
  size_t live = 0, idle = 0, idle_bytes = 0;
};

// every pool registers its release / stats hooks here (one list per process)
struct PoolRegistry {
  std::mutex mu;
  std::vector<std::function<void(PoolStats &, bool release)>> pools;
  std::atomic<size_t> idle_budget{(size_t)8 << 30};  // bytes of idle engines kept per device and pool
  static PoolRegistry &get() {
    static PoolRegistry *r = new PoolRegistry();  // never destroyed: engines may outlive static teardown
    return *r;
  }
  // release: free every idle engine; otherwise (stats) idle engines beyond a
  // lowered idle_budget are trimmed
  void visit(PoolStats &st, bool release) {
    std::vector<std::function<void(PoolStats &, bool)>> copy;
    {
      std::lock_guard<std::mutex> g(mu);
      copy = pools;
    }
    for (auto &f : copy) f(st, release);
  }
};

// E must provide device_bytes(); the pool gives each engine a stream
template <class E>
class EnginePool {
 public:
  typedef std::pair<int, int> Key;  // (device, parameter)
  struct Slot {
    std::unique_ptr<E> e;
    hipStream_t s = nullptr;
    int dev = 0;
  };
  class Lease {
   public:
    Lease(EnginePool *p, Key k, Slot sl) : p_(p), k_(k), sl_(std::move(sl)), exc_(std::uncaught_exceptions()) {}
    Lease(const Lease &) = delete;
    Lease &operator=(const Lease &) = delete;
    // A call that throws (a HIP error, bad arguments) may leave copies reading
    // the caller's buffers or kernels queued on the engine's stream, and the
    // engine in an unknown state: during unwinding (or after poison()) the
    // stream is drained and the engine destroyed instead of returned to the pool.
    ~Lease() {
      if (poisoned_ || std::uncaught_exceptions() > exc_) p_->discard(std::move(sl_));
      else p_->put(k_, std::move(sl_));
    }
    void poison() { poisoned_ = true; }
    E &operator*() { return *sl_.e; }
    E *operator->() { return sl_.e.get(); }
    hipStream_t stream() const { return sl_.s; }

   private:
    EnginePool *p_;
    Key k_;
    Slot sl_;
    int exc_;
    bool poisoned_ = false;
  };

  static EnginePool &get() {
    static EnginePool *p = [] {
      auto *q = new EnginePool();
      std::lock_guard<std::mutex> g(PoolRegistry::get().mu);
      PoolRegistry::get().pools.push_back([q](PoolStats &st, bool release) { q->visit(st, release); });
      return q;
    }();
    return *p;
  }

  template <class Make>
  std::unique_ptr<Lease> lease(int dev, int param, Make make) {
    Key k(dev, param);
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = idle_.find(k);
      if (it != idle_.end() && !it->second.empty()) {
        Slot sl = std::move(it->second.back());
        it->second.pop_back();
        return std::make_unique<Lease>(this, k, std::move(sl));
      }
      ++live_;
    }
    try {
      DeviceGuard dg(dev);
      Slot sl;
      sl.dev = dev;
      sl.e = make();
      MSM_HIP_CHECK(hipStreamCreateWithFlags(&sl.s, hipStreamNonBlocking));
      return std::make_unique<Lease>(this, k, std::move(sl));
    } catch (...) {
      std::lock_guard<std::mutex> g(mu_);
      --live_;
      throw;
    }
  }

 private:
  std::mutex mu_;
  std::map<Key, std::vector<Slot>> idle_;
  size_t live_ = 0;

  size_t idle_bytes_dev(int dev) {  // mu_ held
    size_t b = 0;
    for (auto &kv : idle_)
      if (kv.first.first == dev)
        for (auto &sl : kv.second) b += sl.e->device_bytes();
    return b;
  }
  static void destroy(Slot &sl) noexcept {  // called from ~Lease: never throws
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(sl.dev);
    if (sl.s) {
      (void)hipStreamSynchronize(sl.s);
      (void)hipStreamDestroy(sl.s);
    }
    sl.e.reset();
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  void put(const Key &k, Slot sl) {
    if (!sl.e) return;
    {
      std::lock_guard<std::mutex> g(mu_);
      if (idle_bytes_dev(k.first) + sl.e->device_bytes() <= PoolRegistry::get().idle_budget.load()) {
        idle_[k].push_back(std::move(sl));
        return;
      }
      --live_;
    }
    destroy(sl);
  }
  void discard(Slot sl) noexcept {  // never cached (~Lease during unwinding)
    if (!sl.e) return;
    {
      std::lock_guard<std::mutex> g(mu_);
      --live_;
    }
    destroy(sl);
  }
  void visit(PoolStats &st, bool release) {
    std::vector<Slot> drop;
    {
      std::lock_guard<std::mutex> g(mu_);
      if (release) {
        for (auto &kv : idle_)
          for (auto &sl : kv.second) drop.push_back(std::move(sl));
        idle_.clear();
        live_ -= drop.size();
      } else {  // trim each device's idle engines to the (possibly lowered) budget
        const size_t budget = PoolRegistry::get().idle_budget.load();
        std::map<int, size_t> held;
        for (auto &kv : idle_) {
          auto &v = kv.second;
          for (size_t i = 0; i < v.size();) {
            size_t &h = held[kv.first.first];
            const size_t b = v[i].e->device_bytes();
            if (h + b <= budget) {
              h += b;
              ++i;
            } else {
              drop.push_back(std::move(v[i]));
              v.erase(v.begin() + (long)i);
            }
          }
        }
        live_ -= drop.size();
      }
      st.live += live_;
      for (auto &kv : idle_)
        for (auto &sl : kv.second) st.idle += 1, st.idle_bytes += sl.e->device_bytes();
    }
    for (auto &sl : drop) destroy(sl);
  }
};

}  // namespace msm
