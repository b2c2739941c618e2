// workers.hpp -- the host thread patterns of the engine, free of HIP so the CPU
// sanitizer build (tests/host/sanitize_shim.cpp, ASan/UBSan and TSan) runs the
// same code the library runs.
//
//   WorkerPool  process-wide pool: parallel_for(n, f) runs f(0..n-1) on the
//               workers and the caller (host copies into pinned rings,
//               hoststage.hpp; the batch's per-MSM host Horner, ches.hip; the
//               tiles' row gathers, compat.hip)
//   ThreadTeam  one persistent thread per member: run(f) hands member g the
//               task f(g) on its own thread and waits for all of them -- the
//               multi-device context's shard workers (multi.hpp; a device's
//               calls stay on one host thread)
// The reference is single-threaded (its Go binding's grid, bindings/go/
// blst.go:2064-2197, is the only parallel caller); both patterns are ours.
#pragma once
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace msm {

// Process-wide pool of host worker threads (never destroyed: the workers park
// on a condition variable for the life of the process).  parallel_for runs
// f(0..n-1) on the workers and the calling thread and returns when all are
// done; concurrent callers take turns.  The first exception is rethrown.
class WorkerPool {
 public:
  static WorkerPool &get() {
    static WorkerPool *p = new WorkerPool();
    return *p;
  }
  size_t size() const { return th_.size() + 1; }

  void parallel_for(size_t n, const std::function<void(size_t)> &f) {
    if (n == 0) return;
    if (n == 1 || th_.empty()) {
      for (size_t i = 0; i < n; ++i) f(i);
      return;
    }
    std::lock_guard<std::mutex> turn(call_mu_);
    auto job = std::make_shared<Job>();
    job->f = &f;
    job->n = n;
    job->remaining = n;
    {
      std::lock_guard<std::mutex> g(mu_);
      job_ = job;
      ++gen_;
    }
    cv_.notify_all();
    run(*job);
    {
      std::unique_lock<std::mutex> lk(job->mu);
      job->done.wait(lk, [&] { return job->remaining == 0; });
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      job_.reset();
    }
    if (job->err) std::rethrow_exception(job->err);
  }

 private:
  struct Job {
    const std::function<void(size_t)> *f = nullptr;
    size_t n = 0;
    std::atomic<size_t> next{0};
    size_t remaining = 0;  // guarded by mu
    std::exception_ptr err;
    std::mutex mu;
    std::condition_variable done;
  };
  std::mutex call_mu_, mu_;
  std::condition_variable cv_;
  std::shared_ptr<Job> job_;
  uint64_t gen_ = 0;
  std::vector<std::thread> th_;

  WorkerPool() {
    // the box's CPU share per GPU is 16 threads; host copies saturate at ~8
    // (h2d_stage: 142 GB/s memcpy into pinned memory with 8 threads)
    size_t want = 7;
    if (const char *e = getenv("MSM_HOST_THREADS")) want = (size_t)std::max(1, atoi(e)) - 1;
    const size_t hw = std::thread::hardware_concurrency();
    if (hw) want = std::min(want, hw > 1 ? hw - 1 : 0);
    for (size_t t = 0; t < want; ++t) th_.emplace_back([this] { loop(); });
    for (auto &t : th_) t.detach();
  }
  static void run(Job &j) {
    size_t i;
    while ((i = j.next.fetch_add(1)) < j.n) {
      try {
        (*j.f)(i);
      } catch (...) {
        std::lock_guard<std::mutex> g(j.mu);
        if (!j.err) j.err = std::current_exception();
      }
      std::lock_guard<std::mutex> g(j.mu);
      if (--j.remaining == 0) j.done.notify_all();
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      std::shared_ptr<Job> j;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        j = job_;
      }
      if (j) run(*j);  // a stale job has next >= n: nothing to do
    }
  }
};

// One persistent host thread per member; run(f) runs f(g) on member g's thread
// for every g and waits for all of them (one run at a time; the first exception
// is rethrown).  Joined by the destructor.
class ThreadTeam {
 public:
  explicit ThreadTeam(size_t n) : w_(n) {
    for (Worker &w : w_) w.th = std::thread([&w] { work(w); });
  }
  ~ThreadTeam() {
    for (Worker &w : w_) {
      {
        std::lock_guard<std::mutex> g(w.mu);
        w.quit = true;
      }
      w.cv.notify_all();
      if (w.th.joinable()) w.th.join();
    }
  }
  ThreadTeam(const ThreadTeam &) = delete;
  ThreadTeam &operator=(const ThreadTeam &) = delete;
  size_t size() const { return w_.size(); }

  void run(const std::function<void(size_t)> &f) {
    std::lock_guard<std::mutex> turn(run_mu_);
    for (size_t g = 0; g < w_.size(); ++g) {
      Worker &w = w_[g];
      {
        std::lock_guard<std::mutex> lk(w.mu);
        w.task = [&f, g] { f(g); };
        w.has = true;
        w.done = false;
        w.err = nullptr;
      }
      w.cv.notify_all();
    }
    std::exception_ptr first;
    for (Worker &w : w_) {
      std::unique_lock<std::mutex> lk(w.mu);
      w.cv.wait(lk, [&] { return w.done; });
      if (w.err && !first) first = w.err;
    }
    if (first) std::rethrow_exception(first);
  }

 private:
  struct Worker {
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    std::function<void()> task;
    bool has = false, quit = false, done = false;
    std::exception_ptr err;
  };
  std::vector<Worker> w_;
  std::mutex run_mu_;

  static void work(Worker &w) {
    for (;;) {
      std::function<void()> t;
      {
        std::unique_lock<std::mutex> lk(w.mu);
        w.cv.wait(lk, [&] { return w.has || w.quit; });
        if (w.quit) return;
        t = std::move(w.task);
        w.has = false;
      }
      std::exception_ptr err;
      try {
        t();
      } catch (...) {
        err = std::current_exception();
      }
      {
        std::lock_guard<std::mutex> g(w.mu);
        w.err = err;
        w.done = true;
      }
      w.cv.notify_all();
    }
  }
};

}  // namespace msm
