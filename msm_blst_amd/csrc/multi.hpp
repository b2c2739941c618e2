// multi.hpp -- one CHES MSM over several MI355X devices from ONE process
// (the C/C++ multi-device path behind msm_ches_ctx_create_multi).
//
// MSM is linear: Q = sum_g Q_g with Q_g = sum_{i in shard g} s_i P_i (SURVEY
// 8e).  The n points are split into contiguous, balanced shards, one Ches<G>
// engine per shard on its device; shard g builds (or receives) only its own
// rows of the reference table T[3(i h + j) + m - 1] (main_p1.cpp:155-172: the
// rows of point i are contiguous, so shard g's rows are one contiguous range of
// the reference layout).  A multiplication runs every shard's MSM concurrently
// (one host thread per shard, each driving its own device), and the single
// exchange is the read-back of the shards' 144/288-B Jacobian partials, folded
// on the host with an exact add (hfp::addj, doubling aware) in shard order.
// Each shard has a persistent host worker thread (created with the context; a
// thread per shard per call was a visible fixed cost at 2^18 points per GPU,
// where one MSM takes < 1 ms), and host scalars reach each device through the
// shard's pinned ring (hoststage.hpp) instead of a pageable copy.
// Batches on several DISTINCT devices can exchange over RCCL (the north star's
// "single RCCL reduce of the partial sums over xGMI"; opt-in since round 6,
// MSM_MULTI_RCCL=1, until a run on several devices has checked it): every shard leaves its
// per-MSM window sums (2 Jacobians, 288 B G1 / 576 B G2, per MSM) in a device
// exchange buffer, ONE ncclGather collects all shards' buffers on the first
// shard's device, one read-back, and the host combines and folds them exactly
// (RCCL's reduction ops cannot add curve points, hence gather + fold).
// By default every shard is read back separately (host fold of the shards'
// own read-backs); MSM_MULTI_RCCL=1 selects the RCCL exchange for any context
// of distinct devices, including a single shard (how one GPU tests it).  Single
// MSMs (run) keep the per-shard read-back: their latency path.  The reference
// itself is single-device; its Go binding splits points x windows over threads
// (bindings/go/blst.go:2064-2197), which would replicate points and tables on
// every GPU, so points are sharded.
//
// Shards may share a device (devices = {0, 0, ...}).  Consecutive shards on one
// device are merged into ONE engine over their joint point range (the table
// layout is point-major, so their rows are one contiguous range, and the sum
// of their partials is the MSM of that range): a device then runs one MSM per
// scalar set -- one front, accumulation, level 0 and reduction tail -- instead
// of one per shard (configs[3]'s 8 x 2^18 shards on one device: 8 latency-bound
// 2^18 pipelines became one 2^21 MSM).  MSM_MULTI_MERGE=0 (read when a context
// is created) keeps one engine per shard -- how the 1-GPU tests exercise the
// shard fold -- and MSM_MULTI_PIPELINE=0 additionally runs those engines
// concurrently instead of as one pipeline over (set, shard) jobs.
#pragma once
#include <condition_variable>
#include <cstring>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include <rccl/rccl.h>

#include "engine.hpp"
#include "hoststage.hpp"
#include "workers.hpp"

namespace msm {

template <int G>
class ChesMulti {
 public:
  typedef typename HostField<G>::F HF;
  struct Shard {
    int device = 0;
    int nlog = 1;             // caller's shards merged into this one (consecutive, same device)
    size_t start = 0, n = 0;  // global point range [start, start + n)
    std::unique_ptr<Ches<G>> eng;
    DevBuf scal;               // host scalars of this shard, per call
    HostStager stage;          // pinned ring for those scalars
    hipStream_t stream = nullptr;  // the shard's own stream (shards may share a device)
  };

  ChesMulti(const std::vector<int> &devices, const ChesParams &p) : p_(p), nlogical_(devices.size()) {
    if (devices.empty()) throw std::runtime_error("ChesMulti: no devices");
    const char *me = getenv("MSM_MULTI_MERGE"), *pe = getenv("MSM_MULTI_PIPELINE");
    const bool merge = !me || atoi(me) != 0;
    pipeline_ = !pe || atoi(pe) != 0;
    std::vector<std::pair<int, int>> groups;  // (device, caller shards)
    for (int d : devices)
      if (merge && !groups.empty() && groups.back().first == d) ++groups.back().second;
      else groups.push_back({d, 1});
    shards_ = std::vector<Shard>(groups.size());
    try {
      for (size_t g = 0; g < groups.size(); ++g) {
        Shard &s = shards_[g];
        s.device = groups[g].first;
        s.nlog = groups[g].second;
        s.eng = std::make_unique<Ches<G>>(s.device, p);
        if (groups.size() > 1) {
          DeviceGuard dg(s.device);
          MSM_HIP_CHECK(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
        }
      }
      // one persistent host thread per shard (several shards; workers.hpp)
      if (groups.size() > 1) team_ = std::make_unique<ThreadTeam>(groups.size());
    } catch (...) {
      release();  // the destructor does not run for a constructor that throws
      throw;
    }
  }
  ~ChesMulti() {
    release();
    for (ncclComm_t c : comms_) (void)ncclCommDestroy(c);
  }
  ChesMulti(const ChesMulti &) = delete;
  ChesMulti &operator=(const ChesMulti &) = delete;
  size_t nshards() const { return nlogical_; }  // the caller's shards (merged ones included)
  size_t engines() const { return shards_.size(); }
  Ches<G> &front() { return *shards_[0].eng; }
  const Ches<G> &front() const { return *shards_[0].eng; }
  const ChesParams &params() const { return p_; }
  size_t npoints() const { return n_; }
  size_t rows_per_point() const { return 3 * (size_t)p_.h; }
  size_t table_rows() const { return rows_per_point() * n_; }

  // points: n blst affine points (host memory, or device memory of the single
  // shard's device) -> every shard builds its rows on its own device
  void build_table(const void *pts, size_t n, bool on_device, hipStream_t s) {
    split(n);
    if (shards_.size() == 1) {
      shards_[0].eng->build_table(pts, n, on_device, s);
      return;
    }
    if (on_device) throw std::runtime_error("multi-device build_table takes host points");
    const uint8_t *P = static_cast<const uint8_t *>(pts);
    each([&](Shard &sh) { sh.eng->build_table(P + sh.start * 96 * G, sh.n, false, sh.stream); });
  }
  void reserve_table(size_t n) {
    split(n);
    for (Shard &sh : shards_) sh.eng->reserve_table(sh.n);
  }
  // reference-layout rows [first, first + count) -> the shards that own them
  void put_table(const void *rows, size_t first, size_t count, bool on_device, hipStream_t s) {
    if (shards_.size() == 1) return shards_[0].eng->put_table(rows, first, count, on_device, s);
    if (on_device) throw std::runtime_error("multi-device put_table takes host rows");
    route(first, count, [&](Shard &sh, size_t r0, size_t cnt, size_t off) {
      sh.eng->put_table(static_cast<const uint8_t *>(rows) + off * 96 * G, r0, cnt, false, sh.stream);
    });
  }
  void set_table(const void *tab, size_t n, bool on_device, hipStream_t s) {
    reserve_table(n);
    put_table(tab, 0, table_rows(), on_device, s);
  }
  void get_table(void *out, size_t first, size_t count, hipStream_t s) {
    if (first + count > table_rows()) throw std::runtime_error("table range out of bounds");
    if (shards_.size() == 1) return shards_[0].eng->get_table(out, first, count, s);
    route(first, count, [&](Shard &sh, size_t r0, size_t cnt, size_t off) {
      sh.eng->get_table(static_cast<uint8_t *>(out) + off * 96 * G, r0, cnt, sh.stream);
    });
  }

  // scalars: n strings of `stride` bytes (host memory; device memory only for a
  // single shard, on its device)
  void run(hipStream_t s, const uint8_t *scalars, size_t stride, bool on_device, hfp::Jac<HF> *out) {
    if (shards_.size() == 1) {
      Shard &sh = shards_[0];
      const uint8_t *d = scalars;
      if (!on_device && sh.n) {
        DeviceGuard g(sh.device);
        sh.scal.ensure(sh.n * stride + 16);
        sh.stage.upload(sh.scal.p, scalars, sh.n * stride, s);
        d = static_cast<const uint8_t *>(sh.scal.p);
      }
      sh.eng->run(s, d, stride, out);
      return;
    }
    if (on_device) throw std::runtime_error("multi-device mult takes host scalars");
    std::vector<hfp::Jac<HF>> part(shards_.size());
    each([&](Shard &sh) {
      DeviceGuard g(sh.device);
      hfp::Jac<HF> r;
      if (sh.n) {
        sh.scal.ensure(sh.n * stride + 16);
        sh.stage.upload(sh.scal.p, scalars + sh.start * stride, sh.n * stride, sh.stream);
        sh.eng->run(sh.stream, static_cast<const uint8_t *>(sh.scal.p), stride, &r);
      } else {
        std::memset(&r, 0, sizeof r);
      }
      part[&sh - shards_.data()] = r;
    });
    *out = fold(part);
  }

  // count MSMs: scalar set k at scalars + k * set_stride (host memory for
  // several shards); every shard runs its own pipelined batch on its slice
  void run_batch(hipStream_t s, const uint8_t *scalars, size_t stride, size_t set_stride, size_t count,
                 hfp::Jac<HF> *outs, bool on_host) {
    if (use_rccl()) return run_batch_rccl(s, scalars, stride, set_stride, count, outs, on_host);
    if (shards_.size() == 1) return shards_[0].eng->run_batch(s, scalars, stride, set_stride, count, outs, on_host);
    if (!on_host) throw std::runtime_error("multi-device mult_batch takes host scalars");
    if (one_device_pipeline()) {
      // every shard on one device: ONE pipeline over the count x D jobs (set k,
      // shard d) with each shard's table (Ches::run_jobs), instead of D engines
      // with five streams each competing for the device's four hardware queues
      const size_t D = shards_.size();
      std::vector<const void *> tabs(D);
      for (size_t g = 0; g < D; ++g) tabs[g] = shards_[g].eng->table_ptr();
      std::vector<hfp::Jac<HF>> part(count * D);
      Shard &sh = shards_[0];
      DeviceGuard g(sh.device);
      sh.eng->run_jobs(sh.stream, scalars, stride, set_stride, count, D, tabs.data(), part.data(), true);
      MSM_HIP_CHECK(hipStreamSynchronize(sh.stream));
      for (size_t k = 0; k < count; ++k)
        outs[k] = fold(std::vector<hfp::Jac<HF>>(part.begin() + k * D, part.begin() + (k + 1) * D));
      return;
    }
    std::vector<std::vector<hfp::Jac<HF>>> part(shards_.size(), std::vector<hfp::Jac<HF>>(count));
    each([&](Shard &sh) {
      std::vector<hfp::Jac<HF>> &r = part[&sh - shards_.data()];
      if (sh.n) {
        DeviceGuard g(sh.device);
        sh.eng->run_batch(sh.stream, scalars + sh.start * stride, stride, set_stride, count, r.data(), true);
        MSM_HIP_CHECK(hipStreamSynchronize(sh.stream));
      } else {
        for (auto &j : r) std::memset(&j, 0, sizeof j);
      }
    });
    for (size_t k = 0; k < count; ++k) {
      std::vector<hfp::Jac<HF>> col(shards_.size());
      for (size_t g = 0; g < shards_.size(); ++g) col[g] = part[g][k];
      outs[k] = fold(col);
    }
  }

  void set_profiling(bool on) {
    for (Shard &sh : shards_) sh.eng->set_profiling(on);
  }
  bool rccl_exchange() const { return use_rccl(); }

 private:
  ChesParams p_;
  size_t nlogical_ = 1;
  bool pipeline_ = true;
  std::vector<Shard> shards_;
  size_t n_ = 0;

  // all shards on one device with equal point counts (MSM_MULTI_PIPELINE=0: one
  // engine per shard, concurrently, as on separate devices)
  bool one_device_pipeline() const {
    if (!pipeline_ || shards_.size() < 2 || shards_[0].n == 0) return false;
    for (const Shard &sh : shards_)
      if (sh.device != shards_[0].device || sh.n != shards_[0].n) return false;
    return true;
  }
  // balanced contiguous ranges over the caller's shards; a merged shard owns the
  // union of its members' ranges
  void split(size_t n) {
    const size_t L = nlogical_, base = n / L, rem = n % L;
    size_t at = 0, l = 0;
    for (Shard &sh : shards_) {
      sh.start = at;
      sh.n = 0;
      for (int k = 0; k < sh.nlog; ++k, ++l) sh.n += base + (l < rem ? 1 : 0);
      at += sh.n;
    }
    n_ = n;
  }
  std::unique_ptr<ThreadTeam> team_;  // one thread per shard when there are several (one run at a time)
  // RCCL exchange of batch partials (use_rccl): one communicator per shard
  // device (ncclCommInitAll, created at the first exchange), the shards' send
  // buffers and the gather buffer on shard 0's device
  std::vector<ncclComm_t> comms_;
  std::vector<DevBuf> xsend_;
  DevBuf xrecv_;
  std::vector<hipStream_t> xstreams_;  // the shards' streams (created here for a single shard)

  bool use_rccl() const {
    static const int env = [] {
      const char *e = getenv("MSM_MULTI_RCCL");
      return e ? atoi(e) : -1;
    }();
    // opt-in (MSM_MULTI_RCCL=1): every run so far had one GPU, so the gather has
    // only run on one-rank communicators; the per-shard read-back stays the
    // default until a run on several devices has compared the two
    if (env != 1 || shards_.empty()) return false;
    for (size_t a = 0; a < shards_.size(); ++a)  // distinct devices only (one rank per device)
      for (size_t b = a + 1; b < shards_.size(); ++b)
        if (shards_[a].device == shards_[b].device) return false;
    return true;
  }
  static void nccl_check(ncclResult_t r, const char *what) {
    if (r != ncclSuccess) throw std::runtime_error(std::string("RCCL ") + what + ": " + ncclGetErrorString(r));
  }
  // every shard runs its batch into its send buffer (concurrently, one worker per
  // shard), then one ncclGather onto shard 0's device, one read-back, and the
  // host combine + fold per MSM in shard order
  void run_batch_rccl(hipStream_t s, const uint8_t *scalars, size_t stride, size_t set_stride, size_t count,
                      hfp::Jac<HF> *outs, bool on_host) {
    if (!on_host && shards_.size() > 1) throw std::runtime_error("multi-device mult_batch takes host scalars");
    const size_t D = shards_.size();
    if (comms_.empty()) {
      std::vector<int> devs(D);
      for (size_t g = 0; g < D; ++g) devs[g] = shards_[g].device;
      comms_.resize(D);
      nccl_check(ncclCommInitAll(comms_.data(), (int)D, devs.data()), "ncclCommInitAll");
      xsend_ = std::vector<DevBuf>(D);
      xstreams_.assign(D, nullptr);
      for (size_t g = 0; g < D; ++g) {
        xstreams_[g] = shards_[g].stream;
        if (!xstreams_[g]) {  // a single shard: its own stream for the collective
          DeviceGuard dg(shards_[g].device);
          MSM_HIP_CHECK(hipStreamCreateWithFlags(&shards_[g].stream, hipStreamNonBlocking));
          xstreams_[g] = shards_[g].stream;
        }
      }
    }
    const size_t ob = shards_[0].eng->exchange_bytes();
    for (size_t g = 0; g < D; ++g) {
      DeviceGuard dg(shards_[g].device);
      xsend_[g].ensure(count * ob);
    }
    {
      DeviceGuard dg(shards_[0].device);
      xrecv_.ensure(D * count * ob);
    }
    // prior work on the caller's stream (which may write the scalar sets) is
    // done before any shard reads them: the shards run on their own streams
    MSM_HIP_CHECK(hipStreamSynchronize(s));
    each([&](Shard &sh) {
      const size_t g = &sh - shards_.data();
      DeviceGuard dg(sh.device);
      if (sh.n) {
        std::vector<hfp::Jac<HF>> unused(1);
        sh.eng->run_batch(sh.stream, scalars + sh.start * stride, stride, set_stride, count, unused.data(), on_host,
                          xsend_[g].p);
      } else {
        MSM_HIP_CHECK(hipMemsetAsync(xsend_[g].p, 0, count * ob, sh.stream));  // all-zero Jacobians: infinity
      }
      MSM_HIP_CHECK(hipStreamSynchronize(sh.stream));
    });
    nccl_check(ncclGroupStart(), "ncclGroupStart");
    for (size_t g = 0; g < D; ++g) {
      DeviceGuard dg(shards_[g].device);
      nccl_check(ncclGather(xsend_[g].p, g == 0 ? xrecv_.p : nullptr, count * ob, ncclUint8, 0, comms_[g],
                            shards_[g].stream),
                 "ncclGather");
    }
    nccl_check(ncclGroupEnd(), "ncclGroupEnd");
    std::vector<uint8_t> host(D * count * ob);
    {
      DeviceGuard dg(shards_[0].device);
      MSM_HIP_CHECK(hipMemcpyAsync(host.data(), xrecv_.p, host.size(), hipMemcpyDeviceToHost, shards_[0].stream));
      for (size_t g = 0; g < D; ++g) {
        DeviceGuard dg2(shards_[g].device);
        MSM_HIP_CHECK(hipStreamSynchronize(shards_[g].stream));
      }
    }
    for (size_t k = 0; k < count; ++k) {
      std::vector<hfp::Jac<HF>> col(D);
      for (size_t g = 0; g < D; ++g) {
        const uint8_t *w = host.data() + (g * count + k) * ob;
        bool zero = true;  // a shard without points sent zeros (infinity)
        for (size_t b = 0; b < ob && zero; ++b) zero = w[b] == 0;
        if (zero) std::memset(&col[g], 0, sizeof col[g]);
        else col[g] = shards_[g].eng->combine_exchange(w);
      }
      outs[k] = fold(col);
    }
  }

  void release() {
    team_.reset();  // joins the shard threads
    for (Shard &s : shards_)
      if (s.stream) {
        int prev = -1;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(s.device);
        (void)hipStreamSynchronize(s.stream);
        (void)hipStreamDestroy(s.stream);
        s.stream = nullptr;
        if (prev >= 0) (void)hipSetDevice(prev);
      }
  }
  // run f on every shard, each on its persistent worker thread; the first
  // exception is rethrown
  template <class Fn>
  void each(Fn f) {
    if (!team_) {
      for (Shard &sh : shards_) f(sh);
      return;
    }
    team_->run([&](size_t g) { f(shards_[g]); });
  }
  // split a reference-layout row range over the owning shards:
  // f(shard, first row within the shard, rows, offset into the caller's range)
  template <class Fn>
  void route(size_t first, size_t count, Fn f) {
    const size_t R = rows_per_point();
    for (Shard &sh : shards_) {
      const size_t lo = sh.start * R, hi = (sh.start + sh.n) * R;
      const size_t a = std::max(lo, first), b = std::min(hi, first + count);
      if (a < b) f(sh, a - lo, b - a, a - first);
    }
  }
  static hfp::Jac<HF> fold(const std::vector<hfp::Jac<HF>> &part) {
    hfp::Jac<HF> acc = part[0];
    for (size_t g = 1; g < part.size(); ++g) acc = hfp::addj(acc, part[g]);
    return acc;
  }
};

}  // namespace msm
