// bgmw.hip -- host orchestration of the BGMW95 fixed-base MSM
// (LuoGuiwen/MSM_blst, method `pippenger_variant_BGMW95`, ref
// main_p1.cpp:294-398; tile ref multi_scalar.c:506-547; digits ref
// auxiliaryfunc.h:130-145) on one MI355X.
//
// Setup (once): table T[i h + j] = q^j P_i (ref init_pippenger_BGMW95,
// main_p1.cpp:94-122) built on the GPU by k_ches_table<G, 1> and resident in
// HBM in the engine's 128-B padded affine rows.
//
// Per MSM (one stream): k_bgmw_digits (signed radix-q digits, one entry per
// nonzero digit) -> BucketSort over q/2 buckets (+ copies of the few buckets the
// top digit hits) -> k_accumulate (one lane per bucket, xyzz += +-T[slot]) ->
// WeightedReducer (sum_b b S_b; ref integrate_buckets, multi_scalar.c:281-297).
#include <algorithm>
#include <cstring>

#include "ches_kernels.hpp"
#include "engine.hpp"
#include "pair_kernels.hpp"

#ifndef MSM_GROUP
#error "define MSM_GROUP (1 or 2)"
#endif

namespace msm {

// r (BLS12-381 group order) >> k for k >= 192, as a 64-bit value
static uint64_t r_shift(int k) {
  const uint64_t R[4] = {0xffffffff00000001ULL, 0x53bda402fffe5bfeULL, 0x3339d80809a1d805ULL, 0x73eda753299d7d48ULL};
  if (k >= 256) return 0;
  const int w = k / 64, b = k % 64;
  uint64_t lo = R[w] >> b;
  if (b && w + 1 < 4) lo |= R[w + 1] << (64 - b);
  return lo;
}

template <int G>
Bgmw<G>::Bgmw(int device, int q_exp, int h) : dev_(device), q_exp_(q_exp), h_(h) {
  DeviceGuard g(dev_);
  if (q_exp < 2 || q_exp > 24 || h < 1 || h > 64 || (long)q_exp * h < 255 || (long)q_exp * (h - 1) < 192)
    throw std::runtime_error("bad BGMW95 parameters (need q_exp in [2,24], q_exp h >= 255)");
  nb0_ = (size_t)1 << (q_exp - 1);
  // |top digit| <= floor((r/2) / q^(h-1)) + 1 (the digits are of min(s, r - s))
  uint64_t top = r_shift(q_exp * (h - 1)) / 2 + 2;
  small_ = (uint32_t)std::min<uint64_t>(top, nb0_);
  ev_.resize(6);
  for (auto &e : ev_) MSM_HIP_CHECK(hipEventCreate(&e));
}
template <int G>
Bgmw<G>::~Bgmw() {
  for (auto &e : ev_) (void)hipEventDestroy(e);
}

// copies_ of the small top-digit buckets so that a copy receives ~ the mean
// bucket load (n h / (q/2)) of top-digit entries
template <int G>
void Bgmw<G>::plan_buckets(size_t n) {
  int want = 1;
  if (n > 0 && small_ < nb0_) {
    double mean = std::max(1.0, (double)n * h_ / (double)nb0_);
    double c = (double)n / ((double)small_ * mean);
    want = (int)std::min(256.0, std::max(1.0, std::ceil(c)));
  }
  if (want == copies_ && red_.size()) return;
  copies_ = want;
  std::vector<uint32_t> w(nb0_);
  for (size_t b = 0; b < nb0_; ++b) w[b] = (uint32_t)(b + 1);
  for (int c = 1; c < copies_; ++c)
    for (uint32_t b = 0; b < small_; ++b) w.push_back(b + 1);
  red_.plan(w);
}

template <int G>
void Bgmw<G>::build_table(const void *pts, size_t n, bool on_device, hipStream_t s) {
  typedef typename FieldOf<G>::F F;
  DeviceGuard g(dev_);
  const size_t K = (size_t)h_;
  if (n == 0) {
    n_ = 0;
    return;
  }
  if (K * n >= (1ull << 31)) throw std::runtime_error("BGMW95 table too large for 31-bit slots");
  const size_t raw = n * 96 * G;
  const void *src = pts;
  DevBuf stage, base;
  if (!on_device) {
    stage.ensure(raw);
    MSM_HIP_CHECK(hipMemcpyAsync(stage.p, pts, raw, hipMemcpyHostToDevice, s));
    src = stage.p;
  }
  base.ensure(n * sizeof(Aff<F>));
  hipLaunchKernelGGL(k_convert_points<G>, dim3(nblk(n, 256)), dim3(256), 0, s, (const uint64_t *)src,
                     base.as<Aff<F>>(), n);
  MSM_HIP_CHECK(hipGetLastError());
  table_.ensure(K * n * sizeof(AffP<F>));
  const size_t chunk = std::min<size_t>(n, (size_t)1 << 17);
  DevBuf scratch, pref;
  scratch.ensure(K * chunk * sizeof(Xyzz<F>));
  pref.ensure(K * chunk * sizeof(F));
  for (size_t i0 = 0; i0 < n; i0 += chunk) {
    size_t cnt = std::min(chunk, n - i0);
    if constexpr (G == 2)  // lane pairs (pair_kernels.hpp)
      hipLaunchKernelGGL((k_ches_table2p<1>), dim3(nblk(2 * cnt, 128)), dim3(128), 0, s, base.as<Aff<F>>(), i0, cnt,
                         q_exp_, h_, scratch.as<Xyzz<F>>(), pref.as<F>(), table_.as<AffP<F>>());
    else
      hipLaunchKernelGGL((k_ches_table<G, 1>), dim3(nblk(cnt, 64)), dim3(64), 0, s, base.as<Aff<F>>(), i0, cnt, q_exp_,
                         h_, scratch.as<Xyzz<F>>(), pref.as<F>(), table_.as<AffP<F>>());
    MSM_HIP_CHECK(hipGetLastError());
  }
  MSM_HIP_CHECK(hipStreamSynchronize(s));
  n_ = n;
  plan_buckets(n);
}

template <int G>
void Bgmw<G>::reserve_table(size_t n) {
  typedef typename FieldOf<G>::F F;
  DeviceGuard g(dev_);
  const size_t cnt = (size_t)h_ * n;
  if (cnt >= (1ull << 31)) throw std::runtime_error("table too large for 31-bit slots");
  table_.ensure(std::max<size_t>(cnt, 1) * sizeof(AffP<F>));
  n_ = n;
  plan_buckets(n);
}

template <int G>
void Bgmw<G>::put_table(const void *tab, size_t first, size_t count, bool on_device, hipStream_t s) {
  typedef typename FieldOf<G>::F F;
  DeviceGuard g(dev_);
  if (first + count > table_rows()) throw std::runtime_error("table rows out of range");
  if (!count) return;
  const void *src = tab;
  DevBuf stage;
  if (!on_device) {
    stage.ensure(count * 96 * G);
    MSM_HIP_CHECK(hipMemcpyAsync(stage.p, tab, count * 96 * G, hipMemcpyHostToDevice, s));
    src = stage.p;
  }
  hipLaunchKernelGGL((k_convert_points<G, AffP<F>>), dim3(nblk(count, 256)), dim3(256), 0, s, (const uint64_t *)src,
                     table_.as<AffP<F>>() + first, count);
  MSM_HIP_CHECK(hipGetLastError());
  MSM_HIP_CHECK(hipStreamSynchronize(s));
}

template <int G>
void Bgmw<G>::set_table(const void *tab, size_t n, bool on_device, hipStream_t s) {
  reserve_table(n);
  put_table(tab, 0, table_rows(), on_device, s);
}

template <int G>
void Bgmw<G>::get_table(void *out, size_t first, size_t count, hipStream_t s) {
  typedef typename FieldOf<G>::F F;
  DeviceGuard g(dev_);
  if (first + count > (size_t)h_ * n_) throw std::runtime_error("table range out of bounds");
  if (!count) return;
  DevBuf o;
  o.ensure(count * 96 * G);
  hipLaunchKernelGGL((k_export_affine<G, AffP<F>>), dim3(nblk(count, 256)), dim3(256), 0, s,
                     table_.as<AffP<F>>() + first, o.as<uint64_t>(), count);
  MSM_HIP_CHECK(hipGetLastError());
  MSM_HIP_CHECK(hipMemcpyAsync(out, o.p, count * 96 * G, hipMemcpyDeviceToHost, s));
  MSM_HIP_CHECK(hipStreamSynchronize(s));
}

template <int G>
void Bgmw<G>::run(hipStream_t s, const uint8_t *d_scalars, size_t stride, hfp::Jac<HF> *out) {
  typedef typename FieldOf<G>::F F;
  DeviceGuard g(dev_);
  if (stride < 32) throw std::runtime_error("BGMW95 scalars must be 32-byte strings");
  if (n_ == 0) {
    std::memset(out, 0, sizeof(*out));
    return;
  }
  const size_t n = n_, ne = n * (size_t)h_, NB = bucket_count();
  keys_.ensure(ne * 4);
  vals_.ensure(ne * 4);
  sorted_.ensure(ne * 4 + 64);  // + the accumulation's 16-B payload window past a run's end
  counts_.ensure(NB * 4);
  offsets_.ensure(NB * 4);
  order_.ensure(NB * 4);
  buckets_.ensure(NB * sizeof(Xyzz<F>));
  if (profile_) MSM_HIP_CHECK(hipEventRecord(ev_[0], s));
  hipLaunchKernelGGL(k_bgmw_digits, dim3(nblk(n, 256)), dim3(256), 0, s, d_scalars, stride, n, q_exp_, h_,
                     keys_.as<uint32_t>(), vals_.as<uint32_t>(), (uint32_t)nb0_, small_, (uint32_t)copies_);
  MSM_HIP_CHECK(hipGetLastError());
  if (profile_) MSM_HIP_CHECK(hipEventRecord(ev_[1], s));
  sort_.run(s, keys_.as<uint32_t>(), vals_.as<uint32_t>(), ne, (uint32_t)NB, sorted_.as<uint32_t>(),
            counts_.as<uint32_t>(), offsets_.as<uint32_t>(), order_.as<uint32_t>());
  if (profile_) MSM_HIP_CHECK(hipEventRecord(ev_[2], s));
  launch_accumulate<G>(s, sort_.sched(order_.as<uint32_t>(), sorted_.as<uint32_t>(), 0, NB), table_.as<AffP<F>>(),
                       buckets_.as<Xyzz<F>>(), NB);
  MSM_HIP_CHECK(hipGetLastError());
  if (profile_) MSM_HIP_CHECK(hipEventRecord(ev_[3], s));
  red_.launch(s, buckets_.p);
  if (profile_) MSM_HIP_CHECK(hipEventRecord(ev_[4], s));
  *out = red_.read(s);
  if (profile_) {
    MSM_HIP_CHECK(hipEventRecord(ev_[5], s));
    MSM_HIP_CHECK(hipEventSynchronize(ev_[5]));
    float ms[5];
    for (int k = 0; k < 5; ++k) MSM_HIP_CHECK(hipEventElapsedTime(&ms[k], ev_[k], ev_[k + 1]));
    times_.digits = ms[0];
    times_.sort = ms[1];
    times_.accumulate = ms[2];
    times_.reduce = ms[3];
    times_.finalize = ms[4];
    MSM_HIP_CHECK(hipEventElapsedTime(&times_.total, ev_[0], ev_[5]));
    times_.accumulate_launches = 1;
  }
}

template class Bgmw<MSM_GROUP>;

}  // namespace msm
