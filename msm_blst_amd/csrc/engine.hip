// engine.hip -- host orchestration of the plain Pippenger pipeline on one
// MI355X (see kernels.hpp for the kernels).  All launches go to the caller's
// stream; the only host synchronisation is the final 16-window read-back.
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "bucket_sort.hpp"
#include "engine.hpp"
#include "hoststage.hpp"
#include "kernels.hpp"
#include "pair_kernels.hpp"

// compiled once per group (build.py: -DMSM_GROUP=1 and -DMSM_GROUP=2) so the
// two instantiations build in parallel
#ifndef MSM_GROUP
#error "define MSM_GROUP (1 or 2)"
#endif

namespace msm {

#if MSM_GROUP == 1  // group-independent: compiled once
BucketSort::Geom BucketSort::prepare(hipStream_t s, size_t ne, uint32_t nb, int nsets, int ntiles) {
  // ~256 coarse bins (see bucket_sort.hpp), fine buckets per bin in [2^8, 2^12]
  Geom g;
  g.fb_bits = 8;
  while (g.fb_bits < BS_MAX_FB_BITS && ((size_t)nb >> g.fb_bits) > 384) ++g.fb_bits;
  g.ncb = (int)(((size_t)nb + (1u << g.fb_bits) - 1) >> g.fb_bits);
  if (g.ncb > BS_MAX_CB || g.ncb > 4096) throw std::runtime_error("BucketSort: too many buckets");
  if (nsets < 1 || nsets > 65535) throw std::runtime_error("BucketSort: bad set count");
  if (ne * nsets >= (1ull << 32)) throw std::runtime_error("BucketSort: too many entries");
  g.ntiles = ntiles > 0 ? ntiles : (int)std::max<size_t>(1, (ne + BS_TILE - 1) / BS_TILE);
  g.nslots = (size_t)nsets * g.ncb * g.ntiles;
  if (g.nslots >= (1ull << 31)) throw std::runtime_error("BucketSort: too many histogram slots");
  ghist.ensure(g.nslots * 4);
  gbase.ensure(g.nslots * 4);
  okeys.ensure(std::max<size_t>(ne * nsets, 1) * 4);
  ovals.ensure(std::max<size_t>(ne * nsets, 1) * 4);
  wbase.ensure(groups(nb) * nsets * 4);
  ipay_stride = ne + BS_IPAY_SLACK;
  ipay.ensure(ipay_stride * nsets * 4);
  size_t scan_tmp = 0;
  hipcub::DeviceScan::ExclusiveSum(nullptr, scan_tmp, ghist.as<uint32_t>(), gbase.as<uint32_t>(), (int)g.nslots, s);
  tmp.ensure(scan_tmp);
  g.scan_tmp = scan_tmp;
  classes.ensure((size_t)512 * 4 * nsets);  // per set: 256 class totals + 256 cursors, cleared by the hist pass
  scnt.ensure((size_t)nb * nsets * 4);
  soff.ensure((size_t)nb * nsets * 4);
  return g;
}

void BucketSort::scan(hipStream_t s, const Geom &g) {
  size_t tb = g.scan_tmp;
  MSM_HIP_CHECK(
      hipcub::DeviceScan::ExclusiveSum(tmp.p, tb, ghist.as<uint32_t>(), gbase.as<uint32_t>(), (int)g.nslots, s));
}

void BucketSort::run(hipStream_t s, const uint32_t *keys, const uint32_t *vals, size_t ne, uint32_t nb,
                     uint32_t *sorted, uint32_t *counts, uint32_t *offsets, uint32_t *order, int nsets) {
  const Geom g = prepare(s, ne, nb, nsets, 0);
  hipLaunchKernelGGL(k_bs_hist, dim3(g.ntiles, nsets), dim3(256), 0, s, keys, ne, g.fb_bits, g.ncb, g.ntiles,
                     ghist.as<uint32_t>(), classes.as<uint32_t>());
  MSM_HIP_CHECK(hipGetLastError());
  scan(s, g);
  hipLaunchKernelGGL(k_bs_coarse, dim3(g.ntiles, nsets), dim3(256), (size_t)(2 * g.ncb + 2 * BS_TILE) * 4, s, keys,
                     vals, ne, g.fb_bits, g.ncb, g.ntiles, gbase.as<uint32_t>(), okeys.as<uint32_t>(),
                     ovals.as<uint32_t>());
  MSM_HIP_CHECK(hipGetLastError());
  finish(s, g, ne, nb, sorted, counts, offsets, order, nsets);
}

void BucketSort::finish(hipStream_t s, const Geom &g, size_t ne, uint32_t nb, uint32_t *sorted, uint32_t *counts,
                        uint32_t *offsets, uint32_t *order, int nsets) {
  (void)ne;
  const int fb_bits = g.fb_bits, ncb = g.ncb, ntiles = g.ntiles;
  const size_t nw = groups(nb);
  if (fine_bt == 256)
    hipLaunchKernelGGL(k_bs_fine<256>, dim3(ncb, nsets), dim3(256), 0, s, okeys.as<uint32_t>(),
                       ovals.as<uint32_t>(), fb_bits, ncb, ntiles, gbase.as<uint32_t>(), ghist.as<uint32_t>(), nb,
                       sorted, counts, offsets, classes.as<uint32_t>(), nsets);
  else
    hipLaunchKernelGGL(k_bs_fine<1024>, dim3(ncb, nsets), dim3(1024), 0, s, okeys.as<uint32_t>(),
                       ovals.as<uint32_t>(), fb_bits, ncb, ntiles, gbase.as<uint32_t>(), ghist.as<uint32_t>(), nb,
                       sorted, counts, offsets, classes.as<uint32_t>(), nsets);
  MSM_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_sched_scatter, dim3(nblk(nb, SCHED_PER_BLOCK), nsets), dim3(256), 0, s, counts, offsets, nb,
                     classes.as<uint32_t>(), order, scnt.as<uint32_t>(), soff.as<uint32_t>());
  MSM_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_interleave, dim3((unsigned)nw / 4 + 1, nsets), dim3(256), 0, s, scnt.as<uint32_t>(),
                     soff.as<uint32_t>(), nb, (uint32_t)nw, classes.as<uint32_t>(), sorted, ipay.as<uint32_t>(),
                     ipay_stride, wbase.as<uint32_t>());
  MSM_HIP_CHECK(hipGetLastError());
}
#endif


template <int G>
Pippenger<G>::Pippenger(int device, int window_bits) : dev_(device), c_(window_bits) {
  if (c_ < 8 || c_ > 20) throw std::runtime_error("window_bits out of range [8,20]");
  DeviceGuard g(dev_);
  ev_.resize(8);
  for (auto &e : ev_) MSM_HIP_CHECK(hipEventCreate(&e));
}
template <int G>
Pippenger<G>::~Pippenger() {
  for (auto &e : ev_) (void)hipEventDestroy(e);
  for (auto &e : bev_) (void)hipEventDestroy(e);
  for (hipStream_t q : {fstream_, lane1_, tstream_})
    if (q) {
      (void)hipStreamSynchronize(q);
      (void)hipStreamDestroy(q);
    }
  if (host_out_) (void)hipHostFree(host_out_);
  if (up_) {
    (void)hipStreamSynchronize(up_);
    (void)hipStreamDestroy(up_);
    (void)hipEventDestroy(ev_up_);
    (void)hipEventDestroy(ev_s_);
  }
}

template <int G>
size_t Pippenger<G>::device_bytes() const {
  size_t b = stage_ ? stage_->pinned_bytes() : 0;
  for (const DevBuf *d : {&pts_, &buckets_[0], &buckets_[1], &gbuckets_[0], &gbuckets_[1], &tmp_, &scal_}) b += d->bytes;
  for (const ChesFrontSet &f : fs_) b += f.device_bytes();
  return b + red_.device_bytes() + (batch_red_ != &red_ ? bred_.device_bytes() : 0);
}

template <int G>
void Pippenger<G>::set_points(const void *pts, size_t n, bool on_device, hipStream_t s) {
  typedef typename FieldOf<G>::F F;
  DeviceGuard g(dev_);
  if (n == 0) {
    n_ = 0;
    return;
  }
  if (n >= (1ull << 31)) throw std::runtime_error("too many points");
  size_t raw = n * 96 * G;
  const void *src = pts;
  if (!on_device) {
    tmp_.ensure(raw);
    MSM_HIP_CHECK(hipMemcpyAsync(tmp_.p, pts, raw, hipMemcpyHostToDevice, s));
    src = tmp_.p;
  }
  pts_.ensure(n * sizeof(Aff<F>));
  hipLaunchKernelGGL(k_convert_points<G>, dim3(nblk(n, 256)), dim3(256), 0, s, (const uint64_t *)src, pts_.as<Aff<F>>(),
                     n);
  MSM_HIP_CHECK(hipGetLastError());
  n_ = n;
}

template <int C>
static void launch_digits(hipStream_t s, const uint8_t *sc, size_t stride, size_t n, int nbits, int W, uint32_t *keys,
                          uint32_t *vals, const uint8_t *neg, int tcl, int nsets, size_t set_stride) {
  hipLaunchKernelGGL(k_digits<C>, dim3(nblk(n, 256), nsets), dim3(256), 0, s, sc, stride, n, nbits, W, keys, vals, neg,
                     tcl, set_stride);
}

#define MSM_C_DISPATCH(c, FN, ...)                          \
  switch (c) {                                              \
    case 8: FN<8>(__VA_ARGS__); break;                      \
    case 10: FN<10>(__VA_ARGS__); break;                    \
    case 12: FN<12>(__VA_ARGS__); break;                    \
    case 13: FN<13>(__VA_ARGS__); break;                    \
    case 14: FN<14>(__VA_ARGS__); break;                    \
    case 15: FN<15>(__VA_ARGS__); break;                    \
    case 16: FN<16>(__VA_ARGS__); break;                    \
    case 17: FN<17>(__VA_ARGS__); break;                    \
    case 18: FN<18>(__VA_ARGS__); break;                    \
    default: throw std::runtime_error("unsupported window"); \
  }

template <int G>
void Pippenger<G>::front(hipStream_t s, const uint8_t *d_scalars, size_t stride, int nbits, const uint8_t *neg,
                         ChesFrontSet &f, int nsets, size_t set_stride) {
  const int c = c_;
  const int W = (nbits + 1 + c - 1) / c;
  const size_t NB = (size_t)1 << (c - 1);
  const size_t NT = (size_t)W * NB;
  const size_t n = n_, ne = (size_t)W * n;
  f.keys.ensure(ne * nsets * 4);
  f.vals.ensure(ne * nsets * 4);
  f.sorted.ensure(ne * nsets * 4 + 64);  // + the accumulation's 16-B payload window past a run's end
  f.counts.ensure(NT * nsets * 4);
  f.offsets.ensure(NT * nsets * 4);
  f.order.ensure(NT * nsets * 4);
  const bool prof = profile_ && &f == &fs_[0];
  if (prof) MSM_HIP_CHECK(hipEventRecord(ev_[0], s));
  MSM_C_DISPATCH(c, launch_digits, s, d_scalars, stride, n, nbits, W, f.keys.as<uint32_t>(), f.vals.as<uint32_t>(), neg,
                 top_copies_log2(nbits), nsets, set_stride);
  MSM_HIP_CHECK(hipGetLastError());
  if (prof) MSM_HIP_CHECK(hipEventRecord(ev_[1], s));
  f.sort.run(s, f.keys.as<uint32_t>(), f.vals.as<uint32_t>(), ne, (uint32_t)NT, f.sorted.as<uint32_t>(),
             f.counts.as<uint32_t>(), f.offsets.as<uint32_t>(), f.order.as<uint32_t>(), nsets);
  if (prof) MSM_HIP_CHECK(hipEventRecord(ev_[2], s));
}

template <int G>
void Pippenger<G>::accumulate(hipStream_t s, int nbits, ChesFrontSet &f, DevBuf &bk) {
  typedef typename FieldOf<G>::F F;
  const int W = (nbits + 1 + c_ - 1) / c_;
  const size_t NT = (size_t)W << (c_ - 1);
  bk.ensure(NT * sizeof(Xyzz<F>));
  const AccSched sched = f.sort.sched(f.order.as<uint32_t>(), f.sorted.as<uint32_t>(), 0, NT);
  if (ext_rows_)
    launch_accumulate<G>(s, sched, static_cast<const AffP<F> *>(ext_rows_), bk.as<Xyzz<F>>(), NT);
  else
    launch_accumulate<G>(s, sched, pts_.as<Aff<F>>(), bk.as<Xyzz<F>>(), NT);
  MSM_HIP_CHECK(hipGetLastError());
}

template <int G>
void Pippenger<G>::accumulate_sets(hipStream_t s, int nbits, ChesFrontSet &f, int R, DevBuf &bk) {
  typedef typename FieldOf<G>::F F;
  const int W = (nbits + 1 + c_ - 1) / c_;
  const size_t NT = (size_t)W << (c_ - 1);
  launch_accumulate_sets<G>(s, f.sort.sched(f.order.as<uint32_t>(), f.sorted.as<uint32_t>(), 0, NT), f.sort.stride(NT),
                            pts_.as<Aff<F>>(), bk.as<Xyzz<F>>(), NT, R);
  MSM_HIP_CHECK(hipGetLastError());
}

template <int G>
void Pippenger<G>::plan_reduction(int nbits) {
  const int c = c_;
  const int W = (nbits + 1 + c - 1) / c;
  const size_t NB = (size_t)1 << (c - 1);
  const size_t NT = (size_t)W * NB;
  const int tcl = top_copies_log2(nbits);
  if (red_W_ == W && red_tcl_ == tcl) return;
  // bucket (w, b-1) has weight b in window w; top window: slot k holds a copy
  // of bucket (k mod ntop) + 1
  std::vector<uint32_t> wt(NT), win(NT);
  const size_t ntop = NB >> tcl;
  for (size_t k = 0; k < NT; ++k) {
    const size_t w = k / NB, b = k % NB;
    wt[k] = (uint32_t)((w == (size_t)W - 1 ? b % ntop : b) + 1);
    win[k] = (uint32_t)w;
  }
  red_.plan(wt, win, W);
  // A/B knob: the batch reducer's level-0 chunk; 0 (default): red_'s own
  // (chunks of 2 at 2^16) -- with front groups of 4, 0.360 vs 0.385 ms per 2^16
  // MSM for chunks of 8 (profiles/r05_shard_pip_study.txt)
  static const int bc_env = [] {
    const char *e = getenv("MSM_PIP_L0_CHUNK");
    return e ? std::max(0, std::min(64, atoi(e))) : 0;
  }();
  if (bc_env && red_.level0_chunk() != bc_env) {
    bred_.plan(wt, win, W, bc_env);
    batch_red_ = &bred_;
  } else {
    batch_red_ = &red_;
  }
  red_W_ = W;
  red_tcl_ = tcl;
}

template <int G>
void Pippenger<G>::back(hipStream_t s, int nbits, hfp::Jac<HF> *out) {
  const int c = c_;
  accumulate(s, nbits, fs_[0], buckets_[0]);
  if (profile_) MSM_HIP_CHECK(hipEventRecord(ev_[3], s));
  plan_reduction(nbits);
  red_.launch(s, buckets_[0].p);
  if (profile_) MSM_HIP_CHECK(hipEventRecord(ev_[4], s));
  *out = red_.read_total(s, c);
  if (profile_) MSM_HIP_CHECK(hipEventRecord(ev_[5], s));
  if (profile_) {
    float ms;
    MSM_HIP_CHECK(hipEventSynchronize(ev_[5]));
    MSM_HIP_CHECK(hipEventElapsedTime(&ms, ev_[0], ev_[1]));
    times_.digits = ms;
    MSM_HIP_CHECK(hipEventElapsedTime(&ms, ev_[1], ev_[2]));
    times_.sort = ms;
    MSM_HIP_CHECK(hipEventElapsedTime(&ms, ev_[2], ev_[3]));
    times_.accumulate = ms;
    MSM_HIP_CHECK(hipEventElapsedTime(&ms, ev_[3], ev_[4]));
    times_.reduce = ms;
    MSM_HIP_CHECK(hipEventElapsedTime(&ms, ev_[4], ev_[5]));
    times_.finalize = ms;
    MSM_HIP_CHECK(hipEventElapsedTime(&ms, ev_[0], ev_[5]));
    times_.total = ms;
    times_.accumulate_launches = 1;
  }
}

template <int G>
void Pippenger<G>::run(hipStream_t s, const uint8_t *d_scalars, size_t stride, int nbits, hfp::Jac<HF> *out) {
  DeviceGuard g(dev_);
  if (nbits < 1 || nbits > 256) throw std::runtime_error("nbits must be in [1,256]");
  if (n_ == 0) {
    *out = hfp::Jac<HF>{hfp::fzero(HF()), hfp::fzero(HF()), hfp::fzero(HF())};
    return;
  }
  fs_[0].sort.fine_bt = 1024;  // alone on the chip: the 1024-thread fine pass
  front(s, d_scalars, stride, nbits, nullptr, fs_[0]);
  back(s, nbits, out);
}

template <int G>
void Pippenger<G>::run_batch(hipStream_t s, const uint8_t *d_scalars, size_t stride, size_t set_stride, size_t count,
                             int nbits, hfp::Jac<HF> *outs) {
  typedef typename FieldOf<G>::F F;
  DeviceGuard g(dev_);
  if (nbits < 1 || nbits > 256) throw std::runtime_error("nbits must be in [1,256]");
  if (count == 0) return;
  if (n_ == 0) {
    for (size_t k = 0; k < count; ++k) outs[k] = hfp::Jac<HF>{hfp::fzero(HF()), hfp::fzero(HF()), hfp::fzero(HF())};
    return;
  }
  const int W = (nbits + 1 + c_ - 1) / c_;
  const size_t NT = (size_t)W << (c_ - 1);
  plan_reduction(nbits);
  WeightedReducer<G> &red = *batch_red_;
  if (!fstream_) {
    int least = 0, greatest = 0;
    MSM_HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    MSM_HIP_CHECK(hipStreamCreateWithPriority(&fstream_, hipStreamNonBlocking, greatest));
    MSM_HIP_CHECK(hipStreamCreateWithFlags(&lane1_, hipStreamNonBlocking));
    MSM_HIP_CHECK(hipStreamCreateWithFlags(&tstream_, hipStreamNonBlocking));
  }
  // the dense stage of the batch's last group over 4 waves per add (nothing left
  // to overlap it with; MSM_TAIL_COOP=0: one lane per add)
  static const bool tail_coop = [] {
    const char *e = getenv("MSM_TAIL_COOP");
    return !e || atoi(e) != 0;
  }();
  // groups of R <= kGroup MSMs share one reduction tail (WeightedReducer batch groups)
  static const size_t group_max = [] {  // A/B knob: MSMs per reduction group
    const char *e = getenv("MSM_PIP_GROUP");
    return (size_t)(e ? std::max(1, std::min(32, atoi(e))) : kGroup);
  }();
  // Front groups: the digits + sort of up to fg_max sets in ONE pass per stage
  // (7 launches per group instead of per MSM), the group's accumulations in ONE
  // launch (k_accumulate_sets) and its level 0s in one launch per reduction
  // group.  A 2^16 MSM's front (digits + two-level sort of 1.25 M entries) took
  // as long as its accumulation beside the other lane's work, so one front per
  // MSM on the front stream set the period (profiles/r05_small_trace.txt).
  // Groups ramp 1, 1, 2, 4, ... so the first accumulation starts after one
  // front.  MSM_PIP_FRONT_GROUP=<1..8> (1: one MSM per launch, round 4's schedule).
  static const size_t fg_env = [] {
    const char *e = getenv("MSM_PIP_FRONT_GROUP");
    return (size_t)(e ? std::max(1, std::min(8, atoi(e))) : 4);
  }();
  const size_t fg_max = fg_env;
  const std::vector<size_t> fgb = front_groups(count, fg_max);
  const size_t nfg = fgb.size() - 1;
  const size_t ngroups = (count + group_max - 1) / group_max, R = (count + ngroups - 1) / ngroups;
  const size_t ob = red.out_bytes();
  if (host_out_bytes_ < count * ob) {
    if (host_out_) (void)hipHostFree(host_out_);
    host_out_ = nullptr;
    host_out_bytes_ = 0;
    const size_t bytes = std::max<size_t>(count, 64) * ob;
    MSM_HIP_CHECK(hipHostMalloc(&host_out_, bytes, hipHostMallocDefault));
    host_out_bytes_ = bytes;
  }
  // every buffer the pipeline touches exists before its first launch (an
  // allocation inside the issue loop would synchronise the device): bucket
  // sets for a whole front group on each lane, reducer sets, and every front
  // set sized for a whole group (sized by one untimed front of fg_max copies of
  // set 0, outside the pipeline)
  // Front phase (MSM_FRONT_PHASE=1; off: measured slower, Ches::run_jobs): one
  // front set per front group, up to kFrontPhase (~4 GiB of front sets at
  // most), the first accumulation waiting for every front of the phase
  static const bool phase_env = [] {
    const char *e = getenv("MSM_FRONT_PHASE");
    return e && atoi(e) != 0;
  }();
  const size_t fs_bytes = fg_max * (size_t)W * n_ * 24 + 1;  // ~ one front set (keys, vals, sorted, sort scratch)
  const int nfr = phase_env ? (int)std::max<size_t>(kFronts, std::min<size_t>(kFrontPhase, ((size_t)4 << 30) / fs_bytes))
                            : kFronts;
  if ((int)fs_.size() < nfr) fs_.resize(nfr);
  // the batch fronts' fine-pass workgroup (bucket_sort.hpp k_bs_fine): 1024
  // threads, or MSM_PIP_FINE_BT=256 (fits beside the accumulation waves)
  static const int fine_bt = [] {
    const char *e = getenv("MSM_PIP_FINE_BT");
    return e && atoi(e) == 256 ? 256 : 1024;
  }();
  for (ChesFrontSet &f : fs_) f.sort.fine_bt = fine_bt;
  for (DevBuf &b : gbuckets_) b.ensure(fg_max * NT * sizeof(Xyzz<F>));
  for (int t = 0; t < kRedSets; ++t) red.ensure_group(t, (int)group_max);
  for (int f = 0; f < nfr; ++f)
    if (fs_[f].sorted.bytes < (size_t)W * n_ * fg_max * 4 + 64)
      front(s, d_scalars, stride, nbits, nullptr, fs_[f], (int)fg_max, 0);
  MSM_HIP_CHECK(hipStreamSynchronize(s));
  while (bev_.size() < 2 * count + nfg + ngroups + 1) {
    hipEvent_t e;
    MSM_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    bev_.push_back(e);
  }
  hipEvent_t *eva = bev_.data() + 1, *evh = eva + count, *evf = evh + count, *evt = evf + nfg;
  MSM_HIP_CHECK(hipEventRecord(bev_[0], s));
  for (hipStream_t q : {fstream_, lane1_, tstream_}) MSM_HIP_CHECK(hipStreamWaitEvent(q, bev_[0], 0));
  auto front_group = [&](size_t g) {
    if (g >= nfg) return;
    if (g >= (size_t)nfr)  // front set g % nfr: group g - nfr's accumulation has read it
      MSM_HIP_CHECK(hipStreamWaitEvent(fstream_, eva[fgb[g - nfr + 1] - 1], 0));
    front(fstream_, d_scalars + fgb[g] * set_stride, stride, nbits, nullptr, fs_[g % nfr],
          (int)(fgb[g + 1] - fgb[g]), set_stride);
    MSM_HIP_CHECK(hipEventRecord(evf[g], fstream_));
  };
  // accumulation groups alternate between two lane streams (the caller's and
  // lane1_); group tails on tstream_
  hipStream_t lane[2] = {s, lane1_};
  // fronts run up to kFronts - 1 groups ahead, each ENQUEUED after the
  // accumulation before it (enqueuing four fronts before the first accumulation
  // cost ~0.3 ms of host time per batch); front g + 1 is always enqueued before
  // accumulation g + 1 waits on it
  size_t fronts_issued = 0;
  auto issue_fronts = [&](size_t upto) {
    for (; fronts_issued <= upto && fronts_issued < nfg; ++fronts_issued) front_group(fronts_issued);
  };
  const size_t nphase = phase_env ? std::min(nfg, (size_t)nfr) : 1;  // fronts before the first accumulation
  issue_fronts(nphase - 1);
  for (size_t g = 0; g < nfg; ++g) {
    const size_t k0 = fgb[g], k1 = fgb[g + 1];
    const int gb = (int)(g & 1);
    hipStream_t L = lane[gb];
    MSM_HIP_CHECK(hipStreamWaitEvent(L, evf[g], 0));
    if (g == 0 && nphase > 1) MSM_HIP_CHECK(hipStreamWaitEvent(L, evf[nphase - 1], 0));  // the front phase
    accumulate_sets(L, nbits, fs_[g % nfr], (int)(k1 - k0), gbuckets_[gb]);  // bucket sets: lane gb only, in order
    for (size_t k = k0; k < k1; ++k) MSM_HIP_CHECK(hipEventRecord(eva[k], L));
    for (size_t a = k0; a < k1;) {  // level 0, one launch per reduction group touched
      const size_t q = a / R, b = std::min(k1, (q + 1) * R);
      if (q >= (size_t)kRedSets) MSM_HIP_CHECK(hipStreamWaitEvent(L, evt[q - kRedSets], 0));  // reducer set free again
      red.launch_head_slots(L, gbuckets_[gb].as<uint8_t>() + (a - k0) * NT * sizeof(Xyzz<F>), NT,
                            (int)(q % kRedSets), (int)(a % R), (int)(b - a));
      a = b;
    }
    for (size_t k = k0; k < k1; ++k) MSM_HIP_CHECK(hipEventRecord(evh[k], L));
    for (size_t k = k0; k < k1; ++k) {  // tails of the reduction groups ending in [k0, k1)
      if ((k + 1) % R != 0 && k + 1 != count) continue;
      const size_t q = k / R, first = q * R;
      MSM_HIP_CHECK(hipStreamWaitEvent(tstream_, evh[k], 0));                                     // this lane's level 0s
      if (k0 >= 1 && k0 - 1 >= first) MSM_HIP_CHECK(hipStreamWaitEvent(tstream_, evh[k0 - 1], 0));  // the other lane's
      red.launch_tail_group(tstream_, (int)(q % kRedSets), (int)(k - first + 1), tail_coop && k + 1 == count);
      red.copy_out_group(tstream_, (int)(q % kRedSets), (int)(k - first + 1), (uint8_t *)host_out_ + first * ob);
      MSM_HIP_CHECK(hipEventRecord(evt[q], tstream_));
    }
    issue_fronts(g + nfr - 1);
  }
  // the host Horner of group q (one per MSM, ~W c doublings each) overlaps the
  // GPU work of later groups, spread over the host worker threads
  for (size_t q = 0; q * R < count; ++q) {
    MSM_HIP_CHECK(hipEventSynchronize(evt[q]));
    const size_t k0 = q * R, k1 = std::min(count, (q + 1) * R);
    WorkerPool::get().parallel_for(k1 - k0, [&](size_t i) {
      outs[k0 + i] = red.combine_windows((const uint8_t *)host_out_ + (k0 + i) * ob, c_);
    });
  }
  // the caller's stream observes completion of every stream of the batch
  for (hipStream_t q : {fstream_, lane1_, tstream_}) {
    MSM_HIP_CHECK(hipEventRecord(bev_[0], q));
    MSM_HIP_CHECK(hipStreamWaitEvent(s, bev_[0], 0));
  }
}

// The blst drop-in (abi.cpp blst_p{1,2}s_mult_pippenger / _tile_pippenger):
// points and scalars in the caller's host memory, uploaded through the
// engine's pinned ring (hoststage.hpp).  The scalars go up first and their
// digits + sort are enqueued; the 96 n G bytes of points then upload (and
// convert) on a second stream while the GPU sorts, and the accumulation waits
// for them.  tile != nullptr: one blst window tile -- k_tile_booth turns the
// raw scalars into |Booth digit| + sign on the device, and the plain pipeline
// multiplies with |d| (cbits + 1 bits) and the signs.
template <int G>
void Pippenger<G>::run_host(hipStream_t s, const void *pts_blst, size_t n, const uint8_t *scalars, size_t stride,
                            int nbits, hfp::Jac<HF> *out, const TileSpec *tile, const void *dev_rows) {
  typedef typename FieldOf<G>::F F;
  DeviceGuard g(dev_);
  if (nbits < 1 || nbits > 256) throw std::runtime_error("nbits must be in [1,256]");
  if (n >= (1ull << 31)) throw std::runtime_error("too many points");
  n_ = n;
  if (n == 0) {
    *out = hfp::Jac<HF>{hfp::fzero(HF()), hfp::fzero(HF()), hfp::fzero(HF())};
    return;
  }
  if (!up_) {
    MSM_HIP_CHECK(hipStreamCreateWithFlags(&up_, hipStreamNonBlocking));
    MSM_HIP_CHECK(hipEventCreateWithFlags(&ev_up_, hipEventDisableTiming));
    MSM_HIP_CHECK(hipEventCreateWithFlags(&ev_s_, hipEventDisableTiming));
  }
  if (!stage_) stage_ = std::make_unique<HostStager>();
  // the point upload (stream up_) must not overwrite points an earlier MSM on s
  // still reads: awaited on the host (an earlier call ended with its read-back,
  // so this returns at once), not by a cross-stream wait -- copies enqueued
  // behind such a wait now and then blocked the host for 7-9 ms
  // (profiles/r05_h2d_block.txt).  The upload overlaps this call's digits + sort.
  MSM_HIP_CHECK(hipEventRecord(ev_s_, s));
  MSM_HIP_CHECK(hipEventSynchronize(ev_s_));
  const size_t sbytes = n * stride;
  scal_.ensure(sbytes + (tile ? n * 5 : 0) + 16);
  stage_->upload(scal_.p, scalars, sbytes, s);
  fs_[0].sort.fine_bt = 1024;  // a batch may have left its setting
  if (tile) {
    uint32_t *mag = reinterpret_cast<uint32_t *>(scal_.as<uint8_t>() + ((sbytes + 3) & ~(size_t)3));
    uint8_t *neg = reinterpret_cast<uint8_t *>(mag + n);
    hipLaunchKernelGGL(k_tile_booth, dim3(nblk(n, 256)), dim3(256), 0, s, scal_.as<uint8_t>(), stride, n, nbits,
                       tile->bit0, tile->wbits, tile->cbits, mag, neg);
    MSM_HIP_CHECK(hipGetLastError());
    nbits = tile->cbits + 1;
    front(s, reinterpret_cast<const uint8_t *>(mag), 4, nbits, neg, fs_[0]);
  } else {
    front(s, scal_.as<uint8_t>(), stride, nbits, nullptr, fs_[0]);
  }
  if (dev_rows) {  // registered points: resident already, nothing to upload
    ext_rows_ = dev_rows;
    try {
      back(s, nbits, out);
    } catch (...) {
      ext_rows_ = nullptr;
      throw;
    }
    ext_rows_ = nullptr;
    return;
  }
  const size_t raw = n * 96 * G;
  tmp_.ensure(raw);
  pts_.ensure(n * sizeof(Aff<F>));
  stage_->upload(tmp_.p, pts_blst, raw, up_);
  hipLaunchKernelGGL(k_convert_points<G>, dim3(nblk(n, 256)), dim3(256), 0, up_, tmp_.as<uint64_t>(),
                     pts_.as<Aff<F>>(), n);
  MSM_HIP_CHECK(hipGetLastError());
  MSM_HIP_CHECK(hipEventRecord(ev_up_, up_));
  MSM_HIP_CHECK(hipStreamWaitEvent(s, ev_up_, 0));
  back(s, nbits, out);
}

template class Pippenger<MSM_GROUP>;

// ---------------------------------------------------------------------------
// device unit-test entry points (parity tests of the field / curve layers)
// ---------------------------------------------------------------------------
template <int G>
__global__ void __launch_bounds__(64) k_test_field(int op, const uint64_t *a, const uint64_t *b, uint64_t *out, size_t n) {
  typedef typename FieldOf<G>::F F;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  F x, y, r;
  f_from_blst(x, a + i * 6 * G);
  f_from_blst(y, b + i * 6 * G);
  if (op == 0) {
    f_mul(r, x, y);
  } else if (op == 1) {
    f_add(r, x, y);
  } else if (op == 2) {
    f_sub4(r, x, y);
  } else {
    f_sqr(r, x);
  }
  f_to_blst(out + i * 6 * G, r);
}

// blst Jacobian (X ZZ, Y ZZZ, ZZ) of an xyzz sum, canonical; infinity -> zeros
template <class F>
__device__ __forceinline__ void test_export_jac(uint64_t *o, const Xyzz<F> &a) {
  constexpr int L = (int)(sizeof(F) / sizeof(Fp)) * 18;
  if (xyzz_is_inf(a)) {
    for (int j = 0; j < L; ++j) o[j] = 0;
    return;
  }
  F X, Y;
  f_mul(X, a.x, a.zz);
  f_mul(Y, a.y, a.zzz);
  f_to_blst(o, X);
  f_to_blst(o + L / 3, Y);
  f_to_blst(o + 2 * L / 3, a.zz);
}

// xyzz sequences: thread i applies ops[i*len .. ] = (point index | sign<<31), then 2*acc via xyzz_add
// (G1: one lane per sequence, the arithmetic of k_accumulate / k_segsum)
template <int G>
__global__ void __launch_bounds__(64) k_test_xyzz(const uint64_t *pts_blst, const uint32_t *ops, int len, size_t nseq, uint64_t *out) {
  typedef typename FieldOf<G>::F F;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nseq) return;
  Xyzz<F> acc;
  xyzz_set_inf(acc);
  for (int k = 0; k < len; ++k) {
    uint32_t o = ops[i * len + k];
    if (o == 0xffffffffu) continue;
    Aff<F> p;
    const uint64_t *src = pts_blst + (size_t)(o & 0x7fffffffu) * 12 * G;
    f_from_blst(p.x, src);
    f_from_blst(p.y, src + 6 * G);
    if (f_is_zero_exact(p.x) && f_is_zero_exact(p.y)) continue;
    xyzz_madd(acc, p, (o >> 31) != 0);
  }
  test_export_jac(out + i * 2 * 18 * G, acc);
  Xyzz<F> a1 = acc;
  xyzz_add(acc, a1);
  test_export_jac(out + (i * 2 + 1) * 18 * G, acc);
}

// the same for G2 on lane pairs (fp2l.hpp), the arithmetic every G2 product
// kernel runs (k_accumulate2p, k_segsum2p, the lane-pair tails): lanes 2i,
// 2i + 1 hold component 0 / 1 of sequence i
__device__ __forceinline__ void test_export_jac2l(uint64_t *o, const Xyzz<Fp2L> &a, int comp) {
  if (xyzz_is_inf(a)) {  // uniform per pair
    for (int j = 0; j < 6; ++j) o[6 * comp + j] = o[12 + 6 * comp + j] = o[24 + 6 * comp + j] = 0;
    return;
  }
  Fp2L X, Y;
  f_mul(X, a.x, a.zz);
  f_mul(Y, a.y, a.zzz);
  fp_to_blst(o + 6 * comp, X.c);
  fp_to_blst(o + 12 + 6 * comp, Y.c);
  fp_to_blst(o + 24 + 6 * comp, a.zz.c);
}
static __global__ void __launch_bounds__(64)
    k_test_xyzz2p(const uint64_t *pts_blst, const uint32_t *ops, int len, size_t nseq, uint64_t *out) {
  const size_t tt = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tt >= 2 * nseq) return;  // whole pairs only
  const int comp = (int)(tt & 1);
  const size_t i = tt >> 1;
  Xyzz<Fp2L> acc;
  xyzz_set_inf(acc);
  for (int k = 0; k < len; ++k) {
    uint32_t o = ops[i * len + k];
    if (o == 0xffffffffu) continue;
    Aff<Fp2L> p;
    const uint64_t *src = pts_blst + (size_t)(o & 0x7fffffffu) * 24;
    fp_from_blst(p.x.c, src + 6 * comp);
    fp_from_blst(p.y.c, src + 12 + 6 * comp);
    if (f_is_zero_exact(p.x) && f_is_zero_exact(p.y)) continue;
    xyzz_madd(acc, p, (o >> 31) != 0);
  }
  test_export_jac2l(out + i * 2 * 36, acc, comp);
  Xyzz<Fp2L> a1 = acc;
  xyzz_add(acc, a1);
  test_export_jac2l(out + (i * 2 + 1) * 36, acc, comp);
}

template <int G>
void test_field(int op, const uint64_t *a, const uint64_t *b, uint64_t *out, size_t n) {
  DevBuf da, db, dout;
  size_t bytes = n * 48 * G;
  da.ensure(bytes);
  db.ensure(bytes);
  dout.ensure(bytes);
  MSM_HIP_CHECK(hipMemcpy(da.p, a, bytes, hipMemcpyHostToDevice));
  MSM_HIP_CHECK(hipMemcpy(db.p, b, bytes, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_test_field<G>, dim3(nblk(n, 64)), dim3(64), 0, 0, op, da.as<uint64_t>(), db.as<uint64_t>(),
                     dout.as<uint64_t>(), n);
  MSM_HIP_CHECK(hipGetLastError());
  MSM_HIP_CHECK(hipMemcpy(out, dout.p, bytes, hipMemcpyDeviceToHost));
}
template <int G>
void test_xyzz(const uint64_t *pts, size_t npts, const uint32_t *ops, int len, size_t nseq, uint64_t *out) {
  DevBuf dp, dops, dout;
  dp.ensure(npts * 96 * G);
  dops.ensure(nseq * len * 4 + 4);
  dout.ensure(nseq * 2 * 144 * G);
  MSM_HIP_CHECK(hipMemcpy(dp.p, pts, npts * 96 * G, hipMemcpyHostToDevice));
  MSM_HIP_CHECK(hipMemcpy(dops.p, ops, nseq * len * 4, hipMemcpyHostToDevice));
  if constexpr (G == 2)
    hipLaunchKernelGGL(k_test_xyzz2p, dim3(nblk(2 * nseq, 64)), dim3(64), 0, 0, dp.as<uint64_t>(), dops.as<uint32_t>(),
                       len, nseq, dout.as<uint64_t>());
  else
    hipLaunchKernelGGL(k_test_xyzz<G>, dim3(nblk(nseq, 64)), dim3(64), 0, 0, dp.as<uint64_t>(), dops.as<uint32_t>(),
                       len, nseq, dout.as<uint64_t>());
  MSM_HIP_CHECK(hipGetLastError());
  MSM_HIP_CHECK(hipMemcpy(out, dout.p, nseq * 2 * 144 * G, hipMemcpyDeviceToHost));
}
template void test_field<MSM_GROUP>(int, const uint64_t *, const uint64_t *, uint64_t *, size_t);
template void test_xyzz<MSM_GROUP>(const uint64_t *, size_t, const uint32_t *, int, size_t, uint64_t *);

}  // namespace msm
