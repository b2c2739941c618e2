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
#include <cstring>
#include <map>
#include <memory>

#include "ches_kernels.hpp"
#include "engine.hpp"
#include "pair_kernels.hpp"
#include "pool.hpp"

#ifndef MSM_GROUP
#error "define MSM_GROUP (1 or 2)"
#endif

namespace msm {

template <int G>
struct EntryMsmState {
  DevBuf pts, keys, vals, sorted, counts, offsets, order, buckets, xfer, bx;
  BucketSort sort;
  WeightedReducer<G> red;
  std::vector<uint32_t> planned;  // weights the reducer plan was built for
  size_t device_bytes() const {
    size_t b = 0;
    for (const DevBuf *d : {&pts, &keys, &vals, &sorted, &counts, &offsets, &order, &buckets, &xfer, &bx}) b += d->bytes;
    return b;
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
  S.counts.ensure(nb * 4);
  S.offsets.ensure(nb * 4);
  S.order.ensure(nb * 4);
  S.buckets.ensure(nb * sizeof(Xyzz<F>));
  S.sort.run(s, S.keys.template as<uint32_t>(), S.vals.template as<uint32_t>(), ne, (uint32_t)nb, S.sorted.template as<uint32_t>(),
             S.counts.template as<uint32_t>(), S.offsets.template as<uint32_t>(), S.order.template as<uint32_t>());
  launch_accumulate<G>(s, S.sort.sched(S.order.template as<uint32_t>(), S.sorted.template as<uint32_t>(), 0, nb),
                       S.pts.template as<Aff<F>>(),
                       S.buckets.template as<Xyzz<F>>(), nb);
  MSM_HIP_CHECK(hipGetLastError());
  if (buckets_out) {
    S.bx.ensure(nb * 192 * G);
    hipLaunchKernelGGL(k_export_xyzz<G>, dim3(nblk(nb, 256)), dim3(256), 0, s, S.buckets.template as<Xyzz<F>>(),
                       S.bx.template as<uint64_t>(), nb);
    MSM_HIP_CHECK(hipGetLastError());
    MSM_HIP_CHECK(hipMemcpyAsync(buckets_out, S.bx.p, nb * 192 * G, hipMemcpyDeviceToHost, s));
  }
  plan_if_changed(S, weights, nb);
  S.red.launch(s, S.buckets.p);
  out = S.red.read(s);
  std::memcpy(ret, &out, sizeof out);
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

}  // namespace msm
