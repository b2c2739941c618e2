// acc_sched.hpp -- the view of one sorted set that an accumulation launch
// reads (produced by BucketSort, engine.hpp; consumed by k_accumulate /
// k_accumulate2p, kernels.hpp / pair_kernels.hpp).
#pragma once
#include <stdint.h>

namespace msm {

// What an accumulation launch reads for one sorted set, by schedule position
// t: bucket order[t] with counts[t] entries -- entry k at
// ipay[(wbase[w] + k) 64 + t % 64] if its wave group w = t / 64 is
// interleaved, else (wbase[w] == ~0) at sorted[offsets[t] + k]
// (bucket_sort.hpp, k_interleave).
struct AccSched {
  const uint32_t *order, *counts, *offsets, *wbase, *ipay, *sorted;
};
// Set r of a front group sorted in one pass (BucketSort with nsets > 1): its
// schedule arrays start r nb (order, counts, offsets), r nw (wbase) and r ipay
// (ipay) entries after set 0's; `sorted` is shared (offsets index it).
struct AccStride {
  uint64_t nb, nw, ipay;
};
#ifdef __HIPCC__
__host__ __device__ inline AccSched acc_set(const AccSched &S, const AccStride &st, uint32_t r) {
  return AccSched{S.order + r * st.nb, S.counts + r * st.nb,  S.offsets + r * st.nb,
                  S.wbase + r * st.nw, S.ipay + r * st.ipay, S.sorted};
}
#endif

}  // namespace msm
