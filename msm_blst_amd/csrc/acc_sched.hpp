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

}  // namespace msm
