// ches.hip -- host orchestration of the CHES "nh + q/5" bucket-set MSM
// (LuoGuiwen/MSM_blst, method `pippenger_variant_q_over_5_CHES`,
// ref main_p1.cpp:192-246) on one MI355X.
//
// Setup (once per context): parameters of ref ches_config_files, bucket set B
// (ref auxiliaryfunc.h:257-288), digit hash (ref main_p1.cpp:140-152) and the
// precomputed table T[3(i h + j) + m - 1] = m q^j P_i (ref main_p1.cpp:155-172),
// the latter built on the GPU and kept resident in HBM in the engine's
// internal limb layout.
//
// Per MSM (all on device, one stream):
//   digits   k_ches_digits: MB radix-q digits + per-bucket counts/ranks
//   sort     exclusive scan of counts, k_ches_scatter, bucket schedule by size
//   accum    k_accumulate: one lane per bucket, xyzz += +-T[slot]
//   reduce   WeightedReducer: sum_i B[i] S_i (replaces the d-trick loop of
//            ref multi_scalar.c:301-321 with a GPU-parallel regrouping)
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "ches_kernels.hpp"
#include "coop.hpp"
#include "engine.hpp"
#include "hoststage.hpp"
#include "pair_kernels.hpp"

#ifndef MSM_GROUP
#error "define MSM_GROUP (1 or 2)"
#endif

namespace msm {

#if MSM_GROUP == 1  // group-independent host setup: compiled once
// ------------------------------------------------------------- parameters --
// values of ref ches_config_files/config_file_n_exp_{8..21}.h and the _beta
// variants (n_exp, beta, q exponent, h, a_h, d_max, |B|, BGMW95 q exponent, h)
static const ChesParams kChesTable[] = {
    {8, 0, 12, 22, 7, 6, 857, 10, 26},         {9, 0, 13, 20, 231, 6, 1725, 11, 24},
    {10, 0, 13, 20, 231, 6, 1725, 12, 22},     {11, 0, 14, 19, 7, 6, 3417, 13, 20},
    {12, 0, 14, 19, 7, 6, 3417, 13, 20},       {13, 0, 16, 16, 29677, 6, 18343, 15, 17},
    {14, 0, 16, 16, 29677, 6, 18343, 15, 17},  {15, 0, 16, 16, 29677, 6, 18343, 16, 16},
    {16, 0, 19, 14, 231, 6, 109244, 17, 15},   {16, 1, 18, 15, 7, 6, 54618, 17, 15},
    {17, 0, 20, 13, 29677, 6, 220931, 17, 15}, {17, 1, 19, 14, 231, 6, 109244, 17, 15},
    {18, 0, 20, 13, 29677, 6, 220931, 19, 14}, {19, 0, 20, 13, 29677, 6, 220931, 20, 13},
    {20, 0, 22, 12, 7419, 6, 874437, 20, 13},  {20, 1, 20, 13, 29677, 6, 220931, 20, 13},
    {21, 0, 22, 12, 7419, 6, 874437, 22, 12},
};

bool ches_params_for(int n_exp, int beta, ChesParams *out) {
  for (const ChesParams &p : kChesTable)
    if (p.n_exp == n_exp && p.beta == beta) {
      *out = p;
      return true;
    }
  return false;
}

// omega2(v) + omega3(v) even  (ref auxiliaryfunc.h:217-255)
static bool even23(int v) {
  int e = 0;
  while (v % 2 == 0) v /= 2, ++e;
  while (v % 3 == 0) v /= 3, ++e;
  return (e & 1) == 0;
}

// ref auxiliaryfunc.h:257-288: {0,1} u {i <= q/2 : even23(i)}, then the two
// pruning passes (membership tested as the passes run, as std::set::erase
// does there), then every even23 value <= a_h + 1 re-inserted.
std::vector<int> ches_bucket_set(int q, int a_h) {
  size_t lim = std::max<size_t>((size_t)q / 2 + 1, (size_t)a_h + 2);
  std::vector<uint8_t> in(lim, 0);
  in[0] = in[1] = 1;
  for (int i = 2; i <= q / 2; ++i) in[i] = even23(i);
  for (int i = q / 4; i < q / 2; ++i) {
    int t = q - 2 * i;
    if (in[i] && t >= 0 && (size_t)t < lim && in[t]) in[t] = 0;
  }
  for (int i = q / 6; i < q / 4; ++i) {
    int t = q - 3 * i;
    if (in[i] && t >= 0 && (size_t)t < lim && in[t]) in[t] = 0;
  }
  for (int i = 1; i <= a_h + 1; ++i)
    if (even23(i)) in[i] = 1;
  std::vector<int> B;
  for (size_t v = 0; v < lim; ++v)
    if (in[v]) B.push_back((int)v);
  return B;
}

// ref main_p1.cpp:140-152: every (m, b) writes H[q - m b] = (m, b, alpha=1),
// then H[m b] = (m, b, 0); later writes win.  Packed per ches_kernels.hpp.
std::vector<uint32_t> ches_digit_hash(const std::vector<int> &B, int q) {
  std::vector<uint32_t> H((size_t)q + 1, 0);
  for (int alpha = 1; alpha >= 0; --alpha)
    for (int m = 1; m <= 3; ++m)
      for (size_t i = 0; i < B.size(); ++i) {
        long mb = (long)m * B[i];
        if (mb > q) continue;
        size_t d = alpha ? (size_t)(q - mb) : (size_t)mb;
        H[d] = (uint32_t)i | ((uint32_t)(m - 1) << 24) | ((uint32_t)alpha << 31);
      }
  return H;
}

void ches_digit_code(const std::vector<int> &B, int q, std::vector<uint32_t> &code, std::vector<uint32_t> &rank) {
  const std::vector<uint32_t> H = ches_digit_hash(B, q);
  code.assign(((size_t)q >> 3) + 2, 0);
  for (size_t d = 0; d <= (size_t)q; ++d) {
    const uint32_t m = ((H[d] >> 24) & 3u) + 1, alpha = H[d] >> 31;
    const int b = B[H[d] & CH_IDX_MASK];
    uint32_t c = (m - 1) | (alpha << 2);
    if (b == 0) {
      c |= 8u;  // bucket value 0: entry skipped
    } else {
      const long v = alpha ? (long)q - (long)d : (long)d;
      if (v % m != 0 || v / m != b) throw std::runtime_error("CHES digit map is not arithmetic at d=" + std::to_string(d));
    }
    code[d >> 3] |= c << (4 * (d & 7));
  }
  const size_t words = ((size_t)B.back() >> 5) + 1;
  rank.assign(2 * words, 0);
  for (int v : B) rank[2 * ((size_t)v >> 5)] |= 1u << (v & 31);
  uint32_t run = 0;
  for (size_t w = 0; w < words; ++w) {
    rank[2 * w + 1] = run;
    run += (uint32_t)__builtin_popcount(rank[2 * w]);
  }
}
#endif  // MSM_GROUP == 1

// a tail level of segment sums: few outputs are latency-bound, so one add
// spreads over 4 waves (coop.hpp: G1 one lane per wave, G2 a lane pair per wave);
// nmsm > 1: the MSMs of a batch group, src / dst advanced by their strides
template <int G>
static void launch_segsum_tail(hipStream_t s, const Xyzz<typename FieldOf<G>::F> *src, const uint32_t *ix,
                               const uint32_t *st, Xyzz<typename FieldOf<G>::F> *dst, size_t nout, bool coop,
                               int nmsm = 1, size_t sstride = 0, size_t dstride = 0) {
  if (coop && nout * (size_t)nmsm <= 16384) {
    if constexpr (G == 1)
      hipLaunchKernelGGL(k_segsum_c<G>, dim3(nblk(nout, 64), (unsigned)nmsm), dim3(256), 0, s, src, ix, st, dst, nout,
                         sstride, dstride);
    else
      hipLaunchKernelGGL(k_segsum_c2p, dim3(nblk(nout, 32), (unsigned)nmsm), dim3(256), 0, s, src, ix, st, dst, nout,
                         sstride, dstride);
  } else {
    launch_segsum<G>(s, src, ix, st, dst, nout, nmsm, sstride, dstride);
  }
}

// -------------------------------------------------------------- scan reduce --
// coop levels of the dense stage: only those with at most this many adds.  A
// 4-wave add is the shortest latency for a narrow level, but its waves are 4x
// the one-lane form's: a suffix step over a batch group's 20 x 2 x 1024 slots
// ran 24 us per level coop (0.8 rounds of wave slots, 2.5 waves per SIMD
// sharing issue) -- the batch's last, exposed tail (profiles/r06_small_trace.txt).
// MSM_DENSE_COOP_MAX=<adds> overrides (0: every level one lane per add).
static size_t dense_coop_max() {
  static const size_t v = [] {
    const char *e = getenv("MSM_DENSE_COOP_MAX");
    return e ? (size_t)std::max(0, atoi(e)) : (size_t)16384;
  }();
  return v;
}

template <int G>
void ScanReducer<G>::launch(hipStream_t s, const void *Abuf, int W, int S, bool coop_req) {
  typedef typename FieldOf<G>::F F;
  if (S < 1 || (S & (S - 1))) throw std::runtime_error("ScanReducer: S must be a power of two");
  const size_t NT = (size_t)W * S;
  bool coop = coop_req && NT <= dense_coop_max();  // the suffix steps: NT adds each
  buf[0].ensure(NT * sizeof(Xyzz<F>));
  buf[1].ensure(NT * sizeof(Xyzz<F>));
  fin.ensure((size_t)W * 144 * G);
  const Xyzz<F> *src = reinterpret_cast<const Xyzz<F> *>(Abuf);
  int cur = 0;
  for (int d = 1; d < S; d <<= 1) {  // suffix sums T_k = sum_{b >= k} A_b
    Xyzz<F> *dst = buf[cur].as<Xyzz<F>>();
    if constexpr (G == 2) {  // lane pairs (fp2l.hpp); coop: one add over 4 waves (coop.hpp)
      if (coop)
        hipLaunchKernelGGL(k_suffix_step_c2p, dim3(nblk(NT, 32)), dim3(256), 0, s, src, dst, S, d, W);
      else
        hipLaunchKernelGGL(k_suffix_step2p, dim3(nblk(2 * NT, 64)), dim3(64), 0, s, src, dst, S, d, W);
    } else {
      if (coop) hipLaunchKernelGGL(k_suffix_step_c<G>, dim3(nblk(NT, 64)), dim3(256), 0, s, src, dst, S, d, W);
      else hipLaunchKernelGGL(k_suffix_step<G>, dim3(nblk(NT, 64)), dim3(64), 0, s, src, dst, S, d, W);
    }
    MSM_HIP_CHECK(hipGetLastError());
    src = dst;
    cur ^= 1;
  }
  for (size_t len = NT; len > (size_t)W; len >>= 1) {  // sum_k T_k = sum_b b A_b
    Xyzz<F> *dst = buf[cur].as<Xyzz<F>>();
    coop = coop_req && len / 2 <= dense_coop_max();  // this pair step: len / 2 adds
    if constexpr (G == 2) {
      if (coop)
        hipLaunchKernelGGL(k_pair_step_c2p, dim3(nblk(len / 2, 32)), dim3(256), 0, s, src, dst, len / 2);
      else
        hipLaunchKernelGGL(k_pair_step2p, dim3(nblk(len, 64)), dim3(64), 0, s, src, dst, len / 2);
    } else {
      if (coop) hipLaunchKernelGGL(k_pair_step_c<G>, dim3(nblk(len / 2, 64)), dim3(256), 0, s, src, dst, len / 2);
      else hipLaunchKernelGGL(k_pair_step<G>, dim3(nblk(len / 2, 64)), dim3(64), 0, s, src, dst, len / 2);
    }
    MSM_HIP_CHECK(hipGetLastError());
    src = dst;
    cur ^= 1;
  }
  hipLaunchKernelGGL(k_finalize<G>, dim3(nblk(W, 64)), dim3(64), 0, s, src, fin.as<uint64_t>(), W);
  MSM_HIP_CHECK(hipGetLastError());
}
template <int G>
void ScanReducer<G>::read(hipStream_t s, int W, std::vector<hfp::Jac<HF>> &out) {
  out.resize(W);
  MSM_HIP_CHECK(hipMemcpyAsync(out.data(), fin.p, (size_t)W * sizeof(hfp::Jac<HF>), hipMemcpyDeviceToHost, s));
  MSM_HIP_CHECK(hipStreamSynchronize(s));
}
template struct ScanReducer<MSM_GROUP>;

// ---------------------------------------------------------- reduction plan --
// sum_i w_i S_i = sum_u u L_u + 2^s sum_v v H_v  with u = w_i mod 2^s,
// v = w_i >> s, L_u = sum_{i: low(w_i) = u} S_i, H_v = sum_{i: high(w_i) = v} S_i.
// L and H are segment sums over one list of bucket indices (level 0: chunks of
// <= 8 within a segment; then pairwise levels until one partial per segment;
// then a dense scatter into 2 windows of 2^s slots), followed by the dense
// 2-window ScanReducer and a 2^s Horner step on the host.
template <int G>
void WeightedReducer<G>::plan(const std::vector<uint32_t> &w, const std::vector<uint32_t> &win, int nwin, int c0) {
  typedef typename FieldOf<G>::F F;
  if (nwin < 1 || (!win.empty() && win.size() != w.size())) throw std::runtime_error("WeightedReducer: bad windows");
  bsize_ = w.size();
  nwin_ = nwin;
  starts_.clear();
  nout_.clear();
  uint32_t maxw = 0;
  for (uint32_t x : w) maxw = std::max(maxw, x);
  int bits = 0;
  while (bits < 32 && ((uint64_t)1 << bits) <= maxw) ++bits;
  sbits_ = std::max(1, (bits + 1) / 2);
  const uint32_t S = 1u << sbits_;
  // dense slot layout: window ww -> [L block (2 ww) S | H block (2 ww + 1) S]
  std::vector<std::vector<uint32_t>> byv((size_t)nwin * S), byu((size_t)nwin * S);
  for (size_t i = 0; i < w.size(); ++i) {
    const size_t ww = win.empty() ? 0 : win[i];
    if (ww >= (size_t)nwin) throw std::runtime_error("WeightedReducer: window out of range");
    uint32_t v = w[i] >> sbits_, u = w[i] & (S - 1);
    if (v) byv[ww * S + v].push_back((uint32_t)i);
    if (u) byu[ww * S + u].push_back((uint32_t)i);
  }
  std::vector<uint32_t> idx, seg;
  for (int ww = 0; ww < nwin; ++ww) {
    for (uint32_t v = 1; v < S; ++v)
      for (uint32_t i : byv[(size_t)ww * S + v]) idx.push_back(i), seg.push_back((2 * ww + 1) * S + v - 1);
    for (uint32_t u = 1; u < S; ++u)
      for (uint32_t i : byu[(size_t)ww * S + u]) idx.push_back(i), seg.push_back(2 * ww * S + u - 1);
  }
  // level 0 + pairwise levels
  std::vector<uint32_t> cur_seg = seg;
  // Level-0 chunk length: a chunk of C items is C - 1 dependent adds in one
  // lane.  Large plans keep 8 (few lanes per item, fewest levels); small ones
  // (a few hundred thousand items: plain Pippenger at 2^16, CHES shards of
  // 2^17..2^19) would leave the chip < 1 wave per SIMD deep with 7-add chains
  // (the 2^16 level 0 ran 103 us for 311 K adds, profiles/archive_r01_r04.txt (r04_fixed_cost.txt)),
  // so they take 4 or 2 and one or two more (tail) levels.  The adds are the
  // same in total (items - segments); MSM_L0_CHUNK=<2..64> overrides.
  static const int C0env = [] {
    const char *e = getenv("MSM_L0_CHUNK");  // A/B knob: level-0 chunk length
    return e ? std::max(2, std::min(64, atoi(e))) : 0;
  }();
  const size_t lane_items = idx.size() * (G == 2 ? 2 : 1);  // G2 segment sums run on lane pairs
  int C = C0env ? C0env : c0 ? c0 : lane_items >= ((size_t)3 << 19) ? 8 : lane_items >= ((size_t)600 << 10) ? 4 : 2;
  c0_ = C;
  while (true) {
    std::vector<uint32_t> st, nseg;
    size_t k = 0;
    while (k < cur_seg.size()) {
      st.push_back((uint32_t)k);
      nseg.push_back(cur_seg[k]);
      size_t e = k + 1;
      while (e < cur_seg.size() && e - k < (size_t)C && cur_seg[e] == cur_seg[k]) ++e;
      k = e;
    }
    st.push_back((uint32_t)cur_seg.size());
    bool first = starts_.empty();
    if (!first && nseg.size() == cur_seg.size()) break;  // nothing merged: one partial per segment
    starts_.emplace_back();
    starts_.back().ensure(st.size() * 4);
    MSM_HIP_CHECK(hipMemcpy(starts_.back().p, st.data(), st.size() * 4, hipMemcpyHostToDevice));
    nout_.push_back(nseg.size());
    cur_seg.swap(nseg);
    C = 2;
    if (cur_seg.empty()) break;
  }
  // bit phase (sync tail of one-window plans): segment (block, j) over the
  // final partials p of block = cur_seg[p] / S whose value cur_seg[p] % S + 1
  // has bit j; chunks of 8, pairwise levels, then a scatter to 2 s slots
  std::vector<uint32_t> bidx;
  bits_ = nwin == 1;
  bstarts_.clear();
  bnout_.clear();
  if (bits_) {
    const uint32_t NB2 = 2u * (uint32_t)nwin * (uint32_t)sbits_;
    std::vector<uint32_t> bseg;
    for (uint32_t bs = 0; bs < NB2; ++bs) {
      const uint32_t blk = bs / (uint32_t)sbits_, j = bs % (uint32_t)sbits_;
      for (size_t q = 0; q < cur_seg.size(); ++q)
        if (cur_seg[q] / S == blk && (((cur_seg[q] % S) + 1) >> j & 1u)) bidx.push_back((uint32_t)q), bseg.push_back(bs);
    }
    int Cb = 2;  // pairwise from the first level: the tail is latency-bound (a chunk of 8 is 7 serial adds in one lane)
    while (!bseg.empty()) {
      std::vector<uint32_t> st, nseg;
      size_t k = 0;
      while (k < bseg.size()) {
        st.push_back((uint32_t)k);
        nseg.push_back(bseg[k]);
        size_t e = k + 1;
        while (e < bseg.size() && e - k < (size_t)Cb && bseg[e] == bseg[k]) ++e;
        k = e;
      }
      st.push_back((uint32_t)bseg.size());
      if (!bnout_.empty() && nseg.size() == bseg.size()) break;
      bstarts_.emplace_back();
      bstarts_.back().ensure(st.size() * 4);
      MSM_HIP_CHECK(hipMemcpy(bstarts_.back().p, st.data(), st.size() * 4, hipMemcpyHostToDevice));
      bnout_.push_back(nseg.size());
      bseg.swap(nseg);
      Cb = 2;
    }
    std::vector<uint32_t> bdst(NB2 + 1, 0), bperm;
    std::vector<int> bat(NB2, -1);
    for (size_t k = 0; k < bseg.size(); ++k) bat[bseg[k]] = (int)k;
    for (uint32_t sl = 0; sl < NB2; ++sl) {
      bdst[sl] = (uint32_t)bperm.size();
      if (bat[sl] >= 0) bperm.push_back((uint32_t)bat[sl]);
    }
    bdst[NB2] = (uint32_t)bperm.size();
    bstarts_.emplace_back();
    bstarts_.back().ensure(bdst.size() * 4);
    MSM_HIP_CHECK(hipMemcpy(bstarts_.back().p, bdst.data(), bdst.size() * 4, hipMemcpyHostToDevice));
    bnout_.push_back(NB2);
    bidx.insert(bidx.end(), bperm.begin(), bperm.end());
    bperm_off_ = bidx.size() - bperm.size();
    bfin_.ensure((size_t)NB2 * 144 * G);
  }
  // dense scatter: slot -> its single partial (or empty), via a permutation
  const size_t NS = (size_t)2 * nwin * S;
  std::vector<uint32_t> dst(NS + 1, 0), perm;
  std::vector<int> at(NS, -1);
  for (size_t k = 0; k < cur_seg.size(); ++k) at[cur_seg[k]] = (int)k;
  for (size_t sl = 0; sl < NS; ++sl) {
    dst[sl] = (uint32_t)perm.size();
    if (at[sl] >= 0) perm.push_back((uint32_t)at[sl]);
  }
  dst[NS] = (uint32_t)perm.size();
  starts_.emplace_back();
  starts_.back().ensure(dst.size() * 4);
  MSM_HIP_CHECK(hipMemcpy(starts_.back().p, dst.data(), dst.size() * 4, hipMemcpyHostToDevice));
  nout_.push_back(NS);
  std::vector<uint32_t> all = idx;  // [level-0 item list | final permutation | bit phase items | bit permutation]
  all.insert(all.end(), perm.begin(), perm.end());
  final_perm_off_ = idx.size();
  bidx_off_ = all.size();
  bperm_off_ += bidx_off_;
  all.insert(all.end(), bidx.begin(), bidx.end());
  idx_.ensure(std::max<size_t>(all.size(), 1) * 4);
  if (!all.empty()) MSM_HIP_CHECK(hipMemcpy(idx_.p, all.data(), all.size() * 4, hipMemcpyHostToDevice));
  maxp_ = 1;
  for (size_t l = 0; l + 1 < nout_.size(); ++l) maxp_ = std::max(maxp_, nout_[l]);
  for (size_t l = 0; l + 1 < bnout_.size(); ++l) maxp_ = std::max(maxp_, bnout_[l]);  // bit phase levels
  maxp1_ = 1;  // batch group tails: level l writes part_[l & 1]; the odd levels are at most half of level 0
  for (size_t l = 1; l + 1 < nout_.size(); l += 2) maxp1_ = std::max(maxp1_, nout_[l]);
  // (the group bit tail, launch_tail_group_bits, alternates its levels over both
  // part_ buffers: every bit level fits either)
  for (size_t l = 0; l + 1 < bnout_.size(); ++l) maxp1_ = std::max(maxp1_, bnout_[l]);
  for (int st = 0; st < NSETS; ++st) {  // a new plan: sets are (re)sized on their next use
    part_[st][0].release();
    part_[st][1].release();
    dense_buf_[st].release();
  }
  ensure_set(0);
}

template <int G>
void WeightedReducer<G>::ensure_set(int set) {
  typedef typename FieldOf<G>::F F;
  if (set < 0 || set >= NSETS) throw std::runtime_error("WeightedReducer: bad buffer set");
  part_[set][0].ensure(maxp_ * sizeof(Xyzz<F>));
  part_[set][1].ensure(maxp_ * sizeof(Xyzz<F>));
  dense_buf_[set].ensure((size_t)2 * nwin_ * ((size_t)1 << sbits_) * sizeof(Xyzz<F>));
}

template <int G>
void WeightedReducer<G>::launch_head(hipStream_t s, const void *Sbuf, int set) {
  typedef typename FieldOf<G>::F F;
  ensure_set(set);
  const size_t L = nout_.size();
  const Xyzz<F> *src = reinterpret_cast<const Xyzz<F> *>(Sbuf);
  Xyzz<F> *dst = L == 1 ? dense_buf_[set].as<Xyzz<F>>() : part_[set][0].as<Xyzz<F>>();
  const uint32_t *ix = L == 1 ? idx_.as<uint32_t>() + final_perm_off_ : idx_.as<uint32_t>();
  launch_segsum<G>(s, src, ix, starts_[0].as<uint32_t>(), dst, nout_[0]);
  MSM_HIP_CHECK(hipGetLastError());
}

template <int G>
void WeightedReducer<G>::launch_tail(hipStream_t s, int set, bool coop) {
  typedef typename FieldOf<G>::F F;
  const size_t L = nout_.size();
  const Xyzz<F> *src = part_[set][0].as<Xyzz<F>>();
  if (bits_ && L >= 2) {
    // phase-1 levels 1 .. L-2 (level L-1 is the dense scatter, not used here),
    // then the bit phase: its level 0 reads the final partials through the
    // bit item list, later levels are contiguous, the last scatters to 2 s slots
    int cur = 0;
    auto segsum = [&](const Xyzz<F> *a, const uint32_t *ix, const uint32_t *st, Xyzz<F> *d, size_t nout) {
      if (!nout) return;
      launch_segsum_tail<G>(s, a, ix, st, d, nout, coop);
      MSM_HIP_CHECK(hipGetLastError());
    };
    for (size_t l = 1; l + 1 < L; ++l) {
      Xyzz<F> *dst = part_[set][l & 1].as<Xyzz<F>>();
      segsum(src, nullptr, starts_[l].as<uint32_t>(), dst, nout_[l]);
      src = dst;
      cur = (int)(l & 1);
    }
    const size_t LB = bnout_.size();
    for (size_t l = 0; l < LB; ++l) {
      const bool last = l + 1 == LB;
      Xyzz<F> *dst = last ? dense_buf_[set].as<Xyzz<F>>() : part_[set][cur ^ 1].as<Xyzz<F>>();
      const uint32_t *ix = l == 0 ? idx_.as<uint32_t>() + bidx_off_ : last ? idx_.as<uint32_t>() + bperm_off_ : nullptr;
      segsum(src, ix, bstarts_[l].as<uint32_t>(), dst, bnout_[l]);
      src = dst;
      cur ^= 1;
    }
    hipLaunchKernelGGL(k_finalize<G>, dim3(nblk(bit_slots(), 64)), dim3(64), 0, s, src, bfin_.as<uint64_t>(),
                       (int)bit_slots());
    MSM_HIP_CHECK(hipGetLastError());
    return;
  }
  for (size_t l = 1; l < L; ++l) {
    const bool last = l + 1 == L;
    Xyzz<F> *dst = last ? dense_buf_[set].as<Xyzz<F>>() : part_[set][l & 1].as<Xyzz<F>>();
    const uint32_t *ix = last ? idx_.as<uint32_t>() + final_perm_off_ : nullptr;
    if (nout_[l]) launch_segsum_tail<G>(s, src, ix, starts_[l].as<uint32_t>(), dst, nout_[l], coop);
    MSM_HIP_CHECK(hipGetLastError());
    src = dst;
  }
  dense_[set].launch(s, dense_buf_[set].p, 2 * nwin_, 1 << sbits_, coop);
}

template <int G>
void WeightedReducer<G>::ensure_group(int set, int nmsm) {
  typedef typename FieldOf<G>::F F;
  if (set < 0 || set >= NSETS || nmsm < 1) throw std::runtime_error("WeightedReducer: bad group");
  part_[set][0].ensure((size_t)nmsm * maxp_ * sizeof(Xyzz<F>));
  part_[set][1].ensure((size_t)nmsm * maxp1_ * sizeof(Xyzz<F>));
  if (bits_) bgfin_[set].ensure((size_t)nmsm * bit_bytes());
  dense_buf_[set].ensure((size_t)nmsm * dense_slots() * sizeof(Xyzz<F>));
  const size_t NT = (size_t)nmsm * dense_slots();  // ScanReducer::launch's buffers for W = 2 nwin nmsm
  dense_[set].buf[0].ensure(NT * sizeof(Xyzz<F>));
  dense_[set].buf[1].ensure(NT * sizeof(Xyzz<F>));
  dense_[set].fin.ensure((size_t)nmsm * out_bytes());
}

template <int G>
typename WeightedReducer<G>::HeadArgs WeightedReducer<G>::head_args(int set, int slot) {
  typedef typename FieldOf<G>::F F;
  const bool only = nout_.size() == 1;  // level 0 is also the last level
  Xyzz<F> *dst = only ? dense_buf_[set].as<Xyzz<F>>() + (size_t)slot * dense_slots()
                      : part_[set][0].as<Xyzz<F>>() + (size_t)slot * maxp_;
  const uint32_t *ix = only ? idx_.as<uint32_t>() + final_perm_off_ : idx_.as<uint32_t>();
  return HeadArgs{ix, starts_[0].as<uint32_t>(), dst, nout_[0]};
}

template <int G>
void WeightedReducer<G>::launch_head_slot(hipStream_t s, const void *Sbuf, int set, int slot) {
  typedef typename FieldOf<G>::F F;
  const HeadArgs a = head_args(set, slot);
  launch_segsum<G>(s, reinterpret_cast<const Xyzz<F> *>(Sbuf), a.idx, a.starts, static_cast<Xyzz<F> *>(a.dst),
                   a.nout);
  MSM_HIP_CHECK(hipGetLastError());
}

template <int G>
void WeightedReducer<G>::launch_head_slots(hipStream_t s, const void *Sbuf, size_t sstride, int set, int slot0,
                                           int nmsm) {
  typedef typename FieldOf<G>::F F;
  const bool only = nout_.size() == 1;  // level 0 is also the last level
  const HeadArgs a = head_args(set, slot0);
  launch_segsum<G>(s, reinterpret_cast<const Xyzz<F> *>(Sbuf), a.idx, a.starts, static_cast<Xyzz<F> *>(a.dst), a.nout,
                   nmsm, sstride, only ? dense_slots() : maxp_);
  MSM_HIP_CHECK(hipGetLastError());
}

template <int G>
void WeightedReducer<G>::launch_tail_group(hipStream_t s, int set, int nmsm, bool coop) {
  typedef typename FieldOf<G>::F F;
  const size_t L = nout_.size();
  const Xyzz<F> *src = part_[set][0].as<Xyzz<F>>();
  for (size_t l = 1; l < L; ++l) {
    const bool last = l + 1 == L;
    Xyzz<F> *dst = last ? dense_buf_[set].as<Xyzz<F>>() : part_[set][l & 1].as<Xyzz<F>>();
    const uint32_t *ix = last ? idx_.as<uint32_t>() + final_perm_off_ : nullptr;
    const size_t sstride = (l & 1) ? maxp_ : maxp1_;  // level l - 1 wrote part_[(l - 1) & 1]
    // coop (the batch's last group: nothing left to overlap): the narrow levels
    // over 4 waves per add
    launch_segsum_tail<G>(s, src, ix, starts_[l].as<uint32_t>(), dst, nout_[l], coop, nmsm, sstride,
                          last ? dense_slots() : (l & 1) ? maxp1_ : maxp_);
    MSM_HIP_CHECK(hipGetLastError());
    src = dst;
  }
  dense_[set].launch(s, dense_buf_[set].p, 2 * nwin_ * nmsm, 1 << sbits_, coop);
}

// The group tail ending in bit sums (one-window plans): the segment levels,
// then per MSM the 2 s bit sums B_j (the bit phase of launch_tail, every level
// one launch for the group), finalized to nmsm x 2 s Jacobians; the host
// combines T = sum_j 2^j B_j (combine_bits).  ~10 levels instead of the 2 s of
// the dense stage: for the batch's LAST group, whose tail runs after the last
// accumulation with the chip otherwise idle (Ches::run_jobs).
template <int G>
void WeightedReducer<G>::launch_tail_group_bits(hipStream_t s, int set, int nmsm, bool coop) {
  typedef typename FieldOf<G>::F F;
  const size_t L = nout_.size(), LB = bnout_.size();
  if (!has_bit_tail()) throw std::runtime_error("WeightedReducer: no bit tail in this plan");
  const Xyzz<F> *src = part_[set][0].as<Xyzz<F>>();
  size_t sstride = maxp_;
  int cur = 0;
  for (size_t l = 1; l + 1 < L; ++l) {  // segment levels 1 .. L-2 (L-1 is the dense scatter)
    Xyzz<F> *dst = part_[set][l & 1].as<Xyzz<F>>();
    const size_t dstride = (l & 1) ? maxp1_ : maxp_;
    if (nout_[l]) launch_segsum_tail<G>(s, src, nullptr, starts_[l].as<uint32_t>(), dst, nout_[l], coop, nmsm, sstride,
                                        dstride);
    MSM_HIP_CHECK(hipGetLastError());
    src = dst;
    sstride = dstride;
    cur = (int)(l & 1);
  }
  for (size_t l = 0; l < LB; ++l) {
    const bool last = l + 1 == LB;
    const int nb = cur ^ 1;
    Xyzz<F> *dst = last ? dense_buf_[set].as<Xyzz<F>>() : part_[set][nb].as<Xyzz<F>>();
    const size_t dstride = last ? bit_slots() : nb ? maxp1_ : maxp_;
    const uint32_t *ix = l == 0 ? idx_.as<uint32_t>() + bidx_off_ : last ? idx_.as<uint32_t>() + bperm_off_ : nullptr;
    if (bnout_[l])
      launch_segsum_tail<G>(s, src, ix, bstarts_[l].as<uint32_t>(), dst, bnout_[l], coop, nmsm, sstride, dstride);
    MSM_HIP_CHECK(hipGetLastError());
    src = dst;
    sstride = dstride;
    cur = nb;
  }
  const int W = (int)((size_t)nmsm * bit_slots());
  hipLaunchKernelGGL(k_finalize<G>, dim3(nblk((size_t)W, 64)), dim3(64), 0, s, src, bgfin_[set].as<uint64_t>(), W);
  MSM_HIP_CHECK(hipGetLastError());
}

template <int G>
void WeightedReducer<G>::copy_out_group_bits(hipStream_t s, int set, int nmsm, void *host) {
  MSM_HIP_CHECK(hipMemcpyAsync(host, bgfin_[set].p, (size_t)nmsm * bit_bytes(), hipMemcpyDefault, s));
}

// window 0's sum_b b S_b from its 2 s bit sums (bit j of the weight: low half
// block j < s, high half s + j): Horner from the top bit, as read_windows
template <int G>
hfp::Jac<typename HostField<G>::F> WeightedReducer<G>::combine_bits(const void *host) const {
  const hfp::Jac<HF> *B = reinterpret_cast<const hfp::Jac<HF> *>(host);
  const hfp::Jac<HF> *lo = B, *hi = B + sbits_;
  hfp::Jac<HF> acc = hi[sbits_ - 1];
  for (int j = 2 * sbits_ - 2; j >= 0; --j) {
    acc = hfp::dbl(acc);
    acc = hfp::addj(acc, j >= sbits_ ? hi[j - sbits_] : lo[j]);
  }
  return acc;
}

template <int G>
void WeightedReducer<G>::copy_out_group(hipStream_t s, int set, int nmsm, void *host) {
  // host (read-back) or device (an exchange buffer, ChesMulti's RCCL gather)
  MSM_HIP_CHECK(hipMemcpyAsync(host, dense_[set].fin.p, (size_t)nmsm * out_bytes(), hipMemcpyDefault, s));
}

template <int G>
void WeightedReducer<G>::copy_out(hipStream_t s, int set, void *host) {
  MSM_HIP_CHECK(hipMemcpyAsync(host, dense_[set].fin.p, out_bytes(), hipMemcpyDeviceToHost, s));
}

template <int G>
std::vector<hfp::Jac<typename HostField<G>::F>> WeightedReducer<G>::combine(const void *host) const {
  const hfp::Jac<HF> *T = reinterpret_cast<const hfp::Jac<HF> *>(host);
  std::vector<hfp::Jac<HF>> out(nwin_);
  for (int ww = 0; ww < nwin_; ++ww) out[ww] = horner(std::vector<hfp::Jac<HF>>{T[2 * ww], T[2 * ww + 1]}, sbits_);
  return out;
}

template <int G>
std::vector<hfp::Jac<typename HostField<G>::F>> WeightedReducer<G>::read_windows(hipStream_t s) {
  if (bits_ && nout_.size() >= 2) {  // launch_tail's bit sums: T = sum_j 2^j B_j, Horner from the top bit
    std::vector<hfp::Jac<HF>> B(bit_slots());
    MSM_HIP_CHECK(hipMemcpyAsync(B.data(), bfin_.p, bit_slots() * sizeof(hfp::Jac<HF>), hipMemcpyDeviceToHost, s));
    MSM_HIP_CHECK(hipStreamSynchronize(s));
    std::vector<hfp::Jac<HF>> out(nwin_);
    for (int ww = 0; ww < nwin_; ++ww) {
      // bit j of the window's weight: low half block 2 ww (j < s), high half block 2 ww + 1
      const hfp::Jac<HF> *lo = &B[(size_t)2 * ww * sbits_], *hi = lo + sbits_;
      hfp::Jac<HF> acc = hi[sbits_ - 1];
      for (int j = 2 * sbits_ - 2; j >= 0; --j) {
        acc = hfp::dbl(acc);
        acc = hfp::addj(acc, j >= sbits_ ? hi[j - sbits_] : lo[j]);
      }
      out[ww] = acc;
    }
    return out;
  }
  std::vector<uint8_t> host(out_bytes());
  copy_out(s, 0, host.data());
  MSM_HIP_CHECK(hipStreamSynchronize(s));
  return combine(host.data());
}

template <int G>
hfp::Jac<typename HostField<G>::F> WeightedReducer<G>::combine_windows(const void *host, int c) const {
  const hfp::Jac<HF> *T = reinterpret_cast<const hfp::Jac<HF> *>(host);
  // terms (exponent, point): L_w at c w, H_w at c w + s; Horner from the top
  std::vector<std::pair<long, int>> terms;
  for (int ww = 0; ww < nwin_; ++ww) {
    terms.emplace_back((long)c * ww, 2 * ww);
    terms.emplace_back((long)c * ww + sbits_, 2 * ww + 1);
  }
  std::sort(terms.begin(), terms.end());
  hfp::Jac<HF> acc = T[terms.back().second];
  long e = terms.back().first;
  for (int k = (int)terms.size() - 2; k >= 0; --k) {
    for (; e > terms[k].first; --e) acc = hfp::dbl(acc);
    acc = hfp::addj(acc, T[terms[k].second]);
  }
  for (; e > 0; --e) acc = hfp::dbl(acc);
  return acc;
}

template <int G>
hfp::Jac<typename HostField<G>::F> WeightedReducer<G>::read_total(hipStream_t s, int c) {
  if (bits_ && nout_.size() >= 2) {  // one-window plan ended in bit sums (launch_tail): its T_0 is the total
    const std::vector<hfp::Jac<HF>> T = read_windows(s);
    return horner(T, c);
  }
  std::vector<uint8_t> host(out_bytes());
  copy_out(s, 0, host.data());
  MSM_HIP_CHECK(hipStreamSynchronize(s));
  return combine_windows(host.data(), c);
}

template class WeightedReducer<MSM_GROUP>;

// ------------------------------------------------------------------ Ches --
template <int G>
Ches<G>::Ches(int device, const ChesParams &p) : dev_(device), p_(p) {
  DeviceGuard g(dev_);
  if (p.q_exp < 2 || p.q_exp > 24 || p.h < 1 || p.h > 32 || (long)p.q_exp * p.h < 255)
    throw std::runtime_error("bad CHES parameters");
  const int q = 1 << p.q_exp;
  B_ = ches_bucket_set(q, p.a_h);
  if (p.b_size > 0 && (int)B_.size() != p.b_size)
    throw std::runtime_error("bucket set size " + std::to_string(B_.size()) + " != configured " +
                             std::to_string(p.b_size));
  std::vector<uint32_t> code, rank;
  ches_digit_code(B_, q, code, rank);
  code_.ensure(code.size() * 4);
  rank_.ensure(rank.size() * 4);
  MSM_HIP_CHECK(hipMemcpy(code_.p, code.data(), code.size() * 4, hipMemcpyHostToDevice));
  MSM_HIP_CHECK(hipMemcpy(rank_.p, rank.data(), rank.size() * 4, hipMemcpyHostToDevice));
  for (size_t k = 1; k < B_.size() && B_[k] <= p.a_h + 1; ++k) small_ = (int)k;
  plan_buckets(0);
  ev_.resize(8);
  for (auto &e : ev_) MSM_HIP_CHECK(hipEventCreate(&e));
}
template <int G>
Ches<G>::~Ches() {
  for (auto &e : ev_) (void)hipEventDestroy(e);
  for (auto &e : acc_ev_) (void)hipEventDestroy(e);
  for (auto &e : bev_) (void)hipEventDestroy(e);
  for (int t = 0; t < kBSets; ++t) {
    if (ev_tail_[t]) (void)hipEventDestroy(ev_tail_[t]);
    if (tails_[t]) (void)hipStreamDestroy(tails_[t]);
  }
  if (host_out_) (void)hipHostFree(host_out_);
  if (host_bits_) (void)hipHostFree(host_bits_);
  if (fstream_) (void)hipStreamDestroy(fstream_);
  if (cstream_) (void)hipStreamDestroy(cstream_);
}

// bucket space = B plus (copies_ - 1) copies of the small buckets 1..small_;
// copies_ is chosen so a copy receives ~12 top-digit entries (n / (small_ copies))
template <int G>
void Ches<G>::plan_buckets(size_t n) {
  int want = 1;
  if (small_ > 0 && n > 0) {
    size_t c = (n + (size_t)small_ * 12 - 1) / ((size_t)small_ * 12);
    want = (int)std::min<size_t>(std::max<size_t>(c, 1), 256);
  }
  if (want == copies_ && red_.size()) return;
  copies_ = want;
  std::vector<uint32_t> w(B_.begin(), B_.end());
  for (int c = 1; c < copies_; ++c)
    for (int k = 1; k <= small_; ++k) w.push_back((uint32_t)B_[k]);
  if (w.size() >= (1u << 24)) throw std::runtime_error("CHES bucket space exceeds 24-bit indices");
  red_.plan(w);
  static const int bc_env = [] {  // A/B knob: the batch reducer's level-0 chunk (0: red_'s)
    const char *e = getenv("MSM_BATCH_L0_CHUNK");
    return e ? std::max(0, std::min(64, atoi(e))) : 8;
  }();
  if (bc_env && red_.level0_chunk() != bc_env) {
    bred_.plan(w, bc_env);
    batch_red_ = &bred_;
  } else {
    batch_red_ = &red_;
  }
}

// Accumulation lanes of a batch (run_batch): 3 (G1) or 2 (G2) when one
// accumulation's lanes (one per bucket for G1, two for G2) fill fewer than ~3 rounds of the chip's
// wave slots (1024 SIMDs x the kernel's waves per SIMD x 64 lanes: 3 for
// k_accumulate<1>, 2 for k_accumulate2p), else 1.  MSM_BATCH_LANES=1|2|3
// overrides.
template <int G>
int Ches<G>::batch_lanes() const {
  static const int env = [] {
    const char *e = getenv("MSM_BATCH_LANES");
    return e ? std::max(1, std::min(3, atoi(e))) : 0;
  }();
  if (env) return env;
  // G1 small MSMs take three lanes since round 4's single reduction group per
  // batch (2^17 / 2^18 / 2^19 batches 0.52 / 0.86 / 1.40 -> 0.49 / 0.80 / 1.35
  // ms per MSM, profiles/archive_r01_r04.txt (r04_small_lanes_ab.txt)); G2 keeps two (not measured)
  const size_t lanes = bucket_count() * (G == 2 ? 2 : 1);
  return lanes < (size_t)3 * (G == 2 ? 2 : 3) * 1024 * 64 ? (G == 1 ? 3 : 2) : 1;
}

template <int G>
void Ches<G>::build_table(const void *pts, size_t n, bool on_device, hipStream_t s) {
  typedef typename FieldOf<G>::F F;
  DeviceGuard g(dev_);
  const size_t K = 3 * (size_t)p_.h;
  if (n == 0) {
    n_ = 0;
    return;
  }
  if (K * n >= (1ull << 31)) throw std::runtime_error("CHES table too large for 31-bit slots");
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
  const size_t chunk = std::min<size_t>(n, (size_t)1 << 16);
  DevBuf scratch, pref;
  scratch.ensure(K * chunk * sizeof(Xyzz<F>));
  pref.ensure(K * chunk * sizeof(F));
  for (size_t i0 = 0; i0 < n; i0 += chunk) {
    size_t cnt = std::min(chunk, n - i0);
    if constexpr (G == 2)  // lane pairs: no spills (pair_kernels.hpp)
      hipLaunchKernelGGL((k_ches_table2p<3>), dim3(nblk(2 * cnt, 128)), dim3(128), 0, s, base.as<Aff<F>>(), i0, cnt,
                         p_.q_exp, p_.h, scratch.as<Xyzz<F>>(), pref.as<F>(), table_.as<AffP<F>>());
    else
      hipLaunchKernelGGL((k_ches_table<G, 3>), dim3(nblk(cnt, 64)), dim3(64), 0, s, base.as<Aff<F>>(), i0, cnt,
                         p_.q_exp, p_.h, scratch.as<Xyzz<F>>(), pref.as<F>(), table_.as<AffP<F>>());
    MSM_HIP_CHECK(hipGetLastError());
  }
  MSM_HIP_CHECK(hipStreamSynchronize(s));
  n_ = n;
  plan_buckets(n);
}

template <int G>
void Ches<G>::reserve_table(size_t n) {
  typedef typename FieldOf<G>::F F;
  DeviceGuard g(dev_);
  const size_t cnt = 3 * (size_t)p_.h * n;
  if (cnt >= (1ull << 31)) throw std::runtime_error("table too large for 31-bit slots");
  table_.ensure(std::max<size_t>(cnt, 1) * sizeof(AffP<F>));
  n_ = n;
  plan_buckets(n);
}

template <int G>
void Ches<G>::put_table(const void *tab, size_t first, size_t count, bool on_device, hipStream_t s) {
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
void Ches<G>::set_table(const void *tab, size_t n, bool on_device, hipStream_t s) {
  reserve_table(n);
  put_table(tab, 0, table_rows(), on_device, s);
}

template <int G>
void Ches<G>::get_table(void *out, size_t first, size_t count, hipStream_t s) {
  typedef typename FieldOf<G>::F F;
  DeviceGuard g(dev_);
  if (first + count > 3 * (size_t)p_.h * n_) throw std::runtime_error("table range out of bounds");
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
void Ches<G>::digits_sort(hipStream_t s, const uint8_t *d_scalars, size_t stride, size_t set_stride, int nsets,
                          int set, int fine_bt) {
  const size_t n = n_, h = (size_t)p_.h, ne = n * h, NB = bucket_count();
  ChesFrontSet &f = fs_[set];
  f.sort.fine_bt = fine_bt;
  f.sorted.ensure(ne * nsets * 4 + 64);  // + the accumulation's 16-B payload window past a run's end
  f.counts.ensure(NB * nsets * 4);
  f.offsets.ensure(NB * nsets * 4);
  f.order.ensure(NB * nsets * 4);
  // Fused front (the h of every reference configuration): the digits are
  // computed twice -- counted per coarse bin, then binned -- instead of being
  // written as keys / vals and read back twice by the sort (5 launches after
  // the scan's 2 instead of 8; MSM_FRONT_FUSED=0 selects the unfused front)
  static const bool fused_env = [] {
    const char *e = getenv("MSM_FRONT_FUSED");
    return !e || atoi(e) != 0;
  }();
  if (fused_env && (p_.h == 12 || p_.h == 13 || p_.h == 14 || p_.h == 16 || p_.h == 19 || p_.h == 20)) {
    const int ntiles = (int)nblk(n, 256);
    const BucketSort::Geom g = f.sort.prepare(s, ne, (uint32_t)NB, nsets, ntiles);
#define MSM_CHES_FRONT(HT)                                                                                             \
  do {                                                                                                                 \
    hipLaunchKernelGGL(k_ches_front_hist<HT>, dim3(ntiles, nsets), dim3(256), 0, s, d_scalars, stride, n, p_.q_exp,   \
                       code_.as<uint32_t>(), rank_.as<uint2>(), (uint32_t)B_.size(), (uint32_t)small_,                 \
                       (uint32_t)copies_, set_stride, g.fb_bits, g.ncb, g.ntiles, f.sort.ghist.as<uint32_t>(),         \
                       f.sort.classes.as<uint32_t>());                                                                  \
    MSM_HIP_CHECK(hipGetLastError());                                                                                  \
    if (profile_) MSM_HIP_CHECK(hipEventRecord(ev_[1], s));                                                            \
    f.sort.scan(s, g);                                                                                                 \
    hipLaunchKernelGGL(k_ches_front_coarse<HT>, dim3(ntiles, nsets), dim3(256), (size_t)(2 * g.ncb + 512 * HT) * 4, s, \
                       d_scalars, stride, n, p_.q_exp, code_.as<uint32_t>(), rank_.as<uint2>(), (uint32_t)B_.size(),  \
                       (uint32_t)small_, (uint32_t)copies_, set_stride, g.fb_bits, g.ncb, g.ntiles,                   \
                       f.sort.gbase.as<uint32_t>(), f.sort.okeys.as<uint32_t>(), f.sort.ovals.as<uint32_t>());         \
    MSM_HIP_CHECK(hipGetLastError());                                                                                  \
  } while (0)
    switch (p_.h) {
      case 12: MSM_CHES_FRONT(12); break;
      case 13: MSM_CHES_FRONT(13); break;
      case 14: MSM_CHES_FRONT(14); break;
      case 16: MSM_CHES_FRONT(16); break;
      case 19: MSM_CHES_FRONT(19); break;
      default: MSM_CHES_FRONT(20); break;
    }
#undef MSM_CHES_FRONT
    f.sort.finish(s, g, ne, (uint32_t)NB, f.sorted.as<uint32_t>(), f.counts.as<uint32_t>(), f.offsets.as<uint32_t>(),
                  f.order.as<uint32_t>(), nsets);
    return;
  }
  f.keys.ensure(ne * nsets * 4);
  f.vals.ensure(ne * nsets * 4);
#define MSM_CHES_DIGITS(HT)                                                                                   \
  hipLaunchKernelGGL(k_ches_digits<HT>, dim3(nblk(n, 256), nsets), dim3(256), 0, s, d_scalars, stride, n, p_.q_exp, \
                     p_.h, code_.as<uint32_t>(), rank_.as<uint2>(), f.keys.as<uint32_t>(), f.vals.as<uint32_t>(),     \
                     (uint32_t)B_.size(), (uint32_t)small_, (uint32_t)copies_, set_stride)
  switch (p_.h) {  // the h of the reference configurations (ches_config_files)
    case 12: MSM_CHES_DIGITS(12); break;
    case 13: MSM_CHES_DIGITS(13); break;
    case 14: MSM_CHES_DIGITS(14); break;
    case 16: MSM_CHES_DIGITS(16); break;
    case 19: MSM_CHES_DIGITS(19); break;
    case 20: MSM_CHES_DIGITS(20); break;
    default: MSM_CHES_DIGITS(0); break;
  }
#undef MSM_CHES_DIGITS
  MSM_HIP_CHECK(hipGetLastError());
  if (profile_) MSM_HIP_CHECK(hipEventRecord(ev_[1], s));
  f.sort.run(s, f.keys.as<uint32_t>(), f.vals.as<uint32_t>(), ne, (uint32_t)NB, f.sorted.as<uint32_t>(),
             f.counts.as<uint32_t>(), f.offsets.as<uint32_t>(), f.order.as<uint32_t>(), nsets);
}

template <int G>
void Ches<G>::accumulate(hipStream_t s, int set, int r, int bset, const void *table) {
  typedef typename FieldOf<G>::F F;
  const size_t NB = bucket_count();
  ChesFrontSet &f = fs_[set];
  buckets_[bset].ensure(NB * sizeof(Xyzz<F>));
  launch_accumulate<G>(s, f.sort.sched(f.order.as<uint32_t>(), f.sorted.as<uint32_t>(), r, NB),
                       table ? static_cast<const AffP<F> *>(table) : table_.as<AffP<F>>(),
                       buckets_[bset].as<Xyzz<F>>(), NB);
  MSM_HIP_CHECK(hipGetLastError());
}

template <int G>
void Ches<G>::accumulate_sets(hipStream_t s, int set, int R, int gb, const void *table) {
  typedef typename FieldOf<G>::F F;
  const size_t NB = bucket_count();
  ChesFrontSet &f = fs_[set];
  launch_accumulate_sets<G>(s, f.sort.sched(f.order.as<uint32_t>(), f.sorted.as<uint32_t>(), 0, NB), f.sort.stride(NB),
                            table ? static_cast<const AffP<F> *>(table) : table_.as<AffP<F>>(),
                            gbuckets_[gb].as<Xyzz<F>>(), NB, R);
  MSM_HIP_CHECK(hipGetLastError());
}

template <int G>
float Ches<G>::time_accumulation(hipStream_t s, const uint8_t *d_scalars, size_t set_stride, int nsets, int reps) {
  DeviceGuard g(dev_);
  if (n_ == 0 || nsets < 1 || reps < 1) throw std::runtime_error("time_accumulation: no table / bad arguments");
  digits_sort(s, d_scalars, 32, set_stride, nsets, 0);
  gbuckets_[0].ensure((size_t)nsets * bucket_count() * sizeof(Xyzz<typename FieldOf<G>::F>));
  accumulate_sets(s, 0, nsets, 0, nullptr);  // warm
  hipEvent_t a, b;
  MSM_HIP_CHECK(hipEventCreate(&a));
  MSM_HIP_CHECK(hipEventCreate(&b));
  MSM_HIP_CHECK(hipEventRecord(a, s));
  for (int r = 0; r < reps; ++r) accumulate_sets(s, 0, nsets, 0, nullptr);
  MSM_HIP_CHECK(hipEventRecord(b, s));
  MSM_HIP_CHECK(hipEventSynchronize(b));
  float ms = 0;
  MSM_HIP_CHECK(hipEventElapsedTime(&ms, a, b));
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return ms / (float)reps;
}

template <int G>
void Ches<G>::accumulate_l0(hipStream_t s, int set, int r, int bset, const void *table, int l0_bset, int gset,
                            int slot, int l0_last) {
  typedef typename FieldOf<G>::F F;
  const size_t NB = bucket_count();
  ChesFrontSet &f = fs_[set];
  const typename WeightedReducer<G>::HeadArgs a = batch_red_->head_args(gset, slot);
  const AccSched S = f.sort.sched(f.order.as<uint32_t>(), f.sorted.as<uint32_t>(), r, NB);
  const AffP<F> *T = table ? static_cast<const AffP<F> *>(table) : table_.as<AffP<F>>();
  // lanes: one per bucket / output (G1), two (G2 lane pairs)
  const unsigned l0b = (unsigned)((G * a.nout + 255) / 256), accb = (unsigned)((G * NB + 255) / 256);
  if constexpr (G == 1)
    hipLaunchKernelGGL((k_accumulate_l0<AffP<F>>), dim3(accb + l0b), dim3(256), 0, s, S, T,
                       buckets_[bset].as<Xyzz<F>>(), NB, buckets_[l0_bset].as<Xyzz<F>>(), a.idx, a.starts,
                       static_cast<Xyzz<F> *>(a.dst), a.nout, l0b, l0_last);
  else
    hipLaunchKernelGGL((k_accumulate2p_l0<AffP<F>>), dim3(accb + l0b), dim3(256), 0, s, S, T,
                       buckets_[bset].as<Xyzz<F>>(), NB, buckets_[l0_bset].as<Xyzz<F>>(), a.idx, a.starts,
                       static_cast<Xyzz<F> *>(a.dst), a.nout, l0b, l0_last);
  MSM_HIP_CHECK(hipGetLastError());
}

template <int G>
void Ches<G>::run(hipStream_t s, const uint8_t *d_scalars, size_t stride, hfp::Jac<HF> *out) {
  DeviceGuard g(dev_);
  if (stride < 32) throw std::runtime_error("CHES scalars must be 32-byte strings");
  if (n_ == 0) {
    std::memset(out, 0, sizeof(*out));
    return;
  }
  if (profile_) MSM_HIP_CHECK(hipEventRecord(ev_[0], s));
  digits_sort(s, d_scalars, stride, 0, 1, 0);
  if (profile_) MSM_HIP_CHECK(hipEventRecord(ev_[2], s));
  accumulate(s, 0, 0, 0);
  if (profile_) MSM_HIP_CHECK(hipEventRecord(ev_[3], s));
  red_.launch(s, buckets_[0].p);
  if (profile_) MSM_HIP_CHECK(hipEventRecord(ev_[4], s));
  *out = red_.read(s);
  if (profile_) {
    MSM_HIP_CHECK(hipEventRecord(ev_[5], s));
    MSM_HIP_CHECK(hipEventSynchronize(ev_[5]));
    float ms;
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
void Ches<G>::run_jobs(hipStream_t s, const uint8_t *scalars, size_t stride, size_t set_stride, size_t nsets,
                       size_t nseg, const void *const *tables, hfp::Jac<HF> *outs, bool scalars_on_host,
                       void *dev_out) {
  DeviceGuard g(dev_);
  if (stride < 32) throw std::runtime_error("CHES scalars must be 32-byte strings");
  if (nseg < 1) throw std::runtime_error("run_jobs: no segments");
  WeightedReducer<G> &red = *batch_red_;
  // the dense stage of the batch's LAST group runs its adds over 4 waves each
  // (nothing else left to overlap; MSM_TAIL_COOP=0: one lane per add throughout)
  static const bool tail_coop = [] {
    const char *e = getenv("MSM_TAIL_COOP");
    return !e || atoi(e) != 0;
  }();
  // jobs k = set (k / nseg), segment (k % nseg); every loop below runs over jobs
  const size_t count = nsets * nseg;
  if (count == 0) return;
  if (n_ == 0) {
    std::memset(outs, 0, sizeof(*outs) * count);
    return;
  }
  auto job_scalars = [&](size_t k) { return scalars + (k / nseg) * set_stride + (k % nseg) * n_ * stride; };
  auto job_table = [&](size_t k) { return tables[k % nseg]; };
  // a front group of several jobs reads their scalars with one stride: the
  // segments' slices are n strings apart, so groups > 1 need packed sets
  const size_t jstride = nseg == 1 ? set_stride : n_ * stride;
  const bool packed = nseg == 1 || set_stride == nseg * n_ * stride;
  if (!fstream_) {
    // fronts at the greatest priority: their short memory-bound kernels take the
    // first CU slots an accumulation releases (the next accumulation waits for
    // them); the reductions at normal priority, beside the accumulations (the
    // same priority for both measured equal, tools/batch_sched.py)
    int least = 0, greatest = 0;
    MSM_HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    static const int front_prio = [] {  // A/B knob: 1 greatest (default), 0 normal, -1 least
      const char *e = getenv("MSM_FRONT_PRIO");
      return e ? atoi(e) : 1;
    }();
    MSM_HIP_CHECK(hipStreamCreateWithPriority(&fstream_, hipStreamNonBlocking,
                                              front_prio > 0 ? greatest : front_prio < 0 ? least : 0));
    static const bool tail_hi = [] {  // A/B knob: reduction streams at the front's (greatest) priority
      const char *e = getenv("MSM_TAIL_PRIO");
      return e && atoi(e) != 0;
    }();
    for (int t = 0; t < kBSets; ++t) {
      MSM_HIP_CHECK(hipStreamCreateWithPriority(&tails_[t], hipStreamNonBlocking, tail_hi ? greatest : 0));
      MSM_HIP_CHECK(hipEventCreateWithFlags(&ev_tail_[t], hipEventDisableTiming));
    }
    MSM_HIP_CHECK(hipStreamCreateWithFlags(&cstream_, hipStreamNonBlocking));
    // a stream's hardware queue is set up at its first launch: do that here,
    // not inside the first batch that happens to use the stream
    prime_.ensure(256);
    for (hipStream_t q : {fstream_, tails_[0], tails_[1], cstream_}) MSM_HIP_CHECK(hipMemsetAsync(prime_.p, 0, 256, q));
    for (hipStream_t q : {fstream_, tails_[0], tails_[1], cstream_}) MSM_HIP_CHECK(hipStreamSynchronize(q));
  }
  // one pinned read-back slot per MSM of the batch: the host never waits inside
  // the issue loop, so MSM k+1's front is queued while MSM k still accumulates
  const size_t ob = red.out_bytes();  // a group's read-back lands contiguously
  // reduction groups of <= kGroup MSMs (balanced sizes), alternating between
  // the reducer sets / tail streams.  MSM_LAST_GROUP=m (A/B knob): the batch's
  // last m MSMs form a group of their own, so the earlier group's tail runs
  // beside the last accumulations and only a narrow tail follows the last one
  static const size_t group_max = [] {  // A/B knob: MSMs per reduction group (default kGroup)
    const char *e = getenv("MSM_RED_GROUP");
    return (size_t)(e ? std::max(1, std::min(32, atoi(e))) : kGroup);
  }();
  static const size_t last_env = [] {
    const char *e = getenv("MSM_LAST_GROUP");
    return (size_t)(e ? std::max(0, std::min(32, atoi(e))) : 0);
  }();
  std::vector<size_t> gfirst;  // group q holds MSMs [gfirst[q], gfirst[q + 1])
  {
    const size_t last = last_env && count > last_env ? std::min(last_env, group_max) : 0, nmain = count - last;
    const size_t ng = (nmain + group_max - 1) / group_max, Rm = (nmain + ng - 1) / ng;
    for (size_t k = 0; k < nmain; k += Rm) gfirst.push_back(k);
    if (last) gfirst.push_back(nmain);
    gfirst.push_back(count);
  }
  const size_t ngroups = gfirst.size() - 1;
  std::vector<uint32_t> gof(count);
  for (size_t q = 0; q < ngroups; ++q)
    for (size_t k = gfirst[q]; k < gfirst[q + 1]; ++k) gof[k] = (uint32_t)q;
  auto grp = [&](size_t k) { return (size_t)gof[k]; };              // the reduction group of MSM k
  auto gslot = [&](size_t k) { return k - gfirst[gof[k]]; };        // its slot in the group
  auto gend = [&](size_t k) { return k + 1 == gfirst[gof[k] + 1]; };  // the group's last MSM
  if (host_out_bytes_ < count * ob) {  // at least 256 MSMs' worth (a few hundred KiB): no regrowth per batch size
    if (host_out_) (void)hipHostFree(host_out_);
    host_out_ = nullptr;
    host_out_bytes_ = 0;
    const size_t bytes = std::max<size_t>(count, 256) * ob;
    MSM_HIP_CHECK(hipHostMalloc(&host_out_, bytes, hipHostMallocDefault));
    host_out_bytes_ = bytes;
  }
  // where the groups' window sums land: the pinned read-back slots, or the
  // caller's device exchange buffer (dev_out: ChesMulti gathers it over RCCL
  // and combines on the host; the combine below is then skipped)
  uint8_t *const out_base = dev_out ? static_cast<uint8_t *>(dev_out) : static_cast<uint8_t *>(host_out_);
  // The batch's LAST reduction group ends in bit sums (launch_tail_group_bits):
  // its tail runs after the last accumulation with the chip otherwise idle, and
  // the bit phase is ~10 latency-bound levels instead of the dense stage's 2 s
  // (profiles/r06_small_trace.txt).  Earlier groups keep the dense stage: their
  // tails run beside accumulations, where the 2 s-Jacobian read-backs cost
  // (DESIGN 5).  MSM_BIT_TAIL=0: dense stage for every group.
  static const bool bit_tail_env = [] {
    const char *e = getenv("MSM_BIT_TAIL");
    return !e || atoi(e) != 0;
  }();
  const bool bit_tail = bit_tail_env && !dev_out && red.has_bit_tail();
  const size_t bb = red.bit_bytes();
  if (bit_tail && host_bits_bytes_ < (size_t)group_max * bb) {
    if (host_bits_) (void)hipHostFree(host_bits_);
    host_bits_ = nullptr;
    host_bits_bytes_ = 0;
    const size_t bytes = (size_t)std::max<size_t>(group_max, 32) * bb;
    MSM_HIP_CHECK(hipHostMalloc(&host_bits_, bytes, hipHostMallocDefault));
    host_bits_bytes_ = bytes;
  }
  // a group's tail + read-back: the dense stage into the read-back slots, or
  // (the last group, bit_tail) the bit phase into host_bits_
  auto group_tail = [&](hipStream_t ts, int rset, size_t first, size_t nmsm, bool last_group) {
    if (bit_tail && last_group) {
      red.launch_tail_group_bits(ts, rset, (int)nmsm, tail_coop);
      red.copy_out_group_bits(ts, rset, (int)nmsm, host_bits_);
    } else {
      red.launch_tail_group(ts, rset, (int)nmsm, tail_coop && last_group);
      red.copy_out_group(ts, rset, (int)nmsm, out_base + first * ob);
    }
  };
  // (group size cap: kFrontGroupDefault, or MSM_FRONT_GROUP=<1..8>; engine.hpp)
  // (small MSMs on lanes: groups of 2 on two lanes -- half the front launches,
  // measured 0.551 -> 0.530 ms per 2^17 MSM and 0.874 -> 0.845 at 2^18 -- and 4
  // on three lanes (profiles/archive_r01_r04.txt (r04_small_lanes_ab.txt)); the 2^20 batch keeps 1,
  // its wider fronts starve the accumulation, r03_front_group_ab.txt and
  // r04_front_group_ab.txt)
  static const size_t fg_env = [] {
    const char *e = getenv("MSM_FRONT_GROUP");
    return e ? (size_t)std::min(kFrontGroup, std::max(1, atoi(e))) : (size_t)0;
  }();
  const int nl = batch_lanes();
  // the batch fronts' fine-pass workgroup (bucket_sort.hpp k_bs_fine): 1024
  // threads; MSM_FINE_BT=256 selects the variant that fits beside three
  // accumulation waves per SIMD -- measured slower (H2D 408-411 vs 415-420 M,
  // resident 423-429 vs 434-440 M pairs/s, profiles/archive_r01_r04.txt (r04_fine_bt_ab.txt))
  static const int fine_bt = [] {
    const char *e = getenv("MSM_FINE_BT");
    return e && atoi(e) == 256 ? 256 : 1024;
  }();
  static const bool acc_group_env = [] {  // accumulation groups (below); MSM_ACC_GROUP=0: per-MSM lanes
    const char *e = getenv("MSM_ACC_GROUP");
    return !e || atoi(e) != 0;
  }();
  const bool acc_groups = nl >= 2 && nseg == 1 && acc_group_env;
  // (one lane, the 2^20 headline: one accumulation launch per MSM.  Alone, two
  // 2^20 sets in one grid accumulate in 1.70 ms per set vs 1.96 for one
  // (profiles/r05_acc_rate.txt: a launch's last waves leave the chip half
  // idle), but in the batch the front and level 0 beside it fill that tail:
  // groups of 2 per launch measured 427 vs 431-433 M pairs/s with H2D, the
  // in-batch accumulation 1.75-1.80 vs 1.72-1.77 ms per set, profiles/r05_head_front_group_ab.txt)
  const size_t fg_max = !packed ? 1 : fg_env ? fg_env : acc_groups ? 4 : nl >= 3 ? 4 : nl == 2 ? 2 : (size_t)kFrontGroupDefault;
  // front groups of 1, 1, 2, 4, then fg_max MSMs: the first accumulation
  // starts after one front, and each group's host sets (copied while the earlier
  // groups accumulate: a set copies in ~0.6 ms, an MSM accumulates in ~2.3) are
  // in HBM before its front is due -- a first group of eight stalled the H2D
  // batch by ~5 ms (the 256-MiB copy, then the front, before MSM 1).
  const std::vector<size_t> fgb = front_groups(count, fg_max);
  const size_t nfg = fgb.size() - 1;
  // every buffer the loop touches exists before the first launch (an allocation
  // inside the issue loop could synchronise the device)
  const size_t NB = bucket_count(), n = n_;
  if (acc_groups)
    for (DevBuf &b : gbuckets_) b.ensure(fg_max * NB * sizeof(Xyzz<typename FieldOf<G>::F>));
  else
    for (int b = 0; b < std::max(kBSets, nl); ++b) buckets_[b].ensure(NB * sizeof(Xyzz<typename FieldOf<G>::F>));
  // sized for kGroup whatever this batch's R: a later, larger batch must not
  // reallocate (a hipFree inside the pipelined region would synchronise it)
  // (both reducer sets, and both bucket sets, whatever this batch's length: a
  // short warm-up batch must leave nothing to allocate inside a longer one)
  // front sets and reducer sets in rotation: the lane schedule (small MSMs,
  // periods of a few hundred us) keeps fronts further ahead and lets group q
  // reuse reducer set q % 4 after tail q - 4 (a tail is ~30 latency-bound
  // launches, ~1 ms beside the accumulations: with 2 sets group q + 2 waited
  // for it, profiles/archive_r01_r04.txt (r04_batch_trace_2p17.txt))
  // Front phase (small-MSM accumulation groups; MSM_FRONT_PHASE=1 enables):
  // one front set per front group, up to kFrontPhase (capped at ~4 GiB of
  // front sets), and the first accumulation waits for every front of that
  // phase.  Fronts beside accumulations starve (their 1024-thread fine-pass
  // workgroups wait for a whole CU to drain: 1.1-1.6 ms instead of 34 us in the
  // 2^17 trace, profiles/r05_small_trace.txt); run first, on the whole chip,
  // the batch's fronts take ~60 us per set and the accumulations then run
  // without them.
  // measured slower, so off by default: 2^17 shard 0.461 vs 0.438 ms per MSM,
  // 2^16 plain 0.385 vs 0.368 (profiles/r05_shard_pip_study.txt)
  static const bool phase_env = [] {
    const char *e = getenv("MSM_FRONT_PHASE");
    return e && atoi(e) != 0;
  }();
  const bool phase = acc_groups && phase_env;
  const size_t fs_bytes = fg_max * n * (size_t)p_.h * 16 + 1;  // ~ one front set (sorted, ranks, interleave)
  const int nfr = phase ? (int)std::max<size_t>(kFrontsMax, std::min<size_t>(kFrontPhase, ((size_t)4 << 30) / fs_bytes))
                        : nl >= 2 ? kFrontsMax : kFronts;
  const int nred = nl >= 2 ? 4 : 2;
  if ((int)fs_.size() < nfr) fs_.resize(nfr);
  for (int t = 0; t < nred; ++t) red.ensure_group(t, (int)group_max);
  // front sets sized for a whole front group (the sort's scan scratch too): run
  // one sort of fg_max sets per set before the loop if they are not yet sized
  // (fg_max dummy sets of all-zero scalars, outside the batch timing)
  const size_t sslot = n * stride;  // one device scalar slot
  bool unsized = false;
  for (int f = 0; f < nfr; ++f) unsized |= fs_[f].sorted.bytes < n * (size_t)p_.h * fg_max * 4;
  // host sets: device slots for up to 32 front groups (<= 2 GiB, at least 4),
  // so a batch of up to 32 groups issues every copy at its start and the copy
  // stream runs them back to back, ahead of the fronts; a longer batch copies
  // group g once group g - nsg's front has consumed its slots.  With 4 slots
  // (copies issued 4 MSMs ahead, each after a front event) the 2^20 H2D
  // headline fell into a slow schedule in about half the runs (372-391 vs
  // 411-417 M pairs/s, more often after a 3-set warm-up); with a slot per set
  // every run gave 418-423 M (profiles/archive_r01_r04.txt (r04_h2d_slots_ab.txt))
  static const size_t nsg_env = [] {
    const char *e = getenv("MSM_H2D_SLOTS");  // A/B knob: slot groups (copies issued that far ahead)
    return (size_t)(e ? std::max(2, std::min(256, atoi(e))) : 0);
  }();
  const size_t slot_groups =
      std::max<size_t>(nsg_env ? nsg_env : std::max<size_t>(4, std::min<size_t>(32, ((size_t)2 << 30) / (fg_max * sslot))),
                       (size_t)nfr - 1);
  // (every group's copies are enqueued before its front: nsg >= nfr - 1)
  const size_t nsg = std::max<size_t>(std::min(slot_groups, nfg), (size_t)nfr - 1);
  // sized for slot_groups whatever this batch's length: a later, longer batch
  // must not reallocate inside its pipelined region
  if (scalars_on_host) scal_.ensure(slot_groups * fg_max * sslot + 16);
  if (unsized) scal_.ensure(fg_max * sslot + 16);
  for (int f = 0; f < nfr; ++f)
    if (fs_[f].sorted.bytes < n * (size_t)p_.h * fg_max * 4) {
      MSM_HIP_CHECK(hipMemsetAsync(scal_.p, 0, fg_max * sslot, s));
      digits_sort(s, scal_.as<uint8_t>(), stride, sslot, (int)fg_max, f);
      MSM_HIP_CHECK(hipStreamSynchronize(s));
    }
  const bool prof = profile_;
  profile_ = false;
  if (prof)
    while (acc_ev_.size() < std::max<size_t>(2 * count, 2 * 64)) {
      hipEvent_t e;
      MSM_HIP_CHECK(hipEventCreate(&e));
      acc_ev_.push_back(e);
    }
  // Streams, front groups g (front set g % nfr), bucket sets k % kBSets and,
  // for host scalars, nsg groups of device scalar slots (g % nsg):
  //   fstream_:  digits + sort of front group g: ONE pass per stage over its R_g
  //              scalar sets (bucket_sort.hpp), after group g - 3's accumulations
  //              released the front set.  Issued when group g - 2's accumulations
  //              are enqueued, so it runs beside them or g - 1's; at the greatest priority,
  //              its short memory-bound kernels take the CU slots the
  //              accumulation's retiring workgroups free;
  //   s:         accumulation k into bucket set k % kBSets (after MSM k-2's
  //              reduction head released it) -- back to back, the VALU-bound
  //              critical path;
  //   tails_[t]: the reductions of reduction group q = k / R, t = q % 2: level 0
  //              of each MSM into its slot of reducer set t right after its
  //              accumulation, then, after the group's last MSM, ONE launch per
  //              tail level for the whole group and one read-back.  Every launch
  //              that runs beside an accumulation costs it ~10-20 us
  //              (profiles/archive_r01_r04.txt (r02_batch_sched2.txt)), so the ~35 latency-bound levels
  //              are paid once per group, not once per MSM.  Two streams: group
  //              q+1's level 0s never queue behind group q's tail;
  //   cstream_:  host scalars: the H2D copies of front group g's sets into slot
  //              group g % nsg, after front g - nsg consumed it, on their own stream.
  // No host waits inside the loop: every MSM has its own pinned read-back slot.
  // Reducer set t is reused by group q + 2 only after group q's tail: both are
  // in order on tails_[t].
  // dependency events for at least 64 MSMs, created once (not inside a timed batch)
  while (bev_.size() < std::max<size_t>(3 * count + 2 * nfg + ngroups + 1, 3 * 64 + 3 * 64 + 1)) {
    hipEvent_t e;
    MSM_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    bev_.push_back(e);
  }
  hipEvent_t *eva = bev_.data() + 1, *evh = eva + count, *evf = evh + count, *evc = evf + nfg, *evt = evc + nfg;
  std::vector<size_t> prof_k;  // profiling: acc_ev_ pairs recorded (per MSM, or per accumulation group)
  MSM_HIP_CHECK(hipEventRecord(bev_[0], s));  // the batch starts after prior work on s
  MSM_HIP_CHECK(hipStreamWaitEvent(fstream_, bev_[0], 0));
  // The copy stream does NOT wait on the batch-start event: an SDMA copy
  // enqueued behind a cross-stream event wait now and then blocked the issuing
  // thread -- the one that enqueues the whole pipeline -- for 7-9 ms (rocprofv3
  // HIP API traces of bench.py: the batch's second hipMemcpyAsync took 7.4 ms in
  // 3 of 5 traced runs, the GPU idle meanwhile; tools/microbench/copy_block.hip:
  // blocked calls only with the wait; profiles/r05_h2d_block.txt).  Prior work
  // on the caller's stream (which may write the host sets) is awaited on the
  // host instead; the device slots are only read by this engine's batches,
  // which end synchronised.
  if (scalars_on_host) MSM_HIP_CHECK(hipEventSynchronize(bev_[0]));
  for (int t = 0; t < kBSets; ++t) MSM_HIP_CHECK(hipStreamWaitEvent(tails_[t], bev_[0], 0));
  auto slots = [&](size_t g) { return scal_.as<uint8_t>() + (g % nsg) * fg_max * sslot; };
  // MSM_ZERO_COPY_SCALARS=1 (A/B knob): page-locked host sets are read by the
  // digit kernel straight over PCIe instead of being copied by SDMA first
  static const bool zc_env = [] {
    const char *e = getenv("MSM_ZERO_COPY_SCALARS");
    return e && atoi(e) != 0;
  }();
  bool zero_copy = false;
  if (scalars_on_host && zc_env) {
    hipPointerAttribute_t a;
    zero_copy = hipPointerGetAttributes(&a, scalars) == hipSuccess && a.type == hipMemoryTypeHost;
    if (!zero_copy) (void)hipGetLastError();
  }
  auto copy_group = [&](size_t g) {
    if (!scalars_on_host || zero_copy || g >= nfg) return;
    if (g >= nsg) MSM_HIP_CHECK(hipStreamWaitEvent(cstream_, evf[g - nsg], 0));  // slots consumed by front g - nsg
    for (size_t k = fgb[g]; k < fgb[g + 1]; ++k)
      MSM_HIP_CHECK(hipMemcpyAsync(slots(g) + (k - fgb[g]) * sslot, job_scalars(k), sslot, hipMemcpyHostToDevice,
                                   cstream_));
    MSM_HIP_CHECK(hipEventRecord(evc[g], cstream_));
  };
  static const bool front_after_l0 = [] {
    const char *e = getenv("MSM_FRONT_AFTER_L0");
    return e && atoi(e) != 0;
  }();
  // Paced copies (MSM_COPY_PACE=L, default 8; 0 or < 3: all at the batch
  // start): the first L front groups' sets are copied at the batch start, the
  // copy of group g >= L is issued when the accumulation L MSMs before it has
  // finished (a host wait on its event -- no cross-stream wait on the copy
  // stream), so later copies run one per period beside one MSM instead of back
  // to back beside the first five: 2^20 H2D 436.4 / 439.2 / 439.9 vs 432.4 /
  // 436.2 / 436.7 M pairs/s (L = 8 vs all at the start, tools/h2d_ab.py
  // medians, alternating on one box; profiles/r05_copy_pace_ab.txt).  The wait
  // targets MSM fgb[g] - L clamped to the last accumulation already enqueued in
  // THIS batch (acc_enq; in the accumulation-group schedule front g is issued
  // when only the groups up to g - nfr + 1 are enqueued), so it
  // never waits on a stale or unrecorded event and cannot deadlock.
  static const size_t pace_env = [] {
    const char *e = getenv("MSM_COPY_PACE");
    return (size_t)(e ? std::max(0, std::min(32, atoi(e))) : 8);
  }();
  const size_t pace = scalars_on_host && !zero_copy && pace_env >= 3 ? pace_env : 0;
  size_t acc_enq = 0;  // accumulations whose eva[] event is recorded in this batch
  auto front_group = [&](size_t g) {
    if (g >= nfg) return;
    const bool copied = scalars_on_host && !zero_copy;
    if (pace && g >= pace && g < nsg) {
      if (acc_enq) MSM_HIP_CHECK(hipEventSynchronize(eva[std::min(fgb[g] - pace, acc_enq - 1)]));
      copy_group(g);
    }
    if (copied) MSM_HIP_CHECK(hipStreamWaitEvent(fstream_, evc[g], 0));
    if (g >= (size_t)nfr) {  // front set g % nfr: every accumulation of group g - nfr has read it
      const size_t last = fgb[g - nfr + 1] - 1;
      MSM_HIP_CHECK(hipStreamWaitEvent(fstream_, eva[last], 0));
      // A/B knob: also after that MSM's level 0, so the front starts beside the
      // next accumulation instead of beside level 0 (one-lane schedule);
      // measured no better (profiles/archive_r01_r04.txt (r04_h2d_slots_ab.txt), call 19)
      if (front_after_l0 && nl < 2) MSM_HIP_CHECK(hipStreamWaitEvent(fstream_, evh[last], 0));
      for (size_t d = 1; d < (size_t)nl && last >= d && last - d >= fgb[g - nfr]; ++d)  // its other lanes
        MSM_HIP_CHECK(hipStreamWaitEvent(fstream_, eva[last - d], 0));
    }
    const uint8_t *src = copied ? slots(g) : job_scalars(fgb[g]);
    digits_sort(fstream_, src, stride, copied ? sslot : jstride, (int)(fgb[g + 1] - fgb[g]), (int)(g % nfr),
                fine_bt);
    MSM_HIP_CHECK(hipEventRecord(evf[g], fstream_));
  };
  for (size_t g = 0; g < (pace ? std::min(nsg, pace) : nsg); ++g) copy_group(g);
  // Accumulation k waits for level 0 of MSM k - 1, so level 0 runs beside the
  // fronts, never beside the next accumulation.  Without this wait the batch
  // fell, in about one run in three, into a schedule where fronts ran two MSMs
  // ahead and every accumulation started at once beside the previous level 0:
  // level 0 then took 0.5-1.2 ms instead of 0.41, the accumulations 2.2-2.7 ms
  // instead of 1.8, and the H2D headline 342-386 M pairs/s instead of ~420
  // (kernel traces, profiles/archive_r01_r04.txt (r03_spread_trace.txt)); with it 19 of 19 runs on
  // three boxes gave 410-422 M (profiles/archive_r01_r04.txt (r03_ab_studies.txt) r03a0*).
  // G2 (5-ms accumulations, 1.2-ms level 0) never showed the slow mode and
  // runs 1.5 % faster free-running (r03a0g2), so the wait is the G1 default;
  // MSM_ACC_AFTER_L0=0 / =1 forces either schedule for both groups.
  static const int l0_env = [] {
    const char *e = getenv("MSM_ACC_AFTER_L0");
    return e ? (atoi(e) != 0 ? 1 : 0) : -1;
  }();
  const bool l0_first = l0_env < 0 ? G == 1 : l0_env == 1;
  // Fronts run up to nfr - 1 groups ahead on their own stream, but each is
  // ENQUEUED after the accumulation before it: enqueuing the first nfr - 1
  // fronts (7 launches each) before the first accumulation cost ~0.3 ms of host
  // time at the start of a small-MSM batch (profiles/r05_small_trace.txt).
  // Front g + 1 is always enqueued before accumulation g + 1 waits on it.
  size_t fronts_issued = 0;
  auto issue_fronts = [&](size_t upto) {  // every front group <= upto not yet enqueued
    for (; fronts_issued <= upto && fronts_issued < nfg; ++fronts_issued) front_group(fronts_issued);
  };
  const size_t nphase = phase ? std::min(nfg, (size_t)nfr) : 1;  // fronts before the first accumulation
  issue_fronts(nphase - 1);
  // Two accumulation lanes (small MSMs, batch_lanes()): MSM k accumulates into
  // bucket set k % 2 on lane stream k % 2 (the caller's s, tails_[0]) and its
  // level 0 follows on the same stream, so accumulations k and k + 1 run side
  // by side -- one small accumulation (a few hundred thousand buckets, one lane
  // each) fills the chip's 3 x 1024 wave slots only ~1 round deep, and its last
  // waves run alone -- while the group tails run on tails_[1].  Bucket set k % 2
  // is reused by lane k % 2 only, in stream order; reducer set q % 2 is reused
  // by group q + 2 after tail q (event evt[q]).
  // Three lanes (MSM_BATCH_LANES=3) add tails_[1] as a lane and move the group
  // tails to the front stream (the process has 4 hardware queues by default,
  // GPU_MAX_HW_QUEUES: one stream per queue).
  // Accumulation groups (small MSMs, one table for every job; MSM_ACC_GROUP=0
  // selects the per-MSM lanes below): front group g's R_g sets accumulate in
  // ONE launch (k_accumulate_sets, into bucket sets gbuckets_[g % 2]) on lane
  // stream g % 2, then ONE level-0 launch per reduction group they touch; the
  // reduction-group tails run on tails_[1].  A small MSM's own grid fills the
  // chip's wave slots about one round deep and its last waves run with the chip
  // half idle; side-by-side lanes left the accumulations at ~0.55 of the madd
  // rate (2^17: 0.65 ms each, 1.5 running at a time; profiles/r05_small_trace.txt).
  if (acc_groups) {
    hipStream_t lane[2] = {s, tails_[0]}, ts = tails_[1];
    for (size_t g = 0; g < nfg; ++g) {
      copy_group(g + nsg);
      const size_t k0 = fgb[g], k1 = fgb[g + 1];
      const int gb = (int)(g & 1);
      hipStream_t L = lane[gb];
      MSM_HIP_CHECK(hipStreamWaitEvent(L, evf[g], 0));
      if (g == 0 && nphase > 1) MSM_HIP_CHECK(hipStreamWaitEvent(L, evf[nphase - 1], 0));  // the front phase
      if (prof) MSM_HIP_CHECK(hipEventRecord(acc_ev_[2 * k0], L));
      accumulate_sets(L, (int)(g % nfr), (int)(k1 - k0), gb, job_table(k0));
      if (prof) {
        MSM_HIP_CHECK(hipEventRecord(acc_ev_[2 * k0 + 1], L));
        prof_k.push_back(k0);
      }
      for (size_t k = k0; k < k1; ++k) MSM_HIP_CHECK(hipEventRecord(eva[k], L));
      acc_enq = k1;
      for (size_t a = k0; a < k1;) {  // level 0, one launch per reduction group touched
        const size_t q = grp(a), b = std::min(k1, gfirst[q + 1]);
        if (q >= (size_t)nred) MSM_HIP_CHECK(hipStreamWaitEvent(L, evt[q - nred], 0));  // reducer set free again
        red.launch_head_slots(L, gbuckets_[gb].as<uint8_t>() + (a - k0) * NB * sizeof(Xyzz<typename FieldOf<G>::F>), NB,
                              (int)(q % nred), (int)gslot(a), (int)(b - a));
        a = b;
      }
      for (size_t k = k0; k < k1; ++k) MSM_HIP_CHECK(hipEventRecord(evh[k], L));
      for (size_t k = k0; k < k1; ++k) {  // tails of the reduction groups ending in [k0, k1)
        if (!gend(k)) continue;
        const size_t q = grp(k), first = gfirst[q];
        MSM_HIP_CHECK(hipStreamWaitEvent(ts, evh[k], 0));  // this lane's level 0s of group q
        if (k0 >= 1 && k0 - 1 >= first) MSM_HIP_CHECK(hipStreamWaitEvent(ts, evh[k0 - 1], 0));  // the other lane's
        group_tail(ts, (int)(q % nred), first, k - first + 1, k + 1 == count);
        MSM_HIP_CHECK(hipEventRecord(evt[q], ts));
      }
      issue_fronts(g + nfr - 1);
    }
  }
  if (nl >= 2 && !acc_groups) {
    hipStream_t lane[3] = {s, tails_[0], tails_[1]}, ts = nl == 3 ? fstream_ : tails_[1];
    for (size_t g = 0; g < nfg; ++g) {
      copy_group(g + nsg);
      for (size_t k = fgb[g]; k < fgb[g + 1]; ++k) {
        hipStream_t L = lane[k % nl];
        const size_t q = grp(k);
        const int bset = (int)(k % nl), slot = (int)gslot(k), gset = (int)(q % nred);
        MSM_HIP_CHECK(hipStreamWaitEvent(L, evf[g], 0));
        if (q >= (size_t)nred && slot < nl)  // reducer set q % nred free again
          MSM_HIP_CHECK(hipStreamWaitEvent(L, evt[q - nred], 0));
        if (prof) MSM_HIP_CHECK(hipEventRecord(acc_ev_[2 * k], L));
        accumulate(L, (int)(g % nfr), (int)(k - fgb[g]), bset, job_table(k));
        if (prof) {
          MSM_HIP_CHECK(hipEventRecord(acc_ev_[2 * k + 1], L));
          prof_k.push_back(k);
        }
        MSM_HIP_CHECK(hipEventRecord(eva[k], L));
        acc_enq = k + 1;
        red.launch_head_slot(L, buckets_[bset].p, gset, slot);
        MSM_HIP_CHECK(hipEventRecord(evh[k], L));
        if (gend(k)) {  // the group's level 0s are done on both lanes
          for (int d = 0; d < nl && d <= slot; ++d) MSM_HIP_CHECK(hipStreamWaitEvent(ts, evh[k - d], 0));
          group_tail(ts, gset, k - slot, slot + 1, k + 1 == count);
          MSM_HIP_CHECK(hipEventRecord(evt[q], ts));
        }
      }
      issue_fronts(g + nfr - 1);
    }
  }
  // Level 0 inside the next accumulation's grid (A/B knob, off by default:
  // measured slower, resident 434-438 vs 446-450 M pairs/s, G2 164.4 vs 165.3 M,
  // profiles/archive_r01_r04.txt (r04_l0_fuse_ab.txt); MSM_L0_FUSE=1: level-0 workgroups first, =2:
  // last; k_accumulate_l0 / k_accumulate2p_l0): MSM k's launch also runs
  // level 0 of MSM k - 1 on the caller's stream, the last MSM's level 0 runs
  // alone after the loop, and reducer set q % 2 is reused by group q + 2 only
  // after tail q (event evt[q]: level 0 no longer runs on the tail's stream).
  static const int fuse_env = [] {
    const char *e = getenv("MSM_L0_FUSE");
    return e ? std::max(0, std::min(2, atoi(e))) : 0;
  }();
  const int fuse = nl < 2 ? fuse_env : 0;
  auto l0_group_tail = [&](size_t p) {  // after level 0 of MSM p (recorded as evh[p] on s)
    const size_t pq = grp(p), pslot = gslot(p);
    if (!gend(p)) return;
    hipStream_t ts = tails_[pq % 2];
    MSM_HIP_CHECK(hipStreamWaitEvent(ts, evh[p], 0));
    group_tail(ts, (int)(pq % 2), p - pslot, pslot + 1, p + 1 == count);
    MSM_HIP_CHECK(hipEventRecord(evt[pq], ts));
  };
  auto l0_set_free = [&](size_t p) {  // level 0 of MSM p may write its reducer set
    const size_t pq = grp(p);
    if (gslot(p) == 0 && pq >= 2) MSM_HIP_CHECK(hipStreamWaitEvent(s, evt[pq - 2], 0));
  };
  for (size_t g = 0; g < (nl >= 2 || !fuse ? 0 : nfg); ++g) {
    copy_group(g + nsg);
    MSM_HIP_CHECK(hipStreamWaitEvent(s, evf[g], 0));
    for (size_t k = fgb[g]; k < fgb[g + 1]; ++k) {
      const int bset = (int)(k % kBSets);
      if (k >= 1) l0_set_free(k - 1);
      if (prof) MSM_HIP_CHECK(hipEventRecord(acc_ev_[2 * k], s));
      if (k >= 1)
        accumulate_l0(s, (int)(g % nfr), (int)(k - fgb[g]), bset, job_table(k), (int)((k - 1) % kBSets),
                      (int)(grp(k - 1) % 2), (int)gslot(k - 1), fuse == 2);
      else
        accumulate(s, (int)(g % nfr), (int)(k - fgb[g]), bset, job_table(k));
      if (prof) {
        MSM_HIP_CHECK(hipEventRecord(acc_ev_[2 * k + 1], s));
        prof_k.push_back(k);
      }
      MSM_HIP_CHECK(hipEventRecord(eva[k], s));
      acc_enq = k + 1;
      if (k >= 1) {
        MSM_HIP_CHECK(hipEventRecord(evh[k - 1], s));
        l0_group_tail(k - 1);
      }
    }
    issue_fronts(g + nfr - 1);
  }
  if (fuse && nl < 2) {  // level 0 of the last MSM, alone
    const size_t p = count - 1;
    l0_set_free(p);
    red.launch_head_slot(s, buckets_[p % kBSets].p, (int)(grp(p) % 2), (int)gslot(p));
    MSM_HIP_CHECK(hipEventRecord(evh[p], s));
    l0_group_tail(p);
  }
  for (size_t g = 0; g < (nl >= 2 || fuse ? 0 : nfg); ++g) {
    copy_group(g + nsg);
    MSM_HIP_CHECK(hipStreamWaitEvent(s, evf[g], 0));
    for (size_t k = fgb[g]; k < fgb[g + 1]; ++k) {
      const int bset = (int)(k % kBSets), slot = (int)gslot(k), gset = (int)(grp(k) % 2);
      hipStream_t ts = tails_[gset];
      if (k >= (size_t)kBSets) MSM_HIP_CHECK(hipStreamWaitEvent(s, evh[k - kBSets], 0));  // bucket set free again
      if (l0_first && k >= 1) MSM_HIP_CHECK(hipStreamWaitEvent(s, evh[k - 1], 0));
      if (prof) MSM_HIP_CHECK(hipEventRecord(acc_ev_[2 * k], s));
      accumulate(s, (int)(g % nfr), (int)(k - fgb[g]), bset, job_table(k));
      if (prof) {
        MSM_HIP_CHECK(hipEventRecord(acc_ev_[2 * k + 1], s));
        prof_k.push_back(k);
      }
      MSM_HIP_CHECK(hipEventRecord(eva[k], s));
      acc_enq = k + 1;
      MSM_HIP_CHECK(hipStreamWaitEvent(ts, eva[k], 0));
      red.launch_head_slot(ts, buckets_[bset].p, gset, slot);
      MSM_HIP_CHECK(hipEventRecord(evh[k], ts));
      if (gend(k)) {  // the reduction group's last MSM
        group_tail(ts, gset, k - slot, slot + 1, k + 1 == count);
      }
    }
    issue_fronts(g + nfr - 1);
  }
  // the caller's stream observes completion of every reduction (and front)
  MSM_HIP_CHECK(hipEventRecord(ev_tail_[0], fstream_));
  MSM_HIP_CHECK(hipStreamWaitEvent(s, ev_tail_[0], 0));
  for (int t = 0; t < kBSets; ++t) {
    MSM_HIP_CHECK(hipEventRecord(ev_tail_[t], tails_[t]));
    MSM_HIP_CHECK(hipStreamWaitEvent(s, ev_tail_[t], 0));
  }
  for (int t = 0; t < kBSets; ++t) MSM_HIP_CHECK(hipStreamSynchronize(tails_[t]));
  MSM_HIP_CHECK(hipStreamSynchronize(fstream_));  // three lanes: the group read-backs ran on the front stream
  // the per-MSM host Horner (~20 us each) over the host worker threads: with
  // one reduction group per batch every combine runs after the last tail
  const size_t last_first = gfirst[ngroups - 1];  // the last group's MSMs: host_bits_ when bit_tail
  auto combine_k = [&](size_t k) {
    outs[k] = bit_tail && k >= last_first ? red.combine_bits((const uint8_t *)host_bits_ + (k - last_first) * bb)
                                          : red.combine((const uint8_t *)host_out_ + k * ob)[0];
  };
  if (dev_out) {
    // the window sums stay in dev_out for the caller's exchange
  } else if (count >= 4) {
    WorkerPool::get().parallel_for(count, combine_k);
  } else {
    for (size_t k = 0; k < count; ++k) combine_k(k);
  }
  profile_ = prof;
  if (prof) {  // accumulation time per MSM over the batch (HIP events on the accumulation streams)
    float sum = 0;
    for (size_t k : prof_k) {
      float ms;
      MSM_HIP_CHECK(hipEventSynchronize(acc_ev_[2 * k + 1]));
      MSM_HIP_CHECK(hipEventElapsedTime(&ms, acc_ev_[2 * k], acc_ev_[2 * k + 1]));
      sum += ms;
    }
    times_ = PhaseTimes();
    times_.accumulate = sum / (float)count;
    times_.accumulate_launches = (int)prof_k.size();
  }
}

template class Ches<MSM_GROUP>;

}  // namespace msm
