// engine.hpp -- host-side orchestration of the MSM kernels on one MI355X.
// Internal C++ API; the C ABI (abi.cpp) and the Python mirror sit on top.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "acc_sched.hpp"
#include "host_fp.hpp"

#define MSM_HIP_CHECK(x)                                                                           \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess)                                                                         \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e_) + " at " + #x); \
  } while (0)

namespace msm {

class HostStager;  // hoststage.hpp: pinned-ring uploads from pageable caller memory

inline unsigned nblk(size_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

// Front groups of a batch (MSMs [fgb[g], fgb[g + 1]) share one digits + sort
// pass and, for small MSMs, one accumulation launch): 1, 1, 2, 4, then fg_max
// each.  taper (MSM_FRONT_TAPER=1, A/B knob): the last group split in halves
// down to one MSM (4 -> 2, 1, 1), so the level 0 that follows the batch's last
// accumulation covers one MSM and the earlier level 0s run beside the last
// accumulations.  Measured no better (2^17 shard 0.429 / 0.411 vs 0.414 / 0.436
// ms, configs[1] 0.340 / 0.341 vs 0.334 / 0.339; profiles/r06_taper_prefetch_ab.txt).
inline std::vector<size_t> front_groups(size_t count, size_t fg_max) {
  static const bool taper = [] {
    const char *e = getenv("MSM_FRONT_TAPER");
    return e && atoi(e) != 0;
  }();
  std::vector<size_t> fgb{0};
  while (fgb.back() < count)
    fgb.push_back(std::min(count, fgb.back() + std::min<size_t>(fg_max, std::max<size_t>(1, fgb.back()))));
  if (taper && fgb.size() >= 2) {
    size_t first = fgb[fgb.size() - 2], len = count - first;
    fgb.pop_back();
    while (len > 1) {
      const size_t half = (len + 1) / 2;
      fgb.push_back(first + half);
      first += half;
      len -= half;
    }
    fgb.push_back(count);
  }
  return fgb;
}

struct DevBuf {
  void *p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf &) = delete;
  DevBuf &operator=(const DevBuf &) = delete;
  DevBuf(DevBuf &&o) noexcept : p(o.p), bytes(o.bytes) { o.p = nullptr, o.bytes = 0; }
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  void ensure(size_t b) {
    if (b <= bytes) return;
    release();
    MSM_HIP_CHECK(hipMalloc(&p, b));
    bytes = b;
  }
  template <class T>
  T *as() const {
    return reinterpret_cast<T *>(p);
  }
};

// per-phase device time of the last run (ms), filled when profiling is on
struct PhaseTimes {
  float digits = 0, sort = 0, accumulate = 0, reduce = 0, finalize = 0, total = 0;
  int accumulate_launches = 0;
};

template <int G>
struct HostField;
template <>
struct HostField<1> {
  typedef hfp::Fp F;
};
template <>
struct HostField<2> {
  typedef hfp::Fp2 F;
};

// Two-level LDS counting sort of (bucket, payload) entries (bucket_sort.hpp).
// Produces payloads grouped by bucket, per-bucket counts/offsets and the
// accumulation schedule (bucket ids by descending count).
struct BucketSort {
  DevBuf ghist, gbase, okeys, ovals, classes, tmp;
  // the schedule's per-position count and payload offset (scnt[t] = counts[order[t]],
  // soff[t] = offsets[order[t]]), the wave groups' interleaved rows (wlen, wbase)
  // and the interleaved payload
  DevBuf scnt, soff, wbase, ipay;
  size_t ipay_stride = 0;  // interleaved entries per set (ne + BS_IPAY_SLACK)
  int fine_bt = 1024;      // k_bs_fine workgroup size: 1024 alone, 256 under a batch's accumulations
  static size_t groups(size_t nb) { return (nb + 63) / 64; }
  // set `set` of the last run (nb buckets per set); order/sorted as passed to run
  AccSched sched(const uint32_t *order, const uint32_t *sorted, size_t set, size_t nb) const {
    const size_t nw = groups(nb);
    return AccSched{order + set * nb,
                    scnt.as<uint32_t>() + set * nb,
                    soff.as<uint32_t>() + set * nb,
                    wbase.as<uint32_t>() + set * nw,
                    ipay.as<uint32_t>() + set * ipay_stride,
                    sorted};
  }
  // the per-set offsets between consecutive sets of one multi-set sort
  AccStride stride(size_t nb) const { return AccStride{nb, groups(nb), ipay_stride}; }
  // keys[ne] (bucket < nb or 0xffffffff), vals[ne]; outputs sized ne / nb.
  // nsets > 1: nsets independent sorts in the same launches -- inputs at
  // keys/vals + r ne, outputs counts/offsets/order + r nb (offsets index the one
  // shared `sorted` array of up to nsets ne entries), bucket_sort.hpp
  void run(hipStream_t s, const uint32_t *keys, const uint32_t *vals, size_t ne, uint32_t nb, uint32_t *sorted,
           uint32_t *counts, uint32_t *offsets, uint32_t *order, int nsets = 1);
  // run() in pieces, for a caller that bins its entries itself (the fused CHES
  // front, ches_kernels.hpp k_ches_front_hist / _coarse): prepare sizes every
  // buffer for ntiles histogram tiles per set (0: ceil(ne / BS_TILE)); the
  // caller fills ghist, scan() writes gbase, the caller bins into okeys / ovals,
  // finish() runs the fine pass, the schedule and the interleave.
  struct Geom {
    int fb_bits = 8, ncb = 1, ntiles = 1;
    size_t nslots = 0, scan_tmp = 0;
  };
  Geom prepare(hipStream_t s, size_t ne, uint32_t nb, int nsets, int ntiles);
  void scan(hipStream_t s, const Geom &g);
  void finish(hipStream_t s, const Geom &g, size_t ne, uint32_t nb, uint32_t *sorted, uint32_t *counts,
              uint32_t *offsets, uint32_t *order, int nsets);
  size_t device_bytes() const {
    return ghist.bytes + gbase.bytes + okeys.bytes + ovals.bytes + classes.bytes + tmp.bytes + scnt.bytes + soff.bytes +
           wbase.bytes + ipay.bytes;
  }
};

// sum_w 2^(c w) T_w, Horner from the top window (ref multi_scalar.c:565-575)
template <class HF>
hfp::Jac<HF> horner(const std::vector<hfp::Jac<HF>> &T, int c) {
  hfp::Jac<HF> ret = T.back();
  for (int w = (int)T.size() - 2; w >= 0; --w) {
    for (int k = 0; k < c; ++k) ret = hfp::dbl(ret);
    ret = hfp::addj(ret, T[w]);
  }
  return ret;
}


// ---------------------------------------------------------------------------
// CHES "nh + q/5" bucket-set method (ches.hip)
// ---------------------------------------------------------------------------
// parameters of ref ches_config_files/config_file_n_exp_*.h
struct ChesParams {
  int n_exp, beta, q_exp, h, a_h, d_max, b_size, q_exp_bgmw, h_bgmw;
};
bool ches_params_for(int n_exp, int beta, ChesParams *out);
// bucket set B of ref auxiliaryfunc.h:257-288 (ascending)
std::vector<int> ches_bucket_set(int q, int a_h);
// packed digit hash (ches_kernels.hpp layout) of ref main_p1.cpp:140-152, q+1 entries
std::vector<uint32_t> ches_digit_hash(const std::vector<int> &B, int q);
// The same map in the compact device form (ches_kernels.hpp "digit code"):
// a 4-bit code per digit value, 8 per word, (q >> 3) + 2 words, and the rank
// table {membership bits, prefix count} per 32 values of [0, max B].  Throws if
// some H[d] is not (m, (alpha ? q - d : d) / m, alpha).
void ches_digit_code(const std::vector<int> &B, int q, std::vector<uint32_t> &code, std::vector<uint32_t> &rank);

// Low-depth dense reduction: for each of W windows of S buckets (A[w*S + b-1]
// holds bucket value b, S a power of two), T_w = sum_b b A_b computed as the sum
// of all suffix sums: log2(S) Hillis-Steele suffix-scan steps + log2(S) pairwise
// tree steps, one xyzz add per lane per step.  Depth 2 log2(S) adds (vs ~20
// dependent adds per level of the running-sum recursion), which matters
// because a lone dependent xyzz add costs ~15 us of one SIMD's issue time.
template <int G>
struct ScanReducer {
  typedef typename HostField<G>::F HF;
  DevBuf buf[2], fin;
  // enqueue: fin <- W blst Jacobians (144 G bytes each).  coop: one add per 4
  // waves (coop.hpp; shortest latency when the GPU is otherwise idle) instead of
  // one add per lane (least resource time beside other kernels)
  void launch(hipStream_t s, const void *A, int W, int S, bool coop = true);
  void read(hipStream_t s, int W, std::vector<hfp::Jac<HF>> &out);
};

// sum_i w[i] * S_i for arbitrary non-negative bucket weights w (w = 0: bucket
// ignored) over device xyzz buckets S (replaces ref multi_scalar.c:301-321).
// Two regroupings by the low and high halves of w[i] (2 xyzz adds per bucket),
// then a dense 2-window ScanReducer and one 2^s Horner step on the host.  The
// plan depends only on w and is built once.  Two independent buffer sets let
// the latency-bound tail of one MSM (launch_tail, on a second stream) overlap
// the next MSM's digits/sort/accumulation/level-0 (launch_head).
template <int G>
class WeightedReducer {
 public:
  typedef typename HostField<G>::F HF;
  static constexpr int NSETS = 4;  // buffer sets, allocated on first use (batch reduction groups rotate over them)
  // win[i] in [0, nwin): the window of bucket i (empty = all in window 0)
  // c0: level-0 chunk length (0: by plan size, see plan())
  void plan(const std::vector<uint32_t> &w, const std::vector<uint32_t> &win, int nwin, int c0 = 0);
  void plan(const std::vector<uint32_t> &w, int c0 = 0) { plan(w, {}, 1, c0); }
  int level0_chunk() const { return c0_; }
  void launch_head(hipStream_t s, const void *S, int set);  // level 0 (reads S = xyzz[w.size()])
  // levels >= 1, dense, finalize; coop: see ScanReducer::launch
  void launch_tail(hipStream_t s, int set, bool coop = true);
  void launch(hipStream_t s, const void *S) {
    launch_head(s, S, 0);
    launch_tail(s, 0);
  }
  size_t out_bytes() const { return (size_t)2 * nwin_ * 144 * G; }
  void copy_out(hipStream_t s, int set, void *host);               // async D2H of out_bytes()
  std::vector<hfp::Jac<HF>> combine(const void *host) const;        // per-window sums
  // sum_w 2^(c w) T_w of a copied-out result in ONE Horner pass over the 2 nwin
  // terms L_w (exponent c w) and H_w (c w + s): (nwin - 1) c + s doublings
  // instead of nwin s + (nwin - 1) c (combine, then horner over the windows)
  hfp::Jac<HF> combine_windows(const void *host, int c) const;
  std::vector<hfp::Jac<HF>> read_windows(hipStream_t s);            // set 0, waits
  hfp::Jac<HF> read(hipStream_t s) { return read_windows(s)[0]; }
  // set 0's sum_w 2^(c w) T_w (after launch_tail), waits
  hfp::Jac<HF> read_total(hipStream_t s, int c);
  size_t size() const { return bsize_; }
  // device bytes held: plan tables, every buffer set (partials, dense slots and
  // their ScanReducer buffers), the bit-phase read-back (engine pool budget)
  size_t device_bytes() const {
    size_t b = idx_.bytes + bfin_.bytes;
    for (int t = 0; t < NSETS; ++t) b += bgfin_[t].bytes;
    for (const DevBuf &d : starts_) b += d.bytes;
    for (const DevBuf &d : bstarts_) b += d.bytes;
    for (int t = 0; t < NSETS; ++t)
      b += dense_buf_[t].bytes + part_[t][0].bytes + part_[t][1].bytes + dense_[t].buf[0].bytes +
           dense_[t].buf[1].bytes + dense_[t].fin.bytes;
    return b;
  }

  void ensure_set(int set);  // allocate buffer set `set` for the current plan

  // Batch groups (Ches::run_batch): the reduction plan is the same for every
  // MSM, so nmsm MSMs share buffer set `set` -- each MSM's level 0 writes its
  // own slot, then ONE launch per tail level reduces all slots together.  A
  // batch then issues ~35 tail launches per group instead of per MSM (every
  // launch beside an accumulation costs it time).
  void ensure_group(int set, int nmsm);
  void launch_head_slot(hipStream_t s, const void *S, int set, int slot);
  // level 0 of nmsm consecutive MSMs (slots slot0 .. slot0 + nmsm - 1 of set
  // `set`) in one launch; MSM j's buckets at S + j sstride points
  void launch_head_slots(hipStream_t s, const void *S, size_t sstride, int set, int slot0, int nmsm);
  // the operands launch_head_slot would pass to its k_segsum (level 0 into slot
  // `slot` of set `set`), for a caller that runs level 0 inside another grid
  struct HeadArgs {
    const uint32_t *idx, *starts;
    void *dst;
    size_t nout;
  };
  HeadArgs head_args(int set, int slot);
  // levels >= 1, dense, finalize; coop: the dense stage's adds over 4 waves each
  // (shortest latency when nothing else runs, e.g. the last group of a batch)
  void launch_tail_group(hipStream_t s, int set, int nmsm, bool coop = false);
  void copy_out_group(hipStream_t s, int set, int nmsm, void *host);  // nmsm * out_bytes()
  // the same group tail ending in 2 s bit sums per MSM instead of the dense
  // stage (one-window plans with a segment phase: has_bit_tail()); the host
  // gets nmsm * bit_bytes() and combine_bits(MSM j's bytes) = combine(...)[0]
  bool has_bit_tail() const { return bits_ && nout_.size() >= 2; }
  size_t bit_bytes() const { return bit_slots() * 144 * G; }
  void launch_tail_group_bits(hipStream_t s, int set, int nmsm, bool coop = false);
  void copy_out_group_bits(hipStream_t s, int set, int nmsm, void *host);
  hfp::Jac<HF> combine_bits(const void *host) const;

 private:
  size_t dense_slots() const { return (size_t)2 * nwin_ << sbits_; }
  size_t bit_slots() const { return (size_t)2 * nwin_ * sbits_; }
  size_t bsize_ = 0, final_perm_off_ = 0, maxp_ = 1;
  size_t maxp1_ = 1;  // batch groups: partials per MSM in part_[.][1] (the odd tail levels)
  int sbits_ = 1, nwin_ = 1, c0_ = 8;
  DevBuf idx_, dense_buf_[NSETS], part_[NSETS][2];
  std::vector<DevBuf> starts_;
  std::vector<size_t> nout_;
  ScanReducer<G> dense_[NSETS];
  // Synchronous tail of a one-window plan (launch_tail / read_windows): the
  // dense 2 x 2^s stage (2 s dependent levels) is replaced by 2 s bit sums
  // B_j = sum of the partials whose value has bit j (j < s: low half, j >= s:
  // high half), ~log2(2^s s / 8) + 2 levels, and a 2 s-step host Horner
  // (T = sum_j 2^j B_j).  Batch groups keep the dense stage (one per group).
  bool bits_ = false;
  size_t bidx_off_ = 0, bperm_off_ = 0;
  std::vector<DevBuf> bstarts_;
  std::vector<size_t> bnout_;
  DevBuf bfin_;
  DevBuf bgfin_[NSETS];  // group bit tails: nmsm x 2 s finalized bit sums per set
};

// digit/sort outputs of one MSM (entries sorted by bucket + schedule); the
// CHES and plain Pippenger batches rotate three of them (front k + 2 beside
// accumulation k)
struct ChesFrontSet {
  DevBuf keys, vals, sorted, counts, offsets, order;
  BucketSort sort;
  size_t device_bytes() const {
    return keys.bytes + vals.bytes + sorted.bytes + counts.bytes + offsets.bytes + order.bytes + sort.device_bytes();
  }
};

// one blst window tile (ref multi_scalar.c:383-419): Booth digit over bits
// [bit0 - 1, bit0 + wbits), cbits = wbits (+ 1 for the top, partial window)
struct TileSpec {
  int bit0, wbits, cbits;
};

// Plain Pippenger bucket method (ref src/multi_scalar.c:549-576) on one GPU.
template <int G>
class Pippenger {
 public:
  typedef typename HostField<G>::F HF;
  Pippenger(int device, int window_bits);
  ~Pippenger();
  // points in blst affine layout (Montgomery R=2^384); host or device memory
  void set_points(const void *points_blst, size_t n, bool on_device, hipStream_t s);
  // scalars: n little-endian byte strings with the given stride, on device
  void run(hipStream_t s, const uint8_t *d_scalars, size_t stride, int nbits, hfp::Jac<HF> *out);
  // points (blst affine) and scalars in host memory: set_points + run with the
  // point upload overlapping the scalars' digits and sort (blst drop-in)
  // tile: one blst window tile instead of the whole MSM (blst_p{1,2}s_tile_pippenger)
  // dev_rows: the points already on this device as AffP rows (a registered
  // host table holding them, table_registry.hpp): nothing is uploaded
  void run_host(hipStream_t s, const void *points_blst, size_t n, const uint8_t *scalars, size_t stride, int nbits,
                hfp::Jac<HF> *out, const TileSpec *tile = nullptr, const void *dev_rows = nullptr);
  // `count` MSMs over the resident points, scalar set k at d_scalars + k
  // set_stride (device memory), pipelined: fronts in groups of up to 4 sets (one
  // digits + sort pass per stage) on a front stream, each group's accumulations
  // in one launch on one of two alternating lane streams (followed by its level
  // 0s); the reduction tails of groups of <= 10 MSMs on a tail stream; the host
  // Horner of group q overlaps the GPU work of later groups.  Results equal
  // `count` run() calls.
  void run_batch(hipStream_t s, const uint8_t *d_scalars, size_t stride, size_t set_stride, size_t count, int nbits,
                 hfp::Jac<HF> *outs);
  size_t npoints() const { return n_; }
  void set_profiling(bool on) { profile_ = on; }
  const PhaseTimes &times() const { return times_; }
  int device() const { return dev_; }
  int window_bits() const { return c_; }
  // bytes this engine holds: device buffers plus its pinned upload ring (the
  // engine pool's idle budget and cache stats count both, pool.hpp)
  size_t device_bytes() const;

 private:
  int dev_, c_;
  size_t n_ = 0;
  bool profile_ = false;
  PhaseTimes times_;
  // kGroup: MSMs per reduction group; 10 (two tails for the 20-MSM configs[1]
  // batch) since the host Horner of a group runs on the worker threads: 0.327-
  // 0.339 vs 0.341-0.353 ms per 2^16 MSM with 8 (profiles/r05_pip_group_ab.txt)
  static constexpr int kFronts = 5, kGroup = 10, kRedSets = 4;
  // digit/sort outputs: fs_[0] for run(); run_batch rotates kFronts of them, or
  // with the front phase one per front group (up to kFrontPhase)
  std::vector<ChesFrontSet> fs_ = std::vector<ChesFrontSet>(kFronts);
  static constexpr int kFrontPhase = 16;
  DevBuf pts_, buckets_[2], tmp_, scal_;
  std::unique_ptr<HostStager> stage_;  // run_host: uploads from the caller's pageable memory
  hipStream_t up_ = nullptr;  // run_host: point upload stream
  const void *ext_rows_ = nullptr;  // run_host with dev_rows: the accumulation reads AffP rows from there
  hipEvent_t ev_up_ = nullptr, ev_s_ = nullptr;
  // run_batch: front stream, second accumulation lane, tail stream; events; read-back slots
  // run_batch streams: fronts, lane 1 (lane 0 is the caller's), tails
  hipStream_t fstream_ = nullptr, lane1_ = nullptr, tstream_ = nullptr;
  std::vector<hipEvent_t> bev_;
  void *host_out_ = nullptr;
  size_t host_out_bytes_ = 0;
  // digits + sort into f; neg: optional per-point sign flips (tiles)
  // nsets > 1: a front group of nsets scalar sets set_stride bytes apart in one pass
  void front(hipStream_t s, const uint8_t *d_scalars, size_t stride, int nbits, const uint8_t *neg, ChesFrontSet &f,
             int nsets = 1, size_t set_stride = 0);
  void accumulate(hipStream_t s, int nbits, ChesFrontSet &f, DevBuf &buckets);
  // the R sets of a front group in one launch, set r's buckets at r NT in bk
  void accumulate_sets(hipStream_t s, int nbits, ChesFrontSet &f, int R, DevBuf &bk);
  DevBuf gbuckets_[2];  // run_batch accumulation groups: two lanes x front-group bucket sets
  void plan_reduction(int nbits);  // reducer plan for this window layout (built once)
  void back(hipStream_t s, int nbits, hfp::Jac<HF> *out);  // accumulate + reduce + read-back (fs_[0])
  WeightedReducer<G> red_;
  // run_batch's reducer: red_, or with MSM_PIP_L0_CHUNK=<2..64> the same
  // weights planned with that level-0 chunk (chunks of 8 measured slower than
  // red_'s 2 at 2^16)
  WeightedReducer<G> bred_;
  WeightedReducer<G> *batch_red_ = &red_;
  int red_W_ = 0, red_tcl_ = -1;  // window count / top copies the reducer plan was built for
  // log2 of the top window's bucket copies (k_digits): 2^topbits digit values
  // spread over its 2^(c-1) slots
  int top_copies_log2(int nbits) const {
    const int W = (nbits + 1 + c_ - 1) / c_;
    const int topbits = nbits - (W - 1) * c_;  // in [0, c - 1]
    return c_ - 1 - topbits;
  }
  std::vector<hipEvent_t> ev_;
};


template <int G>
class Ches {
 public:
  typedef typename HostField<G>::F HF;
  Ches(int device, const ChesParams &p);
  ~Ches();
  // base points (blst affine, host or device) -> table T of 3 n h points, built on the GPU
  void build_table(const void *points_blst, size_t n, bool on_device, hipStream_t s);
  // a precomputed table T (blst affine layout, 3 n h points), host or device
  void set_table(const void *table_blst, size_t n, bool on_device, hipStream_t s);
  // copy T[first, first+count) back in blst affine layout (host memory)
  void get_table(void *out_blst, size_t first, size_t count, hipStream_t s);
  // chunked table upload (file cache): reserve rows for n base points, then
  // put rows [first, first + count) from blst affine layout (host or device)
  void reserve_table(size_t n);
  void put_table(const void *rows_blst, size_t first, size_t count, bool on_device, hipStream_t s);
  size_t table_rows() const { return 3 * (size_t)p_.h * n_; }
  // scalars: n 32-byte LE strings (stride >= 32) on device
  void run(hipStream_t s, const uint8_t *d_scalars, size_t stride, hfp::Jac<HF> *out);
  // `count` MSMs over the same points; scalar set k at scalars + k * set_stride,
  // in device memory or (scalars_on_host) host memory -- then each front group's
  // sets are copied into device slots on their own copy stream (cstream_), ahead
  // of the group's front and overlapping earlier accumulations (pinned host
  // memory for a truly asynchronous copy).  Pipelined: front group g + 1 (digits
  // + sort of up to kFrontGroup sets in one pass) beside group g's
  // accumulations, MSM k's reduction on a second stream beside MSM k+1's
  // accumulation.
  // dev_out (device memory of this engine's device, count * exchange_bytes()):
  // the per-MSM window sums are left there instead of being read back and
  // combined (outs untouched) -- ChesMulti's RCCL exchange
  void run_batch(hipStream_t s, const uint8_t *scalars, size_t stride, size_t set_stride, size_t count,
                 hfp::Jac<HF> *outs, bool scalars_on_host = false, void *dev_out = nullptr) {
    const void *t = table_.p;
    run_jobs(s, scalars, stride, set_stride, count, 1, &t, outs, scalars_on_host, dev_out);
  }
  // bytes of one MSM's window sums in a batch exchange buffer, and their combine
  size_t exchange_bytes() const { return batch_red_->out_bytes(); }
  hfp::Jac<HF> combine_exchange(const void *host) const { return batch_red_->combine(host)[0]; }
  // The batch over nseg point segments of n_ points each, one pipeline: segment
  // d's table is tables[d] (engines of the same parameters and n on this
  // device, e.g. the shards of a multi-shard context that share a GPU), its
  // scalars the d-th n-string slice of every set.  outs: count * nseg partial
  // Jacobians, job k nseg + d = (set k, segment d).
  void run_jobs(hipStream_t s, const uint8_t *scalars, size_t stride, size_t set_stride, size_t count, size_t nseg,
                const void *const *tables, hfp::Jac<HF> *outs, bool scalars_on_host, void *dev_out = nullptr);
  const void *table_ptr() const { return table_.p; }
  size_t npoints() const { return n_; }
  const ChesParams &params() const { return p_; }
  size_t bucket_count() const { return B_.size() + (size_t)(copies_ - 1) * small_; }
  void set_profiling(bool on) { profile_ = on; }
  const PhaseTimes &times() const { return times_; }
  int device() const { return dev_; }
  int batch_lanes() const;  // accumulation streams of run_batch (1, 2 or 3)
  // diagnostic: digits + sort of nsets device scalar sets (set_stride apart) in
  // one front, then the ms of ONE launch accumulating all of them (mean of reps
  // launches, HIP events on stream s); nothing else runs beside it
  float time_accumulation(hipStream_t s, const uint8_t *d_scalars, size_t set_stride, int nsets, int reps);

 private:
  int dev_;
  ChesParams p_;
  std::vector<int> B_;
  size_t n_ = 0;
  // top-digit bucket copies: the top MB digit is <= a_h + 1, so its n entries
  // fall into the few buckets k <= small_ (B[k] <= a_h + 1); entry i of the top
  // digit goes to copy i % copies_ of its bucket (copies share the weight B[k])
  int small_ = 0, copies_ = 1;
  void plan_buckets(size_t n);
  bool profile_ = false;
  PhaseTimes times_;
  // bucket sets: MSM k accumulates into set k % kBSets while the reduction of
  // MSM k-1 still reads the other one
  static constexpr int kBSets = 2;
  static constexpr int kLanesMax = 3;  // batch accumulation lanes (batch_lanes), one bucket set each
  DevBuf code_, rank_, table_, buckets_[kLanesMax];
  // digit/sort outputs.  A batch can run the fronts (digits + sort) of up to
  // kFrontGroup MSMs in ONE pass per stage (seven launches for the group instead
  // of seven per MSM), front group g+2 beside group g's accumulations, three
  // front sets in rotation.  Measured on MI355X (tools/ab_env.sh, profiles/
  // r03_front_group_ab.txt) the grouped fronts slow the accumulations they run
  // beside more than the launches they save (resident 2.33-2.38 ms per MSM with
  // groups of 8 vs 2.26-2.27 with groups of 1), so the default group is one
  // MSM; MSM_FRONT_GROUP=<2..8> selects larger groups.  The synchronous MSM uses
  // set 0 with one scalar set.
  // batch: MSMs per reduction group (WeightedReducer::launch_tail_group).  20:
  // a batch of up to 20 runs one tail, after its last accumulation, instead of
  // tails beside accumulations (each costs the one beside it ~0.3 ms); 20 vs
  // 8 measured +1.2 % (profiles/archive_r01_r04.txt (r04_red_group_ab.txt)).  MSM_RED_GROUP overrides.
  static constexpr int kGroup = 20;
  static constexpr int kFrontGroup = 8;  // batch: largest front group (ramping up 1, 1, 2, 4, 8)
  static constexpr int kFrontGroupDefault = 1;
  // front k+1 may start when accumulation k-2 ends (slack for the copies); the
  // lane schedule of small MSMs rotates kFrontsMax sets (fronts further ahead)
  static constexpr int kFronts = 3, kFrontsMax = 5;
  // front sets: kFronts / kFrontsMax in rotation, or with the front phase of
  // the small-MSM batch one per front group (up to kFrontPhase)
  std::vector<ChesFrontSet> fs_ = std::vector<ChesFrontSet>(kFrontsMax);
  static constexpr int kFrontPhase = 16;
  // host scalar sets of a batch: two groups of kFrontGroup device slots, copied on
  // their own stream (cstream_) ahead of the group's front
  DevBuf scal_;
  DevBuf prime_;  // target of the one-time stream priming launches (run_batch)
  WeightedReducer<G> red_;
  // the batch's reducer: red_ when its level-0 chunk is 8, else bred_, the same
  // weights planned with chunks of 8.  Small plans chunk level 0 by 2-4 for the
  // synchronous MSM's latency; in a batch level 0 runs beside other lanes'
  // accumulations while the grouped tail runs exposed after the last one, so
  // the batch moves the adds into level 0 (2^17: the group tail's first segment
  // level alone was 0.51 ms, profiles/archive_r01_r04.txt (r04_batch_trace_2p17_lanes3.txt)).
  // MSM_BATCH_L0_CHUNK=<2..64> overrides 8; =0 reuses red_.
  WeightedReducer<G> bred_;
  WeightedReducer<G> *batch_red_ = &red_;
  std::vector<hipEvent_t> ev_;
  hipStream_t tails_[kBSets] = {nullptr, nullptr}, fstream_ = nullptr, cstream_ = nullptr;  // batch streams (+ the caller's)
  hipEvent_t ev_tail_[kBSets] = {nullptr, nullptr};
  void *host_out_ = nullptr;
  size_t host_out_bytes_ = 0;
  void *host_bits_ = nullptr;  // the last group's bit-tail read-back (WeightedReducer::launch_tail_group_bits)
  size_t host_bits_bytes_ = 0;
  std::vector<hipEvent_t> bev_;     // batch dependency events, one per (MSM, stage)
  std::vector<hipEvent_t> acc_ev_;  // batch profiling: events around each accumulation
  // digits + sort of nsets scalar sets (set_stride bytes apart) into front set `set`
  // fine_bt: k_bs_fine workgroup size (1024 alone; 256 for a batch front that
  // runs under accumulations, bucket_sort.hpp)
  void digits_sort(hipStream_t s, const uint8_t *d_scalars, size_t stride, size_t set_stride, int nsets, int set,
                   int fine_bt = 1024);
  // accumulation of scalar set r of front set `set` into bucket set bset
  // (table: the table_ of this engine, or of a segment's engine in run_jobs)
  void accumulate(hipStream_t s, int set, int r, int bset, const void *table = nullptr);
  // accumulation group: sets 0 .. R-1 of front set `set` in one launch into
  // the R consecutive bucket sets of gbuckets_[gb]
  void accumulate_sets(hipStream_t s, int set, int R, int gb, const void *table);
  DevBuf gbuckets_[2];  // accumulation groups: two lanes x kFrontGroup bucket sets
  // batch: accumulation as above in the same grid as level 0 of the MSM whose
  // buckets are in l0_bset, into reducer set gset / slot (k_accumulate_l0)
  void accumulate_l0(hipStream_t s, int set, int r, int bset, const void *table, int l0_bset, int gset, int slot,
                     int l0_last);
};

// BGMW95 fixed-base variant (ref main_p1.cpp:94-122, 294-398;
// multi_scalar.c:506-547): table T[i h + j] = q^j P_i resident in HBM, signed
// radix-q digits in (-q/2, q/2], all n h digits accumulated into ONE set of
// q/2 buckets, then sum_b b S_b.  (bgmw.hip)
template <int G>
class Bgmw {
 public:
  typedef typename HostField<G>::F HF;
  Bgmw(int device, int q_exp, int h);
  ~Bgmw();
  void build_table(const void *points_blst, size_t n, bool on_device, hipStream_t s);
  void set_table(const void *table_blst, size_t n, bool on_device, hipStream_t s);  // n h points
  void get_table(void *out_blst, size_t first, size_t count, hipStream_t s);
  void reserve_table(size_t n);
  void put_table(const void *rows_blst, size_t first, size_t count, bool on_device, hipStream_t s);
  size_t table_rows() const { return (size_t)h_ * n_; }
  // scalars: n 32-byte LE strings (stride >= 32) on device
  void run(hipStream_t s, const uint8_t *d_scalars, size_t stride, hfp::Jac<HF> *out);
  size_t npoints() const { return n_; }
  int q_exp() const { return q_exp_; }
  int h() const { return h_; }
  size_t bucket_count() const { return nb0_ + (size_t)(copies_ - 1) * small_; }
  void set_profiling(bool on) { profile_ = on; }
  const PhaseTimes &times() const { return times_; }
  int device() const { return dev_; }

 private:
  int dev_, q_exp_, h_;
  size_t n_ = 0, nb0_ = 0;
  uint32_t small_ = 0;
  int copies_ = 1;
  bool profile_ = false;
  PhaseTimes times_;
  DevBuf table_, keys_, vals_, counts_, offsets_, sorted_, order_, buckets_;
  BucketSort sort_;
  WeightedReducer<G> red_;
  std::vector<hipEvent_t> ev_;
  void plan_buckets(size_t n);
};

// blst's fixed-window MSM with a precomputed table of multiples (wbits.hip;
// ref multi_scalar.c:63-261): table row i = (k+1) P_i for k < 2^(wbits-1),
// resident in HBM; run() sums the Booth-digit gathers per window on the GPU and
// combines the window totals on the host.
template <int G>
class Wbits {
 public:
  typedef typename HostField<G>::F HF;
  Wbits(int device, int wbits);
  // base points (blst affine, host or device) -> table built on the GPU
  void precompute(const void *points_blst, size_t n, bool on_device, hipStream_t s);
  // a table in the reference layout (blst affine, n << (wbits-1) rows), host or device
  void set_table(const void *table_blst, size_t n, bool on_device, hipStream_t s);
  void get_table(void *out_blst, size_t first, size_t count, hipStream_t s);
  // scalars: n little-endian strings of `stride` bytes on device (nullptr: the
  // set last given to upload_scalars); low nbits bits used
  void run(hipStream_t s, const uint8_t *d_scalars, size_t stride, int nbits, hfp::Jac<HF> *out);
  void upload_scalars(const void *host, size_t bytes, hipStream_t s);
  size_t npoints() const { return n_; }
  size_t table_rows() const { return n_ << (wbits_ - 1); }
  int wbits() const { return wbits_; }
  int device() const { return dev_; }
  size_t device_bytes() const { return table_.bytes + parts_[0].bytes + parts_[1].bytes + fin_.bytes + scal_.bytes; }

 private:
  int dev_, wbits_;
  size_t n_ = 0;
  DevBuf table_, parts_[2], fin_, scal_;
};

// blst-level tile entry points (compat.hip): sum_b weights[b] * (sum of the
// entries of bucket b), entries (keys[k] = bucket or KEY_NONE, vals[k] = point
// index | sign << 31) over npts blst affine points in host memory; bucket sums
// optionally written back in blst xyzz layout to host memory buckets_out.
template <int G>
void entry_msm(void *ret_jac, const void *pts_blst, size_t npts, const uint32_t *keys, const uint32_t *vals,
               size_t ne, size_t nb, const uint32_t *weights, void *buckets_out);
// The same for entries named by per-entry point pointers (the blst-level CHES /
// BGMW95 tiles: entry t's point is *points[t], ref multi_scalar.c:421-547):
// fill(ctx, t0, t1, keys, vals) writes the keys / vals of entries [t0, t1)
// (called concurrently on disjoint ranges by the host worker pool).  Keys,
// vals and the gathered point rows are staged through page-locked memory in
// chunks, the host gather of chunk c + 1 overlapping the DMA of chunk c.
typedef void (*EntryFill)(void *ctx, size_t t0, size_t t1, uint32_t *keys, uint32_t *vals);
template <int G>
void entry_msm_ptrs(void *ret, const void *const *points, size_t ne, EntryFill fill, void *fill_ctx, size_t nb,
                    const uint32_t *weights, void *buckets_out);
// sum_i weights[i] * buckets[i] for nb blst xyzz buckets in host memory
template <int G>
void weighted_bucket_sum(void *ret_jac, const void *buckets_blst, size_t nb, const uint32_t *weights);

// VALU ceilings of this device, measured now (probe.hip): {mad lane-ops/s,
// Fp-mul/s, G1 madd/s, device ms spent}
void valu_probe(int device, double out[4]);
// device self-tests (engine.hip)
template <int G>
void test_field(int op, const uint64_t *a, const uint64_t *b, uint64_t *out, size_t n);
template <int G>
void test_xyzz(const uint64_t *pts, size_t npts, const uint32_t *ops, int len, size_t nseq, uint64_t *out);

// set/get device of the calling thread around engine calls
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    MSM_HIP_CHECK(hipGetDevice(&prev));
    if (prev != dev) MSM_HIP_CHECK(hipSetDevice(dev));
  }
  ~DeviceGuard() {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur != prev && prev >= 0) (void)hipSetDevice(prev);
  }
};

}  // namespace msm
