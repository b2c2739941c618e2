// abi.cpp -- extern "C" boundary of libmsm_mi355x.so (include/msm_mi355x.h).
//
// The blst-named entry points reproduce the reference's calling convention
// (ref src/multi_scalar.c:581-607: arrays of pointers with the {ptr, NULL}
// flat shortcut, scalars packed with stride (nbits+7)/8) and run the MSM on
// the GPU; the msm_* functions expose device-resident contexts.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <string>

#include "../../include/msm_mi355x.h"
#include "engine.hpp"
#include "multi.hpp"
#include "pool.hpp"
#include "ptr_walk.hpp"
#include "table_registry.hpp"

using namespace msm;

namespace {
thread_local std::string g_err;

int fail(int code, const std::string &msg) {
  g_err = msg;
  return code;
}

// window of the blst drop-in's plain Pippenger: the fastest c measured on
// MI355X per n (tools/window_sweep.py, profiles/archive_r01_r04.txt (r03_window_sweep.json); blst's
// own rule, multi_scalar.c:268-275, picks smaller windows: CPU buckets are
// cache-bound, GPU lanes want enough buckets to fill the chip)
int auto_window(size_t n) {
  int lg = 0;
  while (((size_t)1 << (lg + 1)) <= n) ++lg;
  if (lg <= 8) return 8;
  if (lg <= 10) return 10;
  if (lg <= 12) return 12;
  if (lg == 13) return 13;
  if (lg <= 16) return 14;
  if (lg <= 21) return 16;
  return 17;
}

// Failure inside a void blst-named entry point.  Default: print and abort (a
// wrong answer is never returned silently).  With msm_set_abort_on_error(0) the
// call instead returns with `ret` set to the all-zero point (infinity), the
// message in msm_last_error() and msm_error_pending() raised for the caller.
std::atomic<int> g_abort_on_error{1};
thread_local int g_pending = 0;
void die(const char *where, const std::exception &e, void *ret = nullptr, size_t ret_bytes = 0) {
  if (g_abort_on_error.load()) {
    fprintf(stderr, "msm_mi355x: %s failed: %s\n", where, e.what());
    fflush(stderr);
    abort();
  }
  g_err = std::string(where) + " failed: " + e.what();
  g_pending = 1;
  if (ret) memset(ret, 0, ret_bytes);
}

template <int G>
std::unique_ptr<typename EnginePool<Pippenger<G>>::Lease> pippenger_engine(int window) {
  int dev = 0;
  MSM_HIP_CHECK(hipGetDevice(&dev));
  return EnginePool<Pippenger<G>>::get().lease(dev, window,
                                               [&] { return std::make_unique<Pippenger<G>>(dev, window); });
}

// The device rows of n points at `pts` when a registered host table holds all
// of them (msm_register_host_table; table_registry.hpp), else nullptr.  `hold`
// keeps the table alive for the call.
template <int G>
const void *registered_rows(const uint8_t *pts, size_t n, std::shared_ptr<HostTable> &hold) {
  int dev = 0;
  MSM_HIP_CHECK(hipGetDevice(&dev));
  std::shared_ptr<HostTable> t = TableRegistry::get().find(G, dev, pts);
  if (!t) return nullptr;
  const size_t off = (size_t)(pts - t->base) / (96 * G);
  if (off + n > t->nrows) return nullptr;
  t = fresh<G>(t, off, off + n - 1);  // rows edited since registration: re-uploaded
  if (!t) return nullptr;
  hold = t;
  return t->rows.template as<uint8_t>() + off * t->row_bytes;
}

template <int G>
void mult_pippenger(void *ret, const void *const *points, size_t n, const byte *const *scalars, size_t nbits) {
  typedef typename HostField<G>::F HF;
  hfp::Jac<HF> out;
  if (n == 0) {
    memset(&out, 0, sizeof out);
    memcpy(ret, &out, sizeof out);
    return;
  }
  const size_t nb = (nbits + 7) / 8;
  std::vector<uint8_t> pbuf, sbuf;
  const uint8_t *pts = contiguous(pbuf, points, n, 96 * G);
  const uint8_t *sc = contiguous(sbuf, (const void *const *)scalars, n, nb);
  std::shared_ptr<HostTable> hold;
  const void *rows = registered_rows<G>(pts, n, hold);  // points registered once: no upload
  auto eng = pippenger_engine<G>(auto_window(n));
  (*eng)->run_host(eng->stream(), pts, n, sc, nb, (int)nbits, &out, nullptr, rows);
  memcpy(ret, &out, sizeof out);
}

// one blst window tile (ref multi_scalar.c:383-419, 587-600): sum_i d_i P_i with
// d_i the Booth digit of scalar i at [bit0, bit0+wbits) (lookback bit bit0-1),
// digits and signs computed on the device (k_tile_booth)
template <int G>
void tile_pippenger(void *ret, const void *const *points, size_t n, const byte *const *scalars, size_t nbits,
                    size_t bit0, size_t window) {
  typedef typename HostField<G>::F HF;
  hfp::Jac<HF> out;
  memset(&out, 0, sizeof out);
  // bit0 == nbits is legal: the top tile of nbits = 256 with 8-bit windows holds
  // only the Booth carry of bit 255 (wbits = 0, cbits = 1; ref multi_scalar.c:596-599)
  if (n == 0) {
    memcpy(ret, &out, sizeof out);
    return;
  }
  if (bit0 > nbits || window == 0 || window > 24) throw std::runtime_error("tile outside the scalar bits");
  TileSpec t;
  t.bit0 = (int)bit0;
  if (bit0 + window > nbits) {
    t.wbits = (int)(nbits - bit0);
    t.cbits = t.wbits + 1;
  } else {
    t.wbits = t.cbits = (int)window;
  }
  const size_t nb = (nbits + 7) / 8;
  std::vector<uint8_t> pbuf, sbuf;
  const uint8_t *pts = contiguous(pbuf, points, n, 96 * G);
  const uint8_t *sc = contiguous(sbuf, (const void *const *)scalars, n, nb);
  std::shared_ptr<HostTable> hold;
  const void *rows = registered_rows<G>(pts, n, hold);
  auto eng = pippenger_engine<G>(8);
  (*eng)->run_host(eng->stream(), pts, n, sc, nb, (int)nbits, &out, &t, rows);
  memcpy(ret, &out, sizeof out);
}

// ---- blst-level CHES / BGMW95 tiles (ref multi_scalar.c:421-547, 671-744) ----
constexpr uint32_t kNone = 0xffffffffu;  // entry skipped (bucket sort key)

// The pointer-array tiles below hand the entries to entry_msm_ptrs (compat.hip):
// keys / vals are filled by the host worker pool straight into pinned memory
// and the n pointed-to rows are gathered chunk-wise through a pinned ring, so
// the host work runs in parallel and overlaps the DMA (at 2^20 CHES one call
// moves 12.6 M rows, 1.2 GB).
struct TileFill {
  const int *scalars;
  const unsigned char *signs;
  const int *v2i;    // d_CHES: bucket value -> index (0 = skipped)
  size_t nb;         // noindex / BGMW95: bucket range check
  int mode;          // 0 d_CHES, 1 noindexhash, 2 BGMW95
};
void tile_fill(void *ctx, size_t t0, size_t t1, uint32_t *keys, uint32_t *vals) {
  const TileFill &f = *static_cast<const TileFill *>(ctx);
  for (size_t t = t0; t < t1; ++t) {
    const int v = f.scalars[t];
    uint32_t key;
    if (f.mode == 0) {  // ref multi_scalar.c:421-463: entry t -> bucket v2i[scalars[t]]
      const int idx = f.v2i[v];
      key = idx > 0 ? (uint32_t)idx : kNone;
    } else if (f.mode == 1) {  // ref multi_scalar.c:466-503: buckets indexed by value
      if (v < 0 || (size_t)v >= f.nb) throw std::runtime_error("bucket value outside the bucket set range");
      key = v > 0 ? (uint32_t)v : kNone;
    } else {  // ref multi_scalar.c:506-547: value v in [1, q/2] -> bucket v - 1
      if (v < 0 || (size_t)v > f.nb) throw std::runtime_error("BGMW95 digit outside [0, q/2]");
      key = v > 0 ? (uint32_t)(v - 1) : kNone;
    }
    keys[t - t0] = key;
    vals[t - t0] = (uint32_t)t | ((uint32_t)(f.signs[t] != 0) << 31);
  }
}

// ref multi_scalar.c:421-463: entry t -> bucket v2i[scalars[t]] (0 = skipped),
// weight of bucket k = bucket_set_ascend[k]
template <int G>
void tile_d_ches(void *ret, const void *const *points, size_t n, const int *scalars, const unsigned char *signs,
                 void *buckets, const int *B, const int *v2i, size_t bsize) {
  std::vector<uint32_t> w(bsize);
  for (size_t k = 0; k < bsize; ++k) w[k] = (uint32_t)std::max(B[k], 0);
  TileFill f{scalars, signs, v2i, bsize, 0};
  entry_msm_ptrs<G>(ret, points, n, tile_fill, &f, bsize, w.data(), buckets);
}

// ref multi_scalar.c:466-503: buckets indexed by value; weight v for v in B, else 0
template <int G>
void tile_d_ches_noindex(void *ret, const void *const *points, size_t n, const int *scalars,
                         const unsigned char *signs, void *buckets, const int *B, size_t bsize) {
  if (bsize == 0) throw std::runtime_error("empty bucket set");
  const size_t nb = (size_t)B[bsize - 1] + 1;
  std::vector<uint32_t> w(nb, 0);
  for (size_t k = 1; k < bsize; ++k) w[B[k]] = (uint32_t)B[k];
  TileFill f{scalars, signs, nullptr, nb, 1};
  entry_msm_ptrs<G>(ret, points, n, tile_fill, &f, nb, w.data(), buckets);
}

// ref multi_scalar.c:671-744: standard q-ary digits, hash lookup and carry
// (written back into scalars[t + 1]) here, table slots 3 t + m - 1
template <int G>
void tile_ches_std(void *ret, const void *table, size_t n, int *scalars, const digit_decomposition *H, void *buckets,
                   const int *B, const int *v2i, size_t bsize) {
  std::vector<uint32_t> keys(n), vals(n), w(bsize);
  for (size_t t = 0; t < n; ++t) {
    const digit_decomposition d = H[scalars[t]];
    if (d.alpha) ++scalars[t + 1];
    int idx = v2i[d.b];
    keys[t] = idx > 0 ? (uint32_t)idx : kNone;
    vals[t] = (uint32_t)(3 * t + d.m - 1) | ((uint32_t)(d.alpha != 0) << 31);
  }
  for (size_t k = 0; k < bsize; ++k) w[k] = (uint32_t)std::max(B[k], 0);
  entry_msm<G>(ret, table, 3 * n, keys.data(), vals.data(), n, bsize, w.data(), buckets);
}

// ref multi_scalar.c:506-547: bucket value v in [1, q/2] -> bucket v - 1 of weight v
template <int G>
void tile_bgmw95(void *ret, const void *const *points, size_t n, const int *scalars, const unsigned char *signs,
                 void *buckets, size_t q_exp) {
  if (q_exp < 2 || q_exp > 26) throw std::runtime_error("q_exponent out of range");
  const size_t nb = (size_t)1 << (q_exp - 1);
  std::vector<uint32_t> w(nb);
  for (size_t k = 0; k < nb; ++k) w[k] = (uint32_t)(k + 1);
  TileFill f{scalars, signs, nullptr, nb, 2};
  entry_msm_ptrs<G>(ret, points, n, tile_fill, &f, nb, w.data(), nullptr);
  // the reference's integrate_buckets leaves buckets[0 .. q/2] zeroed
  if (buckets) memset(buckets, 0, (nb + 1) * 192 * G);
}

// sum_i P_i on the GPU: entries spread over up to 4096 buckets of weight 1
// (one lane accumulates each bucket), then the weighted reduction sums them
template <int G>
void points_add(void *ret, const void *const *points, size_t n) {
  std::vector<uint8_t> buf;
  const uint8_t *flat = contiguous(buf, points, n, 96 * G);
  const size_t nb = std::max<size_t>(1, std::min<size_t>(n, 4096));
  std::vector<uint32_t> keys(n), vals(n), w(nb, 1);
  for (size_t i = 0; i < n; ++i) {
    keys[i] = (uint32_t)(i % nb);
    vals[i] = (uint32_t)i;
  }
  entry_msm<G>(ret, flat, n, keys.data(), vals.data(), n, nb, w.data(), nullptr);
}

// ---- fixed-window MSM with a precomputed table (ref multi_scalar.c:63-261) ----
template <int G>
std::unique_ptr<typename EnginePool<Wbits<G>>::Lease> wbits_engine(int wbits) {
  int dev = 0;
  MSM_HIP_CHECK(hipGetDevice(&dev));
  return EnginePool<Wbits<G>>::get().lease(dev, wbits, [&] { return std::make_unique<Wbits<G>>(dev, wbits); });
}

// all points are read (pointer rule of ref multi_scalar.c:136: a NULL entry
// continues after the previous point) before the table is written, so the
// binding's in-place call (points at the end of the table, blst.hpp:383-393) works
template <int G>
void wbits_precompute(void *table, size_t wbits, const void *const *points, size_t n) {
  if (!n) return;
  std::vector<uint8_t> buf;
  const uint8_t *flat = contiguous(buf, points, n, 96 * G);
  auto eng = wbits_engine<G>((int)wbits);
  (*eng)->precompute(flat, n, false, eng->stream());
  (*eng)->get_table(table, 0, (*eng)->table_rows(), eng->stream());
}

// scalar pointer rule of ref multi_scalar.c:165,191: the first pointer is
// taken, then NULL continues after the previous scalar (stride (nbits+7)/8)
template <int G>
void wbits_mult(void *ret, const void *table, size_t wbits, size_t n, const byte *const *scalars, size_t nbits) {
  typedef typename HostField<G>::F HF;
  hfp::Jac<HF> out;
  memset(&out, 0, sizeof out);
  if (n && nbits) {
    const size_t nb = (nbits + 7) / 8;
    std::vector<uint8_t> buf;
    const uint8_t *sc = contiguous(buf, (const void *const *)scalars, n, nb);
    auto eng = wbits_engine<G>((int)wbits);
    hipStream_t s = eng->stream();
    (*eng)->set_table(table, n, false, s);
    (*eng)->upload_scalars(sc, n * nb, s);
    (*eng)->run(s, nullptr, nb, (int)nbits, &out);
  }
  memcpy(ret, &out, sizeof out);
}

size_t blst_window(size_t n) {  // ref multi_scalar.c:268-275
  size_t w = 0;
  while (n >>= 1) ++w;
  return w > 12 ? w - 3 : (w > 4 ? w - 2 : (w ? 2 : 1));
}
}  // namespace

template <class F>
void fixed_points(hfp::Aff<F> *out, size_t n, hfp::Jac<F> g) {
  std::vector<hfp::Jac<F>> j(n);
  for (size_t i = 0; i < n; ++i) {
    g = hfp::dbl(g);
    j[i] = g;
  }
  hfp::to_affine_batch(out, j.data(), n);
}

struct msm_ches_ctx {
  int group = 1;
  int device = 0;      // first shard's device
  bool ready = false;  // a table was built / set / loaded (mult before that: MSM_E_STATE)
  std::unique_ptr<ChesMulti<1>> g1;  // one shard per device (multi.hpp); one shard = one device
  std::unique_ptr<ChesMulti<2>> g2;
};

struct msm_bgmw_ctx {
  int group = 1;
  int device = 0;
  bool ready = false;
  std::unique_ptr<Bgmw<1>> g1;
  std::unique_ptr<Bgmw<2>> g2;
  DevBuf scalars;
};

struct msm_wbits_ctx {
  int group = 1;
  int device = 0;
  bool ready = false;
  std::unique_ptr<Wbits<1>> g1;
  std::unique_ptr<Wbits<2>> g2;
  DevBuf scalars;
};

struct msm_ctx {
  int group = 1;
  int device = 0;
  std::unique_ptr<Pippenger<1>> g1;
  std::unique_ptr<Pippenger<2>> g2;
  DevBuf scalars;
};

namespace {
// ---------------- table file cache ----------------
// file = 64-byte header + rows in blst affine layout (canonical Montgomery,
// byte-identical to the reference's PRECOMPUTATION_POINTS_LIST_3nh / _BGMW95)
struct TableFileHeader {
  char magic[8];  // "MSMTBL01"
  int32_t group, method, q_exp, h;  // method: 1 CHES (3 rows per digit), 2 BGMW95 (1 row)
  uint64_t npoints, rows;
  uint8_t pad[24];
};
static_assert(sizeof(TableFileHeader) == 64, "header");
static const size_t kTableChunk = (size_t)1 << 20;  // rows per I/O chunk

template <class E>
static int save_table_file(E &eng, int group, int method, int q_exp, int h, const char *path) {
  FILE *f = fopen(path, "wb");
  if (!f) return fail(MSM_E_ARG, std::string("cannot open ") + path);
  TableFileHeader hd;
  memset(&hd, 0, sizeof hd);
  memcpy(hd.magic, "MSMTBL01", 8);
  hd.group = group, hd.method = method, hd.q_exp = q_exp, hd.h = h;
  hd.npoints = eng.npoints(), hd.rows = eng.table_rows();
  bool ok = fwrite(&hd, sizeof hd, 1, f) == 1;
  std::vector<uint8_t> buf(std::min<size_t>(kTableChunk, std::max<size_t>(hd.rows, 1)) * 96 * group);
  for (size_t r0 = 0; ok && r0 < hd.rows; r0 += kTableChunk) {
    size_t cnt = std::min(kTableChunk, (size_t)hd.rows - r0);
    eng.get_table(buf.data(), r0, cnt, (hipStream_t)0);
    ok = fwrite(buf.data(), 96 * group, cnt, f) == cnt;
  }
  ok = (fclose(f) == 0) && ok;
  return ok ? MSM_OK : fail(MSM_E_ARG, std::string("write failed: ") + path);
}

template <class E>
static int load_table_file(E &eng, int group, int method, int q_exp, int h, const char *path) {
  FILE *f = fopen(path, "rb");
  if (!f) return fail(MSM_E_ARG, std::string("cannot open ") + path);
  TableFileHeader hd;
  if (fread(&hd, sizeof hd, 1, f) != 1 || memcmp(hd.magic, "MSMTBL01", 8) != 0) {
    fclose(f);
    return fail(MSM_E_ARG, "not a table file");
  }
  if (hd.group != group || hd.method != method || hd.q_exp != q_exp || hd.h != h) {
    fclose(f);
    return fail(MSM_E_ARG, "table file was written for other parameters");
  }
  // validate everything the header claims before the engine is touched: the
  // row count must be the method's (3 h per point for CHES, h for BGMW95) and
  // the file must hold exactly header + rows * affine bytes
  const uint64_t per_point = (uint64_t)(method == 1 ? 3 : 1) * (uint64_t)h;
  const uint64_t row_bytes = 96ull * (uint64_t)group;
  if (hd.npoints >= (1ull << 31) || hd.rows != per_point * hd.npoints) {
    fclose(f);
    return fail(MSM_E_ARG, "table file row count does not match its point count");
  }
  if (fseek(f, 0, SEEK_END) != 0 || (uint64_t)ftell(f) != sizeof hd + hd.rows * row_bytes ||
      fseek(f, (long)sizeof hd, SEEK_SET) != 0) {
    fclose(f);
    return fail(MSM_E_ARG, std::string("table file size does not match its header: ") + path);
  }
  bool ok = true;
  try {
    eng.reserve_table((size_t)hd.npoints);
    std::vector<uint8_t> buf(std::min<size_t>(kTableChunk, std::max<size_t>(hd.rows, 1)) * row_bytes);
    for (size_t r0 = 0; ok && r0 < hd.rows; r0 += kTableChunk) {
      size_t cnt = std::min(kTableChunk, (size_t)hd.rows - r0);
      ok = fread(buf.data(), row_bytes, cnt, f) == cnt;
      if (ok) eng.put_table(buf.data(), r0, cnt, false, (hipStream_t)0);
    }
  } catch (...) {
    fclose(f);
    eng.reserve_table(0);  // no half-loaded table: the context has no points until a good load/build
    throw;
  }
  fclose(f);
  if (!ok) {
    eng.reserve_table(0);
    return fail(MSM_E_ARG, std::string("short read: ") + path);
  }
  return MSM_OK;
}

}  // namespace

extern "C" {

size_t blst_p1s_mult_pippenger_scratch_sizeof(size_t npoints) { return sizeof(blst_p1xyzz) << (blst_window(npoints) - 1); }
size_t blst_p2s_mult_pippenger_scratch_sizeof(size_t npoints) { return sizeof(blst_p2xyzz) << (blst_window(npoints) - 1); }

void blst_p1s_mult_pippenger(blst_p1 *ret, const blst_p1_affine *const points[], size_t npoints,
                             const byte *const scalars[], size_t nbits, limb_t *scratch) {
  (void)scratch;
  try {
    mult_pippenger<1>(ret, (const void *const *)points, npoints, scalars, nbits);
  } catch (const std::exception &e) {
    die("blst_p1s_mult_pippenger", e, ret, sizeof(*ret));
  }
}
void blst_p2s_mult_pippenger(blst_p2 *ret, const blst_p2_affine *const points[], size_t npoints,
                             const byte *const scalars[], size_t nbits, limb_t *scratch) {
  (void)scratch;
  try {
    mult_pippenger<2>(ret, (const void *const *)points, npoints, scalars, nbits);
  } catch (const std::exception &e) {
    die("blst_p2s_mult_pippenger", e, ret, sizeof(*ret));
  }
}
void blst_p1s_tile_pippenger(blst_p1 *ret, const blst_p1_affine *const points[], size_t npoints,
                             const byte *const scalars[], size_t nbits, limb_t *scratch, size_t bit0, size_t window) {
  (void)scratch;
  try {
    tile_pippenger<1>(ret, (const void *const *)points, npoints, scalars, nbits, bit0, window);
  } catch (const std::exception &e) {
    die("blst_p1s_tile_pippenger", e, ret, sizeof(*ret));
  }
}
void blst_p2s_tile_pippenger(blst_p2 *ret, const blst_p2_affine *const points[], size_t npoints,
                             const byte *const scalars[], size_t nbits, limb_t *scratch, size_t bit0, size_t window) {
  (void)scratch;
  try {
    tile_pippenger<2>(ret, (const void *const *)points, npoints, scalars, nbits, bit0, window);
  } catch (const std::exception &e) {
    die("blst_p2s_tile_pippenger", e, ret, sizeof(*ret));
  }
}

// ---- blst-level CHES / BGMW95 entry points ----
size_t blst_p1s_mult_pippenger_scratch_sizeof_CHES(size_t window) { return sizeof(blst_p1xyzz) * (window / 2); }
size_t blst_p2s_mult_pippenger_scratch_sizeof_CHES(size_t window) { return sizeof(blst_p2xyzz) * (window / 2); }

#define MSM_XYZZ_HELPERS(g, F)                                                                                   \
  void blst_p##g##xyzz_dadd_affine(blst_p##g##xyzz *out, const blst_p##g##xyzz *in, const blst_p##g##_affine *p, \
                                   unsigned char booth_sign) {                                                   \
    *reinterpret_cast<hfp::Xyzz<F> *>(out) = hfp::xyzz_madd(*reinterpret_cast<const hfp::Xyzz<F> *>(in),         \
                                                            *reinterpret_cast<const hfp::Aff<F> *>(p),           \
                                                            booth_sign != 0);                                    \
  }                                                                                                              \
  void blst_p##g##xyzz_dadd(blst_p##g##xyzz *p3, const blst_p##g##xyzz *p1, const blst_p##g##xyzz *p2) {         \
    *reinterpret_cast<hfp::Xyzz<F> *>(p3) = hfp::xyzz_add(*reinterpret_cast<const hfp::Xyzz<F> *>(p1),           \
                                                          *reinterpret_cast<const hfp::Xyzz<F> *>(p2));          \
  }                                                                                                              \
  void blst_p##g##xyzz_to_Jacobian(blst_p##g *out, const blst_p##g##xyzz *in) {                                  \
    *reinterpret_cast<hfp::Jac<F> *>(out) = hfp::xyzz_to_jac(*reinterpret_cast<const hfp::Xyzz<F> *>(in));       \
  }                                                                                                              \
  void blst_p##g##_to_xyzz(blst_p##g##xyzz *out, blst_p##g *in) {                                                \
    *reinterpret_cast<hfp::Xyzz<F> *>(out) = hfp::jac_to_xyzz(*reinterpret_cast<const hfp::Jac<F> *>(in));       \
  }                                                                                                              \
  void blst_p##g##_prefetch_CHES(const blst_p##g##xyzz buckets[], size_t booth_idx) {                            \
    (void)buckets;                                                                                               \
    (void)booth_idx;                                                                                             \
  }                                                                                                              \
  void blst_p##g##_bucket_CHES(blst_p##g##xyzz buckets[], int booth_idx, const blst_p##g##_affine *p,            \
                               unsigned char booth_sign) {                                                       \
    blst_p##g##xyzz_dadd_affine(&buckets[booth_idx], &buckets[booth_idx], p, booth_sign);                        \
  }
MSM_XYZZ_HELPERS(1, hfp::Fp)
MSM_XYZZ_HELPERS(2, hfp::Fp2)
#undef MSM_XYZZ_HELPERS

#define MSM_CHES_ENTRIES(g)                                                                                        \
  void blst_p##g##_integrate_buckets_accumulation_d_CHES(blst_p##g *out, blst_p##g##xyzz buckets[],              \
                                                         int bucket_set_ascend[], size_t bucket_set_size,         \
                                                         int d_max) {                                             \
    (void)d_max;                                                                                                  \
    try {                                                                                                         \
      std::vector<uint32_t> w(bucket_set_size);                                                                   \
      for (size_t k = 0; k < bucket_set_size; ++k) w[k] = (uint32_t)std::max(bucket_set_ascend[k], 0);           \
      weighted_bucket_sum<g>(out, buckets, bucket_set_size, w.data());                                            \
    } catch (const std::exception &e) {                                                                           \
      die("blst_p" #g "_integrate_buckets_accumulation_d_CHES", e, out, sizeof(*out));                                               \
    }                                                                                                             \
  }                                                                                                               \
  void blst_p##g##_construct_nh_scalars_nh_points(int nh_scalars[], unsigned char booth_signs[],                  \
                                                  blst_p##g##_affine *nh_points_ptr[], const size_t npoints,     \
                                                  blst_p##g##_affine table[], const digit_decomposition H[]) {   \
    for (size_t i = 0; i < npoints; ++i) {                                                                        \
      const digit_decomposition d = H[nh_scalars[i]];                                                             \
      nh_scalars[i] = d.b;                                                                                        \
      booth_signs[i] = (unsigned char)d.alpha;                                                                    \
      if (d.alpha && i + 1 < npoints) ++nh_scalars[i + 1];                                                        \
      nh_points_ptr[i] = table + 3 * i + d.m - 1;                                                                 \
    }                                                                                                             \
  }                                                                                                               \
  void blst_p##g##_tile_pippenger_d_CHES(blst_p##g *ret, const blst_p##g##_affine *const points[], size_t npoints, \
                                         const int scalars[], const unsigned char booth_signs[],                  \
                                         blst_p##g##xyzz buckets[], int bucket_set_ascend[],                      \
                                         int bucket_value_to_its_index[], size_t bucket_set_size, int d_max) {    \
    (void)d_max;                                                                                                  \
    try {                                                                                                         \
      tile_d_ches<g>(ret, (const void *const *)points, npoints, scalars, booth_signs, buckets, bucket_set_ascend, \
                     bucket_value_to_its_index, bucket_set_size);                                                 \
    } catch (const std::exception &e) {                                                                           \
      die("blst_p" #g "_tile_pippenger_d_CHES", e, ret, sizeof(*ret));                                                               \
    }                                                                                                             \
  }                                                                                                               \
  void blst_p##g##_tile_pippenger_d_CHES_noindexhash(                                                             \
      blst_p##g *ret, const blst_p##g##_affine *const points[], size_t npoints, const int scalars[],               \
      const unsigned char booth_signs[], blst_p##g##xyzz buckets[], int bucket_set_ascend[],                      \
      size_t bucket_set_size, int d_max) {                                                                        \
    (void)d_max;                                                                                                  \
    try {                                                                                                         \
      tile_d_ches_noindex<g>(ret, (const void *const *)points, npoints, scalars, booth_signs, buckets,            \
                             bucket_set_ascend, bucket_set_size);                                                 \
    } catch (const std::exception &e) {                                                                           \
      die("blst_p" #g "_tile_pippenger_d_CHES_noindexhash", e, ret, sizeof(*ret));                                                   \
    }                                                                                                             \
  }                                                                                                               \
  void blst_p##g##_tile_pippenger_CHES_prefetch_2step_ahead_input_std_scalar(                                     \
      blst_p##g *ret, const blst_p##g##_affine table[], size_t npoints, int scalars[],                            \
      digit_decomposition H[], blst_p##g##xyzz buckets[], int bucket_set_ascend[],                                \
      int bucket_value_to_its_index[], size_t bucket_set_size, int d_max) {                                       \
    (void)d_max;                                                                                                  \
    try {                                                                                                         \
      tile_ches_std<g>(ret, table, npoints, scalars, H, buckets, bucket_set_ascend, bucket_value_to_its_index,    \
                       bucket_set_size);                                                                          \
    } catch (const std::exception &e) {                                                                           \
      die("blst_p" #g "_tile_pippenger_CHES_prefetch_2step_ahead_input_std_scalar", e, ret, sizeof(*ret));                           \
    }                                                                                                             \
  }                                                                                                               \
  void blst_p##g##_tile_pippenger_BGMW95(blst_p##g *ret, const blst_p##g##_affine *const points[], size_t npoints, \
                                         const int scalars[], const unsigned char booth_signs[],                  \
                                         blst_p##g##xyzz buckets[], size_t q_exponent) {                          \
    try {                                                                                                         \
      tile_bgmw95<g>(ret, (const void *const *)points, npoints, scalars, booth_signs, buckets, q_exponent);       \
    } catch (const std::exception &e) {                                                                           \
      die("blst_p" #g "_tile_pippenger_BGMW95", e, ret, sizeof(*ret));                                                               \
    }                                                                                                             \
  }
MSM_CHES_ENTRIES(1)
MSM_CHES_ENTRIES(2)
#undef MSM_CHES_ENTRIES

// ---- sum of affine points (replaces ref src/bulk_addition.c:145-164) ----
// point pointer rule of bulk_addition.c:155: a NULL entry continues right after
// the previous point
#define MSM_POINTS_ADD(g)                                                                                         \
  void blst_p##g##s_add(blst_p##g *ret, const blst_p##g##_affine *const points[], size_t npoints) {             \
    try {                                                                                                         \
      points_add<g>(ret, (const void *const *)points, npoints);                                                   \
    } catch (const std::exception &e) {                                                                           \
      die("blst_p" #g "s_add", e, ret, sizeof(*ret));                                                                                \
    }                                                                                                             \
  }
MSM_POINTS_ADD(1)
MSM_POINTS_ADD(2)
#undef MSM_POINTS_ADD

// ---- fixed-window MSM with a precomputed table (replaces ref multi_scalar.c:63-261) ----
#define MSM_WBITS_ENTRIES(g, scratch_pts)                                                                         \
  size_t blst_p##g##s_mult_wbits_precompute_sizeof(size_t wbits, size_t npoints) {                              \
    return (sizeof(blst_p##g##_affine) * npoints) << (wbits - 1);                                                 \
  }                                                                                                               \
  void blst_p##g##s_mult_wbits_precompute(blst_p##g##_affine table[], size_t wbits,                              \
                                          const blst_p##g##_affine *const points[], size_t npoints) {            \
    try {                                                                                                         \
      wbits_precompute<g>(table, wbits, (const void *const *)points, npoints);                                    \
    } catch (const std::exception &e) {                                                                           \
      die("blst_p" #g "s_mult_wbits_precompute", e, table,                                                        \
          blst_p##g##s_mult_wbits_precompute_sizeof(wbits, npoints)); /* no half-written table */                \
    }                                                                                                             \
  }                                                                                                               \
  size_t blst_p##g##s_mult_wbits_scratch_sizeof(size_t npoints) {                                                \
    return sizeof(blst_p##g) * (npoints < scratch_pts ? npoints : scratch_pts);                                   \
  }                                                                                                               \
  void blst_p##g##s_mult_wbits(blst_p##g *ret, const blst_p##g##_affine table[], size_t wbits, size_t npoints,   \
                               const byte *const scalars[], size_t nbits, limb_t *scratch) {                      \
    (void)scratch;                                                                                                \
    try {                                                                                                         \
      wbits_mult<g>(ret, table, wbits, npoints, scalars, nbits);                                                  \
    } catch (const std::exception &e) {                                                                           \
      die("blst_p" #g "s_mult_wbits", e, ret, sizeof(*ret));                                                                         \
    }                                                                                                             \
  }
MSM_WBITS_ENTRIES(1, 8192)  /* SCRATCH_SZ of ref multi_scalar.c:78 */
MSM_WBITS_ENTRIES(2, 4096)
#undef MSM_WBITS_ENTRIES

const char *msm_last_error(void) { return g_err.c_str(); }

int msm_set_abort_on_error(int on) { return g_abort_on_error.exchange(on != 0 ? 1 : 0); }

int msm_error_pending(void) {
  const int p = g_pending;
  g_pending = 0;
  return p;
}

void msm_release_engine_cache(void) {
  PoolStats st;
  PoolRegistry::get().visit(st, true);
}

void msm_engine_cache_stats(size_t out[3]) {
  PoolStats st;
  PoolRegistry::get().visit(st, false);
  out[0] = st.live, out[1] = st.idle, out[2] = st.idle_bytes;
}

size_t msm_set_engine_cache_limit(size_t bytes) {
  const size_t prev = PoolRegistry::get().idle_budget.exchange(bytes);
  PoolStats st;  // a lowered limit trims the engines already idle
  PoolRegistry::get().visit(st, false);
  return prev;
}

int msm_register_host_table(int group, const void *rows, size_t nrows) {
  if ((group != 1 && group != 2) || !rows || !nrows) return fail(MSM_E_ARG, "bad group / rows");
  try {
    if (group == 1) register_host_table<1>(rows, nrows);
    else register_host_table<2>(rows, nrows);
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}

int msm_unregister_host_table(const void *rows) {
  if (!rows) return fail(MSM_E_ARG, "null rows");
  return TableRegistry::get().remove(rows) ? MSM_OK : fail(MSM_E_ARG, "table not registered");
}

int msm_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int msm_valu_probe(int device, double out[4]) {
  if (!out) return fail(MSM_E_ARG, "null out");
  if (msm_device_count() <= device || device < 0) return fail(MSM_E_NODEV, "no such HIP device");
  try {
    valu_probe(device, out);
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}

int msm_ctx_create(msm_ctx **ctx, int group, int device, int window_bits) {
  if (!ctx || (group != 1 && group != 2)) return fail(MSM_E_ARG, "bad ctx/group");
  if (msm_device_count() <= device || device < 0) return fail(MSM_E_NODEV, "no such HIP device");
  try {
    auto c = std::make_unique<msm_ctx>();
    c->group = group;
    c->device = device;
    int wb = window_bits > 0 ? window_bits : 16;
    if (group == 1) c->g1 = std::make_unique<Pippenger<1>>(device, wb);
    else c->g2 = std::make_unique<Pippenger<2>>(device, wb);
    *ctx = c.release();
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}

int msm_ctx_set_points(msm_ctx *ctx, const void *points, size_t n, int on_device, void *stream) {
  if (!ctx || (!points && n)) return fail(MSM_E_ARG, "bad args");
  try {
    if (ctx->group == 1) ctx->g1->set_points(points, n, on_device != 0, (hipStream_t)stream);
    else ctx->g2->set_points(points, n, on_device != 0, (hipStream_t)stream);
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}

int msm_ctx_mult(msm_ctx *ctx, void *ret, const byte *scalars, size_t stride, size_t nbits, int on_device,
                 void *stream) {
  if (!ctx || !ret || nbits == 0 || nbits > 256 || stride < (nbits + 7) / 8) return fail(MSM_E_ARG, "bad args");
  try {
    DeviceGuard g(ctx->device);
    hipStream_t s = (hipStream_t)stream;
    size_t n = ctx->group == 1 ? ctx->g1->npoints() : ctx->g2->npoints();
    const uint8_t *d = scalars;
    if (!on_device && n) {
      ctx->scalars.ensure(n * stride + 16);
      MSM_HIP_CHECK(hipMemcpyAsync(ctx->scalars.p, scalars, n * stride, hipMemcpyHostToDevice, s));
      d = ctx->scalars.as<uint8_t>();
    }
    if (ctx->group == 1) {
      hfp::Jac<hfp::Fp> out;
      ctx->g1->run(s, d, stride, (int)nbits, &out);
      memcpy(ret, &out, sizeof out);
    } else {
      hfp::Jac<hfp::Fp2> out;
      ctx->g2->run(s, d, stride, (int)nbits, &out);
      memcpy(ret, &out, sizeof out);
    }
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}

int msm_ctx_mult_batch(msm_ctx *ctx, void *rets, const byte *scalars, size_t stride, size_t set_stride, size_t nbits,
                       size_t count, int on_device, void *stream) {
  if (!ctx || (!rets && count) || nbits == 0 || nbits > 256 || stride < (nbits + 7) / 8)
    return fail(MSM_E_ARG, "bad args");
  try {
    DeviceGuard g(ctx->device);
    hipStream_t s = (hipStream_t)stream;
    const size_t n = ctx->group == 1 ? ctx->g1->npoints() : ctx->g2->npoints();
    const uint8_t *d = scalars;
    if (!on_device && n && count) {  // the sets, packed, in one upload
      ctx->scalars.ensure(count * n * stride + 16);
      for (size_t k = 0; k < count; ++k)
        MSM_HIP_CHECK(hipMemcpyAsync(ctx->scalars.as<uint8_t>() + k * n * stride, scalars + k * set_stride,
                                     n * stride, hipMemcpyHostToDevice, s));
      d = ctx->scalars.as<uint8_t>();
      set_stride = n * stride;
    }
    if (ctx->group == 1) {
      std::vector<hfp::Jac<hfp::Fp>> out(count);
      ctx->g1->run_batch(s, d, stride, set_stride, count, (int)nbits, out.data());
      memcpy(rets, out.data(), count * sizeof(out[0]));
    } else {
      std::vector<hfp::Jac<hfp::Fp2>> out(count);
      ctx->g2->run_batch(s, d, stride, set_stride, count, (int)nbits, out.data());
      memcpy(rets, out.data(), count * sizeof(out[0]));
    }
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}

int msm_ctx_set_profiling(msm_ctx *ctx, int on) {
  if (!ctx) return fail(MSM_E_ARG, "null ctx");
  if (ctx->group == 1) ctx->g1->set_profiling(on != 0);
  else ctx->g2->set_profiling(on != 0);
  return MSM_OK;
}

int msm_ctx_phase_times(const msm_ctx *ctx, float out[6]) {
  if (!ctx || !out) return fail(MSM_E_ARG, "null");
  const PhaseTimes &t = ctx->group == 1 ? ctx->g1->times() : ctx->g2->times();
  out[0] = t.digits;
  out[1] = t.sort;
  out[2] = t.accumulate;
  out[3] = t.reduce;
  out[4] = t.finalize;
  out[5] = t.total;
  return MSM_OK;
}

void msm_ctx_destroy(msm_ctx *ctx) { delete ctx; }

// ---------------- CHES contexts ----------------
static void params_out(const ChesParams &p, int out[9]) {
  const int v[9] = {p.n_exp, p.beta, p.q_exp, p.h, p.a_h, p.d_max, p.b_size, p.q_exp_bgmw, p.h_bgmw};
  memcpy(out, v, sizeof v);
}

int msm_ches_params(int n_exp, int beta, int out[9]) {
  ChesParams p;
  if (!out || !ches_params_for(n_exp, beta, &p)) return fail(MSM_E_ARG, "no CHES configuration for n_exp/beta");
  params_out(p, out);
  return MSM_OK;
}

int msm_ches_ctx_create_params(msm_ches_ctx **ctx, int group, int device, const int v[9]) {
  if (!ctx || !v || (group != 1 && group != 2)) return fail(MSM_E_ARG, "bad ctx/group/params");
  if (msm_device_count() <= device || device < 0) return fail(MSM_E_NODEV, "no such HIP device");
  ChesParams p{v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8]};
  try {
    auto c = std::make_unique<msm_ches_ctx>();
    c->group = group;
    c->device = device;
    const std::vector<int> devs{device};
    if (group == 1) c->g1 = std::make_unique<ChesMulti<1>>(devs, p);
    else c->g2 = std::make_unique<ChesMulti<2>>(devs, p);
    *ctx = c.release();
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}

int msm_ches_ctx_create(msm_ches_ctx **ctx, int group, int device, int n_exp, int beta) {
  int v[9];
  int rc = msm_ches_params(n_exp, beta, v);
  if (rc) return rc;
  return msm_ches_ctx_create_params(ctx, group, device, v);
}

int msm_ches_ctx_create_multi(msm_ches_ctx **ctx, int group, const int *devices, int ndev, int n_exp, int beta) {
  if (!ctx || !devices || ndev < 1 || (group != 1 && group != 2)) return fail(MSM_E_ARG, "bad ctx/group/devices");
  int v[9];
  int rc = msm_ches_params(n_exp, beta, v);
  if (rc) return rc;
  const int have = msm_device_count();
  std::vector<int> devs(devices, devices + ndev);
  for (int d : devs)
    if (d < 0 || d >= have) return fail(MSM_E_NODEV, "no such HIP device");
  ChesParams p{v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8]};
  try {
    auto c = std::make_unique<msm_ches_ctx>();
    c->group = group;
    c->device = devs[0];
    if (group == 1) c->g1 = std::make_unique<ChesMulti<1>>(devs, p);
    else c->g2 = std::make_unique<ChesMulti<2>>(devs, p);
    *ctx = c.release();
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}

int msm_ches_ctx_shards(const msm_ches_ctx *ctx) {
  if (!ctx) return 0;
  return (int)(ctx->group == 1 ? ctx->g1->nshards() : ctx->g2->nshards());
}

#define CHES_DISPATCH(ctx, CALL) ((ctx)->group == 1 ? (ctx)->g1->CALL : (ctx)->g2->CALL)

int msm_ches_ctx_rccl_exchange(const msm_ches_ctx *ctx) { return ctx ? (int)CHES_DISPATCH(ctx, rccl_exchange()) : 0; }

// several engines take host memory only (each device gets its own slice); shards
// merged into one engine on one device (multi.hpp) take device memory like a
// single-device context
static bool multi_device_arg(const msm_ches_ctx *ctx, int on_device) {
  return on_device && (ctx->group == 1 ? ctx->g1->engines() : ctx->g2->engines()) > 1;
}

int msm_ches_ctx_build_table(msm_ches_ctx *ctx, const void *pts, size_t n, int on_device, void *stream) {
  if (!ctx || (!pts && n)) return fail(MSM_E_ARG, "bad args");
  if (multi_device_arg(ctx, on_device)) return fail(MSM_E_ARG, "a multi-device context takes host points");
  try {
    ctx->ready = false;
    CHES_DISPATCH(ctx, build_table(pts, n, on_device != 0, (hipStream_t)stream));
    ctx->ready = true;
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}

int msm_ches_ctx_set_table(msm_ches_ctx *ctx, const void *tab, size_t n, int on_device, void *stream) {
  if (!ctx || (!tab && n)) return fail(MSM_E_ARG, "bad args");
  if (multi_device_arg(ctx, on_device)) return fail(MSM_E_ARG, "a multi-device context takes a host table");
  try {
    ctx->ready = false;
    CHES_DISPATCH(ctx, set_table(tab, n, on_device != 0, (hipStream_t)stream));
    ctx->ready = true;
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}

int msm_ches_ctx_get_table(msm_ches_ctx *ctx, void *out, size_t first, size_t count) {
  if (!ctx || (!out && count)) return fail(MSM_E_ARG, "bad args");
  try {
    CHES_DISPATCH(ctx, get_table(out, first, count, (hipStream_t)0));
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}

int msm_ches_ctx_mult(msm_ches_ctx *ctx, void *ret, const byte *scalars, size_t stride, int on_device,
                      void *stream) {
  if (!ctx || !ret || stride < 32) return fail(MSM_E_ARG, "bad args (stride must be >= 32)");
  if (!ctx->ready) return fail(MSM_E_STATE, "no table: build_table, set_table or load_table first");
  if (multi_device_arg(ctx, on_device)) return fail(MSM_E_ARG, "a multi-device context takes host scalars");
  try {
    DeviceGuard g(ctx->device);
    hipStream_t s = (hipStream_t)stream;
    if (ctx->group == 1) {
      hfp::Jac<hfp::Fp> out;
      ctx->g1->run(s, scalars, stride, on_device != 0, &out);
      memcpy(ret, &out, sizeof out);
    } else {
      hfp::Jac<hfp::Fp2> out;
      ctx->g2->run(s, scalars, stride, on_device != 0, &out);
      memcpy(ret, &out, sizeof out);
    }
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}

int msm_ches_ctx_mult_batch(msm_ches_ctx *ctx, void *rets, const byte *scalars, size_t stride, size_t set_stride,
                            size_t count, int on_device, void *stream) {
  if (!ctx || (!rets && count) || stride < 32) return fail(MSM_E_ARG, "bad args (stride must be >= 32)");
  if (!ctx->ready) return fail(MSM_E_STATE, "no table: build_table, set_table or load_table first");
  if (multi_device_arg(ctx, on_device)) return fail(MSM_E_ARG, "a multi-device context takes host scalars");
  try {
    DeviceGuard g(ctx->device);
    hipStream_t s = (hipStream_t)stream;
    // host scalars are streamed set by set inside the pipeline (Ches::run_batch)
    const bool on_host = !on_device;
    if (ctx->group == 1) {
      std::vector<hfp::Jac<hfp::Fp>> out(count);
      ctx->g1->run_batch(s, scalars, stride, set_stride, count, out.data(), on_host);
      memcpy(rets, out.data(), count * sizeof(out[0]));
    } else {
      std::vector<hfp::Jac<hfp::Fp2>> out(count);
      ctx->g2->run_batch(s, scalars, stride, set_stride, count, out.data(), on_host);
      memcpy(rets, out.data(), count * sizeof(out[0]));
    }
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}

int msm_ches_ctx_set_profiling(msm_ches_ctx *ctx, int on) {
  if (!ctx) return fail(MSM_E_ARG, "null ctx");
  CHES_DISPATCH(ctx, set_profiling(on != 0));
  return MSM_OK;
}

int msm_ches_ctx_phase_times(const msm_ches_ctx *ctx, float out[6]) {
  if (!ctx || !out) return fail(MSM_E_ARG, "null");
  const PhaseTimes &t = CHES_DISPATCH(ctx, front().times());
  const float v[6] = {t.digits, t.sort, t.accumulate, t.reduce, t.finalize, t.total};
  memcpy(out, v, sizeof v);
  return MSM_OK;
}

size_t msm_ches_ctx_bucket_count(const msm_ches_ctx *ctx) { return ctx ? CHES_DISPATCH(ctx, front().bucket_count()) : 0; }

int msm_ches_ctx_batch_lanes(const msm_ches_ctx *ctx) { return ctx ? CHES_DISPATCH(ctx, front().batch_lanes()) : 0; }

int msm_ches_ctx_time_accumulation(msm_ches_ctx *ctx, const byte *scalars, size_t set_stride, int nsets, int reps,
                                   float *ms) {
  if (!ctx || !scalars || !ms || nsets < 1 || reps < 1) return fail(MSM_E_ARG, "bad args");
  if (!ctx->ready) return fail(MSM_E_STATE, "no table");
  if ((ctx->group == 1 ? ctx->g1->engines() : ctx->g2->engines()) != 1) return fail(MSM_E_ARG, "single-device contexts only");
  try {
    DeviceGuard g(ctx->device);
    *ms = CHES_DISPATCH(ctx, front().time_accumulation((hipStream_t)0, scalars, set_stride, nsets, reps));
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}

void msm_ches_ctx_destroy(msm_ches_ctx *ctx) { delete ctx; }

// ---------------- BGMW95 contexts ----------------
int msm_bgmw_ctx_create(msm_bgmw_ctx **ctx, int group, int device, int q_exp, int h) {
  if (!ctx || (group != 1 && group != 2)) return fail(MSM_E_ARG, "bad ctx/group");
  if (msm_device_count() <= device || device < 0) return fail(MSM_E_NODEV, "no such HIP device");
  try {
    auto c = std::make_unique<msm_bgmw_ctx>();
    c->group = group;
    c->device = device;
    if (group == 1) c->g1 = std::make_unique<Bgmw<1>>(device, q_exp, h);
    else c->g2 = std::make_unique<Bgmw<2>>(device, q_exp, h);
    *ctx = c.release();
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_ARG, e.what());
  }
}

int msm_bgmw_ctx_build_table(msm_bgmw_ctx *ctx, const void *pts, size_t n, int on_device, void *stream) {
  if (!ctx || (!pts && n)) return fail(MSM_E_ARG, "bad args");
  try {
    ctx->ready = false;
    CHES_DISPATCH(ctx, build_table(pts, n, on_device != 0, (hipStream_t)stream));
    ctx->ready = true;
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}

int msm_bgmw_ctx_set_table(msm_bgmw_ctx *ctx, const void *tab, size_t n, int on_device, void *stream) {
  if (!ctx || (!tab && n)) return fail(MSM_E_ARG, "bad args");
  try {
    ctx->ready = false;
    CHES_DISPATCH(ctx, set_table(tab, n, on_device != 0, (hipStream_t)stream));
    ctx->ready = true;
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}

int msm_bgmw_ctx_get_table(msm_bgmw_ctx *ctx, void *out, size_t first, size_t count) {
  if (!ctx || (!out && count)) return fail(MSM_E_ARG, "bad args");
  try {
    CHES_DISPATCH(ctx, get_table(out, first, count, (hipStream_t)0));
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}

int msm_bgmw_ctx_mult(msm_bgmw_ctx *ctx, void *ret, const byte *scalars, size_t stride, int on_device,
                      void *stream) {
  if (!ctx || !ret || stride < 32) return fail(MSM_E_ARG, "bad args (stride must be >= 32)");
  if (!ctx->ready) return fail(MSM_E_STATE, "no table: build_table, set_table or load_table first");
  try {
    DeviceGuard g(ctx->device);
    hipStream_t s = (hipStream_t)stream;
    size_t n = CHES_DISPATCH(ctx, npoints());
    const uint8_t *d = scalars;
    if (!on_device && n) {
      ctx->scalars.ensure(n * stride + 16);
      MSM_HIP_CHECK(hipMemcpyAsync(ctx->scalars.p, scalars, n * stride, hipMemcpyHostToDevice, s));
      d = ctx->scalars.as<uint8_t>();
    }
    if (ctx->group == 1) {
      hfp::Jac<hfp::Fp> out;
      ctx->g1->run(s, d, stride, &out);
      memcpy(ret, &out, sizeof out);
    } else {
      hfp::Jac<hfp::Fp2> out;
      ctx->g2->run(s, d, stride, &out);
      memcpy(ret, &out, sizeof out);
    }
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}

int msm_bgmw_ctx_set_profiling(msm_bgmw_ctx *ctx, int on) {
  if (!ctx) return fail(MSM_E_ARG, "null ctx");
  CHES_DISPATCH(ctx, set_profiling(on != 0));
  return MSM_OK;
}

int msm_bgmw_ctx_phase_times(const msm_bgmw_ctx *ctx, float out[6]) {
  if (!ctx || !out) return fail(MSM_E_ARG, "null");
  const PhaseTimes &t = CHES_DISPATCH(ctx, times());
  const float v[6] = {t.digits, t.sort, t.accumulate, t.reduce, t.finalize, t.total};
  memcpy(out, v, sizeof v);
  return MSM_OK;
}

size_t msm_bgmw_ctx_bucket_count(const msm_bgmw_ctx *ctx) { return ctx ? CHES_DISPATCH(ctx, bucket_count()) : 0; }

void msm_bgmw_ctx_destroy(msm_bgmw_ctx *ctx) { delete ctx; }

int msm_ches_ctx_save_table(msm_ches_ctx *ctx, const char *path) {
  if (!ctx || !path) return fail(MSM_E_ARG, "bad args");
  try {
    DeviceGuard g(ctx->device);
    if (ctx->group == 1) {
      const ChesParams &p = ctx->g1->params();
      return save_table_file(*ctx->g1, 1, 1, p.q_exp, p.h, path);
    }
    const ChesParams &p = ctx->g2->params();
    return save_table_file(*ctx->g2, 2, 1, p.q_exp, p.h, path);
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}
int msm_ches_ctx_load_table(msm_ches_ctx *ctx, const char *path) {
  if (!ctx || !path) return fail(MSM_E_ARG, "bad args");
  try {
    DeviceGuard g(ctx->device);
    ctx->ready = false;
    const ChesParams &p = CHES_DISPATCH(ctx, params());
    const int rc = ctx->group == 1 ? load_table_file(*ctx->g1, 1, 1, p.q_exp, p.h, path)
                                   : load_table_file(*ctx->g2, 2, 1, p.q_exp, p.h, path);
    ctx->ready = rc == MSM_OK;
    return rc;
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}
int msm_bgmw_ctx_save_table(msm_bgmw_ctx *ctx, const char *path) {
  if (!ctx || !path) return fail(MSM_E_ARG, "bad args");
  try {
    DeviceGuard g(ctx->device);
    if (ctx->group == 1) return save_table_file(*ctx->g1, 1, 2, ctx->g1->q_exp(), ctx->g1->h(), path);
    return save_table_file(*ctx->g2, 2, 2, ctx->g2->q_exp(), ctx->g2->h(), path);
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}
int msm_bgmw_ctx_load_table(msm_bgmw_ctx *ctx, const char *path) {
  if (!ctx || !path) return fail(MSM_E_ARG, "bad args");
  try {
    DeviceGuard g(ctx->device);
    ctx->ready = false;
    const int rc = ctx->group == 1 ? load_table_file(*ctx->g1, 1, 2, ctx->g1->q_exp(), ctx->g1->h(), path)
                                   : load_table_file(*ctx->g2, 2, 2, ctx->g2->q_exp(), ctx->g2->h(), path);
    ctx->ready = rc == MSM_OK;
    return rc;
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}

size_t msm_ches_bucket_set(int q, int a_h, int *out, size_t cap) {
  if (q < 4 || a_h < 0) return 0;
  std::vector<int> B = ches_bucket_set(q, a_h);
  if (out) memcpy(out, B.data(), std::min(cap, B.size()) * sizeof(int));
  return B.size();
}

int msm_ches_digit_table(int q, int a_h, digit_decomposition *out) {
  if (q < 4 || a_h < 0 || !out) return fail(MSM_E_ARG, "bad args");
  try {
    // decoded from the compact device tables (code + rank, ches_kernels.hpp)
    // with the device's arithmetic, so the golden digit-table hashes pin them
    std::vector<int> B = ches_bucket_set(q, a_h);
    std::vector<uint32_t> code, rank;
    ches_digit_code(B, q, code, rank);
    for (size_t d = 0; d <= (size_t)q; ++d) {
      const uint32_t c = (code[d >> 3] >> (4 * (d & 7))) & 15u, m = (c & 3u) + 1, alpha = (c >> 2) & 1u;
      int b = 0;
      if (!(c & 8u)) {
        const uint32_t v = (alpha ? (uint32_t)q - (uint32_t)d : (uint32_t)d) / m;
        const uint32_t bits = rank[2 * (v >> 5)], idx = rank[2 * (v >> 5) + 1] +
                                                        (uint32_t)__builtin_popcount(bits & ((1u << (v & 31)) - 1u));
        if (!((bits >> (v & 31)) & 1u)) return fail(MSM_E_ARG, "digit code names a value outside B");
        b = B[idx];
      }
      out[d].m = (int)m;
      out[d].b = b;
      out[d].alpha = (int)alpha;
    }
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_ARG, e.what());
  }
}

// ---------------- boundary helpers ----------------
static uint64_t splitmix64(uint64_t *s) {
  uint64_t z = (*s += 0x9e3779b97f4a7c15ULL);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
void msm_gen_scalars(byte *out, size_t n, uint64_t seed) {
  static const uint64_t R[4] = {0xffffffff00000001ULL, 0x53bda402fffe5bfeULL, 0x3339d80809a1d805ULL,
                                0x73eda753299d7d48ULL};
  uint64_t st = seed;
  for (size_t i = 0; i < n; ++i) {
    uint64_t a[4];
    for (;;) {
      for (int k = 0; k < 4; ++k) a[k] = splitmix64(&st);
      a[3] >>= 1;
      bool lt = false;
      for (int k = 3; k >= 0; --k) {
        if (a[k] != R[k]) {
          lt = a[k] < R[k];
          break;
        }
      }
      if (lt) break;
    }
    for (int k = 0; k < 32; ++k) out[32 * i + k] = (uint8_t)(a[k / 8] >> (8 * (k % 8)));
  }
}

void msm_p1_fixed_points(blst_p1_affine *out, size_t n) { msm_p1_fixed_points_range(out, 0, n); }
void msm_p2_fixed_points(blst_p2_affine *out, size_t n) { msm_p2_fixed_points_range(out, 0, n); }
void msm_p1_fixed_points_range(blst_p1_affine *out, size_t start, size_t n) {
  hfp::Jac<hfp::Fp> g = hfp::g1_generator();
  for (size_t i = 0; i < start; ++i) g = hfp::dbl(g);
  fixed_points<hfp::Fp>(reinterpret_cast<hfp::Aff<hfp::Fp> *>(out), n, g);
}
void msm_p2_fixed_points_range(blst_p2_affine *out, size_t start, size_t n) {
  hfp::Jac<hfp::Fp2> g = hfp::g2_generator();
  for (size_t i = 0; i < start; ++i) g = hfp::dbl(g);
  fixed_points<hfp::Fp2>(reinterpret_cast<hfp::Aff<hfp::Fp2> *>(out), n, g);
}
void msm_p1_to_affine(blst_p1_affine *out, const blst_p1 *in) {
  *reinterpret_cast<hfp::Aff<hfp::Fp> *>(out) = hfp::to_affine(*reinterpret_cast<const hfp::Jac<hfp::Fp> *>(in));
}
void msm_p2_to_affine(blst_p2_affine *out, const blst_p2 *in) {
  *reinterpret_cast<hfp::Aff<hfp::Fp2> *>(out) = hfp::to_affine(*reinterpret_cast<const hfp::Jac<hfp::Fp2> *>(in));
}
void msm_p1_compress(byte out[48], const blst_p1 *in) {
  hfp::compress(out, hfp::to_affine(*reinterpret_cast<const hfp::Jac<hfp::Fp> *>(in)));
}
void msm_p2_compress(byte out[96], const blst_p2 *in) {
  hfp::compress(out, hfp::to_affine(*reinterpret_cast<const hfp::Jac<hfp::Fp2> *>(in)));
}
void msm_p1_add(blst_p1 *out, const blst_p1 *a, const blst_p1 *b) {
  *reinterpret_cast<hfp::Jac<hfp::Fp> *>(out) = hfp::addj(*reinterpret_cast<const hfp::Jac<hfp::Fp> *>(a),
                                                          *reinterpret_cast<const hfp::Jac<hfp::Fp> *>(b));
}
void msm_p2_add(blst_p2 *out, const blst_p2 *a, const blst_p2 *b) {
  *reinterpret_cast<hfp::Jac<hfp::Fp2> *>(out) = hfp::addj(*reinterpret_cast<const hfp::Jac<hfp::Fp2> *>(a),
                                                           *reinterpret_cast<const hfp::Jac<hfp::Fp2> *>(b));
}

int msm_test_field(int group, int op, const limb_t *a, const limb_t *b, limb_t *out, size_t n) {
  try {
    if (group == 1) test_field<1>(op, a, b, out, n);
    else test_field<2>(op, a, b, out, n);
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}
int msm_test_xyzz(int group, const void *pts, size_t npts, const uint32_t *ops, int len, size_t nseq, void *out) {
  try {
    if (group == 1) test_xyzz<1>((const uint64_t *)pts, npts, ops, len, nseq, (uint64_t *)out);
    else test_xyzz<2>((const uint64_t *)pts, npts, ops, len, nseq, (uint64_t *)out);
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}

// ---------------- fixed-window (wbits) contexts ----------------
#define WB_DISPATCH(ctx, CALL) ((ctx)->group == 1 ? (ctx)->g1->CALL : (ctx)->g2->CALL)

int msm_wbits_ctx_create(msm_wbits_ctx **ctx, int group, int device, int wbits) {
  if (!ctx || (group != 1 && group != 2)) return fail(MSM_E_ARG, "bad ctx/group");
  if (msm_device_count() <= device || device < 0) return fail(MSM_E_NODEV, "no such HIP device");
  try {
    auto c = std::make_unique<msm_wbits_ctx>();
    c->group = group;
    c->device = device;
    if (group == 1) c->g1 = std::make_unique<Wbits<1>>(device, wbits);
    else c->g2 = std::make_unique<Wbits<2>>(device, wbits);
    *ctx = c.release();
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_ARG, e.what());
  }
}

int msm_wbits_ctx_precompute(msm_wbits_ctx *ctx, const void *pts, size_t n, int on_device, void *stream) {
  if (!ctx || (!pts && n)) return fail(MSM_E_ARG, "bad args");
  try {
    ctx->ready = false;
    WB_DISPATCH(ctx, precompute(pts, n, on_device != 0, (hipStream_t)stream));
    ctx->ready = true;
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}

int msm_wbits_ctx_set_table(msm_wbits_ctx *ctx, const void *tab, size_t n, int on_device, void *stream) {
  if (!ctx || (!tab && n)) return fail(MSM_E_ARG, "bad args");
  try {
    ctx->ready = false;
    WB_DISPATCH(ctx, set_table(tab, n, on_device != 0, (hipStream_t)stream));
    ctx->ready = true;
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}

int msm_wbits_ctx_get_table(msm_wbits_ctx *ctx, void *out, size_t first, size_t count) {
  if (!ctx || (!out && count)) return fail(MSM_E_ARG, "bad args");
  try {
    WB_DISPATCH(ctx, get_table(out, first, count, (hipStream_t)0));
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_ARG, e.what());
  }
}

int msm_wbits_ctx_mult(msm_wbits_ctx *ctx, void *ret, const byte *scalars, size_t stride, size_t nbits,
                       int on_device, void *stream) {
  if (!ctx || !ret || stride == 0 || (nbits + 7) / 8 > stride) return fail(MSM_E_ARG, "bad args (stride < nbits/8)");
  if (!ctx->ready) return fail(MSM_E_STATE, "no table: precompute or set_table first");
  try {
    DeviceGuard g(ctx->device);
    hipStream_t s = (hipStream_t)stream;
    const size_t n = WB_DISPATCH(ctx, npoints());
    const uint8_t *d = scalars;
    if (!on_device && n) {
      ctx->scalars.ensure(n * stride + 16);
      MSM_HIP_CHECK(hipMemcpyAsync(ctx->scalars.p, scalars, n * stride, hipMemcpyHostToDevice, s));
      d = ctx->scalars.as<uint8_t>();
    }
    if (ctx->group == 1) {
      hfp::Jac<hfp::Fp> out;
      ctx->g1->run(s, d, stride, (int)nbits, &out);
      memcpy(ret, &out, sizeof out);
    } else {
      hfp::Jac<hfp::Fp2> out;
      ctx->g2->run(s, d, stride, (int)nbits, &out);
      memcpy(ret, &out, sizeof out);
    }
    return MSM_OK;
  } catch (const std::exception &e) {
    return fail(MSM_E_HIP, e.what());
  }
}

size_t msm_wbits_ctx_table_rows(const msm_wbits_ctx *ctx) { return ctx ? WB_DISPATCH(ctx, table_rows()) : 0; }

void msm_wbits_ctx_destroy(msm_wbits_ctx *ctx) { delete ctx; }
#undef WB_DISPATCH

}  // extern "C"

