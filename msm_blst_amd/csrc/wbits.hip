// wbits.hip -- blst's fixed-window MSM with a precomputed table of multiples
// (ref src/multi_scalar.c:63-261: blst_p{1,2}s_mult_wbits_precompute,
// blst_p{1,2}s_mult_wbits; declared at ref bindings/blst.h:228-236, :367-375;
// the C++ binding's P1_Affines, bindings/blst.hpp:362-430) on one MI355X.
//
// Table (reference layout, ref multi_scalar.c:82-91): row i holds the nwin =
// 2^(wbits-1) canonical affine multiples (k+1) P_i, k < nwin.  Built on the GPU
// by k_wbits_table (G2: k_wbits_table2p, a lane pair per point): one lane per point, nwin xyzz multiples by repeated mixed
// additions, then one Montgomery batch inversion per lane (the reference does
// the same per stride of rows, ref :94-120).
//
// Multiplication (ref :152-227): signed Booth digits of wbits bits (lookback
// bit below, booth_encode of ref ec_mult.h:46-55) select +-row entries; the
// reference adds, window by window from the top, one gathered point per scalar
// and doubles wbits times between windows.  Here every (window, chunk of C
// points) pair is one lane summing its gathered entries in xyzz
// (k_wbits_sums), the per-window partials are added pairwise (k_wbits_pairs),
// and the host Horner step sum_w 2^(wbits w) T_w combines the window totals --
// the same group element, since only the low nbits bits of each scalar count
// in both.
#include <cstring>

#include "ches_kernels.hpp"
#include "engine.hpp"
#include "pair_kernels.hpp"

#ifndef MSM_GROUP
#error "define MSM_GROUP (1 or 2)"
#endif

namespace msm {

// one lane per point i in [i0, i0 + cnt): T[i nwin + k] = (k+1) P_i
template <int G>
static __global__ void __launch_bounds__(64)
    k_wbits_table(const Aff<typename FieldOf<G>::F> *__restrict__ P, size_t i0, size_t cnt, int nwin,
                  Xyzz<typename FieldOf<G>::F> *__restrict__ scratch, typename FieldOf<G>::F *__restrict__ pref,
                  AffP<typename FieldOf<G>::F> *__restrict__ T) {
  typedef typename FieldOf<G>::F F;
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= cnt) return;
  const size_t i = i0 + t;
  Aff<F> p = ld16(&P[i]);
  AffP<F> *out = T + (size_t)nwin * i;
  if (f_is_zero_exact(p.x) && f_is_zero_exact(p.y)) {  // infinity: every multiple is infinity
    Aff<F> z;
    f_zero(z.x);
    f_zero(z.y);
    for (int k = 0; k < nwin; ++k) st_point(&out[k], z);
    return;
  }
  Xyzz<F> Q;
  xyzz_from_aff(Q, p, false);
  for (int k = 0; k < nwin; ++k) {
    st16(&scratch[(size_t)k * cnt + t], Q);
    if (k + 1 < nwin) xyzz_madd(Q, p, false);  // (k+2) P; the k = 0 step takes the doubling branch
  }
  // Montgomery batch inversion of u_k = ZZ_k ZZZ_k (1/ZZ = ZZZ/u, 1/ZZZ = ZZ/u)
  F c;
  f_one(c);
  for (int k = 0; k < nwin; ++k) {
    Xyzz<F> a = ld16(&scratch[(size_t)k * cnt + t]);
    F u;
    f_mul(u, a.zz, a.zzz);
    f_mul(c, c, u);
    pref[(size_t)k * cnt + t] = c;
  }
  F inv;
  f_inv(inv, c);
  for (int k = nwin - 1; k >= 0; --k) {
    Xyzz<F> a = ld16(&scratch[(size_t)k * cnt + t]);
    F ik;
    if (k > 0) {
      F pk = pref[(size_t)(k - 1) * cnt + t];
      f_mul(ik, inv, pk);
      F u;
      f_mul(u, a.zz, a.zzz);
      f_mul(inv, inv, u);
    } else {
      ik = inv;
    }
    F izz, izzz;
    f_mul(izz, ik, a.zzz);
    f_mul(izzz, ik, a.zz);
    Aff<F> r;
    f_mul(r.x, a.x, izz);
    f_mul(r.y, a.y, izzz);
    f_csub(r.x);
    f_csub(r.y);
    st_point(&out[k], r);
  }
}

// bits [lo, lo + len) of a little-endian scalar of nbits bits (len <= 24);
// positions below 0 or at/after nbits read as 0 (the reference's wmask,
// ref multi_scalar.c:178-183, and the zero lookback of the lowest window)
__device__ __forceinline__ uint32_t wbits_field(const uint8_t *s, int nbits, int lo, int len) {
  uint32_t v = 0;
  const int hi = min(lo + len, nbits);
  for (int b = max(lo, 0) & ~7; b < hi; b += 8) {
    uint32_t byte = s[b >> 3];
    const int sh = b - lo;  // where this byte's bit 0 lands in v
    v |= sh >= 0 ? byte << sh : byte >> -sh;
  }
  const int keep = hi - lo;
  return keep <= 0 ? 0u : v & ((keep >= 32 ? 0xffffffffu : (1u << keep) - 1u));
}

// lane (w, c): sum over points i in chunk c of d_{i,w} P_i, d the signed Booth
// digit of window w (bits [w wbits - 1, w wbits + wbits)); parts[w nch + c]
template <int G>
static __global__ void __launch_bounds__(256)
    k_wbits_sums(const AffP<typename FieldOf<G>::F> *__restrict__ T, int wbits, const uint8_t *__restrict__ sc,
                 size_t stride, int nbits, size_t n, int nw, size_t nch, size_t C,
                 Xyzz<typename FieldOf<G>::F> *__restrict__ parts) {
  typedef typename FieldOf<G>::F F;
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (size_t)nw * nch) return;
  const int w = (int)(t / nch);
  const size_t c = t % nch, nwin = (size_t)1 << (wbits - 1);
  Xyzz<F> acc;
  xyzz_set_inf(acc);
  const size_t e = min(n, (c + 1) * C);
  for (size_t i = c * C; i < e; ++i) {
    const uint32_t wval = wbits_field(sc + i * stride, nbits, w * wbits - 1, wbits + 1);
    const int d = (int)((wval + 1) >> 1) - (int)((wval >> wbits) << wbits);  // booth_encode, ec_mult.h:46-55
    if (d == 0) continue;
    const uint32_t m = (uint32_t)(d < 0 ? -d : d);
    Aff<F> p = ld_point(&T[i * nwin + m - 1]);
    if (f_is_zero_exact(p.x) && f_is_zero_exact(p.y)) continue;  // infinity row
    xyzz_madd(acc, p, d < 0);
  }
  st16(&parts[t], acc);
}

// G2 on lane pairs (fp2l.hpp; as k_ches_table2p / k_accumulate2p): lanes 2t,
// 2t + 1 handle point t, one Fp2 component each.  The one-lane G2 kernels
// needed 256 VGPRs + 256 AGPRs and spilled (k_wbits_table<2>: 140 B of
// scratch; k_wbits_sums<2>: 9 VGPRs to AGPRs); a lane holds half the state here
// (tests/test_kernel_resources.py keeps every product kernel spill-free).
static __global__ void __launch_bounds__(128)
    k_wbits_table2p(const Aff<Fp2> *__restrict__ P, size_t i0, size_t cnt, int nwin, Xyzz<Fp2> *__restrict__ scratch,
                    Fp2 *__restrict__ pref, AffP<Fp2> *__restrict__ T) {
  const size_t tt = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tt >= 2 * cnt) return;  // whole pairs only
  const int comp = (int)(tt & 1);
  const size_t t = tt >> 1, i = i0 + t;
  Aff<Fp2L> p;
  ld_point2l(p, &P[i], comp);
  AffP<Fp2> *out = T + (size_t)nwin * i;
  if (f_is_zero_exact(p.x) && f_is_zero_exact(p.y)) {  // infinity: every multiple is infinity (uniform per pair)
    Fp z;
    fp_zero(z);
    for (int k = 0; k < nwin; ++k) {
      Aff<Fp2> *o = reinterpret_cast<Aff<Fp2> *>(out + k);
      st_comp(&o->x, z, comp);
      st_comp(&o->y, z, comp);
    }
    return;
  }
  Xyzz<Fp2L> Q;
  xyzz_from_aff(Q, p, false);
  for (int k = 0; k < nwin; ++k) {
    st_xyzz2l(&scratch[(size_t)k * cnt + t], Q, comp);
    if (k + 1 < nwin) xyzz_madd(Q, p, false);  // (k+2) P; the k = 0 step takes the doubling branch
  }
  Fp2L c;  // Montgomery batch inversion of u_k = ZZ_k ZZZ_k, as k_wbits_table
  f_one(c);
  for (int k = 0; k < nwin; ++k) {
    Xyzz<Fp2L> a;
    ld_xyzz2l(a, &scratch[(size_t)k * cnt + t], comp);
    Fp2L u;
    f_mul(u, a.zz, a.zzz);
    f_mul(c, c, u);
    st_comp(&pref[(size_t)k * cnt + t], c.c, comp);
  }
  Fp2L inv;
  f_inv(inv, c);
  for (int k = nwin - 1; k >= 0; --k) {
    Xyzz<Fp2L> a;
    ld_xyzz2l(a, &scratch[(size_t)k * cnt + t], comp);
    Fp2L ik;
    if (k > 0) {
      Fp2L pk;
      ld_comp(pk.c, &pref[(size_t)(k - 1) * cnt + t], comp);
      f_mul(ik, inv, pk);
      Fp2L u;
      f_mul(u, a.zz, a.zzz);
      f_mul(inv, inv, u);
    } else {
      ik = inv;
    }
    Fp2L izz, izzz, x, y;
    f_mul(izz, ik, a.zzz);
    f_mul(izzz, ik, a.zz);
    f_mul(x, a.x, izz);
    f_mul(y, a.y, izzz);
    f_csub(x);
    f_csub(y);
    Aff<Fp2> *o = reinterpret_cast<Aff<Fp2> *>(out + k);
    st_comp(&o->x, x.c, comp);
    st_comp(&o->y, y.c, comp);
  }
}

// k_wbits_sums for G2: lane pair (w, c), both lanes read the same digits
static __global__ void __launch_bounds__(256)
    k_wbits_sums2p(const AffP<Fp2> *__restrict__ T, int wbits, const uint8_t *__restrict__ sc, size_t stride, int nbits,
                   size_t n, int nw, size_t nch, size_t C, Xyzz<Fp2> *__restrict__ parts) {
  const size_t tt = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tt >= 2 * (size_t)nw * nch) return;
  const int comp = (int)(tt & 1);
  const size_t t = tt >> 1;
  const int w = (int)(t / nch);
  const size_t c = t % nch, nwin = (size_t)1 << (wbits - 1);
  Xyzz<Fp2L> acc;
  xyzz_set_inf(acc);
  const size_t e = min(n, (c + 1) * C);
  for (size_t i = c * C; i < e; ++i) {
    const uint32_t wval = wbits_field(sc + i * stride, nbits, w * wbits - 1, wbits + 1);
    const int d = (int)((wval + 1) >> 1) - (int)((wval >> wbits) << wbits);  // booth_encode, ec_mult.h:46-55
    if (d == 0) continue;
    const uint32_t m = (uint32_t)(d < 0 ? -d : d);
    Aff<Fp2L> p;
    ld_point2l(p, &T[i * nwin + m - 1], comp);
    if (f_is_zero_exact(p.x) && f_is_zero_exact(p.y)) continue;  // infinity row (uniform per pair)
    xyzz_madd(acc, p, d < 0);
  }
  st_xyzz2l(&parts[t], acc, comp);
}

// per window: dst[w nout + j] = src[w nin + 2j] + src[w nin + 2j + 1]
template <int G>
static __global__ void __launch_bounds__(64)
    k_wbits_pairs(const Xyzz<typename FieldOf<G>::F> *__restrict__ src, Xyzz<typename FieldOf<G>::F> *__restrict__ dst,
                  int nw, size_t nin, size_t nout) {
  typedef typename FieldOf<G>::F F;
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (size_t)nw * nout) return;
  const size_t w = t / nout, j = t % nout;
  Xyzz<F> a = ld16(&src[w * nin + 2 * j]);
  if (2 * j + 1 < nin) {
    Xyzz<F> b = ld16(&src[w * nin + 2 * j + 1]);
    xyzz_add(a, b);
  }
  st16(&dst[t], a);
}

template <int G>
Wbits<G>::Wbits(int device, int wbits) : dev_(device), wbits_(wbits) {
  if (wbits < 2 || wbits > 14) throw std::runtime_error("wbits must be in [2, 14] (ref multi_scalar.c:67)");
}

template <int G>
void Wbits<G>::precompute(const void *pts, size_t n, bool on_device, hipStream_t s) {
  typedef typename FieldOf<G>::F F;
  DeviceGuard g(dev_);
  const size_t nwin = (size_t)1 << (wbits_ - 1);
  if (n == 0) {
    n_ = 0;
    return;
  }
  if (n * nwin >= (1ull << 32)) throw std::runtime_error("wbits table too large");
  const void *src = pts;
  DevBuf stage, base;
  if (!on_device) {
    stage.ensure(n * 96 * G);
    MSM_HIP_CHECK(hipMemcpyAsync(stage.p, pts, n * 96 * G, hipMemcpyHostToDevice, s));
    src = stage.p;
  }
  base.ensure(n * sizeof(Aff<F>));
  hipLaunchKernelGGL(k_convert_points<G>, dim3(nblk(n, 256)), dim3(256), 0, s, (const uint64_t *)src,
                     base.as<Aff<F>>(), n);
  MSM_HIP_CHECK(hipGetLastError());
  table_.ensure(n * nwin * sizeof(AffP<F>));
  // scratch: nwin xyzz points + prefix products per lane, bounded to ~512 MiB
  const size_t per_lane = nwin * (sizeof(Xyzz<F>) + sizeof(F));
  const size_t chunk = std::min<size_t>(n, std::max<size_t>(64, ((size_t)512 << 20) / per_lane));
  DevBuf scratch, pref;
  scratch.ensure(nwin * chunk * sizeof(Xyzz<F>));
  pref.ensure(nwin * chunk * sizeof(F));
  for (size_t i0 = 0; i0 < n; i0 += chunk) {
    const size_t cnt = std::min(chunk, n - i0);
    if constexpr (G == 2)
      hipLaunchKernelGGL(k_wbits_table2p, dim3(nblk(2 * cnt, 128)), dim3(128), 0, s, base.as<Aff<F>>(), i0, cnt,
                         (int)nwin, scratch.as<Xyzz<F>>(), pref.as<F>(), table_.as<AffP<F>>());
    else
      hipLaunchKernelGGL(k_wbits_table<G>, dim3(nblk(cnt, 64)), dim3(64), 0, s, base.as<Aff<F>>(), i0, cnt,
                         (int)nwin, scratch.as<Xyzz<F>>(), pref.as<F>(), table_.as<AffP<F>>());
    MSM_HIP_CHECK(hipGetLastError());
  }
  MSM_HIP_CHECK(hipStreamSynchronize(s));
  n_ = n;
}

template <int G>
void Wbits<G>::set_table(const void *tab, size_t n, bool on_device, hipStream_t s) {
  typedef typename FieldOf<G>::F F;
  DeviceGuard g(dev_);
  const size_t rows = n << (wbits_ - 1);
  n_ = 0;
  if (!n) return;
  table_.ensure(rows * sizeof(AffP<F>));
  const size_t chunk = (size_t)1 << 20;
  DevBuf stage;
  if (!on_device) stage.ensure(std::min(chunk, rows) * 96 * G);
  for (size_t r0 = 0; r0 < rows; r0 += chunk) {
    const size_t cnt = std::min(chunk, rows - r0);
    const uint8_t *src = static_cast<const uint8_t *>(tab) + r0 * 96 * G;
    if (!on_device) {
      MSM_HIP_CHECK(hipMemcpyAsync(stage.p, src, cnt * 96 * G, hipMemcpyHostToDevice, s));
      src = stage.as<uint8_t>();
    }
    hipLaunchKernelGGL((k_convert_points<G, AffP<F>>), dim3(nblk(cnt, 256)), dim3(256), 0, s,
                       (const uint64_t *)src, table_.as<AffP<F>>() + r0, cnt);
    MSM_HIP_CHECK(hipGetLastError());
    if (!on_device) MSM_HIP_CHECK(hipStreamSynchronize(s));  // the staging buffer is reused
  }
  MSM_HIP_CHECK(hipStreamSynchronize(s));
  n_ = n;
}

template <int G>
void Wbits<G>::get_table(void *out, size_t first, size_t count, hipStream_t s) {
  typedef typename FieldOf<G>::F F;
  DeviceGuard g(dev_);
  if (first + count > table_rows()) throw std::runtime_error("table range out of bounds");
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
void Wbits<G>::run(hipStream_t s, const uint8_t *d_scalars, size_t stride, int nbits, hfp::Jac<HF> *out) {
  typedef typename FieldOf<G>::F F;
  DeviceGuard g(dev_);
  std::memset(out, 0, sizeof(*out));
  if (n_ == 0 || nbits <= 0) return;
  if ((size_t)(nbits + 7) / 8 > stride) throw std::runtime_error("scalar stride shorter than nbits");
  if (!d_scalars) d_scalars = scal_.as<uint8_t>();  // upload_scalars()
  const int nw = nbits / wbits_ + 1;  // windows 0..K, K = floor(nbits / wbits) (ref multi_scalar.c:174-227)
  // chunk of points per lane: ~2^17 lanes in flight
  const size_t C = std::max<size_t>(1, (n_ * (size_t)nw + ((size_t)1 << 17) - 1) >> 17);
  size_t nch = (n_ + C - 1) / C;
  parts_[0].ensure((size_t)nw * nch * sizeof(Xyzz<F>));
  parts_[1].ensure((size_t)nw * ((nch + 1) / 2 + 1) * sizeof(Xyzz<F>));
  fin_.ensure((size_t)nw * 144 * G);
  if constexpr (G == 2)
    hipLaunchKernelGGL(k_wbits_sums2p, dim3(nblk(2 * (size_t)nw * nch, 256)), dim3(256), 0, s, table_.as<AffP<F>>(),
                       wbits_, d_scalars, stride, nbits, n_, nw, nch, C, parts_[0].as<Xyzz<F>>());
  else
    hipLaunchKernelGGL(k_wbits_sums<G>, dim3(nblk((size_t)nw * nch, 256)), dim3(256), 0, s, table_.as<AffP<F>>(),
                       wbits_, d_scalars, stride, nbits, n_, nw, nch, C, parts_[0].as<Xyzz<F>>());
  MSM_HIP_CHECK(hipGetLastError());
  int cur = 0;
  while (nch > 1) {
    const size_t nout = (nch + 1) / 2;
    hipLaunchKernelGGL(k_wbits_pairs<G>, dim3(nblk((size_t)nw * nout, 64)), dim3(64), 0, s,
                       parts_[cur].as<Xyzz<F>>(), parts_[cur ^ 1].as<Xyzz<F>>(), nw, nch, nout);
    MSM_HIP_CHECK(hipGetLastError());
    cur ^= 1;
    nch = nout;
  }
  hipLaunchKernelGGL(k_finalize<G>, dim3(nblk(nw, 64)), dim3(64), 0, s, parts_[cur].as<Xyzz<F>>(),
                     fin_.as<uint64_t>(), nw);
  MSM_HIP_CHECK(hipGetLastError());
  std::vector<hfp::Jac<HF>> T(nw);
  MSM_HIP_CHECK(hipMemcpyAsync(T.data(), fin_.p, (size_t)nw * sizeof(hfp::Jac<HF>), hipMemcpyDeviceToHost, s));
  MSM_HIP_CHECK(hipStreamSynchronize(s));
  *out = horner(T, wbits_);  // sum_w 2^(wbits w) T_w
}

template <int G>
void Wbits<G>::upload_scalars(const void *host, size_t bytes, hipStream_t s) {
  DeviceGuard g(dev_);
  scal_.ensure(bytes + 16);
  MSM_HIP_CHECK(hipMemcpyAsync(scal_.p, host, bytes, hipMemcpyHostToDevice, s));
}

template class Wbits<MSM_GROUP>;

}  // namespace msm
