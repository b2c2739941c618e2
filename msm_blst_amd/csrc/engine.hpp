// engine.hpp -- host-side orchestration of the MSM kernels on one MI355X.
// Internal C++ API; the C ABI (abi.cpp) and the Python mirror sit on top.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "host_fp.hpp"

#define MSM_HIP_CHECK(x)                                                                           \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess)                                                                         \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e_) + " at " + #x); \
  } while (0)

namespace msm {

struct DevBuf {
  void *p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf &) = delete;
  DevBuf &operator=(const DevBuf &) = delete;
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
  size_t npoints() const { return n_; }
  void set_profiling(bool on) { profile_ = on; }
  const PhaseTimes &times() const { return times_; }
  int device() const { return dev_; }
  int window_bits() const { return c_; }

 private:
  int dev_, c_;
  size_t n_ = 0;
  bool profile_ = false;
  PhaseTimes times_;
  DevBuf pts_, keys_, ranks_, counts_, offsets_, sorted_, order_, iota_, sortkeys_, buckets_, redA_[2], redY_[2],
      fin_, tmp_;
  std::vector<hipEvent_t> ev_;
};

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
