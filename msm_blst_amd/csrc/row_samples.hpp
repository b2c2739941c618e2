// row_samples.hpp -- the staleness guard of a registered host table
// (table_registry.hpp), free of HIP so the CPU sanitizer build
// (tests/host/sanitize_shim.cpp) runs this same code.
//
// At registration up to kSamples rows at even strides (always the first and
// the last) are copied aside; a call through the table compares the samples
// inside the rows it uses with the caller's memory.  A mismatch means the rows
// changed since their upload (the reference reads them on every call, ref
// multi_scalar.c:421-463, main_p1.cpp:233-236), and the caller re-uploads.
#pragma once
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

namespace msm {

struct RowSamples {
  int group = 1;
  const uint8_t *base = nullptr;  // caller's rows (blst affine, 96 G bytes each)
  size_t nrows = 0;
  std::vector<size_t> sidx;    // sampled rows, ascending (first and last included)
  std::vector<uint8_t> sbytes;  // their bytes at registration
  static constexpr size_t kSamples = 1024;

  size_t psz() const { return 96 * (size_t)group; }
  void take_samples() {
    sidx.clear();
    sbytes.clear();
    if (!nrows) return;
    const size_t k = std::min(nrows, kSamples);
    for (size_t i = 0; i < k; ++i) sidx.push_back(k == 1 ? 0 : i * (nrows - 1) / (k - 1));
    sbytes.resize(k * psz());
    for (size_t i = 0; i < k; ++i) memcpy(&sbytes[i * psz()], base + sidx[i] * psz(), psz());
  }
  // a sampled row in [lo, hi] differs from the caller's memory now
  bool changed(size_t lo, size_t hi) const {
    const size_t a = (size_t)(std::lower_bound(sidx.begin(), sidx.end(), lo) - sidx.begin());
    for (size_t i = a; i < sidx.size() && sidx[i] <= hi; ++i)
      if (memcmp(&sbytes[i * psz()], base + sidx[i] * psz(), psz()) != 0) return true;
    return false;
  }
};

}  // namespace msm
