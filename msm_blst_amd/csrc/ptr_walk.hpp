// ptr_walk.hpp -- the blst pointer-array rule on the host (no HIP: the CPU
// sanitizer build, tests/host/sanitize_shim.cpp, runs this same code).
#pragma once
#include <stdint.h>
#include <string.h>

#include <vector>

namespace msm {

// The n elements of `sz` bytes named by a blst pointer array, with the
// reference's iteration rule (ref multi_scalar.c:390-416): the first pointer is
// always taken; after it, a non-NULL entry names the next element and a NULL
// entry means "the element right after the previous one" -- so {ptr, NULL} is
// one flat array and a NULL after k explicit pointers continues contiguously.
// Returns the elements as one contiguous host range: the caller's own memory
// when they already are one (the flat case; no host copy at all), otherwise a
// gather into `buf` that copies each run of adjacent elements with one memcpy.
inline const uint8_t *contiguous(std::vector<uint8_t> &buf, const void *const *ptrs, size_t n, size_t sz) {
  if (n == 0) return nullptr;
  const uint8_t *base = (const uint8_t *)ptrs[0];
  size_t i = 1;
  const void *const *pp = ptrs + 1;
  // walk the explicit pointers while they stay adjacent
  while (i < n && *pp && (const uint8_t *)*pp == base + i * sz) ++i, ++pp;
  if (i == n || !*pp) return base;  // all adjacent, or a NULL: the rest continues after the previous element
  buf.resize(n * sz);
  memcpy(buf.data(), base, i * sz);
  const uint8_t *p = base + (i - 1) * sz;
  while (i < n) {
    if (!*pp) {  // the rest is contiguous after p
      memcpy(buf.data() + i * sz, p + sz, (n - i) * sz);
      break;
    }
    const uint8_t *run = (const uint8_t *)*pp++;
    size_t k = 1;
    while (i + k < n && *pp && (const uint8_t *)*pp == run + k * sz) ++k, ++pp;
    if (i + k < n && !*pp) {  // a NULL right after the run extends it to the end
      k = n - i;
    }
    memcpy(buf.data() + i * sz, run, k * sz);
    p = run + (k - 1) * sz;
    i += k;
  }
  return buf.data();
}

}  // namespace msm
