// table_registry.hpp -- host tables registered once (msm_register_host_table)
// for the pointer-array CHES / BGMW95 tiles.
//
// The reference driver passes the same host table to every tile call as one
// pointer per entry (ref main_p1.cpp:233-236 / :279-282 into
// PRECOMPUTATION_POINTS_LIST_3nh, built once at :128-178).  A registered table
// lives on its device in the engine's row layout (AffP: one 128-B line per G1
// row); a tile whose pointers all hit row boundaries of one registered table
// then ships 4-B row indices instead of gathering 96/192-B rows on the host
// (compat.hip entry_msm_ptrs); a flat point array inside one feeds the plain
// drop-in and its tiles without an upload (abi.cpp).  Process-wide, thread-safe; a call holds a
// shared_ptr to the table it uses, so unregistering during a call is safe.
//
// Staleness guard (round 6, row_samples.hpp): every call through a table
// compares the rows sampled at registration with the caller's memory and
// re-uploads the table on a mismatch (fresh()).  Bulk rewrites and reused
// buffers are caught; an edit of a single unsampled row is not -- the header's
// contract (do not modify registered rows) still holds.
#pragma once
#include <stdint.h>

#include <memory>
#include <mutex>
#include <vector>

#include "engine.hpp"
#include "row_samples.hpp"

namespace msm {

struct HostTable : RowSamples {  // group, base, nrows + the staleness samples (row_samples.hpp)
  int device = 0;
  DevBuf rows;  // AffP<F> rows on `device`
  size_t row_bytes = 0;  // sizeof(AffP<F>)
};

class TableRegistry {
 public:
  static TableRegistry &get() {
    static TableRegistry *r = new TableRegistry();  // never destroyed (tables may outlive static teardown)
    return *r;
  }
  // the table of `group` on `device` whose row range contains p (row-aligned)
  std::shared_ptr<HostTable> find(int group, int device, const void *p) {
    const uint8_t *q = static_cast<const uint8_t *>(p);
    const size_t psz = 96 * (size_t)group;
    std::lock_guard<std::mutex> g(mu_);
    for (const auto &t : t_)
      if (t->group == group && t->device == device && q >= t->base && q < t->base + t->nrows * psz &&
          (size_t)(q - t->base) % psz == 0)
        return t;
    return nullptr;
  }
  void add(std::shared_ptr<HostTable> t) {
    std::lock_guard<std::mutex> g(mu_);
    for (auto &u : t_)
      if (u->base == t->base && u->device == t->device) {
        u = std::move(t);
        return;
      }
    t_.push_back(std::move(t));
  }
  bool remove(const void *base) {
    std::lock_guard<std::mutex> g(mu_);
    const size_t before = t_.size();
    std::vector<std::shared_ptr<HostTable>> keep;
    for (auto &u : t_)
      if (u->base != base) keep.push_back(std::move(u));
    t_.swap(keep);
    return t_.size() != before;
  }

 private:
  std::mutex mu_;
  std::vector<std::shared_ptr<HostTable>> t_;
};

// upload + convert rows [rows, rows + nrows) to the current device (compat.hip)
template <int G>
void register_host_table(const void *rows, size_t nrows);

// t, or -- when a sampled row in [lo, hi] no longer matches the host memory --
// the table re-uploaded from the host rows (the registry entry is replaced)
template <int G>
std::shared_ptr<HostTable> fresh(std::shared_ptr<HostTable> t, size_t lo, size_t hi) {
  if (!t || !t->changed(lo, hi)) return t;
  DeviceGuard g(t->device);
  register_host_table<G>(t->base, t->nrows);
  return TableRegistry::get().find(G, t->device, t->base);
}

}  // namespace msm
