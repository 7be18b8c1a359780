// lt_host.h -- host-side helpers shared by the lookup, packer and batch code:
// uninitialised arrays (first touched by the worker threads that fill them)
// and contiguous-range thread splits sized to the job's CPU share.
#pragma once
#include <algorithm>
#include <cstdint>
#include <memory>
#include <new>
#include <thread>
#include <vector>

#include "lt_error.h"

namespace lt {

// An uninitialised array (new T[] of a trivial T does not zero it, so the
// pages are first touched by whichever thread fills them).
template <class T>
struct Arr {
  std::unique_ptr<T[]> p;
  int64_t n = 0, cap = 0;
  // k elements; an array recycled with room enough keeps its (already
  // mapped) memory
  bool alloc(int64_t k) {
    if (p && cap >= k) {
      n = k;
      return true;
    }
    cap = std::max<int64_t>(k, 1);
    p.reset(new (std::nothrow) T[(size_t)cap]);
    n = k;
    if (!p) cap = 0;
    return p != nullptr;
  }
  size_t bytes() const { return (size_t)cap * sizeof(T); }
  T* data() const { return p.get(); }
  T& operator[](int64_t i) const { return p[(size_t)i]; }
};

// Split [0, n) into contiguous ranges on up to min(32, host_threads())
// threads, one range per `per` items at least; fn(thread, lo, hi).
template <class F>
void parallel_ranges(int64_t n, F fn, int64_t per = 1 << 16) {
  int nt = (int)std::min<int64_t>((n + per - 1) / per, 32);
  nt = std::max(1, std::min(nt, host_threads()));
  if (nt == 1) {
    fn(0, (int64_t)0, n);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) th.emplace_back(fn, t, n * t / nt, n * (t + 1) / nt);
  fn(0, (int64_t)0, n / nt);
  for (std::thread& x : th) x.join();
}

}  // namespace lt
