// oracle/goslice.hpp — Go slice semantics (shared backing array, len, cap, append growth) for
// pointer-sized elements, so the oracle reproduces the reference's slice-aliasing behaviour
// exactly (test infrastructure only).
//
// Why: pkg/matcher/portmatcher.go:126 `ranges := append(s.PortRanges, other.PortRanges...)`
// writes into s.PortRanges' backing array when cap > len, and the PortMatcher `s` is shared by
// every peer of one rule (pkg/matcher/builder.go:84,102,108).  Its observable effect depends on
// the exact capacities Go 1.16 picks: runtime/slice.go growslice (double while old.len < 1024,
// 1.25x after; jump straight to the needed length when it exceeds double) rounded up by
// runtime/msize.go roundupsize to the Go 1.16 malloc size classes (runtime/sizeclasses.go).
#pragma once
#include <cstddef>
#include <memory>
#include <stdexcept>
#include <vector>

namespace goslice {

// Go 1.16 size classes (bytes), runtime/sizeclasses.go class_to_size.
static const size_t kClassToSize[] = {
    0,     8,     16,    24,    32,    48,    64,    80,    96,    112,   128,   144,   160,   176,
    192,   208,   224,   240,   256,   288,   320,   352,   384,   416,   448,   480,   512,   576,
    640,   704,   768,   896,   1024,  1152,  1280,  1408,  1536,  1792,  2048,  2304,  2688,  3072,
    3200,  3456,  4096,  4864,  5376,  6144,  6528,  6784,  6912,  8192,  9472,  9728,  10240, 10880,
    12288, 13568, 14336, 16384, 18432, 19072, 20480, 21760, 24576, 27264, 28672, 32768};

inline size_t roundupsize(size_t size) {
  if (size <= 32768) {
    for (size_t c : kClassToSize)
      if (c >= size) return c;
  }
  // large allocations round to pages (8 KiB)
  return (size + 8191) / 8192 * 8192;
}

// runtime/slice.go growslice, element size 8 (sys.PtrSize)
inline size_t grow_cap(size_t old_len, size_t old_cap, size_t needed) {
  size_t newcap = old_cap;
  size_t doublecap = newcap + newcap;
  if (needed > doublecap) {
    newcap = needed;
  } else if (old_len < 1024) {
    newcap = doublecap;
  } else {
    while (newcap > 0 && newcap < needed) newcap += newcap / 4;
    if (newcap == 0) newcap = needed;
  }
  return roundupsize(newcap * 8) / 8;
}

template <class T>
struct Slice {
  std::shared_ptr<std::vector<T>> arr;  // backing array, size == cap
  size_t len = 0;
  size_t cap = 0;

  bool is_nil() const { return !arr; }
  size_t size() const { return len; }
  const T& operator[](size_t i) const {
    if (i >= len) throw std::out_of_range("slice index");
    return (*arr)[i];
  }
  T& at(size_t i) {
    if (i >= len) throw std::out_of_range("slice index");
    return (*arr)[i];
  }
  std::vector<T> to_vector() const {
    std::vector<T> v;
    for (size_t i = 0; i < len; i++) v.push_back((*arr)[i]);
    return v;
  }
};

// append(s, xs...)
template <class T>
Slice<T> append(const Slice<T>& s, const std::vector<T>& xs) {
  if (xs.empty()) return s;
  size_t need = s.len + xs.size();
  Slice<T> r;
  if (need <= s.cap) {
    r = s;  // shares the backing array: writes are visible to every slice over it
  } else {
    size_t nc = grow_cap(s.len, s.cap, need);
    r.arr = std::make_shared<std::vector<T>>(nc);
    for (size_t i = 0; i < s.len; i++) (*r.arr)[i] = (*s.arr)[i];
    r.cap = nc;
  }
  for (size_t i = 0; i < xs.size(); i++) (*r.arr)[s.len + i] = xs[i];
  r.len = need;
  return r;
}

template <class T>
Slice<T> append(const Slice<T>& s, const Slice<T>& xs) {
  return append(s, xs.to_vector());
}

template <class T>
Slice<T> append1(const Slice<T>& s, const T& x) {
  return append(s, std::vector<T>{x});
}

}  // namespace goslice
