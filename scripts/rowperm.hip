// Row-order probe (dev tool, not part of the product): does the ORDER in which an emit-shaped
// kernel visits the plane rows change the store rate?  Config #4's shape: two planes of 50,000 rows
// of 25,024 B, written by one block per row (256 x 7 x 16 B), rows of the list cut into 8 XCD
// segments, non-temporal 16-byte stores; the row list in address order or randomly permuted, pure
// stores or copies of one of NCLS source rows (the class rows).  Each case is re-run on fresh
// allocations to expose placement effects.
//   hipcc --offload-arch=gfx950 -O3 scripts/rowperm.hip -o scripts/rowperm && ./scripts/rowperm [rounds]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

#define CHK(x)                                                \
  do {                                                        \
    hipError_t e_ = (x);                                      \
    if (e_ != hipSuccess) {                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      exit(1);                                                \
    }                                                         \
  } while (0)

// row list entry: (plane << 31 | row, source row); src == nullptr: pure stores
__global__ __launch_bounds__(256) void k_emit_like(const uint2* list, size_t n, size_t per_xcd, size_t row16, u64x2* pa,
                                                   u64x2* pb, const u64x2* src) {
  const size_t b = blockIdx.x, x = b & 7, r = x * per_xcd + (b >> 3);
  if (r >= n || r >= (x + 1) * per_xcd) return;
  const uint2 e = list[r];
  u64x2* d = ((e.x >> 31) ? pb : pa) + size_t(e.x & 0x7FFFFFFFu) * row16;
  const u64x2* s = src ? src + size_t(e.y) * row16 : nullptr;
  const u64x2 c = {0x5555555555555555ull, 0xAAAAAAAAAAAAAAAAull};
  constexpr int U = 7;
  for (size_t x0 = threadIdx.x; x0 < row16; x0 += 256 * U) {
    u64x2 v[U];
#pragma unroll
    for (int u = 0; u < U; u++)
      if (x0 + u * 256 < row16) v[u] = s ? s[x0 + u * 256] : c;
#pragma unroll
    for (int u = 0; u < U; u++)
      if (x0 + u * 256 < row16) __builtin_nontemporal_store(v[u], d + x0 + u * 256);
  }
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 3;
  const size_t rows = 50000, row = 25024, row16 = row / 16, ncls = 7500;
  const size_t n = 2 * rows, per = (n + 7) / 8;
  std::mt19937 rng(7);
  // class of each (plane, row): random; lists: address order, class-clustered (the emit's), random
  std::vector<uint32_t> cls(n);
  for (auto& c : cls) c = rng() % ncls;
  std::vector<uint2> addr(n), clus(n), rnd(n);
  for (size_t i = 0; i < n; i++) addr[i] = make_uint2(uint32_t((i >= rows) << 31 | (i % rows)), cls[i]);
  std::vector<size_t> idx(n);
  std::iota(idx.begin(), idx.end(), 0);
  std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) {
    return (a >= rows) != (b >= rows) ? a < b : cls[a] < cls[b];  // plane-major, then class
  });
  for (size_t i = 0; i < n; i++) clus[i] = addr[idx[i]];
  rnd = addr;
  std::shuffle(rnd.begin(), rnd.end(), rng);
  uint2 *d_addr, *d_clus, *d_rnd;
  CHK(hipMalloc(&d_addr, n * sizeof(uint2)));
  CHK(hipMalloc(&d_clus, n * sizeof(uint2)));
  CHK(hipMalloc(&d_rnd, n * sizeof(uint2)));
  CHK(hipMemcpy(d_addr, addr.data(), n * sizeof(uint2), hipMemcpyHostToDevice));
  CHK(hipMemcpy(d_clus, clus.data(), n * sizeof(uint2), hipMemcpyHostToDevice));
  CHK(hipMemcpy(d_rnd, rnd.data(), n * sizeof(uint2), hipMemcpyHostToDevice));
  u64x2* src;
  CHK(hipMalloc(&src, ncls * row));
  CHK(hipMemset(src, 0x3C, ncls * row));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const double bytes = double(n) * row;
  std::vector<std::pair<u64x2*, u64x2*>> keep;
  for (int r = 0; r < rounds; r++) {
    u64x2 *pa, *pb;
    CHK(hipMalloc(&pa, rows * row));
    CHK(hipMalloc(&pb, rows * row));
    keep.push_back({pa, pb});
    printf("round %d: planes %p %p\n", r, (void*)pa, (void*)pb);
    const struct { const char* name; const uint2* list; const u64x2* s; } cases[] = {
        {"stores, address order", d_addr, nullptr}, {"stores, class-clustered", d_clus, nullptr},
        {"stores, random order", d_rnd, nullptr},   {"copies, address order", d_addr, src},
        {"copies, class-clustered", d_clus, src},   {"copies, random order", d_rnd, src}};
    for (const auto& c : cases) {
      k_emit_like<<<unsigned(per * 8), 256>>>(c.list, n, per, row16, pa, pb, c.s);
      CHK(hipDeviceSynchronize());
      const int reps = 20;
      CHK(hipEventRecord(e0));
      for (int i = 0; i < reps; i++) k_emit_like<<<unsigned(per * 8), 256>>>(c.list, n, per, row16, pa, pb, c.s);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      ms /= reps;
      printf("  %-26s %8.1f us  %7.1f GB/s\n", c.name, ms * 1e3, bytes / ms / 1e6);
    }
  }
  for (auto& k : keep) {
    CHK(hipFree(k.first));
    CHK(hipFree(k.second));
  }
  return 0;
}
