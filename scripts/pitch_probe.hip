// Row-pitch probe (dev tool, not part of the product): is the emit's plane-placement sensitivity
// (profiles/r05_plane_placement.txt) a matter of where the ROWS start?  Config #3's shape: two planes
// of 100,000 rows of 100,032 B (8 slots x 1563 words: rows only 64-byte aligned), written by one
// 1024-thread block per row (1024 x 7 x 16 B, non-temporal 16-byte stores, the rows of the list cut
// into 8 XCD segments, ingress / egress rows alternating) — pure stores, no reads.  Each pair of
// planes is allocated once at the largest pitch; every pitch then places the same rows in the same
// physical memory with different row starts: natural (100,032 B), 128-byte multiple (100,096),
// 4 KB multiple (102,400), 2 MB / 20 (a row start offset drifting by 64 KB steps).
//   hipcc --offload-arch=gfx950 -O3 scripts/pitch_probe.hip -o scripts/pitch_probe && ./scripts/pitch_probe [pairs] [reps]
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

// list entry: plane << 31 | row; block b writes list[x * per + (b >> 3)] for XCD x = b % 8
__global__ __launch_bounds__(1024) void k_rows(const uint32_t* list, size_t n, size_t per, size_t row16, size_t pitch16,
                                               u64x2* pa, u64x2* pb) {
  const size_t b = blockIdx.x, x = b & 7, r = x * per + (b >> 3);
  if (r >= n || r >= (x + 1) * per) return;
  const uint32_t e = list[r];
  u64x2* d = ((e >> 31) ? pb : pa) + size_t(e & 0x7FFFFFFFu) * pitch16;
  const u64x2 c = {0x5555555555555555ull, 0xAAAAAAAAAAAAAAAAull};
  constexpr int U = 7;
  for (size_t x0 = threadIdx.x; x0 < row16; x0 += 1024 * U) {
#pragma unroll
    for (int u = 0; u < U; u++)
      if (x0 + u * 1024 < row16) __builtin_nontemporal_store(c, d + x0 + u * 1024);
  }
}

int main(int argc, char** argv) {
  const int pairs = argc > 1 ? atoi(argv[1]) : 4, reps = argc > 2 ? atoi(argv[2]) : 5;
  const size_t rows = 100000, row = 100032, row16 = row / 16;
  const size_t pitches[] = {100032, 100096, 102400, 104857 / 16 * 16};
  const size_t maxp = 104857 / 16 * 16 > 102400 ? 104857 / 16 * 16 : 102400;
  const size_t n = 2 * rows, per = (n + 7) / 8;
  // row lists: address order (alternating planes), and 50-row groups (a deployment's pods: one class)
  // in a random order, as the emit's class-clustered list
  std::vector<uint32_t> addr(n), clus(n);
  for (size_t i = 0; i < n; i++) addr[i] = uint32_t((i & 1) << 31 | (i >> 1));
  std::vector<uint32_t> grp(rows / 50);
  std::iota(grp.begin(), grp.end(), 0);
  std::mt19937 rng(11);
  std::shuffle(grp.begin(), grp.end(), rng);
  size_t k = 0;
  for (uint32_t g : grp)
    for (uint32_t j = 0; j < 50; j++) {
      const uint32_t r = g * 50 + j;
      clus[k++] = r;
      clus[k++] = (1u << 31) | r;
    }
  uint32_t *d_addr, *d_clus;
  CHK(hipMalloc(&d_addr, n * 4));
  CHK(hipMalloc(&d_clus, n * 4));
  CHK(hipMemcpy(d_addr, addr.data(), n * 4, hipMemcpyHostToDevice));
  CHK(hipMemcpy(d_clus, clus.data(), n * 4, hipMemcpyHostToDevice));
  std::vector<u64x2*> pa(pairs), pb(pairs);
  for (int p = 0; p < pairs; p++) {
    CHK(hipMalloc(&pa[p], rows * maxp));
    CHK(hipMalloc(&pb[p], rows * maxp));
    printf("pair %d: %p %p (mod 2 MiB %#zx / %#zx)\n", p, (void*)pa[p], (void*)pb[p], size_t(pa[p]) % (2u << 20),
           size_t(pb[p]) % (2u << 20));
  }
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const double bytes = 2.0 * rows * row;
  auto best = [&](auto&& f) {
    float b = 1e30f;
    for (int r = 0; r < reps; r++) {
      CHK(hipEventRecord(e0));
      f();
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      b = std::min(b, ms);
    }
    return b;
  };
  for (int p = 0; p < pairs; p++) {
    const float fm = best([&] {
      CHK(hipMemsetD32Async(hipDeviceptr_t(pa[p]), 0, rows * row / 4, nullptr));
      CHK(hipMemsetD32Async(hipDeviceptr_t(pb[p]), 0, rows * row / 4, nullptr));
    });
    printf("pair %d fill (natural span)       %8.1f us  %6.0f GB/s\n", p, fm * 1e3, bytes / fm / 1e6);
    for (size_t pitch : pitches)
      for (int o = 0; o < 2; o++) {
        const uint32_t* l = o ? d_clus : d_addr;
        const float ms = best([&] { k_rows<<<unsigned(8 * per), 1024>>>(l, n, per, row16, pitch / 16, pa[p], pb[p]); });
        CHK(hipGetLastError());
        printf("pair %d pitch %6zu %-9s      %8.1f us  %6.0f GB/s\n", p, pitch, o ? "clustered" : "address", ms * 1e3,
               bytes / ms / 1e6);
      }
    fflush(stdout);
  }
  return 0;
}
