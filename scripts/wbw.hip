// Write-bandwidth probe (dev tool, not part of the product): how fast can MI355X store a 20 GB
// buffer, by store form and launch shape?  The emit's ceiling question.
//   hipcc --offload-arch=gfx950 -O3 scripts/wbw.hip -o scripts/wbw && ./scripts/wbw [GB]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

#define CHK(x)                                                        \
  do {                                                                \
    hipError_t e_ = (x);                                              \
    if (e_ != hipSuccess) {                                           \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

// grid-stride over 16-byte chunks, UNROLL chunks per thread per step, NT: non-temporal stores
template <int UNROLL, bool NT>
__global__ void k_fill(u64x2* p, size_t n) {
  const size_t stride = size_t(gridDim.x) * blockDim.x * UNROLL;
  const u64x2 v = {0x5555555555555555ull, 0xAAAAAAAAAAAAAAAAull};
  for (size_t i = size_t(blockIdx.x) * blockDim.x * UNROLL + threadIdx.x; i < n; i += stride) {
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
      const size_t x = i + size_t(u) * blockDim.x;
      if (x < n) {
        if (NT) __builtin_nontemporal_store(v, p + x);
        else p[x] = v;
      }
    }
  }
}

// one block per contiguous "row" of ROW bytes (the emit's shape), rows dealt to XCDs in segments
template <int BS, int UNROLL, bool NT>
__global__ __launch_bounds__(BS) void k_rows(u64x2* p, size_t rows, size_t row16, size_t per_xcd) {
  const size_t b = blockIdx.x, x = b & 7, r = x * per_xcd + (b >> 3);
  if (r >= rows || r >= (x + 1) * per_xcd) return;
  u64x2* d = p + r * row16;
  const u64x2 v = {0x5555555555555555ull, 0xAAAAAAAAAAAAAAAAull};
  for (size_t x0 = threadIdx.x; x0 < row16; x0 += BS * UNROLL) {
#pragma unroll
    for (int u = 0; u < UNROLL; u++)
      if (x0 + u * BS < row16) {
        if (NT) __builtin_nontemporal_store(v, d + x0 + u * BS);
        else d[x0 + u * BS] = v;
      }
  }
}


// the emit's two-plane row list: row r of the list -> plane r & 1 (interleaved) or r >= rows (plane-major),
// plane row r >> 1 / r - rows; the list cut into 8 XCD segments
template <int BS, int UNROLL>
__global__ __launch_bounds__(BS) void k_rows2(u64x2* pa, u64x2* pb, size_t rows, size_t row16, size_t per_xcd, int inter) {
  const size_t b = blockIdx.x, x = b & 7, r = x * per_xcd + (b >> 3);
  if (r >= 2 * rows || r >= (x + 1) * per_xcd) return;
  const size_t pl = inter ? (r & 1) : (r >= rows), pr = inter ? (r >> 1) : (r >= rows ? r - rows : r);
  u64x2* d = (pl ? pb : pa) + pr * row16;
  const u64x2 v = {0x5555555555555555ull, 0xAAAAAAAAAAAAAAAAull};
  for (size_t x0 = threadIdx.x; x0 < row16; x0 += BS * UNROLL) {
#pragma unroll
    for (int u = 0; u < UNROLL; u++)
      if (x0 + u * BS < row16) __builtin_nontemporal_store(v, d + x0 + u * BS);
  }
}

template <class F>
static double time_ms(F f, int reps) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  f();
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(a));
  for (int i = 0; i < reps; i++) f();
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms;
  CHK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const double gb = argc > 1 ? atof(argv[1]) : 20.0;
  const size_t bytes = size_t(gb * 1e9) & ~size_t(4095), n = bytes / 16;
  u64x2* p;
  CHK(hipMalloc(&p, bytes));
  int cus = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int reps = 10;
  auto report = [&](const char* name, double ms) { printf("%-44s %8.3f ms  %7.1f GB/s\n", name, ms, bytes / ms / 1e6); };
  for (int mult : {4, 8, 16, 32}) {
    const unsigned g = cus * mult;
    char nm[96];
    snprintf(nm, sizeof nm, "fill nt   256x8  grid %d x CUs", mult);
    report(nm, time_ms([&] { k_fill<8, true><<<g, 256>>>(p, n); }, reps));
    snprintf(nm, sizeof nm, "fill plain 256x8 grid %d x CUs", mult);
    report(nm, time_ms([&] { k_fill<8, false><<<g, 256>>>(p, n); }, reps));
  }
  report("fill nt   256x1  one chunk per thread", time_ms([&] { k_fill<1, true><<<unsigned((n + 255) / 256), 256>>>(p, n); }, reps));
  for (size_t row : {size_t(25024), size_t(100032)}) {  // config #4 / #3 plane rows
    const size_t row16 = row / 16, rows = bytes / row, per = (rows + 7) / 8;
    char nm[96];
    snprintf(nm, sizeof nm, "rows %zu B: 512x13 nt", row);
    report(nm, time_ms([&] { k_rows<512, 13, true><<<unsigned(per * 8), 512>>>(p, rows, row16, per); }, reps));
    snprintf(nm, sizeof nm, "rows %zu B: 256x7 nt", row);
    report(nm, time_ms([&] { k_rows<256, 7, true><<<unsigned(per * 8), 256>>>(p, rows, row16, per); }, reps));
    snprintf(nm, sizeof nm, "rows %zu B: 512x13 plain", row);
    report(nm, time_ms([&] { k_rows<512, 13, false><<<unsigned(per * 8), 512>>>(p, rows, row16, per); }, reps));
  }
  report("hipMemsetAsync", time_ms([&] { CHK(hipMemsetAsync(p, 0x5A, bytes)); }, reps));
  {  // two planes of 100,032 B rows, as the emit writes them (config #3: 2 x 100,000 rows)
    const size_t row = 100032, row16 = row / 16, rows = bytes / 2 / row, per = (2 * rows + 7) / 8;
    u64x2* pa = p;
    u64x2* pb = p + rows * row16;  // one allocation, planes back to back
    report("2 planes, one buffer, interleaved rows", time_ms([&] { k_rows2<512, 13><<<unsigned(per * 8), 512>>>(pa, pb, rows, row16, per, 1); }, reps));
    report("2 planes, one buffer, plane-major", time_ms([&] { k_rows2<512, 13><<<unsigned(per * 8), 512>>>(pa, pb, rows, row16, per, 0); }, reps));
    CHK(hipFree(p));
    u64x2 *qa, *qb;
    CHK(hipMalloc(&qa, rows * row));
    CHK(hipMalloc(&qb, rows * row));
    report("2 planes, two buffers, interleaved rows", time_ms([&] { k_rows2<512, 13><<<unsigned(per * 8), 512>>>(qa, qb, rows, row16, per, 1); }, reps));
    report("2 planes, two buffers, plane-major", time_ms([&] { k_rows2<512, 13><<<unsigned(per * 8), 512>>>(qa, qb, rows, row16, per, 0); }, reps));
    CHK(hipFree(qa));
    CHK(hipFree(qb));
  }
  return 0;
}
