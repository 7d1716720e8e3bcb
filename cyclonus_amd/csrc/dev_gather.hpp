// dev_gather.hpp — table assembly on the device: a source partition's ingress slices into whole rows.
// Part of engine.hip's single translation unit: included once, by engine.hip, in stage order.
//
// Under CYC_ROWS_SOURCE rank r holds, for EVERY destination d and slot k, the words [a_r, a_r + wr_r)
// of the ingress row (d, k) — its sources' bits (include/cyclonus_hip.h, cyc_rows).  The whole
// ingress plane [P][K][W] on every rank (north_star: "an RCCL all-gather over xGMI only to assemble
// the final table"; Table.Get(from, to) for any pair, pkg/connectivity/probe/table.go:54-56) is the
// ranks' slices side by side: the all-gather moves each rank's slice as it is (contiguous
// [rows][K][wr_r] words), and this kernel scatters the gathered slices into whole rows.
#pragma once

namespace cyc {

constexpr int MERGE_MAX_RANKS = 64;
struct MergeSlice {
  const uint64_t* p;  // [rows][K][wr] words: one rank's slice of the chunk's rows
  uint32_t a, wr;     // the slice's first word in a whole row, and its width in words
};
struct MergeArgs {
  MergeSlice s[MERGE_MAX_RANKS];
  uint64_t* out;  // [rows][K][W]: the chunk's first whole row
  uint32_t n;     // slices
  uint32_t W;
  uint32_t rk;    // (row, slot) pairs of the chunk: rows * K
  uint32_t bps;   // blocks per slice
};

// HBM-bound copy: grid = n * bps blocks of 256 threads, block b copying slice b / bps.  The slice is
// read linearly (word i = (row-slot x, word j), x = i / wr) and written as runs of wr words at
// out[x * W + a + j]; both streams are coalesced.  x is i * (1 / wr) in double precision with one
// correction step (exact for the < 2^40 words of a slice); 4 words a thread in flight, non-temporal
// loads and stores (the gathered slices and the whole plane are touched once).
constexpr uint32_t MERGE_UNROLL = 4;
__global__ __launch_bounds__(256) void k_merge_sources(MergeArgs a) {
  const uint32_t r = blockIdx.x / a.bps, b = blockIdx.x - r * a.bps;
  const MergeSlice s = a.s[r];
  const uint64_t total = uint64_t(a.rk) * s.wr;
  if (!total) return;
  const double inv = 1.0 / double(s.wr);
  const uint64_t step = uint64_t(a.bps) * 256 * MERGE_UNROLL;
  for (uint64_t base = uint64_t(b) * 256 * MERGE_UNROLL + threadIdx.x; base < total; base += step) {
    uint64_t v[MERGE_UNROLL], dst[MERGE_UNROLL];
#pragma unroll
    for (uint32_t u = 0; u < MERGE_UNROLL; u++) {
      const uint64_t i = min(base + u * 256, total - 1);  // clamped: every load issued, none in a branch
      uint64_t x = uint64_t(double(i) * inv);
      if (x * s.wr > i) x--;
      else if ((x + 1) * s.wr <= i) x++;
      dst[u] = x * a.W + s.a + (i - x * s.wr);
      v[u] = __builtin_nontemporal_load(s.p + i);
    }
#pragma unroll
    for (uint32_t u = 0; u < MERGE_UNROLL; u++)
      if (base + u * 256 < total) __builtin_nontemporal_store(v[u], a.out + dst[u]);
  }
}

}  // namespace cyc
