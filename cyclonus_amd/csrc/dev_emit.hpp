// dev_emit.hpp — the emit (the roofline kernel): class rows copied into the ingress / egress planes; batched blocks.
// Part of engine.hip's single translation unit (device bodies inline across stages, host helpers are
// static): included once, by engine.hip, in stage order.
#pragma once

namespace cyc {

// The HBM-bound kernel: every target pod's plane rows are a copy of its class rows.  ONE launch
// writes both planes (and the status plane, in block slices).  The row list is the planes' row
// orders (pods clustered by class) one after the other, or, for planes of >= 8 GB, alternating
// ingress / egress rows so every XCD writes into both planes; it is cut into 8 contiguous
// segments, one per XCD (block b runs on XCD b % 8), so an XCD streams a class-clustered range and
// re-reads a class row from its own L2.  Stores are non-temporal 16-byte writes.
// (Measured and dropped in round 1: persistent grids, chunked XCD deals, rows-per-block groups,
// plain / sc1 stores, address-linear fill-like segments, per-plane launches —
// profiles/r01_emit_*.txt.)
struct EmitArgs {
  uint32_t n_rows[2];         // plane rows of this launch (pods [row_lo, row_lo + n_rows)); 0 = plane not in it
  uint32_t row_lo[2];
  uint32_t per_xcd;           // rows of the n_rows[0] + n_rows[1] row list per XCD segment
  const uint2* order[2];      // (pod, identity) of the pods in [row_lo,row_hi), clustered by the plane's
                              // identity: a row's class is one dependent load away (class_of[identity])
  const uint32_t* class_of[2];
  const uint64_t* A[2];
  const uint32_t* arow[2];    // in-place class rows (RowArgs::arow): the class row is a row of out
  uint64_t* out[2];
  uint64_t row_words;         // words per plane row, the same for every row of a launch (K * W, or
                              // K * window words for a source shard's ingress rows)
  uint32_t chunk;             // k_emit_flat: rows per block
  const uint8_t* st_src;      // job status plane [P][K] (the run's third output), copied by the
  uint8_t* st_dst;            // emit's blocks in slices: no separate copy node ends the step
  uint64_t st_bytes;
  uint32_t interleave;        // the row list alternates ingress / egress rows (n_rows equal)
  // k_emit_units (planes whose rows differ in length, a source shard): per plane its row length in
  // words, rows per unit (a unit = one block's pass) and units; the unit list is [plane 0][plane 1]
  uint64_t pl_words[2];
  uint32_t unit_rows[2], n_units[2];
  uint32_t unit_grp[2];  // k_emit_units: a unit's rows copied a thread group each (8 groups), else 0
  // the IP rows' word-span records (RowArgs::ip_rng), reset to ~0 for the NEXT run in block slices
  // (their readers are all done): no fill launch or memset node before the next front
  uint32_t* reset;
  uint64_t reset_n;
};

// Block blockIdx.x's row r of the n-row list and its XCD x; false when the block has no row.
__device__ __forceinline__ bool emit_slot(const EmitArgs& a, uint32_t n, uint32_t& r, uint32_t& x) {
  const uint32_t b = blockIdx.x;
  x = b & 7;
  r = x * a.per_xcd + (b >> 3);  // XCD x writes its own contiguous segment of the row list
  return r < min(n, (x + 1) * a.per_xcd);
}

// Row r of the row list -> (plane, (pod, identity)).
__device__ __forceinline__ uint2 emit_row_of(const EmitArgs& a, uint32_t r, uint32_t& pl) {
  if (a.interleave) {
    pl = r & 1u;
    return a.order[pl][r >> 1];
  }
  pl = r >= a.n_rows[0] ? 1u : 0u;
  return a.order[pl][r - pl * a.n_rows[0]];
}

// Source of plane pl's row for (pod, identity) pi: its class row; null when the row is itself its
// class's row (in-place class rows: nothing to copy).
__device__ __forceinline__ const uint64_t* emit_src(const EmitArgs& a, uint32_t pl, uint2 pi) {
  const uint32_t p = pi.x, c = a.class_of[pl][pi.y];
  if (!a.arow[pl]) return a.A[pl] + uint64_t(c) * a.pl_words[pl];
  const uint32_t r = a.arow[pl][c];
  return r == p - a.row_lo[pl] ? nullptr : a.out[pl] + uint64_t(r) * a.pl_words[pl];
}

// Block b's slice of the status plane copy and of the word-span reset (every emit kernel calls this first).
__device__ __forceinline__ void emit_status(const EmitArgs& a) {
  if (a.reset_n) {
    const uint64_t per = (a.reset_n + gridDim.x - 1) / gridDim.x, lo = uint64_t(blockIdx.x) * per;
    const uint64_t hi = lo + per < a.reset_n ? lo + per : a.reset_n;
    for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) a.reset[i] = 0xFFFFFFFFu;
  }
  if (!a.st_bytes) return;
  const uint64_t per = (a.st_bytes + gridDim.x - 1) / gridDim.x, lo = uint64_t(blockIdx.x) * per;
  const uint64_t hi = lo + per < a.st_bytes ? lo + per : a.st_bytes;
  for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) a.st_dst[i] = a.st_src[i];
}


// Plane stores are non-temporal: they do not displace the class rows the emit re-reads from L2
// (plain stores: config #4 emit +45 %, profiles/r03_emit_ab.txt).
__device__ __forceinline__ void emit_store(u64x2 v, u64x2* p) { __builtin_nontemporal_store(v, p); }

// i / n for i < 2^22 through a float reciprocal (n block-uniform): the exact quotient after one
// correction either way — a 32-bit integer division by a run-time value is ~40 instructions, once per
// 16-byte chunk in the multi-row emit kernels.
__device__ __forceinline__ uint32_t div_small(uint32_t i, uint32_t n, float inv) {
  uint32_t q = uint32_t(float(i) * inv);
  if (q * n > i) q--;
  else if ((q + 1) * n <= i) q++;
  return q;
}

// Rows of an odd word count or planes not 16-byte aligned: 8-byte copies, one block per row.
__global__ __launch_bounds__(256) void k_emit_words(EmitArgs a) {
  emit_status(a);
  uint32_t r, x;
  if (!emit_slot(a, a.n_rows[0] + a.n_rows[1], r, x)) return;
  uint32_t pl;
  const uint2 pi = emit_row_of(a, r, pl);
  const uint64_t* src = emit_src(a, pl, pi);
  if (!src) return;
  uint64_t* dst = a.out[pl] + uint64_t(pi.x - a.row_lo[pl]) * a.row_words;
  for (uint64_t i = threadIdx.x; i < a.row_words; i += blockDim.x) dst[i] = src[i];
}

// Short rows (< 16 KB, auto): one block per a.chunk consecutive rows of an XCD's segment, the
// threads sweeping the rows' 16-byte chunks as one flat range (row = index / chunks per row), so
// rows shorter than a block's pass still keep every lane storing.  The rows' source and
// destination addresses are staged in LDS first.  (1024-thread blocks over ~128 KB each: config #2
// emit 21.8 -> 25.0 us, profiles/r04_emit_flat_ab.txt.)
constexpr uint32_t EMIT_FLAT_MAX_ROWS = 256;
template <int BS, int UNROLL>
__global__ __launch_bounds__(BS) void k_emit_flat(EmitArgs a) {
  emit_status(a);
  __shared__ const u64x2* s_src[EMIT_FLAT_MAX_ROWS];
  __shared__ u64x2* s_dst[EMIT_FLAT_MAX_ROWS];
  const uint32_t b = blockIdx.x, n = a.n_rows[0] + a.n_rows[1], x = b & 7;
  const uint32_t r0 = x * a.per_xcd + (b >> 3) * a.chunk;
  const uint32_t r_end = min(n, (x + 1) * a.per_xcd);
  if (r0 >= r_end) return;
  __shared__ uint32_t s_cnt[BS / 64];
  uint32_t nr = min(a.chunk, r_end - r0);
  // the block's rows that need a copy (in-place class rows are skipped), compacted in row order
  const u64x2* src = nullptr;
  u64x2* dst = nullptr;
  if (threadIdx.x < nr) {
    uint32_t pl;
    const uint2 pi = emit_row_of(a, r0 + threadIdx.x, pl);
    src = reinterpret_cast<const u64x2*>(emit_src(a, pl, pi));
    dst = reinterpret_cast<u64x2*>(a.out[pl] + uint64_t(pi.x - a.row_lo[pl]) * a.row_words);
  }
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t keep = __ballot(src != nullptr);
  if (lane == 0) s_cnt[wv] = __popcll(keep);
  __syncthreads();
  uint32_t off = __popcll(keep & ((1ull << lane) - 1));
  for (uint32_t x = 0; x < wv; x++) off += s_cnt[x];
  nr = 0;
#pragma unroll
  for (uint32_t x = 0; x < BS / 64; x++) nr += s_cnt[x];
  if (src) {
    s_src[off] = src;
    s_dst[off] = dst;
  }
  __syncthreads();
  const uint32_t n2 = uint32_t(a.row_words / 2), tot = nr * n2;
  const float inv = 1.0f / float(n2);
  for (uint32_t i0 = threadIdx.x; i0 < tot; i0 += BS * UNROLL) {
    u64x2 v[UNROLL];
    uint32_t row[UNROLL], col[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
      const uint32_t i = i0 + u * BS;
      row[u] = div_small(i, n2, inv);
      col[u] = i - row[u] * n2;
      if (i < tot) v[u] = s_src[row[u]][col[u]];
    }
#pragma unroll
    for (int u = 0; u < UNROLL; u++)
      if (i0 + u * BS < tot) emit_store(v[u], &s_dst[row[u]][col[u]]);
  }
}

// Rows of >= 16 KB (auto): one block of BS threads per row, UNROLL chosen on the host so ONE pass
// of BS x UNROLL 16-byte chunks covers the row (config #3: 100 KB rows, 512 x 13 x 16 B; config #4:
// 25 KB rows, 256 x 7 x 16 B): every lane's loads are in flight before its stores and no second,
// partly idle pass follows (profiles/r01_emit_wide_sweep.txt, r01_emit_medium_rows_ab.txt).
template <int BS, int UNROLL>
__global__ __launch_bounds__(BS) void k_emit_wide(EmitArgs a) {
  emit_status(a);
  const uint32_t n = a.n_rows[0] + a.n_rows[1];
  uint32_t r, x;
  if (!emit_slot(a, n, r, x)) return;
  uint32_t pl;
  const uint2 pi = emit_row_of(a, r, pl);
  const u64x2* si = reinterpret_cast<const u64x2*>(emit_src(a, pl, pi));
  if (!si) return;  // in-place class row: already written
  u64x2* di = reinterpret_cast<u64x2*>(a.out[pl] + uint64_t(pi.x - a.row_lo[pl]) * a.row_words);
  const uint32_t n2 = uint32_t(a.row_words / 2);
  // stores aligned to the plane's 128-byte lines, as copy_row_buf: the head chunks first
  const uint32_t h2 = (uint32_t(-reinterpret_cast<uintptr_t>(di)) & 127u) / 16;
  if (threadIdx.x < h2 && threadIdx.x < n2) emit_store(si[threadIdx.x], &di[threadIdx.x]);
  for (uint32_t x0 = h2 + threadIdx.x; x0 < n2; x0 += BS * UNROLL) {
    u64x2 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; u++)
      if (x0 + u * BS < n2) v[u] = si[x0 + u * BS];
#pragma unroll
    for (int u = 0; u < UNROLL; u++)
      if (x0 + u * BS < n2) emit_store(v[u], &di[x0 + u * BS]);
  }
}

// Rows of 16-32 KB through buffer loads / stores: the chunk offsets u x BS x 16 B go to the scalar
// offset, so a lane keeps one offset register and all its data in flight (128 x 13: 53 VGPRs, 8
// waves a SIMD, 13 x 16 B a lane; the flat-address form needs an address pair per chunk: 84 VGPRs);
// offsets past the row (the last pass's idle lanes) fall outside the buffer's range and are dropped.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int BUF_RSRC_W3 = 0x00020000;  // buffer resource word 3 for gfx9 raw buffers
// One row copy through buffer ops, its stores aligned to the 128-byte lines of the plane: a row that
// starts mid-line (config #3's 100,032-byte rows: every other one; config #4's 25,024: the same) first
// stores its head up to the next line boundary (threads of the head's 16-byte chunks), then the rest
// from that boundary, so every wave's 1 KB store covers whole lines and only the row's two ends are
// partial lines.  Stores whose 1 KB straddled lines (rows copied from their own start) wrote ~1 line
// in 9 in two halves, by two waves: pure stores of config #3's shape 3.5 % slower on every placement
// measured (scripts/pitch_probe.hip, profiles/r05_row_alignment.txt).  Offsets past the row fall
// outside the buffer's range and are dropped.
template <int BS, int UNROLL>
__device__ __forceinline__ void copy_row_buf(const uint64_t* si, uint64_t* di, uint32_t bytes, uint32_t tid = threadIdx.x) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint64_t*>(si), 0, bytes, BUF_RSRC_W3);
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(di, 0, bytes, BUF_RSRC_W3);
  const uint32_t head = uint32_t(-reinterpret_cast<uintptr_t>(di)) & 127u;  // bytes to the next line (16-byte multiple)
  if (tid * 16 < head) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, tid * 16, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(v, rd, tid * 16, 0, 2);  // nt
  }
  for (uint32_t x0 = head; x0 < bytes; x0 += BS * UNROLL * 16) {
    u32x4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, tid * 16, x0 + u * BS * 16, 0);
#pragma unroll
    for (int u = 0; u < UNROLL; u++) __builtin_amdgcn_raw_buffer_store_b128(v[u], rd, tid * 16, x0 + u * BS * 16, 2);  // nt
  }
}

template <int BS, int UNROLL>
__global__ __launch_bounds__(BS) void k_emit_wide_buf(EmitArgs a) {
  emit_status(a);
  const uint32_t n = a.n_rows[0] + a.n_rows[1];
  uint32_t r, x;
  if (!emit_slot(a, n, r, x)) return;
  uint32_t pl;
  const uint2 pi = emit_row_of(a, r, pl);
  const uint64_t* si = emit_src(a, pl, pi);
  if (!si) return;  // in-place class row: already written
  uint64_t* di = a.out[pl] + uint64_t(pi.x - a.row_lo[pl]) * a.row_words;
  copy_row_buf<BS, UNROLL>(si, di, uint32_t(a.row_words * 8));
}

// Planes whose rows differ in length (a source shard: ingress rows of every destination over the
// shard's words, egress rows of its sources over all words) in ONE launch: the unit list is plane 0's
// rows in groups of unit_rows[0], then plane 1's in groups of unit_rows[1], each group about one
// block pass (BS x UNROLL x 16 B: config #3 at N = 8 one 100 KB egress row or eight 12.5 KB ingress
// rows), cut into 8 XCD segments.  A block stages its rows' source / destination addresses in LDS
// (in-place class rows skipped), then sweeps their 16-byte chunks as one flat range.  Two launches
// (k_emit_wide + k_emit_flat) ran config #3's N = 8 source shard at 6.0 TB/s against the target
// shard's single launch at 7.0 (r04a).
constexpr uint32_t EMIT_UNIT_MAX_ROWS = 64;
template <int BS, int UNROLL>
__global__ __launch_bounds__(BS) void k_emit_units(EmitArgs a) {
  emit_status(a);
  __shared__ const u64x2* s_src[EMIT_UNIT_MAX_ROWS];
  __shared__ u64x2* s_dst[EMIT_UNIT_MAX_ROWS];
  __shared__ uint32_t s_cnt;
  const uint32_t b = blockIdx.x, n = a.n_units[0] + a.n_units[1], x = b & 7;
  const uint32_t u = x * a.per_xcd + (b >> 3);  // XCD x writes its own contiguous segment of the unit list
  if (u >= min(n, (x + 1) * a.per_xcd)) return;
  const uint32_t pl = u >= a.n_units[0] ? 1u : 0u, r0 = (u - pl * a.n_units[0]) * a.unit_rows[pl];
  const uint32_t nr = min(a.unit_rows[pl], a.n_rows[pl] - r0);
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  if (threadIdx.x < nr) {
    const uint2 pi = a.order[pl][r0 + threadIdx.x];
    const u64x2* src = reinterpret_cast<const u64x2*>(emit_src(a, pl, pi));
    if (src) {  // (row order within the unit does not matter: each row is copied whole)
      const uint32_t k = atomicAdd(&s_cnt, 1u);
      s_src[k] = src;
      s_dst[k] = reinterpret_cast<u64x2*>(a.out[pl] + uint64_t(pi.x - a.row_lo[pl]) * a.pl_words[pl]);
    }
  }
  __syncthreads();
  if (a.unit_rows[pl] == 1) {  // a unit of one long row (a source shard's egress rows): the copy of
                               // k_emit_wide_buf, chunk offsets in the scalar offset, no per-chunk division
    if (!s_cnt) return;
    copy_row_buf<BS, UNROLL>(reinterpret_cast<const uint64_t*>(s_src[0]), reinterpret_cast<uint64_t*>(s_dst[0]),
                             uint32_t(a.pl_words[pl] * 8));
    return;
  }
  if (a.unit_grp[pl]) {  // rows of 7-14 KB (a source shard's ingress rows at N = 8): a row per group of
                         // BS / 8 threads (whole waves), each row one line-aligned buffer-op pass
    constexpr uint32_t G = 8, GS = BS / G;
    const uint32_t j = threadIdx.x / GS;
    if (j < s_cnt)
      copy_row_buf<GS, UNROLL>(reinterpret_cast<const uint64_t*>(s_src[j]), reinterpret_cast<uint64_t*>(s_dst[j]),
                               uint32_t(a.pl_words[pl] * 8), threadIdx.x % GS);
    return;
  }
  const uint32_t n2 = uint32_t(a.pl_words[pl] / 2), tot = s_cnt * n2;
  const float inv = 1.0f / float(n2);
  for (uint32_t i0 = threadIdx.x; i0 < tot; i0 += BS * UNROLL) {
    u64x2 v[UNROLL];
    uint32_t row[UNROLL], col[UNROLL];
#pragma unroll
    for (int q = 0; q < UNROLL; q++) {
      const uint32_t i = i0 + q * BS;
      row[q] = div_small(i, n2, inv);
      col[q] = i - row[q] * n2;
      if (i < tot) v[q] = s_src[row[q]][col[q]];
    }
#pragma unroll
    for (int q = 0; q < UNROLL; q++)
      if (i0 + q * BS < tot) emit_store(v[q], &s_dst[row[q]][col[q]]);
  }
}

// Batched blocks (cyc_probe_prepare_blocks): block b's own table, bits relative to its first pod.
// `split` workgroups per block sweep its output words — ingress[d][k][j], egress[s][k][j] for its pods
// and its probe config's slots — each the class row's words [j, j + 1] of the block's window
// shifted down by the block's first pod's bit, masked to its pods; and its status rows.  The bytes
// written are exactly the answered cells' bits plus their status.
struct BlockArgs {
  uint32_t n_blk, K, AS;               // blocks, slots of the class rows, A row stride (words)
  uint32_t split;                      // workgroups per block (sized on the host from the largest block)
  const uint4* blk;                     // per block: (first pod, pods, first slot, slots)
  const uint64_t* boff;                 // per block: plane slab offset (words), status offset (bytes)
  const uint32_t *pod_id[2], *class_of[2];
  const uint64_t* A[2];
  const uint8_t* st_src;                // [P][K]
  uint64_t* out[2];
  uint8_t* st_out;
};
__global__ __launch_bounds__(256) void k_emit_blocks(BlockArgs a) {
  const uint32_t b = blockIdx.x / a.split, g = blockIdx.x % a.split;  // block b's g-th workgroup
  if (b >= a.n_blk) return;
  const uint32_t t0 = g * blockDim.x + threadIdx.x, stride = a.split * blockDim.x;
  const uint4 bl = a.blk[b];  // (p0, np, k0, nk)
  const uint32_t p0 = bl.x, np = bl.y, k0 = bl.z, nk = bl.w, wb = (np + 63) / 64, sh = p0 % 64;
  const uint32_t wa = (p0 + np + 63) / 64 - p0 / 64;  // the class rows' window words
  const uint64_t n = uint64_t(np) * nk * wb, off = a.boff[2 * b];
  const uint64_t tail = np % 64 ? (1ull << (np % 64)) - 1 : ~0ull;
  for (uint64_t x = t0; x < 2 * n; x += stride) {
    const uint32_t pl = x >= n ? 1u : 0u;
    const uint64_t y = x - pl * n;
    const uint32_t j = uint32_t(y % wb), k = uint32_t((y / wb) % nk), q = uint32_t(y / (uint64_t(wb) * nk));
    const uint32_t c = a.class_of[pl][a.pod_id[pl][p0 + q]];
    const uint64_t* row = a.A[pl] + (uint64_t(c) * a.K + k0 + k) * a.AS;
    uint64_t v = row[j] >> sh;
    if (sh && j + 1 < wa) v |= row[j + 1] << (64 - sh);
    if (j == wb - 1) v &= tail;
    a.out[pl][off + y] = v;
  }
  const uint64_t soff = a.boff[2 * b + 1];
  for (uint32_t x = t0; x < np * nk; x += stride)
    a.st_out[soff + x] = a.st_src[uint64_t(p0 + x / nk) * a.K + k0 + x % nk];
}

// First panicking job of every block in its own job order (key ((s - p0) * np + d - p0) * 65536 +
// job index, resources.go:286-333): thread per (source, destination of its block).
struct BlockErrArgs {
  uint32_t n_blk, P, K, AS;
  const uint4* blk;
  const uint32_t* pod_blk;
  const uint32_t* slot_idx;
  const uint8_t* slot_status;
  const uint32_t *pod_iid, *pod_eid, *class_in, *class_eg;
  const uint8_t *err_in, *err_eg;
  const uint64_t *AE_in, *AE_eg;
  unsigned long long* first;  // [n_blk]
  uint32_t dchunks;           // 256-destination chunks of the largest block
};
__global__ __launch_bounds__(256) void k_first_error_blocks(BlockErrArgs a) {
  const uint64_t n = uint64_t(a.P) * a.dchunks;
  for (uint64_t g = blockIdx.x; g < n; g += gridDim.x) {
    const uint32_t s = uint32_t(g / a.dchunks), b = a.pod_blk[s];
    const uint4 bl = a.blk[b];
    const uint32_t dl = uint32_t(g % a.dchunks) * blockDim.x + threadIdx.x;
    if (dl >= bl.y) continue;
    const uint32_t d = bl.x + dl, w0 = bl.x / 64;
    const bool s_err = a.err_eg[a.pod_eid[s]], d_err = a.err_in[a.pod_iid[d]];
    const uint32_t ci = a.class_in[a.pod_iid[d]], ce = a.class_eg[a.pod_eid[s]];
    unsigned long long best = ~0ull;
    for (uint32_t k = bl.z; k < bl.z + bl.w; k++) {
      if (a.slot_status[uint64_t(d) * a.K + k] != CYC_JOB_VALID) continue;
      bool e = d_err || s_err;
      if (!e) e = (a.AE_in[(uint64_t(ci) * a.K + k) * a.AS + (s / 64 - w0)] >> (s % 64)) & 1;
      if (!e) e = (a.AE_eg[(uint64_t(ce) * a.K + k) * a.AS + (d / 64 - w0)] >> (d % 64)) & 1;
      if (!e) continue;
      const unsigned long long key = (uint64_t(s - bl.x) * bl.y + dl) * 65536ull + a.slot_idx[k];
      best = key < best ? key : best;
    }
    if (best != ~0ull) atomicMin(&a.first[b], best);
  }
}

}  // namespace cyc
