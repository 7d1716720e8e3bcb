// comm.hpp — multi-GPU table assembly: the context's RCCL communicator and the all-gather of row
// shards into whole verdict planes on every rank.  Part of engine.hip's single translation unit
// (included last: it uses the device-resident table and the row layouts defined there).
//
// north_star: "Source-pod rows shard across the 8 GPUs of one node, with an RCCL all-gather over
// xGMI only to assemble the final table."  Every verdict depends only on replicated inputs, so the
// shards are computed with no exchange (cyc_probe_run_rows); this is the one collective, and it is
// optional: a source shard already answers Table.Get(from, *) for its sources alone
// (pkg/connectivity/probe/table.go:54-56).  A Go multi-GPU Runner.RunProbeForConfig
// (pkg/connectivity/probe/jobrunner.go:29-31) that must hand back one whole *Table per rank calls
// cyc_comm_init once and cyc_table_allgather per probe.
//
// How the planes move.  RCCL's all-gather wants equal, contiguous shares; the shards here differ by
// a row or a 64-pod word, and a source shard's ingress share is a column slice of every row.  So:
//   * row shares (both planes of a target partition, a source partition's egress rows): one group
//     of N broadcasts, rank r's rows straight from its shard into their place in the whole plane
//     (an all-gather-v with no padding and no relayout; in place when the shard already sits there);
//   * a source partition's ingress slices: the destination rows in chunks of ~256 MB, per chunk a
//     group of N broadcasts of each rank's contiguous [rows][K][wr_r] slice into a scratch buffer,
//     then k_merge_sources scatters the slices into whole rows on a second stream while the next
//     chunk's broadcasts run (two scratch buffers, events between the streams).
// xGMI is point-to-point (7 links per GPU): a rank receives (N - 1) / N of each plane, and the
// broadcasts of one group share the links like a ring all-gather of the same bytes.
#pragma once

namespace {

#define NCCLCHK(x)                                                                             \
  do {                                                                                         \
    ncclResult_t r_ = (x);                                                                     \
    if (r_ != ncclSuccess) throw RcclErr{std::string(#x) + ": " + ncclGetErrorString(r_)}; \
  } while (0)

constexpr uint64_t COMM_CHUNK_BYTES = 256ull << 20;  // whole-row bytes per assembly chunk (per scratch buffer)

// The library's own partition of the pods over nranks (cyclonus_amd/shard.py restates it): target
// rows balanced to a row, source rows balanced to a 64-pod word (row_lo a multiple of 64, as
// rows_layout requires).
void shard_rows(int64_t P, int part, int n, int r, int64_t& lo, int64_t& hi) {
  if (part == CYC_ROWS_SOURCE) {
    const int64_t W = (P + 63) / 64;
    lo = std::min<int64_t>(P, (int64_t(r) * W / n) * 64);
    hi = std::min<int64_t>(P, (int64_t(r + 1) * W / n) * 64);
  } else {
    lo = int64_t(r) * P / n;
    hi = int64_t(r + 1) * P / n;
  }
}

// k_merge_sources over destination rows [d0, d1): slice r reads ptr[r] (the slice's row d0).
void merge_launch(cyc_ctx* c, hipStream_t st, int n, const uint64_t* const* ptr, const uint32_t* a, const uint32_t* wr,
                  uint64_t* out_row_d0, int64_t d0, int64_t d1) {
  const uint64_t K = c->pb.K, W = c->pb.W;
  // (row, slot) pairs per launch held in 32 bits: chunks of at most 2^30 of them
  const int64_t step = std::max<int64_t>(1, int64_t((1u << 30) / std::max<uint64_t>(K, 1)));
  for (int64_t x0 = d0; x0 < d1; x0 += step) {
    const int64_t x1 = std::min(d1, x0 + step);
    MergeArgs m{};
    m.n = uint32_t(n);
    m.W = uint32_t(W);
    m.rk = uint32_t(uint64_t(x1 - x0) * K);
    m.out = out_row_d0 + uint64_t(x0 - d0) * K * W;
    uint64_t most = 0;
    for (int r = 0; r < n; r++) {
      m.s[r].p = ptr[r] + uint64_t(x0 - d0) * K * wr[r];
      m.s[r].a = a[r];
      m.s[r].wr = wr[r];
      most = std::max<uint64_t>(most, uint64_t(m.rk) * wr[r]);
    }
    if (!most) continue;
    // >= ~4096 blocks over the launch when the slices are that large, one 1024-word pass a block at least
    const uint64_t per = (most + 256 * MERGE_UNROLL - 1) / (256 * MERGE_UNROLL);
    m.bps = uint32_t(std::max<uint64_t>(1, std::min<uint64_t>(per, std::max(1, 4096 / n))));
    k_merge_sources<<<m.bps * uint32_t(n), 256, 0, st>>>(m);
    HIPCHK(hipGetLastError());
  }
}

bool comm_ready(cyc_ctx* c, std::string& why) {
  if (!c->comm.nccl) return why = "cyc_comm_init first", false;
  if (!c->prepared) return why = "cyc_probe_prepare first", false;
  if (!c->pb.blocks.empty()) return why = "context prepared for blocks: nothing to assemble", false;
  return true;
}

void ensure_comm_streams(cyc_ctx* c) {
  auto& m = c->comm;
  if (!m.merge) HIPCHK(hipStreamCreateWithFlags(&m.merge, hipStreamNonBlocking));
  for (int b = 0; b < 2; b++) {
    if (!m.full[b]) HIPCHK(hipEventCreateWithFlags(&m.full[b], EV_SYNC));
    if (!m.free_[b]) HIPCHK(hipEventCreateWithFlags(&m.free_[b], EV_SYNC));
  }
  if (!m.done) {
    HIPCHK(hipEventCreateWithFlags(&m.done, EV_SYNC));
    HIPCHK(hipEventRecord(m.done, m.merge));  // a completed event: the first call's wait below is a no-op
  }
}

// The all-gather proper (comm_ready checked).  in / eg: this rank's shard under `part` (the rows of
// shard_rows(rank)); full_in / full_eg: [P][K][W] planes.
int planes_allgather(cyc_ctx* c, hipStream_t st, int part, const uint64_t* in, const uint64_t* eg, uint64_t* full_in,
                     uint64_t* full_eg) {
  auto& m = c->comm;
  const int n = m.nranks, me = m.rank;
  const uint64_t P = c->pb.P, K = c->pb.K, W = c->pb.W, row_words = K * W;
  ensure_comm_streams(c);
  // the previous call's relayout may still run on the merge stream (a caller may switch streams)
  HIPCHK(hipStreamWaitEvent(st, m.done, 0));
  std::vector<int64_t> lo(static_cast<size_t>(n)), hi(static_cast<size_t>(n));
  for (int r = 0; r < n; r++) shard_rows(int64_t(P), part, n, r, lo[size_t(r)], hi[size_t(r)]);
  const bool src = part == CYC_ROWS_SOURCE;

  // 1. row shares: the egress plane (both partitions) and a target partition's ingress plane
  NCCLCHK(ncclGroupStart());
  for (int pl = src ? 1 : 0; pl < 2; pl++) {
    const uint64_t* mine = pl ? eg : in;
    uint64_t* full = pl ? full_eg : full_in;
    for (int r = 0; r < n; r++) {
      const uint64_t cnt = uint64_t(hi[size_t(r)] - lo[size_t(r)]) * row_words;
      if (!cnt) continue;
      uint64_t* dst = full + uint64_t(lo[size_t(r)]) * row_words;
      NCCLCHK(ncclBroadcast(r == me ? static_cast<const void*>(mine) : dst, dst, cnt, ncclUint64, r, m.nccl, st));
    }
  }
  NCCLCHK(ncclGroupEnd());
  if (!src) {
    HIPCHK(hipEventRecord(m.done, st));
    return (int)CYC_OK;
  }

  // 2. a source partition's ingress slices, chunk by chunk of destination rows
  std::vector<uint32_t> a(static_cast<size_t>(n)), wr(static_cast<size_t>(n));
  for (int r = 0; r < n; r++) {
    int64_t v[5];
    std::string why;
    if (!rows_layout(c, part, lo[size_t(r)], hi[size_t(r)], v, why)) return fail(c, CYC_ERR_ARG, why);
    a[size_t(r)] = uint32_t(v[4]);
    wr[size_t(r)] = uint32_t(v[1]);
  }
  const uint64_t others = W - wr[size_t(me)];  // words per (row, slot) this rank receives
  uint64_t rows_blk = P;
  if (n > 1 && others) {
    rows_blk = std::max<uint64_t>(1, std::min<uint64_t>(P, COMM_CHUNK_BYTES / (row_words * 8)));
    const uint64_t need = rows_blk * K * others * 8;
    for (auto& s : m.scratch)
      if (s.bytes < need) s.alloc(need);
  }
  std::vector<const uint64_t*> ptr(static_cast<size_t>(n));
  for (uint64_t d0 = 0, ch = 0; d0 < P; d0 += rows_blk, ch++) {
    const uint64_t d1 = std::min(P, d0 + rows_blk), b = ch & 1;
    if (ch >= 2) HIPCHK(hipStreamWaitEvent(st, m.free_[b], 0));  // chunk ch - 2's relayout has read the buffer
    uint64_t off = 0;
    NCCLCHK(ncclGroupStart());
    for (int r = 0; r < n; r++) {
      const uint64_t cnt = (d1 - d0) * K * wr[size_t(r)];
      if (r == me) {
        ptr[size_t(r)] = in + d0 * K * wr[size_t(r)];  // (sent in place: root sendbuff == recvbuff)
        if (cnt && n > 1)
          NCCLCHK(ncclBroadcast(ptr[size_t(r)], const_cast<uint64_t*>(ptr[size_t(r)]), cnt, ncclUint64, r, m.nccl, st));
        continue;
      }
      uint64_t* dst = m.scratch[b].as<uint64_t>() + off;
      ptr[size_t(r)] = dst;
      off += cnt;
      if (cnt) NCCLCHK(ncclBroadcast(dst, dst, cnt, ncclUint64, r, m.nccl, st));
    }
    NCCLCHK(ncclGroupEnd());
    HIPCHK(hipEventRecord(m.full[b], st));
    HIPCHK(hipStreamWaitEvent(m.merge, m.full[b], 0));
    merge_launch(c, m.merge, n, ptr.data(), a.data(), wr.data(), full_in + d0 * row_words, int64_t(d0), int64_t(d1));
    HIPCHK(hipEventRecord(m.free_[b], m.merge));
  }
  HIPCHK(hipEventRecord(m.done, m.merge));
  HIPCHK(hipStreamWaitEvent(st, m.done, 0));  // the whole planes are complete in stream order on st
  return (int)CYC_OK;
}

}  // namespace

static void comm_release(cyc_ctx* c) {
  auto& m = c->comm;
  if (m.merge) (void)hipStreamSynchronize(m.merge);
  if (m.nccl) (void)ncclCommDestroy(m.nccl);
  m.nccl = nullptr;
  m.nranks = 0;
  m.rank = -1;
  for (int b = 0; b < 2; b++) {
    if (m.full[b]) (void)hipEventDestroy(m.full[b]);
    if (m.free_[b]) (void)hipEventDestroy(m.free_[b]);
    m.full[b] = m.free_[b] = nullptr;
    m.scratch[b].alloc(0);
  }
  if (m.done) (void)hipEventDestroy(m.done);
  if (m.merge) (void)hipStreamDestroy(m.merge);
  m.done = nullptr;
  m.merge = nullptr;
}

extern "C" {

int cyc_comm_unique_id(uint8_t* id) {
  if (!id) return CYC_ERR_ARG;
  static_assert(sizeof(ncclUniqueId) == CYC_COMM_ID_BYTES, "ncclUniqueId is CYC_COMM_ID_BYTES bytes");
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return CYC_ERR_RCCL;
  memcpy(id, &u, sizeof u);
  return (int)CYC_OK;
}

int cyc_comm_init(cyc_ctx* c, int nranks, int rank, const uint8_t* id) {
  if (!c) return CYC_ERR_ARG;
  if (!id) return fail(c, CYC_ERR_ARG, "null unique id");
  if (nranks < 1 || nranks > MERGE_MAX_RANKS) return fail(c, CYC_ERR_ARG, "nranks must be 1..64");
  if (rank < 0 || rank >= nranks) return fail(c, CYC_ERR_ARG, "rank out of range");
  if (!c->stream) return fail(c, CYC_ERR_HIP, "no HIP device for this context");
  return guarded(c, [&]() -> int {
    DeviceGuard dg(c->device);
    comm_release(c);  // (a context holds one communicator: a new init replaces it)
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    NCCLCHK(ncclCommInitRank(&c->comm.nccl, nranks, u, rank));
    c->comm.nranks = nranks;
    c->comm.rank = rank;
    return (int)CYC_OK;
  });
}

int cyc_comm_destroy(cyc_ctx* c) {
  if (!c) return CYC_ERR_ARG;
  return guarded(c, [&]() -> int {
    DeviceGuard dg(c->device, false);
    comm_release(c);
    return (int)CYC_OK;
  });
}

int cyc_rows_shard(cyc_ctx* c, int part, int nranks, int rank, int64_t* row_lo, int64_t* row_hi) {
  if (!c || !row_lo || !row_hi) return CYC_ERR_ARG;
  if (!c->prepared) return fail(c, CYC_ERR_ARG, "cyc_probe_prepare first");
  if (part != CYC_ROWS_TARGET && part != CYC_ROWS_SOURCE) return fail(c, CYC_ERR_ARG, "unknown partition");
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(c, CYC_ERR_ARG, "rank out of range");
  shard_rows(int64_t(c->pb.P), part, nranks, rank, *row_lo, *row_hi);
  return (int)CYC_OK;
}

int cyc_planes_allgather(cyc_ctx* c, void* stream, int part, const uint64_t* d_in, const uint64_t* d_eg,
                         uint64_t* d_in_full, uint64_t* d_eg_full) {
  if (!c) return CYC_ERR_ARG;
  std::string why;
  if (!comm_ready(c, why)) return fail(c, CYC_ERR_ARG, why);
  if (part != CYC_ROWS_TARGET && part != CYC_ROWS_SOURCE) return fail(c, CYC_ERR_ARG, "unknown partition");
  if (!d_in || !d_eg || !d_in_full || !d_eg_full) return fail(c, CYC_ERR_ARG, "null plane");
  if (part == CYC_ROWS_SOURCE && d_in == d_in_full && c->comm.nranks > 1)
    return fail(c, CYC_ERR_ARG, "source rows: the ingress slices cannot be assembled in place");
  return guarded(c, [&]() -> int {
    DeviceGuard dg(c->device);
    return planes_allgather(c, static_cast<hipStream_t>(stream), part, d_in, d_eg, d_in_full, d_eg_full);
  });
}

int cyc_rows_merge_sources(cyc_ctx* c, void* stream, int nranks, const uint64_t* const* d_slices, uint64_t* d_in_full) {
  if (!c) return CYC_ERR_ARG;
  if (!c->prepared) return fail(c, CYC_ERR_ARG, "cyc_probe_prepare first");
  if (!c->pb.blocks.empty()) return fail(c, CYC_ERR_ARG, "context prepared for blocks: nothing to assemble");
  if (nranks < 1 || nranks > MERGE_MAX_RANKS) return fail(c, CYC_ERR_ARG, "nranks must be 1..64");
  if (!d_slices || !d_in_full) return fail(c, CYC_ERR_ARG, "null plane");
  return guarded(c, [&]() -> int {
    DeviceGuard dg(c->device);
    std::vector<uint32_t> a(static_cast<size_t>(nranks)), wr(static_cast<size_t>(nranks));
    for (int r = 0; r < nranks; r++) {
      int64_t lo, hi, v[5];
      std::string why;
      shard_rows(int64_t(c->pb.P), CYC_ROWS_SOURCE, nranks, r, lo, hi);
      if (!rows_layout(c, CYC_ROWS_SOURCE, lo, hi, v, why)) return fail(c, CYC_ERR_ARG, why);
      if (v[1] && !d_slices[r]) return fail(c, CYC_ERR_ARG, "null slice of rank " + std::to_string(r));
      a[size_t(r)] = uint32_t(v[4]);
      wr[size_t(r)] = uint32_t(v[1]);
    }
    merge_launch(c, static_cast<hipStream_t>(stream), nranks, d_slices, a.data(), wr.data(), d_in_full, 0,
                 int64_t(c->pb.P));
    return (int)CYC_OK;
  });
}

int cyc_table_allgather(cyc_ctx* c, const cyc_table* shard, cyc_table** out) {
  if (!c || !shard || !out) return CYC_ERR_ARG;
  *out = nullptr;
  std::string why;
  if (!comm_ready(c, why)) return fail(c, CYC_ERR_ARG, why);
  if (shard->P != c->pb.P || shard->K != c->pb.K || shard->W != c->pb.W || shard->device != c->device)
    return fail(c, CYC_ERR_ARG, "the shard table is not of this context's prepared probe");
  int64_t lo, hi;
  shard_rows(int64_t(c->pb.P), shard->partition, c->comm.nranks, c->comm.rank, lo, hi);
  if (shard->row_lo != lo || shard->row_hi != hi)
    return fail(c, CYC_ERR_ARG, "the shard table's rows are not this rank's (cyc_rows_shard)");
  return guarded(c, [&]() -> int {
    DeviceGuard dg(c->device);
    cyc_table* t = nullptr;
    int rc = table_new(c, CYC_ROWS_TARGET, 0, int64_t(c->pb.P), &t);
    if (rc != CYC_OK) return rc;
    std::unique_ptr<cyc_table> hold(t);
    const uint64_t words = uint64_t(c->pb.P) * c->pb.K * c->pb.W, st_bytes = uint64_t(c->pb.P) * c->pb.K;
    t->own_in.alloc(std::max<uint64_t>(words * 8, 16));
    t->own_eg.alloc(std::max<uint64_t>(words * 8, 16));
    t->own_st.alloc(std::max<uint64_t>(st_bytes, 16));
    t->in = t->own_in.as<uint64_t>();
    t->eg = t->own_eg.as<uint64_t>();
    t->status = t->own_st.as<uint8_t>();
    if (st_bytes) HIPCHK(hipMemcpyAsync(t->own_st.p, shard->status, st_bytes, hipMemcpyDeviceToDevice, c->stream));
    rc = planes_allgather(c, c->stream, shard->partition, shard->in, shard->eg, t->own_in.as<uint64_t>(),
                          t->own_eg.as<uint64_t>());
    if (rc != CYC_OK) return rc;
    HIPCHK(hipStreamSynchronize(c->stream));
    ncclResult_t async = ncclSuccess;
    NCCLCHK(ncclCommGetAsyncError(c->comm.nccl, &async));
    if (async != ncclSuccess) throw RcclErr{std::string("RCCL: ") + ncclGetErrorString(async)};
    *out = hold.release();
    return (int)CYC_OK;
  });
}

}  // extern "C"
