// dev_member.hpp — membership: targets per identity, class hashes, representative election and the class of every identity.
// Part of engine.hip's single translation unit (device bodies inline across stages, host helpers are
// static): included once, by engine.hip, in stage order.
#pragma once

namespace cyc {

// Target membership per pod identity (TargetsApplyingToPod policy.go:68-82 over the identity's
// namespace's targets), class hash, and election of a representative per distinct class.
struct MemberArgs {
  uint32_t n_ident, L, K;
  const uint32_t *id_ns, *id_ls;
  const int32_t* id_desc;     // ingress: [n_ident][K] descriptor (-1 invalid); egress: null
  const uint8_t* id_status;   // ingress: [n_ident][K]
  const uint32_t *tns_lo, *tns_hi;
  const DTarget* tgt;
  SelView sv;                 // target pod selectors on the identity's label set
  const uint32_t* list_off;   // host-computed upper-bound offsets
  uint32_t* list;             // matching target ids (ascending = primary-key order)
  uint32_t* cnt;
  uint64_t* hash;
  uint8_t* err;               // a target selector panics on this identity
  unsigned long long* ht_key; // hash table (capacity ht_cap, power of two) of 16-byte entries:
                              // u64 key (~0 = empty), u32 min identity per key, u32 unused
  uint32_t ht_cap;
  const uint32_t* act;        // identities used by the rows of this run (range plan)
  const uint4* actrec;        // per act[] entry: (label set, namespace targets lo, hi, list offset)
  uint32_t n_act;
  uint32_t* reps;             // class representatives, act[] order within each block (k_classify)
  uint32_t* rep_cnt;          // [0] set to ~0 by k_member: ends at count - 1 of reps[]'s head; [1] set to 0:
                              // the count of its tail (row phases' phase-2 classes, RowArgs::phase_reps)
  const uint32_t* id_blk;     // batched blocks: each identity's block (classes never span blocks), else null
  // row phases (cyc_ctx::row_phases): a class whose representative's first row of the run is at or
  // after `split` is a phase-2 class, listed from the tail of reps[] (null: no phases)
  const uint32_t* first_row;  // per identity: its first pod's row in the run (cyc_ctx::arow)
  uint32_t split;
};

// Entry s: words 2s (key) and 2s + 1 (low half: representative); a probe reads both in one load.
__device__ __forceinline__ uint32_t* ht_rep_at(unsigned long long* ht, uint32_t s) {
  return reinterpret_cast<uint32_t*>(ht + 2 * uint64_t(s) + 1);
}

__device__ __forceinline__ uint32_t ht_find_or_insert(unsigned long long* ht, uint32_t cap, uint64_t h) {
  uint32_t s = uint32_t(h) & (cap - 1);
  for (uint32_t probe = 0; probe < cap; probe++) {
    unsigned long long cur = ht[2 * uint64_t(s)];
    if (cur == h) return s;
    if (cur == ~0ull) {
      unsigned long long old = atomicCAS(&ht[2 * uint64_t(s)], ~0ull, (unsigned long long)h);
      if (old == ~0ull || old == h) return s;
    }
    s = (s + 1) & (cap - 1);
  }
  return 0xFFFFFFFFu;  // unreachable: cap >= 2 * n_ident
}

// The representative stored under key h (plain 16-byte loads of whole entries), or ~0 when absent.
__device__ __forceinline__ uint32_t ht_find_rep(const unsigned long long* ht, uint32_t cap, uint64_t h) {
  uint32_t s = uint32_t(h) & (cap - 1);
  for (uint32_t probe = 0; probe < cap; probe++) {
    const ulonglong2 e = reinterpret_cast<const ulonglong2*>(ht)[s];
    if (e.x == h) return uint32_t(e.y);
    if (e.x == ~0ull) return 0xFFFFFFFFu;
    s = (s + 1) & (cap - 1);
  }
  return 0xFFFFFFFFu;
}

// Elect identity i as a candidate representative of key h.  A plain read first: the key is
// usually present already with a smaller identity (keys never change once set, reps only
// decrease, so a stale read can only send us to the atomics, never skip them wrongly); only
// otherwise the CAS insert + atomicMin (identities sharing a class then cost one read each
// instead of a serialised atomic on one address).
__device__ __forceinline__ void ht_elect(const MemberArgs& a, uint64_t h, uint32_t i) {
  if (ht_find_rep(a.ht_key, a.ht_cap, h) <= i) return;  // (absent: ~0)
  const uint32_t s = ht_find_or_insert(a.ht_key, a.ht_cap, h);
  atomicMin(ht_rep_at(a.ht_key, s), i);
}

__device__ __forceinline__ void member_blk(MemberArgs a, uint32_t bid_, uint32_t nblk_) {
  if (bid_ == 0 && threadIdx.x == 0) a.rep_cnt[0] = ~0u, a.rep_cnt[1] = 0u;  // k_classify counts up from here
  uint32_t ii = bid_ * blockDim.x + threadIdx.x;
  if (ii >= a.n_act) return;
  const uint32_t i = a.act[ii];
  const uint4 rec = a.actrec[ii];
  const uint32_t ls = rec.x, lo = rec.y, hi = rec.z, off = rec.w;
  uint32_t n = 0;
  uint8_t e = 0;
  uint64_t h = 0x5bd1e9955bd1e995ull;
  constexpr uint32_t MB = 8;  // targets whose selector results are loaded at once
  for (uint32_t t0 = lo; t0 < hi; t0 += MB) {
    uint32_t sel[MB];
    uint8_t r[MB];
#pragma unroll
    for (uint32_t x = 0; x < MB; x++) sel[x] = t0 + x < hi ? a.tgt[t0 + x].sel : 0u;
#pragma unroll
    for (uint32_t x = 0; x < MB; x++) r[x] = t0 + x < hi ? uint8_t(sel_at(a.sv, sel[x], ls)) : 0;
#pragma unroll
    for (uint32_t x = 0; x < MB; x++) {
      const uint32_t t = t0 + x;
      if (r[x] == 2) e = 1;
      if (r[x] == 1) {  // ascending target id = primary-key order
        a.list[off + n++] = t;
        h = mix64(h ^ (uint64_t(t) + 1));
      }
    }
  }
  if (a.id_desc) h = hash_slots(h, a.id_status, a.id_desc, i, a.K);
  if (a.id_blk) h = mix64(h ^ (uint64_t(a.id_blk[i]) << 24) ^ 0xB10Cull);  // a class row covers one block's words
  h &= 0x7FFFFFFFFFFFFFFFull;  // never the empty key (~0)
  a.cnt[i] = n;
  a.hash[i] = h;
  a.err[i] = e;
  // Many identities share a class (e.g. every pod no policy selects): only the lowest lane of a
  // wave holding a key (= lowest identity, act[] is sorted) does the atomics, so a popular key
  // costs one CAS + one atomicMin per wave instead of one per identity, while distinct keys
  // still insert in parallel.  Duplicates are found with register shuffles, not atomics.
  const bool want = !e;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t live = __ballot(want);
  bool leader = want;
  for (uint32_t j = 0; j < 64; j++) {
    const uint64_t hj = __shfl(h, int(j));
    if (j < lane && ((live >> j) & 1) && hj == h) leader = false;
  }
  if (leader) ht_elect(a, h, i);
}
__global__ void k_member(MemberArgs a) { member_blk(a, blockIdx.x, gridDim.x); }

// The same membership with one wave per identity (lanes over its namespace's targets, one ballot
// per 64 targets): a run has few identities per namespace but several targets each, so a thread
// per identity leaves the chip nearly idle behind a chain of dependent loads.  Same list order
// (ascending target id = primary-key order), same hash, same representative election.
__device__ __forceinline__ void member_wave_blk(MemberArgs a, uint32_t bid_, uint32_t nblk_) {
  if (bid_ == 0 && threadIdx.x == 0) a.rep_cnt[0] = ~0u, a.rep_cnt[1] = 0u;  // k_classify counts up from here
  const uint32_t lane = threadIdx.x & 63, ii = __builtin_amdgcn_readfirstlane(bid_ * 4 + (threadIdx.x >> 6));  // wave-uniform
  if (ii >= a.n_act) return;
  const uint32_t i = a.act[ii];
  const uint4 rec = a.actrec[ii];
  const uint32_t ls = rec.x, lo = rec.y, hi = rec.z, off = rec.w;
  uint32_t n = 0;
  bool e = false;
  uint64_t h = 0x5bd1e9955bd1e995ull;
  for (uint32_t t0 = lo; t0 < hi; t0 += 64) {
    const uint32_t t = t0 + lane;
    const uint8_t r = t < hi ? uint8_t(sel_at(a.sv, a.tgt[t].sel, ls)) : 0;
    e |= __ballot(r == 2) != 0;
    const uint64_t m = __ballot(r == 1);
    if (r == 1) a.list[off + n + __popcll(m & ((1ull << lane) - 1))] = t;
    for (uint64_t mm = m; mm; mm &= mm - 1) h = mix64(h ^ (uint64_t(t0 + __ffsll((unsigned long long)mm) - 1) + 1));
    n += __popcll(m);
  }
  if (a.id_desc) h = hash_slots(h, a.id_status, a.id_desc, i, a.K);
  if (a.id_blk) h = mix64(h ^ (uint64_t(a.id_blk[i]) << 24) ^ 0xB10Cull);  // a class row covers one block's words
  h &= 0x7FFFFFFFFFFFFFFFull;  // never the empty key (~0)
  if (lane == 0) {
    a.cnt[i] = n;
    a.hash[i] = h;
    a.err[i] = e;
    if (!e) ht_elect(a, h, i);
  }
}
__global__ __launch_bounds__(256) void k_member_wave(MemberArgs a) { member_wave_blk(a, blockIdx.x, gridDim.x); }

// Also compacts the class representatives: each block appends its representatives, in act[]
// order (ascending identity), at a base taken with one atomicAdd — consecutive identities (one
// namespace) stay adjacent, so consecutive class-row blocks share their targets' peer rows in
// L2.  The counter starts at ~0 (hash-table memset), so it ends at count - 1.
// The class of identity i (a thread's work): the representative the membership elected for its
// hash, verified equal — a 64-bit hash collision must never merge distinct classes — else i itself.
// 8 list entries / job slots of both identities per batch, every load of a batch issued before any
// compare (one memory round trip per batch instead of one per entry).  id_desc null: egress.
__device__ __forceinline__ uint32_t class_of_identity(uint32_t i, const uint8_t* __restrict__ err, const uint64_t* __restrict__ hash,
                                                      const unsigned long long* ht_key, uint32_t ht_cap,
                                                      const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ list_off,
                                                      const uint32_t* __restrict__ list, const uint32_t* __restrict__ id_blk,
                                                      const uint8_t* __restrict__ id_status, const int32_t* __restrict__ id_desc,
                                                      uint32_t K) {
  // identity i's own fields in one round trip with its hash (none depends on the representative); then,
  // once the representative is known, its fields and the first 8 job slots of both in one more, and its
  // list entries (they need its list offset) in the last: three round trips after the probe for the
  // usual short lists and K <= 8, where the batches below took five
  const uint8_t ei = err[i];
  const uint64_t hi = hash[i];
  const uint32_t n = cnt[i], oi = list_off[i], bi = id_blk ? id_blk[i] : 0u;
  if (ei) return i;
  const uint32_t r0 = ht_find_rep(ht_key, ht_cap, hi);
  const uint32_t r = r0 == 0xFFFFFFFFu ? i : r0;
  if (r == i) return i;
  const uint32_t nr = cnt[r], orr = list_off[r], br = id_blk ? id_blk[r] : 0u;
  uint8_t si[8], sr[8];
  int32_t di[8], dr[8];
  if (id_desc && K) {
#pragma unroll
    for (uint32_t u = 0; u < 8; u++) {
      const uint64_t k = min(u, K - 1);
      si[u] = id_status[uint64_t(i) * K + k];
      sr[u] = id_status[uint64_t(r) * K + k];
      di[u] = id_desc[uint64_t(i) * K + k];
      dr[u] = id_desc[uint64_t(r) * K + k];
    }
  }
  bool eq = nr == n && br == bi;
  for (uint32_t j0 = 0; eq && j0 < n; j0 += 8) {
    uint32_t x[8], y[8];
#pragma unroll
    for (uint32_t u = 0; u < 8; u++) {
      const uint32_t j = min(j0 + u, n - 1);
      x[u] = list[oi + j];
      y[u] = list[orr + j];
    }
#pragma unroll
    for (uint32_t u = 0; u < 8; u++) eq = eq && x[u] == y[u];
  }
  if (eq && id_desc) {
    for (uint32_t k0 = 0; eq && k0 < K; k0 += 8) {
      if (k0) {
#pragma unroll
        for (uint32_t u = 0; u < 8; u++) {
          const uint64_t k = min(k0 + u, K - 1);
          si[u] = id_status[uint64_t(i) * K + k];
          sr[u] = id_status[uint64_t(r) * K + k];
          di[u] = id_desc[uint64_t(i) * K + k];
          dr[u] = id_desc[uint64_t(r) * K + k];
        }
      }
#pragma unroll
      for (uint32_t u = 0; u < 8; u++) eq = eq && si[u] == sr[u] && (si[u] != CYC_JOB_VALID || di[u] == dr[u]);
    }
  }
  return eq ? r : i;
}

__device__ __forceinline__ void classify_blk(MemberArgs a, uint32_t* __restrict__ class_of, uint32_t bid_, uint32_t nblk_) {
  __shared__ uint32_t wsum[4], wsum2[4], base, base2;
  const uint32_t ii = bid_ * blockDim.x + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool live = ii < a.n_act;
  const uint32_t i = live ? a.act[ii] : 0;
  const uint32_t c = live ? class_of_identity(i, a.err, a.hash, a.ht_key, a.ht_cap, a.cnt, a.list_off, a.list, a.id_blk,
                                              a.id_status, a.id_desc, a.K)
                          : i;
  if (live) class_of[i] = c;
  // row phases: the representative (the class's smallest identity: identities are numbered in pod
  // order, so its first row is the class's) of a class first used at or after the split is listed from
  // the tail, so each phase's class-row launch covers exactly its own classes
  const bool f = live && c == i, late = f && a.first_row && a.first_row[i] >= a.split;
  const uint64_t m = __ballot(f && !late), m2 = __ballot(late);
  if (lane == 0) wsum[wv] = __popcll(m), wsum2[wv] = __popcll(m2);
  __syncthreads();
  if (threadIdx.x == 0) {
    base = atomicAdd(a.rep_cnt, wsum[0] + wsum[1] + wsum[2] + wsum[3]) + 1u;
    if (a.first_row) base2 = atomicAdd(a.rep_cnt + 1, wsum2[0] + wsum2[1] + wsum2[2] + wsum2[3]);
  }
  __syncthreads();
  uint32_t off = base, off2 = base2;
  for (uint32_t x = 0; x < wv; x++) off += wsum[x], off2 += wsum2[x];
  if (f && !late) a.reps[off + __popcll(m & ((1ull << lane) - 1))] = i;
  if (late) a.reps[a.n_ident - 1u - (off2 + __popcll(m2 & ((1ull << lane) - 1)))] = i;
}
__global__ __launch_bounds__(256) void k_classify(MemberArgs a, uint32_t* __restrict__ class_of) { classify_blk(a, class_of, blockIdx.x, gridDim.x); }

}  // namespace cyc
