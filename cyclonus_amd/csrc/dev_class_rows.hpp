// dev_class_rows.hpp — class rows: the ordered peer walk, identity sets, PM-build (PL) and identity-set (IDO) class rows.
// Part of engine.hip's single translation unit (device bodies inline across stages, host helpers are
// static): included once, by engine.hip, in stage order.
#pragma once

namespace cyc {

// Class rows.  For a class representative i, a chunk of KC job slots and one 64-pod word w, walk
// each of its targets' peers in slice order (target.go:29-36: short-circuit on the first
// allowing peer; a panicking peer ends the walk with a panic, ippeermatcher.go:46-48) for 64
// peer pods at once with bit operations, per slot because the port check differs per slot.
// A peer's PM/ER word is loaded once and used for all KC slots.
// KC (template): job slots per thread, 8 or 4.

struct RowArgs {
  const DTarget* tgt;
  const DPeer* peers;
  const uint64_t *PM, *ER;
  const uint8_t* portok;
  const uint32_t* portbits;  // fused IDO egress: portok row m as bits over descriptors (D <= 32), else null
  uint32_t D;
  uint32_t n_ident, K, W, P;
  // the word window of the class rows: words [w0, w0 + WA) of each row (a source shard's ingress
  // rows: its sources' words; otherwise 0, W); A rows hold WA words, word w at w - w0
  uint32_t w0, WA;
  // batched blocks (cyc_probe_prepare_blocks): each identity's own window (its block's words,
  // (w0, words)), at most WA words; A rows keep the stride WA
  const uint2* id_win;
  const uint32_t* reps;     // class representatives (k_classify)
  const uint32_t* rep_cnt;  // count = value + 1
  uint32_t rep_blocks;      // block rows of the grid; they stride over the representatives
  const uint32_t* class_of;
  const uint32_t *cnt, *list_off, *list;
  const uint8_t* id_err;
  const int32_t* id_desc;    // ingress only [n_ident][K]
  const uint8_t* id_status;  // ingress only
  const uint64_t* VALID;     // egress only [K][W]
  const int32_t* DESCW;      // egress only [K][W]
  const uint64_t* DM;        // egress only [K][D][W]
  const int32_t* udesc;      // egress: per slot the descriptor every destination has VALID (all alike), else null
  uint64_t* A;               // [n_ident][K][W], or the output plane when arow is set
  const uint32_t* arow;      // in-place class rows: identity -> its first pod's row of the output plane
  uint64_t* AE;              // [n_ident][K][W] (ERR builds only)
  // IDO builds (no panic possible, every 64-pod word holds <= IDO_MAX_RUNS identity runs):
  // pod peers are folded per class into identity-space sets B by k_class_ident, and the class
  // rows expand B through each word's runs; only IP peers are walked per pod word.
  const uint64_t* IDOB;      // [pod peers][EW] u64: pod peer matches egress identity e (bit e)
  const uint64_t* zero;      // 256 zero bytes: the target of branch-free loads for absent items
  const uint32_t* peer_ido;  // peer id -> IDOB row
  const uint32_t* prow;      // peer id -> its PM / ER row and IP word-span record (IP peers of one IPBlock share one)
  const struct WordRuns* runs;  // [W] each 64-pod word's identity runs (<= IDO_MAX_RUNS)
  uint64_t* B;               // [n_ident][NB][EW]; NB = K (ingress, per slot) or D (egress, per descriptor)
  const uint32_t* ip_off;    // [n_ident] host upper bound: IP peers of the identity's namespace's targets
  uint32_t* ip_cnt;          // [n_ident] IP peers of the class's targets, listed in ip_list as
  uint4* ip_list;            // (peer, port matcher, first, last nonzero PM word)
  const uint32_t* ip_rng;    // [R][4] per IP peer (no-panic runs): first word, ~last word of its nonzero PM
                             // words, then (u64) ~ the mask of its chunks holding one (chunks < 64)
  const uint32_t* ip_cnz;    // [R][W/64] 1 if the 64-word chunk of an IP peer's PM row was written
  uint32_t pod_sparse;       // PM builds' fused front: pod-peer rows are stored like IP rows (pod_rows_sparse_blk)
  uint32_t E, EW, NB;
  uint32_t ew_lo, ew_hi;     // IDO identity sets: the identity words the class rows read (a source shard's
                             // ingress rows: those of its sources' egress identities; else 0, EW)
  uint32_t rpb;              // IDO class rows: representatives per block (class_rows_ido_blk)
  // the direction's hash table (keys + reps), emptied for the NEXT run by the first class-row
  // kernel in block slices once k_classify is done with it: no memset node precedes k_member
  uint32_t* ht_clear;
  uint64_t ht_clear_words;
  // row phases: 1 = the classes rows [0, split) use, 2 = the others, 0 = every class (phase_reps)
  uint32_t phase;
};
// The representatives: k_classify lists the phase-1 classes' at the head of reps[] (rep_cnt[0] + 1 of
// them) and, on row-phased runs, the phase-2 classes' from its tail backwards (rep_cnt[1]): logical
// index k is reps[k] for k < n1, else reps[n_ident - 1 - (k - n1)].  (A class's representative is its
// smallest identity — the election keeps the minimum — and identities are numbered in pod order, so
// its first row is the class's first row: the representative alone decides the class's phase.)
__device__ __forceinline__ uint32_t rep_at(const RowArgs& a, uint32_t k) {
  const uint32_t n1 = *a.rep_cnt + 1u;
  return k < n1 ? a.reps[k] : a.reps[a.n_ident - 1u - (k - n1)];
}
// This launch's representatives (RowArgs::phase): logical indices [lo, lo + n)
__device__ __forceinline__ void phase_reps(const RowArgs& a, uint32_t& lo, uint32_t& n) {
  const uint32_t n1 = *a.rep_cnt + 1u, n2 = a.rep_cnt[1];
  lo = a.phase == 2 ? n1 : 0u;
  n = a.phase == 1 ? n1 : a.phase == 2 ? n2 : n1 + n2;
}

// Row of A holding representative i's class rows: its identity slot, or (in-place class rows) the
// plane row of the first pod of identity i in the run's rows — that pod's plane row IS the class
// row, so the emit leaves it alone and copies it to the class's other pods.
__device__ __forceinline__ uint64_t arow_of(const RowArgs& a, uint32_t i) { return a.arow ? a.arow[i] : i; }

// Words [w0, w0 + wa) of representative i's class rows: the run's window, or its block's.
__device__ __forceinline__ void rep_window(const RowArgs& a, uint32_t i, uint32_t& w0, uint32_t& wa) {
  if (a.id_win) {
    const uint2 v = a.id_win[i];
    w0 = v.x;
    wa = v.y;
  } else {
    w0 = a.w0;
    wa = a.WA;
  }
}

__device__ __forceinline__ void ht_clear_slice(const RowArgs& a, uint32_t bid, uint32_t nblk) {
  if (!a.ht_clear_words) return;
  const uint64_t per = (a.ht_clear_words + nblk - 1) / nblk, lo = uint64_t(bid) * per;
  const uint64_t hi = lo + per < a.ht_clear_words ? lo + per : a.ht_clear_words;
  for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) a.ht_clear[i] = 0xFFFFFFFFu;
}

// Most 64-pod words hold 1-2 identity runs (pods of a deployment are contiguous); IDO builds are
// used only when no word holds more than IDO_MAX_RUNS runs (host-checked, plan_peers).
constexpr uint32_t IDO_MAX_RUNS = 4;
struct WordRuns {
  uint32_t e[IDO_MAX_RUNS];   // egress identity of each run
  uint64_t m[IDO_MAX_RUNS];   // its pods in the word (0 = unused run)
};
constexpr uint32_t IDO_LDS_BYTES = 48 * 1024;  // staged identity sets per class-row block

// Pod-peer outcomes packed over egress identities: one wave per (64 identities, PB_GROUP pod
// peers): the identities' (namespace, namespace labels, labels) are loaded once and the group's
// outcomes (podpeermatcher.go:21-28: namespace then pod matcher) are independent selres gathers;
// one ballot per peer -> IDOB (no-panic runs only).
constexpr uint32_t PB_GROUP = 16;  // pod peers per identity-set wave (8: +4 % launch B, profiles/r02_pb_group_ab.txt)
// pod peers whose selector loads are in flight together (8: k_front_b 61 -> 81 VGPRs)
constexpr uint32_t PB_HALF_MAX = 4;
#ifndef CYC_PB_WIDE
#define CYC_PB_WIDE 8  // peers whose label-table gathers are in flight together (pb_rec path)
#endif
// Identity words [ew0, ew0 + new) of the rows only (a source shard's ingress peers: the words of the
// egress identities its sources have).
__device__ __forceinline__ void peer_bits_blk(uint32_t Rp, uint32_t E, uint32_t EW, const uint32_t* __restrict__ pod_peers,
                                                   const DPeer* __restrict__ peers, const SelView& sv,
                                                   const uint32_t* __restrict__ id_ns, const uint32_t* __restrict__ id_nsls,
                                                   const uint32_t* __restrict__ id_ls, uint64_t* __restrict__ idob, uint32_t bid_, uint32_t nblk_,
                                                   uint32_t ew0, uint32_t new_, const uint2* __restrict__ grp_ns,
                                                   const uint2* __restrict__ word_ns, const uint4* __restrict__ prec = nullptr) {
  // the wave index is wave-uniform: a scalar, so the peers' records below are scalar loads
  const uint32_t wv = __builtin_amdgcn_readfirstlane(bid_ * 4 + (threadIdx.x >> 6)), lane = threadIdx.x & 63;
  const uint32_t groups = (Rp + PB_GROUP - 1) / PB_GROUP;
  if (wv >= groups * new_) return;
  const uint32_t g = wv / new_, ew = ew0 + wv % new_, g0 = g * PB_GROUP;
  // the identities' own records and (pb_rec) the group's matcher records — 3 x 16 B a row, lane 3x +
  // part, ONE vector load — are issued before the skip test's loads, so their latencies overlap
  const uint32_t e = ew * 64 + lane;
  const bool live = e < E;
  const uint32_t ns = live ? id_ns[e] : 0u, nsls = live ? id_nsls[e] : 0u, ls = live ? id_ls[e] : 0u;
  const bool use_rec = prec && !sv.selres;
  const uint4 R = use_rec ? prec[min(3 * g0 + (lane < 3 * PB_GROUP ? lane : 0u), 3 * Rp - 1)] : uint4{0, 0, 0, 0};
  {  // a group of exact-namespace peers (podpeermatcher.go:115-125: ns == the policy's namespace) whose
     // namespaces the word's identities do not have matches none of them: zeros, no selector loads
    const uint2 gr = grp_ns[g], wr = word_ns[ew];
    if (gr.y < wr.x || gr.x > wr.y) {
      const uint32_t p = g0 + lane;
      if (lane < PB_GROUP && p < Rp) idob[uint64_t(p) * EW + ew] = 0;
      return;
    }
  }
  uint64_t mine = 0;
  if (use_rec) {
    // per PB_WIDE peers every label-table gather at once: two memory round trips a batch fewer than the
    // pod_peers -> peers -> one chain (podpeermatcher.go:21-28)
    constexpr uint32_t PB_WIDE = CYC_PB_WIDE;
#pragma unroll
    for (uint32_t h = 0; h < PB_GROUP; h += PB_WIDE) {
      uint32_t xn[PB_WIDE], xp[PB_WIDE];
#pragma unroll
      for (uint32_t x = 0; x < PB_WIDE; x++) {  // (record fields: scalar reads of lanes 3x + 1 / 2)
        const uint32_t on_x = __builtin_amdgcn_readlane(R.x, 3 * (h + x) + 1), on_y = __builtin_amdgcn_readlane(R.y, 3 * (h + x) + 1);
        const uint32_t op_x = __builtin_amdgcn_readlane(R.x, 3 * (h + x) + 2), op_y = __builtin_amdgcn_readlane(R.y, 3 * (h + x) + 2);
        xn[x] = sv.LVT[uint64_t(on_x < SEL_ALL ? on_y : 0u) * sv.L + nsls];
        xp[x] = sv.LVT[uint64_t(op_x < SEL_ALL ? op_y : 0u) * sv.L + ls];
      }
#pragma unroll
      for (uint32_t x = 0; x < PB_WIDE; x++) {
        const uint32_t q = 3 * (h + x);
        const uint32_t nk = __builtin_amdgcn_readlane(R.x, q), nv = __builtin_amdgcn_readlane(R.y, q),
                       ps = __builtin_amdgcn_readlane(R.z, q);
        const uint32_t on_x = __builtin_amdgcn_readlane(R.x, q + 1), op_x = __builtin_amdgcn_readlane(R.x, q + 2);
        uint32_t rn = 1u, rp = 1u;
        if (nk == 2 && on_x == SEL_WALK) rn = sel_eval(sv, sv.LVT, sv.L, nv, nsls);
        else if (nk == 2 && on_x != SEL_ALL)
          rn = req_holds(on_x & 0xFFu, xn[x], __builtin_amdgcn_readlane(R.z, q + 1), __builtin_amdgcn_readlane(R.w, q + 1), on_x >> 8);
        if (ps != CYC_ALL && op_x == SEL_WALK) rp = sel_eval(sv, sv.LVT, sv.L, ps, ls);
        else if (ps != CYC_ALL && op_x != SEL_ALL)
          rp = req_holds(op_x & 0xFFu, xp[x], __builtin_amdgcn_readlane(R.z, q + 2), __builtin_amdgcn_readlane(R.w, q + 2), op_x >> 8);
        const bool m = live && g0 + h + x < Rp && (nk != 0 || ns == nv) && rn == 1 && rp == 1;
        const uint64_t b = __ballot(m);
        if (lane == h + x) mine = b;
      }
    }
    const uint32_t p = g0 + lane;
    if (lane < PB_GROUP && p < Rp) idob[uint64_t(p) * EW + ew] = mine;
    return;
  }
  // PB_HALF peers at a time, in phases — their records, then every selector outcome, then the ballots —
  // so the loads of all of them are in flight together instead of one dependent chain per peer
  // (podpeermatcher.go:21-28 namespace then pod matcher; no panic on this path, so both matchers
  // can be evaluated for every peer and combined)
  constexpr uint32_t PB_HALF = PB_GROUP < PB_HALF_MAX ? PB_GROUP : PB_HALF_MAX;
#pragma unroll
  for (uint32_t h = 0; h < PB_GROUP; h += PB_HALF) {
    uint32_t nk[PB_HALF], nv[PB_HALF], ps[PB_HALF];
    bool ok[PB_HALF];
#pragma unroll
    for (uint32_t x = 0; x < PB_HALF; x++) {
      const uint32_t p = g * PB_GROUP + h + x;
      ok[x] = p < Rp;
      const DPeer pr = peers[pod_peers[ok[x] ? p : g * PB_GROUP]];
      nk[x] = pr.nskind;
      nv[x] = pr.nsval;
      ps[x] = pr.podsel;
    }
    uint32_t rn[PB_HALF], rp[PB_HALF];
    if (sv.selres) {  // dense selector table: one byte gather per matcher, all issued unconditionally
      uint8_t an[PB_HALF], ap[PB_HALF];
#pragma unroll
      for (uint32_t x = 0; x < PB_HALF; x++) an[x] = sv.selres[uint64_t(nk[x] == 2 ? nv[x] : 0u) * sv.L + nsls];
#pragma unroll
      for (uint32_t x = 0; x < PB_HALF; x++) ap[x] = sv.selres[uint64_t(ps[x] != CYC_ALL ? ps[x] : 0u) * sv.L + ls];
#pragma unroll
      for (uint32_t x = 0; x < PB_HALF; x++) {
        rn[x] = nk[x] == 2 ? an[x] : 1u;
        rp[x] = ps[x] != CYC_ALL ? ap[x] : 1u;
      }
    } else {  // selectors evaluated here: one-requirement records (scalar), then every LVT gather at once
      uint4 on[PB_HALF], op[PB_HALF];
#pragma unroll
      for (uint32_t x = 0; x < PB_HALF; x++) {
        on[x] = sv.one[nk[x] == 2 ? nv[x] : 0u];
        op[x] = sv.one[ps[x] != CYC_ALL ? ps[x] : 0u];
      }
      uint32_t xn[PB_HALF], xp[PB_HALF];
#pragma unroll
      for (uint32_t x = 0; x < PB_HALF; x++) {
        xn[x] = sv.LVT[uint64_t(on[x].x < SEL_ALL ? on[x].y : 0u) * sv.L + nsls];
        xp[x] = sv.LVT[uint64_t(op[x].x < SEL_ALL ? op[x].y : 0u) * sv.L + ls];
      }
#pragma unroll
      for (uint32_t x = 0; x < PB_HALF; x++) {
        rn[x] = 1u;
        if (nk[x] == 2 && on[x].x == SEL_WALK) rn[x] = sel_eval(sv, sv.LVT, sv.L, nv[x], nsls);
        else if (nk[x] == 2 && on[x].x != SEL_ALL) rn[x] = req_holds(on[x].x & 0xFFu, xn[x], on[x].z, on[x].w, on[x].x >> 8);
        rp[x] = 1u;
        if (ps[x] != CYC_ALL && op[x].x == SEL_WALK) rp[x] = sel_eval(sv, sv.LVT, sv.L, ps[x], ls);
        else if (ps[x] != CYC_ALL && op[x].x != SEL_ALL) rp[x] = req_holds(op[x].x & 0xFFu, xp[x], op[x].z, op[x].w, op[x].x >> 8);
      }
    }
#pragma unroll
    for (uint32_t x = 0; x < PB_HALF; x++) {
      const bool m = live && ok[x] && (nk[x] != 0 || ns == nv[x]) && rn[x] == 1 && rp[x] == 1;
      const uint64_t b = __ballot(m);
      if (lane == h + x) mine = b;
    }
  }
  const uint32_t p = g * PB_GROUP + lane;
  if (lane < PB_GROUP && p < Rp) idob[uint64_t(p) * EW + ew] = mine;
}
__global__ __launch_bounds__(256) void k_peer_bits(uint32_t Rp, uint32_t E, uint32_t EW, const uint32_t* __restrict__ pod_peers,
                                                   const DPeer* __restrict__ peers, const uint8_t* __restrict__ selres, uint32_t L,
                                                   const uint32_t* __restrict__ id_ns, const uint32_t* __restrict__ id_nsls,
                                                   const uint32_t* __restrict__ id_ls, uint64_t* __restrict__ idob, uint32_t ew0,
                                                   uint32_t new_, const uint2* __restrict__ grp_ns, const uint2* __restrict__ word_ns) {
  SelView sv{};
  sv.selres = selres;
  sv.L = L;
  peer_bits_blk(Rp, E, EW, pod_peers, peers, sv, id_ns, id_nsls, id_ls, idob, blockIdx.x, gridDim.x, ew0, new_, grp_ns, word_ns);
}

// Per class representative and NB index (ingress: job slot, egress: job descriptor): the set of
// egress identities its targets' pod / all / ports-for-all peers allow on that port (target.go:29-36
// is an OR over peers; without a panic its order only matters for early exit).  One wave per
// (representative, NB index), lanes over 64-identity words.
// The class's peers are first flattened, in target order, into a per-wave LDS list (targets 64 at
// a time, a wave prefix sum over their peer counts), so the walk loads CI_BATCH peers' fields and
// identity-set words at once — one chain of dependent loads per batch instead of per peer (the
// walk dominates this launch on row shards, where few classes leave the chip mostly idle).
// Classes with more than CI_LDS peers walk the targets directly.
constexpr uint32_t CI_LDS = 128;
constexpr int CI_G = 4;  // identity sets: job slots (ingress) / descriptors (egress) per wave
template <bool EGRESS, int G>
__device__ __forceinline__ void class_ident_blk(RowArgs a, uint32_t bid_, uint32_t nblk_) {
  __shared__ uint32_t s_j[4][CI_LDS];
  __shared__ uint32_t s_pid[4][CI_LDS], s_pk[4][CI_LDS];  // per entry: identity-set row; kind << 16 | port-test bits
  ht_clear_slice(a, bid_, nblk_);
  // one wave per (representative, G NB indices): each peer's IDOB word is loaded once for all G
  const uint32_t wi = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), wv = bid_ * 4 + wi, lane = threadIdx.x & 63;
  const uint32_t nbc = (a.NB + G - 1) / G;
  const uint32_t r = wv / nbc, nb0 = (wv % nbc) * G;
  uint32_t rlo, rn;
  phase_reps(a, rlo, rn);
  if (r >= rn) return;
  const uint32_t i = rep_at(a, rlo + r);
  int32_t du[G];
  {  // ingress: the slots' status and descriptor, all G pairs loaded at once
    uint8_t st[G];
    int32_t ds[G];
#pragma unroll
    for (uint32_t x = 0; x < uint32_t(G); x++) {
      const uint64_t ik = EGRESS ? 0u : uint64_t(i) * a.K + min(nb0 + x, a.K - 1);
      st[x] = EGRESS ? uint8_t(0) : a.id_status[ik];
      ds[x] = EGRESS ? 0 : a.id_desc[ik];
    }
#pragma unroll
    for (uint32_t x = 0; x < uint32_t(G); x++) {
      const uint32_t nb = nb0 + x;
      du[x] = -1;
      if (nb < a.NB) du[x] = EGRESS ? int32_t(nb) : (st[x] == CYC_JOB_VALID ? ds[x] : -1);
    }
  }
  const uint32_t n = a.cnt[i];
  const uint32_t* lst = a.list + a.list_off[i];
  uint32_t* sj = s_j[wi];
  uint32_t m = 0;
  for (uint32_t t0 = 0; t0 < n; t0 += 64) {
    uint32_t poff = 0, pc = 0;
    if (t0 + lane < n) {
      const DTarget tg = a.tgt[lst[t0 + lane]];
      poff = tg.poff;
      pc = tg.pcnt;
    }
    uint32_t x = pc;  // inclusive prefix sum over the wave
    for (uint32_t o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    const uint32_t base = m + x - pc;
    for (uint32_t k = 0; k < pc && base + k < CI_LDS; k++) sj[base + k] = poff + k;
    m += __shfl(x, 63);
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the list is read back by other lanes
  const bool flat = m <= CI_LDS;
  if (flat) {  // each entry's record, identity-set row and port test, a lane per entry: two load levels for all
    for (uint32_t x = lane; x < m; x += 64) {
      const uint32_t j = sj[x];
      const DPeer pr = a.peers[j];
      const uint32_t pid = a.peer_ido[j];
      const uint32_t port = pr.kind == 0 ? 0u : pr.port;
      uint32_t okb = 0;
      if (a.portbits) {
        const uint32_t pb = a.portbits[port];
#pragma unroll
        for (uint32_t y = 0; y < uint32_t(G); y++)
          if (du[y] >= 0 && ((pb >> du[y]) & 1u)) okb |= 1u << y;
      } else {
        uint8_t pkb[G];
#pragma unroll
        for (uint32_t y = 0; y < uint32_t(G); y++) pkb[y] = a.portok[uint64_t(port) * a.D + uint32_t(max(du[y], 0))];
#pragma unroll
        for (uint32_t y = 0; y < uint32_t(G); y++)
          if (du[y] >= 0 && pkb[y]) okb |= 1u << y;
      }
      s_pid[wi][x] = pid;
      s_pk[wi][x] = (pr.kind << 16) | okb;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
  for (uint32_t ew0 = a.ew_lo; ew0 < a.ew_hi; ew0 += 64) {
    const uint32_t ew = ew0 + lane;
    uint64_t b[G];
#pragma unroll
    for (uint32_t x = 0; x < uint32_t(G); x++) b[x] = (n == 0 && du[x] >= 0) ? ~0ull : 0ull;  // no target: allowed (policy.go:158-160)
    if (flat) {
      // no panic on this path: the OR over peers is order-free (AllPeersMatcher: every valid cell)
      // entries staged once per wave (below, before this loop): only the identity-set words are
      // loaded here, CI_WB at a time
      constexpr uint32_t CI_WB = 8;
      for (uint32_t x0 = 0; x0 < m; x0 += CI_WB) {
        uint32_t pk[CI_WB];
        uint64_t v[CI_WB];
#pragma unroll
        for (uint32_t u = 0; u < CI_WB; u++) {
          const uint32_t x = min(x0 + u, m - 1);
          const uint32_t pid = __builtin_amdgcn_readfirstlane(s_pid[wi][x]);
          pk[u] = x0 + u < m ? __builtin_amdgcn_readfirstlane(s_pk[wi][x]) : (3u << 16);
          const uint32_t kind = pk[u] >> 16;
          const uint64_t iv = *(kind == 2 && ew < a.EW ? a.IDOB + uint64_t(pid) * a.EW + ew : a.zero);
          v[u] = kind == 0 || kind == 1 ? ~0ull : iv;
        }
#pragma unroll
        for (uint32_t u = 0; u < CI_WB; u++) {
          const uint32_t kind = pk[u] >> 16;
          if (kind == 3) continue;  // IP peers: per pod word, in the class rows
#pragma unroll
          for (uint32_t x = 0; x < uint32_t(G); x++)
            if (du[x] >= 0 && (kind == 0 || ((pk[u] >> x) & 1u))) b[x] |= v[u];
        }
      }
    } else {
      for (uint32_t tj = 0; tj < n; tj++) {
        const DTarget tg = a.tgt[lst[tj]];
        for (uint32_t j = tg.poff; j < tg.poff + tg.pcnt; j++) {
          const DPeer pr = a.peers[j];
          if (pr.kind == 3) continue;  // IP peers: per pod word, in the class rows
          const uint8_t* pok = a.portok + uint64_t(pr.port) * a.D;
          if (pr.kind == 0) {  // AllPeersMatcher
#pragma unroll
            for (uint32_t x = 0; x < uint32_t(G); x++) b[x] = du[x] >= 0 ? ~0ull : 0ull;
            break;
          }
          const uint64_t vv = pr.kind == 1 ? ~0ull : (ew < a.EW ? a.IDOB[uint64_t(a.peer_ido[j]) * a.EW + ew] : 0ull);
#pragma unroll
          for (uint32_t x = 0; x < uint32_t(G); x++)
            if (du[x] >= 0 && pok[du[x]]) b[x] |= vv;  // PortsForAllPeers / pod peer on an allowed port
        }
      }
    }
    if (ew < a.ew_hi) {
#pragma unroll
      for (uint32_t x = 0; x < uint32_t(G); x++)
        if (nb0 + x < a.NB) a.B[(uint64_t(i) * a.NB + nb0 + x) * a.EW + ew] = b[x];
    }
  }
  if (nb0 != 0) return;
  // the class's IP peers (whatever the port) with nonzero rows, walked per pod word by the class rows
  uint4* il = a.ip_list + a.ip_off[i];
  if (flat) {  // lanes over the list, compacted by ballot; none when an AllPeersMatcher allows all
    uint32_t mm = 0;
    bool all = false;
    for (uint32_t e0 = 0; e0 < m; e0 += 64) {
      const uint32_t e = e0 + lane;
      uint32_t j = 0, kind = 3, r0 = 0xFFFFFFFFu;
      if (e < m) {
        j = sj[e];
        kind = a.peers[j].kind;
        if (kind == 3) r0 = a.ip_rng[4 * a.prow[j]];
      }
      all |= __ballot(e < m && kind == 0) != 0;
      const bool keep = e < m && kind == 3 && r0 != 0xFFFFFFFFu;
      const uint64_t bm = __ballot(keep);
      if (keep && !all) {
        const uint32_t row = a.prow[j];
        il[mm + __popcll(bm & ((1ull << lane) - 1))] = make_uint4(row, a.peers[j].port, r0, ~a.ip_rng[4 * row + 1]);
      }
      mm += __popcll(bm);
    }
    if (lane == 0) a.ip_cnt[i] = all ? 0u : mm;
    return;
  }
  if (lane == 0) {
    uint32_t mm = 0;
    for (uint32_t tj = 0; tj < n; tj++) {
      const DTarget tg = a.tgt[lst[tj]];
      for (uint32_t j = tg.poff; j < tg.poff + tg.pcnt; j++) {
        const DPeer pr = a.peers[j];
        if (pr.kind == 0) break;  // AllPeers: the identity sets already allow everything
        if (pr.kind != 3) continue;
        const uint32_t row = a.prow[j];
        if (a.ip_rng[4 * row] != 0xFFFFFFFFu) il[mm++] = make_uint4(row, pr.port, a.ip_rng[4 * row], ~a.ip_rng[4 * row + 1]);
      }
    }
    a.ip_cnt[i] = mm;
  }
}
template <bool EGRESS, int G>
__global__ __launch_bounds__(256) void k_class_ident(RowArgs a) { class_ident_blk<EGRESS, G>(a, blockIdx.x, gridDim.x); }

// Port check of one peer's port matcher row `pok` for job slot k of pod word w: all 64 pods
// (descriptor du >= 0), none (invalid slot), or per destination (egress word whose
// destinations have mixed job descriptors, through DM; rare).
template <bool EGRESS>
__device__ __forceinline__ uint64_t port_mask(const RowArgs& a, const uint8_t* pok, int32_t du, uint32_t k, uint32_t w) {
  if (du >= 0) return pok[du] ? ~0ull : 0ull;
  if (!EGRESS || du == -2) return 0ull;
  uint64_t okm = 0;
  const uint64_t* dm = a.DM + uint64_t(k) * a.D * a.W + w;
  for (uint32_t d = 0; d < a.D; d++)
    if (pok[d]) okm |= dm[uint64_t(d) * a.W];
  return okm;
}
constexpr uint32_t PEER_BATCH = 4;  // IDO class rows: IP peers whose PM words are loaded at once

template <bool EGRESS, bool ERR, int KC>
__device__ __forceinline__ void class_row_word(const RowArgs& a, uint32_t i, uint32_t kc, uint32_t w, uint32_t w0) {
  const uint32_t k0 = kc * KC;
  const uint64_t lastmask = (a.P % 64) ? ((1ull << (a.P % 64)) - 1) : ~0ull;
  const uint64_t wmask = (w == a.W - 1) ? lastmask : ~0ull;

  uint64_t valid[KC], allow[KC], err[KC];
  int32_t du[KC];
#pragma unroll
  for (int kk = 0; kk < KC; kk++) {
    uint32_t k = k0 + kk;
    valid[kk] = 0;
    du[kk] = -2;
    allow[kk] = 0;
    err[kk] = 0;
    if (k < a.K) {
      if (EGRESS) {
        valid[kk] = a.VALID[uint64_t(k) * a.W + w];
        du[kk] = a.DESCW[uint64_t(k) * a.W + w];
      } else {
        bool v = a.id_status[uint64_t(i) * a.K + k] == CYC_JOB_VALID;
        valid[kk] = v ? wmask : 0ull;
        du[kk] = v ? a.id_desc[uint64_t(i) * a.K + k] : -2;
      }
    }
  }
  // A panicking membership (labelselector.go:57 via TargetsApplyingToPod) makes every VALID
  // cell of the row panic, which the error path reports; the row itself is left zero.
  const uint32_t n = a.id_err[i] ? 0xFFFFFFFFu : a.cnt[i];
  if (n == 0) {
#pragma unroll
    for (int kk = 0; kk < KC; kk++) allow[kk] = ~0ull;  // no target applies: allowed (policy.go:158-160)
  } else if (n != 0xFFFFFFFFu) {
    const uint32_t* lst = a.list + a.list_off[i];
    for (uint32_t tj = 0; tj < n; tj++) {
      DTarget tg = a.tgt[lst[tj]];
      uint64_t dec[KC];
#pragma unroll
      for (int kk = 0; kk < KC; kk++) dec[kk] = ~valid[kk];  // invalid slots / dsts / padding: pre-decided
      for (uint32_t j = tg.poff; j < tg.poff + tg.pcnt; j++) {
        DPeer pr = a.peers[j];
        if (pr.kind == 0) {  // AllPeersMatcher: everything undecided is allowed
#pragma unroll
          for (int kk = 0; kk < KC; kk++) allow[kk] |= ~dec[kk];
          break;
        }
        uint64_t pm = ~0ull, er = 0;
        const uint32_t row = pr.kind == 3 ? a.prow[j] : j;
        if (!ERR && pr.kind == 3 && (w < a.ip_rng[4 * row] || w > ~a.ip_rng[4 * row + 1])) continue;  // zero word
        if (pr.kind >= 2) {
          pm = a.PM[uint64_t(row) * a.W + w];
          if (ERR) er = a.ER[uint64_t(row) * a.W + w];
        }
        const uint8_t* pok = a.portok + uint64_t(pr.port) * a.D;
        uint64_t alldec = ~0ull;
#pragma unroll
        for (int kk = 0; kk < KC; kk++) {
          uint64_t okm;
          if (du[kk] >= 0) {
            okm = pok[du[kk]] ? ~0ull : 0ull;
          } else if (!EGRESS || du[kk] == -2) {
            okm = 0;
          } else {  // egress word whose destinations have mixed job descriptors (rare)
            okm = 0;
            const uint64_t* dm = a.DM + uint64_t(k0 + kk) * a.D * a.W + w;
            for (uint32_t d = 0; d < a.D; d++)
              if (pok[d]) okm |= dm[uint64_t(d) * a.W];
          }
          uint64_t ne = er & ~dec[kk];
          uint64_t na = pm & okm & ~dec[kk] & ~er;
          if (ERR) err[kk] |= ne;
          allow[kk] |= na;
          dec[kk] |= ne | na;
          alldec &= dec[kk];
        }
        if (alldec == ~0ull) break;
      }
    }
  }
#pragma unroll
  for (int kk = 0; kk < KC; kk++) {
    uint32_t k = k0 + kk;
    if (k < a.K) {
      uint64_t idx = (uint64_t(i) * a.K + k) * a.WA + (w - w0);
      a.A[idx] = allow[kk] & valid[kk];
      if (ERR) a.AE[idx] = err[kk] & valid[kk];
    }
  }
}

// Panic-capable builds (ordered walk with panic bits).  Grid = representative slots x slot chunks
// x 256-word chunks: one block row per representative slot (the count of classes is only known on
// the device; surplus rows exit at once), 8 job slots per thread.
template <bool EGRESS>
__global__ __launch_bounds__(256) void k_class_rows(RowArgs a) {
  constexpr int KC = 8;
  ht_clear_slice(a, blockIdx.x, gridDim.x);
  const uint32_t chunks = (a.WA + 255) / 256, nkc = (a.K + KC - 1) / KC;
  const uint32_t kc = (blockIdx.x / chunks) % nkc;
  const uint32_t lw = (blockIdx.x % chunks) * 256 + threadIdx.x;
  const uint32_t r = blockIdx.x / (chunks * nkc);
  uint32_t rlo, rn;
  phase_reps(a, rlo, rn);
  if (r >= rn) return;
  const uint32_t i = rep_at(a, rlo + r);
  uint32_t w0, wa;
  rep_window(a, i, w0, wa);
  if (lw < wa) class_row_word<EGRESS, true, KC>(a, i, kc, w0 + lw, w0);
}

// Class rows of PM builds without a panic.  Block = class representative (blocks stride over
// them).  The block first flattens the class's peers cooperatively into LDS — lanes over its
// targets, then over their peers: (PM row, nonzero word span, port test pre-resolved as a bit row:
// ingress = one bit per job slot of this representative, egress = the port matcher's descriptor
// bits) — so the long chain of dependent loads (membership list -> target -> peer -> word span)
// runs once per class with every lane's loads in flight, not once per pod word.  Then each
// (slot chunk, pod word) item ORs its peers' PM words, PL_BATCH loads in flight.  Without a panic
// the verdict is that OR (target.go:29-36 short-circuits only to save work); an AllPeersMatcher
// (peermatcher.go:18) allows every valid cell; no matching target allows (policy.go:158-160).
// Lists longer than the LDS part spill into the identity's ip_list slot (sized for every peer of
// its namespace's targets).
// PL_BATCH: list entries whose PM words are loaded at once (16: occupancy 6 -> 4); PL_THREADS: threads
// per class-row block (one representative per block)
constexpr uint32_t PL_LDS = 256, PL_TGT = 64, PL_BATCH = 8, PL_THREADS = 128;
constexpr uint32_t PL_SKIP = 0xFFFFFFFEu, PL_ONES = 0xFFFFFFFFu;  // entry rows: zero row / PortsForAllPeers
constexpr uint32_t PL_IP = 0x80000000u;

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

// The neighbouring lane's (lane ^ 1) 8-byte value, by DPP quad permutation [1, 0, 3, 2].
__device__ __forceinline__ uint64_t lane_pair_swap(uint64_t v) {
  const uint32_t lo = uint32_t(__builtin_amdgcn_mov_dpp(int(uint32_t(v)), 0xB1, 0xF, 0xF, false));
  const uint32_t hi = uint32_t(__builtin_amdgcn_mov_dpp(int(uint32_t(v >> 32)), 0xB1, 0xF, 0xF, false));
  return (uint64_t(hi) << 32) | lo;
}
// Words off, off ^ 1 (lanes 2j, 2j + 1 hold one word each) of two class-row slot rows as 16-byte
// stores: the even lane writes row ra's pair, the odd lane row rb's — half the store instructions
// of 8-byte stores (the class rows are store-issue bound: config #3 / #4 class rows 30 us faster
// with their stores removed).  Rows 16-byte aligned, off even on even lanes, both lanes live.
__device__ __forceinline__ void store_row_pair(uint64_t* ra, uint64_t* rb, uint64_t off, uint64_t va, uint64_t vb, bool odd) {
  const uint64_t got = lane_pair_swap(odd ? va : vb);
  if (!odd) *reinterpret_cast<u64x2*>(ra + off) = u64x2{va, got};
  else *reinterpret_cast<u64x2*>(rb + off - 1) = u64x2{got, vb};
}

// PM word of list entry e for pod word w (0 outside the entry's span)
__device__ __forceinline__ uint64_t pl_word(const RowArgs& a, const uint4& e, uint32_t w) {
  if (e.x == PL_ONES) return ~0ull;
  const uint32_t lo = e.z & ~PL_IP;
  if (e.x == PL_SKIP || w < lo || w > e.w) return 0ull;
  const uint64_t v = a.PM[uint64_t(e.x) * a.W + w];
  return (e.z & PL_IP) ? v & cnz_mask(a.ip_cnz, a.W, e.x, w) : v;
}
struct PlShared {  // one per block, shared by both directions' instantiations of a fused launch
  uint4 e[PL_LDS];        // (row, port matcher, first word, last word)
  uint32_t bits[PL_LDS];  // port test bits
  uint32_t pre[PL_TGT + 1], poff[PL_TGT];
  uint32_t all;
  int32_t rdu[32];  // ingress, K <= 32: the representative's job descriptor per slot (-1: slot not VALID)
};

constexpr int PL_ITEMS = 1;

// PL_ITEMS (slot chunk, pod word) items of class representative i: items it0, it0 + blockDim.x, ...
template <bool EGRESS>
__device__ __forceinline__ void pl_items(const RowArgs& a, const PlShared& sh, const uint4* spill, uint32_t i, uint32_t m,
                                         bool allow_all, bool kbits, uint32_t it0, uint32_t items, uint64_t lastmask,
                                         uint32_t w0, uint32_t wa) {
  constexpr int KC = 4, NI = PL_ITEMS;
  uint64_t valid[NI][KC], allow[NI][KC];
  int32_t du[NI][KC];
  uint32_t w[NI], k0[NI];
  bool fast = kbits;
#pragma unroll
  for (int q = 0; q < NI; q++) {
    const uint32_t it = it0 + q * blockDim.x;
    const bool live = it < items;
    const uint32_t kc = live ? it / wa : 0u;
    w[q] = w0 + (live ? it - kc * wa : 0u);
    k0[q] = live ? kc * KC : a.K;  // a dead item has no slot
#pragma unroll
    for (int kk = 0; kk < KC; kk++) {
      const uint32_t k = k0[q] + kk;
      valid[q][kk] = 0;
      du[q][kk] = -2;
      if (k < a.K) {
        if (EGRESS) {
          valid[q][kk] = a.VALID[uint64_t(k) * a.W + w[q]];
          du[q][kk] = a.DESCW[uint64_t(k) * a.W + w[q]];
        } else {
          const bool v = a.id_status[uint64_t(i) * a.K + k] == CYC_JOB_VALID;
          valid[q][kk] = v ? (w[q] == a.W - 1 ? lastmask : ~0ull) : 0ull;
          du[q][kk] = v ? a.id_desc[uint64_t(i) * a.K + k] : -2;
        }
      }
      fast = fast && du[q][kk] != -1;  // -1: egress word whose destinations mix descriptors
      allow[q][kk] = allow_all ? ~0ull : 0ull;
    }
  }
  if (!allow_all && fast && m <= PL_LDS) {
    // The entries are the same for every thread of the block: a batch's fields are read from LDS
    // into scalar registers first, then all of the batch's PM (and nonzero-mask) loads are issued,
    // and only then combined — one memory round trip per batch, not one per entry.
    for (uint32_t x0 = 0; x0 < m; x0 += PL_BATCH) {
      uint32_t ex[PL_BATCH], ez[PL_BATCH], ew[PL_BATCH], bits[PL_BATCH];
#pragma unroll
      for (uint32_t u = 0; u < PL_BATCH; u++) {
        const uint32_t x = min(x0 + u, PL_LDS - 1);
        uint4 e = sh.e[x];
        const uint32_t b = sh.bits[x];
        if (x0 + u >= m) e.x = PL_SKIP;
        ex[u] = __builtin_amdgcn_readfirstlane(e.x);
        ez[u] = __builtin_amdgcn_readfirstlane(e.z);
        ew[u] = __builtin_amdgcn_readfirstlane(e.w);
        bits[u] = __builtin_amdgcn_readfirstlane(b);
      }
      uint64_t v[NI][PL_BATCH], c[NI][PL_BATCH];
#pragma unroll
      for (uint32_t u = 0; u < PL_BATCH; u++)
#pragma unroll
        for (int q = 0; q < NI; q++) {
          v[q][u] = 0;
          c[q][u] = ~0ull;
          if (ex[u] < PL_SKIP && w[q] >= (ez[u] & ~PL_IP) && w[q] <= ew[u]) {
            v[q][u] = a.PM[uint64_t(ex[u]) * a.W + w[q]];
            if (ez[u] & PL_IP) c[q][u] = a.ip_cnz[uint64_t(ex[u]) * ((a.W + 63) / 64) + w[q] / 64];
          }
        }
      uint64_t undecided = 0;
#pragma unroll
      for (int q = 0; q < NI; q++) {
        // entries are sorted by port bits: OR each run of equal bits first, then test its slots once
        uint64_t acc = 0;
#pragma unroll
        for (uint32_t u = 0; u < PL_BATCH; u++) {
          acc |= ex[u] == PL_ONES ? ~0ull : (c[q][u] ? v[q][u] : 0ull);
          if (u + 1 < PL_BATCH && bits[u + 1] == bits[u]) continue;  // the run goes on (uniform)
          if (acc) {
#pragma unroll
            for (int kk = 0; kk < KC; kk++) {
              if (du[q][kk] < 0) continue;
              if (EGRESS) allow[q][kk] |= ((bits[u] >> uint32_t(du[q][kk])) & 1u) ? acc : 0ull;
              else if ((bits[u] >> (k0[q] + kk)) & 1u) allow[q][kk] |= acc;  // the same for the whole block
            }
          }
          acc = 0;
        }
#pragma unroll
        for (int kk = 0; kk < KC; kk++) undecided |= valid[q][kk] & ~allow[q][kk];
      }
      if (!undecided) break;
    }
  } else if (!allow_all) {  // mixed descriptors, no bit rows (ingress K > 32), lists past the LDS part
    // ingress with K <= 32: an entry's .y is its slot bits for this representative (class_rows_pl_blk),
    // not a port matcher id; every other entry carries the port matcher
    const bool slot_bits = !EGRESS && a.K <= 32;
    for (uint32_t x = 0; x < m; x++) {
      const uint4 e = x < PL_LDS ? sh.e[x] : spill[x];
#pragma unroll
      for (int q = 0; q < NI; q++) {
        const uint64_t pm = pl_word(a, e, w[q]);
        if (!pm) continue;
#pragma unroll
        for (int kk = 0; kk < KC; kk++) {
          if (slot_bits) {
            if (du[q][kk] >= 0 && ((e.y >> (k0[q] + kk)) & 1u)) allow[q][kk] |= pm;
          } else {
            allow[q][kk] |= pm & port_mask<EGRESS>(a, a.portok + uint64_t(e.y) * a.D, du[q][kk], k0[q] + kk, w[q]);
          }
        }
      }
    }
  }
#pragma unroll
  for (int q = 0; q < NI; q++)
#pragma unroll
    for (int kk = 0; kk < KC; kk++) {
      const uint32_t k = k0[q] + kk;
      if (k < a.K) a.A[(arow_of(a, i) * a.K + k) * a.WA + (w[q] - w0)] = allow[q][kk] & valid[q][kk];
    }
}

// The class rows a WAVE PER 64-WORD CHUNK (port bit rows available, at most PL_NB descriptors /
// slots, at most 64 chunks): lane = pod word.  The class's entries sit one per lane (row, port
// bits, mask of the chunks where the entry's PM row has a nonzero word — for IP rows recorded by
// the IP-row pass, so zero chunks are never read); per chunk one ballot picks the entries that
// matter there (a CIDR covers a few chunks) and their PM words are loaded PL_WBATCH at a time, all
// in flight together, then ORed into an accumulator per descriptor (egress) or slot (ingress)
// bit.  The accumulators become the class rows through each word's slot descriptor (DESCW; the DM
// masks for mixed words).

// PL_WBATCH: PM words in flight per wave-per-chunk batch (8: 78 VGPRs, config #4 class rows +7 us:
// profiles/r03_front_b_d_ab.txt)
constexpr uint32_t PL_WBATCH = 4, PL_NB = 4;
// An entry's lane fields for the wave-per-chunk rows: row, port bits, mask of the 64-word chunks
// holding a nonzero PM word of it (IP rows: from the IP-row pass; other rows: all)
struct PlLane {
  uint32_t row, bits;
  uint64_t cm;
};
__device__ __forceinline__ PlLane pl_lane(const RowArgs& a, const uint4* src, uint32_t x, uint32_t m) {
  PlLane l{PL_SKIP, 0u, 0ull};
  if (x < m) {
    const uint4 e = src[x];  // (row, port bits, first word | PL_IP, last word)
    l.row = e.x;
    l.bits = e.y;
    // the chunk mask is loaded whatever the entry (a zero word for the others): no wait in a branch
    const bool sparse = e.x < PL_SKIP && (e.z & PL_IP);
    const uint64_t nm = *(sparse ? reinterpret_cast<const uint64_t*>(a.ip_rng) + 2 * e.x + 1 : a.zero);
    if (e.x == PL_SKIP || !e.y) l.cm = 0;
    else if (sparse) l.cm = ~nm;
    else l.cm = ~0ull;
  }
  return l;
}

// Pops up to PL_WBATCH entries of `todo` (lanes of the wave's entry group g) and loads their PM words
// of pod word wl, branch-free: all of the batch's loads are in flight together.
__device__ __forceinline__ void pl_load_batch(const RowArgs& a, const PlLane& g, uint64_t& todo, uint32_t wl,
                                              uint64_t (&v)[PL_WBATCH], uint32_t (&bits)[PL_WBATCH]) {
#pragma unroll
  for (uint32_t u = 0; u < PL_WBATCH; u++) {
    uint32_t row = PL_SKIP;
    bits[u] = 0;
    if (todo) {  // wave-uniform
      const uint32_t src = __ffsll((unsigned long long)todo) - 1;
      todo &= todo - 1;
      row = __builtin_amdgcn_readlane(g.row, src);
      bits[u] = __builtin_amdgcn_readlane(g.bits, src);
    }
    const uint64_t x = *(row < PL_SKIP ? a.PM + uint64_t(row) * a.W + wl : a.zero);
    v[u] = row == PL_ONES ? ~0ull : x;
  }
}

template <bool EGRESS, bool UNI = false>
__device__ __forceinline__ void pl_wave_chunks(const RowArgs& a, const PlShared& sh, const uint4* spill, uint32_t i,
                                               uint32_t m, bool allow_all, uint64_t lastmask, uint32_t w0, uint32_t wa) {
  static_assert(PL_LDS % 64 == 0, "a lane group of entries is all in LDS or all spilled");
  const uint32_t lane = threadIdx.x & 63, nwaves = blockDim.x >> 6;
  // the chunks holding the window's words (<= 64 chunks in all: pl_wave_ok)
  const uint32_t cend = (w0 + wa + 63) / 64;
  const PlLane g0 = pl_lane(a, sh.e, lane, m);  // entries 0..63, one per lane, for every chunk
  uint64_t* const rows = a.A + arow_of(a, i) * a.K * a.WA;  // the class row's slot 0
  const bool pair = a.WA % 2 == 0 && w0 % 2 == 0 && reinterpret_cast<uintptr_t>(a.A) % 16 == 0;
  uint32_t vslots = 0;  // ingress: the representative's VALID slots (class_rows_pl_blk staged them)
  if (!EGRESS)
#pragma unroll
    for (uint32_t k = 0; k < PL_NB; k++)
      if (k < a.K && sh.rdu[k] >= 0) vslots |= 1u << k;
  for (uint32_t c = w0 / 64 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); c < cend; c += nwaves) {
    const uint32_t w = c * 64 + lane;
    const bool live = w >= w0 && w < w0 + wa;
    const uint32_t wl = live ? w : w0;  // dead lanes load a valid word and store nothing
    uint64_t valid[PL_NB];
    int32_t du[PL_NB];
#pragma unroll
    for (uint32_t k = 0; k < PL_NB; k++) {  // slot words, loaded with the first batch
      valid[k] = 0;
      du[k] = -2;
      if (k < a.K) {
        if (EGRESS && UNI) {  // one descriptor per slot for every destination (RowArgs::udesc)
          valid[k] = w == a.W - 1 ? lastmask : ~0ull;
          du[k] = a.udesc[k];
        } else if (EGRESS) {
          valid[k] = a.VALID[uint64_t(k) * a.W + wl];
          du[k] = a.DESCW[uint64_t(k) * a.W + wl];
        } else if ((vslots >> k) & 1u) {
          valid[k] = w == a.W - 1 ? lastmask : ~0ull;
        }
      }
    }
    uint64_t acc[PL_NB];
#pragma unroll
    for (uint32_t d = 0; d < PL_NB; d++) acc[d] = allow_all ? ~0ull : 0ull;
    for (uint32_t x0 = 0; x0 < (allow_all ? 0u : m); x0 += 64) {
      PlLane g = g0;  // (uniform branches: an LDS or a global load, never a flat one)
      if (x0 >= PL_LDS) g = pl_lane(a, spill, x0 + lane, m);
      else if (x0) g = pl_lane(a, sh.e, x0 + lane, m);
      // the entries with a nonzero PM word in this chunk; their words are loaded PL_WBATCH at a time
      uint64_t todo = __ballot((g.cm >> c) & 1ull);
      while (todo) {
        uint32_t bits[PL_WBATCH];
        uint64_t v[PL_WBATCH];
        pl_load_batch(a, g, todo, wl, v, bits);
#pragma unroll
        for (uint32_t u = 0; u < PL_WBATCH; u++)
#pragma unroll
          for (uint32_t d = 0; d < PL_NB; d++)
            if ((bits[u] >> d) & 1u) acc[d] |= v[u];
      }
    }
    if (!live) continue;
    uint64_t rr[PL_NB];
#pragma unroll
    for (uint32_t k = 0; k < PL_NB; k++) {
      uint64_t r = 0;
      if (k >= a.K) {
      } else if (!EGRESS) r = acc[k] & valid[k];
      else if (du[k] >= 0) {
#pragma unroll
        for (uint32_t d = 0; d < PL_NB; d++) r = uint32_t(du[k]) == d ? acc[d] : r;
        r &= valid[k];
      } else if (du[k] == -1) {  // destinations with mixed job descriptors (rare)
        const uint64_t* dm = a.DM + uint64_t(k) * a.D * a.W + w;
#pragma unroll
        for (uint32_t d = 0; d < PL_NB; d++)
          if (d < a.D) r |= acc[d] & dm[uint64_t(d) * a.W];
        r &= valid[k];
      }
      rr[k] = r;
    }
    const uint64_t off = w - w0;
    uint32_t k = 0;
    if (pair)
#pragma unroll
      for (; k + 1 < PL_NB; k += 2) {
        if (k + 1 >= a.K) break;
        store_row_pair(rows + uint64_t(k) * a.WA, rows + uint64_t(k + 1) * a.WA, off, rr[k], rr[k + 1], lane & 1);
      }
#pragma unroll
    for (uint32_t kk = 0; kk < PL_NB; kk++)
      if (kk >= k && kk < a.K) rows[uint64_t(kk) * a.WA + off] = rr[kk];
  }
}

template <bool EGRESS, bool WAVE>
__device__ __forceinline__ void class_rows_pl_blk(const RowArgs& a, PlShared& sh, uint32_t bid_, uint32_t nblk_) {
  constexpr int KC = 4;
  ht_clear_slice(a, bid_, nblk_);
  const uint32_t nkc = (a.K + KC - 1) / KC;
  uint32_t rlo, n_reps;
  phase_reps(a, rlo, n_reps);
  const bool kbits = EGRESS ? a.portbits != nullptr : a.K <= 32;
  for (uint32_t r = bid_; r < n_reps; r += nblk_) {
    const uint32_t i = rep_at(a, rlo + r);
    const uint32_t nt = a.cnt[i];
    const uint32_t* lst = a.list + a.list_off[i];
    uint4* spill = a.ip_list + a.ip_off[i] - PL_LDS;  // entries x >= PL_LDS live at spill[x]
    if (threadIdx.x == 0) sh.all = 0;
    // ingress (K <= 32): the representative's descriptor per slot, read by the peers' slot bits below
    // and by the chunk walk (the first barrier of the target loop, or the one after it, publishes it)
    if (!EGRESS && threadIdx.x < min(a.K, 32u)) {
      const uint64_t ik = uint64_t(i) * a.K + threadIdx.x;
      const uint8_t st = a.id_status[ik];
      const int32_t ds = a.id_desc[ik];
      sh.rdu[threadIdx.x] = st == CYC_JOB_VALID ? ds : -1;
    }
    uint32_t m = 0;
    for (uint32_t t0 = 0; t0 < nt; t0 += PL_TGT) {  // targets in chunks: offsets, counts, prefix sums
      const uint32_t ntc = min(PL_TGT, nt - t0);
      static_assert(PL_TGT == 64, "one wave scans a target chunk");
      if (threadIdx.x < 64) {  // wave 0: the chunk's targets a lane each, peer counts prefix-summed in registers
        uint32_t v = 0;
        if (threadIdx.x < ntc) {
          const DTarget tg = a.tgt[lst[t0 + threadIdx.x]];
          sh.poff[threadIdx.x] = tg.poff;
          v = tg.pcnt;
        }
#pragma unroll
        for (uint32_t o = 1; o < 64; o <<= 1) {
          const uint32_t u = __shfl_up(v, o);
          if (threadIdx.x >= o) v += u;
        }
        if (threadIdx.x < ntc) sh.pre[threadIdx.x + 1] = v;
        if (threadIdx.x == 0) sh.pre[0] = 0;
      }
      __syncthreads();
      const uint32_t mc = sh.pre[ntc];
      for (uint32_t e = threadIdx.x; e < mc; e += blockDim.x) {  // the peers, one per lane
        uint32_t lo = 0, hi = ntc;  // target of peer e: pre[lo] <= e < pre[lo + 1]
        while (hi - lo > 1) {
          const uint32_t mid = (lo + hi) >> 1;
          if (sh.pre[mid] <= e) lo = mid;
          else hi = mid;
        }
        const uint32_t j = sh.poff[lo] + (e - sh.pre[lo]);
        // every lane issues the same loads in two levels (peer + its row id, then the row's word span
        // and the port bits), whatever the peer's kind: no load waits inside a divergent branch
        const DPeer pr = a.peers[j];
        const uint32_t prj = a.prow[j];
        const uint32_t row = pr.kind == 3 ? prj : j;
        const uint32_t rlo = a.ip_rng[4 * row], rhi = a.ip_rng[4 * row + 1];
        const uint32_t pbits = a.portbits ? a.portbits[pr.kind == 0 ? 0u : pr.port] : 0u;
        uint4 en = make_uint4(PL_SKIP, 0u, 1u, 0u);
        uint32_t bits = 0;
        if (pr.kind == 0) {
          sh.all = 1;  // AllPeersMatcher
        } else {
          // PortsForAllPeers, and a pod peer of every pod in every namespace (podpeermatcher.go with
          // AllNamespaceMatcher + AllPodMatcher): all-ones rows, never loaded (nor built, sparse rows)
          const bool ones = pr.kind == 1 || (pr.kind == 2 && pr.nskind == 1 && pr.podsel == CYC_ALL);
          en = make_uint4(ones ? PL_ONES : row, pr.port, 0u, a.W - 1);
          if (!ones && (pr.kind == 3 || (pr.kind == 2 && a.pod_sparse))) {  // bit 31 of z: a sparse row (only the cnz-marked words were written)
            en.z = rlo | PL_IP;
            en.w = ~rhi;
            if (rlo == 0xFFFFFFFFu) en.x = PL_SKIP;  // an all-zero row
          }
          if (EGRESS) {
            bits = pbits;
          } else if (a.K <= 32) {  // a bit per job slot of this representative
            for (uint32_t k = 0; k < a.K; k++) {
              const int32_t du = sh.rdu[k];
              if (du < 0) continue;
              if (a.portbits ? ((pbits >> du) & 1u) : a.portok[uint64_t(pr.port) * a.D + du]) bits |= 1u << k;
            }
          }
          // spilled entries (and every entry of the wave-per-chunk rows) carry the bits themselves
          en.y = WAVE || (!EGRESS && a.K <= 32) ? bits : pr.port;
          if (kbits && !bits) en.x = PL_SKIP;  // the port matcher passes no slot / descriptor here
        }
        const uint32_t x = m + e;
        if (x < PL_LDS) {
          sh.e[x] = en;
          sh.bits[x] = bits;
        } else {
          spill[x] = en;
        }
      }
      m += mc;
      __syncthreads();
    }
    if (!WAVE && threadIdx.x == 0 && m <= 64) {  // group entries by port bits: each group's slot test runs once
      for (uint32_t x = 1; x < m; x++) {
        const uint4 e = sh.e[x];
        const uint32_t b = sh.bits[x];
        uint32_t y = x;
        for (; y > 0 && sh.bits[y - 1] > b; y--) {
          sh.e[y] = sh.e[y - 1];
          sh.bits[y] = sh.bits[y - 1];
        }
        sh.e[y] = e;
        sh.bits[y] = b;
      }
    }
    __syncthreads();
    const bool allow_all = nt == 0 || sh.all;
    const uint64_t lastmask = (a.P % 64) ? ((1ull << (a.P % 64)) - 1) : ~0ull;
    // the class's (slot chunk, word) items, PL_ITEMS per thread at once (their loads overlap)
    uint32_t w0, wa;
    rep_window(a, i, w0, wa);
    if (WAVE && EGRESS && a.udesc) {
      pl_wave_chunks<EGRESS, true>(a, sh, spill, i, m, allow_all, lastmask, w0, wa);
    } else if (WAVE) {
      pl_wave_chunks<EGRESS>(a, sh, spill, i, m, allow_all, lastmask, w0, wa);
    } else {
      const uint32_t items = nkc * wa;
      for (uint32_t it0 = threadIdx.x; it0 < items; it0 += PL_ITEMS * blockDim.x)
        pl_items<EGRESS>(a, sh, spill, i, m, allow_all, kbits, it0, items, lastmask, w0, wa);
    }
    __syncthreads();  // LDS reused by the next representative
  }
}
template <bool EGRESS, bool WAVE>
__global__ __launch_bounds__(256) void k_class_rows_pl(RowArgs a) {
  __shared__ PlShared sh;
  class_rows_pl_blk<EGRESS, WAVE>(a, sh, blockIdx.x, gridDim.x);
}

// Class rows from identity sets (IDO builds).  Block = (class representative, KC job slots,
// 256 pod words); the representative's identity sets for those slots (ingress) or for every job
// descriptor (egress) are staged in LDS, each thread expands them over its word's identity runs
// (one 48-byte record), then ORs in the class's IP peers (PM words; the only per-pod peers).
// The staged sets are 32-bit words with the block's rows interleaved (IdoRuns): a run's bit of
// every slot row is one LDS read, and a run adds its pods to a slot's word with a sign-extended
// bit field and two and-or operations (v_bfe_i32, v_and_or_b32) instead of a 64-bit shift, compare
// and two selects: config #3's class rows issued ~1,000 VALU instructions per wave, ~75 % of
// the launch at 4 cycles each (profiles/r04_pmc_config3.txt).
struct IdoRuns {  // a thread's word's identity runs, resolved against the staged layout
  uint32_t off[IDO_MAX_RUNS];  // (identity >> 5) * rows: the run's 32-bit word in a representative's sets
  uint32_t sh[IDO_MAX_RUNS];   // identity & 31
  uint32_t lo[IDO_MAX_RUNS], hi[IDO_MAX_RUNS];  // the run's pods in the word (0: unused run)
};
__device__ __forceinline__ void ido_or_run(uint32_t bits, uint32_t sh, uint32_t lo, uint32_t hi, uint32_t& alo, uint32_t& ahi) {
  const uint32_t sel = uint32_t(__builtin_amdgcn_sbfe(int(bits), sh, 1));  // 0 or ~0
  alo |= lo & sel;
  ahi |= hi & sel;
}
// Row `row` of a representative's staged sets (sq) expanded over the word's runs.
__device__ __forceinline__ uint64_t expand_runs32(const uint32_t* sq, uint32_t row, const IdoRuns& ir) {
  uint32_t alo = 0, ahi = 0;
#pragma unroll
  for (uint32_t x = 0; x < IDO_MAX_RUNS; x++) ido_or_run(sq[ir.off[x] + row], ir.sh[x], ir.lo[x], ir.hi[x], alo, ahi);
  return (uint64_t(ahi) << 32) | alo;
}

constexpr uint32_t IDO_RPB_MAX = 64;  // class_rpb's upper bound
constexpr uint32_t IDO_IPL = 16;      // IP peers per representative staged in LDS (row, span, port bits)
// Grid rows of the IDO class rows per (slot chunk, representative group): 256-word chunks (staging
// once for 2 / 4 / 7 chunks per block measured slower on config #3: profiles/r03_ido_rows_ab.txt).
__host__ __device__ inline uint32_t ido_chunk_groups(uint32_t WA) { return (WA + 255) / 256; }
// The PM words (and chunk marks) of the staged IP peers listed in the bit mask pend (up to N of them, taken off
// pend) for pod word w.
// Branch-free: every lane issues every load (a zero word where the peer is absent or w is outside its
// span), so the batch's loads are in flight together — a load under a divergent branch is waited
// for at the branch's end, which serialises a batch into one memory round trip per peer.
template <uint32_t N>
__device__ __forceinline__ void ido_ip_loads_mask(const RowArgs& a, const uint4* sl, uint32_t& pend, uint32_t w,
                                                  uint64_t (&pm)[N], uint32_t (&pbits)[N]) {
  const uint32_t cw = (a.W + 63) / 64;
  uint4 e[N];
  bool ok[N];
  bool any = false;
#pragma unroll
  for (uint32_t u = 0; u < N; u++) {
    const bool in = pend != 0;
    e[u] = sl[in ? __builtin_ctz(pend) : 0u];
    pend &= pend - 1;
    ok[u] = in && w >= e[u].y && w <= e[u].z;
    pbits[u] = in ? e[u].w : 0u;
    pm[u] = 0;
    any |= ok[u];
  }
  if (!__ballot(any)) return;
  uint64_t v[N];
  uint32_t cm[N];
#pragma unroll
  for (uint32_t u = 0; u < N; u++) {
    v[u] = *(ok[u] ? a.PM + uint64_t(e[u].x) * a.W + w : a.zero);
    cm[u] = *(ok[u] ? a.ip_cnz + uint64_t(e[u].x) * cw + w / 64 : reinterpret_cast<const uint32_t*>(a.zero));
  }
#pragma unroll
  for (uint32_t u = 0; u < N; u++) pm[u] = cm[u] ? v[u] : 0ull;
}

template <int KC>
struct RepHead {  // a class-row block's representative: identity, class-row index, IP-peer list, slot descriptors
  uint32_t i, arow, m, ipoff;
  int32_t du[KC];
};

// UNI (egress): every destination has the same VALID job descriptor in each slot (a.udesc[k]), so the
// slot's descriptor is a scalar and its valid mask every pod: no per-word VALID / DESCW loads, and
// only the block's KC descriptors' identity sets are staged (config #3 / #4: identical containers).
template <bool EGRESS, int KC, bool UNI = false>
__device__ __forceinline__ void class_rows_ido_blk(RowArgs a, uint32_t bid_, uint32_t nblk_) {
  extern __shared__ __attribute__((aligned(16))) uint64_t sB[];
  // block = (a.rpb consecutive class representatives, KC job slots, 256 pod words): each word's runs
  // and slot words are loaded once for all its representatives
  const uint32_t cg = ido_chunk_groups(a.WA), nkc = (a.K + KC - 1) / KC;
  const uint32_t kc = (bid_ / cg) % nkc;
  uint32_t rlo, n_reps;
  phase_reps(a, rlo, n_reps);
  const uint32_t r0 = (bid_ / (cg * nkc)) * a.rpb;
  if (r0 >= n_reps) return;  // whole block
  const uint32_t nr = min(a.rpb, n_reps - r0);
  const uint32_t k0 = kc * KC;
  const uint32_t nrow = EGRESS && !UNI ? a.NB : min(uint32_t(KC), a.K - k0);
  // staged layout: 32-bit word j of row r of representative q at sB32[(q * EW32 + j) * NS + r]
  const uint32_t NS = EGRESS && !UNI ? a.NB : uint32_t(KC), EW32 = 2 * a.EW;
  uint32_t* const sB32 = reinterpret_cast<uint32_t*>(sB);
  const uint32_t wend = a.w0 + a.WA;
  // the word's own loads (runs) are issued before the staging barrier, so their latency overlaps the
  // staging loads instead of following them
  const uint32_t w = a.w0 + (bid_ % cg) * 256 + threadIdx.x;
  WordRuns wr = a.runs[min(w, wend - 1)];  // (lanes past the window load a valid record and store nothing)
  const uint64_t lastmask = (a.P % 64) ? ((1ull << (a.P % 64)) - 1) : ~0ull;
  // Staging in two dependency levels, every load of a level issued unconditionally (clamped
  // indices, zero words) so a level is one memory round trip: (1) each representative's scalars —
  // identity, class-row index, IP-peer list, ingress slot descriptors — a thread each; (2) after a
  // barrier, its identity sets (B) and its first IDO_IPL IP peers with their port bits.  The row
  // loop then reads them from LDS instead of walking reps -> identity -> list chains.
  __shared__ RepHead<KC> s_rep[IDO_RPB_MAX];
  if (threadIdx.x < nr) {
    RepHead<KC> h;
    h.i = rep_at(a, rlo + r0 + threadIdx.x);
    h.arow = uint32_t(arow_of(a, h.i));
    const uint32_t cn = a.cnt[h.i], ipc = a.ip_cnt[h.i];
    h.ipoff = a.ip_off[h.i];
    uint8_t st[KC];
    int32_t ds[KC];
#pragma unroll
    for (int kk = 0; kk < KC; kk++) {
      const uint64_t ik = uint64_t(h.i) * a.K + min(k0 + kk, a.K - 1);
      st[kk] = EGRESS ? uint8_t(0) : a.id_status[ik];
      ds[kk] = EGRESS ? 0 : a.id_desc[ik];
    }
    h.m = cn ? ipc : 0u;
#pragma unroll
    for (int kk = 0; kk < KC; kk++) h.du[kk] = !EGRESS && k0 + kk < a.K && st[kk] == CYC_JOB_VALID ? ds[kk] : -2;
    s_rep[threadIdx.x] = h;
  }
  int32_t ud[KC];  // egress UNI: the block's slots' descriptors (block-uniform)
#pragma unroll
  for (int kk = 0; kk < KC; kk++) ud[kk] = EGRESS && UNI ? a.udesc[min(k0 + kk, a.K - 1)] : 0;
  __syncthreads();
  {  // identity sets: a wave per (representative, row) at a time, lanes over the row's words, 4 rows'
     // loads in flight; (representative, row) is wave-uniform, so the transposing index math is scalar
    const uint32_t nrows = nr * nrow, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint32_t r0 = wv; r0 < nrows; r0 += 4 * nw)
      for (uint32_t j0 = 0; j0 < a.EW; j0 += 64) {
        const uint32_t j = min(j0 + lane, a.EW - 1);
        uint64_t v[4];
#pragma unroll
        for (uint32_t u = 0; u < 4; u++) {
          const uint32_t qr = min(r0 + u * nw, nrows - 1), q = qr / nrow, row = qr - q * nrow;
          const uint64_t i = s_rep[q].i;
          int32_t d = EGRESS ? int32_t(row) : int32_t(k0 + row);  // the set's row in B
          if (EGRESS && UNI) {  // the sets of the block's slots' descriptors, one row each
            d = ud[0];
#pragma unroll
            for (int y = 1; y < KC; y++) d = uint32_t(y) == row ? ud[y] : d;
          }
          v[u] = a.B[(i * a.NB + uint32_t(d)) * a.EW + j];
        }
#pragma unroll
        for (uint32_t u = 0; u < 4; u++) {
          const uint32_t qr = r0 + u * nw, q = qr / nrow, row = qr - q * nrow;
          if (qr >= nrows || j0 + lane >= a.EW) continue;
          uint32_t* dst = sB32 + (q * EW32 + 2 * j) * NS + row;
          dst[0] = uint32_t(v[u]);
          dst[NS] = uint32_t(v[u] >> 32);
        }
      }
  }
  // the first IDO_IPL IP peers of each representative: (PM row, first word, last word, port bits —
  // egress: the descriptor bit row; ingress: a bit per block slot), so the row loop issues only the
  // PM loads (no list -> port table chain per batch)
  uint4* s_il = reinterpret_cast<uint4*>(sB32 + ((nr * EW32 * NS + 3) & ~3u));  // 16-byte aligned
  const bool stage_ip = !EGRESS || a.portbits != nullptr;
  // per representative: which staged peers have nonzero PM words inside the block's words (a CIDR
  // covers a few namespaces' pods, so most (representative, 256-word chunk) pairs have none)
  __shared__ uint32_t s_ipm[IDO_RPB_MAX];
  if (stage_ip) {
    const uint32_t wlo = a.w0 + (bid_ % cg) * 256, whi = min(wlo + 255, wend - 1);
    static_assert(64 % IDO_IPL == 0, "a representative's staged peers lie in one wave");
    for (uint32_t t = threadIdx.x; t < ((nr * IDO_IPL + 63) & ~63u); t += blockDim.x) {
      const RepHead<KC>& h = s_rep[min(t / IDO_IPL, nr - 1)];
      const uint32_t x = t % IDO_IPL;
      const bool ok = t < nr * IDO_IPL && x < h.m;
      const uint4 jp = *(ok ? a.ip_list + h.ipoff + x : reinterpret_cast<const uint4*>(a.zero));
      const uint64_t hit = __ballot(ok && jp.z <= whi && jp.w >= wlo);
      if (x == 0 && t < nr * IDO_IPL) s_ipm[t / IDO_IPL] = uint32_t(hit >> (t & 63 & ~(IDO_IPL - 1))) & ((1u << IDO_IPL) - 1);
      uint32_t bits = 0;
      if (EGRESS) {
        bits = *(ok ? a.portbits + jp.y : reinterpret_cast<const uint32_t*>(a.zero));
      } else {
        uint8_t pk[KC];
#pragma unroll
        for (int kk = 0; kk < KC; kk++)
          pk[kk] = *(ok ? a.portok + uint64_t(jp.y) * a.D + uint32_t(max(h.du[kk], 0)) : reinterpret_cast<const uint8_t*>(a.zero));
#pragma unroll
        for (int kk = 0; kk < KC; kk++)
          if (h.du[kk] >= 0 && pk[kk]) bits |= 1u << kk;
      }
      if (ok) s_il[t] = make_uint4(jp.x, jp.z, jp.w, bits);
    }
  }
  __syncthreads();
  // 16-byte stores of word pairs (store_row_pair): even rows of the class rows' window, aligned base
  const bool pair = a.WA % 2 == 0 && reinterpret_cast<uintptr_t>(a.A) % 16 == 0;
  if (w >= wend) return;  // no barrier below
  IdoRuns ir;
#pragma unroll
  for (uint32_t x = 0; x < IDO_MAX_RUNS; x++) {
    ir.off[x] = (wr.e[x] >> 5) * NS;
    ir.sh[x] = wr.e[x] & 31;
    ir.lo[x] = uint32_t(wr.m[x]);
    ir.hi[x] = uint32_t(wr.m[x] >> 32);
  }
  const uint64_t wmask = (w == a.W - 1) ? lastmask : ~0ull;
  uint64_t valid[KC];
  int32_t du[KC];
#pragma unroll
  for (int kk = 0; kk < KC; kk++) {
    const uint32_t k = k0 + kk;
    valid[kk] = 0;
    du[kk] = -2;
    if (EGRESS && UNI && k < a.K) {
      valid[kk] = wmask;
      du[kk] = a.udesc[k];
    } else if (EGRESS && k < a.K) {
      valid[kk] = a.VALID[uint64_t(k) * a.W + w];
      du[kk] = a.DESCW[uint64_t(k) * a.W + w];
    }
  }
  for (uint32_t q = 0; q < nr; q++) {
    const RepHead<KC>& h = s_rep[q];
    const uint32_t* sq = sB32 + q * EW32 * NS;
    uint64_t allow[KC];
    if (!EGRESS) {  // the destination's slots: per representative (block-uniform)
#pragma unroll
      for (int kk = 0; kk < KC; kk++) {
        du[kk] = k0 + kk < a.K ? h.du[kk] : -2;
        valid[kk] = du[kk] >= 0 ? wmask : 0ull;
      }
    }
    if (EGRESS && !UNI) {  // per destination word: its slots' descriptors' rows
#pragma unroll
      for (int kk = 0; kk < KC; kk++) {
        const uint32_t k = k0 + kk;
        allow[kk] = 0;
        if (k >= a.K) continue;
        if (du[kk] >= 0) {
          allow[kk] = expand_runs32(sq, uint32_t(du[kk]), ir);
        } else if (du[kk] == -1) {  // destinations with mixed job descriptors (rare)
          const uint64_t* dm = a.DM + uint64_t(k) * a.D * a.W + w;
          for (uint32_t d = 0; d < a.D; d++) allow[kk] |= expand_runs32(sq, d, ir) & dm[uint64_t(d) * a.W];
        }
      }
    } else {  // the block's KC slot rows (a slot not VALID is masked by valid[] at the store)
      uint32_t alo[KC], ahi[KC];
#pragma unroll
      for (int kk = 0; kk < KC; kk++) alo[kk] = ahi[kk] = 0;
#pragma unroll
      for (uint32_t x = 0; x < IDO_MAX_RUNS; x++) {
        if constexpr (KC == 4) {
          const uint4 b = *reinterpret_cast<const uint4*>(sq + ir.off[x]);
          ido_or_run(b.x, ir.sh[x], ir.lo[x], ir.hi[x], alo[0], ahi[0]);
          ido_or_run(b.y, ir.sh[x], ir.lo[x], ir.hi[x], alo[1], ahi[1]);
          ido_or_run(b.z, ir.sh[x], ir.lo[x], ir.hi[x], alo[2], ahi[2]);
          ido_or_run(b.w, ir.sh[x], ir.lo[x], ir.hi[x], alo[3], ahi[3]);
        } else {
#pragma unroll
          for (int kk = 0; kk < KC; kk++) ido_or_run(sq[ir.off[x] + kk], ir.sh[x], ir.lo[x], ir.hi[x], alo[kk], ahi[kk]);
        }
      }
#pragma unroll
      for (int kk = 0; kk < KC; kk++) allow[kk] = (uint64_t(ahi[kk]) << 32) | alo[kk];
    }
    // IP peers (ippeermatcher.go:43-50): per pod word through the PM rows, PEER_BATCH peers' words
    // loaded at once (no panic in IDO builds: the OR is order-free; the undecided check only ends
    // the walk early, once per batch)
    const uint32_t m = h.m, ms = stage_ip ? min(m, IDO_IPL) : 0u;
    const uint4* sl = s_il + q * IDO_IPL;
    uint32_t pend = stage_ip ? s_ipm[q] : 0u;  // staged peers with PM words in the block's words
    uint64_t undecided = ~0ull;  // (only ends the walk over unstaged peers early)
    if (!pend && m > ms) {
      undecided = 0;
#pragma unroll
      for (int kk = 0; kk < KC; kk++) undecided |= valid[kk] & ~allow[kk];
    }
    while (pend) {
      uint64_t pm[PEER_BATCH];
      uint32_t pbits[PEER_BATCH];
      ido_ip_loads_mask(a, sl, pend, w, pm, pbits);
      undecided = 0;
#pragma unroll
      for (int kk = 0; kk < KC; kk++) {
#pragma unroll
        for (uint32_t u = 0; u < PEER_BATCH; u++) {
          if (!pm[u]) continue;
          if (!EGRESS) allow[kk] |= ((pbits[u] >> kk) & 1u) ? pm[u] : 0ull;
          else if (du[kk] >= 0) allow[kk] |= ((pbits[u] >> du[kk]) & 1u) ? pm[u] : 0ull;
          else if (!UNI && du[kk] == -1) {  // destinations with mixed job descriptors (rare)
            uint64_t okm = 0;
            const uint64_t* dm = a.DM + uint64_t(k0 + kk) * a.D * a.W + w;
            for (uint32_t d = 0; d < a.D; d++)
              if ((pbits[u] >> d) & 1u) okm |= dm[uint64_t(d) * a.W];
            allow[kk] |= pm[u] & okm;
          }
        }
        undecided |= valid[kk] & ~allow[kk];
      }
      if (!undecided) break;
    }
    const uint4* il = a.ip_list + h.ipoff;
    for (uint32_t x0 = ms; x0 < (undecided ? m : 0u); x0 += PEER_BATCH) {  // peers past the staged ones
      uint64_t pm[PEER_BATCH];
      uint32_t port[PEER_BATCH], pbits[PEER_BATCH];
#pragma unroll
      for (uint32_t u = 0; u < PEER_BATCH; u++) {
        pm[u] = 0;
        port[u] = 0;
        pbits[u] = 0;
        if (x0 + u < m) {
          const uint4 jp = il[x0 + u];
          port[u] = jp.y;
          if (EGRESS && a.portbits) pbits[u] = a.portbits[jp.y];  // block-uniform: one scalar load per peer
          if (w >= jp.z && w <= jp.w)  // inside the peer's nonzero words
            pm[u] = a.PM[uint64_t(jp.x) * a.W + w] & cnz_mask(a.ip_cnz, a.W, jp.x, w);
        }
      }
      uint64_t undecided = 0;
#pragma unroll
      for (int kk = 0; kk < KC; kk++) {
#pragma unroll
        for (uint32_t u = 0; u < PEER_BATCH; u++) {
          if (!pm[u]) continue;
          // egress: the descriptor varies per destination word, so the byte table would cost a
          // vector load per (slot, peer); the bit row is a shift
          if (EGRESS && a.portbits && du[kk] >= 0) allow[kk] |= ((pbits[u] >> du[kk]) & 1u) ? pm[u] : 0ull;
          else if (!UNI) allow[kk] |= pm[u] & port_mask<EGRESS>(a, a.portok + uint64_t(port[u]) * a.D, du[kk], k0 + kk, w);
          else if (du[kk] >= 0 && a.portok[uint64_t(port[u]) * a.D + du[kk]]) allow[kk] |= pm[u];
        }
        undecided |= valid[kk] & ~allow[kk];
      }
      if (!undecided) break;
    }
    uint64_t* const rows = a.A + (uint64_t(h.arow) * a.K + k0) * a.WA;  // slot k0 of the class row
    const uint64_t off = w - a.w0;
    int kk = 0;
    if (pair)
#pragma unroll
      for (; kk + 1 < KC; kk += 2) {
        if (k0 + kk + 1 >= a.K) break;
        store_row_pair(rows + uint64_t(kk) * a.WA, rows + uint64_t(kk + 1) * a.WA, off, allow[kk] & valid[kk],
                       allow[kk + 1] & valid[kk + 1], threadIdx.x & 1);
      }
#pragma unroll
    for (int x = 0; x < KC; x++)
      if (x >= kk && k0 + x < a.K) rows[uint64_t(x) * a.WA + off] = allow[x] & valid[x];
  }
}
template <bool EGRESS, int KC, bool UNI = false>
__global__ __launch_bounds__(256) void k_class_rows_ido(RowArgs a) { class_rows_ido_blk<EGRESS, KC, UNI>(a, blockIdx.x, gridDim.x); }

}  // namespace cyc
