// dev_front.hpp — the fused front: launches A-E as concatenations of the per-block bodies above.
// Part of engine.hip's single translation unit (device bodies inline across stages, host helpers are
// static): included once, by engine.hip, in stage order.
#pragma once

namespace cyc {

// Fused front (cyc_set_option "front_fused", IDO builds): the front's ~15 kernels of two graph
// branches become 5 launches on ONE stream, each launch a concatenation of independent block
// ranges (every range calls the same per-block body as its stand-alone kernel, with its own
// block index and count).  A launch depends on the previous one only, so the graph needs no
// cross-stream edges (each cost ~10 us of join latency on the critical path) and both
// directions' blocks share every launch.
//   A: IP word spans reset | port table | slot words | selectors        (independent)
//   B: IP rows (both directions) | pod-peer identity sets (both) | membership in | membership eg
//      (membership dispatched first unless the IP rows fill the chip: FrontB::member_first)
//   C: class election in | eg           D: identity sets in | eg         E: class rows in | eg
struct FrontA {
  uint32_t nb[4];
  uint32_t* fill_p;
  uint64_t fill_n;
  uint32_t M, D, P, K, W, S, L;
  const DPortM* pms;
  const DPortEntry* pents;
  const DDesc* descs;
  uint8_t* portok;
  const int32_t* slot_desc;
  const uint8_t* slot_status;
  uint64_t* VALID;
  int32_t* DESCW;
  uint64_t* DM;
  const uint32_t *sel_off, *req_vals, *LVT, *sel_list;
  const DReq* dreqs;
  uint8_t* selres;
};
__global__ __launch_bounds__(256) void k_front_a(FrontA f) {
  uint32_t b = blockIdx.x;
  if (b < f.nb[0]) return fill_u32_blk(f.fill_p, f.fill_n, 0xFFFFFFFFu, b, f.nb[0]);
  b -= f.nb[0];
  if (b < f.nb[1]) return portok_blk(f.M, f.D, f.pms, f.pents, f.descs, f.portok, b, f.nb[1]);
  b -= f.nb[1];
  if (b < f.nb[2]) return slot_words_blk(f.P, f.K, f.W, f.D, f.slot_desc, f.slot_status, f.VALID, f.DESCW, f.DM, b, f.nb[2]);
  b -= f.nb[2];
  if (b < f.nb[3]) selectors_dense_blk(f.S, f.L, f.sel_off, f.dreqs, f.req_vals, f.LVT, f.selres, f.sel_list, b, f.nb[3]);
}

// Peer rows are built over a word window per direction: a source shard's ingress peers only over
// its sources' words (chunks [c0, c0 + nch)), everything else over all words.  Segment x of the IP
// rows and of the per-pod pod-peer rows is one direction's sub-list (target-row runs put both
// directions into segment 0: one window).
struct FrontB {
  uint32_t nb[13];      // IP rows x2 | pod-peer rows x2 (or identity sets, segment 2) | membership in | eg | port bits |
                        // port table | slot words (the last two: runs without launch A, enq_front_fused) |
                        // IP rows from address ranges x2 | IP rows as pod intervals x2
  uint32_t Rv[2];       // interval-built IP rows per segment (ip_rows_iv_blk)
  const DIPIv* vtests[2];
  const uint2* ipv_iv;
  uint32_t Rr[2];       // range-built IP rows per segment (ip_rows_range_blk)
  const DIPRange* rtests[2];
  const uint2* ipr_iv;
  const uint32_t* ipsort;
  FrontA pre;           // launch A's port table and slot-word arguments
  uint32_t bits_direct; // port bits from the matchers (pre.pms ...), not from the byte table
  uint32_t ip_grp;      // IP rows: peers per wave
  uint32_t pod_direct;  // PM builds with few pod-peer words: segments 2-3 = full pod-peer rows per pod
                        // (pod_rows_direct_blk), else segment 2 = identity sets (IDO)
  SelView sv;           // IDO identity sets: selector outcomes (SELRES or evaluated where used)
  uint32_t Rp[2];
  const uint32_t* plist[2];
  uint32_t pw0[2], pnw[2];  // per-pod pod-peer rows: word window per segment
  const uint32_t* pod_eid;
  uint32_t M, D;
  const uint8_t* portok;
  uint32_t* portbits;
  uint32_t Ri[2], P, W;
  const DIPTest* tests[2];
  uint32_t ic0[2], inch[2];  // IP rows: chunk window per segment
  const DIPItem* ip_items[2];  // IP rows as work items (non-null: segments 0-1 are items, a wave each)
  uint32_t n_ip_items[2];
  const uint32_t* ip_ilist;
  const DCidr* ip_ex;
  const DIP* pod_ip;
  const DWordIP* words;
  uint64_t* PM;
  uint32_t* rng;
  uint32_t* cnz;
  uint32_t E, EW, L;
  // identity sets (IDO builds) per segment x: its pod peers and identity word window
  uint32_t Ru_[2], ew0[2], new_[2];
  const uint32_t* pod_peers_u_[2];
  uint64_t* idob_[2];
  const uint2* grp_ns_[2];   // per group of PB_GROUP rows: the namespace range of its exact-namespace peers
  const uint4* pbrec_[2];    // per row its matcher records (pb_rec; null: the peers' chains)
  const uint2* word_ns;      // per egress identity word: its identities' namespace range
  const DPeer* peers;
  const uint8_t* selres;
  const uint32_t *id_ns, *id_nsls, *id_ls;
  MemberArgs ma[2];
  uint32_t member_wave[2];  // 1: a wave per identity (k_member_wave), 0: a thread per identity
  // membership blocks dispatched first (1) or after the pod-peer rows (0): few blocks, each a chain
  // of dependent loads, which first start at once instead of waiting for slots behind thousands of
  // short pod-row blocks (config #2: B 23.1 -> 16.5 us); behind a chip-full of IP rows they go last,
  // filling the tail instead of holding slots the IP rows need (config #4: first 66.6, last 64.1 us)
  uint32_t member_first;
};
__device__ __forceinline__ void front_b_member(const FrontB& f, uint32_t b) {
  if (b < f.nb[4]) {
    if (f.member_wave[0]) member_wave_blk(f.ma[0], b, f.nb[4]);
    else member_blk(f.ma[0], b, f.nb[4]);
    return;
  }
  b -= f.nb[4];
  if (f.member_wave[1]) member_wave_blk(f.ma[1], b, f.nb[5]);
  else member_blk(f.ma[1], b, f.nb[5]);
}
__global__ __launch_bounds__(256) void k_front_b(FrontB f) {
  uint32_t b = blockIdx.x;
  const uint32_t nm = f.nb[4] + f.nb[5];
  if (f.member_first) {
    if (b < nm) return front_b_member(f, b);
    b -= nm;
  }
#pragma unroll
  for (int x = 0; x < 2; x++) {
    if (b < f.nb[11 + x]) return ip_rows_iv_blk(f.Rv[x], f.W, f.vtests[x], f.ipv_iv, f.words, f.PM, f.rng, f.cnz, b, f.ic0[x], f.inch[x]);
    b -= f.nb[11 + x];
  }
#pragma unroll
  for (int x = 0; x < 2; x++) {
    if (b < f.nb[x]) {
      if (f.ip_items[x])
        return ip_rows_items_blk(f.n_ip_items[x], f.ip_items[x], f.ip_ilist, f.P, f.W, f.tests[x], f.ip_ex, f.pod_ip, f.words,
                                 f.PM, f.rng, f.cnz, b);
      return ip_rows_fast_blk(f.Ri[x], f.P, f.W, f.tests[x], f.ip_ex, f.pod_ip, f.words, f.PM, f.rng, f.cnz, b, f.nb[x], f.ip_grp,
                              f.ic0[x], f.inch[x]);
    }
    b -= f.nb[x];
  }
#pragma unroll
  for (int x = 0; x < 2; x++) {
    if (b < f.nb[2 + x]) {
      if (f.pod_direct)
        return pod_rows_direct_blk<false>(f.Rp[x], f.P, f.W, f.plist[x], f.peers, f.sv, f.pod_eid, f.id_ns, f.id_nsls,
                                          f.id_ls, f.PM, nullptr, b, f.nb[2 + x], f.pw0[x], f.pnw[x]);
      return peer_bits_blk(f.Ru_[x], f.E, f.EW, f.pod_peers_u_[x], f.peers, f.sv, f.id_ns, f.id_nsls, f.id_ls, f.idob_[x], b,
                           f.nb[2 + x], f.ew0[x], f.new_[x], f.grp_ns_[x], f.word_ns, f.pbrec_[x]);
    }
    b -= f.nb[2 + x];
  }
  if (!f.member_first) {
    if (b < nm) return front_b_member(f, b);
    b -= nm;
  }
  if (b < f.nb[6]) {  // for the identity sets and the class rows
    if (f.bits_direct) return portbits_direct_blk(f.M, f.D, f.pre.pms, f.pre.pents, f.pre.descs, f.portbits, b);
    return portbits_blk(f.M, f.D, f.portok, f.portbits, b);
  }
  b -= f.nb[6];
  if (b < f.nb[7]) return portok_blk(f.pre.M, f.pre.D, f.pre.pms, f.pre.pents, f.pre.descs, f.pre.portok, b, f.nb[7]);
  b -= f.nb[7];
  if (b < f.nb[8])
    return slot_words_blk(f.pre.P, f.pre.K, f.pre.W, f.pre.D, f.pre.slot_desc, f.pre.slot_status, f.pre.VALID, f.pre.DESCW,
                          f.pre.DM, b, f.nb[8]);
  b -= f.nb[8];
#pragma unroll
  for (int x = 0; x < 2; x++) {
    if (b < f.nb[9 + x])
      return ip_rows_range_blk(f.Rr[x], f.W, f.rtests[x], f.ipr_iv, f.ipsort, f.PM, f.rng, f.cnz, b, f.ic0[x], f.inch[x]);
    b -= f.nb[9 + x];
  }
}

// Pod-peer rows from posting lists: a pod selector that is ONE requirement `k = v` or `k in (v0,
// v1)` (matchLabels, the common shape) matches exactly the pods listed under (k, v) in the host's
// label postings, so its row is built from those few pods instead of testing every pod: block =
// one such peer; the row is assembled in LDS PR_POST_WORDS words at a time (each pod of the
// postings whose namespace the peer's namespace matcher accepts sets its bit with an LDS atomic
// OR), then stored chunk-dense with span and chunk masks (pod_chunk_store).  Cost ~ postings +
// nonzero chunks, not pods.
constexpr uint32_t PR_POST_WORDS = 1024;  // 16 chunks of the row per LDS pass (8 KB)
__device__ __forceinline__ void pod_rows_post_blk(uint32_t P, uint32_t W, const uint32_t* __restrict__ plist,
                                                  const DPeer* __restrict__ peers, const SelView& sv,
                                                  const uint4* __restrict__ req_post, const uint32_t* __restrict__ post_pods,
                                                  const uint32_t* __restrict__ pod_ns, const uint32_t* __restrict__ pod_nsls,
                                                  uint64_t* __restrict__ PM, uint32_t* __restrict__ rng, uint32_t* __restrict__ cnz,
                                                  uint32_t bid_, uint32_t c0, uint32_t nch) {
  __shared__ unsigned long long s_row[PR_POST_WORDS];
  const uint32_t j = plist[bid_];
  const DPeer pr = peers[j];
  const uint4 pp = req_post[sv.sel_off[pr.podsel]];  // (offset, count) of value 0, then of value 1
  // chunks [c0, c0 + nch) of the row (a source shard's ingress peers: the chunks of its word window)
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, chunks = c0 + nch;
  for (uint32_t w0 = c0 * 64; w0 < min(W, chunks * 64); w0 += PR_POST_WORDS) {
    for (uint32_t x = threadIdx.x; x < PR_POST_WORDS; x += blockDim.x) s_row[x] = 0;
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < pp.y + pp.w; e += blockDim.x) {
      const uint32_t q = post_pods[e < pp.y ? pp.x + e : pp.z + (e - pp.y)];
      const uint32_t w = q >> 6;
      if (w < w0 || w >= w0 + PR_POST_WORDS) continue;
      bool ok = pr.nskind == 1;  // podpeermatcher.go:21-28: the namespace matcher
      if (pr.nskind == 0) ok = pod_ns[q] == pr.nsval;
      else if (pr.nskind == 2) ok = sel_at(sv, pr.nsval, pod_nsls[q]) == 1;
      if (ok) atomicOr(&s_row[w - w0], 1ull << (q & 63));
    }
    __syncthreads();
    for (uint32_t c = w0 / 64 + wave; c < min(chunks, (w0 + PR_POST_WORDS) / 64); c += blockDim.x >> 6)
      pod_chunk_store(j, c, W, lane, c * 64 + lane < W ? s_row[c * 64 + lane - w0] : 0ull, PM, rng, cnz);
    __syncthreads();  // s_row is cleared for the next pass
  }
}

// Launch C also carries PM builds' sparse pod-peer rows (they need only launch A's selector table
// and precede the class rows): the light class election keeps them off launch B, whose IP rows and
// membership would otherwise run at the pod rows' register budget (occupancy 8 -> 5-7).
struct FrontC {
  uint32_t nb[6];  // class election in | eg | sparse pod-peer rows x2 | posting-built rows x2
  MemberArgs ma[2];
  uint32_t* class_of[2];
  // sparse pod-peer rows (pod_rows_sparse_blk over plist, then pod_rows_post_blk over plist_post),
  // one segment per word window (ingress peers of a source shard / the rest)
  uint32_t Rp[2], P, W, pr_grp;
  const uint32_t* plist[2];
  uint32_t c0[2], nch[2];
  const DPeer* peers;
  SelView sv;
  const uint32_t *pod_ns, *pod_nsls, *pod_ls;
  const DWordNS* nsw;  // per word, then per chunk: namespace ranges
  uint64_t* PM;
  uint32_t *rng, *cnz;
  const uint32_t* plist_post[2];  // pod peers whose rows come from label postings (pod_rows_post_blk)
  const uint4* req_post;
  const uint32_t* post_pods;
};
__global__ __launch_bounds__(256) void k_front_c(FrontC f) {
  uint32_t b = blockIdx.x;
  if (b < f.nb[0]) return classify_blk(f.ma[0], f.class_of[0], b, f.nb[0]);
  b -= f.nb[0];
  if (b < f.nb[1]) return classify_blk(f.ma[1], f.class_of[1], b, f.nb[1]);
  b -= f.nb[1];
#pragma unroll
  for (int x = 0; x < 2; x++) {
    if (b < f.nb[2 + x])
      return pod_rows_sparse_blk(f.Rp[x], f.P, f.W, f.plist[x], f.peers, f.sv, f.pod_ns, f.pod_nsls, f.pod_ls, f.nsw, f.PM, f.rng,
                                 f.cnz, f.pr_grp, b, f.c0[x], f.nch[x]);
    b -= f.nb[2 + x];
  }
#pragma unroll
  for (int x = 0; x < 2; x++) {
    if (b < f.nb[4 + x])
      return pod_rows_post_blk(f.P, f.W, f.plist_post[x], f.peers, f.sv, f.req_post, f.post_pods, f.pod_ns, f.pod_nsls, f.PM, f.rng,
                               f.cnz, b, f.c0[x], f.nch[x]);
    b -= f.nb[4 + x];
  }
}

struct FrontRows {
  uint32_t nb[2];
  RowArgs ra[2];
};
__global__ __launch_bounds__(256) void k_front_d(FrontRows f) {
  const uint32_t b = blockIdx.x;
  if (b < f.nb[0]) class_ident_blk<false, CI_G>(f.ra[0], b, f.nb[0]);
  else class_ident_blk<true, CI_G>(f.ra[1], b - f.nb[0], f.nb[1]);
}
// PM builds (pod-peer words from materialised rows): the class rows, egress blocks first
template <bool WAVE>
__global__ __launch_bounds__(256) void k_front_d_pm(FrontRows f) {
  __shared__ PlShared sh;
  const uint32_t b = blockIdx.x;
  if (b < f.nb[1]) class_rows_pl_blk<true, WAVE>(f.ra[1], sh, b, f.nb[1]);
  else class_rows_pl_blk<false, WAVE>(f.ra[0], sh, b - f.nb[1], f.nb[0]);
}

// egress blocks first: they are the slower ones (per-destination port masks), so the launch's
// tail is made of the shorter ingress blocks (4 job slots per thread: profiles/r01_front_e_kc_ab.txt)
constexpr int E_KC = 4;  // job slots per thread in the IDO class rows of the fused front
// Launch E as one kernel when the egress rows take the one-descriptor-per-slot form (UNI): both
// bodies then stay near 60 VGPRs, so the fused launch keeps their occupancy and saves a launch.
__global__ __launch_bounds__(256) void k_front_e_uni(FrontRows f) {
  uint32_t b = blockIdx.x;
  const bool eg = b < f.nb[1];
  if (!eg) b -= f.nb[1];
  if (eg) class_rows_ido_blk<true, E_KC, true>(f.ra[1], b, f.nb[1]);
  else class_rows_ido_blk<false, E_KC>(f.ra[0], b, f.nb[0]);
}

}  // namespace cyc
