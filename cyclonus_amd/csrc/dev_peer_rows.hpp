// dev_peer_rows.hpp — peer rows: pod-peer rows and identity sets, IP rows (per word, as work items, from address ranges).
// Part of engine.hip's single translation unit (device bodies inline across stages, host helpers are
// static): included once, by engine.hip, in stage order.
#pragma once

namespace cyc {

// Pod peers depend on a peer pod only through its (namespace, labels) identity, so they are
// evaluated once per (pod peer, egress identity) -> IDO u8 [Rpod][E] ...
__global__ void k_peer_ident(uint32_t Rp, uint32_t E, const uint32_t* __restrict__ pod_peers, const DPeer* __restrict__ peers,
                             const uint8_t* __restrict__ selres, uint32_t L, const uint32_t* __restrict__ id_ns,
                             const uint32_t* __restrict__ id_nsls, const uint32_t* __restrict__ id_ls,
                             uint8_t* __restrict__ ido) {
  uint64_t n = uint64_t(Rp) * E;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    uint32_t p = uint32_t(i / E), e = uint32_t(i % E);
    DPeer pr = peers[pod_peers[p]];
    ido[i] = uint8_t(pod_peer_outcome(pr, selres, L, id_ns[e], id_nsls[e], id_ls[e]));
  }
}

// ... then expanded to packed pod rows through each 64-pod word's identity runs (word_off /
// run_e / run_mask; pods of one identity are usually contiguous, so a word holds 1-2 runs).
template <bool ERR>
__global__ __launch_bounds__(256) void k_pod_rows(uint32_t Rp, uint32_t E, uint32_t W, const uint32_t* __restrict__ pod_peers,
                                                  const uint8_t* __restrict__ ido, const uint32_t* __restrict__ word_off,
                                                  const uint32_t* __restrict__ run_e, const uint64_t* __restrict__ run_mask,
                                                  uint64_t* __restrict__ PM, uint64_t* __restrict__ ER, uint32_t w0, uint32_t nw) {
  uint32_t chunks = (nw + 255) / 256;
  uint32_t p = blockIdx.x / chunks;
  uint32_t w = w0 + (blockIdx.x % chunks) * 256 + threadIdx.x;
  if (p >= Rp || w >= w0 + nw) return;
  const uint8_t* row = ido + uint64_t(p) * E;
  uint64_t m = 0, e = 0;
  for (uint32_t x = word_off[w]; x < word_off[w + 1]; x++) {
    uint8_t o = row[run_e[x]];
    uint64_t mk = run_mask[x];
    m |= o == 1 ? mk : 0ull;
    if (ERR) e |= o == 2 ? mk : 0ull;
  }
  uint64_t j = pod_peers[p];
  PM[j * W + w] = m;
  if (ERR) ER[j * W + w] = e;
}

struct DWordNS {
  uint32_t lo, hi;  // namespace string ids of the word's (chunk's) pods: min, max
  uint32_t nsls;    // their namespace label set when lo == hi
  uint32_t pad;
};

// Pod-peer rows straight from each pod's egress identity: one wave per (pod peer, 64-pod word),
// lane = pod, one ballot per word.  Used when identities are about as many as pods (every pod
// labelled apart, e.g. a `pod: <name>` label): then the identity-space outcomes cost as much as
// this and the run expansion above loops over up to 64 runs per word.
// Words [w0, w0 + nw) of each row (a source shard's ingress peers: its word window).
constexpr uint32_t PR_DIRECT_G = 4;  // pod peers per wave of the direct pod-peer rows
// Wave = (PR_DIRECT_G pod peers, one 64-pod word), lane = pod: the word's pod identities (pod ->
// identity -> namespace, namespace labels, labels) are loaded once for the group, then every
// peer's two matcher bytes at once, one ballot per peer.
__host__ __device__ inline uint64_t pod_direct_waves(uint32_t Rp, uint32_t nw) {
  return uint64_t((Rp + PR_DIRECT_G - 1) / PR_DIRECT_G) * nw;
}
// No panic possible (the fused front): both matchers through a SelView — the dense selector table, or
// selectors evaluated here (one-requirement records: one label-table gather each) when the front builds
// no table (sel_lazy), so a PM build with full pod-peer rows needs no launch A.
__device__ __forceinline__ uint32_t pod_peer_match_sv(const DPeer& pr, const SelView& sv, uint32_t ns, uint32_t nsls, uint32_t ls) {
  const bool nsel = pr.nskind == 2, psel = pr.podsel != CYC_ALL;
  const uint32_t rn = nsel ? sel_at(sv, pr.nsval, nsls) : 1u;
  const uint32_t rp = psel ? sel_at(sv, pr.podsel, ls) : 1u;
  if (pr.nskind == 0) return ns == pr.nsval && rp == 1 ? 1u : 0u;
  return rn == 1 && rp == 1 ? 1u : 0u;
}
template <bool ERR>
__device__ __forceinline__ void pod_rows_direct_blk(uint32_t Rp, uint32_t P, uint32_t W,
                                                         const uint32_t* __restrict__ pod_peers,
                                                         const DPeer* __restrict__ peers, const SelView& sv,
                                                         const uint32_t* __restrict__ pod_eid,
                                                         const uint32_t* __restrict__ id_ns, const uint32_t* __restrict__ id_nsls,
                                                         const uint32_t* __restrict__ id_ls, uint64_t* __restrict__ PM,
                                                         uint64_t* __restrict__ ER, uint32_t bid_, uint32_t nblk_, uint32_t w0,
                                                         uint32_t nw) {
  const uint32_t lane = threadIdx.x & 63, gw = __builtin_amdgcn_readfirstlane(bid_ * 4 + (threadIdx.x >> 6));  // wave-uniform
  const uint32_t g = gw / nw, w = w0 + (gw - g * nw), p0 = g * PR_DIRECT_G;
  if (p0 >= Rp) return;
  uint32_t j[PR_DIRECT_G];
  DPeer pr[PR_DIRECT_G];
#pragma unroll
  for (uint32_t u = 0; u < PR_DIRECT_G; u++) {
    j[u] = pod_peers[min(p0 + u, Rp - 1)];
    pr[u] = peers[j[u]];
  }
  const uint32_t q = w * 64 + lane;
  const uint32_t e = pod_eid[min(q, P - 1)];  // (clamped: no load inside a branch)
  const uint32_t ns = id_ns[e], nsls = id_nsls[e], ls = id_ls[e];
  uint32_t o[PR_DIRECT_G];
#pragma unroll
  for (uint32_t u = 0; u < PR_DIRECT_G; u++)
    o[u] = ERR || sv.selres ? pod_peer_outcome(pr[u], sv.selres, sv.L, ns, nsls, ls) : pod_peer_match_sv(pr[u], sv, ns, nsls, ls);
#pragma unroll
  for (uint32_t u = 0; u < PR_DIRECT_G; u++) {
    if (p0 + u >= Rp) break;  // wave-uniform
    const uint32_t ou = q < P ? o[u] : 0u;
    const uint64_t m = __ballot(ou == 1);
    const uint64_t er = ERR ? __ballot(ou == 2) : 0ull;
    if (lane == 0) {
      PM[uint64_t(j[u]) * W + w] = m;
      if (ERR) ER[uint64_t(j[u]) * W + w] = er;
    }
  }
}
template <bool ERR>
__global__ __launch_bounds__(256) void k_pod_rows_direct(uint32_t Rp, uint32_t P, uint32_t W,
                                                         const uint32_t* __restrict__ pod_peers,
                                                         const DPeer* __restrict__ peers, const uint8_t* __restrict__ selres,
                                                         uint32_t L, const uint32_t* __restrict__ pod_eid,
                                                         const uint32_t* __restrict__ id_ns, const uint32_t* __restrict__ id_nsls,
                                                         const uint32_t* __restrict__ id_ls, uint64_t* __restrict__ PM,
                                                         uint64_t* __restrict__ ER, uint32_t w0, uint32_t nw) {
  SelView sv{};
  sv.selres = selres;
  sv.L = L;
  pod_rows_direct_blk<ERR>(Rp, P, W, pod_peers, peers, sv, pod_eid, id_ns, id_nsls, id_ls, PM, ER, blockIdx.x, gridDim.x, w0, nw);
}

// Pod-peer rows of the fused front on PM builds (no panic possible), stored sparse, 64-word chunks
// at a time with lane = pod word (block shapes: pod_rows_sparse_blk).  The namespace
// matcher runs first (podpeermatcher.go:21-28) and decides most words without looking at a pod:
// an exact namespace (nskind 0: the policy's own) matches only the words holding that namespace's
// pods — pods of a namespace are normally listed together, so a chunk whose namespace range
// misses it is skipped whole — and a namespace selector is ONE lookup for a word whose pods share
// a namespace.  The remaining words are evaluated a pod per lane, PR_WB words at once per wave
// (their loads in flight together).  Rows are stored chunk-dense with their nonzero word span and chunk masks,
// exactly like the IP rows (ip_row_word), so the class rows skip their zero chunks: with every pod
// labelled apart (identities ~ pods) most pod-peer rows are a namespace's worth of words.
constexpr uint32_t PR_WB = 8;  // words evaluated at once per wave

// Word masks of pod peer pr over chunk `chunk` (this lane's word w): the namespace outcome per word
// first, then a pod per lane for the words it leaves open — only those of rank part, part + parts,
// ... among them (a chunk's words split over `parts` waves).
__device__ __forceinline__ uint64_t pod_chunk_words(const DPeer& pr, const SelView& sv, uint32_t P, uint32_t W, uint32_t chunk,
                                                    uint32_t lane, uint32_t part, uint32_t parts,
                                                    const uint32_t* __restrict__ pod_ns, const uint32_t* __restrict__ pod_nsls,
                                                    const uint32_t* __restrict__ pod_ls, const DWordNS* __restrict__ nsw) {
  const uint32_t w = chunk * 64 + lane;
  const bool valid = w < W;
  DWordNS wn{0xFFFFFFFFu, 0u, 0u, 0u};
  if (valid) wn = nsw[w];
  uint32_t nsm = 0;  // the word's namespace outcome: 0 no pod, 1 every pod, 2 per pod
  if (valid) {
    if (pr.nskind == 1) nsm = 1;
    else if (pr.nskind == 0) nsm = (pr.nsval < wn.lo || pr.nsval > wn.hi) ? 0u : (wn.lo == wn.hi ? 1u : 2u);
    else nsm = wn.lo == wn.hi ? (sel_at(sv, pr.nsval, wn.nsls) == 1 ? 1u : 0u) : 2u;
  }
  uint64_t mine = 0;
  if (part == 0 && nsm == 1 && pr.podsel == CYC_ALL) mine = (w == W - 1 && P % 64) ? ((1ull << (P % 64)) - 1) : ~0ull;
  uint64_t todo = __ballot(nsm == 2 || (nsm == 1 && pr.podsel != CYC_ALL));
  // a pod selector of ONE requirement with <= 2 values (matchLabels {k: v}, the common shape) is
  // held in scalar registers: a batch's PLVT loads then all go out together instead of one
  // requirement walk (dependent loads) per word; other shapes walk the requirements (sel_at_pod)
  // or, with the dense table, gather SELRES through the pod's label set
  uint32_t r_op = REQ_INVALID, r_key = 0, r_v0 = 0, r_v1 = 0, r_vc = 0;
  if (pr.podsel != CYC_ALL && sv.sel_off[pr.podsel + 1] - sv.sel_off[pr.podsel] == 1) {
    const DReq q1 = sv.dreqs[sv.sel_off[pr.podsel]];
    if (q1.op != REQ_INVALID && q1.vcnt <= 2) {
      r_op = q1.op;
      r_key = q1.key;
      r_vc = q1.vcnt;
      r_v0 = q1.vcnt > 0 ? sv.req_vals[q1.voff] : 0u;
      r_v1 = q1.vcnt > 1 ? sv.req_vals[q1.voff + 1] : 0u;
    }
  }
  const bool one = r_op != REQ_INVALID;
  if (parts > 1) {  // this wave's share
    uint64_t sub = 0;
    for (uint32_t r = 0; todo; r++, todo &= todo - 1)
      if (r % parts == part) sub |= todo & (~todo + 1);
    todo = sub;
  }
  while (todo) {
    uint32_t wl[PR_WB], nsv[PR_WB], q[PR_WB], xv[PR_WB];
    bool live[PR_WB];
#pragma unroll
    for (uint32_t u = 0; u < PR_WB; u++) {
      wl[u] = 64;
      if (todo) {
        wl[u] = __ffsll((unsigned long long)todo) - 1;
        todo &= todo - 1;
      }
      q[u] = (chunk * 64 + wl[u]) * 64 + lane;
      live[u] = wl[u] < 64 && q[u] < P;
      // the pod's namespace (exact matcher) or namespace label set (selector), when needed
      nsv[u] = live[u] && pr.nskind != 1 ? (pr.nskind == 0 ? pod_ns[q[u]] : pod_nsls[q[u]]) : 0u;
      // the selector's key value of the pod (one requirement), or the pod's label set (dense table,
      // or no PLVT: the selector is then evaluated on the label set)
      xv[u] = 0;
      if (live[u] && pr.podsel != CYC_ALL) {
        if (one) xv[u] = sv.PLVT ? sv.PLVT[uint64_t(r_key) * P + q[u]] : sv.LVT[uint64_t(r_key) * sv.L + pod_ls[q[u]]];
        else if (sv.selres || !sv.PLVT) xv[u] = pod_ls[q[u]];
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < PR_WB; u++) {
      // no panic is possible here: outcomes are 0 / 1 only, so both matchers can be evaluated
      bool a = pr.nskind == 1 || (pr.nskind == 0 && nsv[u] == pr.nsval);
      if (pr.nskind == 2) a = live[u] && sel_at(sv, pr.nsval, nsv[u]) == 1;
      bool b = pr.podsel == CYC_ALL;
      if (!b && live[u])
        b = one ? req_holds(r_op, xv[u], r_v0, r_v1, r_vc)
                : (sv.selres ? sv.selres[uint64_t(pr.podsel) * sv.L + xv[u]]
                   : sv.PLVT ? sel_at_pod(sv, pr.podsel, q[u]) : sel_at(sv, pr.podsel, xv[u])) == 1;
      const uint64_t m = __ballot(live[u] && a && b);
      if (lane == wl[u]) mine = m;
    }
  }
  return mine;
}

// One wave stores chunk `chunk` of peer j's row (v = this lane's word) chunk-dense, with its
// nonzero flag, and widens the row's word span and nonzero-chunk mask.
__device__ __forceinline__ void pod_chunk_store(uint32_t j, uint32_t chunk, uint32_t W, uint32_t lane, uint64_t v,
                                                uint64_t* __restrict__ PM, uint32_t* __restrict__ rng, uint32_t* __restrict__ cnz) {
  const uint32_t w = chunk * 64 + lane;
  const uint64_t nzc = __ballot(v != 0);
  if (nzc && w < W) PM[uint64_t(j) * W + w] = v;  // a nonzero chunk stores all its words
  if (lane == 0) {
    cnz[uint64_t(j) * ((W + 63) / 64) + chunk] = nzc ? 1u : 0u;
    if (nzc) {
      atomicMin(&rng[4 * j], chunk * 64 + __ffsll((unsigned long long)nzc) - 1);
      atomicMin(&rng[4 * j + 1], ~(chunk * 64 + 63 - __clzll((long long)nzc)));
      if (chunk < 64) atomicAnd(reinterpret_cast<unsigned long long*>(rng) + 2 * j + 1, ~(1ull << chunk));
    }
  }
}

// grp > 1: block = (grp pod peers, 4 chunks), a wave per chunk walking the group's peers (many
// peers: the grid is large anyway).  grp == 1: block = (pod peer, 4 chunks) taken one chunk at a
// time, each chunk's open words split over the 4 waves and met in LDS (few peers with dense rows:
// config #2 26 us, where a wave per chunk leaves 3 waves per peer and takes 100 us).
__device__ __forceinline__ void pod_rows_sparse_blk(uint32_t Rp, uint32_t P, uint32_t W, const uint32_t* __restrict__ plist,
                                                    const DPeer* __restrict__ peers, const SelView& sv,
                                                    const uint32_t* __restrict__ pod_ns,
                                                    const uint32_t* __restrict__ pod_nsls, const uint32_t* __restrict__ pod_ls,
                                                    const DWordNS* __restrict__ nsw, uint64_t* __restrict__ PM,
                                                    uint32_t* __restrict__ rng, uint32_t* __restrict__ cnz, uint32_t grp,
                                                    uint32_t bid_, uint32_t c0, uint32_t nch) {
  __shared__ uint64_t s_m[4][64];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t chunks = (W + 63) / 64, cb = (nch + 3) / 4;  // chunks [c0, c0 + nch) of each row
  const uint32_t x0 = (bid_ / cb) * grp;
  if (x0 >= Rp) return;  // whole block
  if (grp > 1) {
    const uint32_t chunk = __builtin_amdgcn_readfirstlane(c0 + (bid_ % cb) * 4 + wave);
    if (chunk >= c0 + nch) return;
    const DWordNS ck = nsw[W + chunk];
    for (uint32_t x = x0; x < min(Rp, x0 + grp); x++) {
      const uint32_t j = plist[x];
      const DPeer pr = peers[j];
      if (pr.nskind == 0 && (pr.nsval < ck.lo || pr.nsval > ck.hi)) {  // no pod of the namespace here
        if (lane == 0) cnz[uint64_t(j) * chunks + chunk] = 0;
        continue;
      }
      const uint64_t v = pod_chunk_words(pr, sv, P, W, chunk, lane, 0, 1, pod_ns, pod_nsls, pod_ls, nsw);
      pod_chunk_store(j, chunk, W, lane, v, PM, rng, cnz);
    }
    return;
  }
  const uint32_t j = plist[x0];
  const DPeer pr = peers[j];
  for (uint32_t ci = 0; ci < 4; ci++) {
    const uint32_t chunk = c0 + (bid_ % cb) * 4 + ci;  // block-uniform
    if (chunk >= c0 + nch) break;
    const DWordNS ck = nsw[W + chunk];
    if (pr.nskind == 0 && (pr.nsval < ck.lo || pr.nsval > ck.hi)) {
      if (threadIdx.x == 0) cnz[uint64_t(j) * chunks + chunk] = 0;
      continue;
    }
    s_m[wave][lane] = pod_chunk_words(pr, sv, P, W, chunk, lane, wave, 4, pod_ns, pod_nsls, pod_ls, nsw);
    __syncthreads();
    if (wave == 0) pod_chunk_store(j, chunk, W, lane, s_m[0][lane] | s_m[1][lane] | s_m[2][lane] | s_m[3][lane], PM, rng, cnz);
    __syncthreads();  // s_m is reused by the next chunk
  }
}

// IP peers depend on each pod's own address: one wave per 64-pod word (one lane per pod).  A
// block owns IPB_BATCH IP peers: their CIDR and except records (host-flattened, in evaluation
// order) are staged once into LDS, then every wave tests its lane's IP (loaded once) against
// the whole batch with LDS-broadcast reads — no dependent global loads in the inner loop.
constexpr uint32_t IPB_BATCH = 64;
constexpr uint32_t IPB_EX_LDS = 192;  // except records staged per batch (more => global reads)
struct DIPTest {
  uint32_t peer, exoff, excnt, pad;  // exoff: into ip_ex (flattened DCidr list)
  DCidr cidr;
};

// Words [w0, w0 + nw) of the rows only (a source shard's ingress peers: the shard's word window).
template <bool ERR>
__global__ __launch_bounds__(256) void k_ip_rows(uint32_t Ri, uint32_t P, uint32_t W, const DIPTest* __restrict__ tests,
                                                 const DCidr* __restrict__ ip_ex, const DIP* __restrict__ pod_ip,
                                                 uint64_t* __restrict__ PM, uint64_t* __restrict__ ER, uint32_t batch,
                                                 uint32_t w0, uint32_t nw) {
  __shared__ DIPTest s_t[IPB_BATCH];
  __shared__ DCidr s_ex[IPB_EX_LDS];
  const uint32_t wchunks = (nw + 3) / 4;
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t w = w0 + (blockIdx.x % wchunks) * 4 + wave;
  const uint32_t r0 = (blockIdx.x / wchunks) * batch;
  const uint32_t nr = min(Ri - r0, batch);
  const uint32_t ex0 = tests[r0].exoff;
  const uint32_t nex = tests[r0 + nr - 1].exoff + tests[r0 + nr - 1].excnt - ex0;
  for (uint32_t t = threadIdx.x; t < nr; t += blockDim.x) s_t[t] = tests[r0 + t];
  for (uint32_t t = threadIdx.x; t < min(nex, IPB_EX_LDS); t += blockDim.x) s_ex[t] = ip_ex[ex0 + t];
  __syncthreads();
  if (w >= w0 + nw) return;
  const uint32_t q = w * 64 + lane;
  DIP ip{};
  if (q < P) ip = pod_ip[q];
  const bool live = q < P;
  for (uint32_t r = 0; r < nr; r++) {
    const DIPTest& t = s_t[r];
    // ipaddress.go:22-40: CIDR parse, IP parse, contains, then each except in order
    uint32_t o;
    if (!t.cidr.valid || !ip.valid) o = 2;
    else if (!cidr_contains(t.cidr, ip)) o = 0;
    else {
      o = 1;
      for (uint32_t e = 0; e < t.excnt; e++) {
        uint32_t xi = t.exoff + e - ex0;
        const DCidr& x = xi < IPB_EX_LDS ? s_ex[xi] : ip_ex[t.exoff + e];
        if (!x.valid) {
          o = 2;
          break;
        }
        if (cidr_contains(x, ip)) {
          o = 0;
          break;
        }
      }
    }
    if (!live) o = 0;
    uint64_t m = __ballot(o == 1);
    uint64_t e = ERR ? __ballot(o == 2) : 0ull;
    if (lane == 0) {
      PM[uint64_t(t.peer) * W + w] = m;
      if (ERR) ER[uint64_t(t.peer) * W + w] = e;
    }
  }
}

// Fast IP rows (no-panic inputs: every pod address parses).  One wave = (IP peer, 64
// consecutive words); lane = word.  A CIDR (and each except) is an address interval of its
// family, so a word is decided per family from the [min, max] address of its pods of that family
// (an IPv4 network never contains an IPv6 address and vice versa, ippeermatcher / net.Contains):
// fully outside, fully inside (then each except of the family fully out / fully in), or mixed.
// Only mixed words fall back to the lane-per-pod test.  Pods numbered in address order (the
// usual case: addresses handed out per namespace) leave almost no mixed words.
struct DWordIP {
  uint32_t min4, max4;         // over the word's IPv4 pods
  uint64_t m4, m6;             // bits of the IPv4 / IPv6 pods
  uint32_t min6[4], max6[4];   // over the word's IPv6 pods (big-endian 128-bit)
  // per family (v4: bits 0-7, v6: bits 8-15): bit 7 set when the family's pods of the word have
  // AFFINE addresses — the pod in lane i holds min + (i - first), first = bits 0-5 = the lowest lane of
  // the family (addresses handed out in pod order); a network then covers a lane range computed from
  // its bounds, no per-pod address load (word records of chunks: 0)
  uint32_t aff, pad;
};
static_assert(sizeof(DWordIP) == 64, "DWordIP is one 64-byte record");

__device__ __forceinline__ bool lt128(const uint32_t* a, const uint32_t* b) {
  for (int i = 0; i < 4; i++)
    if (a[i] != b[i]) return a[i] < b[i];
  return false;
}

// Position of the interval [mn, mx] against the network c of the same family:
// 0 disjoint, 1 inside, 2 straddles.
__device__ __forceinline__ uint32_t span_vs_cidr4(uint32_t mn, uint32_t mx, const DCidr& c) {
  const uint32_t lo = c.net[3] & c.mask[3], hi = lo | ~c.mask[3];
  if (mx < lo || mn > hi) return 0;
  return (mn >= lo && mx <= hi) ? 1 : 2;
}
__device__ __forceinline__ uint32_t span_vs_cidr6(const uint32_t* mn, const uint32_t* mx, const DCidr& c) {
  uint32_t lo[4], hi[4];
  for (int i = 0; i < 4; i++) {
    lo[i] = c.net[i] & c.mask[i];
    hi[i] = lo[i] | ~c.mask[i];
  }
  if (lt128(mx, lo) || lt128(hi, mn)) return 0;
  return (!lt128(mn, lo) && !lt128(hi, mx)) ? 1 : 2;
}

// Also records each IP peer's nonzero word span in rng[4 * peer] (first word) and
// rng[4 * peer + 1] (~last word), both atomicMin'd from 0xFFFFFFFF, and the complement of its
// nonzero-chunk mask in the u64 at rng + 4 * peer + 2 (atomicAnd'd from ~0; chunks < 64 — the
// wave-per-chunk class rows test an entry against their chunk with it): CIDRs are address ranges and
// pods of a namespace have neighbouring addresses, so a peer's row is mostly zero words the
// class rows can skip without loading them.  Rows are stored chunk-dense: cnz[peer][chunk] (one
// u32 per 64-word chunk, written by the chunk's wave) is 1 if the chunk has a nonzero word; a chunk with
// none stores no PM word at all, any other chunk stores all 64.  Readers issue the PM and cnz loads
// together and drop the PM word of an all-zero chunk, so the zero chunks — most of a row — cost
// no HBM writes.
// Lanes of a word whose pods of family `v4` hold addresses in network c, when those addresses are
// affine in the lane (DWordIP::aff): lane i holds min + (i - first), so the network's bounds
// [lo, hi] give the lane range [first + (lo - min), first + (hi - min)] clamped to the word.  Both
// differences are taken only where the bound lies in [min, max] (a span under 64), so 64-bit
// arithmetic on the low words is exact for IPv6 too.
__device__ __forceinline__ uint64_t lanes_in_range(uint32_t first, uint32_t span, uint64_t lo_off, bool lo_below, bool lo_above,
                                                   uint64_t hi_off, bool hi_below, bool hi_above) {
  // lo_below: lo <= min (range starts at the first lane); lo_above: lo > max (no lane)
  // hi_above: hi >= max (range ends at the last lane); hi_below: hi < min (no lane)
  if (lo_above || hi_below) return 0ull;
  const uint32_t a = lo_below ? first : first + uint32_t(lo_off);
  const uint32_t b = hi_above ? first + span : first + uint32_t(hi_off);
  if (b < a) return 0ull;
  const uint64_t upto = b >= 63 ? ~0ull : ((1ull << (b + 1)) - 1);
  return upto & ~((1ull << a) - 1);
}
__device__ __forceinline__ uint64_t affine_lanes4(const DWordIP& wd, const DCidr& c) {
  const uint32_t lo = c.net[3] & c.mask[3], hi = lo | ~c.mask[3];
  const uint32_t first = wd.aff & 63u;
  return lanes_in_range(first, wd.max4 - wd.min4, uint64_t(lo - wd.min4), lo <= wd.min4, lo > wd.max4, uint64_t(hi - wd.min4),
                        hi < wd.min4, hi >= wd.max4);
}
__device__ __forceinline__ uint64_t low64(const uint32_t* x) { return (uint64_t(x[2]) << 32) | x[3]; }
__device__ __forceinline__ uint64_t affine_lanes6(const DWordIP& wd, const DCidr& c) {
  uint32_t lo[4], hi[4];
  for (int i = 0; i < 4; i++) {
    lo[i] = c.net[i] & c.mask[i];
    hi[i] = lo[i] | ~c.mask[i];
  }
  const uint32_t first = (wd.aff >> 8) & 63u;
  const uint64_t mn = low64(wd.min6), mx = low64(wd.max6);
  return lanes_in_range(first, uint32_t(mx - mn), low64(lo) - mn, !lt128(wd.min6, lo), lt128(wd.max6, lo), low64(hi) - mn,
                        lt128(hi, wd.min6), !lt128(hi, wd.max6));
}

constexpr uint32_t IP_MIXB = 1;  // straddling words of an IP row whose pod addresses are loaded at once (2: config #4 launch B +4 us)
__device__ __forceinline__ void ip_row_word(const DIPTest& t, const DCidr* ex, const DIP* __restrict__ pod_ip,
                                            const DWordIP& wd, bool valid, uint32_t w, uint32_t chunk, uint32_t P, uint32_t W,
                                            uint32_t lane, uint64_t* __restrict__ PM, uint32_t* __restrict__ rng,
                                            uint32_t* __restrict__ cnz) {
  bool uniform = true;
  uint64_t res = 0;
  if (valid) {
    const bool v4 = t.cidr.fam == 4;
    const uint64_t fm = v4 ? wd.m4 : wd.m6;  // pods of the network's family; the others never match
    if (fm && ((wd.aff >> (v4 ? 7 : 15)) & 1u)) {
      // affine addresses: the network and each except of its family are lane ranges (ipaddress.go:22-40:
      // in the CIDR and in none of the excepts)
      res = fm & (v4 ? affine_lanes4(wd, t.cidr) : affine_lanes6(wd, t.cidr));
      for (uint32_t e = 0; e < t.excnt && res; e++) {
        const DCidr x = ex[e];
        if (x.fam == t.cidr.fam) res &= ~(v4 ? affine_lanes4(wd, x) : affine_lanes6(wd, x));
      }
    } else if (fm) {
      uint32_t pos = v4 ? span_vs_cidr4(wd.min4, wd.max4, t.cidr) : span_vs_cidr6(wd.min6, wd.max6, t.cidr);
      if (pos == 2) uniform = false;
      else if (pos == 1) {
        res = fm;
        for (uint32_t e = 0; e < t.excnt; e++) {
          const DCidr x = ex[e];
          if (x.fam != t.cidr.fam) continue;
          uint32_t xp = v4 ? span_vs_cidr4(wd.min4, wd.max4, x) : span_vs_cidr6(wd.min6, wd.max6, x);
          if (xp == 0) continue;
          if (xp == 1) res = 0;
          else uniform = false;
          break;
        }
      }
    }
  }
  uint64_t nz = __ballot(valid && uniform && res != 0);
  // chunk-dense: a chunk with any nonzero word (or a straddling word still to test) stores all its
  // words; an all-zero chunk stores none, only its mask word below
  if ((nz | __ballot(valid && !uniform)) && valid && uniform) PM[uint64_t(t.peer) * W + w] = res;
  const uint32_t w0 = chunk * 64;
  uint32_t lo = nz ? w0 + __ffsll((unsigned long long)nz) - 1 : 0xFFFFFFFFu;
  uint32_t hi = nz ? w0 + 63 - __clzll((long long)nz) : 0u;
  uint64_t mixed = __ballot(valid && !uniform);
  // words whose pods straddle the network (or an except) are tested a pod per lane, IP_MIXB words at
  // once: only the network family's address words are loaded (a pod of the other family never
  // matches, ippeermatcher / net.Contains), all of the batch's loads in flight together
  const bool v4net = t.cidr.fam == 4;
  while (mixed) {
    uint32_t wl[IP_MIXB], fam[IP_MIXB], a[IP_MIXB][4];
#pragma unroll
    for (uint32_t u = 0; u < IP_MIXB; u++) {
      wl[u] = 64;
      if (mixed) {
        wl[u] = __ffsll((unsigned long long)mixed) - 1;
        mixed &= mixed - 1;
      }
      const uint32_t q = (chunk * 64 + wl[u]) * 64 + lane;
      // loaded unconditionally (a clamped pod), so the batch's loads are in flight together
      const DIP* ip = pod_ip + min(q, P - 1);
      const bool live = wl[u] < 64 && q < P;
      const uint32_t f = ip->fam;
      a[u][3] = ip->w[3];
      a[u][0] = v4net ? 0u : ip->w[0];
      a[u][1] = v4net ? 0u : ip->w[1];
      a[u][2] = v4net ? 0u : ip->w[2];
      fam[u] = live ? f : 0u;
    }
#pragma unroll
    for (uint32_t u = 0; u < IP_MIXB; u++) {
      if (wl[u] >= 64) break;  // wave-uniform
      DIP ip{};
      ip.valid = 1;
      ip.fam = fam[u];
      ip.w[0] = a[u][0];
      ip.w[1] = a[u][1];
      ip.w[2] = a[u][2];
      ip.w[3] = a[u][3];
      uint32_t o = 0;
      if (fam[u] && cidr_contains(t.cidr, ip)) {
        o = 1;
        for (uint32_t e = 0; e < t.excnt; e++)
          if (cidr_contains(ex[e], ip)) {
            o = 0;
            break;
          }
      }
      const uint32_t ww = chunk * 64 + wl[u];
      const uint64_t m = __ballot(o == 1);
      if (lane == 0) PM[uint64_t(t.peer) * W + ww] = m;
      if (m) {
        nz |= 1ull << wl[u];
        lo = min(lo, ww);
        hi = max(hi, ww);
      }
    }
  }
  if (lane == 0) {
    cnz[uint64_t(t.peer) * ((W + 63) / 64) + chunk] = nz ? 1u : 0u;
    if (lo != 0xFFFFFFFFu) {
      atomicMin(&rng[4 * t.peer], lo);
      atomicMin(&rng[4 * t.peer + 1], ~hi);
      if (chunk < 64) atomicAnd(reinterpret_cast<unsigned long long*>(rng) + 2 * t.peer + 1, ~(1ull << chunk));
    }
  }
}

// ~0 if word w of IP peer j's PM row was stored (its chunk has a nonzero word; see ip_row_word).
__device__ __forceinline__ uint64_t cnz_mask(const uint32_t* __restrict__ cnz, uint32_t W, uint32_t j, uint32_t w) {
  return cnz[uint64_t(j) * ((W + 63) / 64) + w / 64] ? ~0ull : 0ull;
}

// IP rows by address ranges (no-panic runs): an IPBlock that matches few pods
// is built from the host's address index instead of a test per word — the pods of each family
// sorted by address, so the CIDR less its same-family excepts (ipaddress.go:22-40: in the network,
// in none of the excepts) is a few intervals of sorted positions, found by binary search once per
// problem.  A wave per IPBlock sets its pods' bits in an LDS copy of the row window (64-bit LDS
// ORs), then stores the chunks holding a bit, chunk-dense like k_ip_rows_fast, with the row's word
// span and chunk masks.  Cost ~ matching pods + window words, with no per-pod address loads or
// straddling-word round trips (config #2's pod addresses step by 256 within a namespace, so every
// word a /16 touches straddled it).
struct DIPRange {
  uint32_t peer, ivoff, ivcnt;  // intervals iv[ivoff .. ivoff + ivcnt) of sorted positions
  uint32_t sw0;                 // first word of the matching pods' span (< IPR_SPAN words long)
};
constexpr uint32_t IPR_MAX_MATCH = 4096;  // pods an IPBlock may match to be built from ranges
constexpr uint32_t IPR_SPAN = 256;        // words of a range row's LDS window (the matching pods' span)
constexpr uint32_t IP_GROUP_MAX = 64, IP_EX_LDS = 256;
// LDS of the two IP-row bodies, one allocation in a kernel that holds both (k_front_b): the fast
// rows' staged tests and excepts, or the range rows' per-wave row windows
union IpRowsLds {
  struct {
    DIPTest t[IP_GROUP_MAX];
    DCidr ex[IP_EX_LDS];
  } fast;
  unsigned long long row[4][IPR_SPAN];
};
__shared__ IpRowsLds ip_lds;
__device__ __forceinline__ void ip_rows_range_blk(uint32_t Rr, uint32_t W, const DIPRange* __restrict__ rt,
                                                  const uint2* __restrict__ iv, const uint32_t* __restrict__ sorted,
                                                  uint64_t* __restrict__ PM, uint32_t* __restrict__ rng, uint32_t* __restrict__ cnz,
                                                  uint32_t bid_, uint32_t c0, uint32_t nch) {
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t r = __builtin_amdgcn_readfirstlane(bid_ * 4 + wv);  // wave-uniform
  unsigned long long* row = ip_lds.row[wv];
  const bool live = r < Rr;
  for (uint32_t x = lane; x < IPR_SPAN; x += 64) row[x] = 0;
  DIPRange t{};
  if (live) t = rt[r];
  // the LDS window: the span's words inside the run's word window (a source shard's ingress peers)
  const uint32_t lo_w = max(t.sw0, c0 * 64), hi_w = min(min(t.sw0 + IPR_SPAN, (c0 + nch) * 64), W);
  __syncthreads();
  for (uint32_t i = 0; live && i < t.ivcnt; i++) {
    const uint2 v = iv[t.ivoff + i];
    for (uint32_t p0 = v.x; p0 < v.y; p0 += 4 * 64) {  // 4 pods a lane in flight
      uint32_t q[4];
#pragma unroll
      for (uint32_t u = 0; u < 4; u++) q[u] = sorted[min(p0 + u * 64 + lane, v.y - 1)];
#pragma unroll
      for (uint32_t u = 0; u < 4; u++) {
        const uint32_t w = q[u] >> 6;
        if (p0 + u * 64 + lane < v.y && w >= lo_w && w < hi_w) atomicOr(&row[w - t.sw0], 1ull << (q[u] & 63));
      }
    }
  }
  __syncthreads();
  if (!live) return;
  const uint32_t j = t.peer, cw = (W + 63) / 64;
  uint32_t lo = 0xFFFFFFFFu, hi = 0;
  uint64_t chunks = 0;
  for (uint32_t c = c0; c < c0 + nch; c++) {
    const uint32_t w = c * 64 + lane;
    const bool in = c * 64 + 63 >= lo_w && c * 64 < hi_w;  // wave-uniform: the chunk meets the window
    const uint64_t v = in && w >= lo_w && w < hi_w ? row[w - t.sw0] : 0ull;
    const uint64_t nz = __ballot(v != 0);
    if (nz && w < W) PM[uint64_t(j) * W + w] = v;  // chunk-dense: every word of a chunk with a bit
    if (lane == 0) cnz[uint64_t(j) * cw + c] = nz ? 1u : 0u;
    if (nz) {
      lo = min(lo, c * 64 + uint32_t(__ffsll((unsigned long long)nz) - 1));
      hi = max(hi, c * 64 + 63 - uint32_t(__clzll((long long)nz)));
      if (c < 64) chunks |= 1ull << c;
    }
  }
  if (lane == 0) {  // the row's only writer: its span and nonzero-chunk mask (as k_ip_rows_fast's atomics leave them)
    rng[4 * j] = lo;
    rng[4 * j + 1] = lo == 0xFFFFFFFFu ? 0xFFFFFFFFu : ~hi;
    reinterpret_cast<unsigned long long*>(rng)[2 * j + 1] = ~chunks;
  }
}
__global__ __launch_bounds__(256) void k_ip_rows_range(uint32_t Rr, uint32_t W, const DIPRange* __restrict__ rt, const uint2* __restrict__ iv,
                                                       const uint32_t* __restrict__ sorted, uint64_t* __restrict__ PM,
                                                       uint32_t* __restrict__ rng, uint32_t* __restrict__ cnz, uint32_t c0, uint32_t nch) {
  ip_rows_range_blk(Rr, W, rt, iv, sorted, PM, rng, cnz, blockIdx.x, c0, nch);
}

// IP rows as pod intervals (no-panic runs whose network family is address-monotone in pod order, the
// usual case: addresses handed out in pod order).  The host's address index turns the network less
// its same-family excepts (ipaddress.go:22-40; ippeermatcher.go:43-50) into <= IPV_MAX pod-index
// intervals [x, y) of that family's pods, once per range plan; a row word is then the family's pods of
// the word (DWordIP::m4 / m6) AND the intervals' lanes — no pod address is loaded and no word
// straddles.  A wave per row: the chunks outside the rows' pod span get their chunk flag cleared (one
// vector store), each chunk of the span is one pass (lane = word) storing the chunk dense when it has
// a bit, and the row's word span and chunk mask are plain stores (the row's only writer), as
// ip_rows_range_blk leaves them.
struct DIPIv {
  uint32_t peer, fam, ivoff, ivcnt;  // fam 0 = IPv4, 1 = IPv6; intervals ipv_iv[ivoff .. ivoff + ivcnt), ascending
};
constexpr uint32_t IPV_MAX = 16;  // intervals an interval-built row may have (1 + its same-family excepts)
__device__ __forceinline__ uint64_t pod_span_bits(uint32_t w, uint32_t x, uint32_t y) {  // pods [x, y) in word w
  const uint32_t b0 = w * 64, a = max(x, b0), b = min(y, b0 + 64);
  if (b <= a) return 0ull;
  const uint32_t lo = a - b0, n = b - a;
  return (n == 64 ? ~0ull : ((1ull << n) - 1)) << lo;
}
__device__ __forceinline__ void ip_rows_iv_blk(uint32_t Rv, uint32_t W, const DIPIv* __restrict__ rt,
                                               const uint2* __restrict__ iv, const DWordIP* __restrict__ words,
                                               uint64_t* __restrict__ PM, uint32_t* __restrict__ rng, uint32_t* __restrict__ cnz,
                                               uint32_t bid_, uint32_t c0, uint32_t nch) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t r = __builtin_amdgcn_readfirstlane(bid_ * 4 + (threadIdx.x >> 6));  // wave-uniform
  if (r >= Rv) return;
  const DIPIv t = rt[r];
  const uint32_t j = t.peer, cw = (W + 63) / 64;
  // the rows' pod span [p0, p1) -> its chunks [s0, s1] (empty: s0 > s1)
  const uint32_t p0 = t.ivcnt ? iv[t.ivoff].x : 0u, p1 = t.ivcnt ? iv[t.ivoff + t.ivcnt - 1].y : 0u;
  const uint32_t s0 = max(c0, p0 / 4096), s1 = p1 > p0 ? min(c0 + nch, (p1 - 1) / 4096 + 1) : 0u;  // [s0, s1)
  // chunks of the window outside the span: no bit (their PM words are not written)
  for (uint32_t c = c0 + lane; c < c0 + nch; c += 64)
    if (c < s0 || c >= s1) cnz[uint64_t(j) * cw + c] = 0;
  uint32_t lo = 0xFFFFFFFFu, hi = 0;
  uint64_t chunks = 0;
  for (uint32_t c = s0; c < s1; c++) {
    const uint32_t w = c * 64 + lane;
    uint64_t v = 0;
    if (w < W) {
      const DWordIP& wd = words[w];
      const uint64_t fm = t.fam ? wd.m6 : wd.m4;
      for (uint32_t i = 0; i < t.ivcnt; i++) {  // (scalar loads: the intervals are wave-uniform)
        const uint2 x = iv[t.ivoff + i];
        v |= pod_span_bits(w, x.x, x.y);
      }
      v &= fm;
    }
    const uint64_t nz = __ballot(v != 0);
    if (nz && w < W) PM[uint64_t(j) * W + w] = v;  // chunk-dense: every word of a chunk with a bit
    if (lane == 0) cnz[uint64_t(j) * cw + c] = nz ? 1u : 0u;
    if (nz) {
      lo = min(lo, c * 64 + uint32_t(__ffsll((unsigned long long)nz) - 1));
      hi = max(hi, c * 64 + 63 - uint32_t(__clzll((long long)nz)));
      if (c < 64) chunks |= 1ull << c;
    }
  }
  if (lane == 0) {
    rng[4 * j] = lo;
    rng[4 * j + 1] = lo == 0xFFFFFFFFu ? 0xFFFFFFFFu : ~hi;
    reinterpret_cast<unsigned long long*>(rng)[2 * j + 1] = ~chunks;
  }
}
__global__ __launch_bounds__(256) void k_ip_rows_iv(uint32_t Rv, uint32_t W, const DIPIv* __restrict__ rt, const uint2* __restrict__ iv,
                                                    const DWordIP* __restrict__ words, uint64_t* __restrict__ PM,
                                                    uint32_t* __restrict__ rng, uint32_t* __restrict__ cnz, uint32_t c0, uint32_t nch) {
  ip_rows_iv_blk(Rv, W, rt, iv, words, PM, rng, cnz, blockIdx.x, c0, nch);
}

// A block handles one group of `grp` IP peers over 4 chunks of 64 words (a wave per chunk, lane =
// word): the group's tests and their except records are staged into LDS once (one coalesced load
// per block, instead of a chain of dependent scalar loads per peer and except), and each wave loads
// its words' [min, max] records once for the whole group.
constexpr uint32_t IP_GROUP = 16;  // IP peers per block (profiles/r02_ip_group_ab.txt)
// Chunks [c0, c0 + nch) of the rows (a source shard's ingress peers: the chunks of its word window).
__device__ __forceinline__ void ip_rows_fast_blk(uint32_t Ri, uint32_t P, uint32_t W, const DIPTest* __restrict__ tests,
                                                      const DCidr* __restrict__ ip_ex, const DIP* __restrict__ pod_ip,
                                                      const DWordIP* __restrict__ words, uint64_t* __restrict__ PM,
                                                      uint32_t* __restrict__ rng, uint32_t* __restrict__ cnz, uint32_t bid_, uint32_t nblk_,
                                                      uint32_t grp, uint32_t c0, uint32_t nch) {
  DIPTest* const s_t = ip_lds.fast.t;
  DCidr* const s_ex = ip_lds.fast.ex;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t cb = (nch + 3) / 4;
  const uint32_t r0 = (bid_ / cb) * grp;
  if (r0 >= Ri) return;  // whole block
  const uint32_t nr = min(Ri - r0, grp), chunk = c0 + (bid_ % cb) * 4 + (threadIdx.x >> 6);
  // the wave's word records are loaded first (clamped, unconditionally): their latency overlaps the
  // staging below instead of following its barrier
  const uint32_t w = chunk * 64 + lane;
  const bool valid = w < W && chunk < c0 + nch;
  const DWordIP wd = words[min(w, W - 1)];
  // the chunk's own [min, max] per family (records W.. of `words`): a peer whose network misses
  // the whole chunk leaves all 64 words zero — the wave only clears the chunk's cnz mask
  const DWordIP ck = words[W + min(uint32_t(__builtin_amdgcn_readfirstlane(chunk)), (W + 63) / 64 - 1)];
  const uint32_t ex0 = tests[r0].exoff, nex = tests[r0 + nr - 1].exoff + tests[r0 + nr - 1].excnt - ex0;
  const bool ex_lds = nex <= IP_EX_LDS;
  for (uint32_t x = threadIdx.x; x < nr; x += blockDim.x) s_t[x] = tests[r0 + x];
  if (ex_lds)
    for (uint32_t x = threadIdx.x; x < nex; x += blockDim.x) s_ex[x] = ip_ex[ex0 + x];
  __syncthreads();
  if (chunk >= c0 + nch) return;
  // the chunk test of the group's peers a lane each (lane x: peer r0 + x; grp <= 64): a peer whose
  // network misses the chunk's addresses only gets its chunk mask cleared, here, by its lane — the
  // wave then walks only the peers that touch the chunk (config #4: ~1 in 5)
  bool touch = false;
  if (lane < nr) {
    const DIPTest& tx = s_t[lane];
    const bool v4 = tx.cidr.fam == 4;
    touch = !(tx.cidr.valid && (v4 ? !ck.m4 || span_vs_cidr4(ck.min4, ck.max4, tx.cidr) == 0
                                   : !ck.m6 || span_vs_cidr6(ck.min6, ck.max6, tx.cidr) == 0));
    if (!touch) cnz[uint64_t(tx.peer) * ((W + 63) / 64) + chunk] = 0;
  }
  for (uint64_t todo = __ballot(touch); todo; todo &= todo - 1) {
    const DIPTest t = s_t[__builtin_amdgcn_readfirstlane(__ffsll((unsigned long long)todo) - 1)];
    ip_row_word(t, ex_lds ? s_ex + (t.exoff - ex0) : ip_ex + t.exoff, pod_ip, wd, valid, w, chunk, P, W, lane, PM, rng, cnz);
  }
}
__global__ __launch_bounds__(256) void k_ip_rows_fast(uint32_t Ri, uint32_t P, uint32_t W, const DIPTest* __restrict__ tests,
                                                      const DCidr* __restrict__ ip_ex, const DIP* __restrict__ pod_ip,
                                                      const DWordIP* __restrict__ words, uint64_t* __restrict__ PM,
                                                      uint32_t* __restrict__ rng, uint32_t* __restrict__ cnz, uint32_t grp,
                                                      uint32_t c0, uint32_t nch) {
  ip_rows_fast_blk(Ri, P, W, tests, ip_ex, pod_ip, words, PM, rng, cnz, blockIdx.x, gridDim.x, grp, c0, nch);
}

// IP rows as work items (the fused front's default, cyc_set_option "ip_items"): the host lists, per
// 64-word chunk of the run's window, the IP rows whose network meets the chunk's address range
// (the test ip_rows_fast_blk makes per wave, made once per range plan), so a wave handles up to
// IPI_TOUCH rows that all touch its chunk — its word records loaded once for all of them, their tests
// held one per lane and broadcast with readlane — instead of a group of IP_GROUP rows of which a
// few touch (config #4: ~1 in 5).  A "zero" item clears the chunk flag of up to 64 rows that miss it.
struct DIPItem {
  uint32_t chunk, off, cnt, touch;  // rows ilist[off .. off + cnt) (indices into the segment's tests)
};
constexpr uint32_t IPI_TOUCH = 16;  // touching rows per wave
__device__ __forceinline__ void ip_rows_items_blk(uint32_t n_items, const DIPItem* __restrict__ items,
                                                  const uint32_t* __restrict__ ilist, uint32_t P, uint32_t W,
                                                  const DIPTest* __restrict__ tests, const DCidr* __restrict__ ip_ex,
                                                  const DIP* __restrict__ pod_ip, const DWordIP* __restrict__ words,
                                                  uint64_t* __restrict__ PM, uint32_t* __restrict__ rng, uint32_t* __restrict__ cnz,
                                                  uint32_t bid_) {
  const uint32_t wv = __builtin_amdgcn_readfirstlane(bid_ * 4 + (threadIdx.x >> 6)), lane = threadIdx.x & 63;
  if (wv >= n_items) return;
  const DIPItem it = items[wv];
  const uint32_t cw = (W + 63) / 64;
  const uint32_t mi = ilist[it.off + min(lane, it.cnt - 1)];
  if (!it.touch) {
    const uint32_t peer = tests[mi].peer;
    if (lane < it.cnt) cnz[uint64_t(peer) * cw + it.chunk] = 0;
    return;
  }
  const uint32_t w = it.chunk * 64 + lane;
  const bool valid = w < W;
  const DWordIP wd = words[min(w, W - 1)];
  const DIPTest mine = tests[mi];  // lane x < cnt holds row x's test
  for (uint32_t x = 0; x < it.cnt; x++) {
    DIPTest t;
    t.peer = __builtin_amdgcn_readlane(mine.peer, x);
    t.exoff = __builtin_amdgcn_readlane(mine.exoff, x);
    t.excnt = __builtin_amdgcn_readlane(mine.excnt, x);
    t.pad = 0;
    t.cidr.valid = __builtin_amdgcn_readlane(mine.cidr.valid, x);
    t.cidr.fam = __builtin_amdgcn_readlane(mine.cidr.fam, x);
    t.cidr.pad0 = t.cidr.pad1 = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      t.cidr.net[i] = __builtin_amdgcn_readlane(mine.cidr.net[i], x);
      t.cidr.mask[i] = __builtin_amdgcn_readlane(mine.cidr.mask[i], x);
    }
    ip_row_word(t, ip_ex + t.exoff, pod_ip, wd, valid, w, it.chunk, P, W, lane, PM, rng, cnz);
  }
}

// Grid of k_ip_rows_fast / an IP-row range of k_front_b: peer groups x blocks of 4 of the nch chunks.
__host__ __device__ inline uint64_t ip_rows_blocks(uint32_t Ri, uint32_t nch, uint32_t grp) {
  return uint64_t((Ri + grp - 1) / grp) * ((nch + 3) / 4);
}

}  // namespace cyc
