// engine.hip — CDNA4 (gfx950) verdict engine for cyclonus's simulated-connectivity path.
//
// What the reference does per cell (pkg/connectivity/probe/jobrunner.go:68-94 ->
// pkg/matcher/policy.go:131-174): for the ingress direction, walk EVERY ingress target, keep the
// ones whose namespace equals the destination's and whose pod selector matches its labels
// (TargetsApplyingToPod :68-82); the cell is allowed iff no target matched, or some matched
// target's ordered peer list (target.go:29-36) allows the source on the job's port; same for
// egress with source and destination swapped.
//
// What this engine does instead (exact rewriting, no per-cell walk):
//   k_selectors     every (selector, label set) pair once            -> SELRES u8 [S][L]
//   k_peer_rows     every pod/IP peer over all pods as packed bits    -> PM / ER [R][W] u64
//                   (ER = the peer would panic for that pod: bad CIDR/IP/operator)
//   k_portok        every (port matcher, job descriptor)              -> PORTOK u8 [M][D]
//   k_slot_words    per (slot, 64-pod word): valid bits, desc masks   -> VALID, DESCW, DM
//   k_member        per pod IDENTITY (ns, labels[, job descriptors]): matching targets,
//                   a 64-bit hash, and a device hash table that elects one representative
//                   identity per distinct target set                  -> classes
//   k_class_rows    per class representative, slot, word: OR over its targets of the ordered
//                   peer walk done 64 pods at a time with bit ops     -> A_in / A_eg rows
//   k_emit          per target pod: copy its class rows into the output planes (HBM-bound;
//                   the roofline kernel)
//   k_first_error / k_error_detail   only when the inputs can panic: first panicking job in
//                   the reference's job order and the panic message.
#include <dlfcn.h>
#include <execinfo.h>
#include <hip/hip_runtime.h>

#include <csignal>
#include <cstdlib>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <unordered_map>
#include <vector>

#include "cyclonus_hip.h"
#include "host.hpp"

namespace cyc {

// ----------------------------------------------------------------------------- device helpers
__device__ __forceinline__ uint64_t mix64(uint64_t z) {  // splitmix64 finaliser
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Evaluate selector `sel` on label set `ls`: 0 no match, 1 match, 2 panic (invalid operator).
// labelselector.go:66-86: matchLabels first (all must hold), then expressions in order.
__device__ uint8_t eval_selector(const uint32_t* __restrict__ sel_off, const DReq* __restrict__ reqs,
                                 const uint32_t* __restrict__ req_vals, const uint32_t* __restrict__ ls_off,
                                 const uint32_t* __restrict__ ls_key, const uint32_t* __restrict__ ls_val,
                                 uint32_t sel, uint32_t ls) {
  uint32_t r0 = sel_off[sel], r1 = sel_off[sel + 1];
  uint32_t l0 = ls_off[ls], l1 = ls_off[ls + 1];
  for (uint32_t r = r0; r < r1; r++) {
    DReq q = reqs[r];
    if (q.op == REQ_INVALID) return 2;
    // binary search the key in the (sorted) label set
    uint32_t lo = l0, hi = l1;
    while (lo < hi) {
      uint32_t mid = (lo + hi) >> 1;
      if (ls_key[mid] < q.key) lo = mid + 1;
      else hi = mid;
    }
    bool present = lo < l1 && ls_key[lo] == q.key;
    uint32_t v = present ? ls_val[lo] : 0xFFFFFFFFu;
    bool ok;
    switch (q.op) {
      case REQ_EQ: ok = present && v == req_vals[q.voff]; break;
      case REQ_EQ_EMPTY: ok = !present || v == req_vals[q.voff]; break;
      case REQ_IN:
      case REQ_NOTIN: {
        bool in = false;
        for (uint32_t i = 0; i < q.vcnt; i++) in |= (req_vals[q.voff + i] == v);
        ok = present && (q.op == REQ_IN ? in : !in);
        break;
      }
      case REQ_EXISTS: ok = present; break;
      default: ok = !present; break;  // REQ_DNE
    }
    if (!ok) return 0;
  }
  return 1;
}

// sel_list (optional): only these selectors' rows are evaluated (range plan); S = its length.
__global__ void k_selectors(uint32_t S, uint32_t L, const uint32_t* sel_off, const DReq* reqs, const uint32_t* req_vals,
                            const uint32_t* ls_off, const uint32_t* ls_key, const uint32_t* ls_val,
                            uint8_t* __restrict__ selres, const uint32_t* __restrict__ sel_list = nullptr) {
  uint64_t n = uint64_t(S) * L;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    uint32_t s = uint32_t(i / L), l = uint32_t(i % L);
    if (sel_list) s = sel_list[s];
    selres[uint64_t(s) * L + l] = eval_selector(sel_off, reqs, req_vals, ls_off, ls_key, ls_val, s, l);
  }
}

// Same evaluation over a dense label table: LVT[kx][l] = value id of dense key kx in label set l
// (~0 = key absent; column NK is all-absent for selector keys no label set has), and dreqs with
// the key replaced by its dense index.  One coalesced load per requirement instead of a binary
// search over the label set (a chain of dependent loads).
constexpr uint32_t SEL_LPT = 4;  // label sets per thread in k_selectors_dense (independent loads in flight)
__device__ __forceinline__ void selectors_dense_blk(uint32_t S, uint32_t L, const uint32_t* __restrict__ sel_off,
                                                         const DReq* __restrict__ dreqs, const uint32_t* __restrict__ req_vals,
                                                         const uint32_t* __restrict__ LVT, uint8_t* __restrict__ selres,
                                                         const uint32_t* __restrict__ sel_list, uint32_t bid_, uint32_t nblk_) {
  // block = (selector, 256 * SEL_LPT label sets): the requirement walk is block-uniform (scalar
  // loads); each thread evaluates SEL_LPT label sets with their table loads issued together
  const uint32_t lchunks = (L + 256 * SEL_LPT - 1) / (256 * SEL_LPT);
  uint32_t s = bid_ / lchunks;
  const uint32_t l0 = (bid_ % lchunks) * 256 * SEL_LPT + threadIdx.x;
  if (s >= S) return;
  if (sel_list) s = sel_list[s];
  uint8_t res[SEL_LPT];
#pragma unroll
  for (uint32_t x = 0; x < SEL_LPT; x++) res[x] = 1;
  for (uint32_t r = sel_off[s]; r < sel_off[s + 1]; r++) {
    const DReq q = dreqs[r];
    if (q.op == REQ_INVALID) {  // reached only by label sets every earlier requirement matched
#pragma unroll
      for (uint32_t x = 0; x < SEL_LPT; x++) res[x] = res[x] == 1 ? 2 : res[x];
      break;
    }
    uint32_t v[SEL_LPT];
#pragma unroll
    for (uint32_t x = 0; x < SEL_LPT; x++) {
      const uint32_t l = l0 + x * 256;
      v[x] = l < L ? LVT[uint64_t(q.key) * L + l] : 0xFFFFFFFFu;
    }
    const uint32_t v0 = (q.op == REQ_EQ || q.op == REQ_EQ_EMPTY) ? req_vals[q.voff] : 0u;
#pragma unroll
    for (uint32_t x = 0; x < SEL_LPT; x++) {
      const bool present = v[x] != 0xFFFFFFFFu;
      bool ok;
      switch (q.op) {
        case REQ_EQ: ok = present && v[x] == v0; break;
        case REQ_EQ_EMPTY: ok = !present || v[x] == v0; break;
        case REQ_IN:
        case REQ_NOTIN: {
          bool in = false;
          for (uint32_t j = 0; j < q.vcnt; j++) in |= (req_vals[q.voff + j] == v[x]);
          ok = present && (q.op == REQ_IN ? in : !in);
          break;
        }
        case REQ_EXISTS: ok = present; break;
        default: ok = !present; break;  // REQ_DNE
      }
      if (!ok && res[x] == 1) res[x] = 0;
    }
  }
#pragma unroll
  for (uint32_t x = 0; x < SEL_LPT; x++) {
    const uint32_t l = l0 + x * 256;
    if (l < L) selres[uint64_t(s) * L + l] = res[x];
  }
}
__global__ __launch_bounds__(256) void k_selectors_dense(uint32_t S, uint32_t L, const uint32_t* __restrict__ sel_off,
                                                         const DReq* __restrict__ dreqs, const uint32_t* __restrict__ req_vals,
                                                         const uint32_t* __restrict__ LVT, uint8_t* __restrict__ selres,
                                                         const uint32_t* __restrict__ sel_list) { selectors_dense_blk(S, L, sel_off, dreqs, req_vals, LVT, selres, sel_list, blockIdx.x, gridDim.x); }

// A selector's outcome on a label set, from SELRES (dense builds) or evaluated on the spot from the
// dense label table (lazy builds: PM builds, whose pods carry ~as many label sets as there are pods,
// evaluate only the (selector, label set) pairs a membership walk or a pod-peer word reaches instead
// of every pair).  Same result as selectors_dense_blk: requirements in order, the first failing one
// decides 0, an invalid operator reached with every earlier requirement matched is a panic (2).
struct SelView {
  const uint8_t* selres;  // null: evaluate through LVT
  uint32_t L;
  const uint32_t *sel_off, *req_vals, *LVT;
  const DReq* dreqs;
  const uint32_t* PLVT;   // LVT's columns per pod: PLVT[kx][q] = LVT[kx][label set of pod q]
  uint32_t P;
  const uint4* one;       // per selector: (op | values << 8, dense key, value 0, value 1) when it is ONE
                          // requirement of <= 2 values; x = SEL_ALL (no requirement) / SEL_WALK (other)
};
constexpr uint32_t SEL_ALL = 0xFFFFFFFEu, SEL_WALK = 0xFFFFFFFFu;
// (tab, n) = (LVT, L) with l a label set, or (PLVT, P) with l a pod: the key's value column
__device__ __forceinline__ uint32_t sel_eval(const SelView& v, const uint32_t* __restrict__ tab, uint32_t n, uint32_t s, uint32_t l) {
  for (uint32_t r = v.sel_off[s]; r < v.sel_off[s + 1]; r++) {
    const DReq q = v.dreqs[r];
    if (q.op == REQ_INVALID) return 2;
    const uint32_t x = tab[uint64_t(q.key) * n + l];
    const bool present = x != 0xFFFFFFFFu;
    bool ok;
    switch (q.op) {
      case REQ_EQ: ok = present && x == v.req_vals[q.voff]; break;
      case REQ_EQ_EMPTY: ok = !present || x == v.req_vals[q.voff]; break;
      case REQ_IN:
      case REQ_NOTIN: {
        bool in = false;
        for (uint32_t j = 0; j < q.vcnt; j++) in |= (v.req_vals[q.voff + j] == x);
        ok = present && (q.op == REQ_IN ? in : !in);
        break;
      }
      case REQ_EXISTS: ok = present; break;
      default: ok = !present; break;  // REQ_DNE
    }
    if (!ok) return 0;
  }
  return 1;
}
// labelselector.go:66-86 for one requirement, x = the pod's value of the key (~0: absent), with at
// most two values (v0, v1; vc of them)
__device__ __forceinline__ bool req_holds(uint32_t op, uint32_t x, uint32_t v0, uint32_t v1, uint32_t vc) {
  const bool present = x != 0xFFFFFFFFu;
  const bool in = (vc > 0 && x == v0) || (vc > 1 && x == v1);
  switch (op) {
    case REQ_EQ: return present && x == v0;
    case REQ_EQ_EMPTY: return !present || x == v0;
    case REQ_IN: return present && in;
    case REQ_NOTIN: return present && !in;
    case REQ_EXISTS: return present;
    default: return !present;  // REQ_DNE
  }
}

__device__ __forceinline__ uint32_t sel_at(const SelView& v, uint32_t s, uint32_t l) {
  if (v.selres) return v.selres[uint64_t(s) * v.L + l];
  // one requirement: one table load, no walk (so several evaluations' loads can be in flight)
  const uint4 d = v.one[s];
  if (d.x == SEL_ALL) return 1;
  if (d.x != SEL_WALK) return req_holds(d.x & 0xFFu, v.LVT[uint64_t(d.y) * v.L + l], d.z, d.w, d.x >> 8) ? 1u : 0u;
  return sel_eval(v, v.LVT, v.L, s, l);
}
// Mixes identity i's ingress slot descriptors into its class hash (status and descriptor of every
// slot), 8 slots' loads in flight at once.
__device__ __forceinline__ uint64_t hash_slots(uint64_t h, const uint8_t* __restrict__ id_status, const int32_t* __restrict__ id_desc,
                                               uint32_t i, uint32_t K) {
  for (uint32_t k0 = 0; k0 < K; k0 += 8) {
    uint8_t st[8];
    int32_t ds[8];
#pragma unroll
    for (uint32_t x = 0; x < 8; x++) {
      const uint64_t ik = uint64_t(i) * K + min(k0 + x, K - 1);
      st[x] = id_status[ik];
      ds[x] = id_desc[ik];
    }
#pragma unroll
    for (uint32_t x = 0; x < 8; x++) {
      if (k0 + x >= K) break;
      const uint64_t sk = st[x];
      const int32_t d = sk == CYC_JOB_VALID ? ds[x] : -1;
      h = mix64(h ^ ((sk << 40) | uint32_t(d + 1)) ^ (uint64_t(k0 + x) << 48));
    }
  }
  return h;
}

// Pod selector s on pod q's own labels through PLVT: one coalesced load per requirement for a wave
// of consecutive pods, instead of a pod -> label set -> table gather chain.
__device__ __forceinline__ uint32_t sel_at_pod(const SelView& v, uint32_t s, uint32_t q) { return sel_eval(v, v.PLVT, v.P, s, q); }

__device__ __forceinline__ void fill_u32_blk(uint32_t* p, uint64_t n, uint32_t v, uint32_t bid_, uint32_t nblk_) {
  const uint64_t i = bid_ * uint64_t(blockDim.x) + threadIdx.x;
  if (i < n) p[i] = v;
}
__global__ void k_fill_u32(uint32_t* p, uint64_t n, uint32_t v) { fill_u32_blk(p, n, v, blockIdx.x, gridDim.x); }

// PLVT[kx][q] = LVT[kx][label set of pod q] (SelView::PLVT), one word per thread (grid-stride)
__global__ __launch_bounds__(256) void k_plvt(const uint32_t* __restrict__ LVT, const uint32_t* __restrict__ pod_ls, uint32_t L,
                                              uint32_t P, uint64_t n, uint32_t* __restrict__ PLVT) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t kx = i / P, q = i - kx * P;
    PLVT[i] = LVT[kx * L + pod_ls[q]];
  }
}

// IPNet.Contains after To4 collapse (ipaddress.go:10-20): families must agree.
__device__ __forceinline__ bool cidr_contains(const DCidr& c, const DIP& ip) {
  if (c.fam != ip.fam) return false;
  if (c.fam == 4) return ((c.net[3] ^ ip.w[3]) & c.mask[3]) == 0;
  return (((c.net[0] ^ ip.w[0]) & c.mask[0]) | ((c.net[1] ^ ip.w[1]) & c.mask[1]) |
          ((c.net[2] ^ ip.w[2]) & c.mask[2]) | ((c.net[3] ^ ip.w[3]) & c.mask[3])) == 0;
}

// Outcome of a pod peer for a peer pod with namespace `ns`, namespace label set `nsls` and pod
// label set `ls`: 0 no, 1 match (before the port check), 2 panic.  podpeermatcher.go:21-28:
// namespace matcher first, pod matcher only if it matched.
__device__ __forceinline__ uint32_t pod_peer_outcome(const DPeer& pr, const uint8_t* __restrict__ selres, uint32_t L,
                                                     uint32_t ns, uint32_t nsls, uint32_t ls) {
  // both matchers' table bytes are loaded up front (byte 0 when a matcher needs none), so neither
  // load waits inside a branch; the outcome still follows the matchers' order
  const bool nsel = pr.nskind == 2, psel = pr.podsel != CYC_ALL;
  const uint8_t rn = selres[nsel ? uint64_t(pr.nsval) * L + nsls : 0u];
  const uint8_t rp = selres[psel ? uint64_t(pr.podsel) * L + ls : 0u];
  if (pr.nskind == 0) {
    if (ns != pr.nsval) return 0;
  } else if (nsel && rn != 1) {
    return rn == 2 ? 2u : 0u;
  }
  return psel ? rp : 1u;
}

// IP peer outcome for one pod IP: ippeermatcher.go:43-50 -> ipaddress.go:22-40 (CIDR parse,
// IP parse, contains, then each except in order; a parse error is a panic).
__device__ __forceinline__ uint32_t ip_peer_outcome(const DIPBlock& b, const DCidr* __restrict__ cidrs,
                                                    const uint32_t* __restrict__ ipb_ex, const DIP& ip) {
  DCidr cd = cidrs[b.cidr];
  if (!cd.valid) return 2;
  if (!ip.valid) return 2;
  if (!cidr_contains(cd, ip)) return 0;
  for (uint32_t e = 0; e < b.excnt; e++) {
    DCidr x = cidrs[ipb_ex[b.exoff + e]];
    if (!x.valid) return 2;
    if (cidr_contains(x, ip)) return 0;
  }
  return 1;
}

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
template <bool ERR>
__device__ __forceinline__ void pod_rows_direct_blk(uint32_t Rp, uint32_t P, uint32_t W,
                                                         const uint32_t* __restrict__ pod_peers,
                                                         const DPeer* __restrict__ peers, const uint8_t* __restrict__ selres,
                                                         uint32_t L, const uint32_t* __restrict__ pod_eid,
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
  for (uint32_t u = 0; u < PR_DIRECT_G; u++) o[u] = pod_peer_outcome(pr[u], selres, L, ns, nsls, ls);
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
  pod_rows_direct_blk<ERR>(Rp, P, W, pod_peers, peers, selres, L, pod_eid, id_ns, id_nsls, id_ls, PM, ER, blockIdx.x, gridDim.x, w0, nw);
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

// PortMatcher.Allows(ResolvedPort, ResolvedPortName, Protocol) — portmatcher.go:10-92, 190-199.
__device__ __forceinline__ void portok_blk(uint32_t M, uint32_t D, const DPortM* pms, const DPortEntry* pents, const DDesc* descs,
                         uint8_t* __restrict__ portok, uint32_t bid_, uint32_t nblk_) {
  uint32_t i = bid_ * blockDim.x + threadIdx.x;
  if (i >= M * D) return;
  uint32_t m = i / D, e = i % D;
  DPortM pm = pms[m];
  DDesc d = descs[e];
  uint8_t ok = pm.all ? 1 : 0;
  for (uint32_t j = 0; j < pm.ecnt && !ok; j++) {
    DPortEntry pe = pents[pm.eoff + j];
    if (pe.proto != d.proto) continue;  // raw protocol string compare ("tcp" != "TCP")
    switch (pe.kind) {
      case PE_PROTO: ok = 1; break;
      case PE_INT: ok = pe.a == d.port; break;
      case PE_NAME: ok = uint32_t(pe.a) == d.name; break;
      default: ok = pe.a <= d.port && d.port <= pe.b; break;
    }
  }
  portok[i] = ok;
}
__global__ void k_portok(uint32_t M, uint32_t D, const DPortM* pms, const DPortEntry* pents, const DDesc* descs,
                         uint8_t* __restrict__ portok) { portok_blk(M, D, pms, pents, descs, portok, blockIdx.x, gridDim.x); }

// Port table rows as descriptor bit masks (D <= 32): the egress class rows test a peer's port
// matcher against a per-word descriptor with a shift of one block-uniform word instead of a
// vector byte load per (slot, peer).
__device__ __forceinline__ void portbits_blk(uint32_t M, uint32_t D, const uint8_t* __restrict__ portok,
                                             uint32_t* __restrict__ portbits, uint32_t bid_) {
  const uint32_t m = bid_ * 256 + threadIdx.x;
  if (m >= M) return;
  uint32_t bits = 0;
  for (uint32_t e = 0; e < D; e++) bits |= portok[uint64_t(m) * D + e] ? (1u << e) : 0u;
  portbits[m] = bits;
}
// The same bit rows straight from the port matchers (no byte table first): launch B builds them next
// to the byte table when there is no launch A, so the identity sets of launch D can read them.
__device__ __forceinline__ void portbits_direct_blk(uint32_t M, uint32_t D, const DPortM* pms, const DPortEntry* pents,
                                                    const DDesc* descs, uint32_t* __restrict__ portbits, uint32_t bid_) {
  const uint32_t m = bid_ * 256 + threadIdx.x;
  if (m >= M) return;
  const DPortM pm = pms[m];
  uint32_t bits = pm.all ? (D >= 32 ? ~0u : (1u << D) - 1u) : 0u;
  // the matcher's entries PB_ENT at a time, all loaded before any test (one memory round trip per
  // batch, not one per (descriptor, entry)), each tested against every descriptor (block-uniform
  // loads): launch B config #3 81.4 -> 79.9 us, its N = 8 source shard 33 -> 26.5 us (the port bits
  // were that shard's longest chain); 4 at a time: the same times at +5 VGPRs for all of launch B
  // (profiles/r04_front_b_ab.txt)
  constexpr uint32_t PB_ENT = 2;
  for (uint32_t j0 = 0; !pm.all && j0 < pm.ecnt; j0 += PB_ENT) {
    DPortEntry pe[PB_ENT];
#pragma unroll
    for (uint32_t x = 0; x < PB_ENT; x++) pe[x] = pents[pm.eoff + min(j0 + x, pm.ecnt - 1)];
    for (uint32_t e = 0; e < D; e++) {
      const DDesc d = descs[e];
      bool ok = false;
#pragma unroll
      for (uint32_t x = 0; x < PB_ENT; x++)  // raw protocol string compare ("tcp" != "TCP")
        ok = ok || (pe[x].proto == d.proto &&
                    (pe[x].kind == PE_PROTO ? true
                     : pe[x].kind == PE_INT ? pe[x].a == d.port
                     : pe[x].kind == PE_NAME ? uint32_t(pe[x].a) == d.name
                                             : pe[x].a <= d.port && d.port <= pe[x].b));
      bits |= ok ? 1u << e : 0u;
    }
  }
  portbits[m] = bits;
}
__global__ __launch_bounds__(256) void k_portbits(uint32_t M, uint32_t D, const uint8_t* __restrict__ portok,
                                                  uint32_t* __restrict__ portbits) {
  portbits_blk(M, D, portok, portbits, blockIdx.x);
}

// Per (slot k, word w over pods-as-destinations): VALID bits, the word's common descriptor
// (DESCW >= 0), none valid (-2) or mixed (-1), and per-descriptor masks DM for mixed words.
__device__ __forceinline__ void slot_words_blk(uint32_t P, uint32_t K, uint32_t W, uint32_t D,
                                                    const int32_t* __restrict__ slot_desc,
                                                    const uint8_t* __restrict__ slot_status, uint64_t* __restrict__ VALID,
                                                    int32_t* __restrict__ DESCW, uint64_t* __restrict__ DM, uint32_t bid_, uint32_t nblk_) {
  uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t idx = __builtin_amdgcn_readfirstlane(bid_ * 4 + wave);  // (k, w), wave-uniform
  if (idx >= K * W) return;
  uint32_t k = idx / W, w = idx % W;
  uint32_t q = w * 64 + lane;
  int32_t e = -1;
  bool valid = false;
  if (q < P) {
    valid = slot_status[uint64_t(q) * K + k] == CYC_JOB_VALID;
    e = valid ? slot_desc[uint64_t(q) * K + k] : -1;
  }
  uint64_t vm = __ballot(valid);
  // first valid lane's descriptor, broadcast
  int32_t first = -2;
  if (vm) first = __shfl(e, __ffsll((unsigned long long)vm) - 1);
  bool same = !valid || e == first;
  uint64_t sm = __ballot(same);
  int32_t dw = vm == 0 ? -2 : (sm == ~0ull ? first : -1);
  if (lane == 0) {
    VALID[uint64_t(k) * W + w] = vm;
    DESCW[uint64_t(k) * W + w] = dw;
  }
  if (dw == -1) {
    for (uint32_t d = 0; d < D; d++) {
      uint64_t m = __ballot(valid && e == int32_t(d));
      if (lane == 0) DM[(uint64_t(k) * D + d) * W + w] = m;
    }
  }
}
__global__ __launch_bounds__(256) void k_slot_words(uint32_t P, uint32_t K, uint32_t W, uint32_t D,
                                                    const int32_t* __restrict__ slot_desc,
                                                    const uint8_t* __restrict__ slot_status, uint64_t* __restrict__ VALID,
                                                    int32_t* __restrict__ DESCW, uint64_t* __restrict__ DM) { slot_words_blk(P, K, W, D, slot_desc, slot_status, VALID, DESCW, DM, blockIdx.x, gridDim.x); }

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
  uint32_t* rep_cnt;          // set to ~0 by k_member: ends at count - 1
  const uint32_t* id_blk;     // batched blocks: each identity's block (classes never span blocks), else null
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
  if (bid_ == 0 && threadIdx.x == 0) *a.rep_cnt = ~0u;  // k_classify counts up from here
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
  if (bid_ == 0 && threadIdx.x == 0) *a.rep_cnt = ~0u;  // k_classify counts up from here
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
  if (err[i]) return i;
  const uint32_t r0 = ht_find_rep(ht_key, ht_cap, hash[i]);
  const uint32_t r = r0 == 0xFFFFFFFFu ? i : r0;
  if (r == i) return i;
  const uint32_t n = cnt[i], oi = list_off[i], orr = list_off[r];
  bool eq = cnt[r] == n && (!id_blk || id_blk[r] == id_blk[i]);
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
      uint8_t si[8], sr[8];
      int32_t di[8], dr[8];
#pragma unroll
      for (uint32_t u = 0; u < 8; u++) {
        const uint64_t k = min(k0 + u, K - 1);
        si[u] = id_status[uint64_t(i) * K + k];
        sr[u] = id_status[uint64_t(r) * K + k];
        di[u] = id_desc[uint64_t(i) * K + k];
        dr[u] = id_desc[uint64_t(r) * K + k];
      }
#pragma unroll
      for (uint32_t u = 0; u < 8; u++) eq = eq && si[u] == sr[u] && (si[u] != CYC_JOB_VALID || di[u] == dr[u]);
    }
  }
  return eq ? r : i;
}

__device__ __forceinline__ void classify_blk(MemberArgs a, uint32_t* __restrict__ class_of, uint32_t bid_, uint32_t nblk_) {
  __shared__ uint32_t wsum[4], base;
  const uint32_t ii = bid_ * blockDim.x + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool live = ii < a.n_act;
  const uint32_t i = live ? a.act[ii] : 0;
  const uint32_t c = live ? class_of_identity(i, a.err, a.hash, a.ht_key, a.ht_cap, a.cnt, a.list_off, a.list, a.id_blk,
                                              a.id_status, a.id_desc, a.K)
                          : i;
  if (live) class_of[i] = c;
  const bool f = live && c == i;
  const uint64_t m = __ballot(f);
  if (lane == 0) wsum[wv] = __popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) base = atomicAdd(a.rep_cnt, wsum[0] + wsum[1] + wsum[2] + wsum[3]) + 1u;
  __syncthreads();
  uint32_t off = base;
  for (uint32_t x = 0; x < wv; x++) off += wsum[x];
  if (f) a.reps[off + __popcll(m & ((1ull << lane) - 1))] = i;
}
__global__ __launch_bounds__(256) void k_classify(MemberArgs a, uint32_t* __restrict__ class_of) { classify_blk(a, class_of, blockIdx.x, gridDim.x); }


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
};

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
// Identity words [ew0, ew0 + new) of the rows only (a source shard's ingress peers: the words of the
// egress identities its sources have).
__device__ __forceinline__ void peer_bits_blk(uint32_t Rp, uint32_t E, uint32_t EW, const uint32_t* __restrict__ pod_peers,
                                                   const DPeer* __restrict__ peers, const SelView& sv,
                                                   const uint32_t* __restrict__ id_ns, const uint32_t* __restrict__ id_nsls,
                                                   const uint32_t* __restrict__ id_ls, uint64_t* __restrict__ idob, uint32_t bid_, uint32_t nblk_,
                                                   uint32_t ew0, uint32_t new_, const uint2* __restrict__ grp_ns,
                                                   const uint2* __restrict__ word_ns) {
  // the wave index is wave-uniform: a scalar, so the peers' records below are scalar loads
  const uint32_t wv = __builtin_amdgcn_readfirstlane(bid_ * 4 + (threadIdx.x >> 6)), lane = threadIdx.x & 63;
  const uint32_t groups = (Rp + PB_GROUP - 1) / PB_GROUP;
  if (wv >= groups * new_) return;
  const uint32_t g = wv / new_, ew = ew0 + wv % new_;
  {  // a group of exact-namespace peers (podpeermatcher.go:115-125: ns == the policy's namespace) whose
     // namespaces the word's identities do not have matches none of them: zeros, no selector loads
    const uint2 gr = grp_ns[g], wr = word_ns[ew];
    if (gr.y < wr.x || gr.x > wr.y) {
      const uint32_t p = g * PB_GROUP + lane;
      if (lane < PB_GROUP && p < Rp) idob[uint64_t(p) * EW + ew] = 0;
      return;
    }
  }
  const uint32_t e = ew * 64 + lane;
  const bool live = e < E;
  const uint32_t ns = live ? id_ns[e] : 0u, nsls = live ? id_nsls[e] : 0u, ls = live ? id_ls[e] : 0u;
  uint64_t mine = 0;
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
  if (r >= *a.rep_cnt + 1u) return;
  const uint32_t i = a.reps[r];
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
  if (r >= *a.rep_cnt + 1u) return;
  const uint32_t i = a.reps[r];
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
  const uint32_t n_reps = *a.rep_cnt + 1u, nkc = (a.K + KC - 1) / KC;
  const bool kbits = EGRESS ? a.portbits != nullptr : a.K <= 32;
  for (uint32_t r = bid_; r < n_reps; r += nblk_) {
    const uint32_t i = a.reps[r];
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
  const uint32_t r0 = (bid_ / (cg * nkc)) * a.rpb, n_reps = *a.rep_cnt + 1u;
  if (r0 >= n_reps) return;  // whole block
  const uint32_t nr = min(a.rpb, n_reps - r0), k0 = kc * KC;
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
    h.i = a.reps[r0 + threadIdx.x];
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
  uint32_t nb[11];      // IP rows x2 | pod-peer rows x2 (or identity sets, segment 2) | membership in | eg | port bits |
                        // port table | slot words (the last two: runs without launch A, enq_front_fused) |
                        // IP rows from address ranges x2
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
        return pod_rows_direct_blk<false>(f.Rp[x], f.P, f.W, f.plist[x], f.peers, f.selres, f.L, f.pod_eid, f.id_ns, f.id_nsls,
                                          f.id_ls, f.PM, nullptr, b, f.nb[2 + x], f.pw0[x], f.pnw[x]);
      return peer_bits_blk(f.Ru_[x], f.E, f.EW, f.pod_peers_u_[x], f.peers, f.sv, f.id_ns, f.id_nsls, f.id_ls, f.idob_[x], b,
                           f.nb[2 + x], f.ew0[x], f.new_[x], f.grp_ns_[x], f.word_ns);
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
  // the IP rows' word-span records (RowArgs::ip_rng), reset to ~0 for the NEXT run in block slices
  // (their readers are all done): no fill launch or memset node before the next front
  uint32_t* reset;
  uint64_t reset_n;
  uint32_t buf;        // 56-104 KB rows through k_emit_wide_buf<512,13> (else k_emit_wide<1024,7>)
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
  for (uint32_t x0 = threadIdx.x; x0 < n2; x0 += BS * UNROLL) {
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
  const uint32_t bytes = uint32_t(a.row_words * 8);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint64_t*>(si), 0, bytes, BUF_RSRC_W3);
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(di, 0, bytes, BUF_RSRC_W3);
  for (uint32_t x0 = 0; x0 < bytes; x0 += BS * UNROLL * 16) {
    u32x4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, threadIdx.x * 16, x0 + u * BS * 16, 0);
#pragma unroll
    for (int u = 0; u < UNROLL; u++) __builtin_amdgcn_raw_buffer_store_b128(v[u], rd, threadIdx.x * 16, x0 + u * BS * 16, 2);  // nt
  }
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
    const uint32_t bytes = uint32_t(a.pl_words[pl] * 8);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<u64x2*>(s_src[0]), 0, bytes, BUF_RSRC_W3);
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(s_dst[0], 0, bytes, BUF_RSRC_W3);
    for (uint32_t x0 = 0; x0 < bytes; x0 += BS * UNROLL * 16) {
      u32x4 v[UNROLL];
#pragma unroll
      for (int q = 0; q < UNROLL; q++) v[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, threadIdx.x * 16, x0 + q * BS * 16, 0);
#pragma unroll
      for (int q = 0; q < UNROLL; q++) __builtin_amdgcn_raw_buffer_store_b128(v[q], rd, threadIdx.x * 16, x0 + q * BS * 16, 2);  // nt
    }
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

// ---------------------------------------------------------------- panic path (rare)
struct ErrArgs {
  uint32_t P, K, W, n_cfg;
  uint32_t row_lo, row_hi;
  uint32_t src;                    // source-row run: rows [row_lo, row_hi) are sources for both directions
  uint32_t w0, WA;                 // ingress class rows' word window (RowArgs)
  const uint8_t* slot_status;  // [P][K]
  const uint32_t *slot_cfg, *slot_idx;
  const uint32_t *pod_iid, *pod_eid, *class_in, *class_eg;
  const uint8_t *err_in, *err_eg;  // per identity: a target selector panics
  const uint64_t *AE_in, *AE_eg;
  unsigned long long* first;       // [n_cfg] min job-order key within each probe config
};

// Per probe config (each config is its own table, built in order: the lowest config with a panic
// is the one the reference hits first), key = (s*P + d)*65536 + idx_in_cfg = the reference's job
// order (resources.go:286-333).  The host guarantees P < 2^24 and idx < 65536 on this path, so the
// key never overflows.  Grid-stride over (s, 256-destination chunk): no grid-size limit on P.
__global__ __launch_bounds__(256) void k_first_error(ErrArgs a) {
  const uint64_t chunks = (a.P + 255) / 256, n = chunks * a.P;
  for (uint64_t b = blockIdx.x; b < n; b += gridDim.x) {
    const uint32_t s = uint32_t(b / chunks);
    const uint32_t d = uint32_t(b % chunks) * blockDim.x + threadIdx.x;
    if (d >= a.P) continue;
    // only the directions whose rows this run computes (the whole table when [lo,hi) = [0,P)); a
    // source-row run computes both directions of its sources' cells
    const bool sin = s >= a.row_lo && s < a.row_hi, din = a.src ? sin : d >= a.row_lo && d < a.row_hi;
    if (!din && !sin) continue;
    const bool s_err = sin && a.err_eg[a.pod_eid[s]];
    const bool d_err = din && a.err_in[a.pod_iid[d]];
    const uint32_t ci = din ? a.class_in[a.pod_iid[d]] : 0, ce = sin ? a.class_eg[a.pod_eid[s]] : 0;
    uint32_t cfg = 0xFFFFFFFFu;
    unsigned long long best = ~0ull;
    for (uint32_t k = 0; k < a.K; k++) {
      if (a.slot_status[uint64_t(d) * a.K + k] != CYC_JOB_VALID) continue;
      bool e = d_err || s_err;
      if (!e && din && a.AE_in) e = (a.AE_in[(uint64_t(ci) * a.K + k) * a.WA + (s / 64 - a.w0)] >> (s % 64)) & 1;
      if (!e && sin && a.AE_eg) e = (a.AE_eg[(uint64_t(ce) * a.K + k) * a.W + d / 64] >> (d % 64)) & 1;
      if (!e) continue;
      const uint32_t kc = a.slot_cfg[k];
      const unsigned long long key = (uint64_t(s) * a.P + d) * 65536ull + a.slot_idx[k];
      if (kc != cfg) {  // slots of one config are contiguous, configs ascending
        if (best != ~0ull) atomicMin(&a.first[cfg], best);
        cfg = kc;
        best = key;
      } else {
        best = key < best ? key : best;
      }
    }
    if (best != ~0ull) atomicMin(&a.first[cfg], best);
  }
}

// ---------------------------------------------------------------- single-cell queries
// Policy.IsTrafficAllowed (policy.go:131-174) for arbitrary matcher.Traffic values, one thread per
// traffic.  Endpoint 2i is the source, 2i+1 the destination; ext[e] = Internal == nil.
// res[i] = ingress | egress << 1; pan[i] = panic code | (string kind << 8), pid[i] = string id.
struct QueryArgs {
  uint32_t n, L, D;
  const uint32_t *pod_ns, *pod_ls, *pod_nsls, *ext, *tdesc;
  const DIP* pod_ip;
  const uint8_t* selres;
  const uint8_t* portok;
  const DTarget* tgt[2];
  const uint32_t *tns_lo[2], *tns_hi[2];
  const DPeer* peers;
  const DIPBlock* ipbs;
  const DCidr* cidrs;
  const uint32_t* ipb_ex;
  uint8_t* res;
  uint32_t *pan, *pid;
  uint8_t* tflags;        // optional: per (traffic, direction) matching-target verdicts
  const uint64_t* toff;   // [n][2] offsets into tflags (entry t - tns_lo: 0 no match, 1 allows, 2 denies)
  uint32_t members_only;  // query-target: TargetsApplyingToPod only (flag 1 = applies)
};

enum { QP_NONE = 0, QP_SELECTOR = 1, QP_IP = 2, QP_CIDR = 3 };

// returns 1 allowed / 0 denied, or sets *code and returns 2 (panic)
__device__ uint32_t query_direction(const QueryArgs& a, int dir, uint32_t T, uint32_t Q, uint32_t desc, uint32_t* code,
                                    uint32_t* sid, uint8_t* fl) {
  if (a.ext[T]) return 1;  // policy.go:151-153
  const uint32_t ns = a.pod_ns[T], ls = a.pod_ls[T];
  const uint32_t lo = a.tns_lo[dir][ns], hi = a.tns_hi[dir][ns];
  uint32_t nmatch = 0;
  for (uint32_t t = lo; t < hi; t++) {  // TargetsApplyingToPod evaluates every target first
    uint8_t r = a.selres[uint64_t(a.tgt[dir][t].sel) * a.L + ls];
    if (r == 2) {
      *code = QP_SELECTOR;
      return 2;
    }
    nmatch += r;
  }
  if (a.members_only) {  // analyze.go:189-192 TargetsApplyingToPod
    if (fl)
      for (uint32_t t = lo; t < hi; t++) fl[t - lo] = a.selres[uint64_t(a.tgt[dir][t].sel) * a.L + ls];
    return 1;
  }
  if (nmatch == 0) return 1;  // :158-160
  uint32_t allowed = 0;
  for (uint32_t t = lo; t < hi; t++) {
    if (a.selres[uint64_t(a.tgt[dir][t].sel) * a.L + ls] != 1) continue;
    DTarget tg = a.tgt[dir][t];
    uint32_t tallow = 0;  // policy.go:165-171: this target goes to AllowingTargets or DenyingTargets
    for (uint32_t j = tg.poff; j < tg.poff + tg.pcnt; j++) {  // Target.Allows: every matching target runs
      DPeer pr = a.peers[j];
      if (pr.kind == 0) {
        tallow = 1;
        break;
      }
      bool pok = a.portok[uint64_t(pr.port) * a.D + desc] != 0;
      if (pr.kind == 1) {
        if (pok) {
          tallow = 1;
          break;
        }
        continue;
      }
      uint32_t o;
      if (pr.kind == 2) {
        if (a.ext[Q]) continue;  // podpeermatcher.go:22-24
        o = pod_peer_outcome(pr, a.selres, a.L, a.pod_ns[Q], a.pod_nsls[Q], a.pod_ls[Q]);
        if (o == 2) {
          *code = QP_SELECTOR;
          return 2;
        }
      } else {
        DIPBlock b = a.ipbs[pr.ipb];
        if (!a.cidrs[b.cidr].valid) {
          *code = QP_CIDR;
          *sid = b.cidr;
          return 2;
        }
        DIP ip = a.pod_ip[Q];
        if (!ip.valid) {
          *code = QP_IP;
          *sid = Q;
          return 2;
        }
        o = ip_peer_outcome(b, a.cidrs, a.ipb_ex, ip);
        if (o == 2) {  // an except failed to parse: find which (evaluation order)
          for (uint32_t e = 0; e < b.excnt; e++) {
            uint32_t x = a.ipb_ex[b.exoff + e];
            if (!a.cidrs[x].valid) {
              *code = QP_CIDR;
              *sid = x;
              return 2;
            }
            if (cidr_contains(a.cidrs[x], ip)) break;
          }
        }
      }
      if (o == 1 && pok) {
        tallow = 1;
        break;
      }
    }
    allowed |= tallow;
    if (fl) fl[t - lo] = tallow ? 1 : 2;
  }
  return allowed;
}

__global__ void k_query(QueryArgs a) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  uint32_t code = 0, sid = 0;
  uint8_t* fi = a.tflags ? a.tflags + a.toff[2 * i] : nullptr;
  uint8_t* fe = a.tflags ? a.tflags + a.toff[2 * i + 1] : nullptr;
  uint32_t in = query_direction(a, 0, 2 * i + 1, 2 * i, a.tdesc[i], &code, &sid, fi);
  uint32_t eg = 0;
  if (in != 2) eg = query_direction(a, 1, 2 * i, 2 * i + 1, a.tdesc[i], &code, &sid, fe);
  a.res[i] = uint8_t((in == 1 ? 1 : 0) | (eg == 1 ? 2 : 0));
  a.pan[i] = code;
  a.pid[i] = sid;
}


// ---------------------------------------------------------------- table cells (lazy probe.Table)
// One (source s, destination d, job slot k) cell per thread, as the reference's Table would hold
// it after NewTableFromJobResults (table.go:38-48): VALID jobs take Ingress / Egress from the
// planes and Combined = both allowed (jobrunner.go:85-93); BadPortProtocol and BadNamedPort jobs
// get the fixed results of jobrunner.go:36-55; slots without a job are CYC_CONN_NO_JOB.
struct CellArgs {
  uint32_t K, W, row_lo, row_hi;
  uint32_t src, w0, WA;      // source-row table: ingress rows of every destination over words [w0, w0 + WA)
  const uint64_t *in, *eg;   // planes of rows [row_lo, row_hi) (layout: include/cyclonus_hip.h)
  const uint8_t* status;     // [P][K]
  uint32_t s_lo, d_lo, k_lo, nd, nk;
  uint64_t n;                // cells
  uint8_t *o_in, *o_eg, *o_comb;  // each optional
};
__global__ __launch_bounds__(256) void k_table_cells(CellArgs a) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < a.n; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t k = a.k_lo + uint32_t(i % a.nk);
    const uint64_t sd = i / a.nk;
    const uint32_t d = a.d_lo + uint32_t(sd % a.nd), s = a.s_lo + uint32_t(sd / a.nd);
    const uint8_t st = a.status[uint64_t(d) * a.K + k];
    uint8_t ci = CYC_CONN_NO_JOB, ce = CYC_CONN_NO_JOB, cc = CYC_CONN_NO_JOB;
    if (st == CYC_JOB_VALID) {
      // the host checked that the requested planes cover these rows
      const uint64_t iw = a.src ? (uint64_t(d) * a.K + k) * a.WA + (s / 64 - a.w0) : (uint64_t(d - a.row_lo) * a.K + k) * a.W + s / 64;
      const bool ai = a.o_in || a.o_comb ? (a.in[iw] >> (s % 64)) & 1 : false;
      const bool ae = a.o_eg || a.o_comb ? (a.eg[(uint64_t(s - a.row_lo) * a.K + k) * a.W + d / 64] >> (d % 64)) & 1 : false;
      ci = ai ? CYC_CONN_ALLOWED : CYC_CONN_BLOCKED;
      ce = ae ? CYC_CONN_ALLOWED : CYC_CONN_BLOCKED;
      cc = ai && ae ? CYC_CONN_ALLOWED : CYC_CONN_BLOCKED;
    } else if (st == CYC_JOB_BAD_PORT_PROTOCOL) {
      ci = cc = CYC_CONN_INVALID_PORT_PROTOCOL;
      ce = CYC_CONN_UNKNOWN;
    } else if (st == CYC_JOB_BAD_NAMED_PORT) {
      ci = cc = CYC_CONN_INVALID_NAMED_PORT;
      ce = CYC_CONN_UNKNOWN;
    }
    if (a.o_in) a.o_in[i] = ci;
    if (a.o_eg) a.o_eg[i] = ce;
    if (a.o_comb) a.o_comb[i] = cc;
  }
}

}  // namespace cyc

// ============================================================================ context + C ABI
using namespace cyc;

#define HIPCHK(x)                                                                   \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) throw HipErr{std::string(#x) + ": " + hipGetErrorString(e_)}; \
  } while (0)

namespace {
struct HipErr {
  std::string msg;
};

// Makes `device` current for the scope of an entry point and restores the caller's current device
// afterwards: a binding calling in from a thread whose current device is another GPU (e.g. PyTorch
// on cuda:1 with a context on device 0) keeps its own current device.
// Events of a run (stream order, completion, phase timing) release to device scope: a default
// (system-scope) event writes back and invalidates the caches when it is recorded, which left a
// ~15 us idle gap after every step's emit (config #3 timeline, r04c) and inflated the phase timings.
// Nothing here hands memory to the host through an event: host reads are hipMemcpy calls.
constexpr unsigned EV_SYNC = hipEventDisableTiming | hipEventReleaseToDevice;
constexpr unsigned EV_TIMING = hipEventReleaseToDevice;

struct DeviceGuard {
  int prev = -1;
  bool set = false;
  explicit DeviceGuard(int device, bool strict = true) {
    hipError_t e = hipGetDevice(&prev);
    if (e == hipSuccess && prev == device) return;
    e = hipSetDevice(device);
    if (e != hipSuccess) {
      if (strict) throw HipErr{std::string("hipSetDevice: ") + hipGetErrorString(e)};
      return;
    }
    set = prev >= 0;
  }
  ~DeviceGuard() {
    if (set) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  void alloc(size_t n) {
    if (p) {
      (void)hipFree(p);
      p = nullptr;
    }
    bytes = n;
    if (n) HIPCHK(hipMalloc(&p, n));
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

template <class T>
void upload(DevBuf& b, const std::vector<T>& v) {
  b.alloc(std::max<size_t>(v.size() * sizeof(T), 16));
  if (!v.empty()) HIPCHK(hipMemcpy(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
}

struct Identities {  // pod identities for one direction
  std::vector<uint32_t> ns, ls, nsls, list_off;
  std::vector<int32_t> desc;     // ingress: [n][K]
  std::vector<uint8_t> status;   // ingress: [n][K]
  std::vector<uint32_t> of_pod;  // [P]
  uint64_t list_total = 0;
  uint32_t ht_cap = 0;
};

struct DirDev {
  DevBuf id_ns, id_ls, id_desc, id_status, list_off, list, cnt, hash, err, ht_key, ht_rep, class_of, A, AE, tns_lo,
      tns_hi, tgt, pod_id, reps, B, ip_off, ip_cnt, ip_list;
  uint32_t n = 0, ht_cap = 0;
  // hash table buffer = [cap] u64 keys, [cap] u32 reps, 1 u32 representative counter: one
  // 0xFF memset per run empties the table and sets the counter to ~0 (= count - 1 for 0)
  uint32_t* rep_cnt() { return reinterpret_cast<uint32_t*>(static_cast<char*>(ht_key.p) + uint64_t(ht_cap) * 16); }
};
}  // namespace

struct PeerPlan {
  std::vector<uint32_t> pod_peers, ip_peers, word_off, run_e;
  std::vector<uint64_t> run_mask;
  std::vector<DIPTest> ip_tests;
  std::vector<DCidr> ip_ex;
  uint32_t max_runs = 0;  // most identity runs in one 64-pod word
  std::vector<WordRuns> runs;  // [W] when max_runs <= IDO_MAX_RUNS
};
struct cyc_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  bool have_policy = false, have_res = false, prepared = false;
  PolicyIR policy;
  Resources res;
  Problem pb;
  Identities ids[2];
  // device tables
  DevBuf ls_off, ls_key, ls_val, sel_off, reqs, req_vals, pod_ns, pod_ls, pod_nsls, pod_ip, cidrs, ipbs, ipb_ex, pms,
      pents, peers, descs, slot_desc, slot_status, slot_cfg, slot_idx;
  DevBuf selres, PM, ER, portok, portbits, VALID, DESCW, DM, first_err, order[2];
  DevBuf status_sink;  // status plane target of graph runs given no status pointer (see capture_pipeline)
  // peer-row stage: pod peers in identity space + per-word identity runs; IP peers per pod
  DevBuf pod_peers_u;  // identity-set (IDOB) rows: the needed pod peers, one per distinct
                       // (namespace matcher, pod selector) of a direction (peer_ido maps every peer)
  DevBuf pod_peers, ip_peers, ip_tests, ip_ex, id_nsls, word_off, run_e, run_mask, ido, ip_words, peer_ido, peer_row, zeros, idob, runs, ip_rng, lvt, dreqs;
  std::vector<uint32_t> prow_host;  // peer_row on the host (the panic describer reads PM / ER rows by it)
  DevBuf udesc;     // per slot the one VALID descriptor every pod has, when all slots are so (uni_desc)
  bool uni_desc = false;
  DevBuf plvt;      // LVT per pod (SelView::PLVT), built by ensure_plvt when it fits PLVT_MAX_BYTES
  uint32_t n_lkeys = 0;     // dense label keys (LVT rows - 1)
  bool plvt_ready = false;
  int64_t plvt_max_mb = 1024;  // "plvt_max_mb": largest PLVT built (0: never, the LVT gathers instead)
  DevBuf sel_one;   // SelView::one
  DevBuf req_post, post_pods;  // label postings: per requirement (offset, count) x 2 values; pod lists
  std::vector<uint8_t> req_post_ok;  // the requirement's pods are its postings (EQ, IN of <= 2 values)
  DevBuf pp_scan, pp_post;     // sparse pod rows: pod peers scanned per word / built from postings
  uint32_t n_scan = 0, n_post = 0;
  DevBuf ns_words;  // DWordNS per 64-pod word, then per 64-word chunk (sparse pod rows)
  bool dense_sel = false;  // k_selectors_dense (LVT fits)
  uint32_t Rp = 0, Ri = 0;
  uint32_t rp_off[3] = {0, 0, 0}, ri_off[3] = {0, 0, 0};  // per-direction sub-lists (ingress, egress)
  // IP rows built from address ranges (ip_rows_range_blk): the pods of each family sorted by
  // address (host keys for the binary searches; the pod order on the device), and per direction the
  // range-built rows
  std::vector<uint32_t> ip4_key, ipsort_host;
  std::vector<uint8_t> word_aff;  // per 64-pod word: bit f set when family f's pods there are affine (or absent)
  std::vector<std::array<uint32_t, 4>> ip6_key;
  DevBuf ipsort, ipr_tests, ipr_iv;
  uint32_t rr_off[3] = {0, 0, 0}, Rr = 0;
  uint32_t rpu_off[3] = {0, 0, 0};  // sub-lists of pod_peers_u: one pod peer per distinct matcher
  DevBuf ipi_items, ipi_list;   // IP-row work items of the fused front (DIPItem; ip_rows_items_blk) and their rows
  uint32_t ipi_off[3] = {0, 0, 0};  // items of segment x: [ipi_off[x], ipi_off[x + 1])
  bool ip_items = false;        // the current plan's items are built (option "ip_items" on and fast IP rows present)
  int ip_items_opt = -1;        // "ip_items": -1 auto (on) / 0 / 1
  std::vector<DWordIP> ipw_h;   // host copy of the IP word and chunk records (ip_words)
  DevBuf ido_grp_ns, ido_word_ns;  // identity-set namespace skip (peer_bits_blk): per row group, per identity word
  uint32_t ido_goff[2] = {0, 0};   // first group of each direction's sub-list in ido_grp_ns
  PeerPlan plan;                 // all pod / IP peers (host); filtered per row range
  DevBuf act[2], actrec[2], sel_list;
  DevBuf arow[2];  // per identity: its first pod's row in the run's row range (in-place class rows)
  uint32_t n_act[2] = {0, 0}, n_sel = 0;
  double act_targets[2] = {0, 0};  // mean namespace targets per active identity (range plan)
  // Diagnostic path selectors (cyc_set_option; results never change, the GPU tests force each path):
  int use_graphs = -1;  // "graphs": 1 = graph replay, 2 = the same DAG enqueued eagerly on three
                        // streams with events (no graph launch), 0 = eager on one stream with phase
                        // events, -1 = auto: 2 when the fused front applies (its launches on one
                        // stream start ~8 us sooner after the previous step's emit than a graph
                        // replay: profiles/r01_front_fused_ab.txt), else 1
  int ip_range = -1;    // "ip_range": IP rows of few, close pods from the address index: -1 auto (where the
                        // words are not affine), 1 wherever they fit, 0 never
  int pod_rows = -1;    // "pod_rows": pod-peer PM rows per pod directly (1), through identity outcomes
                        // and word runs (0), or -1 = direct when identities >= pods / 2
  int member_wave = -1; // "member_wave": membership with a wave (1) or a thread (0) per identity,
                        // -1 = auto by identity count
  int pod_words = -1;   // "pod_words": pod-peer words in the class rows from identity sets (1, IDO),
                        // from materialised PM rows (0), or IDO when every word has <= IDO_MAX_RUNS runs
  int64_t class_rpb_opt = 0;  // "class_rpb": IDO class-row representatives per block; 0 = auto
                              // (profiles/r04_class_rpb_ab.txt)
  int step_events = 0;  // "step_events": graph / eager-DAG runs record the whole-step timing events (1);
                        // off by default: the two timing events cost ~9 us of idle GPU per step
                        // (config #2 0.077 -> 0.069 ms/step, profiles/r02_step_events_ab.txt)
  int pl_wave = 1;      // "pl_wave": PM-build class rows a wave per 64-word chunk where they fit (1),
                        // or a thread per (slot chunk, word) item (0)
  int class_inplace = -1; // "class_inplace": fused-front class rows written straight into the output
                          // planes (the first member pod's row), the emit copying only the others (1);
                          // -1 = auto (inplace_ok)
  int pr_group = -1;   // "pr_group": sparse pod-peer rows, pod peers per block (1..64; -1 = auto)
  int sel_lazy = -1;    // "sel_lazy": selectors evaluated where used (1) or as the dense SELRES table
                        // first (0); -1 = lazy on the fused front of PM builds
  int front_fused = 1;  // "front_fused": the front as block-range-fused launches on one stream
                        // (enq_front_fused), 0 = the two-branch DAG
  int emit_interleave = -1;  // "emit_interleave": a target-row emit's row list alternates the planes'
                             // rows (1) or is [plane 0][plane 1] (0); -1 = auto (planes >= 8 GB)
  int emit_split = 1;   // "emit_split": a target-row emit as this many launches over consecutive parts
                        // of each plane's row list (1..8)
  int emit_buf = 2;      // "emit_buf": 56-104 KB plane rows through 1024 x 7 buffer-op blocks (2), 512 x 13
                         // buffer-op blocks (1) or 1024 x 7 flat-address blocks (0).  The emit's rate depends
                         // on the planes' physical placement; over 14 placements of config #3's planes 1024 x 7
                         // averaged 3.389 ms per step against 3.542 for 512 x 13 (1-2 % behind on the best
                         // placements, up to 8 % ahead on the worst; a target shard at N = 8 -5.7 %),
                         // profiles/r05_plane_placement.txt, r05_shard_ab.txt
  // what the last enqueued emit launched (cyc_last_emit): kernel name(s) and launch count
  std::string emit_kernel;
  int emit_launches = 0;
  hipStream_t cap_stream = nullptr, cap_stream2 = nullptr, cap_stream3 = nullptr;  // graph capture branches
  hipEvent_t fork_ev = nullptr, join_ev = nullptr, sel_ev = nullptr, ports_ev = nullptr;
  hipGraphExec_t graph_exec = nullptr;
  hipGraph_t graph = nullptr;  // kept alive with its exec
  hipEvent_t graph_done = nullptr;  // recorded on the caller's stream after each launch of graph_exec
  // An exec replaced by a re-capture (new output pointers, row range or tuning knob) may still have
  // a launch queued on the caller's stream: cyc_probe_run returns without synchronising.  It is
  // retired with the event recorded after its last launch and destroyed only once that event has
  // completed (reap_graphs).  Destroying it at once freed an exec a queued launch still used — the
  // intermittent crash inside hipGraphLaunch seen in round 1.
  struct Retired {
    hipGraphExec_t exec;
    hipGraph_t graph;
    hipEvent_t done;  // null: never launched
  };
  std::vector<Retired> retired;
  const void* graph_key[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  bool timed_graph = false;
  DirDev dir[2];
  int64_t order_lo = -1, order_hi = -1;
  bool order_src = false;  // the range plan partitions sources (CYC_ROWS_SOURCE), not target rows
  // the current plan: plane rows per direction (ingress keyed by destination, egress by source) and
  // the ingress word window (a source shard's sources: its peers' rows and class rows cover only
  // those words); target-row plans: both directions [lo, hi), window [0, W)
  int64_t rl[2] = {0, 0}, rh[2] = {0, 0};
  uint32_t win_w0 = 0, win_wa = 0;
  uint32_t ido_ew0 = 0, ido_ew1 = 0;  // ingress identity sets: egress-identity words of the window's sources
  uint32_t scan_off[3] = {0, 0, 0}, post_off[3] = {0, 0, 0};  // pp_scan / pp_post: ingress peers, then egress
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  double last_ms[3] = {0, 0, 0};
  bool timed = false;  // the last run recorded the step timing events
  // the IP rows' word-span records are all ~0: the last enqueued run's emit reset them (EmitArgs::reset),
  // so the next fused front needs no fill before its IP rows (and, without a selector table, no launch A)
  bool ip_rng_clean = false;
  bool capturing = false;  // a hipGraph capture is in progress (captured steps always fill the spans themselves)
  bool ran = false;    // a run has been enqueued
  hipEvent_t run_done = nullptr;  // recorded on the run's stream after every run (cyc_last_classes)
  // batched blocks (cyc_probe_prepare_blocks; pb.blocks non-empty)
  DevBuf blk, blk_off, id_blk[2], id_win[2], first_blk;
  uint32_t blk_wa_max = 0, blk_np_max = 0;
  std::vector<uint64_t> blk_off_h;          // per block: plane slab offset (words), status offset (bytes); then totals
  std::vector<int> blk_rc;                  // per block status of the last run
  std::vector<std::string> blk_msg;         // and its message
};

int describe_panic(cyc_ctx* c, uint32_t s, uint32_t d, uint32_t cfg, uint32_t idx);
static bool rows_layout(const cyc_ctx* c, int part, int64_t lo, int64_t hi, int64_t v[5], std::string& why);

static int fail(cyc_ctx* c, int code, const std::string& m) {
  if (c) c->err = m;
  return code;
}

template <class F>
static int guarded(cyc_ctx* c, F&& f) {
  try {
    return f();
  } catch (Panic& p) {
    return fail(c, p.code, p.msg);
  } catch (HipErr& h) {
    return fail(c, CYC_ERR_HIP, h.msg);
  } catch (std::bad_alloc&) {
    return fail(c, CYC_ERR_OOM, "host allocation failed");
  } catch (std::exception& e) {
    return fail(c, CYC_ERR_JSON, e.what());
  }
}

static inline uint64_t hmix(uint64_t z) {  // splitmix64 finaliser (host)
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Pod identities per direction, numbered by first appearance in pod order: egress (namespace, label
// set), ingress (namespace, label set, every slot's job status and descriptor).  Hashed into an
// open-addressing table whose entries hold their first pod; a probe compares the pods' fields.
static void build_identities(cyc_ctx* c) {
  Problem& pb = c->pb;
  const uint32_t K = pb.K;
  uint32_t cap = 2;
  while (cap < 2 * std::max<uint32_t>(pb.P, 1)) cap <<= 1;
  std::vector<uint32_t> slot_pod(cap), slot_id(cap);
  for (int d = 0; d < 2; d++) {
    Identities& I = c->ids[d];
    I = Identities{};
    I.of_pod.resize(pb.P);
    const bool slots = d == 0 && K;  // the ingress identity includes the pod's job descriptors
    std::fill(slot_pod.begin(), slot_pod.end(), UINT32_MAX);
    for (uint32_t p = 0; p < pb.P; p++) {
      uint64_t h = hmix((uint64_t(pb.pod_ns[p]) << 32) | pb.pod_ls[p]);
      if (slots)
        for (uint32_t k = 0; k < K; k++)
          h = hmix(h ^ (uint64_t(uint32_t(pb.slot_desc[size_t(p) * K + k])) << 8 | pb.slot_status[size_t(p) * K + k]));
      uint32_t x = uint32_t(h) & (cap - 1);
      for (;; x = (x + 1) & (cap - 1)) {
        const uint32_t q = slot_pod[x];
        if (q == UINT32_MAX) break;
        if (pb.pod_ns[q] == pb.pod_ns[p] && pb.pod_ls[q] == pb.pod_ls[p] &&
            (!slots || (memcmp(&pb.slot_desc[size_t(q) * K], &pb.slot_desc[size_t(p) * K], 4 * size_t(K)) == 0 &&
                        memcmp(&pb.slot_status[size_t(q) * K], &pb.slot_status[size_t(p) * K], K) == 0)))
          break;
      }
      if (slot_pod[x] == UINT32_MAX) {
        slot_pod[x] = p;
        slot_id[x] = uint32_t(I.ns.size());
        I.ns.push_back(pb.pod_ns[p]);
        I.ls.push_back(pb.pod_ls[p]);
        I.nsls.push_back(pb.pod_nsls[p]);
        if (d == 0)
          for (uint32_t k = 0; k < K; k++) {
            I.desc.push_back(pb.slot_desc[size_t(p) * K + k]);
            I.status.push_back(pb.slot_status[size_t(p) * K + k]);
          }
      }
      I.of_pod[p] = slot_id[x];
    }
    I.list_off.resize(I.ns.size());
    uint64_t tot = 0;
    for (size_t i = 0; i < I.ns.size(); i++) {
      I.list_off[i] = uint32_t(tot);
      tot += pb.tns_hi[d][I.ns[i]] - pb.tns_lo[d][I.ns[i]];
      if (tot > 0xFFFFFFFFull) throw Panic{CYC_ERR_OOM, "membership lists exceed 2^32 entries"};
    }
    I.list_total = tot;
    uint32_t hc = 2;
    while (hc < 2 * I.ns.size()) hc <<= 1;
    I.ht_cap = hc;
  }
}

// Host side of the peer-row stage: which peers are pod peers / IP peers, and for every 64-pod
// word the runs of equal egress identity (a pod peer's outcome is a function of that identity).
static PeerPlan plan_peers(const Problem& pb, const Identities& eg) {
  PeerPlan pl;
  for (uint32_t j = 0; j < pb.peers.size(); j++) {
    if (pb.peers[j].kind == PK_POD) pl.pod_peers.push_back(j);
    else if (pb.peers[j].kind == PK_IP) {
      pl.ip_peers.push_back(j);
      const DIPBlock& b = pb.ipbs[pb.peers[j].ipb];
      DIPTest t{};
      t.peer = j;
      t.exoff = uint32_t(pl.ip_ex.size());
      t.excnt = b.excnt;
      t.cidr = pb.cidrs[b.cidr];
      for (uint32_t e = 0; e < b.excnt; e++) pl.ip_ex.push_back(pb.cidrs[pb.ipb_ex[b.exoff + e]]);
      pl.ip_tests.push_back(t);
    }
  }
  pl.word_off.push_back(0);
  for (uint32_t w = 0; w < pb.W; w++) {
    uint32_t q0 = w * 64, q1 = std::min<uint32_t>(pb.P, q0 + 64);
    for (uint32_t q = q0; q < q1; q++) {
      uint32_t e = eg.of_pod[q];
      size_t start = pl.word_off.back();
      size_t x = pl.run_e.size();
      // merge with an earlier run of the same identity in this word (keeps runs short)
      size_t hit = x;
      for (size_t y = start; y < x; y++)
        if (pl.run_e[y] == e) {
          hit = y;
          break;
        }
      if (hit == x) {
        pl.run_e.push_back(e);
        pl.run_mask.push_back(0);
      }
      pl.run_mask[hit] |= 1ull << (q - q0);
    }
    pl.word_off.push_back(uint32_t(pl.run_e.size()));
    pl.max_runs = std::max(pl.max_runs, pl.word_off.back() - pl.word_off[pl.word_off.size() - 2]);
  }
  if (pl.max_runs <= IDO_MAX_RUNS) {
    pl.runs.assign(pb.W, WordRuns{});
    for (uint32_t w = 0; w < pb.W; w++)
      for (uint32_t x = pl.word_off[w]; x < pl.word_off[w + 1]; x++) {
        pl.runs[w].e[x - pl.word_off[w]] = pl.run_e[x];
        pl.runs[w].m[x - pl.word_off[w]] = pl.run_mask[x];
      }
  }
  return pl;
}

static uint64_t ido_b_bytes(const cyc_ctx* c, int d) {
  const uint64_t EW = (c->ids[1].ns.size() + 63) / 64, D = std::max<size_t>(c->pb.descs.size(), 1);
  return uint64_t(c->ids[d].ns.size()) * (d == 0 ? c->pb.K : D) * EW * 8;
}

static uint64_t ido_lds_bytes(const cyc_ctx* c) {  // k_class_rows_ido: staged identity-set rows
  const uint64_t EW = (c->ids[1].ns.size() + 63) / 64, D = std::max<size_t>(c->pb.descs.size(), 1);
  return std::max<uint64_t>(std::min<uint64_t>(8, c->pb.K), D) * EW * 8;  // KC <= 8 slot rows or D
}

static bool ido_possible(const cyc_ctx* c) {
  return !c->pb.may_err && c->plan.max_runs <= IDO_MAX_RUNS && ido_lds_bytes(c) <= IDO_LDS_BYTES &&
         ido_b_bytes(c, 0) + ido_b_bytes(c, 1) <= (1ull << 30);
}

// Batched blocks: per block (first pod, pods, first slot, slots) and its output slab offsets; per
// identity its block and class-row window (its block's words).
static void prepare_blocks_device(cyc_ctx* c) {
  Problem& pb = c->pb;
  c->blk_off_h.clear();
  c->blk_wa_max = c->blk_np_max = 0;
  if (pb.blocks.empty()) return;
  std::vector<uint32_t> cfg_k0(pb.n_cfg + 1, pb.K), cfg_nk(pb.n_cfg, 0);
  for (uint32_t k = pb.K; k-- > 0;) cfg_k0[pb.slot_cfg[k]] = k;
  for (uint32_t k = 0; k < pb.K; k++) cfg_nk[pb.slot_cfg[k]]++;
  std::vector<uint4> bl(pb.blocks.size());
  uint64_t words = 0, bytes = 0;
  for (size_t b = 0; b < pb.blocks.size(); b++) {
    const ProbeBlock& x = pb.blocks[b];
    const uint32_t np = x.p1 - x.p0, nk = cfg_nk[x.cfg];
    bl[b] = uint4{x.p0, np, cfg_k0[x.cfg], nk};
    c->blk_off_h.push_back(words);
    c->blk_off_h.push_back(bytes);
    words += uint64_t(np) * nk * ((np + 63) / 64);
    bytes += uint64_t(np) * nk;
    c->blk_wa_max = std::max<uint32_t>(c->blk_wa_max, np ? (x.p1 + 63) / 64 - x.p0 / 64 : 0u);
    c->blk_np_max = std::max(c->blk_np_max, np);
  }
  c->blk_off_h.push_back(words);
  c->blk_off_h.push_back(bytes);
  upload(c->blk, bl);
  upload(c->blk_off, c->blk_off_h);
  for (int d = 0; d < 2; d++) {
    const Identities& I = c->ids[d];
    std::vector<uint32_t> ib(I.ns.size(), 0);
    std::vector<uint2> iw(I.ns.size(), uint2{0, 0});
    for (uint32_t q = 0; q < pb.P; q++) {
      const ProbeBlock& x = pb.blocks[pb.pod_blk[q]];
      ib[I.of_pod[q]] = pb.pod_blk[q];
      iw[I.of_pod[q]] = uint2{x.p0 / 64, (x.p1 + 63) / 64 - x.p0 / 64};
    }
    upload(c->id_blk[d], ib);
    upload(c->id_win[d], iw);
  }
  c->first_blk.alloc(std::max<uint64_t>(pb.blocks.size() * 8, 16));
}

static void prepare_device(cyc_ctx* c) {
  Problem& pb = c->pb;
  PhaseClock clk("prepare_device");
  upload(c->ls_off, pb.ls_off);
  upload(c->ls_key, pb.ls_key);
  upload(c->ls_val, pb.ls_val);
  upload(c->sel_off, pb.sel_off);
  upload(c->reqs, pb.reqs);
  upload(c->req_vals, pb.req_vals);
  upload(c->pod_ns, pb.pod_ns);
  upload(c->pod_ls, pb.pod_ls);
  upload(c->pod_nsls, pb.pod_nsls);
  upload(c->pod_ip, pb.pod_ip);
  {  // the address index of the range-built IP rows: IPv4 pods by address, then IPv6 pods
    std::vector<uint32_t> p4, p6;
    for (uint32_t q = 0; q < pb.P; q++)
      if (pb.pod_ip[q].valid) (pb.pod_ip[q].fam == 4 ? p4 : p6).push_back(q);
    std::stable_sort(p4.begin(), p4.end(), [&](uint32_t x, uint32_t y) { return pb.pod_ip[x].w[3] < pb.pod_ip[y].w[3]; });
    auto a6 = [&](uint32_t q) { return std::array<uint32_t, 4>{pb.pod_ip[q].w[0], pb.pod_ip[q].w[1], pb.pod_ip[q].w[2], pb.pod_ip[q].w[3]}; };
    std::stable_sort(p6.begin(), p6.end(), [&](uint32_t x, uint32_t y) { return a6(x) < a6(y); });
    c->ip4_key.resize(p4.size());
    c->ip6_key.resize(p6.size());
    for (size_t x = 0; x < p4.size(); x++) c->ip4_key[x] = pb.pod_ip[p4[x]].w[3];
    for (size_t x = 0; x < p6.size(); x++) c->ip6_key[x] = a6(p6[x]);
    c->ipsort_host = p4;
    c->ipsort_host.insert(c->ipsort_host.end(), p6.begin(), p6.end());
    upload(c->ipsort, c->ipsort_host);
  }
  upload(c->cidrs, pb.cidrs);
  upload(c->ipbs, pb.ipbs);
  upload(c->ipb_ex, pb.ipb_ex);
  upload(c->pms, pb.pms);
  upload(c->pents, pb.pents);
  upload(c->peers, pb.peers);
  upload(c->descs, pb.descs);
  upload(c->slot_desc, pb.slot_desc);
  upload(c->slot_status, pb.slot_status);
  upload(c->slot_cfg, pb.slot_cfg);
  upload(c->slot_idx, pb.slot_idx);
  clk.lap("uploads");
  uint64_t R = pb.peers.size(), W = pb.W, D = std::max<size_t>(pb.descs.size(), 1), K = pb.K;
  c->selres.alloc(std::max<uint64_t>(uint64_t(pb.S) * pb.L, 16));
  {  // dense label table for k_selectors_dense: label keys -> dense index kx, LVT[kx][l]
    std::vector<int32_t> kx(pb.strings.size(), -1);
    uint32_t nk = 0;
    for (uint32_t k : pb.ls_key)
      if (kx[k] < 0) kx[k] = int32_t(nk++);
    c->dense_sel = uint64_t(nk + 1) * pb.L * 4 <= (256ull << 20);
    if (c->dense_sel) {
      std::vector<uint32_t> lvt(uint64_t(nk + 1) * pb.L, 0xFFFFFFFFu);
      for (uint32_t l = 0; l < pb.L; l++)
        for (uint32_t x = pb.ls_off[l]; x < pb.ls_off[l + 1]; x++) lvt[uint64_t(kx[pb.ls_key[x]]) * pb.L + l] = pb.ls_val[x];
      std::vector<DReq> dr = pb.reqs;
      for (DReq& q : dr) q.key = (q.op != REQ_INVALID && q.key < kx.size() && kx[q.key] >= 0) ? uint32_t(kx[q.key]) : nk;
      upload(c->lvt, lvt);
      upload(c->dreqs, dr);
      {  // one-requirement selectors in a single record each (SelView::one)
        std::vector<uint4> one(std::max<size_t>(pb.S, 1), uint4{SEL_WALK, 0, 0, 0});
        for (uint32_t sid = 0; sid < pb.S; sid++) {
          const uint32_t r0 = pb.sel_off[sid], nr = pb.sel_off[sid + 1] - r0;
          if (nr == 0) {
            one[sid].x = SEL_ALL;
            continue;
          }
          const DReq& q = dr[r0];
          if (nr != 1 || q.op == REQ_INVALID || q.vcnt > 2) continue;
          const bool has_v = q.op == REQ_EQ || q.op == REQ_EQ_EMPTY || q.op == REQ_IN || q.op == REQ_NOTIN;
          const uint32_t vc = has_v ? (q.op == REQ_EQ || q.op == REQ_EQ_EMPTY ? 1u : q.vcnt) : 0u;
          one[sid] = uint4{q.op | (vc << 8), q.key, vc > 0 ? pb.req_vals[q.voff] : 0u, vc > 1 ? pb.req_vals[q.voff + 1] : 0u};
        }
        upload(c->sel_one, one);
      }
      // the same table per pod (PLVT, sparse pod-peer rows) is gathered on the device when a run
      // first needs it (ensure_plvt): IDO builds never read it, and it is (keys + 1) x P words
      c->n_lkeys = nk;
      c->plvt.alloc(0);
      c->plvt_ready = false;
      // label postings: the pods under each (dense key, value) of their own labels, and per EQ / IN
      // (<= 2 values) requirement the postings of its values (pod_rows_post_blk)
      // (key, value, pod) triples sorted by (key, value), pods ascending within: two counting-sort
      // passes (value, then key; both are dictionary ids), O(pairs + dictionary)
      std::vector<std::pair<uint64_t, uint32_t>> kv;
      {
        const size_t NV = pb.strings.size() + 1, NK = nk + 1;
        size_t n = 0;
        for (uint32_t q = 0; q < pb.P; q++) n += pb.ls_off[pb.pod_ls[q] + 1] - pb.ls_off[pb.pod_ls[q]];
        std::vector<uint32_t> kk(n), vv(n), qq(n), cnt(std::max(NV, NK) + 1);
        size_t x0 = 0;
        for (uint32_t q = 0; q < pb.P; q++) {
          const uint32_t l = pb.pod_ls[q];
          for (uint32_t x = pb.ls_off[l]; x < pb.ls_off[l + 1]; x++, x0++) {
            kk[x0] = uint32_t(kx[pb.ls_key[x]]);
            vv[x0] = pb.ls_val[x];
            qq[x0] = q;
          }
        }
        std::vector<uint32_t> ord(n), ord2(n);
        auto pass = [&](const std::vector<uint32_t>& key, size_t range, const std::vector<uint32_t>& in, std::vector<uint32_t>& out) {
          std::fill(cnt.begin(), cnt.begin() + range + 1, 0u);
          for (uint32_t i : in) cnt[key[i] + 1]++;
          for (size_t r = 0; r < range; r++) cnt[r + 1] += cnt[r];
          for (uint32_t i : in) out[cnt[key[i]]++] = i;
        };
        std::iota(ord.begin(), ord.end(), 0u);  // pod order (q ascending)
        pass(vv, NV, ord, ord2);
        pass(kk, NK, ord2, ord);
        kv.resize(n);
        for (size_t i = 0; i < n; i++) kv[i] = {(uint64_t(kk[ord[i]]) << 32) | vv[ord[i]], qq[ord[i]]};
      }
      std::vector<uint32_t> pods(kv.size());
      for (size_t i = 0; i < kv.size(); i++) pods[i] = kv[i].second;
      auto range = [&](uint32_t key, uint32_t v) {
        const uint64_t k = (uint64_t(key) << 32) | v;
        auto lo = std::lower_bound(kv.begin(), kv.end(), std::make_pair(k, 0u));
        auto hi = std::lower_bound(kv.begin(), kv.end(), std::make_pair(k + 1, 0u));
        return std::make_pair(uint32_t(lo - kv.begin()), uint32_t(hi - lo));
      };
      std::vector<uint4> rp(dr.size(), uint4{0, 0, 0, 0});
      c->req_post_ok.assign(dr.size(), 0);
      for (size_t r = 0; r < dr.size(); r++) {
        const DReq& q = dr[r];
        if (q.key >= nk || !(q.op == REQ_EQ || (q.op == REQ_IN && q.vcnt >= 1 && q.vcnt <= 2))) continue;
        const auto a = range(q.key, pb.req_vals[q.voff]);
        rp[r] = uint4{a.first, a.second, 0, 0};
        if (q.op == REQ_IN && q.vcnt == 2 && pb.req_vals[q.voff + 1] != pb.req_vals[q.voff]) {
          const auto b = range(q.key, pb.req_vals[q.voff + 1]);
          rp[r].z = b.first;
          rp[r].w = b.second;
        }
        c->req_post_ok[r] = 1;
      }
      upload(c->req_post, rp);
      upload(c->post_pods, pods);
    }
  }
  clk.lap("label tables");
  c->PM.alloc(std::max<uint64_t>(R * W * 8, 16));
  c->ip_rng.alloc(std::max<uint64_t>(R * 16 + R * ((W + 63) / 64) * 4, 16));  // [R][4] word spans + chunk masks, then [R][W/64] cnz
  c->ip_rng_clean = false;  // a new buffer: the next fused front fills it (no emit has reset it yet)
  c->ER.alloc(pb.may_err ? std::max<uint64_t>(R * W * 8, 16) : 16);
  {
    c->plan = plan_peers(pb, c->ids[1]);
    PeerPlan& pl = c->plan;
    upload(c->word_off, pl.word_off);
    upload(c->run_e, pl.run_e);
    upload(c->run_mask, pl.run_mask);
    upload(c->runs, pl.runs);
    upload(c->id_nsls, c->ids[1].nsls);
    {  // per-word, per-family address intervals for k_ip_rows_fast, then one record per 64-word chunk
      const uint32_t NC = (pb.W + 63) / 64;
      std::vector<DWordIP> wi(pb.W + NC);
      c->word_aff.assign(pb.W, 3);
      for (uint32_t w = 0; w < pb.W; w++) {
        DWordIP d{};
        d.min4 = 0xFFFFFFFFu;
        for (int i = 0; i < 4; i++) d.min6[i] = 0xFFFFFFFFu;
        // affine check per family: every pod of the family at lane i holds base + i (128-bit, big-endian
        // words; v4 in w[3]) for one base (DWordIP::aff)
        bool aff[2] = {true, true};
        int first[2] = {-1, -1};
        uint32_t base[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
        for (uint32_t q = w * 64; q < std::min<uint32_t>(pb.P, w * 64 + 64); q++) {
          const DIP& ip = pb.pod_ip[q];
          if (!ip.valid) continue;  // only with may_err, where the fast kernel is not used
          const uint32_t lane = q - w * 64;
          const int f = ip.fam == 4 ? 0 : 1;
          uint32_t a[4] = {f ? ip.w[0] : 0u, f ? ip.w[1] : 0u, f ? ip.w[2] : 0u, ip.w[3]};
          // b = a - lane (128-bit): the pod's base
          uint32_t b[4];
          uint64_t borrow = lane;
          for (int i = 3; i >= 0; i--) {
            const uint64_t v = uint64_t(a[i]) - borrow;
            b[i] = uint32_t(v);
            borrow = (v >> 63) & 1u;  // went below zero
          }
          if (borrow) aff[f] = false;  // address < lane: no base (never affine)
          if (first[f] < 0) {
            first[f] = int(lane);
            std::copy(b, b + 4, base[f]);
          } else if (!std::equal(b, b + 4, base[f])) {
            aff[f] = false;
          }
          if (ip.fam == 4) {
            d.m4 |= 1ull << lane;
            d.min4 = std::min(d.min4, ip.w[3]);
            d.max4 = std::max(d.max4, ip.w[3]);
          } else {
            d.m6 |= 1ull << lane;
            if (std::lexicographical_compare(ip.w, ip.w + 4, d.min6, d.min6 + 4)) std::copy(ip.w, ip.w + 4, d.min6);
            if (std::lexicographical_compare(d.max6, d.max6 + 4, ip.w, ip.w + 4)) std::copy(ip.w, ip.w + 4, d.max6);
          }
        }
        for (int f = 0; f < 2; f++)
          if (first[f] >= 0 && aff[f]) d.aff |= (uint32_t(first[f]) | 0x80u) << (8 * f);
        c->word_aff[w] = uint8_t((first[0] < 0 || aff[0] ? 1u : 0u) | (first[1] < 0 || aff[1] ? 2u : 0u));
        wi[w] = d;
      }
      for (uint32_t ch = 0; ch < NC; ch++) {
        DWordIP d{};
        d.min4 = 0xFFFFFFFFu;
        for (int i = 0; i < 4; i++) d.min6[i] = 0xFFFFFFFFu;
        for (uint32_t w = ch * 64; w < std::min<uint32_t>(pb.W, ch * 64 + 64); w++) {
          const DWordIP& x = wi[w];
          if (x.m4) {
            d.m4 |= 1ull << (w - ch * 64);
            d.min4 = std::min(d.min4, x.min4);
            d.max4 = std::max(d.max4, x.max4);
          }
          if (x.m6) {
            d.m6 |= 1ull << (w - ch * 64);
            if (std::lexicographical_compare(x.min6, x.min6 + 4, d.min6, d.min6 + 4)) std::copy(x.min6, x.min6 + 4, d.min6);
            if (std::lexicographical_compare(d.max6, d.max6 + 4, x.max6, x.max6 + 4)) std::copy(x.max6, x.max6 + 4, d.max6);
          }
        }
        wi[pb.W + ch] = d;
      }
      upload(c->ip_words, wi);
      c->ipw_h = wi;
      // namespace range of every word's and chunk's pods (pod_rows_sparse_blk)
      std::vector<DWordNS> nw(pb.W + NC, DWordNS{0xFFFFFFFFu, 0u, 0u, 0u});
      for (uint32_t q = 0; q < pb.P; q++) {
        for (DWordNS* x : {&nw[q / 64], &nw[pb.W + q / 4096]}) {
          if (x->lo == 0xFFFFFFFFu) x->nsls = pb.pod_nsls[q];
          else if (x->lo != pb.pod_ns[q] || x->hi != pb.pod_ns[q]) x->nsls = 0xFFFFFFFFu;
          x->lo = std::min(x->lo, pb.pod_ns[q]);
          x->hi = std::max(x->hi, pb.pod_ns[q]);
        }
      }
      upload(c->ns_words, nw);
    }
    c->ido.alloc(std::max<uint64_t>(uint64_t(pl.pod_peers.size()) * c->ids[1].ns.size(), 16));
    c->idob.alloc(std::max<uint64_t>(uint64_t(pl.pod_peers.size()) * ((c->ids[1].ns.size() + 63) / 64) * 8, 16));
  }
  clk.lap("peer plan");
  {  // one VALID descriptor per slot across all pods? (egress class rows then skip the per-word slot words)
    std::vector<int32_t> ud(std::max<uint32_t>(pb.K, 1), -1);
    bool uni = pb.P > 0 && pb.K > 0;
    for (uint32_t k = 0; k < pb.K && uni; k++) {
      ud[k] = pb.slot_desc[k];
      for (uint32_t q = 0; q < pb.P && uni; q++)
        uni = pb.slot_status[size_t(q) * pb.K + k] == CYC_JOB_VALID && pb.slot_desc[size_t(q) * pb.K + k] == ud[k];
    }
    c->uni_desc = uni;
    upload(c->udesc, ud);
  }
  c->portok.alloc(std::max<uint64_t>(pb.pms.size() * D, 16));
  c->portbits.alloc(std::max<uint64_t>(pb.pms.size() * 4, 16));
  c->VALID.alloc(std::max<uint64_t>(K * W * 8, 16));
  c->DESCW.alloc(std::max<uint64_t>(K * W * 4, 16));
  c->DM.alloc(std::max<uint64_t>(K * D * W * 8, 16));
  c->first_err.alloc(std::max<uint64_t>(uint64_t(pb.n_cfg) * 8, 16));  // per probe config (k_first_error)
  c->status_sink.alloc(std::max<uint64_t>(uint64_t(pb.P) * K, 16));
  for (int d = 0; d < 2; d++) {
    Identities& I = c->ids[d];
    DirDev& dd = c->dir[d];
    dd.n = uint32_t(I.ns.size());
    dd.ht_cap = I.ht_cap;
    upload(dd.id_ns, I.ns);
    upload(dd.id_ls, I.ls);
    upload(dd.id_desc, I.desc);
    upload(dd.id_status, I.status);
    upload(dd.list_off, I.list_off);
    upload(dd.tns_lo, pb.tns_lo[d]);
    upload(dd.tns_hi, pb.tns_hi[d]);
    upload(dd.tgt, pb.tgt[d]);
    upload(dd.pod_id, I.of_pod);
    dd.list.alloc(std::max<uint64_t>(I.list_total * 4, 16));
    dd.cnt.alloc(std::max<uint64_t>(dd.n * 4ull, 16));
    dd.hash.alloc(std::max<uint64_t>(dd.n * 8ull, 16));
    dd.err.alloc(std::max<uint64_t>(dd.n, 16));
    dd.ht_key.alloc(uint64_t(dd.ht_cap) * 16 + 16);  // [cap] 16-byte entries (key ~0 = empty, rep), counter
    HIPCHK(hipMemset(dd.ht_key.p, 0xFF, dd.ht_key.bytes));  // empty; afterwards every run's class rows empty it
    if (!c->zeros.p) {
      c->zeros.alloc(256);
      HIPCHK(hipMemset(c->zeros.p, 0, 256));
    }
    dd.reps.alloc(std::max<uint64_t>(dd.n * 4ull, 16));
    dd.class_of.alloc(std::max<uint64_t>(dd.n * 4ull, 16));
    dd.A.alloc(std::max<uint64_t>(uint64_t(dd.n) * K * W * 8, 16));
    if (pb.may_err) dd.AE.alloc(std::max<uint64_t>(uint64_t(dd.n) * K * W * 8, 16));
    else dd.AE.alloc(0);
    dd.B.alloc(ido_possible(c) ? std::max<uint64_t>(ido_b_bytes(c, d), 16) : 16);
    {  // IP-peer list bounds per identity: the IP peers of its namespace's targets
      // (upper bound for both list uses: IDO builds list the IP peers, PM builds every peer)
      std::vector<uint32_t> ns_ip(pb.strings.size(), 0), off(dd.n + 1, 0);
      for (const DTarget& t : pb.tgt[d]) ns_ip[t.ns] += t.pcnt;
      for (uint32_t i = 0; i < dd.n; i++) off[i + 1] = off[i] + ns_ip[I.ns[i]];
      upload(dd.ip_off, off);
      dd.ip_cnt.alloc(std::max<uint64_t>(dd.n * 4ull, 16));
      dd.ip_list.alloc(std::max<uint64_t>(uint64_t(off[dd.n]) * 16, 16));
    }
  }
  clk.lap("scratch");
  prepare_blocks_device(c);
  c->order_lo = c->order_hi = -1;
  c->order_src = false;
}

// nonzero-chunk flags of the IP peers' PM rows, after the word spans and chunk masks in the ip_rng buffer
static uint32_t* ip_cnz(cyc_ctx* c) { return c->ip_rng.as<uint32_t>() + 4 * c->pb.peers.size(); }

static unsigned grid1(uint64_t n, unsigned block) { return unsigned(std::min<uint64_t>((n + block - 1) / block, 1u << 20)); }

static bool front_fused_ok(const cyc_ctx* c);
static bool ido_mode(const cyc_ctx* c);
// Selectors evaluated where used (sel_at through LVT), not as the dense SELRES table: the fused
// front of PM builds (its pod-peer rows and membership are the only selector users, and PM builds
// are the ones whose label sets number ~ the pods).  The DAG path computes SELRES regardless.
// PM builds' fused front: sparse pod-peer rows (pod_rows_sparse_blk, launch C) once the rows are
// large (>= 2M pod-peer words: config #3u), else full rows a wave per (pod peer, word) in launch B,
// which has the parallelism small problems need (config #2: 125k peer words, B + C 33 vs 52 us).
// pr_group > 0 forces the sparse rows.
static bool pod_sparse(const cyc_ctx* c) {
  if (ido_mode(c)) return false;
  const uint64_t Rp = c->rp_off[2] - c->rp_off[0];
  return c->pr_group > 0 || Rp * c->pb.W >= (2ull << 20);
}
// PLVT (each pod's value of every dense label key) for the sparse pod-peer rows: gathered on the
// device from LVT once per prepare, on the run's stream ahead of the step, when a run needs it
// and it fits PLVT_MAX_BYTES; otherwise the rows read LVT through each pod's label set (SelView
// with PLVT null), one more dependent load per pod.
static void ensure_plvt(cyc_ctx* c, hipStream_t st) {
  if (c->plvt_ready || !c->dense_sel || !pod_sparse(c)) return;
  const uint64_t n = uint64_t(c->n_lkeys + 1) * c->pb.P;
  if (!n || n * 4 > (uint64_t(c->plvt_max_mb) << 20)) return;
  c->plvt.alloc(n * 4);
  k_plvt<<<grid1(n, 256), 256, 0, st>>>(c->lvt.as<uint32_t>(), c->pod_ls.as<uint32_t>(), c->pb.L, c->pb.P, n,
                                        c->plvt.as<uint32_t>());
  HIPCHK(hipGetLastError());
  c->plvt_ready = true;
}
static bool lazy_sel(const cyc_ctx* c) {
  if (!c->dense_sel || c->pb.may_err || c->sel_lazy == 0 || !front_fused_ok(c)) return false;
  const bool pod_peers = c->rp_off[2] > c->rp_off[0];
  // the full pod-peer rows read the dense selector table
  if (!ido_mode(c) && !pod_sparse(c) && pod_peers) return false;
  // no pod-peer rows at all (IPBlock-only policies, config #4): the membership is the only selector
  // user, one record and one label-table load per target — no table, and no launch A
  if (!pod_peers && c->sel_lazy < 0) return true;
  // auto: lazy once the dense table would take ~0.1 ms (>= 64M pairs; config #3u: 0.75G pairs,
  // 1.1 ms; config #2 stays dense — its multi-requirement selectors cost more evaluated per use)
  // IDO builds always: their identity sets and membership evaluate fewer pairs than the table
  // holds (config #3: A + B 118 -> 111 us; its N = 8 shard 35 -> 31 us, profiles/r02_sel_lazy_ab.txt)
  return c->sel_lazy == 1 || ido_mode(c) || uint64_t(c->n_sel) * c->pb.L >= (64ull << 20);
}
static SelView sel_view(cyc_ctx* c) {
  SelView v{};
  v.selres = lazy_sel(c) ? nullptr : c->selres.as<uint8_t>();
  v.L = c->pb.L;
  v.sel_off = c->sel_off.as<uint32_t>();
  v.req_vals = c->req_vals.as<uint32_t>();
  v.LVT = c->lvt.as<uint32_t>();
  v.dreqs = c->dreqs.as<DReq>();
  v.PLVT = c->plvt_ready ? c->plvt.as<uint32_t>() : nullptr;  // null: pod -> label set -> LVT gathers
  v.P = c->pb.P;
  v.one = c->sel_one.as<uint4>();
  return v;
}

static MemberArgs member_args(cyc_ctx* c, int d) {
  Problem& pb = c->pb;
  DirDev& dd = c->dir[d];
  MemberArgs a{};
  a.n_ident = dd.n;
  a.L = pb.L;
  a.K = pb.K;
  a.id_ns = dd.id_ns.as<uint32_t>();
  a.id_ls = dd.id_ls.as<uint32_t>();
  a.id_desc = d == 0 ? dd.id_desc.as<int32_t>() : nullptr;
  a.id_status = d == 0 ? dd.id_status.as<uint8_t>() : nullptr;
  a.tns_lo = dd.tns_lo.as<uint32_t>();
  a.tns_hi = dd.tns_hi.as<uint32_t>();
  a.tgt = dd.tgt.as<DTarget>();
  a.sv = sel_view(c);
  a.list_off = dd.list_off.as<uint32_t>();
  a.list = dd.list.as<uint32_t>();
  a.cnt = dd.cnt.as<uint32_t>();
  a.hash = dd.hash.as<uint64_t>();
  a.err = dd.err.as<uint8_t>();
  a.ht_key = dd.ht_key.as<unsigned long long>();
  a.ht_cap = dd.ht_cap;
  a.act = c->act[d].as<uint32_t>();
  a.actrec = c->actrec[d].as<uint4>();
  a.n_act = c->n_act[d];
  a.reps = dd.reps.as<uint32_t>();
  a.rep_cnt = dd.rep_cnt();
  a.id_blk = c->pb.blocks.empty() ? nullptr : c->id_blk[d].as<uint32_t>();
  return a;
}

// PM-build class rows (k_class_rows_pl): threads per block — PL_THREADS, or 256 for rows of >= 16
// chunks (the wave-per-chunk rows then split a class's chunks over 4 waves: config #3u -5 %,
// config #4's 13 chunks +9 %: profiles/r02_pl_threads_ab.txt) — and blocks per direction, striding
// over the representatives, about two blocks in flight per CU slot
static uint32_t pl_threads(const cyc_ctx* c) { return (c->pb.W + 63) / 64 >= 16 ? 256u : PL_THREADS; }
static uint32_t pl_blocks(const cyc_ctx* c, int d) { return std::min<uint32_t>(c->n_act[d], 2048u * 256u / pl_threads(c)); }

// Range plan for rows [lo,hi): (1) the rows ordered so pods sharing class rows are adjacent
// (L2 / Infinity-Cache reuse in k_emit); (2) the identities those rows use, per direction —
// only their classes are elected and their class rows computed; (3) the peers of the targets
// in those identities' namespaces — only their PM rows are built.  A rank of an N-GPU run thus
// does ~1/N of the front work too, not just 1/N of the emit.
// Source-row plans (src): rows [lo, hi) are SOURCES; the run computes every cell (s in [lo, hi), d,
// k): egress rows of sources [lo, hi) (full rows) and the ingress rows of EVERY destination, but
// only their words [lo / 64, ceil(hi / 64)) — the shard's sources as peers.  lo must be a multiple
// of 64 and hi too unless it is P (checked by the caller), so the windows of a partition tile the words.
static void peer_chunks(const cyc_ctx* c, int d, uint32_t& c0, uint32_t& nch);
static bool one_window(const cyc_ctx* c);
// Host restatement of ip_rows_fast_blk's chunk test: false when network n misses the chunk's pods'
// addresses of its family (or the chunk has none of that family).
static bool ip_chunk_touch(const DCidr& n, const DWordIP& ck) {
  if (!n.valid) return true;
  if (n.fam == 4) {
    const uint32_t lo = n.net[3] & n.mask[3], hi = lo | ~n.mask[3];
    return ck.m4 && !(ck.max4 < lo || ck.min4 > hi);
  }
  uint32_t lo[4], hi[4];
  for (int i = 0; i < 4; i++) {
    lo[i] = n.net[i] & n.mask[i];
    hi[i] = lo[i] | ~n.mask[i];
  }
  auto lt = [](const uint32_t* a, const uint32_t* b) { return std::lexicographical_compare(a, a + 4, b, b + 4); };
  return ck.m6 && !(lt(ck.max6, lo) || lt(hi, ck.min6));
}

static void ensure_range(cyc_ctx* c, int64_t lo, int64_t hi, bool src = false) {
  if (c->order_lo == lo && c->order_hi == hi && c->order_src == src) return;
  Problem& pb = c->pb;
  PhaseClock clk("range plan");
  c->rl[0] = src ? 0 : lo;
  c->rh[0] = src ? int64_t(pb.P) : hi;
  c->rl[1] = lo;
  c->rh[1] = hi;
  c->win_w0 = src ? uint32_t(lo / 64) : 0u;
  c->win_wa = src ? uint32_t((hi + 63) / 64 - lo / 64) : pb.W;
  if (src && hi <= lo) c->win_wa = 0;
  {  // the egress identities of the window's pods (identity ids follow first appearance in pod order, so a
     // source shard's are mostly one range): the ingress identity sets need only their words
    const uint32_t EW = uint32_t((c->ids[1].ns.size() + 63) / 64);
    c->ido_ew0 = 0;
    c->ido_ew1 = EW;
    if (src) {
      uint32_t e0 = UINT32_MAX, e1 = 0;
      for (int64_t q = c->win_w0 * 64ll; q < std::min<int64_t>(int64_t(c->win_w0 + c->win_wa) * 64, pb.P); q++) {
        e0 = std::min(e0, c->ids[1].of_pod[size_t(q)]);
        e1 = std::max(e1, c->ids[1].of_pod[size_t(q)] + 1);
      }
      c->ido_ew0 = e0 == UINT32_MAX ? 0u : e0 / 64;
      c->ido_ew1 = e0 == UINT32_MAX ? 0u : (e1 + 63) / 64;
    }
  }
  for (int d = 0; d < 2; d++) {  // emit row order: clustered by this direction's identity, (pod, identity) pairs
    std::vector<uint32_t> ord(size_t(c->rh[d] - c->rl[d]));
    std::iota(ord.begin(), ord.end(), uint32_t(c->rl[d]));
    const auto& i1 = c->ids[d].of_pod;
    const auto& i2 = c->ids[1 - d].of_pod;
    std::stable_sort(ord.begin(), ord.end(),
                     [&](uint32_t x, uint32_t y) { return i1[x] != i1[y] ? i1[x] < i1[y] : i2[x] < i2[y]; });
    std::vector<uint32_t> pairs(ord.size() * 2);
    for (size_t r = 0; r < ord.size(); r++) {
      pairs[2 * r] = ord[r];
      pairs[2 * r + 1] = i1[ord[r]];
    }
    upload(c->order[d], pairs);
  }
  std::vector<uint8_t> peer_needed(pb.peers.size(), 0), peer_dir(pb.peers.size(), 0);
  for (const DTarget& t : pb.tgt[1])
    for (uint32_t j = t.poff; j < t.poff + t.pcnt; j++) peer_dir[j] = 1;
  for (int d = 0; d < 2; d++) {
    const Identities& I = c->ids[d];
    std::vector<uint8_t> used(I.ns.size(), 0);
    std::vector<uint32_t> act;
    const bool empty_window = d == 0 && c->win_wa == 0;  // a source shard without sources: no ingress words
    for (int64_t p = c->rl[d]; p < c->rh[d] && !empty_window; p++) {
      uint32_t i = I.of_pod[size_t(p)];
      if (!used[i]) {
        used[i] = 1;
        act.push_back(i);
      }
    }
    std::sort(act.begin(), act.end());
    {  // each active identity's first pod in the range: its plane row holds the class row in place
      std::vector<uint32_t> ar(I.ns.size(), 0xFFFFFFFFu);
      for (int64_t p = c->rh[d] - 1; p >= c->rl[d]; p--) ar[I.of_pod[size_t(p)]] = uint32_t(p - c->rl[d]);
      upload(c->arow[d], ar);
    }
    std::vector<uint8_t> ns_needed(pb.strings.size(), 0);
    for (uint32_t i : act) ns_needed[I.ns[i]] = 1;
    for (const DTarget& t : pb.tgt[d])
      if (ns_needed[t.ns])
        for (uint32_t j = t.poff; j < t.poff + t.pcnt; j++) peer_needed[j] = 1;
    c->n_act[d] = uint32_t(act.size());
    uint64_t tsum = 0;  // namespace targets each active identity's membership walk visits
    for (uint32_t i : act) tsum += pb.tns_hi[d][I.ns[i]] - pb.tns_lo[d][I.ns[i]];
    c->act_targets[d] = act.empty() ? 0.0 : double(tsum) / double(act.size());
    upload(c->act[d], act);
    // the membership's per-identity inputs in one 16-byte record (one load instead of the chain
    // act -> id_ls / id_ns / list_off -> tns_lo / tns_hi)
    std::vector<uint32_t> rec(act.size() * 4);
    for (size_t x = 0; x < act.size(); x++) {
      const uint32_t i = act[x], ns = I.ns[i];
      rec[4 * x] = I.ls[i];
      rec[4 * x + 1] = pb.tns_lo[d][ns];
      rec[4 * x + 2] = pb.tns_hi[d][ns];
      rec[4 * x + 3] = I.list_off[i];
    }
    upload(c->actrec[d], rec);
  }
  // selectors the range can reach: its targets' pod selectors and their peers' selectors
  std::vector<uint8_t> sel_needed(pb.S, 0);
  for (int d = 0; d < 2; d++)
    for (const DTarget& t : pb.tgt[d]) {
      bool needed = false;
      for (uint32_t j = t.poff; j < t.poff + t.pcnt && !needed; j++) needed = peer_needed[j];
      if (needed || t.pcnt == 0) sel_needed[t.sel] = 1;
    }
  for (int d = 0; d < 2; d++) {  // targets of active namespaces (also those without peers)
    const Identities& I = c->ids[d];
    std::vector<uint8_t> ns_needed(pb.strings.size(), 0);
    for (int64_t p = c->rl[d]; p < c->rh[d]; p++) ns_needed[I.ns[I.of_pod[size_t(p)]]] = 1;
    for (const DTarget& t : pb.tgt[d])
      if (ns_needed[t.ns]) sel_needed[t.sel] = 1;
  }
  for (uint32_t j = 0; j < pb.peers.size(); j++)
    if (peer_needed[j] && pb.peers[j].kind == PK_POD) {
      if (pb.peers[j].nskind == NS_LABEL) sel_needed[pb.peers[j].nsval] = 1;
      if (pb.peers[j].podsel != CYC_ALL) sel_needed[pb.peers[j].podsel] = 1;
    }
  std::vector<uint32_t> sl;
  for (uint32_t i = 0; i < pb.S; i++)
    if (sel_needed[i]) sl.push_back(i);
  c->n_sel = uint32_t(sl.size());
  {  // sparse pod rows: peers whose pod selector is one posting requirement are built from postings
    // (ingress peers first, then egress: each sub-list has its direction's word window)
    std::vector<uint32_t> scan, post;
    for (int d = 0; d < 2; d++) {
      c->scan_off[d] = uint32_t(scan.size());
      c->post_off[d] = uint32_t(post.size());
      for (uint32_t j : c->plan.pod_peers) {
        if (!peer_needed[j] || peer_dir[j] != d) continue;
        const DPeer& pr = pb.peers[j];
        if (pr.nskind == NS_ALL && pr.podsel == CYC_ALL) continue;  // all-ones row: the class rows need none
        const bool one = pr.podsel != CYC_ALL && pb.sel_off[pr.podsel + 1] - pb.sel_off[pr.podsel] == 1;
        if (one && c->dense_sel && !c->req_post_ok.empty() && c->req_post_ok[pb.sel_off[pr.podsel]]) post.push_back(j);
        else scan.push_back(j);
      }
    }
    c->scan_off[2] = uint32_t(scan.size());
    c->post_off[2] = uint32_t(post.size());
    c->n_scan = uint32_t(scan.size());
    c->n_post = uint32_t(post.size());
    upload(c->pp_scan, scan);
    upload(c->pp_post, post);
  }
  upload(c->sel_list, sl);
  std::vector<uint32_t> pp, ip;
  std::vector<DIPTest> tests;
  // An IP peer's row depends only on its IPBlock (ippeermatcher.go:43-50; the port is tested by the
  // class rows): peers of one direction whose (cidr, except) strings are equal share the row of
  // the first (config #4: the 0.0.0.0/0-style blocks of ~2,500 peers are 5 rows).  prow maps every
  // peer to its row; only the first of each IPBlock gets an IP-row test.
  std::vector<uint32_t> prow(std::max<size_t>(pb.peers.size(), 1));
  for (uint32_t j = 0; j < prow.size(); j++) prow[j] = j;
  std::vector<DIPRange> rtests;
  std::vector<uint2> riv;
  // an IPBlock's matching pods as intervals of the address index (its family's block, less each
  // same-family except), their count and word span: built from ranges when few and close
  // (no-panic runs only: the ordered walk with panic bits keeps its dense rows)
  const uint32_t n4 = uint32_t(c->ip4_key.size());
  auto range_rows = [&](const DIPTest& t, DIPRange& out) -> bool {
    if (pb.may_err || !t.cidr.valid || c->ip_range == 0) return false;
    auto bounds = [&](const DCidr& cd, uint32_t& a, uint32_t& b) {
      if (cd.fam == 4) {
        const uint32_t lo = cd.net[3] & cd.mask[3], hi = lo | ~cd.mask[3];
        a = uint32_t(std::lower_bound(c->ip4_key.begin(), c->ip4_key.end(), lo) - c->ip4_key.begin());
        b = uint32_t(std::upper_bound(c->ip4_key.begin(), c->ip4_key.end(), hi) - c->ip4_key.begin());
      } else {
        std::array<uint32_t, 4> lo, hi;
        for (int i = 0; i < 4; i++) {
          lo[i] = cd.net[i] & cd.mask[i];
          hi[i] = lo[i] | ~cd.mask[i];
        }
        a = n4 + uint32_t(std::lower_bound(c->ip6_key.begin(), c->ip6_key.end(), lo) - c->ip6_key.begin());
        b = n4 + uint32_t(std::upper_bound(c->ip6_key.begin(), c->ip6_key.end(), hi) - c->ip6_key.begin());
      }
    };
    std::vector<uint2> iv(1);
    bounds(t.cidr, iv[0].x, iv[0].y);
    for (uint32_t e = 0; e < t.excnt; e++) {
      const DCidr& x = c->plan.ip_ex[t.exoff + e];
      if (!x.valid) return false;
      if (x.fam != t.cidr.fam) continue;  // an except of the other family never contains a pod of this one
      uint32_t ea, eb;
      bounds(x, ea, eb);
      std::vector<uint2> next;
      for (const uint2& v : iv) {
        if (ea > v.x) next.push_back(make_uint2(v.x, std::min(v.y, ea)));
        if (eb < v.y) next.push_back(make_uint2(std::max(v.x, eb), v.y));
      }
      iv.clear();
      for (const uint2& v : next)
        if (v.y > v.x) iv.push_back(v);
    }
    uint64_t n = 0;
    for (const uint2& v : iv) n += v.y - v.x;
    if (n > IPR_MAX_MATCH) return false;
    uint32_t wlo = 0xFFFFFFFFu, whi = 0;
    for (const uint2& v : iv)
      for (uint32_t x = v.x; x < v.y; x++) {
        wlo = std::min(wlo, c->ipsort_host[x] / 64);
        whi = std::max(whi, c->ipsort_host[x] / 64);
      }
    if (n && whi - wlo >= IPR_SPAN) return false;
    // words whose pods of the family hold affine addresses get the network's lanes from its bounds
    // in k_ip_rows_fast (no per-pod test): keep those rows there (config #4: range-built rows
    // made launch B 64 -> 70 us; config #2's addresses step by 256, so its words are not affine)
    const uint8_t fbit = t.cidr.fam == 4 ? 1u : 2u;
    bool all_aff = c->word_aff.size() == pb.W;
    for (uint32_t w = wlo; all_aff && n && w <= whi; w++) all_aff = (c->word_aff[w] & fbit) != 0;
    if (all_aff && c->ip_range < 0) return false;
    out = DIPRange{t.peer, uint32_t(riv.size()), uint32_t(iv.size()), n ? wlo : 0u};
    riv.insert(riv.end(), iv.begin(), iv.end());
    return true;
  };
  for (int d = 0; d < 2; d++) {  // ingress peers first, then egress: one sub-list per branch
    c->rp_off[d] = uint32_t(pp.size());
    c->ri_off[d] = uint32_t(ip.size());
    c->rr_off[d] = uint32_t(rtests.size());
    for (uint32_t j : c->plan.pod_peers)
      if (peer_needed[j] && peer_dir[j] == d) pp.push_back(j);
    std::map<std::vector<uint32_t>, uint32_t> ipb_row;
    std::vector<uint32_t> key;
    for (size_t r = 0; r < c->plan.ip_peers.size(); r++) {
      const uint32_t j = c->plan.ip_peers[r];
      if (!peer_needed[j] || peer_dir[j] != d) continue;
      const DIPBlock& b = pb.ipbs[pb.peers[j].ipb];
      key.assign(1, b.cidr);
      key.insert(key.end(), pb.ipb_ex.begin() + b.exoff, pb.ipb_ex.begin() + b.exoff + b.excnt);
      auto it = ipb_row.emplace(key, j);
      if (!it.second) {
        prow[j] = it.first->second;
        continue;
      }
      DIPRange rt{};
      if (range_rows(c->plan.ip_tests[r], rt)) {
        rtests.push_back(rt);
        continue;
      }
      ip.push_back(j);
      tests.push_back(c->plan.ip_tests[r]);
    }
  }
  c->rr_off[2] = uint32_t(rtests.size());
  c->Rr = uint32_t(rtests.size());
  upload(c->ipr_tests, rtests);
  upload(c->ipr_iv, riv);
  upload(c->peer_row, prow);
  c->prow_host = prow;
  c->rp_off[2] = uint32_t(pp.size());
  c->ri_off[2] = uint32_t(ip.size());
  c->Rp = uint32_t(pp.size());
  c->Ri = uint32_t(ip.size());
  upload(c->pod_peers, pp);
  {
    // IDOB rows depend on a pod peer only through (namespace matcher, pod selector)
    // (podpeermatcher.go:21-28; the port is checked per peer by the class rows), so peers sharing
    // them share one row: config #3 has 17k pod peers over 7.8k distinct matchers
    // The rows are ordered exact-namespace matchers first, by namespace, so a group of PB_GROUP rows
    // mostly names one or two namespaces: its identity-set waves over words of other namespaces'
    // identities skip every selector (grp_ns / word_ns below).
    std::vector<uint32_t> pi(std::max<size_t>(pb.peers.size(), 1), 0), ppu;
    std::vector<uint2> gns;
    for (int d = 0; d < 2; d++) {
      c->rpu_off[d] = uint32_t(ppu.size());
      c->ido_goff[d] = uint32_t(gns.size());
      std::map<std::tuple<uint32_t, uint32_t, uint32_t>, uint32_t> row;  // matcher -> its first peer
      for (uint32_t x = c->rp_off[d]; x < c->rp_off[d + 1]; x++) {
        const DPeer& pr = pb.peers[pp[x]];
        row.emplace(std::make_tuple(pr.nskind, pr.nsval, pr.podsel), pp[x]);
      }
      const uint32_t u0 = uint32_t(ppu.size());
      std::map<std::tuple<uint32_t, uint32_t, uint32_t>, uint32_t> at;
      for (const auto& kv : row) {  // (nskind 0 = exact namespace sorts first, then by namespace)
        at[kv.first] = uint32_t(ppu.size());
        ppu.push_back(kv.second);
      }
      for (uint32_t x = c->rp_off[d]; x < c->rp_off[d + 1]; x++) {
        const DPeer& pr = pb.peers[pp[x]];
        pi[pp[x]] = at[std::make_tuple(pr.nskind, pr.nsval, pr.podsel)];
      }
      for (uint32_t g0 = u0; g0 < ppu.size(); g0 += PB_GROUP) {
        uint2 r{0xFFFFFFFFu, 0u};
        for (uint32_t x = g0; x < std::min<uint32_t>(g0 + PB_GROUP, uint32_t(ppu.size())); x++) {
          const DPeer& pr = pb.peers[ppu[x]];
          if (pr.nskind != 0) r = uint2{0u, 0xFFFFFFFFu};  // a namespace / all-namespace matcher: never skipped
          if (r.x == 0 && r.y == 0xFFFFFFFFu) break;
          r.x = std::min(r.x, pr.nsval);
          r.y = std::max(r.y, pr.nsval);
        }
        gns.push_back(r);
      }
    }
    c->rpu_off[2] = uint32_t(ppu.size());
    upload(c->pod_peers_u, ppu);
    upload(c->peer_ido, pi);
    gns.push_back(uint2{0u, 0xFFFFFFFFu});
    upload(c->ido_grp_ns, gns);
    const auto& ins = c->ids[1].ns;  // egress identities' namespaces, per 64-identity word
    std::vector<uint2> wns(std::max<size_t>((ins.size() + 63) / 64, 1), uint2{0xFFFFFFFFu, 0u});
    for (size_t e = 0; e < ins.size(); e++) {
      wns[e / 64].x = std::min(wns[e / 64].x, ins[e]);
      wns[e / 64].y = std::max(wns[e / 64].y, ins[e]);
    }
    upload(c->ido_word_ns, wns);
  }
  upload(c->ip_peers, ip);
  upload(c->ip_tests, tests);
  upload(c->ip_ex, c->plan.ip_ex);
  {  // IP-row work items of the fused front's segments (ip_rows_items_blk): per chunk of a segment's
     // window, its rows whose network meets the chunk's addresses (the chunk test of
     // ip_rows_fast_blk), IPI_TOUCH to a wave, and the others 64 to a wave (their chunk flags cleared)
    std::vector<DIPItem> items;
    std::vector<uint32_t> il;
    const bool one = one_window(c);
    const uint32_t NCH = (pb.W + 63) / 64;
    const bool on = c->ip_items_opt != 0 && c->ipw_h.size() == size_t(pb.W) + NCH && !pb.may_err;
    for (int x = 0; x < 2; x++) {
      c->ipi_off[x] = uint32_t(items.size());
      if (!on || (one && x)) continue;
      const int dlo = one ? 0 : x, dhi = one ? 2 : x + 1;
      const uint32_t i0 = c->ri_off[dlo], n = c->ri_off[dhi] - i0;
      uint32_t c0, nch;
      peer_chunks(c, one ? 1 : x, c0, nch);
      std::vector<uint32_t> hit, miss;
      for (uint32_t ch = c0; n && ch < c0 + nch; ch++) {
        const DWordIP& ck = c->ipw_h[pb.W + ch];
        hit.clear();
        miss.clear();
        for (uint32_t r = 0; r < n; r++) (ip_chunk_touch(tests[i0 + r].cidr, ck) ? hit : miss).push_back(r);
        for (const auto* v : {&hit, &miss}) {
          const uint32_t per = v == &hit ? IPI_TOUCH : 64u;
          for (size_t a = 0; a < v->size(); a += per) {
            const uint32_t cnt = uint32_t(std::min<size_t>(per, v->size() - a));
            items.push_back(DIPItem{ch, uint32_t(il.size()), cnt, v == &hit ? 1u : 0u});
            il.insert(il.end(), v->begin() + a, v->begin() + a + cnt);
          }
        }
      }
    }
    c->ipi_off[2] = uint32_t(items.size());
    c->ip_items = on && !items.empty();
    upload(c->ipi_items, items);
    upload(c->ipi_list, il);
  }
  clk.lap("done");
  c->order_lo = lo;
  c->order_hi = hi;
  c->order_src = src;
}

// Word window of direction d's peer rows in the current plan: [w0, w0 + nw); as 64-word chunks
// [c0, c0 + nch).
static void peer_window(const cyc_ctx* c, int d, uint32_t& w0, uint32_t& nw) {
  w0 = d == 0 ? c->win_w0 : 0u;
  nw = d == 0 ? c->win_wa : c->pb.W;
}
static void peer_chunks(const cyc_ctx* c, int d, uint32_t& c0, uint32_t& nch) {
  uint32_t w0, nw;
  peer_window(c, d, w0, nw);
  c0 = w0 / 64;
  nch = nw ? (w0 + nw + 63) / 64 - c0 : 0u;
}
// the two directions' peer rows share one window (target-row plans): one launch segment for both
static bool one_window(const cyc_ctx* c) { return c->win_w0 == 0 && c->win_wa == c->pb.W; }

// Pipeline pieces.  Steps 1, 3, 4 are shared; steps 2 and 5-7 run per direction (ingress peers,
// targets, class rows and plane are disjoint from egress ones), so the two directions can run
// as two independent branches: one direction's front hides under the other's HBM-bound emit.
enum { COMMON_SELECTORS = 1, COMMON_PORTS = 2, COMMON_FILL = 4, COMMON_ALL = 7 };
// Descriptor bit rows of the port table for the egress class rows (cyc_set_option "port_bits")
static bool port_bits_on(const cyc_ctx* c) { return std::max<size_t>(c->pb.descs.size(), 1) <= 32; }

static void enq_common(cyc_ctx* c, hipStream_t st, int parts = COMMON_ALL) {
  Problem& pb = c->pb;
  const uint32_t P = pb.P, K = pb.K, W = pb.W, D = uint32_t(std::max<size_t>(pb.descs.size(), 1));
  const uint32_t M = uint32_t(pb.pms.size());
  if ((parts & COMMON_FILL) && !pb.may_err && (c->Ri || c->Rr))  // IP-peer word spans (k_ip_rows_fast)
    k_fill_u32<<<grid1(c->pb.peers.size() * 4, 256), 256, 0, st>>>(c->ip_rng.as<uint32_t>(), c->pb.peers.size() * 4, 0xFFFFFFFFu);
  if (!(parts & COMMON_SELECTORS)) goto ports;
  // 1. selectors x label sets
  if (uint64_t(c->n_sel) * pb.L && c->dense_sel)
    k_selectors_dense<<<unsigned(uint64_t(c->n_sel) * ((pb.L + 256 * SEL_LPT - 1) / (256 * SEL_LPT))), 256, 0, st>>>(
        c->n_sel, pb.L, c->sel_off.as<uint32_t>(), c->dreqs.as<DReq>(), c->req_vals.as<uint32_t>(), c->lvt.as<uint32_t>(),
        c->selres.as<uint8_t>(), c->sel_list.as<uint32_t>());
  else if (uint64_t(c->n_sel) * pb.L)
    k_selectors<<<grid1(uint64_t(c->n_sel) * pb.L, 256), 256, 0, st>>>(
        c->n_sel, pb.L, c->sel_off.as<uint32_t>(), c->reqs.as<DReq>(), c->req_vals.as<uint32_t>(), c->ls_off.as<uint32_t>(),
        c->ls_key.as<uint32_t>(), c->ls_val.as<uint32_t>(), c->selres.as<uint8_t>(), c->sel_list.as<uint32_t>());
ports:
  if (!(parts & COMMON_PORTS)) return;
  // 3. port matchers x job descriptors
  if (M && pb.descs.size())
    k_portok<<<grid1(uint64_t(M) * D, 256), 256, 0, st>>>(M, D, c->pms.as<DPortM>(), c->pents.as<DPortEntry>(),
                                                          c->descs.as<DDesc>(), c->portok.as<uint8_t>());
  if (M && pb.descs.size() && port_bits_on(c))
    k_portbits<<<(M + 255) / 256, 256, 0, st>>>(M, D, c->portok.as<uint8_t>(), c->portbits.as<uint32_t>());
  // 4. per-slot destination words
  if (uint64_t(K) * W)
    k_slot_words<<<unsigned((uint64_t(K) * W + 3) / 4), 256, 0, st>>>(
        P, K, W, D, c->slot_desc.as<int32_t>(), c->slot_status.as<uint8_t>(), c->VALID.as<uint64_t>(),
        c->DESCW.as<int32_t>(), c->DM.as<uint64_t>());
}

// Pod peers folded into per-class identity sets, expanded by the class rows over each word's
// identity runs (no PM pod rows)?  Needs: no panic possible (the panic path walks PM / ER rows in
// peer order), few runs per word, and identity sets of bounded size.
static bool ido_mode(const cyc_ctx* c) { return c->pod_words != 0 && c->pb.blocks.empty() && ido_possible(c); }

// 2. peer rows of direction d's peers: pod peers in identity space, expanded over word runs
// (skipped in IDO mode: the class rows expand them); IP peers per pod
enum { PEERS_POD = 1, PEERS_IP = 2 };
static void enq_peer_rows(cyc_ctx* c, int d, hipStream_t st, int which = PEERS_POD | PEERS_IP) {
  Problem& pb = c->pb;
  const uint32_t P = pb.P, W = pb.W;
  const uint32_t E = c->dir[1].n;
  // d = 2: both directions in one launch (their peer sub-lists are adjacent) when they share a window
  if (d == 2 && !one_window(c)) {
    enq_peer_rows(c, 0, st, which);
    enq_peer_rows(c, 1, st, which);
    return;
  }
  const int dlo = d == 2 ? 0 : d, dhi = d == 2 ? 2 : d + 1;
  uint32_t w0, nw, c0, nch;  // the rows' word window (a source shard's ingress peers: its sources' words)
  peer_window(c, d == 2 ? 1 : d, w0, nw);
  peer_chunks(c, d == 2 ? 1 : d, c0, nch);
  const uint32_t r0 = c->rp_off[dlo], Rp = (which & PEERS_POD) ? c->rp_off[dhi] - r0 : 0u;
  if (Rp && E && W && ido_mode(c)) {
    const uint32_t EW = (E + 63) / 64;
    for (int x = dlo; x < dhi; x++) {  // per direction: its identity word window
      const uint32_t u0 = c->rpu_off[x], Ru = c->rpu_off[x + 1] - u0;  // distinct matchers only
      const uint32_t ew0 = x == 0 ? c->ido_ew0 : 0u, new_ = x == 0 ? c->ido_ew1 - c->ido_ew0 : EW;
      if (Ru && new_)
        k_peer_bits<<<unsigned((uint64_t((Ru + PB_GROUP - 1) / PB_GROUP) * new_ + 3) / 4), 256, 0, st>>>(
            Ru, E, EW, c->pod_peers_u.as<uint32_t>() + u0, c->peers.as<DPeer>(), c->selres.as<uint8_t>(), pb.L,
            c->dir[1].id_ns.as<uint32_t>(), c->id_nsls.as<uint32_t>(), c->dir[1].id_ls.as<uint32_t>(),
            c->idob.as<uint64_t>() + uint64_t(u0) * EW, ew0, new_, c->ido_grp_ns.as<uint2>() + c->ido_goff[x],
            c->ido_word_ns.as<uint2>());
    }
  } else if (Rp && E && nw && (c->pod_rows >= 0 ? c->pod_rows == 1 : uint64_t(E) * 2 >= P)) {
    const uint32_t* plist = c->pod_peers.as<uint32_t>() + r0;
    const unsigned g = unsigned((pod_direct_waves(Rp, nw) + 3) / 4);
    const uint32_t* eid = c->dir[1].pod_id.as<uint32_t>();
    if (pb.may_err)
      k_pod_rows_direct<true><<<g, 256, 0, st>>>(Rp, P, W, plist, c->peers.as<DPeer>(), c->selres.as<uint8_t>(), pb.L, eid,
                                                 c->dir[1].id_ns.as<uint32_t>(), c->id_nsls.as<uint32_t>(),
                                                 c->dir[1].id_ls.as<uint32_t>(), c->PM.as<uint64_t>(), c->ER.as<uint64_t>(), w0, nw);
    else
      k_pod_rows_direct<false><<<g, 256, 0, st>>>(Rp, P, W, plist, c->peers.as<DPeer>(), c->selres.as<uint8_t>(), pb.L, eid,
                                                  c->dir[1].id_ns.as<uint32_t>(), c->id_nsls.as<uint32_t>(),
                                                  c->dir[1].id_ls.as<uint32_t>(), c->PM.as<uint64_t>(), c->ER.as<uint64_t>(), w0, nw);
  } else if (Rp && E && nw) {
    const uint32_t* plist = c->pod_peers.as<uint32_t>() + r0;
    uint8_t* ido = c->ido.as<uint8_t>() + uint64_t(r0) * E;
    k_peer_ident<<<grid1(uint64_t(Rp) * E, 256), 256, 0, st>>>(Rp, E, plist, c->peers.as<DPeer>(), c->selres.as<uint8_t>(),
                                                               pb.L, c->dir[1].id_ns.as<uint32_t>(),
                                                               c->id_nsls.as<uint32_t>(), c->dir[1].id_ls.as<uint32_t>(), ido);
    unsigned g = unsigned(uint64_t((nw + 255) / 256) * Rp);
    if (pb.may_err)
      k_pod_rows<true><<<g, 256, 0, st>>>(Rp, E, W, plist, ido, c->word_off.as<uint32_t>(), c->run_e.as<uint32_t>(),
                                          c->run_mask.as<uint64_t>(), c->PM.as<uint64_t>(), c->ER.as<uint64_t>(), w0, nw);
    else
      k_pod_rows<false><<<g, 256, 0, st>>>(Rp, E, W, plist, ido, c->word_off.as<uint32_t>(), c->run_e.as<uint32_t>(),
                                           c->run_mask.as<uint64_t>(), c->PM.as<uint64_t>(), c->ER.as<uint64_t>(), w0, nw);
  }
  const uint32_t q0 = c->rr_off[dlo], Rr = (which & PEERS_IP) ? c->rr_off[dhi] - q0 : 0u;
  if (Rr && nw)
    k_ip_rows_range<<<(Rr + 3) / 4, 256, 0, st>>>(Rr, W, c->ipr_tests.as<DIPRange>() + q0, c->ipr_iv.as<uint2>(),
                                                c->ipsort.as<uint32_t>(), c->PM.as<uint64_t>(), c->ip_rng.as<uint32_t>(), ip_cnz(c), c0, nch);
  const uint32_t i0 = c->ri_off[dlo], Ri = (which & PEERS_IP) ? c->ri_off[dhi] - i0 : 0u;
  if (Ri && nw) {
    const DIPTest* tests = c->ip_tests.as<DIPTest>() + i0;
    if (pb.may_err) {
      // batch size: as many peers per block as keep >= ~2048 blocks in flight, at most IPB_BATCH
      const uint64_t wch = (nw + 3) / 4;
      const uint64_t nb_want = (2048 + wch - 1) / wch;
      const uint32_t bat = uint32_t(std::max<uint64_t>(1, std::min<uint64_t>(IPB_BATCH, (Ri + nb_want - 1) / nb_want)));
      unsigned g = unsigned(wch * ((Ri + bat - 1) / bat));
      k_ip_rows<true><<<g, 256, 0, st>>>(Ri, P, W, tests, c->ip_ex.as<DCidr>(), c->pod_ip.as<DIP>(), c->PM.as<uint64_t>(),
                                         c->ER.as<uint64_t>(), bat, w0, nw);
    } else {
      const uint32_t grp = IP_GROUP;
      k_ip_rows_fast<<<unsigned(ip_rows_blocks(Ri, nch, grp)), 256, 0, st>>>(
          Ri, P, W, tests, c->ip_ex.as<DCidr>(), c->pod_ip.as<DIP>(), c->ip_words.as<DWordIP>(), c->PM.as<uint64_t>(),
          c->ip_rng.as<uint32_t>(), ip_cnz(c), grp, c0, nch);
    }
  }
}

// 5. membership + classes of direction d
static void enq_member_clear(cyc_ctx* c, int d, hipStream_t st) {
  DirDev& dd = c->dir[d];
  if (dd.n) HIPCHK(hipMemsetAsync(dd.ht_key.p, 0xFF, dd.ht_key.bytes, st));  // keys and reps: one buffer
}

// The class rows of a run empty the hash table for the next one (ht_clear_slice); only runs whose
// class rows do not launch (no slots or no pods) need the memset (prepare_device empties it once).
static bool class_rows_clear_ht(const cyc_ctx* c, int d) {
  return c->dir[d].n && c->pb.K && c->pb.W && c->n_act[d];
}

static void enq_member(cyc_ctx* c, int d, hipStream_t st, bool clear = true) {
  DirDev& dd = c->dir[d];
  if (!dd.n) return;
  if (clear && !class_rows_clear_ht(c, d)) enq_member_clear(c, d, st);
  MemberArgs ma = member_args(c, d);
  if (!c->n_act[d]) return;
  // auto (-1): a wave per identity while identities are few (<= 4096) and each walks several
  // targets (>= 4 on average): config #3 (2000 identities, ~6 targets each) gains, configs #2
  // (10k identities), #4 (38k) and #5 (~0.3 targets each) lose (profiles/r01_member_wave_ab.txt)
  if (c->member_wave > 0 || (c->member_wave < 0 && c->n_act[d] <= 4096 && c->act_targets[d] >= 4.0)) k_member_wave<<<unsigned((uint64_t(c->n_act[d]) + 3) / 4), 256, 0, st>>>(ma);
  else k_member<<<grid1(c->n_act[d], 128), 128, 0, st>>>(ma);
  k_classify<<<grid1(c->n_act[d], 256), 256, 0, st>>>(ma, dd.class_of.as<uint32_t>());
}

// 6. class rows of direction d
// IDO class rows: representatives per block (cyc_set_option "class_rpb"; 0 = auto: 4, or more in
// the fused front, enq_front_fused), as many as fit the staged identity-set budget
static uint32_t class_rpb(const cyc_ctx* c, size_t per_rep_lds, uint32_t want = 0) {
  const uint64_t fit = std::max<uint64_t>(1, IDO_LDS_BYTES / std::max<size_t>(per_rep_lds, 1));
  const int64_t w = want ? int64_t(want) : c->class_rpb_opt ? c->class_rpb_opt : 4;
  return uint32_t(std::max<int64_t>(1, std::min<int64_t>(w, int64_t(fit))));
}

static RowArgs row_args(cyc_ctx* c, int d) {
  Problem& pb = c->pb;
  const uint32_t P = pb.P, K = pb.K, W = pb.W, D = uint32_t(std::max<size_t>(pb.descs.size(), 1));
  DirDev& dd = c->dir[d];
  RowArgs ra{};
  ra.tgt = dd.tgt.as<DTarget>();
  ra.peers = c->peers.as<DPeer>();
  ra.PM = c->PM.as<uint64_t>();
  ra.ER = c->ER.as<uint64_t>();
  ra.portok = c->portok.as<uint8_t>();
  // descriptor bit rows of the port table (k_portbits; computed whenever D <= 32)
  ra.portbits = port_bits_on(c) && pb.pms.size() && pb.descs.size() ? c->portbits.as<uint32_t>() : nullptr;
  ra.D = D;
  ra.n_ident = dd.n;
  ra.K = K;
  ra.W = W;
  ra.P = P;
  peer_window(c, d, ra.w0, ra.WA);  // the class rows cover their peers' word window
  if (!c->pb.blocks.empty()) {     // batched blocks: each class row covers its block's words
    ra.w0 = 0;
    ra.WA = c->blk_wa_max;
    ra.id_win = c->id_win[d].as<uint2>();
  }
  ra.class_of = dd.class_of.as<uint32_t>();
  ra.cnt = dd.cnt.as<uint32_t>();
  ra.list_off = dd.list_off.as<uint32_t>();
  ra.list = dd.list.as<uint32_t>();
  ra.id_err = dd.err.as<uint8_t>();
  ra.id_desc = dd.id_desc.as<int32_t>();
  ra.id_status = dd.id_status.as<uint8_t>();
  ra.VALID = c->VALID.as<uint64_t>();
  ra.DESCW = c->DESCW.as<int32_t>();
  ra.DM = c->DM.as<uint64_t>();
  ra.A = dd.A.as<uint64_t>();
  ra.AE = pb.may_err ? dd.AE.as<uint64_t>() : nullptr;
  ra.rep_blocks = c->n_act[d];  // k_class_rows (panic path): a block row per representative slot
  ra.reps = dd.reps.as<uint32_t>();
  ra.rep_cnt = dd.rep_cnt();
  ra.IDOB = c->idob.as<uint64_t>();
  ra.peer_ido = c->peer_ido.as<uint32_t>();
  ra.prow = c->peer_row.as<uint32_t>();
  ra.zero = c->zeros.as<uint64_t>();
  ra.runs = c->runs.as<WordRuns>();
  ra.B = dd.B.as<uint64_t>();
  ra.ip_off = dd.ip_off.as<uint32_t>();
  ra.ip_cnt = dd.ip_cnt.as<uint32_t>();
  ra.ip_list = dd.ip_list.as<uint4>();
  ra.ip_rng = c->ip_rng.as<uint32_t>();
  ra.ip_cnz = ip_cnz(c);
  ra.E = c->dir[1].n;
  ra.EW = (ra.E + 63) / 64;
  ra.ew_lo = d == 0 ? c->ido_ew0 : 0u;
  ra.ew_hi = d == 0 ? c->ido_ew1 : ra.EW;
  ra.NB = d == 0 ? K : D;
  // the first kernel below empties the hash table for the next run (keys + reps; not the counter)
  ra.ht_clear = reinterpret_cast<uint32_t*>(dd.ht_key.p);
  ra.ht_clear_words = uint64_t(dd.ht_cap) * 4;
  ra.rpb = 1;
  return ra;
}

// PM-build class rows a wave per 64-word chunk (pl_wave_chunks): both directions' accumulators fit
// (descriptors and slots <= PL_NB) and every peer's port bits are available.
static bool pl_wave_ok(const cyc_ctx* c) {
  const Problem& pb = c->pb;
  return c->pl_wave && pb.K <= PL_NB && pb.descs.size() <= PL_NB && pb.descs.size() && pb.pms.size() &&
         port_bits_on(c) && pb.W <= 64 * 64;
}

static void enq_class_rows(cyc_ctx* c, int d, hipStream_t st) {
  Problem& pb = c->pb;
  const uint32_t K = pb.K, W = pb.W, D = uint32_t(std::max<size_t>(pb.descs.size(), 1));
  DirDev& dd = c->dir[d];
  if (!dd.n || !K || !W || !c->n_act[d]) return;
  RowArgs ra = row_args(c, d);
  if (!ra.WA) return;
  if (pb.may_err) {  // the ordered walk with panic bits: one block row per identity, 8 slots per thread
    const unsigned g = unsigned(uint64_t((ra.WA + 255) / 256) * ((K + 7) / 8) * ra.rep_blocks);
    if (d == 0) k_class_rows<false><<<g, 256, 0, st>>>(ra);
    else k_class_rows<true><<<g, 256, 0, st>>>(ra);
  } else if (ido_mode(c)) {
    // identity sets first (one wave per representative and 4 slots / descriptors), then the rows
    const uint64_t waves = uint64_t(c->n_act[d]) * ((ra.NB + CI_G - 1) / CI_G);
    if (d == 0) k_class_ident<false, CI_G><<<unsigned((waves + 3) / 4), 256, 0, st>>>(ra);
    else k_class_ident<true, CI_G><<<unsigned((waves + 3) / 4), 256, 0, st>>>(ra);
    ra.ht_clear_words = 0;
    const uint32_t rows = d == 0 ? 4u : D;  // (class_rows_ido_blk stages KC = 4 slot rows, or D descriptor rows)
    const size_t per = size_t(rows) * ra.EW * 8 + IDO_IPL * sizeof(uint4) + 16;  // identity sets + staged IP peers (+ alignment)
    ra.rpb = class_rpb(c, per);
    const unsigned gi = unsigned(uint64_t(ido_chunk_groups(ra.WA)) * ((K + 3) / 4) * ((c->n_act[d] + ra.rpb - 1) / ra.rpb));
    if (d == 0) k_class_rows_ido<false, 4><<<gi, 256, per * ra.rpb, st>>>(ra);
    else k_class_rows_ido<true, 4><<<gi, 256, per * ra.rpb, st>>>(ra);
  } else {  // per-class flattened peer lists (the IP word spans are final here)
    const bool wave = pl_wave_ok(c);
    if (d == 0 && wave) k_class_rows_pl<false, true><<<pl_blocks(c, d), pl_threads(c), 0, st>>>(ra);
    else if (d == 0) k_class_rows_pl<false, false><<<pl_blocks(c, d), pl_threads(c), 0, st>>>(ra);
    else if (wave) k_class_rows_pl<true, true><<<pl_blocks(c, d), pl_threads(c), 0, st>>>(ra);
    else k_class_rows_pl<true, false><<<pl_blocks(c, d), pl_threads(c), 0, st>>>(ra);
  }
}

// 7. the emit: both planes (ingress rows to out_in, egress rows to out_eg) in one launch — two
// when their rows differ in length (a source shard: ingress rows of every destination over the
// shard's word window, egress rows of its sources over all words).  d_status (may be null): the
// status plane, copied by the (first) emit's blocks.  Returns false if no emit was launched (no rows
// in the plan; the caller then copies the status plane itself).
constexpr uint64_t EMIT_WIDE_MIN = 16384;  // shortest plane row (bytes) emitted a block per row; shorter: k_emit_flat
// k_emit_units over ea.n_rows[] rows of ea.pl_words[] words per plane (16-byte aligned planes, even
// row words): units of about one 1024 x 7 x 16 B block pass (114 KB) — whole rows of up to that, or
// several shorter rows — so a block resolves its rows' order -> identity -> class chains together
static const char* enq_emit_units(EmitArgs ea, hipStream_t st) {
  constexpr uint64_t pass = 1024 * 7 * 16;
  for (int pl = 0; pl < 2; pl++) {
    const uint64_t rb = std::max<uint64_t>(ea.pl_words[pl] * 8, 1);
    ea.unit_rows[pl] = uint32_t(std::min<uint64_t>(EMIT_UNIT_MAX_ROWS, std::max<uint64_t>(1, pass / rb)));
    ea.n_units[pl] = (ea.n_rows[pl] + ea.unit_rows[pl] - 1) / ea.unit_rows[pl];
  }
  ea.per_xcd = (ea.n_units[0] + ea.n_units[1] + 7) / 8;
  k_emit_units<1024, 7><<<ea.per_xcd * 8, 1024, 0, st>>>(ea);
  return "k_emit_units<1024,7>";
}


static const char* enq_emit_launch(const EmitArgs& ea_in, hipStream_t st, uint64_t* out_in, uint64_t* out_eg) {
  EmitArgs ea = ea_in;
  const uint32_t nr = ea.n_rows[0] + ea.n_rows[1];
  ea.per_xcd = (nr + 7) / 8;
  const uint64_t row_bytes0 = ea.row_words * 8;
  const bool aligned = reinterpret_cast<uintptr_t>(out_in) % 16 == 0 && reinterpret_cast<uintptr_t>(out_eg) % 16 == 0;
  const unsigned g = ea.per_xcd * 8;  // one block per row slot of the 8 XCD segments
  if (ea.row_words % 2 || !aligned) {
    k_emit_words<<<g, 256, 0, st>>>(ea);
    return "k_emit_words";
  }
  const uint64_t row_bytes = ea.row_words * 8;
  // A 512 x 13 one-pass block with flat addresses held 84 VGPRs, 5 waves a SIMD, and ran config #3
  // 3.5 % slower per step (profiles/r03_emit_ab.txt); through buffer ops it holds 54 (8 waves a
  // SIMD) and beats flat 1024 x 7 on a good plane placement: config #3 emit 3000 vs 3058-3070 us
  // (profiles/r04_emit_buf_ab.txt) — but over many placements 1024 x 7 through buffer ops wins on
  // average (cyc_ctx::emit_buf).
  // (128 x 13 buffer blocks for config #4's 25 KB rows lost: 442-447 vs 419-424 us.)
  if (row_bytes > 512 * 7 * 16 && row_bytes <= 512 * 13 * 16 && ea.buf == 1) {  // 56-104 KB: config #3's 98 KB rows, one pass
    k_emit_wide_buf<512, 13><<<g, 512, 0, st>>>(ea);
    return "k_emit_wide_buf<512,13>";
  } else if (row_bytes > 512 * 7 * 16 && row_bytes <= 1024 * 7 * 16 && ea.buf == 2) {
    k_emit_wide_buf<1024, 7><<<g, 1024, 0, st>>>(ea);
    return "k_emit_wide_buf<1024,7>";
  } else if (row_bytes > 512 * 7 * 16) {  // > 104 KB: 1024 x 7 passes
    k_emit_wide<1024, 7><<<g, 1024, 0, st>>>(ea);
    return "k_emit_wide<1024,7>";
  } else if (row_bytes > 256 * 8 * 16) {  // 32-56 KB: 512 x 7 (source shards at N = 2)
    k_emit_wide<512, 7><<<g, 512, 0, st>>>(ea);
    return "k_emit_wide<512,7>";
  } else if (row_bytes >= EMIT_WIDE_MIN) {  // 256-thread single pass (16-32 KB rows; buffer-op 256 x 8,
                                            // 512 x 4 and 1024 x 2 blocks were no better over 4 plane
                                            // placements of config #4, profiles/r05_plane_placement.txt)
    const uint64_t need = (ea.row_words / 2 + 255) / 256;
    if (need <= 2) k_emit_wide<256, 2><<<g, 256, 0, st>>>(ea);
    else if (need <= 4) k_emit_wide<256, 4><<<g, 256, 0, st>>>(ea);
    else if (need <= 6) k_emit_wide<256, 6><<<g, 256, 0, st>>>(ea);
    else if (need <= 7) k_emit_wide<256, 7><<<g, 256, 0, st>>>(ea);
    else k_emit_wide<256, 8><<<g, 256, 0, st>>>(ea);
    return need <= 2 ? "k_emit_wide<256,2>" : need <= 4 ? "k_emit_wide<256,4>" : need <= 6 ? "k_emit_wide<256,6>"
         : need <= 7 ? "k_emit_wide<256,7>" : "k_emit_wide<256,8>";
  } else {  // flat multi-row sweep over ~32 KB per block
    ea.chunk = uint32_t(std::min<uint64_t>(EMIT_FLAT_MAX_ROWS, std::max<uint64_t>(1, 32768 / row_bytes)));
    k_emit_flat<256, 8><<<(ea.per_xcd + ea.chunk - 1) / ea.chunk * 8, 256, 0, st>>>(ea);
    return "k_emit_flat<256,8>";
  }
}

static bool enq_emit_blocks(cyc_ctx* c, hipStream_t st, uint64_t* out_in, uint64_t* out_eg, uint8_t* d_status) {
  Problem& pb = c->pb;
  if (pb.blocks.empty()) return false;
  if (!pb.K || !d_status) return true;  // nothing to write (the status plane of blocks is their slabs)
  BlockArgs ba{};
  ba.n_blk = uint32_t(pb.blocks.size());
  ba.K = pb.K;
  ba.AS = c->blk_wa_max;
  ba.blk = c->blk.as<uint4>();
  ba.boff = c->blk_off.as<uint64_t>();
  for (int pl = 0; pl < 2; pl++) {
    ba.pod_id[pl] = c->dir[pl].pod_id.as<uint32_t>();
    ba.class_of[pl] = c->dir[pl].class_of.as<uint32_t>();
    ba.A[pl] = c->dir[pl].A.as<uint64_t>();
  }
  ba.st_src = c->slot_status.as<uint8_t>();
  ba.out[0] = out_in;
  ba.out[1] = out_eg;
  ba.st_out = d_status;
  // a block's slab words split over workgroups of ~16 words per thread (one workgroup per block
  // left a few large blocks on a few CUs); small blocks' extra workgroups exit at once
  const unsigned bs = c->blk_np_max * 2 > 128 ? 256 : 128;
  const uint64_t most = 2ull * c->blk_np_max * pb.K * ((c->blk_np_max + 63) / 64);  // largest slab, both planes
  ba.split = uint32_t(std::min<uint64_t>(64, std::max<uint64_t>(1, most / (uint64_t(bs) * 16))));
  k_emit_blocks<<<ba.n_blk * ba.split, bs, 0, st>>>(ba);
  return true;
}

static bool enq_emit(cyc_ctx* c, hipStream_t st, uint64_t* out_in, uint64_t* out_eg, uint8_t* d_status, bool inplace = false) {
  Problem& pb = c->pb;
  c->ip_rng_clean = false;  // (set again below when this emit resets the spans for the next run)
  const uint32_t K = pb.K;
  const uint64_t rw[2] = {uint64_t(K) * c->win_wa, uint64_t(K) * pb.W};  // words per plane row
  uint32_t nr[2];
  for (int d = 0; d < 2; d++) nr[d] = rw[d] ? uint32_t(c->rh[d] - c->rl[d]) : 0u;
  c->emit_kernel.clear();
  c->emit_launches = 0;
  if (!pb.blocks.empty()) {
    const bool r = enq_emit_blocks(c, st, out_in, out_eg, d_status);
    if (r && pb.K && d_status) c->emit_kernel = "k_emit_blocks", c->emit_launches = 1;
    return r;
  }
  if (!nr[0] && !nr[1]) return false;
  EmitArgs ea{};
  ea.st_src = c->slot_status.as<uint8_t>();
  ea.st_dst = d_status;
  ea.st_bytes = d_status ? uint64_t(pb.P) * K : 0;
  ea.reset = c->ip_rng.as<uint32_t>();
  ea.reset_n = pb.may_err ? 0u : uint64_t(pb.peers.size()) * 4;  // (k_ip_rows with panics keeps no spans)
  ea.buf = uint32_t(c->emit_buf);
  c->ip_rng_clean = ea.reset_n != 0;
  for (uint32_t pl = 0; pl < 2; pl++) {
    ea.row_lo[pl] = uint32_t(c->rl[pl]);
    ea.order[pl] = c->order[pl].as<uint2>();
    ea.class_of[pl] = c->dir[pl].class_of.as<uint32_t>();
    ea.A[pl] = c->dir[pl].A.as<uint64_t>();
    ea.arow[pl] = inplace ? c->arow[pl].as<uint32_t>() : nullptr;
  }
  ea.out[0] = out_in;
  ea.out[1] = out_eg;
  ea.pl_words[0] = rw[0];
  ea.pl_words[1] = rw[1];
  auto note = [&](const char* k) {  // what cyc_last_emit reports
    if (c->emit_kernel.find(k) == std::string::npos) c->emit_kernel += (c->emit_kernel.empty() ? "" : " + ") + std::string(k);
    c->emit_launches++;
  };
  if (rw[0] == rw[1] && nr[0] == nr[1]) {  // target rows: both planes in one launch
    ea.row_words = rw[0];
    // alternate the planes' rows when each plane is >= 8 GB (config #3 on one GPU: emit 3.42 ->
    // 3.11 ms on two of three boxes, -1 % on the third; 1-4 % slower for planes of <= 5 GB — 2, 4
    // and 8 shards — profiles/r01_emit_interleave_sweep.txt)
    ea.interleave = c->emit_interleave >= 0 ? uint32_t(c->emit_interleave)
                                            : uint64_t(nr[0]) * rw[0] * 8 >= (8ull << 30) ? 1u : 0u;
    // emit_split > 1: consecutive parts of both planes' row lists (class-clustered, so nearly address
    // order) as separate launches, the first carrying the status copy and the span reset
    const uint32_t parts = uint32_t(std::max(1, std::min<int>(c->emit_split, int(std::max<uint32_t>(nr[0], 1)))));
    for (uint32_t h = 0; h < parts; h++) {
      const uint32_t r0 = uint32_t(uint64_t(nr[0]) * h / parts), r1 = uint32_t(uint64_t(nr[0]) * (h + 1) / parts);
      EmitArgs e1 = ea;
      e1.n_rows[0] = e1.n_rows[1] = r1 - r0;
      for (int pl = 0; pl < 2; pl++) e1.order[pl] = ea.order[pl] + r0;
      if (h) e1.st_bytes = e1.reset_n = 0;
      note(enq_emit_launch(e1, st, out_in, out_eg));
    }
    return true;
  }
  // rows of different lengths (a source shard): ONE launch over units of about one block pass each
  const bool aligned = reinterpret_cast<uintptr_t>(out_in) % 16 == 0 && reinterpret_cast<uintptr_t>(out_eg) % 16 == 0;
  if (aligned && rw[0] % 2 == 0 && rw[1] % 2 == 0) {
    ea.n_rows[0] = nr[0];
    ea.n_rows[1] = nr[1];
    note(enq_emit_units(ea, st));
    return true;
  }
  bool first = true;
  for (int pl = 0; pl < 2; pl++) {  // (8-byte row words or unaligned planes) one launch per plane
    if (!nr[pl]) continue;
    EmitArgs e1 = ea;
    e1.n_rows[0] = pl == 0 ? nr[0] : 0u;  // the row list is [plane 0 rows][plane 1 rows]
    e1.n_rows[1] = pl == 1 ? nr[1] : 0u;
    e1.row_words = rw[pl];
    if (!first) e1.st_bytes = e1.reset_n = 0;
    first = false;
    note(enq_emit_launch(e1, st, pl == 0 ? out_in : reinterpret_cast<uint64_t*>(16), pl == 1 ? out_eg : reinterpret_cast<uint64_t*>(16)));
  }
  return true;
}

// The fused front (k_front_a..e, one stream): the same block ranges the two-branch DAG launches
// as ~15 kernels (enq_common, enq_peer_rows, enq_member, enq_class_rows), grouped by dependency
// level.  Applies to no-panic builds with dense selectors whose pod-peer rows (PM builds) are
// computed per pod in one level; returns false (nothing enqueued) otherwise.
static bool front_fused_ok(const cyc_ctx* c) {
  const Problem& pb = c->pb;
  if (!c->front_fused || pb.may_err) return false;
  if (!pb.P || !pb.K || !pb.W) return false;
  if (uint64_t(c->n_sel) * pb.L && !c->dense_sel) return false;
  if (ido_mode(c)) return true;
  const uint32_t E = c->dir[1].n, Rp = c->rp_off[2] - c->rp_off[0];
  return !(Rp && E) || (c->pod_rows >= 0 ? c->pod_rows == 1 : uint64_t(E) * 2 >= pb.P);
}

// In-place class rows: the fused front with both output planes given.
// Auto (-1): when the rows' identities are >= 1/16 of the rows (PM builds: config #4 emit -8 %,
// #3u -7 %), and for identity-set (IDO) runs: config #3's class rows are 2 % of its rows,
// and writing them into the planes saves their 400 MB of separate writes (3.286 -> 3.191 ms/step,
// profiles/r05_inplace_sweep_ab.txt; over 5 plane placements in one process -2.1 / -0.0 / -0.1 /
// -2.8 / -2.2 %, never slower: profiles/r05_plane_placement.txt; a source shard at N = 8 -1.2 %,
// r05_shard_ab.txt; in round 2, before the current launch E, it lost 1 %).
static bool inplace_ok(const cyc_ctx* c, const uint64_t* d_in, const uint64_t* d_eg) {
  if (!c->class_inplace || !d_in || !d_eg || !front_fused_ok(c) || !c->pb.blocks.empty()) return false;
  const uint64_t rows = uint64_t(std::max<int64_t>((c->rh[0] - c->rl[0] + c->rh[1] - c->rl[1]) / 2, 1));
  return c->class_inplace == 1 || uint64_t(c->n_act[0] + c->n_act[1]) * 16 >= 2 * rows || ido_mode(c);
}

// out_in / out_eg non-null: the class rows go straight into those planes (in-place class rows; the
// emit must then be enqueued with inplace = true).
static bool enq_front_fused(cyc_ctx* c, hipStream_t st, hipEvent_t ev_front = nullptr, hipEvent_t ev_rows = nullptr,
                            uint64_t* out_in = nullptr, uint64_t* out_eg = nullptr) {
  Problem& pb = c->pb;
  const uint32_t P = pb.P, K = pb.K, W = pb.W, D = uint32_t(std::max<size_t>(pb.descs.size(), 1));
  const uint32_t M = uint32_t(pb.pms.size()), E = c->dir[1].n, EW = (E + 63) / 64;
  bool fits = true;  // every launch's block count below 2^31 (else the DAG path runs)
  auto blocks = [&fits](uint64_t n) {
    fits = fits && n < (1ull << 30);
    return uint32_t(n);
  };
  // A: IP word spans | port table | slot words | selectors
  FrontA fa{};
  fa.fill_p = c->ip_rng.as<uint32_t>();
  // the word spans and chunk masks of the IP rows and of PM builds' sparse pod rows (cnz needs no reset)
  fa.fill_n = (c->Ri || c->Rr || (!ido_mode(c) && c->Rp)) ? pb.peers.size() * 4 : 0;
  fa.nb[0] = blocks((fa.fill_n + 255) / 256);
  fa.M = M;
  fa.D = D;
  fa.P = P;
  fa.K = K;
  fa.W = W;
  fa.pms = c->pms.as<DPortM>();
  fa.pents = c->pents.as<DPortEntry>();
  fa.descs = c->descs.as<DDesc>();
  fa.portok = c->portok.as<uint8_t>();
  fa.nb[1] = (M && pb.descs.size()) ? blocks((uint64_t(M) * D + 255) / 256) : 0u;
  fa.slot_desc = c->slot_desc.as<int32_t>();
  fa.slot_status = c->slot_status.as<uint8_t>();
  fa.VALID = c->VALID.as<uint64_t>();
  fa.DESCW = c->DESCW.as<int32_t>();
  fa.DM = c->DM.as<uint64_t>();
  // the slot words (VALID / DESCW / DM per 64 destinations) serve only egress class rows whose
  // destinations do not all share each slot's descriptor (uni_desc: the UNI class rows read udesc)
  const bool slot_words = !c->uni_desc || !(ido_mode(c) || pl_wave_ok(c)) || !c->pb.blocks.empty();
  fa.nb[2] = slot_words ? blocks((uint64_t(K) * W + 3) / 4) : 0u;
  fa.S = c->n_sel;
  fa.L = pb.L;
  fa.sel_off = c->sel_off.as<uint32_t>();
  fa.dreqs = c->dreqs.as<DReq>();
  fa.req_vals = c->req_vals.as<uint32_t>();
  fa.LVT = c->lvt.as<uint32_t>();
  fa.selres = c->selres.as<uint8_t>();
  fa.sel_list = c->sel_list.as<uint32_t>();
  fa.nb[3] = uint64_t(c->n_sel) * pb.L && !lazy_sel(c) ? blocks(uint64_t(c->n_sel) * ((pb.L + 256 * SEL_LPT - 1) / (256 * SEL_LPT))) : 0u;
  // B: IP rows | pod-peer identity sets (both directions' adjacent sub-lists) | membership x 2
  // Segments x = 0, 1 of the IP rows and per-pod pod rows: the directions' sub-lists with their own
  // word windows (source shards), or both directions in segment 0 (one window)
  const bool one_win = one_window(c);
  FrontB fb{};
  fb.P = P;
  fb.W = W;
  fb.ip_ex = c->ip_ex.as<DCidr>();
  fb.pod_ip = c->pod_ip.as<DIP>();
  fb.words = c->ip_words.as<DWordIP>();
  fb.PM = c->PM.as<uint64_t>();
  fb.rng = c->ip_rng.as<uint32_t>();
  fb.cnz = ip_cnz(c);
  fb.ip_grp = IP_GROUP;
  fb.ipr_iv = c->ipr_iv.as<uint2>();
  fb.ipsort = c->ipsort.as<uint32_t>();
  fb.ip_ilist = c->ipi_list.as<uint32_t>();
  for (int x = 0; x < 2; x++) {
    const int dlo = one_win ? 0 : x, dhi = one_win ? 2 : x + 1;
    const uint32_t i0 = c->ri_off[dlo];
    fb.Ri[x] = one_win && x ? 0u : c->ri_off[dhi] - i0;
    fb.tests[x] = c->ip_tests.as<DIPTest>() + i0;
    peer_chunks(c, one_win ? 1 : x, fb.ic0[x], fb.inch[x]);
    fb.nb[x] = fb.Ri[x] && fb.inch[x] ? blocks(ip_rows_blocks(fb.Ri[x], fb.inch[x], fb.ip_grp)) : 0u;
    if (c->ip_items && fb.nb[x]) {  // the range plan's work items of this segment
      fb.ip_items[x] = c->ipi_items.as<DIPItem>() + c->ipi_off[x];
      fb.n_ip_items[x] = c->ipi_off[x + 1] - c->ipi_off[x];
      fb.nb[x] = blocks((uint64_t(fb.n_ip_items[x]) + 3) / 4);
    }
    fb.Rr[x] = one_win && x ? 0u : c->rr_off[dhi] - c->rr_off[dlo];
    fb.rtests[x] = c->ipr_tests.as<DIPRange>() + c->rr_off[dlo];
    fb.nb[9 + x] = fb.Rr[x] && fb.inch[x] ? blocks((uint64_t(fb.Rr[x]) + 3) / 4) : 0u;
  }
  fb.E = E;
  fb.EW = EW;
  fb.L = pb.L;
  fb.peers = c->peers.as<DPeer>();
  fb.selres = c->selres.as<uint8_t>();
  fb.id_ns = c->dir[1].id_ns.as<uint32_t>();
  fb.id_nsls = c->id_nsls.as<uint32_t>();
  fb.id_ls = c->dir[1].id_ls.as<uint32_t>();
  fb.sv = sel_view(c);
  fb.word_ns = c->ido_word_ns.as<uint2>();
  for (int x = 0; x < 2; x++) {  // identity sets per direction: the ingress ones over the window's identity words
    const uint32_t ux = c->rpu_off[x];
    fb.Ru_[x] = c->rpu_off[x + 1] - ux;
    fb.pod_peers_u_[x] = c->pod_peers_u.as<uint32_t>() + ux;
    fb.idob_[x] = c->idob.as<uint64_t>() + uint64_t(ux) * EW;
    fb.grp_ns_[x] = c->ido_grp_ns.as<uint2>() + c->ido_goff[x];
    fb.ew0[x] = x == 0 ? c->ido_ew0 : 0u;
    fb.new_[x] = x == 0 ? c->ido_ew1 - c->ido_ew0 : EW;
    fb.nb[2 + x] = (fb.Ru_[x] && E && fb.new_[x]) ? blocks((uint64_t((fb.Ru_[x] + PB_GROUP - 1) / PB_GROUP) * fb.new_[x] + 3) / 4) : 0u;
  }
  const bool ido = ido_mode(c);
  FrontC fc{};
  if (!ido && !pod_sparse(c)) {  // PM builds, few pod-peer words: full rows, a wave per (pod peer, word)
    fb.pod_direct = 1;
    fb.pod_eid = c->dir[1].pod_id.as<uint32_t>();
    for (int x = 0; x < 2; x++) {
      const int dlo = one_win ? 0 : x, dhi = one_win ? 2 : x + 1;
      fb.Rp[x] = one_win && x ? 0u : c->rp_off[dhi] - c->rp_off[dlo];
      fb.plist[x] = c->pod_peers.as<uint32_t>() + c->rp_off[dlo];
      peer_window(c, one_win ? 1 : x, fb.pw0[x], fb.pnw[x]);
      fb.nb[2 + x] = (fb.Rp[x] && E && fb.pnw[x]) ? blocks((pod_direct_waves(fb.Rp[x], fb.pnw[x]) + 3) / 4) : 0u;
    }
  } else if (!ido) {  // PM builds: sparse pod-peer rows in launch C (k_front_c)
    fb.nb[2] = fb.nb[3] = 0;
    fc.P = P;
    fc.W = W;
    fc.req_post = c->req_post.as<uint4>();
    fc.post_pods = c->post_pods.as<uint32_t>();
    fc.peers = c->peers.as<DPeer>();
    fc.pod_ns = c->pod_ns.as<uint32_t>();
    fc.pod_nsls = c->pod_nsls.as<uint32_t>();
    fc.pod_ls = c->pod_ls.as<uint32_t>();
    fc.nsw = c->ns_words.as<DWordNS>();
    fc.sv = sel_view(c);
    fc.PM = c->PM.as<uint64_t>();
    fc.rng = c->ip_rng.as<uint32_t>();
    fc.cnz = ip_cnz(c);
    // a wave per chunk over groups of 8 peers once that fills the chip (>= 64k peer chunks:
    // config #3u 2.6 vs 3.2 ms), else the 4 waves of a block share each chunk (config #2)
    uint64_t peer_chunks_all = 0;
    for (int x = 0; x < 2; x++) {
      const int dlo = one_win ? 0 : x, dhi = one_win ? 2 : x + 1;
      fc.Rp[x] = one_win && x ? 0u : c->scan_off[dhi] - c->scan_off[dlo];
      fc.plist[x] = c->pp_scan.as<uint32_t>() + c->scan_off[dlo];
      fc.plist_post[x] = c->pp_post.as<uint32_t>() + c->post_off[dlo];
      peer_chunks(c, one_win ? 1 : x, fc.c0[x], fc.nch[x]);
      peer_chunks_all += uint64_t(fc.Rp[x]) * fc.nch[x];
    }
    fc.pr_grp = c->pr_group > 0 ? uint32_t(c->pr_group) : (peer_chunks_all >= 65536 ? 8u : 1u);
    for (int x = 0; x < 2; x++) {
      const int dlo = one_win ? 0 : x, dhi = one_win ? 2 : x + 1;
      const uint64_t cb = (fc.nch[x] + 3) / 4;
      fc.nb[2 + x] = (fc.Rp[x] && E && cb) ? blocks((uint64_t(fc.Rp[x]) + fc.pr_grp - 1) / fc.pr_grp * cb) : 0u;
      fc.nb[4 + x] = E && fc.nch[x] && !(one_win && x) ? c->post_off[dhi] - c->post_off[dlo] : 0u;  // a block per posting-built peer
    }
  }
  FrontRows fd{}, fe{};
  size_t lds = 0, lds_uni = 0, e_per[2] = {0, 0};
  uint32_t e_na[2] = {0, 0};
  for (int d = 0; d < 2; d++) {
    const uint32_t na = c->dir[d].n ? c->n_act[d] : 0u;
    fb.ma[d] = member_args(c, d);
    fc.ma[d] = fb.ma[d];
    fc.class_of[d] = c->dir[d].class_of.as<uint32_t>();
    fb.member_wave[d] = c->member_wave > 0 || (c->member_wave < 0 && na <= 4096 && c->act_targets[d] >= 4.0);
    fb.nb[4 + d] = na ? blocks(fb.member_wave[d] ? (uint64_t(na) + 3) / 4 : (uint64_t(na) + 255) / 256) : 0u;
    fc.nb[d] = na ? blocks((uint64_t(na) + 255) / 256) : 0u;
    if (!na) continue;
    fd.ra[d] = row_args(c, d);  // its blocks empty the direction's hash table for the next run
    if (out_in && out_eg) {
      fd.ra[d].A = d == 0 ? out_in : out_eg;
      fd.ra[d].arow = c->arow[d].as<uint32_t>();
    }
    // (the class election keeps a launch of its own, C: electing inside the next launch's blocks put
    // the election chain on every block — IDO identity sets C + D 29 -> 45 us, PM class rows C + D
    // 79 -> 117 us on config #4: profiles/r04_elect_ab.txt)
    if (!ido) {  // PM builds: launch D (k_front_d_pm) is the class rows from flattened peer lists
      fd.nb[d] = pl_blocks(c, d);
      if (d == 1 && c->uni_desc && c->pb.blocks.empty()) fd.ra[d].udesc = c->udesc.as<int32_t>();
      fd.ra[d].pod_sparse = pod_sparse(c);  // pod rows from pod_rows_sparse_blk (launch C)
      continue;
    }
    fe.ra[d] = fd.ra[d];
    fe.ra[d].ht_clear_words = 0;  // (launch D's identity sets empty it)
    fd.nb[d] = blocks((uint64_t(na) * ((fd.ra[d].NB + CI_G - 1) / CI_G) + 3) / 4);
    // egress with one descriptor per slot (udesc): only the block's slots' sets are staged
    if (d == 1 && c->uni_desc) fe.ra[d].udesc = c->udesc.as<int32_t>();
    e_per[d] = size_t(d == 0 || fe.ra[d].udesc ? uint32_t(E_KC) : D) * fd.ra[d].EW * 8 +
               IDO_IPL * sizeof(uint4) + 16;  // identity sets + staged IP peers (+ alignment)
    e_na[d] = na;
  }
  // launch E's representatives per block: the most of 16 / 8 that still leaves >= 3000 blocks
  // (about two rounds of the chip's resident blocks: one block's staging latency is paid once per
  // 16 representatives), else 4 (config #3: E 106 -> 96 us at N = 1 with 16; at N = 8 a source
  // shard's ~1,900 blocks of 4 ran 22.8 us, of 8 24.0 — profiles/r04_class_rpb_ab.txt)
  auto e_blocks = [&](int d, uint32_t rpb) {
    return uint64_t(ido_chunk_groups(fe.ra[d].WA)) * ((K + E_KC - 1) / E_KC) * ((e_na[d] + rpb - 1) / rpb);
  };
  uint32_t e_want = uint32_t(c->class_rpb_opt);
  if (!e_want) {
    e_want = 4;
    for (uint32_t cand : {16u, 8u}) {
      uint64_t tot = 0;
      for (int d = 0; d < 2; d++)
        if (e_per[d]) tot += e_blocks(d, class_rpb(c, e_per[d], cand));
      if (tot >= 3000) {
        e_want = cand;
        break;
      }
    }
  }
  for (int d = 0; d < 2; d++) {
    if (!e_per[d]) continue;
    fe.ra[d].rpb = class_rpb(c, e_per[d], e_want);
    fe.nb[d] = blocks(e_blocks(d, fe.ra[d].rpb));
    if (d == 1 && fe.ra[d].udesc) lds_uni = e_per[d] * fe.ra[d].rpb;
    else lds = std::max<size_t>(lds, e_per[d] * fe.ra[d].rpb);
  }
  // membership ahead of the rest of launch B unless the IP rows alone fill the chip (~2k resident blocks)
  fb.member_first = uint64_t(fb.nb[0]) + fb.nb[1] < 2048;
  const bool bits = fa.nb[1] && port_bits_on(c);
  const uint32_t nb_bits = bits ? blocks((uint64_t(M) + 255) / 256) : 0u;
  fb.M = M;
  fb.D = D;
  fb.portok = c->portok.as<uint8_t>();
  fb.portbits = c->portbits.as<uint32_t>();
  fb.nb[6] = nb_bits;
  fe.ra[1].portbits = bits && fe.nb[1] ? c->portbits.as<uint32_t>() : nullptr;
  // Without a selector table to build (lazy selectors) launch A is dropped: its port table, slot
  // words and port bits (from the matchers directly) join launch B — their readers are the class
  // rows, launches D / E — and the IP rows' word spans were reset by the previous run's emit
  // (EmitArgs::reset; a memset when they were not).  Captured graphs keep launch A: a replay must not
  // depend on the step before it.
  if (fa.nb[3] == 0 && !c->capturing) {
    fb.pre = fa;
    fb.bits_direct = 1;
    fb.nb[7] = fa.nb[1];
    fb.nb[8] = fa.nb[2];
    if (fa.fill_n && !c->ip_rng_clean) HIPCHK(hipMemsetAsync(fa.fill_p, 0xFF, fa.fill_n * 4, st));
    fa.nb[0] = fa.nb[1] = fa.nb[2] = 0;
  }
  const uint64_t ga = uint64_t(fa.nb[0]) + fa.nb[1] + fa.nb[2] + fa.nb[3];
  uint64_t gb = 0, gc = 0;
  for (uint32_t x : fb.nb) gb += x;
  for (uint32_t x : fc.nb) gc += x;
  if (!fits || gb >= (1ull << 31) || gc >= (1ull << 31)) return false;
  if (ga) k_front_a<<<unsigned(ga), 256, 0, st>>>(fa);
  if (gb) k_front_b<<<unsigned(gb), 256, 0, st>>>(fb);
  if (gc) k_front_c<<<unsigned(gc), 256, 0, st>>>(fc);
  if (ev_front) HIPCHK(hipEventRecord(ev_front, st));  // eager runs: phase timings
  if (!ido) {
    const unsigned gd = fd.nb[0] + fd.nb[1];
    if (gd && pl_wave_ok(c)) k_front_d_pm<true><<<gd, pl_threads(c), 0, st>>>(fd);
    else if (gd) k_front_d_pm<false><<<gd, pl_threads(c), 0, st>>>(fd);
    if (ev_rows) HIPCHK(hipEventRecord(ev_rows, st));
    return true;
  }
  if (fd.nb[0] + fd.nb[1]) k_front_d<<<fd.nb[0] + fd.nb[1], 256, 0, st>>>(fd);
  if (fe.nb[0] && fe.nb[1] && fe.ra[1].udesc) {
    k_front_e_uni<<<fe.nb[0] + fe.nb[1], 256, std::max(lds, lds_uni), st>>>(fe);
  } else {  // the directions' class rows as two launches, each at its own register budget (egress 101
            // VGPRs, ingress 61: one launch at 101 ran config #3 189 -> 170 us, profiles/r03_e_split_ab.txt)
    if (fe.nb[1] && fe.ra[1].udesc) k_class_rows_ido<true, E_KC, true><<<fe.nb[1], 256, lds_uni, st>>>(fe.ra[1]);
    else if (fe.nb[1]) k_class_rows_ido<true, E_KC><<<fe.nb[1], 256, lds, st>>>(fe.ra[1]);
    if (fe.nb[0]) k_class_rows_ido<false, E_KC><<<fe.nb[0], 256, lds, st>>>(fe.ra[0]);
  }
  if (ev_rows) HIPCHK(hipEventRecord(ev_rows, st));
  return true;
}

// Eager launch, in phase order with the timing events: [0] start, [1] after the front (peer
// rows, classes), [2] after the class rows, [3] after both emits.
static void enqueue_pipeline(cyc_ctx* c, hipStream_t st, uint64_t* d_in, uint64_t* d_eg, uint8_t* d_status) {
  Problem& pb = c->pb;
  HIPCHK(hipEventRecord(c->ev[0], st));
  const bool ip = inplace_ok(c, d_in, d_eg);
  const bool fused = front_fused_ok(c) && enq_front_fused(c, st, c->ev[1], c->ev[2], ip ? d_in : nullptr, ip ? d_eg : nullptr);
  if (!fused) {
    enq_common(c, st);
    for (int d = 0; d < 2; d++) enq_peer_rows(c, d, st);
    for (int d = 0; d < 2; d++) enq_member(c, d, st);
    HIPCHK(hipEventRecord(c->ev[1], st));
    for (int d = 0; d < 2; d++) enq_class_rows(c, d, st);
    HIPCHK(hipEventRecord(c->ev[2], st));
  }
  const bool status_done = enq_emit(c, st, d_in, d_eg, d_status, ip && fused);
  HIPCHK(hipEventRecord(c->ev[3], st));
  if (!status_done && d_status && uint64_t(pb.P) * pb.K)
    HIPCHK(hipMemcpyAsync(d_status, c->slot_status.p, uint64_t(pb.P) * pb.K, hipMemcpyDeviceToDevice, st));
}

// Graph capture / eager DAG: the fused front on st when it applies; else the two-branch DAG:
// [st3] IP rows of both directions + port tables || [st] selectors, then per direction (ingress on
// st, egress on st2) pod-peer sets -> membership / classes -> (wait for st3) class rows, joined
// into one emit of both planes (fork / join through events, graph dependencies when captured).
static void capture_pipeline(cyc_ctx* c, hipStream_t st, hipStream_t st2, hipStream_t st3, uint64_t* d_in, uint64_t* d_eg,
                             uint8_t* d_status) {
  Problem& pb = c->pb;
  const bool ip = inplace_ok(c, d_in, d_eg);
  if (front_fused_ok(c) && enq_front_fused(c, st, nullptr, nullptr, ip ? d_in : nullptr, ip ? d_eg : nullptr)) {
    if (enq_emit(c, st, d_in, d_eg, d_status, ip)) return;
  } else {
    HIPCHK(hipEventRecord(c->fork_ev, st));
    HIPCHK(hipStreamWaitEvent(st3, c->fork_ev, 0));
    enq_common(c, st3, COMMON_FILL | COMMON_PORTS);
    enq_peer_rows(c, 2, st3, PEERS_IP);  // both directions' IP rows in one launch
    HIPCHK(hipEventRecord(c->ports_ev, st3));
    enq_common(c, st, COMMON_SELECTORS);
    HIPCHK(hipEventRecord(c->sel_ev, st));
    HIPCHK(hipStreamWaitEvent(st2, c->sel_ev, 0));
    for (int d = 1; d >= 0; d--) {
      hipStream_t s = d ? st2 : st;
      enq_peer_rows(c, d, s, PEERS_POD);
      enq_member(c, d, s);
      HIPCHK(hipStreamWaitEvent(s, c->ports_ev, 0));
      enq_class_rows(c, d, s);
    }
    HIPCHK(hipEventRecord(c->join_ev, st2));
    HIPCHK(hipStreamWaitEvent(st, c->join_ev, 0));
    // the emit also writes the status plane; the copy node below only ends steps without rows
    if (enq_emit(c, st, d_in, d_eg, d_status)) return;
  }
  // The step always ends with the status-plane copy (into a sink buffer when the caller passed no
  // status pointer), so every captured graph has the same shape: one node after the join.
  const uint64_t nst = uint64_t(pb.P) * pb.K;
  uint8_t* dst = d_status && nst ? d_status : c->status_sink.as<uint8_t>();  // sink: >= 16 B (prepare_device)
  HIPCHK(hipMemcpyAsync(dst, c->slot_status.p, std::max<uint64_t>(nst, 1), hipMemcpyDeviceToDevice, st));
}

// Destroy the retired execs whose last launch has completed (all of them when `wait`).
static void reap_graphs(cyc_ctx* c, bool wait) {
  size_t keep = 0;
  for (size_t i = 0; i < c->retired.size(); i++) {
    cyc_ctx::Retired& r = c->retired[i];
    if (r.done && wait) (void)hipEventSynchronize(r.done);
    const bool done = !r.done || wait || hipEventQuery(r.done) != hipErrorNotReady;
    if (!done) {
      c->retired[keep++] = r;
      continue;
    }
    (void)hipGraphExecDestroy(r.exec);
    if (r.graph) (void)hipGraphDestroy(r.graph);
    if (r.done) (void)hipEventDestroy(r.done);
  }
  c->retired.resize(keep);
}

static void drop_graph(cyc_ctx* c) {
  if (c->graph_exec) c->retired.push_back({c->graph_exec, c->graph, c->graph_done});
  c->graph_exec = nullptr;
  c->graph = nullptr;
  c->graph_done = nullptr;
  reap_graphs(c, false);
}

static void ensure_cap_streams(cyc_ctx* c) {
  if (c->cap_stream) return;
  HIPCHK(hipStreamCreateWithFlags(&c->cap_stream, hipStreamNonBlocking));
  HIPCHK(hipStreamCreateWithFlags(&c->cap_stream2, hipStreamNonBlocking));
  HIPCHK(hipStreamCreateWithFlags(&c->cap_stream3, hipStreamNonBlocking));
  HIPCHK(hipEventCreateWithFlags(&c->sel_ev, EV_SYNC));
  HIPCHK(hipEventCreateWithFlags(&c->ports_ev, EV_SYNC));
  HIPCHK(hipEventCreateWithFlags(&c->fork_ev, EV_SYNC));
  HIPCHK(hipEventCreateWithFlags(&c->join_ev, EV_SYNC));
}

// Batched blocks: each block's status, as its stand-alone run would end — the job expansion's
// panic, else its first panicking job (its own job order), else its table build's duplicate key —
// into c->blk_rc / c->blk_msg.  Synchronises only when the inputs can panic.
static int blocks_status(cyc_ctx* c, hipStream_t st) {
  Problem& pb = c->pb;
  const size_t nb = pb.blocks.size();
  c->blk_rc.assign(nb, CYC_OK);
  c->blk_msg.assign(nb, "");
  std::vector<unsigned long long> first(nb, ~0ull);
  if (pb.may_err && pb.P && pb.K) {
    HIPCHK(hipMemsetAsync(c->first_blk.p, 0xFF, nb * 8, st));
    BlockErrArgs e{};
    e.n_blk = uint32_t(nb);
    e.P = pb.P;
    e.K = pb.K;
    e.AS = c->blk_wa_max;
    e.blk = c->blk.as<uint4>();
    e.pod_blk = nullptr;
    e.slot_idx = c->slot_idx.as<uint32_t>();
    e.slot_status = c->slot_status.as<uint8_t>();
    e.pod_iid = c->dir[0].pod_id.as<uint32_t>();
    e.pod_eid = c->dir[1].pod_id.as<uint32_t>();
    e.class_in = c->dir[0].class_of.as<uint32_t>();
    e.class_eg = c->dir[1].class_of.as<uint32_t>();
    e.err_in = c->dir[0].err.as<uint8_t>();
    e.err_eg = c->dir[1].err.as<uint8_t>();
    e.AE_in = c->dir[0].AE.as<uint64_t>();
    e.AE_eg = c->dir[1].AE.as<uint64_t>();
    e.first = c->first_blk.as<unsigned long long>();
    e.dchunks = (c->blk_np_max + 255) / 256;
    DevBuf pod_blk;
    upload(pod_blk, pb.pod_blk);
    e.pod_blk = pod_blk.as<uint32_t>();
    if (c->dir[0].n && c->dir[1].n)
      k_first_error_blocks<<<grid1(uint64_t(pb.P) * e.dchunks, 1), 256, 0, st>>>(e);
    HIPCHK(hipMemcpyAsync(first.data(), c->first_blk.p, nb * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  const std::string saved = c->err;
  for (size_t b = 0; b < nb; b++) {
    const ProbeBlock& x = pb.blocks[b];
    if (pb.blk_expand_panic[b]) {
      c->blk_rc[b] = CYC_ERR_PANIC_RUNTIME;
      c->blk_msg[b] = "runtime error: index out of range [0] with length 0";
    } else if (first[b] != ~0ull) {
      const uint32_t np = x.p1 - x.p0, idx = uint32_t(first[b] % 65536);
      const uint64_t rest = first[b] / 65536;
      c->blk_rc[b] = describe_panic(c, x.p0 + uint32_t(rest / np), x.p0 + uint32_t(rest % np), x.cfg, idx);
      c->blk_msg[b] = c->err;
    } else if (!pb.blk_dup_msg[b].empty()) {
      c->blk_rc[b] = CYC_ERR_DUPLICATE_KEY;
      c->blk_msg[b] = pb.blk_dup_msg[b];
    }
  }
  c->err = saved;
  return (int)CYC_OK;
}

// allow_capture = false: never capture a graph for this run (cyc_table_run's planes are new on
// every call, so a captured graph would be re-instantiated each time): graphs = 1 runs as 2.
// src: rows [lo, hi) are a source shard (CYC_ROWS_SOURCE), else target rows.
static int run_pipeline(cyc_ctx* c, hipStream_t st, uint64_t* d_in, uint64_t* d_eg, uint8_t* d_status, int64_t lo,
                        int64_t hi, bool allow_capture = true, bool src = false) {
  Problem& pb = c->pb;
  const uint32_t P = pb.P, K = pb.K, W = pb.W;
  if (lo < 0 || hi > int64_t(P) || lo > hi) return fail(c, CYC_ERR_ARG, "row range out of bounds");
  if (src && (lo % 64 || (hi % 64 && hi != int64_t(P))))
    return fail(c, CYC_ERR_ARG, "source rows: row_lo must be a multiple of 64, row_hi too unless it is the pod count");
  if (c->order_lo != lo || c->order_hi != hi || c->order_src != src) drop_graph(c);  // range plan buffers are re-made
  ensure_range(c, lo, hi, src);
  if (!c->plvt_ready && front_fused_ok(c) && pod_sparse(c)) {
    drop_graph(c);  // a graph captured without the per-pod table would keep the slower gathers
    ensure_plvt(c, st);
  }
  int graphs = c->use_graphs >= 0 ? c->use_graphs : (front_fused_ok(c) ? 2 : 1);
  if (graphs == 1 && !allow_capture) graphs = 2;
  if (graphs == 2 && !pb.may_err) {
    // the graph's DAG, enqueued directly: the caller's stream forks to two internal streams and
    // joins them back before the emit (events), without hipGraphLaunch's per-replay latency
    ensure_cap_streams(c);
    if (c->step_events) HIPCHK(hipEventRecord(c->ev[0], st));
    capture_pipeline(c, st, c->cap_stream2, c->cap_stream3, d_in, d_eg, d_status);
    if (c->step_events) HIPCHK(hipEventRecord(c->ev[3], st));
    c->timed = c->step_events != 0;
    c->timed_graph = true;
  } else if (graphs && !pb.may_err) {
    // The whole pipeline as one hipGraph (captured once per output buffers / row range):
    // removes the host launch cost of ~16 launches per run (dominant on small problems).
    const void* key[6] = {d_in, d_eg, d_status, reinterpret_cast<void*>(lo), reinterpret_cast<void*>(hi),
                          reinterpret_cast<void*>(intptr_t(src))};
    if (!c->graph_exec || memcmp(key, c->graph_key, sizeof(key)) != 0) {
      drop_graph(c);
      ensure_cap_streams(c);
      hipGraph_t g = nullptr;
      HIPCHK(hipStreamBeginCapture(c->cap_stream, hipStreamCaptureModeThreadLocal));
      c->capturing = true;
      try {
        capture_pipeline(c, c->cap_stream, c->cap_stream2, c->cap_stream3, d_in, d_eg, d_status);
      } catch (...) {
        c->capturing = false;
        throw;
      }
      c->capturing = false;
      HIPCHK(hipStreamEndCapture(c->cap_stream, &g));
      c->graph = g;  // destroyed with the exec (drop_graph / reap_graphs)
      HIPCHK(hipGraphInstantiate(&c->graph_exec, g, nullptr, nullptr, 0));
      HIPCHK(hipEventCreateWithFlags(&c->graph_done, EV_SYNC));
      memcpy(c->graph_key, key, sizeof(key));
    }
    if (c->step_events) HIPCHK(hipEventRecord(c->ev[0], st));
    HIPCHK(hipGraphLaunch(c->graph_exec, st));
    HIPCHK(hipEventRecord(c->graph_done, st));  // the exec may be retired once this completes
    if (c->step_events) HIPCHK(hipEventRecord(c->ev[3], st));
    c->timed = c->step_events != 0;
    c->timed_graph = true;
  } else {
    enqueue_pipeline(c, st, d_in, d_eg, d_status);
    c->timed = true;
    c->timed_graph = false;
  }
  c->ran = true;
  HIPCHK(hipEventRecord(c->run_done, st));

  if (!pb.blocks.empty()) return blocks_status(c, st);

  // 8. panic path: the first panicking job in job order, as the reference would hit it.  Configs
  // run in order (one RunProbeForConfig each); within one, the job expansion (may panic on a pod
  // without containers) precedes the evaluation, which precedes the table build (duplicate keys).
  uint32_t eval_cfg = pb.n_cfg, eval_s = 0, eval_d = 0, eval_idx = 0;
  if (pb.may_err) {
    if (P >= (1u << 24) || K > 65536)  // k_first_error's job-order key: (s*P + d)*65536 + idx < 2^64
      throw Panic{CYC_ERR_ARG, "inputs that can panic are limited to 2^24 pods and 65536 job slots"};
    HIPCHK(hipMemsetAsync(c->first_err.p, 0xFF, uint64_t(pb.n_cfg) * 8, st));
    ErrArgs e{};
    e.P = P;
    e.K = K;
    e.W = W;
    e.n_cfg = pb.n_cfg;
    e.row_lo = uint32_t(lo);
    e.row_hi = uint32_t(hi);
    e.src = src ? 1u : 0u;
    e.w0 = c->win_w0;
    e.WA = c->win_wa;
    e.slot_status = c->slot_status.as<uint8_t>();
    e.slot_cfg = c->slot_cfg.as<uint32_t>();
    e.slot_idx = c->slot_idx.as<uint32_t>();
    e.pod_iid = c->dir[0].pod_id.as<uint32_t>();
    e.pod_eid = c->dir[1].pod_id.as<uint32_t>();
    e.class_in = c->dir[0].class_of.as<uint32_t>();
    e.class_eg = c->dir[1].class_of.as<uint32_t>();
    e.err_in = c->dir[0].err.as<uint8_t>();
    e.err_eg = c->dir[1].err.as<uint8_t>();
    e.AE_in = c->dir[0].n ? c->dir[0].AE.as<uint64_t>() : nullptr;
    e.AE_eg = c->dir[1].n ? c->dir[1].AE.as<uint64_t>() : nullptr;
    e.first = c->first_err.as<unsigned long long>();
    if (P && K) k_first_error<<<grid1(uint64_t((P + 255) / 256) * P, 1), 256, 0, st>>>(e);
    std::vector<unsigned long long> first(std::max<uint32_t>(pb.n_cfg, 1), ~0ull);
    HIPCHK(hipMemcpyAsync(first.data(), c->first_err.p, uint64_t(pb.n_cfg) * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    for (uint32_t cc = 0; cc < pb.n_cfg; cc++)
      if (first[cc] != ~0ull) {
        eval_cfg = cc;
        eval_idx = uint32_t(first[cc] % 65536);
        const uint64_t rest = first[cc] / 65536;
        eval_d = uint32_t(rest % P);
        eval_s = uint32_t(rest / P);
        break;
      }
  }
  for (uint32_t cc = 0; cc < pb.n_cfg; cc++) {
    if (pb.expand_panic[cc]) return fail(c, CYC_ERR_PANIC_RUNTIME, "runtime error: index out of range [0] with length 0");
    if (cc == eval_cfg) return describe_panic(c, eval_s, eval_d, eval_cfg, eval_idx);
    if (!pb.dup_key_msg[cc].empty()) return fail(c, CYC_ERR_DUPLICATE_KEY, pb.dup_key_msg[cc]);
  }
  return (int)CYC_OK;
}

// Host-side formatting of the panic message for the identified first panicking job.  The
// device found WHICH job panics; this re-derives the reference's message text for it by
// replaying that single job's evaluation order over the compiled tables (error path only).
int describe_panic(cyc_ctx* c, uint32_t s, uint32_t d, uint32_t cfg, uint32_t idx) {
  Problem& pb = c->pb;
  uint32_t k = 0;
  for (uint32_t kk = 0; kk < pb.K; kk++)
    if (pb.slot_cfg[kk] == cfg && pb.slot_idx[kk] == idx) k = kk;
  std::vector<uint8_t> selres(size_t(pb.S) * pb.L);
  HIPCHK(hipMemcpy(selres.data(), c->selres.p, selres.size(), hipMemcpyDeviceToHost));
  auto sel = [&](uint32_t sid, uint32_t ls) { return selres[size_t(sid) * pb.L + ls]; };
  auto ip_err = [&](const DPeer& pr, uint32_t q, std::string& msg) -> int {
    const DIPBlock& b = pb.ipbs[pr.ipb];
    auto cidr_msg = [&](uint32_t id) {
      return "unable to parse CIDR '" + pb.cidr_str[id] + "': invalid CIDR address: " + pb.cidr_str[id];
    };
    if (!pb.cidrs[b.cidr].valid) {
      msg = cidr_msg(b.cidr);
      return CYC_ERR_PANIC_CIDR;
    }
    if (!pb.pod_ip[q].valid) {
      msg = "unable to parse IP '" + pb.pod_ip_str[q] + "'";
      return CYC_ERR_PANIC_IP;
    }
    for (uint32_t e = 0; e < b.excnt; e++) {
      uint32_t x = pb.ipb_ex[b.exoff + e];
      if (!pb.cidrs[x].valid) {
        msg = cidr_msg(x);
        return CYC_ERR_PANIC_CIDR;
      }
    }
    return 0;
  };
  // direction 0 (ingress): target d, peer s; direction 1 (egress): target s, peer d
  for (int dir = 0; dir < 2; dir++) {
    uint32_t tp = dir == 0 ? d : s, peer = dir == 0 ? s : d;
    uint32_t ns = pb.pod_ns[tp], ls = pb.pod_ls[tp];
    uint32_t lo = pb.tns_lo[dir][ns], hi = pb.tns_hi[dir][ns];
    for (uint32_t t = lo; t < hi; t++)
      if (sel(pb.tgt[dir][t].sel, ls) == 2) return fail(c, CYC_ERR_PANIC_SELECTOR, "invalid operator");
    // copy of the device outcome rows for the peer pod's word
    for (uint32_t t = lo; t < hi; t++) {
      if (sel(pb.tgt[dir][t].sel, ls) != 1) continue;
      const DTarget& tg = pb.tgt[dir][t];
      for (uint32_t j = tg.poff; j < tg.poff + tg.pcnt; j++) {
        const DPeer& pr = pb.peers[j];
        if (pr.kind == 0) break;
        int32_t de = pb.slot_desc[size_t(d) * pb.K + k];
        std::vector<uint8_t> ok(1);
        HIPCHK(hipMemcpy(ok.data(), c->portok.as<uint8_t>() + size_t(pr.port) * std::max<size_t>(pb.descs.size(), 1) + de, 1,
                         hipMemcpyDeviceToHost));
        if (pr.kind == 1) {
          if (ok[0]) break;
          continue;
        }
        uint64_t pm, er;
        const size_t row = pr.kind == 3 && j < c->prow_host.size() ? c->prow_host[j] : j;  // IP peers share their IPBlock's row
        HIPCHK(hipMemcpy(&pm, c->PM.as<uint64_t>() + row * pb.W + peer / 64, 8, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(&er, c->ER.as<uint64_t>() + row * pb.W + peer / 64, 8, hipMemcpyDeviceToHost));
        if ((er >> (peer % 64)) & 1) {
          if (pr.kind == 2) return fail(c, CYC_ERR_PANIC_SELECTOR, "invalid operator");
          std::string msg;
          int code = ip_err(pr, peer, msg);
          return fail(c, code ? code : CYC_ERR_PANIC_CIDR, msg);
        }
        if (((pm >> (peer % 64)) & 1) && ok[0]) break;
      }
    }
  }
  return fail(c, CYC_ERR_PANIC_CIDR, "panic (unresolved message)");
}

static void destroy_events(cyc_ctx* c) {
  for (auto& e : c->ev)
    if (e) {
      (void)hipEventDestroy(e);
      e = nullptr;
    }
}

extern "C" {

const char* cyc_version(void) { return "cyclonus_hip 0.1 (gfx950)"; }

// Diagnostic (env CYC_SEGV_TRACE=1): on SIGSEGV print the native frames as module + offset
// (resolve offline with addr2line -e <module> <offset>), then die with the default action.
static void segv_trace(int sig) {
  void* bt[64];
  const int n = backtrace(bt, 64);
  char line[512];
  for (int i = 0; i < n; i++) {
    Dl_info di{};
    int len;
    if (dladdr(bt[i], &di) && di.dli_fname)
      len = snprintf(line, sizeof line, "cyc-segv #%d %s +0x%lx %s\n", i, di.dli_fname,
                     (unsigned long)((char*)bt[i] - (char*)di.dli_fbase), di.dli_sname ? di.dli_sname : "");
    else
      len = snprintf(line, sizeof line, "cyc-segv #%d %p\n", i, bt[i]);
    if (len > 0) (void)!write(2, line, size_t(len));
  }
  signal(sig, SIG_DFL);
  raise(sig);
}

int cyc_ctx_create(int device_id, cyc_ctx** out) {
  if (!out) return CYC_ERR_ARG;
  static const bool trace = [] {
    const char* e = getenv("CYC_SEGV_TRACE");
    if (e && *e == '1') signal(SIGSEGV, segv_trace);
    return true;
  }();
  (void)trace;
  // Policy compilation / IR export work on a host without a GPU: when the device is not there, the
  // context is created without HIP state and the first call that needs it (cyc_probe_prepare) fails.
  // When it is, the context's stream and events are made here — the first HIP stream of a process
  // costs ~100 ms (queue creation), paid once per context instead of inside the first prepare.
  auto* c = new cyc_ctx();
  c->device = device_id;
  int n_dev = 0;
  if (hipGetDeviceCount(&n_dev) == hipSuccess && device_id >= 0 && device_id < n_dev) {
    DeviceGuard dg(device_id, false);
    int cur = -1;
    bool ok = hipGetDevice(&cur) == hipSuccess && cur == device_id;
    ok = ok && hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess;
    for (auto& e : c->ev) ok = ok && hipEventCreateWithFlags(&e, EV_TIMING) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&c->run_done, EV_SYNC) == hipSuccess;
    if (!ok) {  // (left to the first prepare, which reports the error)
      for (auto& e : c->ev)
        if (e) (void)hipEventDestroy(e), e = nullptr;
      if (c->run_done) (void)hipEventDestroy(c->run_done), c->run_done = nullptr;
      if (c->stream) (void)hipStreamDestroy(c->stream), c->stream = nullptr;
    }
  } else {
    (void)hipGetLastError();  // (no device: nothing to initialise)
  }
  *out = c;
  return (int)CYC_OK;
}

void cyc_ctx_destroy(cyc_ctx* c) {
  if (!c) return;
  if (c->stream) {
    DeviceGuard dg(c->device, false);
    drop_graph(c);
    reap_graphs(c, true);  // waits for each retired exec's last launch only
    destroy_events(c);
    if (c->cap_stream) (void)hipStreamDestroy(c->cap_stream);
    if (c->cap_stream2) (void)hipStreamDestroy(c->cap_stream2);
    if (c->cap_stream3) (void)hipStreamDestroy(c->cap_stream3);
    if (c->sel_ev) (void)hipEventDestroy(c->sel_ev);
    if (c->ports_ev) (void)hipEventDestroy(c->ports_ev);
    if (c->fork_ev) (void)hipEventDestroy(c->fork_ev);
    if (c->join_ev) (void)hipEventDestroy(c->join_ev);
    if (c->run_done) (void)hipEventDestroy(c->run_done);
    (void)hipStreamDestroy(c->stream);
  }
  delete c;
}

const char* cyc_last_error(const cyc_ctx* c) { return c ? c->err.c_str() : "null context"; }

int cyc_policy_build_json(cyc_ctx* c, int simplify, const char* js, size_t len) {
  if (!c || !js) return CYC_ERR_ARG;
  return guarded(c, [&] {
    json::Node n = json::parse(js, len);
    c->policy = build_network_policies(n, simplify != 0);
    c->have_policy = true;
    c->prepared = false;
    return (int)CYC_OK;
  });
}

int cyc_policy_load_ir_json(cyc_ctx* c, const char* js, size_t len) {
  if (!c || !js) return CYC_ERR_ARG;
  return guarded(c, [&] {
    c->policy = load_policy_ir(json::parse(js, len));
    c->have_policy = true;
    c->prepared = false;
    return (int)CYC_OK;
  });
}

// The JSON dumps: bytes needed (+1), the text copied when buf holds it all; -(cyc_status) on failure
// (nothing loaded, or the dump itself failed, e.g. out of memory) with cyc_last_error set.
static int64_t json_out(cyc_ctx* c, bool have, const char* what, const std::function<std::string()>& dump, char* buf,
                        size_t cap) {
  if (!c) return -int64_t(CYC_ERR_ARG);
  if (!have) return -int64_t(fail(c, CYC_ERR_ARG, std::string("no ") + what + " loaded"));
  int64_t need = 0;
  const int rc = guarded(c, [&] {
    const std::string s = dump();
    if (buf && cap > s.size()) {
      memcpy(buf, s.data(), s.size());
      buf[s.size()] = 0;
    }
    need = int64_t(s.size()) + 1;
    return (int)CYC_OK;
  });
  return rc == CYC_OK ? need : -int64_t(rc);
}

int64_t cyc_policy_ir_json(cyc_ctx* c, char* buf, size_t cap) {
  return json_out(c, c && c->have_policy, "policy", [&] { return dump_policy_ir(c->policy); }, buf, cap);
}

int cyc_resources_load_json(cyc_ctx* c, const char* js, size_t len) {
  if (!c || !js) return CYC_ERR_ARG;
  return guarded(c, [&] {
    c->res = load_resources(json::parse(js, len));
    c->have_res = true;
    c->prepared = false;
    return (int)CYC_OK;
  });
}

int64_t cyc_resources_json(cyc_ctx* c, char* buf, size_t cap) {
  return json_out(c, c && c->have_res, "resources", [&] { return dump_resources(c->res); }, buf, cap);
}

int cyc_resources_load(cyc_ctx* c, const cyc_resource_tables* t) {
  if (!c || !t) return CYC_ERR_ARG;
  return guarded(c, [&] {
    c->res = load_resources_tables(*t);
    c->have_res = true;
    c->prepared = false;
    return (int)CYC_OK;
  });
}

int cyc_policy_load(cyc_ctx* c, const cyc_policy_tables* t) {
  if (!c || !t) return CYC_ERR_ARG;
  return guarded(c, [&] {
    c->policy = load_policy_tables(*t);
    c->have_policy = true;
    c->prepared = false;
    return (int)CYC_OK;
  });
}

// `probes` decodes the probe configs (JSON or flat) inside the guarded call
static int probe_prepare(cyc_ctx* c, const std::function<std::vector<ProbeConfig>()>& probes_of, cyc_probe_shape* shape,
                         const std::vector<ProbeBlock>* blocks) {
  if (!c) return CYC_ERR_ARG;
  if (!c->have_policy || !c->have_res) return fail(c, CYC_ERR_ARG, "load a policy and resources first");
  return guarded(c, [&] {
    PhaseClock clk("prepare");
    DeviceGuard dg(c->device);
    clk.lap("device");
    if (!c->stream) {
      HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
      for (auto& e : c->ev) HIPCHK(hipEventCreateWithFlags(&e, EV_TIMING));
      HIPCHK(hipEventCreateWithFlags(&c->run_done, EV_SYNC));
    }
    clk.lap("stream");
    const std::vector<ProbeConfig> probes = probes_of();
    c->prepared = false;
    clk.lap("probe configs");
    c->pb = build_problem(c->policy, c->res, probes, blocks);
    clk.lap("build_problem");
    drop_graph(c);
    build_identities(c);
    clk.lap("identities");
    prepare_device(c);
    clk.lap("device tables");
    c->prepared = true;
    if (shape) {
      shape->pods = c->pb.P;
      shape->slots = c->pb.K;
      shape->words = c->pb.W;
      shape->configs = c->pb.n_cfg;
      shape->targets_in = int64_t(c->pb.tgt[0].size());
      shape->targets_eg = int64_t(c->pb.tgt[1].size());
      shape->peers = int64_t(c->pb.peers.size());
      shape->classes_in = c->dir[0].n;
      shape->classes_eg = c->dir[1].n;
      shape->may_panic = c->pb.may_err ? 1 : 0;
      shape->selectors = c->pb.S;
      shape->label_sets = c->pb.L;
      shape->pod_peers = int64_t(c->plan.pod_peers.size());
      shape->ip_peers = int64_t(c->plan.ip_peers.size());
      shape->descriptors = int64_t(c->pb.descs.size());
      shape->max_word_runs = c->plan.max_runs;
    }
    return (int)CYC_OK;
  });
}

int cyc_probe_prepare(cyc_ctx* c, const char* js, size_t len, cyc_probe_shape* shape) {
  if (!c || !js) return CYC_ERR_ARG;
  return probe_prepare(c, [&] { return load_probes(json::parse(js, len)); }, shape, nullptr);
}

int cyc_probe_prepare_configs(cyc_ctx* c, const cyc_probe_config* cfgs, int64_t n, cyc_probe_shape* shape) {
  if (!c || (n && !cfgs) || n < 0) return CYC_ERR_ARG;
  return probe_prepare(c, [&] { return load_probe_configs(cfgs, n); }, shape, nullptr);
}

int cyc_probe_prepare_blocks(cyc_ctx* c, const char* js, size_t len, const int64_t* block_end, const int32_t* block_config,
                             int64_t n_blocks, cyc_probe_shape* shape) {
  if (!c || !js || n_blocks < 1 || !block_end || !block_config) return CYC_ERR_ARG;
  std::vector<ProbeBlock> bl(static_cast<size_t>(n_blocks));
  int64_t at = 0;
  for (int64_t b = 0; b < n_blocks; b++) {
    if (block_end[b] < at || block_end[b] > int64_t(UINT32_MAX) || block_config[b] < 0)
      return fail(c, CYC_ERR_ARG, "blocks must be consecutive pod ranges with a probe config each");
    bl[size_t(b)] = ProbeBlock{uint32_t(at), uint32_t(block_end[b]), uint32_t(block_config[b])};
    at = block_end[b];
  }
  if (!js) return CYC_ERR_ARG;
  return probe_prepare(c, [&] { return load_probes(json::parse(js, len)); }, shape, &bl);
}

int cyc_blocks_layout(cyc_ctx* c, int64_t* out, int64_t n) {
  if (!c || !out) return CYC_ERR_ARG;
  if (!c->prepared || c->pb.blocks.empty()) return fail(c, CYC_ERR_ARG, "cyc_probe_prepare_blocks first");
  const size_t nb = c->pb.blocks.size();
  if (n < int64_t(nb + 1) * 2) return fail(c, CYC_ERR_ARG, "layout buffer needs 2 * (blocks + 1) entries");
  for (size_t i = 0; i < 2 * (nb + 1); i++) out[i] = int64_t(c->blk_off_h[i]);
  return (int)CYC_OK;
}

int cyc_probe_run_blocks(cyc_ctx* c, void* stream, uint64_t* d_in, uint64_t* d_eg, uint8_t* d_status, int32_t* block_status) {
  if (!c) return CYC_ERR_ARG;
  if (!c->prepared || c->pb.blocks.empty()) return fail(c, CYC_ERR_ARG, "cyc_probe_prepare_blocks first");
  const uint64_t words = c->blk_off_h[2 * c->pb.blocks.size()];
  if ((words && (!d_in || !d_eg)) || !d_status) return fail(c, CYC_ERR_ARG, "null output slab");
  return guarded(c, [&]() -> int {
    DeviceGuard dg(c->device);
    hipStream_t st = static_cast<hipStream_t>(stream);
    const int rc = run_pipeline(c, st, d_in, d_eg, d_status, 0, c->pb.P, false, false);
    if (rc == CYC_OK && block_status)
      for (size_t b = 0; b < c->blk_rc.size(); b++) block_status[b] = c->blk_rc[b];
    return rc;
  });
}

const char* cyc_block_error(const cyc_ctx* c, int64_t b) {
  if (!c || b < 0 || size_t(b) >= c->blk_msg.size()) return "";
  return c->blk_msg[size_t(b)].c_str();
}

int cyc_probe_run_rows(cyc_ctx* c, void* stream, uint64_t* d_in, uint64_t* d_eg, uint8_t* d_status, int part, int64_t lo,
                       int64_t hi) {
  if (!c) return CYC_ERR_ARG;
  if (!c->prepared) return fail(c, CYC_ERR_ARG, "cyc_probe_prepare first");
  if ((!d_in || !d_eg) && hi > lo) return fail(c, CYC_ERR_ARG, "null output plane");
  if (part != CYC_ROWS_TARGET && part != CYC_ROWS_SOURCE) return fail(c, CYC_ERR_ARG, "unknown partition");
  if (!c->pb.blocks.empty()) return fail(c, CYC_ERR_ARG, "context prepared for blocks: use cyc_probe_run_blocks");
  return guarded(c, [&] {
    DeviceGuard dg(c->device);
    hipStream_t st = static_cast<hipStream_t>(stream);  // NULL = the HIP default (null) stream
    return run_pipeline(c, st, d_in, d_eg, d_status, lo, hi, true, part == CYC_ROWS_SOURCE);
  });
}

int cyc_probe_run(cyc_ctx* c, void* stream, uint64_t* d_in, uint64_t* d_eg, uint8_t* d_status, int64_t lo, int64_t hi) {
  return cyc_probe_run_rows(c, stream, d_in, d_eg, d_status, CYC_ROWS_TARGET, lo, hi);
}

int cyc_probe_run_host_rows(cyc_ctx* c, uint64_t* h_in, uint64_t* h_eg, uint8_t* h_status, int part, int64_t lo, int64_t hi) {
  if (!c) return CYC_ERR_ARG;
  if (!c->prepared) return fail(c, CYC_ERR_ARG, "cyc_probe_prepare first");
  return guarded(c, [&]() -> int {
    DeviceGuard dg(c->device);
    int64_t v[5];
    std::string why;
    if (!rows_layout(c, part, lo, hi, v, why)) return fail(c, CYC_ERR_ARG, why);
    const uint64_t words_in = uint64_t(v[0]) * c->pb.K * v[1], words_eg = uint64_t(v[2]) * c->pb.K * v[3];
    DevBuf din, deg, dst;
    din.alloc(std::max<uint64_t>(words_in * 8, 16));
    deg.alloc(std::max<uint64_t>(words_eg * 8, 16));
    dst.alloc(std::max<uint64_t>(uint64_t(c->pb.P) * c->pb.K, 16));
    int rc = run_pipeline(c, c->stream, din.as<uint64_t>(), deg.as<uint64_t>(), dst.as<uint8_t>(), lo, hi, true,
                          part == CYC_ROWS_SOURCE);
    HIPCHK(hipStreamSynchronize(c->stream));
    if (rc != CYC_OK) return rc;
    if (h_in && words_in) HIPCHK(hipMemcpy(h_in, din.p, words_in * 8, hipMemcpyDeviceToHost));
    if (h_eg && words_eg) HIPCHK(hipMemcpy(h_eg, deg.p, words_eg * 8, hipMemcpyDeviceToHost));
    if (h_status && uint64_t(c->pb.P) * c->pb.K)
      HIPCHK(hipMemcpy(h_status, dst.p, uint64_t(c->pb.P) * c->pb.K, hipMemcpyDeviceToHost));
    return (int)CYC_OK;
  });
}

int cyc_probe_run_host(cyc_ctx* c, uint64_t* h_in, uint64_t* h_eg, uint8_t* h_status, int64_t lo, int64_t hi) {
  return cyc_probe_run_host_rows(c, h_in, h_eg, h_status, CYC_ROWS_TARGET, lo, hi);
}

// ---------------------------------------------------------------- device-resident tables
struct cyc_table {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  uint32_t P = 0, K = 0, W = 0;
  int64_t row_lo = 0, row_hi = 0;
  int partition = CYC_ROWS_TARGET;  // CYC_ROWS_SOURCE: rows are sources; ingress rows cover words [w0, w0 + wa)
  uint32_t w0 = 0, wa = 0;
  const uint64_t *in = nullptr, *eg = nullptr;
  const uint8_t* status = nullptr;
  DevBuf own_in, own_eg, own_st;  // cyc_table_run: the table owns its planes
};

// Plane shapes of rows [lo, hi) under a partition: ingress rows, words per ingress row slot, egress
// rows, words per egress row slot, first word of the ingress window.
static bool rows_layout(const cyc_ctx* c, int part, int64_t lo, int64_t hi, int64_t v[5], std::string& why) {
  const int64_t P = c->pb.P, W = c->pb.W;
  // a context prepared for batched blocks has per-block slabs, not row planes (cyc_probe_run_blocks)
  if (!c->pb.blocks.empty()) return why = "context prepared for blocks: use cyc_probe_run_blocks", false;
  if (part != CYC_ROWS_TARGET && part != CYC_ROWS_SOURCE) return why = "unknown partition", false;
  if (lo < 0 || hi > P || lo > hi) return why = "row range out of bounds", false;
  if (part == CYC_ROWS_SOURCE && (lo % 64 || (hi % 64 && hi != P)))
    return why = "source rows: row_lo must be a multiple of 64, row_hi too unless it is the pod count", false;
  const bool src = part == CYC_ROWS_SOURCE;
  const int64_t wa = src ? (hi > lo ? (hi + 63) / 64 - lo / 64 : 0) : W;
  v[0] = src ? P : hi - lo;
  v[1] = wa;
  v[2] = hi - lo;
  v[3] = W;
  v[4] = src ? lo / 64 : 0;
  return true;
}

static int table_new(cyc_ctx* c, int part, int64_t lo, int64_t hi, cyc_table** out) {
  int64_t v[5];
  std::string why;
  if (!rows_layout(c, part, lo, hi, v, why)) return fail(c, CYC_ERR_ARG, why);
  auto* t = new cyc_table();
  t->device = c->device;
  t->P = c->pb.P;
  t->K = c->pb.K;
  t->W = c->pb.W;
  t->row_lo = lo;
  t->row_hi = hi;
  t->partition = part;
  t->w0 = uint32_t(v[4]);
  t->wa = uint32_t(v[1]);
  *out = t;
  return (int)CYC_OK;
}

int cyc_table_run_rows(cyc_ctx* c, int part, int64_t lo, int64_t hi, cyc_table** out) {
  if (!c || !out) return CYC_ERR_ARG;
  *out = nullptr;
  if (!c->prepared) return fail(c, CYC_ERR_ARG, "cyc_probe_prepare first");
  return guarded(c, [&]() -> int {
    DeviceGuard dg(c->device);
    cyc_table* t = nullptr;
    int rc = table_new(c, part, lo, hi, &t);
    if (rc != CYC_OK) return rc;
    std::unique_ptr<cyc_table> hold(t);
    const uint64_t words_in = uint64_t(part == CYC_ROWS_SOURCE ? c->pb.P : hi - lo) * c->pb.K * t->wa;
    const uint64_t words_eg = uint64_t(hi - lo) * c->pb.K * c->pb.W;
    t->own_in.alloc(std::max<uint64_t>(words_in * 8, 16));
    t->own_eg.alloc(std::max<uint64_t>(words_eg * 8, 16));
    t->own_st.alloc(std::max<uint64_t>(uint64_t(c->pb.P) * c->pb.K, 16));
    t->in = t->own_in.as<uint64_t>();
    t->eg = t->own_eg.as<uint64_t>();
    t->status = t->own_st.as<uint8_t>();
    rc = run_pipeline(c, c->stream, t->own_in.as<uint64_t>(), t->own_eg.as<uint64_t>(), t->own_st.as<uint8_t>(), lo, hi,
                      false, part == CYC_ROWS_SOURCE);
    HIPCHK(hipStreamSynchronize(c->stream));
    if (rc != CYC_OK) return rc;
    *out = hold.release();
    return (int)CYC_OK;
  });
}

int cyc_table_run(cyc_ctx* c, int64_t lo, int64_t hi, cyc_table** out) { return cyc_table_run_rows(c, CYC_ROWS_TARGET, lo, hi, out); }

int cyc_table_wrap_rows(cyc_ctx* c, const uint64_t* d_in, const uint64_t* d_eg, const uint8_t* d_status, int part, int64_t lo,
                        int64_t hi, cyc_table** out) {
  if (!c || !out) return CYC_ERR_ARG;
  *out = nullptr;
  if (!c->prepared) return fail(c, CYC_ERR_ARG, "cyc_probe_prepare first");
  if (!d_status || ((!d_in || !d_eg) && hi > lo)) return fail(c, CYC_ERR_ARG, "null plane");
  cyc_table* t = nullptr;
  int rc = table_new(c, part, lo, hi, &t);
  if (rc != CYC_OK) return rc;
  t->in = d_in;
  t->eg = d_eg;
  t->status = d_status;
  *out = t;
  return (int)CYC_OK;
}

int cyc_table_wrap(cyc_ctx* c, const uint64_t* d_in, const uint64_t* d_eg, const uint8_t* d_status, int64_t lo, int64_t hi,
                   cyc_table** out) {
  return cyc_table_wrap_rows(c, d_in, d_eg, d_status, CYC_ROWS_TARGET, lo, hi, out);
}

int cyc_rows_layout(cyc_ctx* c, int part, int64_t lo, int64_t hi, int64_t* out, int n) {
  if (!c || !out) return CYC_ERR_ARG;
  if (!c->prepared) return fail(c, CYC_ERR_ARG, "cyc_probe_prepare first");
  int64_t v[5];
  std::string why;
  if (!rows_layout(c, part, lo, hi, v, why)) return fail(c, CYC_ERR_ARG, why);
  for (int i = 0; i < n && i < 5; i++) out[i] = v[i];
  return (int)CYC_OK;
}

const char* cyc_table_error(const cyc_table* t) { return t ? t->err.c_str() : "null table"; }

int cyc_table_shape(const cyc_table* t, int64_t* out, int n) {
  if (!t || !out) return CYC_ERR_ARG;
  const int64_t v[8] = {t->P, t->K, t->W, t->row_lo, t->row_hi, t->partition, t->w0, t->wa};
  for (int i = 0; i < n && i < 8; i++) out[i] = v[i];
  return (int)CYC_OK;
}

int cyc_table_cells(cyc_table* t, int64_t s_lo, int64_t s_hi, int64_t d_lo, int64_t d_hi, int64_t k_lo, int64_t k_hi,
                    uint8_t* ingress, uint8_t* egress, uint8_t* combined) {
  if (!t) return CYC_ERR_ARG;
  auto bad = [&](const char* m) {
    t->err = m;
    return (int)CYC_ERR_ARG;
  };
  if (s_lo < 0 || s_hi > int64_t(t->P) || s_lo > s_hi || d_lo < 0 || d_hi > int64_t(t->P) || d_lo > d_hi || k_lo < 0 ||
      k_hi > int64_t(t->K) || k_lo > k_hi)
    return bad("cell range out of bounds");
  // ingress rows are keyed by destination, egress rows by source (include/cyclonus_hip.h); a
  // source-row table holds both directions of its sources' cells
  const bool src = t->partition == CYC_ROWS_SOURCE;
  const bool need_d = !src && (ingress || combined), need_s = egress || combined || (src && ingress);
  if (s_hi > s_lo && d_hi > d_lo && k_hi > k_lo) {
    if (need_d && (d_lo < t->row_lo || d_hi > t->row_hi)) return bad("ingress cells need destinations inside the table's rows");
    if (need_s && (s_lo < t->row_lo || s_hi > t->row_hi))
      return bad(src ? "cells of a source-row table need sources inside its rows" : "egress cells need sources inside the table's rows");
  }
  const uint64_t n = uint64_t(s_hi - s_lo) * uint64_t(d_hi - d_lo) * uint64_t(k_hi - k_lo);
  if (!n) return (int)CYC_OK;
  try {
    DeviceGuard dg(t->device);
    if (!t->stream) HIPCHK(hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking));
    DevBuf o[3];
    uint8_t* host[3] = {ingress, egress, combined};
    for (int x = 0; x < 3; x++)
      if (host[x]) o[x].alloc(n);
    CellArgs a{};
    a.K = t->K;
    a.W = t->W;
    a.row_lo = uint32_t(t->row_lo);
    a.row_hi = uint32_t(t->row_hi);
    a.src = src ? 1u : 0u;
    a.w0 = t->w0;
    a.WA = t->wa;
    a.in = t->in;
    a.eg = t->eg;
    a.status = t->status;
    a.s_lo = uint32_t(s_lo);
    a.d_lo = uint32_t(d_lo);
    a.k_lo = uint32_t(k_lo);
    a.nd = uint32_t(d_hi - d_lo);
    a.nk = uint32_t(k_hi - k_lo);
    a.n = n;
    a.o_in = o[0].as<uint8_t>();
    a.o_eg = o[1].as<uint8_t>();
    a.o_comb = o[2].as<uint8_t>();
    k_table_cells<<<grid1(n, 256), 256, 0, t->stream>>>(a);
    HIPCHK(hipGetLastError());
    for (int x = 0; x < 3; x++)
      if (host[x]) HIPCHK(hipMemcpyAsync(host[x], o[x].p, n, hipMemcpyDeviceToHost, t->stream));
    HIPCHK(hipStreamSynchronize(t->stream));
  } catch (HipErr& h) {
    t->err = h.msg;
    return (int)CYC_ERR_HIP;
  } catch (std::bad_alloc&) {
    t->err = "host allocation failed";
    return (int)CYC_ERR_OOM;
  }
  return (int)CYC_OK;
}

void cyc_table_destroy(cyc_table* t) {
  if (!t) return;
  DeviceGuard dg(t->device, false);
  if (t->stream) {
    (void)hipStreamSynchronize(t->stream);
    (void)hipStreamDestroy(t->stream);
  }
  delete t;  // owned planes are freed by their DevBufs
}

int cyc_last_timings(cyc_ctx* c, double* ms, int n) {
  if (!c || !ms) return CYC_ERR_ARG;
  if (!c->timed) return fail(c, CYC_ERR_ARG, c->ran ? "the last run recorded no timing events (step_events = 0)" : "no run yet");
  return guarded(c, [&] {
    DeviceGuard dg(c->device);
    HIPCHK(hipEventSynchronize(c->ev[3]));
    float a = 0, b = 0, r = 0;
    HIPCHK(hipEventElapsedTime(&a, c->ev[0], c->ev[3]));
    if (!c->timed_graph) {
      HIPCHK(hipEventElapsedTime(&b, c->ev[2], c->ev[3]));
      HIPCHK(hipEventElapsedTime(&r, c->ev[1], c->ev[2]));
    }
    double v[3] = {a, c->timed_graph ? -1.0 : b, c->timed_graph ? -1.0 : r};
    for (int i = 0; i < n && i < 3; i++) ms[i] = v[i];
    return (int)CYC_OK;
  });
}

int cyc_last_classes(cyc_ctx* c, int64_t* out, int n) {
  if (!c || !out || n < 2) return CYC_ERR_ARG;
  if (!c->ran) return fail(c, CYC_ERR_ARG, "no run yet");
  return guarded(c, [&]() -> int {
    DeviceGuard dg(c->device);
    HIPCHK(hipEventSynchronize(c->run_done));  // the last run's stream, not the whole device
    for (int d = 0; d < 2; d++) {
      uint32_t v = 0xFFFFFFFFu;
      if (c->dir[d].n && c->n_act[d]) HIPCHK(hipMemcpy(&v, c->dir[d].rep_cnt(), 4, hipMemcpyDeviceToHost));
      out[d] = int64_t(uint32_t(v + 1u));
    }
    return (int)CYC_OK;
  });
}

int cyc_last_emit(cyc_ctx* c, char* name, size_t cap, int64_t* launches) {
  if (!c) return CYC_ERR_ARG;
  if (!c->ran) return fail(c, CYC_ERR_ARG, "no run yet");
  if (name && cap) {
    const size_t n = std::min(cap - 1, c->emit_kernel.size());
    std::memcpy(name, c->emit_kernel.data(), n);
    name[n] = 0;
  }
  if (launches) *launches = c->emit_launches;
  return CYC_OK;
}

int cyc_set_option(cyc_ctx* c, const char* name, int64_t value) {
  if (!c || !name) return CYC_ERR_ARG;
  std::unique_ptr<DeviceGuard> dg;
  if (c->stream) dg.reset(new DeviceGuard(c->device, false));  // drop_graph may destroy this context's execs
  const std::string n(name);
  auto range = [&](int64_t lo, int64_t hi) {
    if (value < lo || value > hi) throw Panic{CYC_ERR_ARG, n + " must be in " + std::to_string(lo) + ".." + std::to_string(hi)};
  };
  return guarded(c, [&]() -> int {
    if (n == "graphs") range(-1, 2), c->use_graphs = int(value);
    else if (n == "front_fused") range(0, 1), c->front_fused = int(value);
    else if (n == "pod_words") range(-1, 1), c->pod_words = int(value);
    else if (n == "pod_rows") range(-1, 1), c->pod_rows = int(value);
    else if (n == "ip_range") {
      range(-1, 1);
      c->ip_range = int(value);
      c->order_lo = c->order_hi = -1;  // the next run re-plans which IP rows are range-built
    }
    else if (n == "member_wave") range(-1, 1), c->member_wave = int(value);
    else if (n == "class_rpb") range(0, 64), c->class_rpb_opt = value;
    else if (n == "pl_wave") range(0, 1), c->pl_wave = int(value);
    else if (n == "sel_lazy") range(-1, 1), c->sel_lazy = int(value);
    else if (n == "pr_group") range(-1, 64), c->pr_group = int(value == 0 ? -1 : value);
    else if (n == "class_inplace") range(-1, 1), c->class_inplace = int(value);
    else if (n == "step_events") range(0, 1), c->step_events = int(value);
    else if (n == "emit_interleave") range(-1, 1), c->emit_interleave = int(value);
    else if (n == "emit_split") range(1, 8), c->emit_split = int(value);
    else if (n == "emit_buf") range(0, 2), c->emit_buf = int(value);
    else if (n == "ip_items") {
      range(-1, 1);
      c->ip_items_opt = int(value);
      c->order_lo = c->order_hi = -1;  // the next run re-plans the items
    }
    else if (n == "plvt_max_mb") {
      range(0, 1 << 20);
      c->plvt_max_mb = value;
      c->plvt_ready = false;  // rebuilt (or not) by the next run
      c->plvt.alloc(0);
    }
    else return fail(c, CYC_ERR_ARG, "unknown option " + n);
    drop_graph(c);
    return (int)CYC_OK;
  });
}

int cyc_get_option(cyc_ctx* c, const char* name, int64_t* value) {
  if (!c || !name || !value) return CYC_ERR_ARG;
  const std::string n(name);
  if (n == "graphs") *value = c->use_graphs;
  else if (n == "front_fused") *value = c->front_fused;
  else if (n == "pod_rows") *value = c->pod_rows;
  else if (n == "ip_range") *value = c->ip_range;
  else if (n == "member_wave") *value = c->member_wave;
  else if (n == "class_rpb") *value = c->class_rpb_opt;
  else if (n == "pl_wave") *value = c->pl_wave;
  else if (n == "sel_lazy") *value = c->sel_lazy;
  else if (n == "pr_group") *value = c->pr_group;
  else if (n == "class_inplace") *value = c->class_inplace;
  else if (n == "class_inplace_active") {
    if (!c->prepared || c->order_lo < 0) return fail(c, CYC_ERR_ARG, "class_inplace_active: run a probe first");
    *value = inplace_ok(c, reinterpret_cast<const uint64_t*>(16), reinterpret_cast<const uint64_t*>(16)) ? 1 : 0;
  }
  else if (n == "step_events") *value = c->step_events;
  else if (n == "emit_interleave") *value = c->emit_interleave;
  else if (n == "emit_split") *value = c->emit_split;
  else if (n == "ip_items") *value = c->ip_items_opt;
  else if (n == "emit_buf") *value = c->emit_buf;
  else if (n == "plvt_max_mb") *value = c->plvt_max_mb;
  else if (n == "plvt_active") *value = c->plvt_ready ? 1 : 0;
  else if (n == "pl_wave_active") {
    if (!c->prepared) return fail(c, CYC_ERR_ARG, "pl_wave_active: call cyc_probe_prepare first");
    *value = !ido_mode(c) && pl_wave_ok(c) ? 1 : 0;
  } else if (n == "launch") *value = c->use_graphs >= 0 ? c->use_graphs : (front_fused_ok(c) ? 2 : 1);  // in effect
  else if (n == "front_fused_active") *value = front_fused_ok(c) ? 1 : 0;
  else if (n == "pod_words") {
    if (!c->prepared) return fail(c, CYC_ERR_ARG, "pod_words: call cyc_probe_prepare first");
    *value = ido_mode(c) ? 1 : 0;
  } else return fail(c, CYC_ERR_ARG, std::string("unknown option ") + name);
  return (int)CYC_OK;
}

// Shared single-cell runner (k_query).  tlist (optional): per (traffic, direction) the matching
// targets in primary-key order, t for an allowing target and -t-1 for a denying one.
static int run_query(cyc_ctx* c, const std::vector<QueryTraffic>& ts, uint8_t* out,
                     std::vector<std::vector<int64_t>>* tlist, bool members_only = false) {
  DeviceGuard dg(c->device);
  std::vector<uint32_t> ext, tdesc;
  Problem q = build_query_problem(c->policy, ts, ext, tdesc);
  DevBuf ls_off, ls_key, ls_val, sel_off, reqs, req_vals, pod_ns, pod_ls, pod_nsls, pod_ip, cidrs, ipbs, ipb_ex, pms, pents,
      peers, descs, dext, dtdesc, tgt0, tgt1, lo0, lo1, hi0, hi1, selres, portok, res, pan, pid;
  upload(ls_off, q.ls_off);
  upload(ls_key, q.ls_key);
  upload(ls_val, q.ls_val);
  upload(sel_off, q.sel_off);
  upload(reqs, q.reqs);
  upload(req_vals, q.req_vals);
  upload(pod_ns, q.pod_ns);
  upload(pod_ls, q.pod_ls);
  upload(pod_nsls, q.pod_nsls);
  upload(pod_ip, q.pod_ip);
  upload(cidrs, q.cidrs);
  upload(ipbs, q.ipbs);
  upload(ipb_ex, q.ipb_ex);
  upload(pms, q.pms);
  upload(pents, q.pents);
  upload(peers, q.peers);
  upload(descs, q.descs);
  upload(dext, ext);
  upload(dtdesc, tdesc);
  upload(tgt0, q.tgt[0]);
  upload(tgt1, q.tgt[1]);
  upload(lo0, q.tns_lo[0]);
  upload(lo1, q.tns_lo[1]);
  upload(hi0, q.tns_hi[0]);
  upload(hi1, q.tns_hi[1]);
  const uint32_t D = uint32_t(std::max<size_t>(q.descs.size(), 1)), M = uint32_t(q.pms.size());
  selres.alloc(std::max<uint64_t>(uint64_t(q.S) * q.L, 16));
  portok.alloc(std::max<uint64_t>(uint64_t(M) * D, 16));
  res.alloc(std::max<size_t>(ts.size(), 16));
  pan.alloc(std::max<size_t>(ts.size() * 4, 16));
  pid.alloc(std::max<size_t>(ts.size() * 4, 16));
  hipStream_t st = nullptr;
  if (uint64_t(q.S) * q.L)
    k_selectors<<<grid1(uint64_t(q.S) * q.L, 256), 256, 0, st>>>(q.S, q.L, sel_off.as<uint32_t>(), reqs.as<DReq>(),
                                                                  req_vals.as<uint32_t>(), ls_off.as<uint32_t>(),
                                                                  ls_key.as<uint32_t>(), ls_val.as<uint32_t>(),
                                                                  selres.as<uint8_t>());
  if (M) k_portok<<<grid1(uint64_t(M) * D, 256), 256, 0, st>>>(M, D, pms.as<DPortM>(), pents.as<DPortEntry>(), descs.as<DDesc>(),
                                                              portok.as<uint8_t>());
  QueryArgs qa{};
  qa.n = uint32_t(ts.size());
  qa.L = q.L;
  qa.D = D;
  qa.pod_ns = pod_ns.as<uint32_t>();
  qa.pod_ls = pod_ls.as<uint32_t>();
  qa.pod_nsls = pod_nsls.as<uint32_t>();
  qa.ext = dext.as<uint32_t>();
  qa.tdesc = dtdesc.as<uint32_t>();
  qa.pod_ip = pod_ip.as<DIP>();
  qa.selres = selres.as<uint8_t>();
  qa.portok = portok.as<uint8_t>();
  qa.tgt[0] = tgt0.as<DTarget>();
  qa.tgt[1] = tgt1.as<DTarget>();
  qa.tns_lo[0] = lo0.as<uint32_t>();
  qa.tns_lo[1] = lo1.as<uint32_t>();
  qa.tns_hi[0] = hi0.as<uint32_t>();
  qa.tns_hi[1] = hi1.as<uint32_t>();
  qa.peers = peers.as<DPeer>();
  qa.ipbs = ipbs.as<DIPBlock>();
  qa.cidrs = cidrs.as<DCidr>();
  qa.ipb_ex = ipb_ex.as<uint32_t>();
  qa.res = res.as<uint8_t>();
  qa.pan = pan.as<uint32_t>();
  qa.pid = pid.as<uint32_t>();
  // per (traffic, direction): one flag per target of the end's namespace
  std::vector<uint64_t> hoff;
  DevBuf doff, dfl;
  uint64_t nfl = 0;
  if (tlist) {
    for (size_t i = 0; i < ts.size(); i++)
      for (int d = 0; d < 2; d++) {
        uint32_t T = uint32_t(d == 0 ? 2 * i + 1 : 2 * i);  // ingress target = dst, egress = src
        uint32_t ns = q.pod_ns[T];
        hoff.push_back(nfl);
        nfl += q.tns_hi[d][ns] - q.tns_lo[d][ns];
      }
    upload(doff, hoff);
    dfl.alloc(std::max<uint64_t>(nfl, 16));
    HIPCHK(hipMemsetAsync(dfl.p, 0, std::max<uint64_t>(nfl, 16), st));
    qa.tflags = dfl.as<uint8_t>();
    qa.toff = doff.as<uint64_t>();
  }
  qa.members_only = members_only ? 1u : 0u;
  k_query<<<grid1(ts.size(), 128), 128, 0, st>>>(qa);
  std::vector<uint8_t> hres(ts.size());
  std::vector<uint32_t> hpan(ts.size()), hpid(ts.size());
  HIPCHK(hipMemcpy(hres.data(), res.p, ts.size(), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(hpan.data(), pan.p, ts.size() * 4, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(hpid.data(), pid.p, ts.size() * 4, hipMemcpyDeviceToHost));
  for (size_t i = 0; i < ts.size(); i++) {
    if (hpan[i]) {  // analyze.go:209-225 prints the earlier traffics, then the reference panics
      if (hpan[i] == QP_SELECTOR) return fail(c, CYC_ERR_PANIC_SELECTOR, "invalid operator");
      if (hpan[i] == QP_IP) return fail(c, CYC_ERR_PANIC_IP, "unable to parse IP '" + q.pod_ip_str[hpid[i]] + "'");
      const std::string& cs = q.cidr_str[hpid[i]];
      return fail(c, CYC_ERR_PANIC_CIDR, "unable to parse CIDR '" + cs + "': invalid CIDR address: " + cs);
    }
    out[i] = hres[i];
  }
  if (tlist) {
    std::vector<uint8_t> hfl(nfl);
    if (nfl) HIPCHK(hipMemcpy(hfl.data(), dfl.p, nfl, hipMemcpyDeviceToHost));
    tlist->assign(ts.size() * 2, {});
    for (size_t i = 0; i < ts.size(); i++)
      for (int d = 0; d < 2; d++) {
        uint32_t T = uint32_t(d == 0 ? 2 * i + 1 : 2 * i);
        uint32_t lo = q.tns_lo[d][q.pod_ns[T]], hi = q.tns_hi[d][q.pod_ns[T]];
        for (uint32_t t = lo; t < hi; t++) {
          uint8_t f = hfl[hoff[2 * i + d] + (t - lo)];
          if (f) (*tlist)[2 * i + d].push_back(f == 1 ? int64_t(t) : -int64_t(t) - 1);
        }
      }
  }
  return (int)CYC_OK;
}

int cyc_query_traffic(cyc_ctx* c, const char* js, size_t len, uint8_t* out, int64_t n) {
  if (!c || !js) return CYC_ERR_ARG;
  if (!c->have_policy) return fail(c, CYC_ERR_ARG, "load a policy first");
  return guarded(c, [&]() -> int {
    auto ts = load_traffics(json::parse(js, len));
    if (int64_t(ts.size()) > n) return fail(c, CYC_ERR_ARG, "output buffer smaller than the traffic list");
    if (ts.empty()) return (int)CYC_OK;
    return run_query(c, ts, out, nullptr);
  });
}

int cyc_query_traffic_tables(cyc_ctx* c, const cyc_traffic_tables* t, uint8_t* out, int64_t n) {
  if (!c || !t) return CYC_ERR_ARG;
  if (!c->have_policy) return fail(c, CYC_ERR_ARG, "load a policy first");
  return guarded(c, [&]() -> int {
    auto ts = load_traffic_tables(*t);
    if (int64_t(ts.size()) > n || (!ts.empty() && !out)) return fail(c, CYC_ERR_ARG, "output buffer smaller than the traffic list");
    if (ts.empty()) return (int)CYC_OK;
    return run_query(c, ts, out, nullptr);
  });
}

static void json_str(std::string& o, const std::string& v) {
  o += '"';
  for (unsigned char ch : v) {
    if (ch == '"' || ch == '\\') {
      o += '\\';
      o += char(ch);
    } else if (ch < 0x20) {
      char b[8];
      snprintf(b, sizeof(b), "\\u%04x", ch);
      o += b;
    } else {
      o += char(ch);
    }
  }
  o += '"';
}

int cyc_query_traffic_targets(cyc_ctx* c, const char* js, size_t len, char* out_json, size_t cap, size_t* needed) {
  if (!c || !js) return CYC_ERR_ARG;
  if (!c->have_policy) return fail(c, CYC_ERR_ARG, "load a policy first");
  return guarded(c, [&]() -> int {
    auto ts = load_traffics(json::parse(js, len));
    std::vector<uint8_t> res(ts.size());
    std::vector<std::vector<int64_t>> tl;
    if (!ts.empty()) {
      int rc = run_query(c, ts, res.data(), &tl);
      if (rc != CYC_OK) return rc;
    }
    std::string o = "[";
    for (size_t i = 0; i < ts.size(); i++) {
      if (i) o += ',';
      o += '{';
      for (int d = 0; d < 2; d++) {
        o += d ? ",\"Egress\":{" : "\"Ingress\":{";
        for (int allow = 1; allow >= 0; allow--) {
          o += allow ? "\"AllowingTargets\":[" : ",\"DenyingTargets\":[";
          bool first = true;
          for (int64_t t : tl[2 * i + d]) {
            if ((t >= 0) != bool(allow)) continue;
            if (!first) o += ',';
            first = false;
            json_str(o, c->policy.dir[d][size_t(t >= 0 ? t : -t - 1)].pk);
          }
          o += ']';
        }
        o += ",\"IsAllowed\":";
        o += (res[i] >> d) & 1 ? "true" : "false";
        o += '}';
      }
      o += ",\"IsAllowed\":";
      o += (res[i] & 3) == 3 ? "true" : "false";
      o += '}';
    }
    o += ']';
    if (needed) *needed = o.size() + 1;
    if (!out_json || cap < o.size() + 1) return fail(c, CYC_ERR_ARG, "output buffer too small (see *needed)");
    memcpy(out_json, o.c_str(), o.size() + 1);
    return (int)CYC_OK;
  });
}

int cyc_query_targets(cyc_ctx* c, const char* js, size_t len, char* out_json, size_t cap, size_t* needed) {
  if (!c || !js) return CYC_ERR_ARG;
  if (!c->have_policy) return fail(c, CYC_ERR_ARG, "load a policy first");
  return guarded(c, [&]() -> int {
    auto ts = load_target_pods(json::parse(js, len));
    std::vector<uint8_t> res(ts.size());
    std::vector<std::vector<int64_t>> tl;
    if (!ts.empty()) {
      int rc = run_query(c, ts, res.data(), &tl, true);
      if (rc != CYC_OK) return rc;
    }
    std::string o = "[";
    for (size_t i = 0; i < ts.size(); i++) {
      o += i ? ",{" : "{";
      for (int d = 0; d < 2; d++) {
        o += d ? "],\"Egress\":[" : "\"Ingress\":[";
        for (size_t x = 0; x < tl[2 * i + d].size(); x++) {
          if (x) o += ',';
          json_str(o, c->policy.dir[d][size_t(tl[2 * i + d][x])].pk);
        }
      }
      o += "]}";
    }
    o += ']';
    if (needed) *needed = o.size() + 1;
    if (!out_json || cap < o.size() + 1) return fail(c, CYC_ERR_ARG, "output buffer too small (see *needed)");
    memcpy(out_json, o.c_str(), o.size() + 1);
    return (int)CYC_OK;
  });
}

}  // extern "C"
