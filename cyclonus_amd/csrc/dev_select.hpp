// dev_select.hpp — device helpers: selector evaluation on label sets, the PLVT gather table, fills, CIDR and peer outcomes.
// Part of engine.hip's single translation unit (device bodies inline across stages, host helpers are
// static): included once, by engine.hip, in stage order.
#pragma once

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

}  // namespace cyc
