// dev_query.hpp — the panic path, single-cell queries and lazy table cells.
// Part of engine.hip's single translation unit (device bodies inline across stages, host helpers are
// static): included once, by engine.hip, in stage order.
#pragma once

namespace cyc {

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
