// ctx.hpp — the context: device buffers, options, error handling.
// Part of engine.hip's single translation unit (device bodies inline across stages, host helpers are
// static): included once, by engine.hip, in stage order.
#pragma once

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
struct RcclErr {  // an RCCL call failed (CYC_ERR_RCCL)
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
  std::vector<uint4> sel_one_h;  // its host copy (the identity-set peer records, pb_rec)
  // per identity-set row (pod_peers_u): its matcher as three 16-byte records — (namespace matcher kind,
  // namespace / selector, pod selector, 0), then the namespace selector's and the pod selector's
  // one-requirement records (SelView::one; SEL_ALL when there is none): peer_bits_blk loads a row
  // group's records in one vector load instead of pod_peers -> peers -> one chains
  DevBuf pb_rec;
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
  // IP rows as pod intervals (ip_rows_iv_blk): when a family's pods hold non-decreasing addresses in
  // pod order (ip_mono[0] IPv4, [1] IPv6), a network less its excepts matches that family's pods in
  // a few pod-index intervals; per direction the rows built that way
  bool ip_mono[2] = {false, false};
  DevBuf ipv_tests, ipv_iv;
  uint32_t rv_off[3] = {0, 0, 0}, Rv = 0;
  uint32_t rpu_off[3] = {0, 0, 0};  // sub-lists of pod_peers_u: one pod peer per distinct matcher
  DevBuf ipi_items, ipi_list;   // IP-row work items of the fused front (DIPItem; ip_rows_items_blk) and their rows
  uint32_t ipi_off[3] = {0, 0, 0};  // items of segment x: [ipi_off[x], ipi_off[x + 1])
  bool ip_items = false;        // the current plan's items are built (option "ip_items" on and fast IP rows present)
  int ip_items_opt = -1;        // "ip_items": -1 auto (whole-table runs) / 0 / 1
  std::vector<DWordIP> ipw_h;   // host copy of the IP word and chunk records (ip_words)
  DevBuf ido_grp_ns, ido_word_ns;  // identity-set namespace skip (peer_bits_blk): per row group, per identity word
  uint32_t ido_goff[2] = {0, 0};   // first group of each direction's sub-list in ido_grp_ns
  PeerPlan plan;                 // all pod / IP peers (host); filtered per row range
  DevBuf act[2], actrec[2], sel_list;
  DevBuf arow[2];  // per identity: its first pod's row in the run's row range (in-place class rows)
  uint32_t n_act[2] = {0, 0}, n_sel = 0;
  uint32_t n_act_ph1[2] = {0, 0};  // row phases: active identities whose first row is before the split (every
                                   // phase-1 class's representative is one of them)
  double act_targets[2] = {0, 0};  // mean namespace targets per active identity (range plan)
  // Diagnostic path selectors (cyc_set_option; results never change, the GPU tests force each path):
  int use_graphs = -1;  // "graphs": 1 = graph replay, 2 = the same DAG enqueued eagerly on three
                        // streams with events (no graph launch), 0 = eager on one stream with phase
                        // events, -1 = auto: 2 when the fused front applies (its launches on one
                        // stream start ~8 us sooner after the previous step's emit than a graph
                        // replay: profiles/r01_front_fused_ab.txt), else 1
  int ip_iv = -1;       // "ip_iv": IP rows as pod intervals where the network's family is address-monotone
                        // in pod order (-1 auto = 1), 0 never
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
  hipStream_t last_stream = nullptr;  // the stream the last run was enqueued on
  // batched blocks (cyc_probe_prepare_blocks; pb.blocks non-empty)
  DevBuf blk, blk_off, id_blk[2], id_win[2], first_blk;
  uint32_t blk_wa_max = 0, blk_np_max = 0;
  std::vector<uint64_t> blk_off_h;          // per block: plane slab offset (words), status offset (bytes); then totals
  std::vector<int> blk_rc;                  // per block status of the last run
  std::vector<std::string> blk_msg;         // and its message
  // Row phases ("row_phases"): a whole-table run's class rows and emit in two phases — the class rows
  // of the classes rows [0, P/2) use, the emit of those rows, then the other classes' rows and the emit
  // of rows [P/2, P) — so a phase's class rows (~200 MB for config #3) are still in the 256 MB MALL when
  // its emit re-reads them; the whole table's (~400 MB) are not, and its emit reads them from HBM
  // between its writes (round 6, profiles/r06_emit_footprint_ab.txt).  The front before the class rows
  // runs once.
  int row_phases = -1;     // -1 auto (whole no-panic tables of >= 8 GB planes), 1 = off, 2 = whenever possible
  uint32_t phase_split = 0;   // the range plan's split row (0: no phases): emit lists are [rows < split][rows >= split]
  uint32_t phase_n1[2] = {0, 0};  // per plane: rows before the split in its emit list
  int phase_used = 0;      // the last run's phases (2, or 0 for a plain run)
  hipEvent_t ev_p[2] = {nullptr, nullptr};  // eager runs: around phase 2's class rows (cyc_last_timings)
  // multi-GPU table assembly (comm.hpp): the context's RCCL communicator, a second stream on which
  // gathered chunks are relaid out under the next chunk's all-gather, and the chunks' double buffer
  struct Comm {
    ncclComm_t nccl = nullptr;
    int nranks = 0, rank = -1;
    hipStream_t merge = nullptr;
    hipEvent_t full[2] = {nullptr, nullptr}, free_[2] = {nullptr, nullptr}, done = nullptr;
    DevBuf scratch[2];
  } comm;
};

int describe_panic(cyc_ctx* c, uint32_t s, uint32_t d, uint32_t cfg, uint32_t idx);
static void comm_release(cyc_ctx* c);  // comm.hpp
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
  } catch (RcclErr& r) {
    return fail(c, CYC_ERR_RCCL, r.msg);
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
