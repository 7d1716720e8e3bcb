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
#include <rccl/rccl.h>

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

// Device code, by stage (namespace cyc)
#include "dev_select.hpp"
#include "dev_peer_rows.hpp"
#include "dev_slots.hpp"
#include "dev_member.hpp"
#include "dev_class_rows.hpp"
#include "dev_front.hpp"
#include "dev_emit.hpp"
#include "dev_query.hpp"
#include "dev_gather.hpp"

// Host side: context, planner, enqueueing; the C ABI below
#include "ctx.hpp"
#include "plan.hpp"
#include "enqueue.hpp"

extern "C" {

const char* cyc_version(void) { return "cyclonus_hip 0.2 (gfx950, ABI 2)"; }
int cyc_abi_version(void) { return CYC_ABI_VERSION; }

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
    for (auto& e : c->ev_p) ok = ok && hipEventCreateWithFlags(&e, EV_TIMING) == hipSuccess;
    if (!ok) {  // (left to the first prepare, which reports the error)
      for (auto& e : c->ev)
        if (e) (void)hipEventDestroy(e), e = nullptr;
      for (auto& e : c->ev_p)
        if (e) (void)hipEventDestroy(e), e = nullptr;
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
    comm_release(c);
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
      for (auto& e : c->ev_p) HIPCHK(hipEventCreateWithFlags(&e, EV_TIMING));
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
      if (c->phase_used) {  // row phases: phase 2's class rows ran between the emits (ev_p)
        float p2 = 0;
        HIPCHK(hipEventElapsedTime(&p2, c->ev_p[0], c->ev_p[1]));
        b -= p2;
        r += p2;
      }
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
    // the last run's stream, not an event recorded after every run: an event at each step's end held
    // the next step's first launch ~4.5 us (config #2: 0.0640 -> 0.0598 ms per step without it, r05at)
    HIPCHK(hipStreamSynchronize(c->last_stream));
    for (int d = 0; d < 2; d++) {
      uint32_t v[2] = {0xFFFFFFFFu, 0u};  // reps[]'s head (count - 1) and tail (row phases' phase-2 classes)
      if (c->dir[d].n && c->n_act[d]) HIPCHK(hipMemcpy(v, c->dir[d].rep_cnt(), 8, hipMemcpyDeviceToHost));
      out[d] = int64_t(uint32_t(v[0] + 1u)) + int64_t(v[1]);
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
    else if (n == "ip_iv") {
      range(-1, 1);
      c->ip_iv = int(value);
      c->order_lo = c->order_hi = -1;  // the next run re-plans which IP rows are interval-built
    }
    else if (n == "member_wave") range(-1, 1), c->member_wave = int(value);
    else if (n == "class_rpb") range(0, 64), c->class_rpb_opt = value;
    else if (n == "pl_wave") range(0, 1), c->pl_wave = int(value);
    else if (n == "sel_lazy") range(-1, 1), c->sel_lazy = int(value);
    else if (n == "pr_group") range(-1, 64), c->pr_group = int(value == 0 ? -1 : value);
    else if (n == "class_inplace") range(-1, 1), c->class_inplace = int(value);
    else if (n == "step_events") range(0, 1), c->step_events = int(value);
    else if (n == "emit_interleave") range(-1, 1), c->emit_interleave = int(value);
    else if (n == "row_phases") {
      range(-1, 4);
      if (value == 0 || value > 2) throw Panic{CYC_ERR_ARG, "row_phases must be -1 (auto), 1 (off) or 2"};
      c->row_phases = int(value);
      c->order_lo = c->order_hi = -1;  // the emit lists are re-planned
    }
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
  else if (n == "ip_iv") *value = c->ip_iv;
  else if (n == "ip_iv_rows") *value = c->Rv;  // (the last range plan's interval-built rows)
  else if (n == "member_wave") *value = c->member_wave;
  else if (n == "class_rpb") *value = c->class_rpb_opt;
  else if (n == "pl_wave") *value = c->pl_wave;
  else if (n == "sel_lazy") *value = c->sel_lazy;
  else if (n == "pr_group") *value = c->pr_group;
  else if (n == "class_inplace") *value = c->class_inplace;
  else if (n == "row_phases") *value = c->row_phases;
  else if (n == "row_phases_active") *value = c->phase_used;  // (the last run's phases; 0: a plain run)
  else if (n == "class_inplace_active") {
    if (!c->prepared || c->order_lo < 0) return fail(c, CYC_ERR_ARG, "class_inplace_active: run a probe first");
    *value = inplace_ok(c, reinterpret_cast<const uint64_t*>(16), reinterpret_cast<const uint64_t*>(16)) ? 1 : 0;
  }
  else if (n == "step_events") *value = c->step_events;
  else if (n == "emit_interleave") *value = c->emit_interleave;
  else if (n == "ip_items") *value = c->ip_items_opt;
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

// Multi-GPU table assembly: the RCCL communicator and the all-gather of row shards (C ABI included)
#include "comm.hpp"
