// host.hpp — host side of libcyclonus_hip: the policy compiler (reference pkg/matcher/builder.go +
// simplifier.go restated), the probe model (pkg/connectivity/probe/resources.go, pod.go) and the
// flattening of both into the device tables consumed by engine.hip.
//
// The host does only O(input) work here: decoding, interning strings / label maps / selectors,
// parsing CIDR and IP strings into fixed-width words, and resolving each destination pod's probe
// jobs (resources.go:284-364; O(pods x containers)).  Every O(pods x policies) and O(pods^2 x
// ports) step of the verdict path runs on the GPU (engine.hip).
#pragma once
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <optional>
#include <string>
#include <unordered_map>
#include <vector>

#include "cjson.hpp"
#include "cyclonus_hip.h"
#include "tables.h"

namespace cyc {

// CYC_TRACE_PREPARE=1: host phase times of cyc_probe_prepare on stderr (development aid)
struct PhaseClock {
  const char* what;
  bool on = getenv("CYC_TRACE_PREPARE") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  explicit PhaseClock(const char* w) : what(w) {}
  void lap(const char* phase) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    fprintf(stderr, "[cyc %s] %-14s %8.2f ms\n", what, phase, std::chrono::duration<double, std::milli>(n - t).count());
    t = n;
  }
};


// A Go panic the reference would raise (message text follows the reference).
struct Panic {
  int code;
  std::string msg;
};

struct IntStr {
  bool is_str = false;
  int32_t i = 0;
  std::string s;
  bool operator==(const IntStr& o) const { return is_str == o.is_str && (is_str ? s == o.s : i == o.i); }
};

struct Requirement {
  std::string key, op;
  std::vector<std::string> values;
};

// metav1.LabelSelector (matchLabels kept sorted: only AND semantics and sorted serialisation matter)
struct Selector {
  std::map<std::string, std::string> labels;
  std::vector<Requirement> exprs;
  bool empty() const { return labels.empty() && exprs.empty(); }
  std::string serialize() const;  // kube.SerializeLabelSelector (labelselector.go:94-112)
  std::string to_json() const;    // json.Marshal(metav1.LabelSelector)
};

// ----------------------------------------------------------------------------- compiled IR
// Mirrors *matcher.Policy after BuildNetworkPolicies (+ Simplify).
struct PortEntry {  // matcher.PortProtocolMatcher (port nil => has_port false)
  bool has_port = false;
  IntStr port;
  std::string proto;
  bool equals(const PortEntry& o) const {
    return proto == o.proto && has_port == o.has_port && (!has_port || port == o.port);
  }
};
struct PortRange {  // matcher.PortRangeMatcher
  int32_t from = 0, to = 0;
  std::string proto;
};
// Go []*PortRangeMatcher: a (backing array, len, cap) view, so slice aliasing in
// SpecificPortMatcher.Combine (portmatcher.go:126) is reproduced exactly.
struct RangeSlice {
  int arr = -1;
  uint32_t len = 0, cap = 0;
};
struct PortMatcher {  // AllPortMatcher | SpecificPortMatcher
  bool all = false;
  std::vector<PortEntry> ports;
  bool ports_nil = true;
  RangeSlice ranges;
};

enum PeerKind : uint32_t { PK_ALL = 0, PK_PORTS = 1, PK_POD = 2, PK_IP = 3 };
enum NsKind : uint32_t { NS_EXACT = 0, NS_ALL = 1, NS_LABEL = 2 };

struct Peer {
  PeerKind kind = PK_ALL;
  int port = -1;  // index into PolicyIR::pm (shared between peers of one rule, builder.go:84)
  NsKind ns_kind = NS_EXACT;
  std::string ns;   // NS_EXACT
  Selector ns_sel;  // NS_LABEL
  bool pod_all = true;
  Selector pod_sel;
  std::string cidr;  // PK_IP
  std::vector<std::string> except;
  bool except_nil = true;
  std::string pod_pk() const;  // PodPeerMatcher.PrimaryKey (podpeermatcher.go:17-19)
  std::string ip_pk() const;   // IPPeerMatcher.PrimaryKey (ippeermatcher.go:21-31)
};

struct Target {
  std::string ns;
  Selector sel;
  std::vector<Peer> peers;
  bool peers_nil = true;
  std::vector<std::string> rules;  // SourceRules (names only)
  std::string pk;                  // GetPrimaryKey (target.go:57-62)
};

struct PolicyIR {
  std::vector<PortMatcher> pm;
  std::vector<std::vector<PortRange>> range_arrays;  // Go backing arrays (size == cap)
  std::vector<Target> dir[2];                        // 0 = ingress, 1 = egress; sorted by pk
  std::vector<PortRange> ranges_of(const PortMatcher& m) const;
};

// builder.go:11-26 BuildNetworkPolicies(simplify, netpols); `netpols` is a JSON array of
// k8s NetworkPolicy objects (or a List with "items", or a single object).  Throws Panic.
PolicyIR build_network_policies(const json::Node& netpols, bool simplify);
// Load json.Marshal(*matcher.Policy) — what a cgo binding hands over.
PolicyIR load_policy_ir(const json::Node& ir);
std::string dump_policy_ir(const PolicyIR& p);
// The same IR from the flat tables of include/cyclonus_hip.h (cyc_policy_tables); throws Panic{CYC_ERR_ARG}.
PolicyIR load_policy_tables(const cyc_policy_tables& t);

// ----------------------------------------------------------------------------- probe model
// probe.Resources (resources.go:15-19, pod.go:44-51,173-179) in interned form: every string is an
// index into `str` (duplicates allowed: the flat tables of a binding may repeat a string), maps and
// lists are offset ranges.  Both loaders fill it — the JSON one (cyc_resources_load_json) and the
// flat tables a cgo binding passes without JSON (cyc_resources_load) — and build_problem reads only
// this, mapping each distinct string to the problem's dictionary once instead of once per use.
struct Container {  // probe.Container: Name, Port, Protocol, PortName
  uint32_t name = 0, proto = 0, port_name = 0;
  int32_t port = 0;
};
struct Resources {
  std::vector<std::string> str;
  // Namespaces map[string]map[string]string: key, nil-ness of the label map, its labels
  std::vector<uint32_t> ns_name;
  std::vector<uint8_t> ns_nil;
  std::vector<uint32_t> ns_lab_off{0}, ns_lab_key, ns_lab_val;
  // Pods, in Resources.Pods order
  std::vector<uint32_t> pod_ns, pod_name, pod_ip;
  std::vector<uint32_t> pod_lab_off{0}, lab_key, lab_val;  // a Go map: duplicate keys, if given, last wins
  std::vector<uint32_t> pod_cont_off{0};
  std::vector<Container> conts;
  std::vector<uint8_t> pod_nil;  // per pod: bit 0 Labels == nil, bit 1 Containers == nil (json.Marshal: null)
  size_t pods() const { return pod_ns.size(); }
  uint32_t n_conts(size_t p) const { return pod_cont_off[p + 1] - pod_cont_off[p]; }
  const Container& cont(size_t p, uint32_t i) const { return conts[pod_cont_off[p] + i]; }
  const std::string& s(uint32_t id) const { return str[id]; }
  std::string pod_string(size_t p) const { return str[pod_ns[p]] + "/" + str[pod_name[p]]; }  // PodString
};
struct ProbeConfig {  // generator.ProbeConfig (AllAvailable | PortProtocol)
  bool all_available = false;
  IntStr port;
  std::string proto;
};

Resources load_resources(const json::Node& n);
// The flat tables of include/cyclonus_hip.h, validated (a bad index or offset throws Panic{CYC_ERR_ARG}).
Resources load_resources_tables(const cyc_resource_tables& t);
std::string dump_resources(const Resources& r);  // json.Marshal(*probe.Resources) of the kept fields
std::vector<ProbeConfig> load_probes(const json::Node& n);
std::vector<ProbeConfig> load_probe_configs(const cyc_probe_config* cfgs, int64_t n);

// A batched problem's block (cyc_probe_prepare_blocks): pods [p0, p1) of the Resources form an
// independent probe problem answering probe config `cfg` only, over its own pods only.
struct ProbeBlock {
  uint32_t p0 = 0, p1 = 0, cfg = 0;
};

// ----------------------------------------------------------------------------- device tables
// Everything engine.hip uploads, flattened and interned.
struct Problem {
  // dictionaries
  std::vector<std::string> strings;  // interned strings (namespaces, keys, values, protocols, port names)
  std::unordered_map<std::string, uint32_t> string_id;
  uint32_t intern(const std::string& s);

  uint32_t P = 0, K = 0, W = 0;  // pods, job slots, 64-bit words per bit-row
  uint32_t L = 0, S = 0;         // label sets, selectors
  // label sets (0 == empty / nil map)
  std::vector<uint32_t> ls_off, ls_key, ls_val;
  // selectors
  std::vector<uint32_t> sel_off;
  std::vector<DReq> reqs;
  std::vector<uint32_t> req_vals;
  // pods
  std::vector<uint32_t> pod_ns, pod_ls, pod_nsls;
  std::vector<DIP> pod_ip;
  std::vector<std::string> pod_ip_str;  // pod IP strings (panic messages; only the unparsable ones are kept)
  // CIDRs / IP blocks
  std::vector<DCidr> cidrs;
  std::vector<std::string> cidr_str;
  std::vector<DIPBlock> ipbs;
  std::vector<uint32_t> ipb_ex;
  // port matchers
  std::vector<DPortM> pms;
  std::vector<DPortEntry> pents;
  // peers + targets
  std::vector<DPeer> peers;
  std::vector<DTarget> tgt[2];
  std::vector<uint32_t> tns_lo[2], tns_hi[2];  // per namespace string id: target range
  // job descriptors (port, port-name id, protocol id) and per-(pod, slot) table
  std::vector<DDesc> descs;
  std::vector<int32_t> slot_desc;  // [P][K], -1 => no valid job
  std::vector<uint8_t> slot_status;
  std::vector<uint32_t> slot_cfg, slot_idx;  // slot -> (probe config, job index in config)
  uint32_t n_cfg = 0;
  // evaluation can reach a Go panic (invalid selector operator / CIDR / IP)
  bool may_err = false;
  // first duplicate table key per config, if any (table.go:45 via utils.DoOrDie)
  std::vector<std::string> dup_key_msg;
  // per config: the job expansion itself panics (a pod without containers is some job's podFrom:
  // FromContainer = podFrom.Containers[0].Name, resources.go:296,349 -> index out of range)
  std::vector<uint8_t> expand_panic;
  // batched blocks (empty: one problem over all pods); per block its own expansion panic and
  // duplicate-key fatal, computed over its pods and config only
  std::vector<ProbeBlock> blocks;
  std::vector<uint32_t> pod_blk;  // [P] block of each pod
  std::vector<uint8_t> blk_expand_panic;
  std::vector<std::string> blk_dup_msg;
};

Problem build_problem(const PolicyIR& pol, const Resources& res, const std::vector<ProbeConfig>& probes,
                      const std::vector<ProbeBlock>* blocks = nullptr);

// matcher.Traffic (traffic.go:11-18) for the single-cell query API.
struct QueryEnd {
  bool external = true;  // Internal == nil
  std::string ns, ip;
  std::map<std::string, std::string> labels, ns_labels;
};
struct QueryTraffic {
  QueryEnd src, dst;
  int32_t port = 0;
  std::string port_name, proto;
};
std::vector<QueryTraffic> load_traffics(const json::Node& n);
std::vector<QueryTraffic> load_traffic_tables(const cyc_traffic_tables& t);
std::vector<QueryTraffic> load_target_pods(const json::Node& n);
Problem build_query_problem(const PolicyIR& pol, const std::vector<QueryTraffic>& ts, std::vector<uint32_t>& ext,
                            std::vector<uint32_t>& tdesc);

}  // namespace cyc
