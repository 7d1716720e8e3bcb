// oracle/oracle.cpp — CPU restatement of cyclonus's simulated-connectivity verdict path.
//
// TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
// leg may load this library, and only as the checker / the timed CPU baseline.  The product
// (cyclonus_amd/, libcyclonus_hip.so) never links, calls or falls back to it.
//
// Parity pinning: the Go reference cannot be built here (no Go toolchain; k8s.io deps not
// vendored).  This restatement is pinned by the reference's own golden vectors,
// transcribed under tests/golden/ (README.md:294-313 combined table, pkg/matcher/policy_tests.go,
// builder_tests.go, simplifier_tests.go, pkg/kube/ipaddress_tests.go, labelselector_tests.go).
// IPv6 / v4-mapped IP semantics and the Q2 slice-aliasing quirk are parity-UNPINNED by those
// fixtures (ipaddress_tests.go:49-53 is empty); they follow Go 1.16 source semantics.
//
// Structure mirrors the reference one-to-one, per cell, with no class compression:
//   pkg/matcher/builder.go      BuildNetworkPolicies / BuildTarget / BuildPeerMatcher / ...
//   pkg/matcher/policy.go       Policy.AddTarget / TargetsApplyingToPod / IsTrafficAllowed
//   pkg/matcher/target.go       Target.IsMatch / Allows / Combine / GetPrimaryKey
//   pkg/matcher/*peermatcher.go PeerMatcher kinds and PrimaryKeys
//   pkg/matcher/portmatcher.go  PortMatcher kinds, Combine (incl. quirk Q1), Subtract
//   pkg/matcher/simplifier.go   Simplify
//   pkg/kube/labelselector.go   IsLabelsMatchLabelSelector / SerializeLabelSelector
//   pkg/kube/ipaddress.go       IsIPInCIDR / IsIPAddressMatchForIPBlock
//   pkg/connectivity/probe/{resources,pod,job,jobrunner}.go  jobs + simulated runner
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <optional>
#include <set>
#include <sstream>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "gonet.hpp"
#include "goslice.hpp"
#include "ojson.hpp"

using goslice::Slice;
using ojson::go_quote;
using ojson::Value;
using ojson::VP;

namespace orc {

struct GoPanic {
  std::string msg;
};
[[noreturn]] static void go_panic(const std::string& m) { throw GoPanic{m}; }

using Labels = std::map<std::string, std::string>;
// Go `map[string]string` that may be nil; nil behaves as an empty map for reads.
using LabelsP = std::shared_ptr<Labels>;

// ---------------------------------------------------------------- k8s API types (decoded JSON)
struct IntOrString {
  bool is_str = false;
  int32_t ival = 0;
  std::string sval;
};
struct Requirement {
  std::string key, op;
  std::vector<std::string> values;
};
struct LabelSelector {
  Labels matchLabels;
  std::vector<Requirement> matchExpressions;
};
struct IPBlock {
  std::string cidr;
  std::vector<std::string> except;
  bool except_nil = true;
};
struct NetpolPort {
  std::optional<std::string> protocol;
  std::optional<IntOrString> port;
  std::optional<int32_t> endPort;
};
struct NetpolPeer {
  std::optional<LabelSelector> podSelector, namespaceSelector;
  std::shared_ptr<IPBlock> ipBlock;
};
struct NetpolRule {
  std::vector<NetpolPort> ports;
  std::vector<NetpolPeer> peers;
};
struct NetworkPolicy {
  std::string name, ns;
  LabelSelector podSelector;
  std::vector<NetpolRule> ingress, egress;
  std::vector<std::string> policyTypes;
};

static IntOrString decode_intstr(const Value& v) {
  // k8s.io/apimachinery/pkg/util/intstr/intstr.go UnmarshalJSON: '"' => String else Int
  IntOrString r;
  if (v.kind == Value::String) {
    r.is_str = true;
    r.sval = v.s;
  } else {
    r.ival = int32_t(v.as_int());
  }
  return r;
}

static LabelSelector decode_selector(const Value& v) {
  LabelSelector s;
  if (auto ml = v.get("matchLabels"); ml && ml->kind == Value::Object)
    for (auto& kv : ml->obj) s.matchLabels[kv.first] = kv.second->is_null() ? "" : kv.second->as_str();
  if (auto me = v.get("matchExpressions"); me && me->kind == Value::Array)
    for (auto& e : me->arr) {
      Requirement r;
      if (auto k = e->get("key")) r.key = k->as_str();
      if (auto o = e->get("operator")) r.op = o->as_str();
      if (auto vs = e->get("values"); vs && vs->kind == Value::Array)
        for (auto& x : vs->arr) r.values.push_back(x->as_str());
      s.matchExpressions.push_back(r);
    }
  return s;
}

static std::vector<NetpolPort> decode_ports(const Value* v) {
  std::vector<NetpolPort> out;
  if (!v || v->kind != Value::Array) return out;
  for (auto& p : v->arr) {
    NetpolPort np;
    if (auto pr = p->get("protocol"); pr && !pr->is_null()) np.protocol = pr->as_str();
    if (auto po = p->get("port"); po && !po->is_null()) np.port = decode_intstr(*po);
    if (auto ep = p->get("endPort"); ep && !ep->is_null()) np.endPort = int32_t(ep->as_int());
    out.push_back(np);
  }
  return out;
}

static std::vector<NetpolPeer> decode_peers(const Value* v) {
  std::vector<NetpolPeer> out;
  if (!v || v->kind != Value::Array) return out;
  for (auto& p : v->arr) {
    NetpolPeer np;
    if (auto ps = p->get("podSelector"); ps && !ps->is_null()) np.podSelector = decode_selector(*ps);
    if (auto ns = p->get("namespaceSelector"); ns && !ns->is_null()) np.namespaceSelector = decode_selector(*ns);
    if (auto ib = p->get("ipBlock"); ib && !ib->is_null()) {
      np.ipBlock = std::make_shared<IPBlock>();
      if (auto c = ib->get("cidr")) np.ipBlock->cidr = c->as_str();
      if (auto ex = ib->get("except"); ex && ex->kind == Value::Array) {
        np.ipBlock->except_nil = false;
        for (auto& e : ex->arr) np.ipBlock->except.push_back(e->as_str());
      }
    }
    out.push_back(np);
  }
  return out;
}

static NetworkPolicy decode_netpol(const Value& v) {
  NetworkPolicy np;
  if (auto md = v.get("metadata")) {
    if (auto n = md->get("name"); n && !n->is_null()) np.name = n->as_str();
    if (auto n = md->get("namespace"); n && !n->is_null()) np.ns = n->as_str();
  }
  const Value* spec = v.get("spec");
  if (!spec) return np;
  if (auto ps = spec->get("podSelector"); ps && !ps->is_null()) np.podSelector = decode_selector(*ps);
  if (auto pt = spec->get("policyTypes"); pt && pt->kind == Value::Array)
    for (auto& t : pt->arr) np.policyTypes.push_back(t->as_str());
  if (auto in = spec->get("ingress"); in && in->kind == Value::Array)
    for (auto& r : in->arr) np.ingress.push_back({decode_ports(r->get("ports")), decode_peers(r->get("from"))});
  if (auto eg = spec->get("egress"); eg && eg->kind == Value::Array)
    for (auto& r : eg->arr) np.egress.push_back({decode_ports(r->get("ports")), decode_peers(r->get("to"))});
  return np;
}

// ---------------------------------------------------------------- pkg/kube/labelselector.go
static bool has(const LabelsP& l, const std::string& k, std::string* v = nullptr) {
  if (!l) return false;
  auto it = l->find(k);
  if (it == l->end()) return false;
  if (v) *v = it->second;
  return true;
}

// labelselector.go:24-59 IsMatchExpressionMatchForLabels
static bool is_match_expression(const LabelsP& labels, const Requirement& exp) {
  std::string val;
  if (exp.op == "In") {
    if (!has(labels, exp.key, &val)) return false;
    for (auto& v : exp.values)
      if (v == val) return true;
    return false;
  } else if (exp.op == "NotIn") {
    if (!has(labels, exp.key, &val)) return false;  // absent key: NOT a match (:37-42)
    for (auto& v : exp.values)
      if (v == val) return false;
    return true;
  } else if (exp.op == "Exists") {
    return has(labels, exp.key);
  } else if (exp.op == "DoesNotExist") {
    return !has(labels, exp.key);
  }
  go_panic("invalid operator");  // :57
}

// labelselector.go:66-86 IsLabelsMatchLabelSelector
static bool is_labels_match(const LabelsP& labels, const LabelSelector& sel) {
  for (auto& kv : sel.matchLabels) {
    std::string v;
    has(labels, kv.first, &v);  // labels[key] ("" when absent)
    if (v != kv.second) return false;
  }
  for (auto& e : sel.matchExpressions)
    if (!is_match_expression(labels, e)) return false;
  return true;
}

static bool is_selector_empty(const LabelSelector& s) {  // :88-90
  return s.matchLabels.empty() && s.matchExpressions.empty();
}

// Go json.Marshal of metav1.LabelSelectorRequirement / []LabelSelectorRequirement
static std::string requirement_json(const Requirement& r) {
  std::string o = "{\"key\":" + go_quote(r.key) + ",\"operator\":" + go_quote(r.op);
  if (!r.values.empty()) {
    o += ",\"values\":[";
    for (size_t i = 0; i < r.values.size(); i++) o += (i ? "," : "") + go_quote(r.values[i]);
    o += "]";
  }
  return o + "}";
}

// labelselector.go:94-112 SerializeLabelSelector
static std::string serialize_selector(const LabelSelector& ls) {
  std::string o = "[\"MatchLabels\",";
  if (ls.matchLabels.empty()) {
    o += "null";
  } else {
    o += "[";
    bool first = true;
    for (auto& kv : ls.matchLabels) {  // std::map: sorted by key, as sort.Slice(labelKeys)
      o += (first ? "" : ",") + go_quote(kv.first + ": " + kv.second);
      first = false;
    }
    o += "]";
  }
  o += ",\"MatchExpression\",";
  if (ls.matchExpressions.empty()) {
    o += "null";
  } else {
    o += "[";
    for (size_t i = 0; i < ls.matchExpressions.size(); i++)
      o += (i ? "," : "") + requirement_json(ls.matchExpressions[i]);
    o += "]";
  }
  return o + "]";
}

// Go json.Marshal(metav1.LabelSelector)
static std::string selector_json(const LabelSelector& ls) {
  std::string o = "{";
  bool comma = false;
  if (!ls.matchLabels.empty()) {
    o += "\"matchLabels\":{";
    bool first = true;
    for (auto& kv : ls.matchLabels) {
      o += (first ? "" : ",") + go_quote(kv.first) + ":" + go_quote(kv.second);
      first = false;
    }
    o += "}";
    comma = true;
  }
  if (!ls.matchExpressions.empty()) {
    o += comma ? "," : "";
    o += "\"matchExpressions\":[";
    for (size_t i = 0; i < ls.matchExpressions.size(); i++)
      o += (i ? "," : "") + requirement_json(ls.matchExpressions[i]);
    o += "]";
  }
  return o + "}";
}

// ---------------------------------------------------------------- pkg/kube/ipaddress.go
struct IPResult {
  bool ok;  // false => error
  bool member;
  std::string err;
};

// ipaddress.go:10-20 IsIPInCIDR
static IPResult is_ip_in_cidr(const std::string& ip, const std::string& cidr) {
  gonet::IPNet net;
  if (!gonet::ParseCIDR(cidr, net))
    return {false, false, "unable to parse CIDR '" + cidr + "': invalid CIDR address: " + cidr};
  gonet::IP tip = gonet::ParseIP(ip);
  if (tip.empty()) return {false, false, "unable to parse IP '" + ip + "'"};
  return {true, gonet::Contains(net, tip), ""};
}

// ipaddress.go:22-40 IsIPAddressMatchForIPBlock
static IPResult is_ip_match_block(const std::string& ip, const IPBlock& b) {
  IPResult r = is_ip_in_cidr(ip, b.cidr);
  if (!r.ok || !r.member) return r;
  for (auto& e : b.except) {
    IPResult x = is_ip_in_cidr(ip, e);
    if (!x.ok) return x;
    if (x.member) return {true, false, ""};
  }
  return {true, true, ""};
}

// ---------------------------------------------------------------- pkg/matcher/traffic.go
struct InternalPeer {
  LabelsP podLabels, nsLabels;
  std::string ns;
};
struct TrafficPeer {
  std::shared_ptr<InternalPeer> internal;  // nil => external
  std::string ip;
};
struct Traffic {
  TrafficPeer src, dst;
  int port = 0;
  std::string portName, protocol;
};

// ---------------------------------------------------------------- pkg/matcher/portmatcher.go
struct PortProtocolMatcher {
  std::optional<IntOrString> port;
  std::string protocol;
  bool allows(int portInt, const std::string& portName, const std::string& proto) const {  // :33-38
    if (port) {
      bool pm = port->is_str ? port->sval == portName : int(port->ival) == portInt;  // isPortMatch :190
      return pm && protocol == proto;
    }
    return protocol == proto;
  }
  bool equals(const PortProtocolMatcher& o) const {  // :40-51
    if (protocol != o.protocol) return false;
    if (!port && !o.port) return true;
    if (!port || !o.port) return false;
    if (port->is_str != o.port->is_str) return false;
    return port->is_str ? port->sval == o.port->sval : port->ival == o.port->ival;
  }
};
using PPMp = std::shared_ptr<PortProtocolMatcher>;

struct PortRangeMatcher {
  int from, to;
  std::string protocol;
  bool allows(int portInt, const std::string& proto) const { return from <= portInt && portInt <= to && protocol == proto; }
};
using PRMp = std::shared_ptr<PortRangeMatcher>;

struct PortMatcher {
  bool all = false;  // AllPortMatcher
  Slice<PPMp> ports;
  Slice<PRMp> ranges;
  bool allows(int portInt, const std::string& portName, const std::string& proto) const {  // :80-92
    if (all) return true;
    for (size_t i = 0; i < ports.len; i++)
      if (ports[i]->allows(portInt, portName, proto)) return true;
    for (size_t i = 0; i < ranges.len; i++)
      if (ranges[i]->allows(portInt, proto)) return true;
    return false;
  }
};
using PMp = std::shared_ptr<PortMatcher>;

// isPortLessThan :158-188 (nil < string < int)
static bool port_less(const std::optional<IntOrString>& a, const std::optional<IntOrString>& b) {
  if (!a) return bool(b);
  if (!b) return false;
  if (!a->is_str) return !b->is_str ? a->ival < b->ival : false;
  return !b->is_str ? true : a->sval < b->sval;
}

// SpecificPortMatcher.Combine :102-131 — restated INCLUDING quirk Q1 (the inner loop never
// runs when s.Ports is empty, dropping other.Ports) and Q2 (ranges appended into s's backing array)
static PMp specific_combine(const PortMatcher& s, const PortMatcher& other) {
  Slice<PPMp> empty_lit;  // []*PortProtocolMatcher{} (non-nil, cap 0)
  empty_lit.arr = std::make_shared<std::vector<PPMp>>();
  Slice<PPMp> pps = goslice::append(empty_lit, s.ports);
  for (size_t oi = 0; oi < other.ports.len; oi++) {
    PPMp otherPP = other.ports[oi];
    Slice<PPMp> snapshot = pps;  // `for _, pp := range pps` evaluates pps once
    for (size_t i = 0; i < snapshot.len; i++) {
      if (snapshot[i]->equals(*otherPP)) break;
      pps = goslice::append1(pps, otherPP);
    }
  }
  {
    std::vector<PPMp> v = pps.to_vector();
    std::stable_sort(v.begin(), v.end(), [](const PPMp& a, const PPMp& b) {
      if (port_less(a->port, b->port)) return true;
      if (port_less(b->port, a->port)) return false;
      return a->protocol < b->protocol;
    });
    for (size_t i = 0; i < v.size(); i++) pps.at(i) = v[i];
  }
  auto r = std::make_shared<PortMatcher>();
  r->ports = pps;
  r->ranges = goslice::append(s.ranges, other.ranges);  // :126
  return r;
}

// SpecificPortMatcher.Subtract :133-153
static std::pair<bool, PMp> specific_subtract(const PortMatcher& s, const PortMatcher& other) {
  Slice<PRMp> remainingRanges = s.ranges;
  Slice<PPMp> remaining;
  for (size_t i = 0; i < s.ports.len; i++) {
    bool found = false;
    for (size_t j = 0; j < other.ports.len; j++)
      if (s.ports[i]->equals(*other.ports[j])) {
        found = true;
        break;
      }
    if (!found) remaining = goslice::append1(remaining, s.ports[i]);
  }
  if (remainingRanges.len == 0 && remaining.len == 0) return {true, nullptr};
  auto r = std::make_shared<PortMatcher>();
  r->ports = remaining;
  r->ranges = remainingRanges;
  return {false, r};
}

// simplifier.go:142-159 CombinePortMatchers
static PMp combine_port_matchers(const PMp& a, const PMp& b) {
  if (a->all) return a;
  if (b->all) return b;
  return specific_combine(*a, *b);
}

// simplifier.go:164-189 SubtractPortMatchers
static std::pair<bool, PMp> subtract_port_matchers(const PMp& a, const PMp& b) {
  if (a->all) {
    if (b->all) return {true, nullptr};
    return {false, a};
  }
  if (b->all) return {true, nullptr};
  return specific_subtract(*a, *b);
}

// ---------------------------------------------------------------- pkg/matcher peer matchers
enum class NsKind { Exact, Label, All };
struct NsMatcher {
  NsKind kind;
  std::string ns;
  LabelSelector sel;
  bool allows(const std::string& n, const LabelsP& nsLabels) const {
    if (kind == NsKind::Exact) return ns == n;
    if (kind == NsKind::All) return true;
    return is_labels_match(nsLabels, sel);
  }
  std::string pk() const {
    if (kind == NsKind::Exact) return "{\"type\": \"exact-namespace\", \"namespace\": \"" + ns + "\"}";
    if (kind == NsKind::All) return "{\"type\": \"all-namespaces\"}";
    return "{\"type\": \"label-selector\", \"selector\": \"" + serialize_selector(sel) + "\"}";
  }
  std::string json() const {
    if (kind == NsKind::Exact) return "{\"Namespace\":" + go_quote(ns) + ",\"Type\":\"specific namespace\"}";
    if (kind == NsKind::All) return "{\"Type\":\"all namespaces\"}";
    return "{\"Selector\":" + selector_json(sel) + ",\"Type\":\"matching namespace by label\"}";
  }
};
struct PodMatcher {
  bool all;
  LabelSelector sel;
  bool allows(const LabelsP& l) const { return all || is_labels_match(l, sel); }
  std::string pk() const {
    if (all) return "{\"type\": \"all-pods\"}";
    return "{\"type\": \"label-selector\", \"selector\": \"" + serialize_selector(sel) + "\"}";
  }
  std::string json() const {
    if (all) return "{\"Type\":\"all pods\"}";
    return "{\"Selector\":" + selector_json(sel) + ",\"Type\":\"matching pods by label\"}";
  }
};

enum class PeerKind { AllPeers, PortsForAll, Pod, IP };
struct PeerMatcher {
  PeerKind kind;
  PMp port;
  std::shared_ptr<NsMatcher> ns;
  std::shared_ptr<PodMatcher> pod;
  std::shared_ptr<IPBlock> ip;

  // peermatcher.go:18,32; podpeermatcher.go:21-28; ippeermatcher.go:43-50
  bool allows(const TrafficPeer& peer, int portInt, const std::string& portName, const std::string& proto) const {
    switch (kind) {
      case PeerKind::AllPeers: return true;
      case PeerKind::PortsForAll: return port->allows(portInt, portName, proto);
      case PeerKind::Pod:
        if (!peer.internal) return false;
        return ns->allows(peer.internal->ns, peer.internal->nsLabels) && pod->allows(peer.internal->podLabels) &&
               port->allows(portInt, portName, proto);
      case PeerKind::IP: {
        IPResult r = is_ip_match_block(peer.ip, *ip);
        if (!r.ok) go_panic(r.err);
        return r.member && port->allows(portInt, portName, proto);
      }
    }
    return false;
  }
  std::string pod_pk() const { return ns->pk() + "---" + pod->pk(); }  // podpeermatcher.go:17
  std::string ip_pk() const {                                          // ippeermatcher.go:21-31
    std::vector<std::string> ex = ip->except;
    std::sort(ex.begin(), ex.end());
    std::string j;
    for (size_t i = 0; i < ex.size(); i++) j += (i ? ", " : "") + ex[i];
    return ip->cidr + ": [" + j + "]";
  }
};
using PeerP = std::shared_ptr<PeerMatcher>;
static PeerP kAllPeersPorts = std::make_shared<PeerMatcher>(PeerMatcher{PeerKind::AllPeers, nullptr, nullptr, nullptr, nullptr});

// ---------------------------------------------------------------- pkg/matcher/target.go
struct Target {
  std::string ns;
  LabelSelector podSelector;
  std::vector<PeerP> peers;
  bool peers_nil = true;
  std::vector<std::string> sourceRules;
  std::string pk_cache;
  bool is_match(const std::string& n, const LabelsP& podLabels) const {  // :25-27
    return ns == n && is_labels_match(podLabels, podSelector);
  }
  bool allows(const TrafficPeer& peer, int portInt, const std::string& portName, const std::string& proto) const {
    for (auto& p : peers)  // :29-36 (short-circuit, slice order)
      if (p->allows(peer, portInt, portName, proto)) return true;
    return false;
  }
  const std::string& pk() {  // :57-62
    if (pk_cache.empty())
      pk_cache = "{\"Namespace\": \"" + ns + "\", \"PodSelector\": " + serialize_selector(podSelector) + "}";
    return pk_cache;
  }
};
using TargetP = std::shared_ptr<Target>;

// ---------------------------------------------------------------- pkg/matcher/simplifier.go
static std::vector<PeerP> simplify(const std::vector<PeerP>& matchers, bool& out_nil) {
  bool matchesAll = false;
  std::vector<PeerP> pfa, ips, pods;
  for (auto& m : matchers) {
    switch (m->kind) {
      case PeerKind::AllPeers: matchesAll = true; break;
      case PeerKind::PortsForAll: pfa.push_back(m); break;
      case PeerKind::IP: ips.push_back(m); break;
      case PeerKind::Pod: pods.push_back(m); break;
    }
  }
  // simplifyPortsForAllPeers :36-45
  PeerP pfaM;
  if (!pfa.empty()) {
    PMp port = pfa[0]->port;
    for (size_t i = 1; i < pfa.size(); i++) port = combine_port_matchers(port, pfa[i]->port);
    pfaM = std::make_shared<PeerMatcher>(PeerMatcher{PeerKind::PortsForAll, port, nullptr, nullptr, nullptr});
  }
  // simplifyIPMatchers :68-88 (grouping in slice order; result sorted by pk)
  {
    std::vector<std::string> order;
    std::map<std::string, PeerP> grouped;
    for (auto& im : ips) {
      std::string k = im->ip_pk();
      auto it = grouped.find(k);
      if (it == grouped.end()) {
        grouped[k] = im;
        order.push_back(k);
      } else {
        it->second = std::make_shared<PeerMatcher>(
            PeerMatcher{PeerKind::IP, combine_port_matchers(it->second->port, im->port), nullptr, nullptr, it->second->ip});
      }
    }
    ips.clear();
    for (auto& kv : grouped) ips.push_back(kv.second);
  }
  // simplifyPodMatchers :47-66
  {
    std::map<std::string, PeerP> grouped;
    for (auto& pm : pods) {
      std::string k = pm->pod_pk();
      auto it = grouped.find(k);
      if (it == grouped.end()) {
        grouped[k] = pm;
      } else {
        it->second = std::make_shared<PeerMatcher>(PeerMatcher{
            PeerKind::Pod, combine_port_matchers(it->second->port, pm->port), it->second->ns, it->second->pod, nullptr});
      }
    }
    pods.clear();
    for (auto& kv : grouped) pods.push_back(kv.second);
  }
  // simplifyIPsAndPodsIntoAlls :90-120
  if (pfaM) {
    std::vector<PeerP> nips, npods;
    for (auto& ip : ips) {
      auto r = subtract_port_matchers(ip->port, pfaM->port);
      if (!r.first) nips.push_back(std::make_shared<PeerMatcher>(PeerMatcher{PeerKind::IP, r.second, nullptr, nullptr, ip->ip}));
    }
    for (auto& pd : pods) {
      auto r = subtract_port_matchers(pd->port, pfaM->port);
      if (!r.first)
        npods.push_back(std::make_shared<PeerMatcher>(PeerMatcher{PeerKind::Pod, r.second, pd->ns, pd->pod, nullptr}));
    }
    ips = nips;
    pods = npods;
  }
  // GenerateSimplifiedMatchers :122-140
  std::vector<PeerP> out;
  if (matchesAll) {
    out_nil = false;
    return {kAllPeersPorts};
  }
  if (pfaM) out.push_back(pfaM);
  for (auto& p : ips) out.push_back(p);
  for (auto& p : pods) out.push_back(p);
  out_nil = out.empty();
  return out;
}

// ---------------------------------------------------------------- pkg/matcher/builder.go
static PMp build_port_matcher(const std::vector<NetpolPort>& npPorts) {  // :144-159
  auto m = std::make_shared<PortMatcher>();
  if (npPorts.empty()) {
    m->all = true;
    return m;
  }
  for (auto& p : npPorts) {
    // BuildSinglePortMatcher :161-187
    std::string protocol = p.protocol ? *p.protocol : "TCP";
    if (!p.endPort) {
      m->ports = goslice::append1(m->ports, std::make_shared<PortProtocolMatcher>(PortProtocolMatcher{p.port, protocol}));
      continue;
    }
    if (!p.port) go_panic("invalid port range: start port is nil");
    if (p.port->is_str) go_panic("invalid port range: start port is string");
    if (*p.endPort < p.port->ival) go_panic("invalid port range: end port < start port");
    m->ranges =
        goslice::append1(m->ranges, std::make_shared<PortRangeMatcher>(PortRangeMatcher{p.port->ival, *p.endPort, protocol}));
  }
  return m;
}

static std::vector<PeerP> build_peer_matcher(const std::string& policyNs, const NetpolRule& rule) {  // :79-113
  if (rule.ports.empty() && rule.peers.empty()) return {kAllPeersPorts};
  PMp port = build_port_matcher(rule.ports);
  if (rule.peers.empty())
    return {std::make_shared<PeerMatcher>(PeerMatcher{PeerKind::PortsForAll, port, nullptr, nullptr, nullptr})};
  std::vector<PeerP> out;
  for (auto& from : rule.peers) {
    // BuildIPBlockNamespacePodMatcher :115-142
    // An IPBlock peer yields (ip, nil, nil), so the :97-99 "IPBlock must be nil" guard can never
    // fire: selectors next to an ipBlock are silently ignored.
    if (from.ipBlock) {
      out.push_back(std::make_shared<PeerMatcher>(PeerMatcher{PeerKind::IP, port, nullptr, nullptr, from.ipBlock}));
      continue;
    }
    auto pod = std::make_shared<PodMatcher>();
    if (!from.podSelector || is_selector_empty(*from.podSelector)) {
      pod->all = true;
    } else {
      pod->all = false;
      pod->sel = *from.podSelector;
    }
    auto ns = std::make_shared<NsMatcher>();
    if (!from.namespaceSelector) {
      ns->kind = NsKind::Exact;
      ns->ns = policyNs;
    } else if (is_selector_empty(*from.namespaceSelector)) {
      ns->kind = NsKind::All;
    } else {
      ns->kind = NsKind::Label;
      ns->sel = *from.namespaceSelector;
    }
    // (the all-nil guard at :94-96 is unreachable: pod/ns matchers are always built)
    out.push_back(std::make_shared<PeerMatcher>(PeerMatcher{PeerKind::Pod, port, ns, pod, nullptr}));
  }
  return out;
}

struct Policy {
  std::map<std::string, TargetP> ingress, egress;  // Go map; iteration order irrelevant to verdicts

  void add_target(bool isIngress, TargetP t) {  // policy.go:51-66 (+ Target.Combine target.go:41-54)
    auto& dict = isIngress ? ingress : egress;
    const std::string& pk = t->pk();
    auto it = dict.find(pk);
    if (it != dict.end()) {
      auto c = std::make_shared<Target>();
      c->ns = it->second->ns;
      c->podSelector = it->second->podSelector;
      c->peers = it->second->peers;
      c->peers.insert(c->peers.end(), t->peers.begin(), t->peers.end());
      c->peers_nil = c->peers.empty() && it->second->peers_nil && t->peers_nil;
      c->sourceRules = it->second->sourceRules;
      c->sourceRules.insert(c->sourceRules.end(), t->sourceRules.begin(), t->sourceRules.end());
      it->second = c;
    } else {
      dict[pk] = t;
    }
  }

  // policy.go:138-174
  struct Dir {
    bool allowed;
  };
  bool direction_allowed(const Traffic& tr, bool isIngress) const {
    const TrafficPeer& target = isIngress ? tr.dst : tr.src;
    const TrafficPeer& peer = isIngress ? tr.src : tr.dst;
    if (!target.internal) return true;  // :151-153
    return allowed_given(targets_applying(target, isIngress), peer, tr);
  }
  // TargetsApplyingToPod :68-82 walks EVERY target of the direction
  std::vector<const Target*> targets_applying(const TrafficPeer& target, bool isIngress) const {
    const auto& dict = isIngress ? ingress : egress;
    std::vector<const Target*> matching;
    for (auto& kv : dict)
      if (kv.second->is_match(target.internal->ns, target.internal->podLabels)) matching.push_back(kv.second.get());
    return matching;
  }
  // :158-171 given the matching targets (every matching target's Allows runs, in order)
  static bool allowed_given(const std::vector<const Target*>& matching, const TrafficPeer& peer, const Traffic& tr) {
    if (matching.empty()) return true;  // :158-160
    size_t allowers = 0, deniers = 0;
    for (auto* t : matching) {
      if (t->allows(peer, tr.port, tr.portName, tr.protocol)) allowers++;
      else deniers++;
    }
    return allowers > 0 || deniers == 0;  // DirectionResult.IsAllowed :89-91
  }

  // IsIngressOrEgressAllowed with its DirectionResult lists (policy.go:138-174), as primary keys
  // (the map keys) in map order.
  void direction_result(const Traffic& tr, bool isIngress, std::vector<std::string>& allow,
                        std::vector<std::string>& deny) const {
    const TrafficPeer& target = isIngress ? tr.dst : tr.src;
    const TrafficPeer& peer = isIngress ? tr.src : tr.dst;
    if (!target.internal) return;
    const auto& dict = isIngress ? ingress : egress;
    std::vector<std::pair<std::string, const Target*>> matching;
    for (auto& kv : dict)
      if (kv.second->is_match(target.internal->ns, target.internal->podLabels)) matching.push_back({kv.first, kv.second.get()});
    for (auto& m : matching) (m.second->allows(peer, tr.port, tr.portName, tr.protocol) ? allow : deny).push_back(m.first);
  }
};

// builder.go:11-26 BuildNetworkPolicies + :35-61 BuildTarget
static std::shared_ptr<Policy> build_network_policies(bool doSimplify, const std::vector<NetworkPolicy>& netpols) {
  auto np = std::make_shared<Policy>();
  for (auto& pol : netpols) {
    if (pol.policyTypes.empty()) go_panic("invalid network policy: need at least 1 type");
    std::string ns = pol.ns.empty() ? "default" : pol.ns;
    TargetP ingress, egress;
    for (auto& pt : pol.policyTypes) {
      if (pt == "Ingress") {
        ingress = std::make_shared<Target>();
        ingress->ns = ns;
        ingress->podSelector = pol.podSelector;
        ingress->sourceRules = {pol.name};
        for (auto& r : pol.ingress) {
          auto ps = build_peer_matcher(ns, r);
          ingress->peers.insert(ingress->peers.end(), ps.begin(), ps.end());
        }
        ingress->peers_nil = ingress->peers.empty();
      } else if (pt == "Egress") {
        egress = std::make_shared<Target>();
        egress->ns = ns;
        egress->podSelector = pol.podSelector;
        egress->sourceRules = {pol.name};
        for (auto& r : pol.egress) {
          auto ps = build_peer_matcher(ns, r);
          egress->peers.insert(egress->peers.end(), ps.begin(), ps.end());
        }
        egress->peers_nil = egress->peers.empty();
      }
    }
    if (ingress) np->add_target(true, ingress);
    if (egress) np->add_target(false, egress);
  }
  if (doSimplify) {  // policy.go:176-183
    for (auto* dict : {&np->ingress, &np->egress})
      for (auto& kv : *dict) {
        bool nil;
        kv.second->peers = simplify(kv.second->peers, nil);
        kv.second->peers_nil = nil;
      }
  }
  return np;
}

// ---------------------------------------------------------------- json.Marshal(*matcher.Policy)
static std::string port_json(const PMp& p) {
  if (p->all) return "{\"Type\":\"all ports\"}";
  std::string o = "{\"PortRanges\":";
  if (p->ranges.len == 0 && !p->ranges.arr) o += "null";
  else {
    o += "[";
    for (size_t i = 0; i < p->ranges.len; i++) {
      auto& r = p->ranges[i];
      o += (i ? "," : "") + std::string("{\"From\":") + std::to_string(r->from) + ",\"Protocol\":" + go_quote(r->protocol) +
           ",\"To\":" + std::to_string(r->to) + ",\"Type\":\"port range\"}";
    }
    o += "]";
  }
  o += ",\"Ports\":";
  if (p->ports.len == 0 && !p->ports.arr) o += "null";
  else {
    o += "[";
    for (size_t i = 0; i < p->ports.len; i++) {
      auto& pp = p->ports[i];
      std::string port = !pp->port ? "null" : pp->port->is_str ? go_quote(pp->port->sval) : std::to_string(pp->port->ival);
      o += (i ? "," : "") + std::string("{\"Port\":") + port + ",\"Protocol\":" + go_quote(pp->protocol) + "}";
    }
    o += "]";
  }
  return o + ",\"Type\":\"specific ports\"}";
}

static std::string peer_json(const PeerP& p) {
  switch (p->kind) {
    case PeerKind::AllPeers: return "{\"Type\":\"all peers\"}";
    case PeerKind::PortsForAll: return "{\"Port\":" + port_json(p->port) + ",\"Type\":\"all peers for port\"}";
    case PeerKind::Pod:
      return "{\"Namespace\":" + p->ns->json() + ",\"Pod\":" + p->pod->json() + ",\"Port\":" + port_json(p->port) + "}";
    case PeerKind::IP: {
      std::string ex;
      if (p->ip->except_nil) ex = "null";
      else {
        ex = "[";
        for (size_t i = 0; i < p->ip->except.size(); i++) ex += (i ? "," : "") + go_quote(p->ip->except[i]);
        ex += "]";
      }
      return "{\"CIDR\":" + go_quote(p->ip->cidr) + ",\"Except\":" + ex + ",\"Port\":" + port_json(p->port) +
             ",\"Type\":\"IPBlock\"}";
    }
  }
  return "null";
}

static std::string policy_json(Policy& pol) {
  std::string o = "{";
  for (int dir = 0; dir < 2; dir++) {
    auto& dict = dir == 0 ? pol.ingress : pol.egress;
    o += dir == 0 ? "\"Ingress\":{" : ",\"Egress\":{";
    bool first = true;
    for (auto& kv : dict) {
      auto& t = kv.second;
      o += (first ? "" : ",") + go_quote(kv.first) + ":{\"Namespace\":" + go_quote(t->ns) +
           ",\"PodSelector\":" + selector_json(t->podSelector) + ",\"Peers\":";
      if (t->peers_nil && t->peers.empty()) o += "null";
      else {
        o += "[";
        for (size_t i = 0; i < t->peers.size(); i++) o += (i ? "," : "") + peer_json(t->peers[i]);
        o += "]";
      }
      o += ",\"SourceRules\":[";
      for (size_t i = 0; i < t->sourceRules.size(); i++)
        o += (i ? "," : "") + std::string("{\"metadata\":{\"name\":") + go_quote(t->sourceRules[i]) + "}}";
      o += "]}";
      first = false;
    }
    o += "}";
  }
  return o + "}";
}

// ---------------------------------------------------------------- pkg/connectivity/probe
struct Container {
  std::string name;
  int port = 0;
  std::string protocol, portName;
};
struct Pod {
  std::string ns, name, ip;
  LabelsP labels;
  std::vector<Container> containers;
};
struct Resources {
  std::map<std::string, LabelsP> namespaces;
  std::vector<Pod> pods;
  LabelsP ns_labels(const std::string& ns) const {  // r.Namespaces[ns] (nil when absent)
    auto it = namespaces.find(ns);
    return it == namespaces.end() ? nullptr : it->second;
  }
};

static LabelsP decode_labels(const Value* v) {
  if (!v || v->is_null()) return nullptr;
  auto l = std::make_shared<Labels>();
  for (auto& kv : v->obj) (*l)[kv.first] = kv.second->is_null() ? "" : kv.second->as_str();
  return l;
}

static Resources decode_resources(const Value& v) {
  Resources r;
  if (auto ns = v.get("Namespaces"); ns && ns->kind == Value::Object)
    for (auto& kv : ns->obj) r.namespaces[kv.first] = decode_labels(kv.second.get());
  if (auto pods = v.get("Pods"); pods && pods->kind == Value::Array)
    for (auto& p : pods->arr) {
      Pod pod;
      if (auto x = p->get("Namespace")) pod.ns = x->as_str();
      if (auto x = p->get("Name")) pod.name = x->as_str();
      if (auto x = p->get("IP"); x && !x->is_null()) pod.ip = x->as_str();
      pod.labels = decode_labels(p->get("Labels"));
      if (auto cs = p->get("Containers"); cs && cs->kind == Value::Array)
        for (auto& c : cs->arr) {
          Container ct;
          if (auto x = c->get("Name"); x && !x->is_null()) ct.name = x->as_str();
          if (auto x = c->get("Port"); x && !x->is_null()) ct.port = int(x->as_int());
          if (auto x = c->get("Protocol"); x && !x->is_null()) ct.protocol = x->as_str();
          if (auto x = c->get("PortName"); x && !x->is_null()) ct.portName = x->as_str();
          pod.containers.push_back(ct);
        }
      r.pods.push_back(pod);
    }
  return r;
}

// generator.ProbeConfig: AllAvailable, or PortProtocol{Port intstr, Protocol}
struct ProbeConfig {
  bool allAvailable = false;
  IntOrString port;
  std::string protocol;
};

static std::vector<ProbeConfig> decode_probes(const Value& v) {
  std::vector<ProbeConfig> out;
  for (auto& p : v.arr) {
    ProbeConfig c;
    if (auto a = p->get("AllAvailable"); a && a->kind == Value::Bool && a->b) {
      c.allAvailable = true;
    } else {
      const Value* pp = p->get("PortProtocol");
      const Value* src = pp ? pp : p.get();
      if (auto x = src->get("Port"); x && !x->is_null()) c.port = decode_intstr(*x);
      if (auto x = src->get("Protocol"); x && !x->is_null()) c.protocol = x->as_str();
    }
    out.push_back(c);
  }
  return out;
}

enum Status : uint8_t { ST_NONE = 0, ST_VALID = 1, ST_BAD_NAMED_PORT = 2, ST_BAD_PORT_PROTOCOL = 3 };

// A job's port/protocol triple as built by resources.go:284-334 / :336-364
struct JobDesc {
  uint8_t status = ST_NONE;
  int port = -1;
  std::string portName, protocol;
};

// slots per config: PortProtocol => 1; AllAvailable => max containers over pods
static std::vector<int> slot_offsets(const Resources& r, const std::vector<ProbeConfig>& cfgs, int& K) {
  std::vector<int> off;
  K = 0;
  int maxc = 0;
  for (auto& p : r.pods) maxc = std::max<int>(maxc, int(p.containers.size()));
  for (auto& c : cfgs) {
    off.push_back(K);
    K += c.allAvailable ? maxc : 1;
  }
  return off;
}

// Job descriptor for (dst pod, config, index): resources.go:284-334 (PortProtocol, port resolved on
// the DESTINATION pod: pod.go:132-148) and :336-364 (AllAvailable, raw container protocol)
static JobDesc job_desc(const Pod& podTo, const ProbeConfig& c, int idx) {
  JobDesc j;
  if (c.allAvailable) {
    if (idx >= int(podTo.containers.size())) return j;  // no job
    auto& ct = podTo.containers[idx];
    j.status = ST_VALID;
    j.port = ct.port;
    j.portName = ct.portName;
    j.protocol = ct.protocol;
    return j;
  }
  j.protocol = c.protocol;
  j.port = -1;
  if (c.port.is_str) {
    j.portName = c.port.sval;
    for (auto& ct : podTo.containers)  // ResolveNamedPort pod.go:132-139
      if (ct.portName == c.port.sval) {
        j.port = ct.port;
        j.status = ST_VALID;
        return j;
      }
    j.status = ST_BAD_NAMED_PORT;
    return j;
  }
  j.port = c.port.ival;
  for (auto& ct : podTo.containers)  // ResolveNumberedPort pod.go:141-148 (protocol ignored)
    if (ct.port == c.port.ival) {
      j.portName = ct.portName;
      j.status = ST_VALID;
      return j;
    }
  j.status = ST_BAD_PORT_PROTOCOL;
  return j;
}

// Job.Traffic job.go:81-103
static Traffic job_traffic(const Resources& r, const Pod& from, const Pod& to, const JobDesc& j) {
  Traffic t;
  t.src.internal = std::make_shared<InternalPeer>(InternalPeer{from.labels, r.ns_labels(from.ns), from.ns});
  t.src.ip = from.ip;
  t.dst.internal = std::make_shared<InternalPeer>(InternalPeer{to.labels, r.ns_labels(to.ns), to.ns});
  t.dst.ip = to.ip;
  t.port = j.port;
  t.portName = j.portName;
  t.protocol = j.protocol;
  return t;
}

struct Handle {
  std::shared_ptr<Policy> policy;
  Resources res;
};

// NewTableFromJobResults (table.go:38-48) over runProbe's result list (jobrunner.go:33-58): the
// valid jobs in RunJobs order (resources.go:286-287 podFrom, podTo[, container]), then every
// BadPortProtocol job, then every BadNamedPort job, each added to the Item of (FromKey, ToKey) —
// PodString ns/name, so pods sharing a name share Items — under JobResult.Key() = Protocol/ResolvedPort
// (job.go:23-25); Item.AddJobResult (table.go:16-22) rejects a key the Item already holds and
// utils.DoOrDie (utils.go:10-14) ends the program.  Returns "" or the error text.  The reference's
// text continues with the whole Job as %+v (its ToHost depends on the probe mode) and the stack
// pkg/errors prints; here the job is named by FromKey, ToKey and ToContainer.
static std::string table_build_error(const Resources& r, const ProbeConfig& c, int nslot) {
  const auto& pods = r.pods;
  const size_t P = pods.size();
  std::unordered_map<std::string, uint64_t> pod_id, key_id;
  std::vector<uint64_t> pid(P);
  for (size_t p = 0; p < P; p++) pid[p] = pod_id.emplace(pods[p].ns + "/" + pods[p].name, pod_id.size()).first->second;
  std::unordered_set<std::string> held;  // (FromKey id, ToKey id, key) of every added result
  auto add = [&](size_t s, size_t d, const JobDesc& j, const std::string& to_cont) -> std::string {
    const std::string key = j.protocol + "/" + std::to_string(j.port);
    std::string item = std::to_string(pid[s]) + "|" + std::to_string(pid[d]) + "|" + key;
    if (held.insert(item).second) return "";
    return "unable to add job result: duplicate key " + key + " (job {FromKey:" + pods[s].ns + "/" + pods[s].name +
           " ToKey:" + pods[d].ns + "/" + pods[d].name + " ToContainer:" + to_cont + "})";
  };
  for (int pass = 0; pass < 3; pass++) {  // valid jobs, BadPortProtocol, BadNamedPort
    const int want = pass == 0 ? ST_VALID : pass == 1 ? ST_BAD_PORT_PROTOCOL : ST_BAD_NAMED_PORT;
    for (size_t s = 0; s < P; s++)
      for (size_t d = 0; d < P; d++)
        for (int i = 0; i < nslot; i++) {
          JobDesc j = job_desc(pods[d], c, i);
          if (j.status != want) continue;
          std::string e = add(s, d, j, c.allAvailable ? pods[d].containers[i].name : "");
          if (!e.empty()) return e;
        }
  }
  return "";
}

static void set_err(char* err, size_t cap, const std::string& m) {
  if (!err || !cap) return;
  size_t n = std::min(cap - 1, m.size());
  memcpy(err, m.data(), n);
  err[n] = 0;
}

static std::vector<NetworkPolicy> decode_netpols(const std::string& json) {
  VP v = ojson::parse(json);
  std::vector<NetworkPolicy> out;
  if (v->kind == Value::Array) {
    for (auto& p : v->arr) out.push_back(decode_netpol(*p));
  } else if (v->kind == Value::Object) {
    if (auto items = v->get("items"); items && items->kind == Value::Array) {
      for (auto& p : items->arr) out.push_back(decode_netpol(*p));
    } else {
      out.push_back(decode_netpol(*v));
    }
  }
  return out;
}

}  // namespace orc

using namespace orc;

extern "C" {

void* orc_new(const char* policies_json, int simplify, const char* resources_json, char* err, size_t errcap) {
  try {
    auto h = new Handle();
    h->policy = build_network_policies(simplify != 0, decode_netpols(policies_json ? policies_json : "[]"));
    if (resources_json && *resources_json) h->res = decode_resources(*ojson::parse(resources_json));
    return h;
  } catch (GoPanic& p) {
    set_err(err, errcap, p.msg);
  } catch (std::exception& e) {
    set_err(err, errcap, e.what());
  }
  return nullptr;
}

void orc_free(void* h) { delete static_cast<Handle*>(h); }

int orc_policy_json(void* hv, char* buf, size_t cap) {
  auto* h = static_cast<Handle*>(hv);
  std::string s = policy_json(*h->policy);
  if (buf && cap > s.size()) {
    memcpy(buf, s.data(), s.size());
    buf[s.size()] = 0;
  }
  return int(s.size());
}

int orc_probe_shape(void* hv, const char* probes_json, int* P, int* K, char* err, size_t errcap) {
  try {
    auto* h = static_cast<Handle*>(hv);
    auto cfgs = decode_probes(*ojson::parse(probes_json));
    slot_offsets(h->res, cfgs, *K);
    *P = int(h->res.pods.size());
    return 0;
  } catch (std::exception& e) {
    set_err(err, errcap, e.what());
    return -1;
  }
}

// Full truth table, per cell, in the reference's job order (for each config: for podFrom, for
// podTo, for job).  Layout (shared with the product): status[d*K+k];
// in_plane[(d*K+k)*W + s/64] bit s%64 (ingress verdict of s->d, keyed by the ingress TARGET d);
// eg_plane[(s*K+k)*W + d/64] bit d%64 (egress verdict of s->d, keyed by the egress TARGET s).
// Returns 0 OK, 1 on a Go panic (message in err; *panic_cell = s*P*K + d*K + k of the first
// panicking job in job order), -1 on a decode error.
int orc_probe_run(void* hv, const char* probes_json, uint8_t* status, uint64_t* in_plane, uint64_t* eg_plane,
                  long long* panic_cell, char* err, size_t errcap) {
  auto* h = static_cast<Handle*>(hv);
  try {
    auto cfgs = decode_probes(*ojson::parse(probes_json));
    int K;
    auto off = slot_offsets(h->res, cfgs, K);
    const auto& pods = h->res.pods;
    size_t P = pods.size(), W = (P + 63) / 64;
    memset(status, 0, P * K);
    memset(in_plane, 0, P * K * W * 8);
    memset(eg_plane, 0, P * K * W * 8);
    for (size_t c = 0; c < cfgs.size(); c++) {
      int nslot = (c + 1 < cfgs.size() ? off[c + 1] : K) - off[c];
      for (size_t d = 0; d < P; d++)
        for (int i = 0; i < nslot; i++) status[d * K + off[c] + i] = job_desc(pods[d], cfgs[c], i).status;
    }
    for (size_t c = 0; c < cfgs.size(); c++) {
      int nslot = (c + 1 < cfgs.size() ? off[c + 1] : K) - off[c];
      // GetJobsForProbeConfig (resources.go:284-364) builds every job of this config first, and each
      // job reads podFrom.Containers[0].Name (:296, :349): a container-less source pod panics there
      for (size_t s = 0; s < P; s++)
        for (size_t d = 0; d < P; d++) {
          const bool builds_job = !cfgs[c].allAvailable || !pods[d].containers.empty();
          if (builds_job && pods[s].containers.empty()) {
            set_err(err, errcap, "runtime error: index out of range [0] with length 0");
            if (panic_cell) *panic_cell = -1;
            return 1;
          }
        }
      for (size_t s = 0; s < P; s++)
        for (size_t d = 0; d < P; d++)
          for (int i = 0; i < nslot; i++) {
            JobDesc j = job_desc(pods[d], cfgs[c], i);
            if (j.status != ST_VALID) continue;
            int k = off[c] + i;
            Traffic t = job_traffic(h->res, pods[s], pods[d], j);
            try {
              bool in = h->policy->direction_allowed(t, true);
              bool eg = h->policy->direction_allowed(t, false);
              if (in) in_plane[(d * K + k) * W + s / 64] |= 1ull << (s % 64);
              if (eg) eg_plane[(s * K + k) * W + d / 64] |= 1ull << (d % 64);
            } catch (GoPanic& p) {
              set_err(err, errcap, p.msg);
              if (panic_cell) *panic_cell = (long long)((s * P + d) * K + k);
              return 1;
            }
          }
      // the config's table is built after its jobs ran (jobrunner.go:29-31)
      std::string dup = table_build_error(h->res, cfgs[c], nslot);
      if (!dup.empty()) {
        set_err(err, errcap, dup);
        if (panic_cell) *panic_cell = -2;
        return 1;
      }
    }
    return 0;
  } catch (std::exception& e) {
    set_err(err, errcap, e.what());
    return -1;
  }
}

// Sampled cells (s[i], d[i], k[i]) => out[i] = status | ingress<<4 | egress<<5 | panic<<6.
int orc_probe_cells(void* hv, const char* probes_json, const int32_t* ss, const int32_t* dd, const int32_t* kk, int n,
                    uint8_t* out, char* err, size_t errcap) {
  auto* h = static_cast<Handle*>(hv);
  try {
    auto cfgs = decode_probes(*ojson::parse(probes_json));
    int K;
    auto off = slot_offsets(h->res, cfgs, K);
    const auto& pods = h->res.pods;
    for (int i = 0; i < n; i++) {
      int k = kk[i];
      size_t c = 0;
      while (c + 1 < cfgs.size() && off[c + 1] <= k) c++;
      JobDesc j = job_desc(pods[dd[i]], cfgs[c], k - off[c]);
      uint8_t o = j.status;
      if (j.status == ST_VALID) {
        Traffic t = job_traffic(h->res, pods[ss[i]], pods[dd[i]], j);
        try {
          if (h->policy->direction_allowed(t, true)) o |= 1 << 4;
          if (h->policy->direction_allowed(t, false)) o |= 1 << 5;
        } catch (GoPanic&) {
          o |= 1 << 6;
        }
      }
      out[i] = o;
    }
    return 0;
  } catch (std::exception& e) {
    set_err(err, errcap, e.what());
    return -1;
  }
}

// Same as orc_probe_cells with the cells split statically over `threads` std::threads (the
// multi-core CPU baseline of SURVEY §8d).  The per-cell walk is read-only on the Policy, so the
// threads share it; each thread decodes the probe configs itself.
int orc_probe_cells_mt(void* hv, const char* probes_json, const int32_t* ss, const int32_t* dd, const int32_t* kk, int n,
                       uint8_t* out, int threads, char* err, size_t errcap) {
  if (threads <= 1) return orc_probe_cells(hv, probes_json, ss, dd, kk, n, out, err, errcap);
  std::vector<std::thread> pool;
  std::vector<int> rc(threads, 0);
  std::vector<std::string> msg(threads);
  for (int t = 0; t < threads; t++) {
    int lo = int(int64_t(n) * t / threads), hi = int(int64_t(n) * (t + 1) / threads);
    pool.emplace_back([&, t, lo, hi] {
      char e[1024] = {0};
      rc[t] = orc_probe_cells(hv, probes_json, ss + lo, dd + lo, kk + lo, hi - lo, out + lo, e, sizeof(e));
      msg[t] = e;
    });
  }
  for (auto& th : pool) th.join();
  for (int t = 0; t < threads; t++)
    if (rc[t] != 0) {
      set_err(err, errcap, msg[t]);
      return rc[t];
    }
  return 0;
}

// analyze --mode query-traffic (analyze.go:209-225): JSON list of matcher.Traffic.
// out[i] = ingress | egress<<1 | panic<<2
// One plane row: dir 0 = ingress row of destination `pod` (bit s over every source), dir 1 = egress
// row of source `pod` (bit d over every destination), slot k; row[W] as in the planes.  The same
// per-cell IsIngressOrEgressAllowed walk as orc_probe_run, with the row's fixed target pod's
// TargetsApplyingToPod list computed once (it depends on that pod alone, policy.go:68-82).  Cells
// without a VALID job are 0.  `threads` split the row's cells.  Returns 0, 1 on a Go panic.
int orc_probe_row(void* hv, const char* probes_json, int dir, int pod, int k, uint64_t* row, int threads, char* err,
                  size_t errcap) {
  auto* h = static_cast<Handle*>(hv);
  try {
    auto cfgs = decode_probes(*ojson::parse(probes_json));
    int K;
    auto off = slot_offsets(h->res, cfgs, K);
    const auto& pods = h->res.pods;
    const int P = int(pods.size()), W = (P + 63) / 64;
    if (pod < 0 || pod >= P || k < 0 || k >= K) {
      set_err(err, errcap, "row out of range");
      return -1;
    }
    size_t c = 0;
    while (c + 1 < cfgs.size() && off[c + 1] <= k) c++;
    memset(row, 0, size_t(W) * 8);
    const bool ingress = dir == 0;
    // the fixed pod is the target of this direction (ingress: destination, egress: source)
    TrafficPeer tp;
    tp.internal = std::make_shared<InternalPeer>(InternalPeer{pods[pod].labels, h->res.ns_labels(pods[pod].ns), pods[pod].ns});
    tp.ip = pods[pod].ip;
    const auto matching = h->policy->targets_applying(tp, ingress);
    const JobDesc jd = ingress ? job_desc(pods[pod], cfgs[c], k - int(off[c])) : JobDesc{};
    threads = std::max(1, std::min(threads, 64));
    std::vector<std::thread> pool;
    std::vector<int> rc(threads, 0);
    std::vector<std::string> msg(threads);
    for (int t = 0; t < threads; t++) {
      // whole 64-pod words per thread: no two threads write one word
      const int w0 = int(int64_t(W) * t / threads), w1 = int(int64_t(W) * (t + 1) / threads);
      pool.emplace_back([&, t, w0, w1] {
        try {
          for (int q = w0 * 64; q < std::min(P, w1 * 64); q++) {
            const int s = ingress ? q : pod, d = ingress ? pod : q;
            const JobDesc j = ingress ? jd : job_desc(pods[d], cfgs[c], k - int(off[c]));
            if (j.status != ST_VALID) continue;
            const Traffic tr = job_traffic(h->res, pods[s], pods[d], j);
            if (Policy::allowed_given(matching, ingress ? tr.src : tr.dst, tr)) row[q / 64] |= 1ull << (q % 64);
          }
        } catch (GoPanic& p) {
          rc[t] = 1;
          msg[t] = p.msg;
        }
      });
    }
    for (auto& th : pool) th.join();
    for (int t = 0; t < threads; t++)
      if (rc[t]) {
        set_err(err, errcap, msg[t]);
        return 1;
      }
    return 0;
  } catch (std::exception& e) {
    set_err(err, errcap, e.what());
    return -1;
  }
}

static std::vector<Traffic> decode_traffics(const char* traffic_json) {
  VP v = ojson::parse(traffic_json);
  auto peer = [](const Value* p) {
    TrafficPeer tp;
    if (!p || p->is_null()) return tp;
    if (auto ip = p->get("IP"); ip && !ip->is_null()) tp.ip = ip->as_str();
    if (auto in = p->get("Internal"); in && !in->is_null()) {
      tp.internal = std::make_shared<InternalPeer>();
      tp.internal->podLabels = decode_labels(in->get("PodLabels"));
      tp.internal->nsLabels = decode_labels(in->get("NamespaceLabels"));
      if (auto ns = in->get("Namespace"); ns && !ns->is_null()) tp.internal->ns = ns->as_str();
    }
    return tp;
  };
  std::vector<Traffic> out;
  for (auto& t : v->arr) {
    Traffic tr;
    tr.src = peer(t->get("Source"));
    tr.dst = peer(t->get("Destination"));
    if (auto x = t->get("ResolvedPort"); x && !x->is_null()) tr.port = int(x->as_int());
    if (auto x = t->get("ResolvedPortName"); x && !x->is_null()) tr.portName = x->as_str();
    if (auto x = t->get("Protocol"); x && !x->is_null()) tr.protocol = x->as_str();
    out.push_back(std::move(tr));
  }
  return out;
}

// AllowedResult lists per traffic as JSON (same shape as cyc_query_traffic_targets):
// [{"Ingress": {"AllowingTargets": [pk..], "DenyingTargets": [..], "IsAllowed": b}, "Egress": {..},
//   "IsAllowed": b}, ..].  Returns 0, 1 on a Go panic (message in err), -1 on bad input / small buffer.
int orc_query_traffic_targets(void* hv, const char* traffic_json, char* out, size_t cap, char* err, size_t errcap) {
  auto* h = static_cast<Handle*>(hv);
  try {
    std::string o = "[";
    bool first = true;
    for (auto& tr : decode_traffics(traffic_json)) {
      o += first ? "{" : ",{";
      first = false;
      bool all = true;
      for (int d = 0; d < 2; d++) {
        std::vector<std::string> allow, deny;
        try {
          h->policy->direction_result(tr, d == 0, allow, deny);
        } catch (GoPanic& p) {
          set_err(err, errcap, p.msg);
          return 1;
        }
        bool ok = !allow.empty() || deny.empty();
        all = all && ok;
        o += d ? ",\"Egress\":{" : "\"Ingress\":{";
        for (int a = 0; a < 2; a++) {
          o += a == 0 ? "\"AllowingTargets\":[" : ",\"DenyingTargets\":[";
          auto& L = a == 0 ? allow : deny;
          for (size_t i = 0; i < L.size(); i++) {
            if (i) o += ',';
            o += ojson::go_quote(L[i]);
          }
          o += ']';
        }
        o += std::string(",\"IsAllowed\":") + (ok ? "true" : "false") + "}";
      }
      o += std::string(",\"IsAllowed\":") + (all ? "true" : "false") + "}";
    }
    o += "]";
    if (o.size() + 1 > cap) {
      set_err(err, errcap, "buffer too small: need " + std::to_string(o.size() + 1));
      return -1;
    }
    memcpy(out, o.c_str(), o.size() + 1);
    return 0;
  } catch (std::exception& e) {
    set_err(err, errcap, e.what());
    return -1;
  }
}

// analyze --mode query-target (analyze.go:163-204): per QueryTargetPod {Namespace, Labels},
// TargetsApplyingToPod per direction as primary keys: [{"Ingress": [..], "Egress": [..]}, ..].
int orc_query_targets(void* hv, const char* pods_json, char* out, size_t cap, char* err, size_t errcap) {
  auto* h = static_cast<Handle*>(hv);
  try {
    VP v = ojson::parse(pods_json);
    std::string o = "[";
    bool first = true;
    for (auto& p : v->arr) {
      std::string ns;
      if (auto x = p->get("Namespace"); x && !x->is_null()) ns = x->as_str();
      auto labels = decode_labels(p->get("Labels"));
      o += first ? "{" : ",{";
      first = false;
      for (int d = 0; d < 2; d++) {
        o += d ? "],\"Egress\":[" : "\"Ingress\":[";
        bool f2 = true;
        try {
          for (auto& kv : d == 0 ? h->policy->ingress : h->policy->egress)  // policy.go:68-82
            if (kv.second->is_match(ns, labels)) {
              o += f2 ? "" : ",";
              f2 = false;
              o += ojson::go_quote(kv.first);
            }
        } catch (GoPanic& e) {
          set_err(err, errcap, e.msg);
          return 1;
        }
      }
      o += "]}";
    }
    o += "]";
    if (o.size() + 1 > cap) {
      set_err(err, errcap, "buffer too small: need " + std::to_string(o.size() + 1));
      return -1;
    }
    memcpy(out, o.c_str(), o.size() + 1);
    return 0;
  } catch (std::exception& e) {
    set_err(err, errcap, e.what());
    return -1;
  }
}

int orc_query_traffic(void* hv, const char* traffic_json, uint8_t* out, int n, char* err, size_t errcap) {
  auto* h = static_cast<Handle*>(hv);
  try {
    VP v = ojson::parse(traffic_json);
    auto peer = [](const Value* p) {
      TrafficPeer tp;
      if (!p || p->is_null()) return tp;
      if (auto ip = p->get("IP"); ip && !ip->is_null()) tp.ip = ip->as_str();
      if (auto in = p->get("Internal"); in && !in->is_null()) {
        tp.internal = std::make_shared<InternalPeer>();
        tp.internal->podLabels = decode_labels(in->get("PodLabels"));
        tp.internal->nsLabels = decode_labels(in->get("NamespaceLabels"));
        if (auto ns = in->get("Namespace"); ns && !ns->is_null()) tp.internal->ns = ns->as_str();
      }
      return tp;
    };
    int i = 0;
    for (auto& t : v->arr) {
      if (i >= n) break;
      Traffic tr;
      tr.src = peer(t->get("Source"));
      tr.dst = peer(t->get("Destination"));
      if (auto x = t->get("ResolvedPort"); x && !x->is_null()) tr.port = int(x->as_int());
      if (auto x = t->get("ResolvedPortName"); x && !x->is_null()) tr.portName = x->as_str();
      if (auto x = t->get("Protocol"); x && !x->is_null()) tr.protocol = x->as_str();
      uint8_t o = 0;
      try {
        if (h->policy->direction_allowed(tr, true)) o |= 1;
        if (h->policy->direction_allowed(tr, false)) o |= 2;
      } catch (GoPanic& p) {
        o = 4;
        set_err(err, errcap, p.msg);
      }
      out[i++] = o;
    }
    return i;
  } catch (std::exception& e) {
    set_err(err, errcap, e.what());
    return -1;
  }
}

// KAT helpers: pkg/kube/ipaddress.go, labelselector.go.  Return 1/0, or -1 on error/panic.
int orc_ip_in_cidr(const char* ip, const char* cidr) {
  IPResult r = is_ip_in_cidr(ip, cidr);
  return r.ok ? (r.member ? 1 : 0) : -1;
}

int orc_ipblock_match(const char* ip, const char* cidr, const char* const* except, int n_except) {
  IPBlock b;
  b.cidr = cidr;
  for (int i = 0; i < n_except; i++) b.except.push_back(except[i]);
  IPResult r = is_ip_match_block(ip, b);
  return r.ok ? (r.member ? 1 : 0) : -1;
}

int orc_selector_match(const char* labels_json, const char* selector_json) {
  try {
    VP l = ojson::parse(labels_json);
    VP s = ojson::parse(selector_json);
    return is_labels_match(decode_labels(l.get()), decode_selector(*s)) ? 1 : 0;
  } catch (GoPanic&) {
    return -1;
  } catch (std::exception&) {
    return -2;
  }
}

// MakeIPV4CIDR ipaddress.go:42-46
int orc_make_ipv4_cidr(const char* ip, int bits, char* buf, size_t cap) {
  gonet::IP p = gonet::ParseIP(ip);
  gonet::IP m = gonet::CIDRMask(bits, 32);
  gonet::IP x = gonet::Mask(p, m);
  std::string s = (x.size() == 4 ? gonet::IPv4String(x) : std::string("<nil>")) + "/" + std::to_string(bits);
  set_err(buf, cap, s);
  return 0;
}

}  // extern "C"
