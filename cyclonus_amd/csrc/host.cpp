// host.cpp — policy compiler, probe model and table flattening (see host.hpp).
#include "host.hpp"

#include <algorithm>
#include <cstring>
#include <functional>
#include <set>
#include <stdexcept>

#include "cyclonus_hip.h"

namespace cyc {

using json::Node;
using json::quote;

// ============================================================================ selectors
static std::string req_json(const Requirement& r) {
  std::string o = "{\"key\":" + quote(r.key) + ",\"operator\":" + quote(r.op);
  if (!r.values.empty()) {
    o += ",\"values\":[";
    for (size_t i = 0; i < r.values.size(); i++) o += (i ? "," : "") + quote(r.values[i]);
    o += "]";
  }
  return o + "}";
}

std::string Selector::serialize() const {
  // json.Marshal([]interface{}{"MatchLabels", keyVals, "MatchExpression", MatchExpressions})
  std::string o = "[\"MatchLabels\",";
  if (labels.empty()) o += "null";
  else {
    o += "[";
    bool first = true;
    for (auto& kv : labels) {
      o += (first ? "" : ",") + quote(kv.first + ": " + kv.second);
      first = false;
    }
    o += "]";
  }
  o += ",\"MatchExpression\",";
  if (exprs.empty()) o += "null";
  else {
    o += "[";
    for (size_t i = 0; i < exprs.size(); i++) o += (i ? "," : "") + req_json(exprs[i]);
    o += "]";
  }
  return o + "]";
}

std::string Selector::to_json() const {
  std::string o = "{";
  if (!labels.empty()) {
    o += "\"matchLabels\":{";
    bool first = true;
    for (auto& kv : labels) {
      o += (first ? "" : ",") + quote(kv.first) + ":" + quote(kv.second);
      first = false;
    }
    o += "}";
  }
  if (!exprs.empty()) {
    o += labels.empty() ? "" : ",";
    o += "\"matchExpressions\":[";
    for (size_t i = 0; i < exprs.size(); i++) o += (i ? "," : "") + req_json(exprs[i]);
    o += "]";
  }
  return o + "}";
}

static Selector decode_selector(const Node& n) {
  Selector s;
  if (auto ml = n.val("matchLabels"); ml && ml->is_obj())
    for (auto& kv : ml->o) s.labels[kv.first] = kv.second.null() ? "" : kv.second.str();
  if (auto me = n.val("matchExpressions"); me && me->is_arr())
    for (auto& e : me->a) {
      Requirement r;
      if (auto k = e.sval("key")) r.key = k->str();
      if (auto op = e.sval("operator")) r.op = op->str();
      if (auto vs = e.val("values"); vs && vs->is_arr())
        for (auto& v : vs->a) r.values.push_back(v.str());
      s.exprs.push_back(std::move(r));
    }
  return s;
}

static IntStr decode_intstr(const Node& n) {  // intstr.IntOrString.UnmarshalJSON
  IntStr v;
  if (n.t == Node::Str) {
    v.is_str = true;
    v.s = n.s;
  } else {
    v.i = int32_t(n.i64());
  }
  return v;
}

// ============================================================================ peer keys
static std::string ns_pk(const Peer& p) {  // podpeermatcher.go:135,150,166
  switch (p.ns_kind) {
    case NS_EXACT: return "{\"type\": \"exact-namespace\", \"namespace\": \"" + p.ns + "\"}";
    case NS_ALL: return "{\"type\": \"all-namespaces\"}";
    default: return "{\"type\": \"label-selector\", \"selector\": \"" + p.ns_sel.serialize() + "\"}";
  }
}
std::string Peer::pod_pk() const {
  std::string pod = pod_all ? "{\"type\": \"all-pods\"}"
                            : "{\"type\": \"label-selector\", \"selector\": \"" + pod_sel.serialize() + "\"}";
  return ns_pk(*this) + "---" + pod;
}
std::string Peer::ip_pk() const {
  std::vector<std::string> ex = except;
  std::sort(ex.begin(), ex.end());
  std::string j;
  for (size_t i = 0; i < ex.size(); i++) j += (i ? ", " : "") + ex[i];
  return cidr + ": [" + j + "]";
}

// ============================================================================ Go slice model
// runtime/slice.go growslice (Go 1.16) for 8-byte elements + runtime/msize.go roundupsize.
static uint32_t go_roundup_cap(uint64_t elems) {
  static const uint32_t classes[] = {8,    16,   24,   32,   48,   64,   80,   96,   112,  128,  144,  160,
                                     176,  192,  208,  224,  240,  256,  288,  320,  352,  384,  416,  448,
                                     480,  512,  576,  640,  704,  768,  896,  1024, 1152, 1280, 1408, 1536,
                                     1792, 2048, 2304, 2688, 3072, 3200, 3456, 4096, 4864, 5376, 6144, 6528,
                                     6784, 6912, 8192, 9472, 9728, 10240, 10880, 12288, 13568, 14336, 16384,
                                     18432, 19072, 20480, 21760, 24576, 27264, 28672, 32768};
  uint64_t bytes = elems * 8;
  for (uint32_t c : classes)
    if (c >= bytes) return c / 8;
  return uint32_t(((bytes + 8191) / 8192 * 8192) / 8);
}
static uint32_t go_grow(uint32_t old_len, uint32_t old_cap, uint32_t need) {
  uint64_t nc = old_cap, dbl = uint64_t(old_cap) * 2;
  if (need > dbl) nc = need;
  else if (old_len < 1024) nc = dbl;
  else {
    while (nc > 0 && nc < need) nc += nc / 4;
    if (nc == 0) nc = need;
  }
  return go_roundup_cap(nc);
}

struct Compiler {
  PolicyIR ir;

  // append(s, xs...) on []*PortRangeMatcher
  RangeSlice append_ranges(RangeSlice s, const std::vector<PortRange>& xs) {
    if (xs.empty()) return s;
    uint32_t need = s.len + uint32_t(xs.size());
    RangeSlice r = s;
    if (s.arr < 0 || need > s.cap) {
      uint32_t nc = go_grow(s.len, s.arr < 0 ? 0 : s.cap, need);
      std::vector<PortRange> arr(nc);
      for (uint32_t i = 0; i < s.len; i++) arr[i] = ir.range_arrays[s.arr][i];
      ir.range_arrays.push_back(std::move(arr));
      r.arr = int(ir.range_arrays.size() - 1);
      r.cap = nc;
    }
    for (size_t i = 0; i < xs.size(); i++) ir.range_arrays[r.arr][s.len + i] = xs[i];  // may alias s's array
    r.len = need;
    return r;
  }

  int new_pm(PortMatcher m) {
    ir.pm.push_back(std::move(m));
    return int(ir.pm.size() - 1);
  }

  // builder.go:144-187 BuildPortMatcher / BuildSinglePortMatcher
  int build_port_matcher(const Node* ports) {
    PortMatcher m;
    if (!ports || !ports->is_arr() || ports->a.empty()) {
      m.all = true;
      return new_pm(m);
    }
    for (auto& p : ports->a) {
      std::string proto = "TCP";
      if (auto pr = p.val("protocol")) proto = pr->str();
      const Node* port = p.val("port");
      const Node* end = p.val("endPort");
      if (!end) {
        PortEntry e;
        e.proto = proto;
        if (port) {
          e.has_port = true;
          e.port = decode_intstr(*port);
        }
        m.ports.push_back(e);
        m.ports_nil = false;
        continue;
      }
      if (!port) throw Panic{CYC_ERR_INVALID_POLICY, "invalid port range: start port is nil"};
      IntStr start = decode_intstr(*port);
      if (start.is_str) throw Panic{CYC_ERR_INVALID_POLICY, "invalid port range: start port is string"};
      int32_t endp = int32_t(end->i64());
      if (endp < start.i) throw Panic{CYC_ERR_INVALID_POLICY, "invalid port range: end port < start port"};
      m.ranges = append_ranges(m.ranges, {PortRange{start.i, endp, proto}});
    }
    return new_pm(m);
  }

  // builder.go:79-142 BuildPeerMatcher / BuildIPBlockNamespacePodMatcher
  void build_peers(const std::string& policy_ns, const Node& rule, const char* peers_key, std::vector<Peer>& out) {
    const Node* ports = rule.val("ports");
    const Node* peers = rule.val(peers_key);
    bool no_ports = !ports || !ports->is_arr() || ports->a.empty();
    bool no_peers = !peers || !peers->is_arr() || peers->a.empty();
    if (no_ports && no_peers) {
      out.push_back(Peer{});  // AllPeersPorts
      return;
    }
    int port = build_port_matcher(ports);
    if (no_peers) {
      Peer p;
      p.kind = PK_PORTS;
      p.port = port;
      out.push_back(p);
      return;
    }
    for (auto& from : peers->a) {
      Peer p;
      p.port = port;
      if (auto ib = from.val("ipBlock")) {  // selectors next to an ipBlock are ignored (:116-121)
        p.kind = PK_IP;
        if (auto c = ib->sval("cidr")) p.cidr = c->str();
        if (auto ex = ib->val("except"); ex && ex->is_arr()) {
          p.except_nil = false;
          for (auto& e : ex->a) p.except.push_back(e.str());
        }
        out.push_back(p);
        continue;
      }
      p.kind = PK_POD;
      const Node* ps = from.val("podSelector");
      if (ps) {
        p.pod_sel = decode_selector(*ps);
        p.pod_all = p.pod_sel.empty();
      }
      const Node* nss = from.val("namespaceSelector");
      if (!nss) {
        p.ns_kind = NS_EXACT;
        p.ns = policy_ns;
      } else {
        p.ns_sel = decode_selector(*nss);
        p.ns_kind = p.ns_sel.empty() ? NS_ALL : NS_LABEL;
      }
      out.push_back(p);
    }
  }

  // ---------------------------------------------------------------- simplifier.go
  int combine(int a, int b) {  // CombinePortMatchers :142-159
    if (ir.pm[a].all) return a;
    if (ir.pm[b].all) return b;
    // SpecificPortMatcher.Combine portmatcher.go:102-131, quirks Q1 + Q2 included
    std::vector<PortEntry> pps = ir.pm[a].ports;
    std::vector<PortEntry> other = ir.pm[b].ports;
    for (auto& op : other) {
      size_t n = pps.size();  // range over the slice header taken before the loop
      for (size_t i = 0; i < n; i++) {
        if (pps[i].equals(op)) break;
        pps.push_back(op);
      }
    }
    std::stable_sort(pps.begin(), pps.end(), [](const PortEntry& x, const PortEntry& y) {
      auto less = [](const PortEntry& p, const PortEntry& q) {  // isPortLessThan: nil < string < int
        if (!p.has_port) return q.has_port;
        if (!q.has_port) return false;
        if (!p.port.is_str) return !q.port.is_str && p.port.i < q.port.i;
        return !q.port.is_str || p.port.s < q.port.s;
      };
      if (less(x, y)) return true;
      if (less(y, x)) return false;
      return x.proto < y.proto;
    });
    PortMatcher m;
    m.ports = std::move(pps);
    m.ports_nil = false;
    RangeSlice ra = ir.pm[a].ranges, rb = ir.pm[b].ranges;
    m.ranges = append_ranges(ra, ir.ranges_of(ir.pm[b]));
    (void)rb;
    return new_pm(m);
  }

  // SubtractPortMatchers :164-189 + SpecificPortMatcher.Subtract portmatcher.go:133-153
  int subtract(int a, int b, bool& empty) {
    empty = false;
    if (ir.pm[a].all) {
      if (ir.pm[b].all) {
        empty = true;
        return -1;
      }
      return a;
    }
    if (ir.pm[b].all) {
      empty = true;
      return -1;
    }
    PortMatcher m;
    for (auto& p : ir.pm[a].ports) {
      bool found = false;
      for (auto& q : ir.pm[b].ports)
        if (p.equals(q)) {
          found = true;
          break;
        }
      if (!found) {
        m.ports.push_back(p);
        m.ports_nil = false;
      }
    }
    m.ranges = ir.pm[a].ranges;  // remainingRanges := s.PortRanges (shares the backing array)
    if (m.ranges.len == 0 && m.ports.empty()) {
      empty = true;
      return -1;
    }
    return new_pm(m);
  }

  std::vector<Peer> simplify(const std::vector<Peer>& in, bool& nil) {  // Simplify :8-34
    bool matches_all = false;
    std::vector<const Peer*> pfa, ips, pods;
    for (auto& p : in) {
      if (p.kind == PK_ALL) matches_all = true;
      else if (p.kind == PK_PORTS) pfa.push_back(&p);
      else if (p.kind == PK_IP) ips.push_back(&p);
      else pods.push_back(&p);
    }
    int pfa_port = -1;
    if (!pfa.empty()) {  // simplifyPortsForAllPeers :36-45
      pfa_port = pfa[0]->port;
      for (size_t i = 1; i < pfa.size(); i++) pfa_port = combine(pfa_port, pfa[i]->port);
    }
    std::map<std::string, Peer> gips, gpods;  // sorted by primary key, as the sort.Slice calls
    for (auto* p : ips) {                     // simplifyIPMatchers :68-88
      std::string k = p->ip_pk();
      auto it = gips.find(k);
      if (it == gips.end()) gips.emplace(k, *p);
      else it->second.port = combine(it->second.port, p->port);
    }
    for (auto* p : pods) {  // simplifyPodMatchers :47-66
      std::string k = p->pod_pk();
      auto it = gpods.find(k);
      if (it == gpods.end()) gpods.emplace(k, *p);
      else it->second.port = combine(it->second.port, p->port);
    }
    std::vector<Peer> out;
    if (matches_all) {  // GenerateSimplifiedMatchers :122-140
      nil = false;
      return {Peer{}};
    }
    if (pfa_port >= 0) {
      Peer p;
      p.kind = PK_PORTS;
      p.port = pfa_port;
      out.push_back(p);
    }
    for (auto* g : {&gips, &gpods})
      for (auto& kv : *g) {
        Peer p = kv.second;
        if (pfa_port >= 0) {  // simplifyIPsAndPodsIntoAlls :90-120
          bool empty;
          int rem = subtract(p.port, pfa_port, empty);
          if (empty) continue;
          p.port = rem;
        }
        out.push_back(p);
      }
    nil = out.empty();
    return out;
  }
};

std::vector<PortRange> PolicyIR::ranges_of(const PortMatcher& m) const {
  std::vector<PortRange> v;
  for (uint32_t i = 0; i < m.ranges.len; i++) v.push_back(range_arrays[m.ranges.arr][i]);
  return v;
}

static std::string target_pk(const std::string& ns, const Selector& s) {
  return "{\"Namespace\": \"" + ns + "\", \"PodSelector\": " + s.serialize() + "}";
}

static void for_each_netpol(const Node& root, const std::function<void(const Node&)>& f) {
  if (root.is_arr()) {
    for (auto& p : root.a) f(p);
  } else if (root.is_obj()) {
    if (auto items = root.val("items"); items && items->is_arr()) {
      for (auto& p : items->a) f(p);
    } else {
      f(root);
    }
  }
}

PolicyIR build_network_policies(const Node& netpols, bool simplify) {
  Compiler c;
  std::map<std::string, Target> dict[2];
  for_each_netpol(netpols, [&](const Node& pol) {
    const Node* md = pol.sval("metadata");
    const Node* spec = pol.sval("spec");
    std::string name, ns;
    if (md) {
      if (auto n = md->sval("name")) name = n->str();
      if (auto n = md->sval("namespace")) ns = n->str();
    }
    if (ns.empty()) ns = "default";  // builder.go:28-33
    const Node* types = spec ? spec->val("policyTypes") : nullptr;
    if (!types || !types->is_arr() || types->a.empty())
      throw Panic{CYC_ERR_INVALID_POLICY, "invalid network policy: need at least 1 type"};  // :38-40
    Selector sel;
    if (auto ps = spec->sval("podSelector")) sel = decode_selector(*ps);
    bool have[2] = {false, false};
    Target built[2];
    for (auto& t : types->a) {  // BuildTarget :35-61 (a repeated type rebuilds the same target)
      int d = t.str() == "Ingress" ? 0 : t.str() == "Egress" ? 1 : -1;
      if (d < 0) continue;
      Target tg;
      tg.ns = ns;
      tg.sel = sel;
      tg.rules = {name};
      if (auto rules = spec->val(d == 0 ? "ingress" : "egress"); rules && rules->is_arr())
        for (auto& r : rules->a) c.build_peers(ns, r, d == 0 ? "from" : "to", tg.peers);
      tg.peers_nil = tg.peers.empty();
      built[d] = std::move(tg);
      have[d] = true;
    }
    for (int d = 0; d < 2; d++) {
      if (!have[d]) continue;
      std::string pk = target_pk(built[d].ns, built[d].sel);
      auto it = dict[d].find(pk);
      if (it == dict[d].end()) {  // Policy.AddTarget policy.go:51-66
        built[d].pk = pk;
        dict[d].emplace(pk, std::move(built[d]));
      } else {  // Target.Combine target.go:41-54
        Target& prev = it->second;
        prev.peers.insert(prev.peers.end(), built[d].peers.begin(), built[d].peers.end());
        prev.peers_nil = prev.peers.empty();
        prev.rules.insert(prev.rules.end(), built[d].rules.begin(), built[d].rules.end());
      }
    }
  });
  for (int d = 0; d < 2; d++)
    for (auto& kv : dict[d]) {
      Target t = std::move(kv.second);
      if (simplify) {  // Policy.Simplify policy.go:176-183
        bool nil;
        t.peers = c.simplify(t.peers, nil);
        t.peers_nil = nil;
      }
      c.ir.dir[d].push_back(std::move(t));
    }
  return std::move(c.ir);
}

// ============================================================================ IR JSON (json.Marshal)
static std::string port_json(const PolicyIR& ir, int idx) {
  const PortMatcher& m = ir.pm[idx];
  if (m.all) return "{\"Type\":\"all ports\"}";
  std::string o = "{\"PortRanges\":";
  auto rs = ir.ranges_of(m);
  if (m.ranges.arr < 0) o += "null";
  else {
    o += "[";
    for (size_t i = 0; i < rs.size(); i++)
      o += (i ? "," : "") + std::string("{\"From\":") + std::to_string(rs[i].from) + ",\"Protocol\":" + quote(rs[i].proto) +
           ",\"To\":" + std::to_string(rs[i].to) + ",\"Type\":\"port range\"}";
    o += "]";
  }
  o += ",\"Ports\":";
  if (m.ports_nil) o += "null";
  else {
    o += "[";
    for (size_t i = 0; i < m.ports.size(); i++) {
      auto& p = m.ports[i];
      std::string port = !p.has_port ? "null" : p.port.is_str ? quote(p.port.s) : std::to_string(p.port.i);
      o += (i ? "," : "") + std::string("{\"Port\":") + port + ",\"Protocol\":" + quote(p.proto) + "}";
    }
    o += "]";
  }
  return o + ",\"Type\":\"specific ports\"}";
}

static std::string peer_json(const PolicyIR& ir, const Peer& p) {
  switch (p.kind) {
    case PK_ALL: return "{\"Type\":\"all peers\"}";
    case PK_PORTS: return "{\"Port\":" + port_json(ir, p.port) + ",\"Type\":\"all peers for port\"}";
    case PK_IP: {
      std::string ex = "null";
      if (!p.except_nil) {
        ex = "[";
        for (size_t i = 0; i < p.except.size(); i++) ex += (i ? "," : "") + quote(p.except[i]);
        ex += "]";
      }
      return "{\"CIDR\":" + quote(p.cidr) + ",\"Except\":" + ex + ",\"Port\":" + port_json(ir, p.port) + ",\"Type\":\"IPBlock\"}";
    }
    default: {
      std::string ns = p.ns_kind == NS_EXACT ? "{\"Namespace\":" + quote(p.ns) + ",\"Type\":\"specific namespace\"}"
                       : p.ns_kind == NS_ALL ? std::string("{\"Type\":\"all namespaces\"}")
                                             : "{\"Selector\":" + p.ns_sel.to_json() + ",\"Type\":\"matching namespace by label\"}";
      std::string pod = p.pod_all ? std::string("{\"Type\":\"all pods\"}")
                                  : "{\"Selector\":" + p.pod_sel.to_json() + ",\"Type\":\"matching pods by label\"}";
      return "{\"Namespace\":" + ns + ",\"Pod\":" + pod + ",\"Port\":" + port_json(ir, p.port) + "}";
    }
  }
}

std::string dump_policy_ir(const PolicyIR& ir) {
  std::string o = "{";
  for (int d = 0; d < 2; d++) {
    o += d == 0 ? "\"Ingress\":{" : ",\"Egress\":{";
    for (size_t i = 0; i < ir.dir[d].size(); i++) {
      const Target& t = ir.dir[d][i];
      o += (i ? "," : "") + quote(t.pk) + ":{\"Namespace\":" + quote(t.ns) + ",\"PodSelector\":" + t.sel.to_json() + ",\"Peers\":";
      if (t.peers_nil && t.peers.empty()) o += "null";
      else {
        o += "[";
        for (size_t j = 0; j < t.peers.size(); j++) o += (j ? "," : "") + peer_json(ir, t.peers[j]);
        o += "]";
      }
      o += ",\"SourceRules\":[";
      for (size_t j = 0; j < t.rules.size(); j++) o += (j ? "," : "") + std::string("{\"metadata\":{\"name\":") + quote(t.rules[j]) + "}}";
      o += "]}";
    }
    o += "}";
  }
  return o + "}";
}

static const std::string& type_of(const Node& n) {
  static const std::string none;
  const Node* t = n.val("Type");
  return t ? t->str() : none;
}

PolicyIR load_policy_ir(const Node& root) {
  PolicyIR ir;
  auto load_port = [&](const Node* n) {
    PortMatcher m;
    if (!n || type_of(*n) == "all ports") {
      m.all = true;
    } else {
      if (auto ps = n->val("Ports"); ps && ps->is_arr()) {
        m.ports_nil = false;
        for (auto& p : ps->a) {
          PortEntry e;
          if (auto pr = p.sval("Protocol")) e.proto = pr->str();
          if (auto po = p.val("Port")) {
            e.has_port = true;
            e.port = decode_intstr(*po);
          }
          m.ports.push_back(e);
        }
      }
      if (auto rs = n->val("PortRanges"); rs && rs->is_arr()) {
        std::vector<PortRange> v;
        for (auto& r : rs->a) {
          PortRange pr;
          if (auto x = r.sval("From")) pr.from = int32_t(x->i64());
          if (auto x = r.sval("To")) pr.to = int32_t(x->i64());
          if (auto x = r.sval("Protocol")) pr.proto = x->str();
          v.push_back(pr);
        }
        ir.range_arrays.push_back(v);
        m.ranges = RangeSlice{int(ir.range_arrays.size() - 1), uint32_t(v.size()), uint32_t(v.size())};
      }
    }
    ir.pm.push_back(m);
    return int(ir.pm.size() - 1);
  };
  for (int d = 0; d < 2; d++) {
    const Node* dict = root.val(d == 0 ? "Ingress" : "Egress");
    if (!dict || !dict->is_obj()) continue;
    for (auto& kv : dict->o) {
      const Node& tn = kv.second;
      Target t;
      if (auto ns = tn.sval("Namespace")) t.ns = ns->str();
      if (auto ps = tn.val("PodSelector")) t.sel = decode_selector(*ps);
      t.pk = target_pk(t.ns, t.sel);
      if (auto sr = tn.val("SourceRules"); sr && sr->is_arr())
        for (auto& r : sr->a) {
          const Node* md = r.val("metadata");
          const Node* nm = md ? md->val("name") : nullptr;
          t.rules.push_back(nm ? nm->str() : std::string());
        }
      if (auto peers = tn.val("Peers"); peers && peers->is_arr()) {
        t.peers_nil = false;
        for (auto& pn : peers->a) {
          Peer p;
          const std::string& ty = type_of(pn);
          if (ty == "all peers") {
            p.kind = PK_ALL;
          } else if (ty == "all peers for port") {
            p.kind = PK_PORTS;
            p.port = load_port(pn.val("Port"));
          } else if (ty == "IPBlock") {
            p.kind = PK_IP;
            if (auto c = pn.sval("CIDR")) p.cidr = c->str();
            if (auto ex = pn.val("Except"); ex && ex->is_arr()) {
              p.except_nil = false;
              for (auto& e : ex->a) p.except.push_back(e.str());
            }
            p.port = load_port(pn.val("Port"));
          } else {
            p.kind = PK_POD;
            const Node* ns = pn.val("Namespace");
            const std::string nty = ns ? type_of(*ns) : std::string("all namespaces");
            if (nty == "specific namespace") {
              p.ns_kind = NS_EXACT;
              if (auto x = ns->sval("Namespace")) p.ns = x->str();
            } else if (nty == "matching namespace by label") {
              p.ns_kind = NS_LABEL;
              if (auto x = ns->val("Selector")) p.ns_sel = decode_selector(*x);
            } else {
              p.ns_kind = NS_ALL;
            }
            const Node* pod = pn.val("Pod");
            if (pod && type_of(*pod) == "matching pods by label") {
              p.pod_all = false;
              if (auto x = pod->val("Selector")) p.pod_sel = decode_selector(*x);
            }
            p.port = load_port(pn.val("Port"));
          }
          t.peers.push_back(p);
        }
      }
      ir.dir[d].push_back(std::move(t));
    }
    std::sort(ir.dir[d].begin(), ir.dir[d].end(), [](const Target& a, const Target& b) { return a.pk < b.pk; });
  }
  return ir;
}

// ============================================================================ probe model
static void decode_labels(const Node* n, bool& nil, std::map<std::string, std::string>& out) {
  nil = !n || n->null();
  if (nil) return;
  for (auto& kv : n->o) out[kv.first] = kv.second.null() ? "" : kv.second.str();
}

Resources load_resources(const Node& n) {
  Resources r;
  if (auto ns = n.val("Namespaces"); ns && ns->is_obj())
    for (auto& kv : ns->o) {
      if (kv.second.null()) {
        r.namespaces[kv.first] = std::nullopt;
      } else {
        std::map<std::string, std::string> l;
        bool nil;
        decode_labels(&kv.second, nil, l);
        r.namespaces[kv.first] = l;
      }
    }
  if (auto pods = n.val("Pods"); pods && pods->is_arr()) {
    r.pods.reserve(pods->a.size());
    for (auto& p : pods->a) {
      Pod pod;
      if (auto x = p.sval("Namespace")) pod.ns = x->str();
      if (auto x = p.sval("Name")) pod.name = x->str();
      if (auto x = p.sval("IP")) pod.ip = x->str();
      decode_labels(p.val("Labels"), pod.labels_nil, pod.labels);
      if (auto cs = p.val("Containers"); cs && cs->is_arr())
        for (auto& c : cs->a) {
          Container ct;
          if (auto x = c.sval("Name")) ct.name = x->str();
          if (auto x = c.sval("Port")) ct.port = int32_t(x->i64());
          if (auto x = c.sval("Protocol")) ct.proto = x->str();
          if (auto x = c.sval("PortName")) ct.port_name = x->str();
          pod.conts.push_back(ct);
        }
      r.pods.push_back(std::move(pod));
    }
  }
  return r;
}

std::vector<ProbeConfig> load_probes(const Node& n) {
  std::vector<ProbeConfig> out;
  auto one = [&](const Node& p) {
    ProbeConfig c;
    if (auto a = p.sval("AllAvailable"); a && a->t == Node::Bool && a->b) {
      c.all_available = true;
    } else {
      const Node* src = p.val("PortProtocol") ? p.val("PortProtocol") : &p;
      if (auto x = src->val("Port")) c.port = decode_intstr(*x);
      if (auto x = src->sval("Protocol")) c.proto = x->str();
    }
    out.push_back(c);
  };
  if (n.is_arr()) for (auto& p : n.a) one(p);
  else if (n.is_obj()) one(n);
  return out;
}

// ============================================================================ Go net parsing
// Restates Go 1.16 net.ParseIP / ParseCIDR / networkNumberAndMask into fixed-width words.
static bool go_dtoi(const std::string& s, size_t off, int& n, size_t& used) {
  n = 0;
  used = 0;
  while (off + used < s.size() && s[off + used] >= '0' && s[off + used] <= '9') {
    n = n * 10 + (s[off + used] - '0');
    used++;
    if (n >= 0xFFFFFF) return false;
  }
  return used > 0;
}
static bool go_v4(const std::string& s, uint8_t out[4]) {
  size_t pos = 0;
  for (int i = 0; i < 4; i++) {
    if (pos >= s.size()) return false;
    if (i > 0) {
      if (s[pos] != '.') return false;
      pos++;
    }
    int n;
    size_t c;
    if (!go_dtoi(s, pos, n, c) || n > 255) return false;
    pos += c;
    out[i] = uint8_t(n);
  }
  return pos == s.size();
}
static bool go_v6(std::string s, uint8_t ip[16]) {
  memset(ip, 0, 16);
  int ellipsis = -1;
  if (s.size() >= 2 && s[0] == ':' && s[1] == ':') {
    ellipsis = 0;
    s = s.substr(2);
    if (s.empty()) return true;
  }
  int i = 0;
  while (i < 16) {
    int n = 0;
    size_t c = 0;
    for (; c < s.size(); c++) {
      char h = s[c];
      int d = (h >= '0' && h <= '9') ? h - '0' : (h >= 'a' && h <= 'f') ? h - 'a' + 10 : (h >= 'A' && h <= 'F') ? h - 'A' + 10 : -1;
      if (d < 0) break;
      n = n * 16 + d;
      if (n >= 0xFFFFFF) return false;
    }
    if (c == 0 || n > 0xFFFF) return false;
    if (c < s.size() && s[c] == '.') {
      if (ellipsis < 0 && i != 12) return false;
      if (i + 4 > 16) return false;
      uint8_t v4[4];
      if (!go_v4(s, v4)) return false;
      memcpy(ip + i, v4, 4);
      s.clear();
      i += 4;
      break;
    }
    ip[i] = uint8_t(n >> 8);
    ip[i + 1] = uint8_t(n);
    i += 2;
    s = s.substr(c);
    if (s.empty()) break;
    if (s[0] != ':' || s.size() == 1) return false;
    s = s.substr(1);
    if (s[0] == ':') {
      if (ellipsis >= 0) return false;
      ellipsis = i;
      s = s.substr(1);
      if (s.empty()) break;
    }
  }
  if (!s.empty()) return false;
  if (i < 16) {
    if (ellipsis < 0) return false;
    int n = 16 - i;
    for (int j = i - 1; j >= ellipsis; j--) ip[j + n] = ip[j];
    for (int j = ellipsis + n - 1; j >= ellipsis; j--) ip[j] = 0;
  } else if (ellipsis >= 0) {
    return false;
  }
  return true;
}
static bool mapped(const uint8_t b[16]) {
  for (int i = 0; i < 10; i++)
    if (b[i]) return false;
  return b[10] == 0xff && b[11] == 0xff;
}
static void words(const uint8_t* b, int nbytes, uint32_t* w) {
  for (int k = 0; k < nbytes / 4; k++)
    w[k] = (uint32_t(b[4 * k]) << 24) | (uint32_t(b[4 * k + 1]) << 16) | (uint32_t(b[4 * k + 2]) << 8) | b[4 * k + 3];
}

static DIP parse_ip(const std::string& s) {  // ParseIP + To4
  DIP r{};
  bool v4 = false;
  for (char c : s) {
    if (c == '.') {
      v4 = true;
      break;
    }
    if (c == ':') break;
  }
  bool any = s.find_first_of(".:") != std::string::npos;
  if (!any) return r;
  uint8_t b[16];
  if (v4) {
    uint8_t q[4];
    if (!go_v4(s, q)) return r;
    r.valid = 1;
    r.fam = 4;
    words(q, 4, &r.w[3]);
    return r;
  }
  if (!go_v6(s, b)) return r;
  r.valid = 1;
  if (mapped(b)) {
    r.fam = 4;
    words(b + 12, 4, &r.w[3]);
  } else {
    r.fam = 6;
    words(b, 16, r.w);
  }
  return r;
}

static DCidr parse_cidr(const std::string& s) {  // ParseCIDR + networkNumberAndMask
  DCidr r{};
  size_t slash = s.find('/');
  if (slash == std::string::npos) return r;
  std::string addr = s.substr(0, slash), mask = s.substr(slash + 1);
  uint8_t b[16], q[4];
  int iplen;
  if (go_v4(addr, q)) iplen = 4;
  else if (go_v6(addr, b)) iplen = 16;
  else return r;
  int n;
  size_t used;
  if (!go_dtoi(mask, 0, n, used) || used != mask.size() || n > 8 * iplen) return r;
  uint8_t m[16] = {0};
  for (int i = 0, left = n; i < iplen; i++, left -= 8) m[i] = left >= 8 ? 0xff : left > 0 ? uint8_t(~(0xff >> left)) : 0;
  r.valid = 1;
  if (iplen == 4) {
    for (int i = 0; i < 4; i++) q[i] &= m[i];
    r.fam = 4;
    words(q, 4, &r.net[3]);
    words(m, 4, &r.mask[3]);
    return r;
  }
  for (int i = 0; i < 16; i++) b[i] &= m[i];
  if (mapped(b)) {  // To4() of the masked network is non-nil => IPv4 semantics with mask[12:]
    r.fam = 4;
    words(b + 12, 4, &r.net[3]);
    words(m + 12, 4, &r.mask[3]);
  } else {
    r.fam = 6;
    words(b, 16, r.net);
    words(m, 16, r.mask);
  }
  return r;
}

// ============================================================================ flattening
uint32_t Problem::intern(const std::string& s) {
  auto it = string_id.find(s);
  if (it != string_id.end()) return it->second;
  uint32_t id = uint32_t(strings.size());
  strings.push_back(s);
  string_id.emplace(s, id);
  return id;
}

namespace {
struct Flattener {
  Problem& pb;
  std::unordered_map<std::string, uint32_t> ls_ids, sel_ids, cidr_ids, desc_ids;
  std::unordered_map<int, uint32_t> pm_ids;
  const PolicyIR& ir;

  Flattener(Problem& p, const PolicyIR& i) : pb(p), ir(i) {
    pb.ls_off = {0};
    ls_ids[""] = 0;  // label set 0 == empty map (nil behaves the same for reads)
    pb.ls_off.push_back(0);
    pb.sel_off = {0};
  }

  uint32_t label_set(const std::map<std::string, std::string>& l) {
    if (l.empty()) return 0;
    std::string key;
    for (auto& kv : l) {
      key += kv.first;
      key += '\0';
      key += kv.second;
      key += '\0';
    }
    auto it = ls_ids.find(key);
    if (it != ls_ids.end()) return it->second;
    std::vector<std::pair<uint32_t, uint32_t>> kvs;
    for (auto& kv : l) kvs.emplace_back(pb.intern(kv.first), pb.intern(kv.second));
    std::sort(kvs.begin(), kvs.end());
    for (auto& kv : kvs) {
      pb.ls_key.push_back(kv.first);
      pb.ls_val.push_back(kv.second);
    }
    uint32_t id = uint32_t(pb.ls_off.size() - 1);
    pb.ls_off.push_back(uint32_t(pb.ls_key.size()));
    ls_ids.emplace(key, id);
    return id;
  }

  uint32_t selector(const Selector& s) {
    std::string key = s.serialize();
    for (auto& e : s.exprs) key += "\x01" + e.op;  // operators are part of serialize; keep explicit
    auto it = sel_ids.find(key);
    if (it != sel_ids.end()) return it->second;
    for (auto& kv : s.labels) {  // matchLabels first (labelselector.go:69-74), then expressions
      DReq r{};
      r.key = pb.intern(kv.first);
      r.op = kv.second.empty() ? REQ_EQ_EMPTY : REQ_EQ;
      r.voff = uint32_t(pb.req_vals.size());
      r.vcnt = 1;
      pb.req_vals.push_back(pb.intern(kv.second));
      pb.reqs.push_back(r);
    }
    for (auto& e : s.exprs) {
      DReq r{};
      r.key = pb.intern(e.key);
      r.op = e.op == "In" ? REQ_IN : e.op == "NotIn" ? REQ_NOTIN : e.op == "Exists" ? REQ_EXISTS
             : e.op == "DoesNotExist" ? REQ_DNE : REQ_INVALID;
      if (r.op == REQ_INVALID) pb.may_err = true;
      r.voff = uint32_t(pb.req_vals.size());
      if (r.op == REQ_IN || r.op == REQ_NOTIN) {
        for (auto& v : e.values) pb.req_vals.push_back(pb.intern(v));
        r.vcnt = uint32_t(e.values.size());
      }
      pb.reqs.push_back(r);
    }
    uint32_t id = uint32_t(pb.sel_off.size() - 1);
    pb.sel_off.push_back(uint32_t(pb.reqs.size()));
    sel_ids.emplace(key, id);
    return id;
  }

  uint32_t cidr(const std::string& s) {
    auto it = cidr_ids.find(s);
    if (it != cidr_ids.end()) return it->second;
    DCidr c = parse_cidr(s);
    if (!c.valid) pb.may_err = true;
    uint32_t id = uint32_t(pb.cidrs.size());
    pb.cidrs.push_back(c);
    pb.cidr_str.push_back(s);
    cidr_ids.emplace(s, id);
    return id;
  }

  uint32_t port_matcher(int idx) {
    auto it = pm_ids.find(idx);
    if (it != pm_ids.end()) return it->second;
    const PortMatcher& m = ir.pm[idx];
    DPortM d{};
    d.all = m.all ? 1 : 0;
    d.eoff = uint32_t(pb.pents.size());
    if (!m.all) {
      for (auto& p : m.ports) {
        DPortEntry e{};
        e.proto = pb.intern(p.proto);
        if (!p.has_port) e.kind = PE_PROTO;
        else if (p.port.is_str) {
          e.kind = PE_NAME;
          e.a = int32_t(pb.intern(p.port.s));
        } else {
          e.kind = PE_INT;
          e.a = p.port.i;
        }
        pb.pents.push_back(e);
      }
      for (auto& r : ir.ranges_of(m)) {
        DPortEntry e{};
        e.kind = PE_RANGE;
        e.a = r.from;
        e.b = r.to;
        e.proto = pb.intern(r.proto);
        pb.pents.push_back(e);
      }
    }
    d.ecnt = uint32_t(pb.pents.size()) - d.eoff;
    uint32_t id = uint32_t(pb.pms.size());
    pb.pms.push_back(d);
    pm_ids.emplace(idx, id);
    return id;
  }

  uint32_t desc(int32_t port, const std::string& name, const std::string& proto) {
    uint32_t n = pb.intern(name), p = pb.intern(proto);
    std::string key = std::to_string(port) + "/" + std::to_string(n) + "/" + std::to_string(p);
    auto it = desc_ids.find(key);
    if (it != desc_ids.end()) return it->second;
    uint32_t id = uint32_t(pb.descs.size());
    pb.descs.push_back(DDesc{port, n, p, 0});
    desc_ids.emplace(key, id);
    return id;
  }
};
}  // namespace

// Targets and their ordered peers (both directions) -> DTarget / DPeer / port / CIDR tables.
static bool flatten_targets(Problem& pb, Flattener& F, const PolicyIR& ir) {
  bool any_ip_peer = false;
  for (int d = 0; d < 2; d++) {
    for (auto& t : ir.dir[d]) {
      DTarget dt{};
      dt.ns = pb.intern(t.ns);
      dt.sel = F.selector(t.sel);
      dt.poff = uint32_t(pb.peers.size());
      dt.pcnt = uint32_t(t.peers.size());
      for (auto& p : t.peers) {
        DPeer dp{};
        dp.kind = p.kind;
        dp.port = (p.kind == PK_ALL) ? CYC_ALL : F.port_matcher(p.port);
        dp.podsel = CYC_ALL;
        dp.ipb = CYC_ALL;
        if (p.kind == PK_POD) {
          dp.nskind = p.ns_kind;
          dp.nsval = p.ns_kind == NS_EXACT ? pb.intern(p.ns) : p.ns_kind == NS_LABEL ? F.selector(p.ns_sel) : 0;
          dp.podsel = p.pod_all ? CYC_ALL : F.selector(p.pod_sel);
        } else if (p.kind == PK_IP) {
          any_ip_peer = true;
          DIPBlock b{};
          b.cidr = F.cidr(p.cidr);
          b.exoff = uint32_t(pb.ipb_ex.size());
          for (auto& e : p.except) pb.ipb_ex.push_back(F.cidr(e));
          b.excnt = uint32_t(p.except.size());
          dp.ipb = uint32_t(pb.ipbs.size());
          pb.ipbs.push_back(b);
        }
        pb.peers.push_back(dp);
      }
      pb.tgt[d].push_back(dt);
    }
  }
  return any_ip_peer;
}

static void finish_tables(Problem& pb) {
  // ---- per-namespace target ranges (targets are sorted by primary key, which starts with the
  //      namespace, so each namespace's targets are contiguous)
  pb.L = uint32_t(pb.ls_off.size() - 1);
  pb.S = uint32_t(pb.sel_off.size() - 1);
  for (int d = 0; d < 2; d++) {
    pb.tns_lo[d].assign(pb.strings.size(), 0);
    pb.tns_hi[d].assign(pb.strings.size(), 0);
    for (uint32_t t = 0; t < pb.tgt[d].size(); t++) {
      uint32_t ns = pb.tgt[d][t].ns;
      if (pb.tns_hi[d][ns] == 0) pb.tns_lo[d][ns] = t;
      else if (pb.tns_hi[d][ns] != t) throw std::runtime_error("internal: namespace targets not contiguous");
      pb.tns_hi[d][ns] = t + 1;
    }
  }
}

// NewTableFromJobResults (table.go:38-48) for one probe config: the first result whose Item already
// holds its key (Item.AddJobResult table.go:16-22 -> utils.DoOrDie), or "".  Results come in
// runProbe's order (jobrunner.go:33-58): valid jobs in RunJobs order (podFrom, podTo[, container],
// resources.go:286-287, 345-347), then BadPortProtocol, then BadNamedPort jobs; an Item is the
// (FromKey, ToKey) = ns/name pair, so pods sharing a name share Items; the key is Protocol/ResolvedPort
// (job.go:23-25).  The reference walks all P^2 K results; this finds the same first duplicate in
// O(P K) from the structure of that order.  A job's category c (0 valid, 1 BadPortProtocol,
// 2 BadNamedPort) and key depend on the destination only, so the results are, per category, every
// source times the destination jobs J_c = (d[, container]) of that category in (d, container) order:
//  (A) a destination job j of J_c whose key its destination's name group (pods sharing its ns/name)
//      already produced in an earlier category or earlier in J_c repeats for EVERY source, first at
//      (c, source 0, j) — source 0 adds the earlier one before it;
//  (B) a source that is not the first pod of its name group repeats at its first job, because the
//      group's first pod added the same (Item, key) earlier in the same category.
// In the first category where either happens, (A) at source 0 precedes (B) at a later source.  The
// reference's message continues with the Job as %+v and the stack pkg/errors prints; the job is
// named here by FromKey, ToKey and ToContainer (the oracle's text, oracle/oracle.cpp).
// Pods [q0, q1) are the problem's pods (a batched block's, or all).
static std::string table_build_error(const Resources& res, const Problem& pb, const ProbeConfig& pc, size_t c, uint32_t koff,
                                     uint32_t q0, uint32_t q1) {
  const uint32_t P = q1;
  if (q1 <= q0) return "";
  std::unordered_map<std::string, uint32_t> first_of;  // name group: first pod with the ns/name
  std::vector<uint32_t> grp(P);
  uint32_t s_b = P;  // the first pod that is not the first of its name group
  for (uint32_t p = q0; p < P; p++) {
    grp[p] = first_of.emplace(pb.pod_key[p], p).first->second;
    if (grp[p] != p && s_b == P) s_b = p;
  }
  struct DJob {
    uint32_t d, i;  // destination pod, container index (AllAvailable) or 0
    std::string key;
  };
  std::vector<DJob> jobs[3];
  for (uint32_t d = q0; d < P; d++) {
    const Pod& pod = res.pods[d];
    const size_t base = size_t(d) * pb.K + koff;
    if (pc.all_available) {
      for (uint32_t i = 0; i < pod.conts.size(); i++)
        jobs[0].push_back({d, i, pod.conts[i].proto + "/" + std::to_string(pod.conts[i].port)});
      continue;
    }
    const uint8_t st = pb.slot_status[base];
    int port = -1;  // ResolvedPort: -1 for a named port that does not resolve (resources.go:303-308)
    if (st == CYC_JOB_VALID) port = pb.descs[size_t(pb.slot_desc[base])].port;
    else if (st == CYC_JOB_BAD_PORT_PROTOCOL) port = pc.port.i;
    const int cat = st == CYC_JOB_VALID ? 0 : st == CYC_JOB_BAD_PORT_PROTOCOL ? 1 : 2;
    jobs[cat].push_back({d, 0, pc.proto + "/" + std::to_string(port)});
  }
  std::set<std::pair<uint32_t, std::string>> seen;  // (name group of the destination, key)
  for (int cat = 0; cat < 3; cat++) {
    const DJob* hit = nullptr;
    for (const DJob& j : jobs[cat])
      if (!seen.insert({grp[j.d], j.key}).second) {
        hit = &j;
        break;
      }
    if (!hit && s_b < P && !jobs[cat].empty()) {
      hit = &jobs[cat][0];
      const std::string to_cont = pc.all_available ? res.pods[hit->d].conts[hit->i].name : "";
      return "unable to add job result: duplicate key " + hit->key + " (job {FromKey:" + pb.pod_key[s_b] +
             " ToKey:" + pb.pod_key[hit->d] + " ToContainer:" + to_cont + "})";
    }
    if (hit) {
      const std::string to_cont = pc.all_available ? res.pods[hit->d].conts[hit->i].name : "";
      return "unable to add job result: duplicate key " + hit->key + " (job {FromKey:" + pb.pod_key[q0] + " ToKey:" +
             pb.pod_key[hit->d] + " ToContainer:" + to_cont + "})";
    }
  }
  return "";
}

Problem build_problem(const PolicyIR& ir, const Resources& res, const std::vector<ProbeConfig>& probes,
                      const std::vector<ProbeBlock>* blocks) {
  Problem pb;
  Flattener F(pb, ir);
  pb.P = uint32_t(res.pods.size());
  pb.W = (pb.P + 63) / 64;
  if (blocks) {  // batched blocks: consecutive pod ranges covering the pods, namespaces private to a block
    pb.blocks = *blocks;
    pb.pod_blk.assign(pb.P, 0);
    uint32_t at = 0;
    std::unordered_map<std::string, uint32_t> ns_blk;
    for (uint32_t b = 0; b < blocks->size(); b++) {
      const ProbeBlock& bl = (*blocks)[b];
      if (bl.p0 != at || bl.p1 < bl.p0 || bl.p1 > pb.P || bl.cfg >= probes.size())
        throw Panic{CYC_ERR_ARG, "blocks must be consecutive pod ranges covering the pods, each with a probe config"};
      for (uint32_t q = bl.p0; q < bl.p1; q++) {
        pb.pod_blk[q] = b;
        // a namespace's targets apply to all its pods (TargetsApplyingToPod policy.go:68-82): a block's
        // problem is its own only if no other block has pods in its namespaces
        auto it = ns_blk.emplace(res.pods[q].ns, b).first;
        if (it->second != b) throw Panic{CYC_ERR_ARG, "namespace " + res.pods[q].ns + " has pods in two blocks"};
      }
      at = bl.p1;
    }
    if (at != pb.P) throw Panic{CYC_ERR_ARG, "blocks must cover every pod"};
  }

  // ---- pods
  bool any_bad_ip = false;
  std::vector<uint32_t> ns_ls_cache;
  std::unordered_map<std::string, uint32_t> nsls;
  for (auto& p : res.pods) {
    pb.pod_ns.push_back(pb.intern(p.ns));
    pb.pod_ls.push_back(F.label_set(p.labels));
    auto it = nsls.find(p.ns);
    if (it == nsls.end()) {
      uint32_t id = 0;
      auto nit = res.namespaces.find(p.ns);  // r.Namespaces[ns]: nil when absent
      if (nit != res.namespaces.end() && nit->second) id = F.label_set(*nit->second);
      it = nsls.emplace(p.ns, id).first;
    }
    pb.pod_nsls.push_back(it->second);
    DIP ip = parse_ip(p.ip);
    if (!ip.valid) any_bad_ip = true;
    pb.pod_ip.push_back(ip);
    pb.pod_ip_str.push_back(p.ip);
    pb.pod_key.push_back(p.ns + "/" + p.name);
  }

  bool any_ip_peer = flatten_targets(pb, F, ir);
  if (any_ip_peer && any_bad_ip) pb.may_err = true;

  // ---- probe job slots (resources.go:274-364, resolved per destination pod)
  size_t maxc = 0;
  for (auto& p : res.pods) maxc = std::max(maxc, p.conts.size());
  std::vector<uint32_t> cfg_off;
  for (size_t c = 0; c < probes.size(); c++) {
    cfg_off.push_back(pb.K);
    uint32_t n = probes[c].all_available ? uint32_t(maxc) : 1u;
    for (uint32_t i = 0; i < n; i++) {
      pb.slot_cfg.push_back(uint32_t(c));
      pb.slot_idx.push_back(i);
    }
    pb.K += n;
  }
  pb.n_cfg = uint32_t(probes.size());
  pb.slot_desc.assign(size_t(pb.P) * pb.K, -1);
  pb.slot_status.assign(size_t(pb.P) * pb.K, 0);
  pb.dup_key_msg.assign(probes.size(), "");
  pb.expand_panic.assign(probes.size(), 0);
  {
    bool bare = false, any_cont = false;
    for (auto& p : res.pods) (p.conts.empty() ? bare : any_cont) = true;
    for (size_t c = 0; c < probes.size(); c++)  // PortProtocol: every (from, to) pair builds a job;
      pb.expand_panic[c] = bare && (probes[c].all_available ? any_cont : true);  // AllAvailable: one per dst container
    pb.blk_expand_panic.assign(pb.blocks.size(), 0);
    for (size_t b = 0; b < pb.blocks.size(); b++) {  // the same, per block over its own pods
      bool bb = false, bc = false;
      for (uint32_t q = pb.blocks[b].p0; q < pb.blocks[b].p1; q++) (res.pods[q].conts.empty() ? bb : bc) = true;
      pb.blk_expand_panic[b] = bb && (probes[pb.blocks[b].cfg].all_available ? bc : true);
    }
  }
  for (size_t c = 0; c < probes.size(); c++) {
    const ProbeConfig& pc = probes[c];
    for (uint32_t d = 0; d < pb.P; d++) {
      if (!pb.blocks.empty() && pb.blocks[pb.pod_blk[d]].cfg != c) continue;  // a block answers its config only
      const Pod& pod = res.pods[d];
      size_t base = size_t(d) * pb.K + cfg_off[c];
      if (pc.all_available) {  // GetJobsAllAvailableServers :336-364
        for (size_t i = 0; i < pod.conts.size(); i++) {
          auto& ct = pod.conts[i];
          pb.slot_desc[base + i] = int32_t(F.desc(ct.port, ct.port_name, ct.proto));
          pb.slot_status[base + i] = CYC_JOB_VALID;
        }
        continue;
      }
      // GetJobsForNamedPortProtocol :284-334 (every pair gets a job)
      if (pc.port.is_str) {  // ResolveNamedPort pod.go:132-139
        const Container* hit = nullptr;
        for (auto& ct : pod.conts)
          if (ct.port_name == pc.port.s) {
            hit = &ct;
            break;
          }
        if (hit) {
          pb.slot_desc[base] = int32_t(F.desc(hit->port, pc.port.s, pc.proto));
          pb.slot_status[base] = CYC_JOB_VALID;
        } else {
          pb.slot_status[base] = CYC_JOB_BAD_NAMED_PORT;
        }
      } else {  // ResolveNumberedPort pod.go:141-148 (protocol ignored)
        const Container* hit = nullptr;
        for (auto& ct : pod.conts)
          if (ct.port == pc.port.i) {
            hit = &ct;
            break;
          }
        if (hit) {
          pb.slot_desc[base] = int32_t(F.desc(pc.port.i, hit->port_name, pc.proto));
          pb.slot_status[base] = CYC_JOB_VALID;
        } else {
          pb.slot_status[base] = CYC_JOB_BAD_PORT_PROTOCOL;
        }
      }
    }
    if (pb.blocks.empty()) pb.dup_key_msg[c] = table_build_error(res, pb, pc, c, cfg_off[c], 0, pb.P);
  }
  pb.blk_dup_msg.assign(pb.blocks.size(), "");
  for (size_t b = 0; b < pb.blocks.size(); b++) {
    const ProbeBlock& bl = pb.blocks[b];
    pb.blk_dup_msg[b] = table_build_error(res, pb, probes[bl.cfg], bl.cfg, cfg_off[bl.cfg], bl.p0, bl.p1);
  }

  finish_tables(pb);
  return pb;
}

std::vector<QueryTraffic> load_traffics(const Node& n) {
  std::vector<QueryTraffic> out;
  if (!n.is_arr()) return out;
  auto end = [](const Node* p) {
    QueryEnd e;
    if (!p) return e;
    if (auto ip = p->sval("IP")) e.ip = ip->str();
    if (auto in = p->val("Internal")) {
      e.external = false;
      if (auto ns = in->sval("Namespace")) e.ns = ns->str();
      bool nil;
      decode_labels(in->val("PodLabels"), nil, e.labels);
      decode_labels(in->val("NamespaceLabels"), nil, e.ns_labels);
    }
    return e;
  };
  for (auto& t : n.a) {
    QueryTraffic q;
    q.src = end(t.val("Source"));
    q.dst = end(t.val("Destination"));
    if (auto x = t.val("ResolvedPort")) q.port = int32_t(x->i64());
    if (auto x = t.val("ResolvedPortName")) q.port_name = x->str();
    if (auto x = t.val("Protocol")) q.proto = x->str();
    out.push_back(std::move(q));
  }
  return out;
}

// analyze --mode query-target input (analyze.go:163-187): a JSON list of QueryTargetPod
// {Namespace, Labels}; each becomes a traffic from the pod to itself (only membership is used).
std::vector<QueryTraffic> load_target_pods(const Node& n) {
  std::vector<QueryTraffic> out;
  if (!n.is_arr()) return out;
  for (auto& t : n.a) {
    QueryEnd e;
    e.external = false;
    if (auto ns = t.val("Namespace")) e.ns = ns->str();
    bool nil;
    decode_labels(t.val("Labels"), nil, e.labels);
    QueryTraffic q;
    q.src = e;
    q.dst = e;
    out.push_back(std::move(q));
  }
  return out;
}

// Query mode (analyze --mode query-traffic, analyze.go:209-225): endpoint 2i is traffic i's
// source, 2i+1 its destination; namespace labels come from the Traffic itself.
Problem build_query_problem(const PolicyIR& ir, const std::vector<QueryTraffic>& ts, std::vector<uint32_t>& ext,
                            std::vector<uint32_t>& tdesc) {
  Problem pb;
  Flattener F(pb, ir);
  pb.P = uint32_t(ts.size() * 2);
  pb.W = (pb.P + 63) / 64;
  bool any_bad_ip = false;
  ext.clear();
  tdesc.clear();
  for (auto& t : ts)
    for (const QueryEnd* e : {&t.src, &t.dst}) {
      pb.pod_ns.push_back(pb.intern(e->ns));
      pb.pod_ls.push_back(F.label_set(e->labels));
      pb.pod_nsls.push_back(F.label_set(e->ns_labels));
      DIP ip = parse_ip(e->ip);
      any_bad_ip |= !ip.valid;
      pb.pod_ip.push_back(ip);
      pb.pod_ip_str.push_back(e->ip);
      ext.push_back(e->external ? 1u : 0u);
    }
  for (auto& t : ts) tdesc.push_back(F.desc(t.port, t.port_name, t.proto));
  bool any_ip_peer = flatten_targets(pb, F, ir);
  if (any_ip_peer && any_bad_ip) pb.may_err = true;
  finish_tables(pb);
  return pb;
}

}  // namespace cyc
