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

// ============================================================================ byte-string maps
// Open-addressing map from byte strings to dense ids (first-insertion order), keys in one arena:
// no allocation per key, one hash per lookup (the interning of 10^5-10^6 short strings and label maps
// is the bulk of cyc_resources_load / cyc_probe_prepare's host time).
static inline uint64_t bytes_hash(const char* p, size_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ (n * 0xBF58476D1CE4E5B9ull);
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    memcpy(&w, p + i, 8);
    h = (h ^ w) * 0x94D049BB133111EBull;
    h ^= h >> 29;
  }
  uint64_t w = 0;
  memcpy(&w, p + i, n - i);
  h = (h ^ w) * 0xBF58476D1CE4E5B9ull;
  h ^= h >> 31;
  h *= 0x94D049BB133111EBull;
  return h ^ (h >> 32);
}
struct BytesMap {
  std::vector<uint32_t> slot;  // id + 1; 0 = empty
  std::vector<uint64_t> off{0};
  std::string arena;
  size_t size() const { return off.size() - 1; }
  void reserve(size_t keys, size_t bytes) {
    off.reserve(keys + 1);
    arena.reserve(bytes);
    size_t cap = 64;
    while (cap < 2 * keys + 2) cap <<= 1;
    if (cap > slot.size()) {
      slot.assign(cap / 2, 0);  // grow() doubles it and re-inserts the (no) keys
      grow();
    }
  }
  std::string_view key(uint32_t id) const { return std::string_view(arena.data() + off[id], size_t(off[id + 1] - off[id])); }
  // id of the key, adding it if absent (added = true)
  uint32_t get(const char* p, size_t n, bool* added = nullptr) {
    if (2 * (size() + 1) > slot.size()) grow();
    const size_t mask = slot.size() - 1;
    for (size_t x = bytes_hash(p, n) & mask;; x = (x + 1) & mask) {
      const uint32_t s = slot[x];
      if (!s) {
        arena.append(p, n);
        off.push_back(arena.size());
        slot[x] = uint32_t(size());
        if (added) *added = true;
        return uint32_t(size() - 1);
      }
      const std::string_view k = key(s - 1);
      if (k.size() == n && (n == 0 || memcmp(k.data(), p, n) == 0)) {
        if (added) *added = false;
        return s - 1;
      }
    }
  }
  void grow() {
    std::vector<uint32_t> old(std::max<size_t>(slot.size() * 2, 64), 0);
    old.swap(slot);
    const size_t mask = slot.size() - 1;
    for (uint32_t id = 0; id < size(); id++) {
      const std::string_view k = key(id);
      size_t x = bytes_hash(k.data(), k.size()) & mask;
      while (slot[x]) x = (x + 1) & mask;
      slot[x] = id + 1;
    }
  }
};

// Open-addressing map from 64-bit keys to 32-bit values (first insertion wins).
struct U64Map {
  std::vector<uint64_t> key;
  std::vector<uint32_t> val;  // ~0 = empty slot
  explicit U64Map(size_t n) {
    size_t cap = 64;
    while (cap < 2 * n + 2) cap <<= 1;
    key.assign(cap, 0);
    val.assign(cap, ~0u);
  }
  // the value stored under k, storing v first if k is absent
  uint32_t emplace(uint64_t k, uint32_t v) {
    const size_t mask = key.size() - 1;
    uint64_t h = k * 0x9E3779B97F4A7C15ull;
    for (size_t x = (h ^ (h >> 29)) & mask;; x = (x + 1) & mask) {
      if (val[x] == ~0u) {
        key[x] = k;
        val[x] = v;
        return v;
      }
      if (key[x] == k) return val[x];
    }
  }
};

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

// ============================================================================ IR flat tables
// The already-built Go *matcher.Policy as cyc_policy_tables (include/cyclonus_hip.h): the same IR
// load_policy_ir reads from json.Marshal(*Policy), without JSON.
PolicyIR load_policy_tables(const cyc_policy_tables& t) {
  const struct Check {
    [[noreturn]] void bad(const std::string& m) const { throw Panic{CYC_ERR_ARG, "cyc_policy_tables: " + m}; }
    void need(const void* p, const char* name) const {
      if (!p) bad(std::string("null ") + name);
    }
    int64_t offsets(const int64_t* off, int64_t n, const char* name) const {
      if (n < 0) bad(std::string("negative count for ") + name);
      need(off, name);
      if (off[0] < 0) bad(std::string(name) + "[0] < 0");
      for (int64_t i = 0; i < n; i++)
        if (off[i + 1] < off[i]) bad(std::string(name) + " decreases at " + std::to_string(i));
      return off[n];
    }
    void index(int64_t v, int64_t n, const char* name, int64_t at) const {
      if (v < 0 || v >= n) bad(std::string(name) + "[" + std::to_string(at) + "] = " + std::to_string(v) + " out of range");
    }
  } ck;
  // strings
  constexpr int64_t U32 = int64_t(1) << 32;  // ids, counts and offsets are kept as 32-bit values
  if (t.str.n >= U32) ck.bad("str.n = " + std::to_string(t.str.n) + ": more than 2^32 - 1 strings");
  ck.offsets(t.str.off, t.str.n, "str.off");
  if (t.str.n && t.str.off[t.str.n] > t.str.off[0]) ck.need(t.str.bytes, "str.bytes");
  auto S = [&](int64_t i, const char* name, int64_t at) {
    ck.index(i, t.str.n, name, at);
    return std::string(t.str.bytes + t.str.off[i], size_t(t.str.off[i + 1] - t.str.off[i]));
  };
  // selectors
  const int64_t NS = t.n_selectors;
  std::vector<Selector> sels(size_t(std::max<int64_t>(NS, 0)));
  if (NS) {
    const int64_t nl = ck.offsets(t.sel_label_off, NS, "sel_label_off");
    const int64_t ne = ck.offsets(t.sel_expr_off, NS, "sel_expr_off");
    if (nl > t.sel_label_off[0]) {
      ck.need(t.sel_label_key, "sel_label_key");
      ck.need(t.sel_label_val, "sel_label_val");
    }
    if (ne > t.sel_expr_off[0]) {
      ck.need(t.expr_key, "expr_key");
      ck.need(t.expr_op, "expr_op");
      ck.need(t.expr_value_off, "expr_value_off");
    }
    for (int64_t i = 0; i < NS; i++) {
      Selector& s = sels[size_t(i)];
      for (int64_t j = t.sel_label_off[i]; j < t.sel_label_off[i + 1]; j++)
        s.labels[S(t.sel_label_key[j], "sel_label_key", j)] = S(t.sel_label_val[j], "sel_label_val", j);
      for (int64_t e = t.sel_expr_off[i]; e < t.sel_expr_off[i + 1]; e++) {
        Requirement r;
        r.key = S(t.expr_key[e], "expr_key", e);
        r.op = S(t.expr_op[e], "expr_op", e);
        if (t.expr_value_off[e + 1] < t.expr_value_off[e] || t.expr_value_off[e] < 0) ck.bad("expr_value_off decreases at " + std::to_string(e));
        if (t.expr_value_off[e + 1] > t.expr_value_off[e]) ck.need(t.expr_value, "expr_value");
        for (int64_t v = t.expr_value_off[e]; v < t.expr_value_off[e + 1]; v++) r.values.push_back(S(t.expr_value[v], "expr_value", v));
        s.exprs.push_back(std::move(r));
      }
    }
  }
  auto sel = [&](int64_t i, const char* name, int64_t at) -> const Selector& {
    ck.index(i, NS, name, at);
    return sels[size_t(i)];
  };
  // port matchers (each keeps its own range array, as loaded from Go: aliasing already happened there)
  PolicyIR ir;
  const int64_t NM = t.n_port_matchers;
  if (NM < 0) ck.bad("negative n_port_matchers");
  if (NM) {
    ck.need(t.pm_all, "pm_all");
    const int64_t np = ck.offsets(t.pm_port_off, NM, "pm_port_off");
    const int64_t nr = ck.offsets(t.pm_range_off, NM, "pm_range_off");
    if (np > t.pm_port_off[0]) {
      ck.need(t.port_kind, "port_kind");
      ck.need(t.port_value, "port_value");
      ck.need(t.port_proto, "port_proto");
    }
    if (nr > t.pm_range_off[0]) {
      ck.need(t.range_from, "range_from");
      ck.need(t.range_to, "range_to");
      ck.need(t.range_proto, "range_proto");
    }
    for (int64_t m = 0; m < NM; m++) {
      PortMatcher pm;
      pm.all = t.pm_all[m] != 0;
      if (!pm.all) {
        pm.ports_nil = t.pm_ports_nil ? t.pm_ports_nil[m] != 0 : t.pm_port_off[m + 1] == t.pm_port_off[m];
        for (int64_t j = t.pm_port_off[m]; j < t.pm_port_off[m + 1]; j++) {
          PortEntry e;
          e.proto = S(t.port_proto[j], "port_proto", j);
          if (t.port_kind[j] == CYC_PORT_NUMBER) {
            e.has_port = true;
            e.port.i = t.port_value[j];
          } else if (t.port_kind[j] == CYC_PORT_NAME) {
            e.has_port = true;
            e.port.is_str = true;
            e.port.s = S(t.port_value[j], "port_value", j);
          } else if (t.port_kind[j] != CYC_PORT_ANY) {
            ck.bad("port_kind[" + std::to_string(j) + "] unknown");
          }
          pm.ports.push_back(std::move(e));
          pm.ports_nil = false;
        }
        const bool rnil = t.pm_ranges_nil ? t.pm_ranges_nil[m] != 0 : t.pm_range_off[m + 1] == t.pm_range_off[m];
        if (!rnil || t.pm_range_off[m + 1] > t.pm_range_off[m]) {
          std::vector<PortRange> v;
          for (int64_t j = t.pm_range_off[m]; j < t.pm_range_off[m + 1]; j++)
            v.push_back(PortRange{t.range_from[j], t.range_to[j], S(t.range_proto[j], "range_proto", j)});
          ir.range_arrays.push_back(v);
          pm.ranges = RangeSlice{int(ir.range_arrays.size() - 1), uint32_t(v.size()), uint32_t(v.size())};
        }
      }
      ir.pm.push_back(std::move(pm));
    }
  }
  // targets and their ordered peers
  if (t.n_targets[0] < 0 || t.n_targets[1] < 0) ck.bad("negative n_targets");
  const int64_t NT = t.n_targets[0] + t.n_targets[1];
  if (NT) {
    ck.need(t.target_ns, "target_ns");
    ck.need(t.target_sel, "target_sel");
    const int64_t npeer = ck.offsets(t.target_peer_off, NT, "target_peer_off");
    if (t.target_rule_off) {
      const int64_t nrule = ck.offsets(t.target_rule_off, NT, "target_rule_off");
      if (nrule > t.target_rule_off[0]) ck.need(t.rule_name, "rule_name");
    }
    if (npeer > t.target_peer_off[0]) {
      ck.need(t.peer_kind, "peer_kind");
      ck.need(t.peer_port, "peer_port");
    }
    for (int64_t x = 0; x < NT; x++) {
      const int d = x < t.n_targets[0] ? 0 : 1;
      Target tg;
      tg.ns = S(t.target_ns[x], "target_ns", x);
      tg.sel = sel(t.target_sel[x], "target_sel", x);
      tg.pk = target_pk(tg.ns, tg.sel);
      tg.peers_nil = t.target_peers_nil ? t.target_peers_nil[x] != 0 : t.target_peer_off[x + 1] == t.target_peer_off[x];
      if (t.target_rule_off)
        for (int64_t r = t.target_rule_off[x]; r < t.target_rule_off[x + 1]; r++) tg.rules.push_back(S(t.rule_name[r], "rule_name", r));
      for (int64_t j = t.target_peer_off[x]; j < t.target_peer_off[x + 1]; j++) {
        Peer p;
        const uint8_t kind = t.peer_kind[j];
        if (kind > CYC_PEER_IP) ck.bad("peer_kind[" + std::to_string(j) + "] unknown");
        p.kind = PeerKind(kind);
        if (kind != CYC_PEER_ALL) {
          ck.index(t.peer_port[j], NM, "peer_port", j);
          p.port = t.peer_port[j];
        }
        if (kind == CYC_PEER_POD) {
          ck.need(t.peer_ns_kind, "peer_ns_kind");
          ck.need(t.peer_pod_sel, "peer_pod_sel");
          const uint8_t nk = t.peer_ns_kind[j];
          if (nk == CYC_NS_EXACT) {
            ck.need(t.peer_ns, "peer_ns");
            p.ns_kind = NS_EXACT;
            p.ns = S(t.peer_ns[j], "peer_ns", j);
          } else if (nk == CYC_NS_LABEL) {
            ck.need(t.peer_ns, "peer_ns");
            p.ns_kind = NS_LABEL;
            p.ns_sel = sel(t.peer_ns[j], "peer_ns", j);
          } else if (nk == CYC_NS_ALL) {
            p.ns_kind = NS_ALL;
          } else {
            ck.bad("peer_ns_kind[" + std::to_string(j) + "] unknown");
          }
          p.pod_all = t.peer_pod_sel[j] < 0;
          if (!p.pod_all) p.pod_sel = sel(t.peer_pod_sel[j], "peer_pod_sel", j);
        } else if (kind == CYC_PEER_IP) {
          ck.need(t.peer_cidr, "peer_cidr");
          ck.need(t.peer_except_off, "peer_except_off");
          p.cidr = S(t.peer_cidr[j], "peer_cidr", j);
          const int64_t e0 = t.peer_except_off[j], e1 = t.peer_except_off[j + 1];
          if (e0 < 0 || e1 < e0) ck.bad("peer_except_off decreases at " + std::to_string(j));
          if (e1 > e0) ck.need(t.except_cidr, "except_cidr");
          for (int64_t e = e0; e < e1; e++) p.except.push_back(S(t.except_cidr[e], "except_cidr", e));
          p.except_nil = t.peer_except_nil ? t.peer_except_nil[j] != 0 : e1 == e0;
          if (e1 > e0) p.except_nil = false;
        }
        tg.peers.push_back(std::move(p));
      }
      if (!tg.peers.empty()) tg.peers_nil = false;
      ir.dir[d].push_back(std::move(tg));
    }
  }
  for (int d = 0; d < 2; d++) {  // Policy.Ingress / Egress are maps keyed by primary key: one target per key
    std::sort(ir.dir[d].begin(), ir.dir[d].end(), [](const Target& a, const Target& b) { return a.pk < b.pk; });
    for (size_t i = 1; i < ir.dir[d].size(); i++)
      if (ir.dir[d][i].pk == ir.dir[d][i - 1].pk) ck.bad("two targets with primary key " + ir.dir[d][i].pk);
  }
  return ir;
}

// ============================================================================ probe model
static void decode_labels(const Node* n, bool& nil, std::map<std::string, std::string>& out) {
  nil = !n || n->null();
  if (nil) return;
  for (auto& kv : n->o) out[kv.first] = kv.second.null() ? "" : kv.second.str();
}

// Strings of the interned probe model: one table entry per distinct decoded string.
namespace {
struct StrTab {
  Resources& r;
  std::unordered_map<std::string, uint32_t> ids;
  explicit StrTab(Resources& res) : r(res) {}
  uint32_t operator()(const std::string& v) {
    auto it = ids.find(v);
    if (it != ids.end()) return it->second;
    const uint32_t id = uint32_t(r.str.size());
    r.str.push_back(v);
    ids.emplace(v, id);
    return id;
  }
};
}  // namespace

Resources load_resources(const Node& n) {
  Resources r;
  StrTab S(r);
  const uint32_t empty = S("");
  if (auto ns = n.val("Namespaces"); ns && ns->is_obj()) {
    std::unordered_map<std::string, size_t> last;  // a repeated key: the last one wins (Go map decode)
    for (size_t i = 0; i < ns->o.size(); i++) last[ns->o[i].first] = i;
    for (size_t i = 0; i < ns->o.size(); i++) {
      auto& kv = ns->o[i];
      if (last[kv.first] != i) continue;
      r.ns_name.push_back(S(kv.first));
      r.ns_nil.push_back(kv.second.null() ? 1 : 0);
      if (!kv.second.null())
        for (auto& l : kv.second.o) {
          r.ns_lab_key.push_back(S(l.first));
          r.ns_lab_val.push_back(l.second.null() ? empty : S(l.second.str()));
        }
      r.ns_lab_off.push_back(uint32_t(r.ns_lab_key.size()));
    }
  }
  if (auto pods = n.val("Pods"); pods && pods->is_arr()) {
    const size_t np = pods->a.size();
    r.pod_ns.reserve(np);
    r.pod_name.reserve(np);
    r.pod_ip.reserve(np);
    r.pod_lab_off.reserve(np + 1);
    r.pod_cont_off.reserve(np + 1);
    for (auto& p : pods->a) {
      const Node* x;
      r.pod_ns.push_back((x = p.sval("Namespace")) ? S(x->str()) : empty);
      r.pod_name.push_back((x = p.sval("Name")) ? S(x->str()) : empty);
      r.pod_ip.push_back((x = p.sval("IP")) ? S(x->str()) : empty);
      const Node* ls = p.val("Labels");
      const Node* cs = p.val("Containers");
      r.pod_nil.push_back(uint8_t((ls && ls->is_obj() ? 0 : 1) | (cs && cs->is_arr() ? 0 : 2)));
      if (ls && ls->is_obj())
        for (auto& kv : ls->o) {
          r.lab_key.push_back(S(kv.first));
          r.lab_val.push_back(kv.second.null() ? empty : S(kv.second.str()));
        }
      r.pod_lab_off.push_back(uint32_t(r.lab_key.size()));
      if (cs && cs->is_arr())
        for (auto& c : cs->a) {
          Container ct;
          ct.name = (x = c.sval("Name")) ? S(x->str()) : empty;
          ct.port = (x = c.sval("Port")) ? int32_t(x->i64()) : 0;
          ct.proto = (x = c.sval("Protocol")) ? S(x->str()) : empty;
          ct.port_name = (x = c.sval("PortName")) ? S(x->str()) : empty;
          r.conts.push_back(ct);
        }
      r.pod_cont_off.push_back(uint32_t(r.conts.size()));
    }
  }
  return r;
}

// json.Marshal(*probe.Resources) of the fields the verdict path reads (Pod.ServiceIP and
// Container.BatchJobs are not kept); map keys sorted as encoding/json writes them, a label map with
// a repeated key as Go would hold it (last value); nil maps and slices as null.
std::string dump_resources(const Resources& r) {
  auto labels = [&](const std::vector<uint32_t>& key, const std::vector<uint32_t>& val, uint32_t lo, uint32_t hi) {
    std::map<std::string, std::string> m;
    for (uint32_t j = lo; j < hi; j++) m[r.s(key[j])] = r.s(val[j]);
    std::string o = "{";
    for (auto& kv : m) o += (o.size() > 1 ? "," : "") + quote(kv.first) + ":" + quote(kv.second);
    return o + "}";
  };
  std::map<std::string, std::string> nss;
  for (size_t i = 0; i < r.ns_name.size(); i++)
    nss[r.s(r.ns_name[i])] = r.ns_nil[i] ? "null" : labels(r.ns_lab_key, r.ns_lab_val, r.ns_lab_off[i], r.ns_lab_off[i + 1]);
  std::string o = "{\"Namespaces\":{";
  bool first = true;
  for (auto& kv : nss) {
    o += (first ? "" : ",") + quote(kv.first) + ":" + kv.second;
    first = false;
  }
  o += "},\"Pods\":[";
  for (size_t p = 0; p < r.pods(); p++) {
    const uint8_t nil = p < r.pod_nil.size() ? r.pod_nil[p] : 0;
    o += (p ? "," : "") + std::string("{\"Namespace\":") + quote(r.s(r.pod_ns[p])) + ",\"Name\":" + quote(r.s(r.pod_name[p])) +
         ",\"Labels\":" + (nil & 1 ? std::string("null") : labels(r.lab_key, r.lab_val, r.pod_lab_off[p], r.pod_lab_off[p + 1])) +
         ",\"IP\":" + quote(r.s(r.pod_ip[p])) + ",\"Containers\":";
    if (nil & 2) {
      o += "null}";
      continue;
    }
    o += "[";
    for (uint32_t i = 0; i < r.n_conts(p); i++) {
      const Container& c = r.cont(p, i);
      o += (i ? "," : "") + std::string("{\"Name\":") + quote(r.s(c.name)) + ",\"Port\":" + std::to_string(c.port) +
           ",\"Protocol\":" + quote(r.s(c.proto)) + ",\"PortName\":" + quote(r.s(c.port_name)) + "}";
    }
    o += "]}";
  }
  return o + "]}";
}

// ---- flat tables (include/cyclonus_hip.h): validation helpers
namespace {
struct FlatCheck {
  const char* what;
  [[noreturn]] void bad(const std::string& m) const { throw Panic{CYC_ERR_ARG, std::string(what) + ": " + m}; }
  void need(const void* p, const char* name) const {
    if (!p) bad(std::string("null ") + name);
  }
  // offsets [n + 1], non-decreasing from >= 0: returns the element count they cover
  int64_t offsets(const int64_t* off, int64_t n, const char* name) const {
    if (n < 0) bad(std::string("negative count for ") + name);
    need(off, name);
    if (off[0] < 0) bad(std::string(name) + "[0] < 0");
    for (int64_t i = 0; i < n; i++)
      if (off[i + 1] < off[i]) bad(std::string(name) + " decreases at " + std::to_string(i));
    return off[n];
  }
  uint32_t index(int64_t v, int64_t n, const char* name, int64_t at) const {
    if (v < 0 || v >= n) bad(std::string(name) + "[" + std::to_string(at) + "] = " + std::to_string(v) + " out of range");
    return uint32_t(v);
  }
};
}  // namespace

Resources load_resources_tables(const cyc_resource_tables& t) {
  const FlatCheck ck{"cyc_resource_tables"};
  PhaseClock clk("resources_load");
  Resources r;
  // the caller's string table may repeat a string: every index maps to one canonical entry, so equal
  // ids <=> equal strings (Resources' invariant, which the name groups of the table build rely on)
  constexpr int64_t U32 = int64_t(1) << 32;  // ids, counts and offsets are kept as 32-bit values
  if (t.str.n >= U32) ck.bad("str.n = " + std::to_string(t.str.n) + ": more than 2^32 - 1 strings");
  ck.offsets(t.str.off, t.str.n, "str.off");
  if (t.str.n && t.str.off[t.str.n] > t.str.off[0]) ck.need(t.str.bytes, "str.bytes");
  std::vector<uint32_t> canon(size_t(t.str.n));
  {
    BytesMap seen;
    seen.reserve(size_t(t.str.n), size_t(t.str.n ? t.str.off[t.str.n] - t.str.off[0] : 0));
    for (int64_t i = 0; i < t.str.n; i++) canon[size_t(i)] = seen.get(t.str.bytes + t.str.off[i], size_t(t.str.off[i + 1] - t.str.off[i]));
    r.str.resize(seen.size());
    for (uint32_t k = 0; k < seen.size(); k++) r.str[k] = std::string(seen.key(k));
  }
  clk.lap("strings");
  const int64_t n_str = t.str.n;
  auto id = [&](int64_t v, const char* name, int64_t at) { return canon[ck.index(v, n_str, name, at)]; };
  if (t.n_namespaces < 0 || t.n_pods < 0) ck.bad("negative count");
  if (t.n_namespaces >= U32) ck.bad("n_namespaces = " + std::to_string(t.n_namespaces) + ": more than 2^32 - 1 namespaces");
  if (t.n_pods >= U32) ck.bad("n_pods = " + std::to_string(t.n_pods) + ": more than 2^32 - 1 pods");
  if (t.n_namespaces) {
    ck.need(t.ns_name, "ns_name");
    const int64_t nl = ck.offsets(t.ns_label_off, t.n_namespaces, "ns_label_off");
    if (nl - t.ns_label_off[0] >= U32) ck.bad("more than 2^32 - 1 namespace labels");
    if (nl) {
      ck.need(t.ns_label_key, "ns_label_key");
      ck.need(t.ns_label_val, "ns_label_val");
    }
    // a repeated key: the last one wins (a Go map has none; this mirrors the JSON loader)
    std::unordered_map<uint32_t, int64_t> last;
    for (int64_t i = 0; i < t.n_namespaces; i++) last[id(t.ns_name[i], "ns_name", i)] = i;
    for (int64_t i = 0; i < t.n_namespaces; i++) {
      const uint32_t name = canon[uint32_t(t.ns_name[i])];
      if (last[name] != i) continue;
      r.ns_name.push_back(name);
      r.ns_nil.push_back(t.ns_nil && t.ns_nil[i] ? 1 : 0);
      for (int64_t j = t.ns_label_off[i]; j < t.ns_label_off[i + 1] && !r.ns_nil.back(); j++) {
        r.ns_lab_key.push_back(id(t.ns_label_key[j], "ns_label_key", j));
        r.ns_lab_val.push_back(id(t.ns_label_val[j], "ns_label_val", j));
      }
      r.ns_lab_off.push_back(uint32_t(r.ns_lab_key.size()));
    }
  }
  const int64_t P = t.n_pods;
  if (P) {
    ck.need(t.pod_ns, "pod_ns");
    ck.need(t.pod_name, "pod_name");
    ck.need(t.pod_ip, "pod_ip");
    const int64_t nl = ck.offsets(t.pod_label_off, P, "pod_label_off");
    const int64_t nc = ck.offsets(t.pod_cont_off, P, "pod_cont_off");
    const int64_t l0 = t.pod_label_off[0], c0 = t.pod_cont_off[0];
    if (nl > l0) {
      ck.need(t.label_key, "label_key");
      ck.need(t.label_val, "label_val");
    }
    if (nc > c0) {
      ck.need(t.cont_name, "cont_name");
      ck.need(t.cont_port, "cont_port");
      ck.need(t.cont_proto, "cont_proto");
      ck.need(t.cont_port_name, "cont_port_name");
    }
    if (nl - l0 >= U32 || nc - c0 >= U32) ck.bad("more than 2^32 - 1 labels or containers");
    r.pod_ns.resize(size_t(P));
    r.pod_name.resize(size_t(P));
    r.pod_ip.resize(size_t(P));
    r.pod_lab_off.assign(size_t(P) + 1, 0);
    r.pod_cont_off.assign(size_t(P) + 1, 0);
    r.pod_nil.assign(size_t(P), 0);
    for (int64_t p = 0; p < P; p++) {
      r.pod_ns[size_t(p)] = id(t.pod_ns[p], "pod_ns", p);
      r.pod_name[size_t(p)] = id(t.pod_name[p], "pod_name", p);
      r.pod_ip[size_t(p)] = id(t.pod_ip[p], "pod_ip", p);
      r.pod_lab_off[size_t(p) + 1] = uint32_t(t.pod_label_off[p + 1] - l0);
      r.pod_cont_off[size_t(p) + 1] = uint32_t(t.pod_cont_off[p + 1] - c0);
      if (t.pod_nil) {  // a nil map / slice holds nothing
        r.pod_nil[size_t(p)] = t.pod_nil[p] & 3;
        if ((t.pod_nil[p] & 1) && t.pod_label_off[p + 1] > t.pod_label_off[p]) ck.bad("pod_nil[" + std::to_string(p) + "]: nil Labels with labels");
        if ((t.pod_nil[p] & 2) && t.pod_cont_off[p + 1] > t.pod_cont_off[p]) ck.bad("pod_nil[" + std::to_string(p) + "]: nil Containers with containers");
      }
    }
    r.lab_key.resize(size_t(nl - l0));
    r.lab_val.resize(size_t(nl - l0));
    for (int64_t j = l0; j < nl; j++) {
      r.lab_key[size_t(j - l0)] = id(t.label_key[j], "label_key", j);
      r.lab_val[size_t(j - l0)] = id(t.label_val[j], "label_val", j);
    }
    r.conts.resize(size_t(nc - c0));
    for (int64_t j = c0; j < nc; j++) {
      Container& c = r.conts[size_t(j - c0)];
      c.name = id(t.cont_name[j], "cont_name", j);
      c.port = t.cont_port[j];
      c.proto = id(t.cont_proto[j], "cont_proto", j);
      c.port_name = id(t.cont_port_name[j], "cont_port_name", j);
    }
  }
  if (r.str.empty()) r.str.push_back("");  // (ids of absent fields are never read; keep the table non-empty)
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

std::vector<ProbeConfig> load_probe_configs(const cyc_probe_config* cfgs, int64_t n) {
  if (n < 0 || (n && !cfgs)) throw Panic{CYC_ERR_ARG, "cyc_probe_config: null or negative count"};
  std::vector<ProbeConfig> out(static_cast<size_t>(n));
  for (int64_t i = 0; i < n; i++) {
    ProbeConfig& c = out[size_t(i)];
    c.all_available = cfgs[i].all_available != 0;
    if (c.all_available) continue;
    auto str = [&](const char* p, int64_t n, const char* name) {
      if (n < 0 || (n && !p))
        throw Panic{CYC_ERR_ARG, "cyc_probe_config[" + std::to_string(i) + "]." + name + ": null pointer or negative length"};
      return std::string(p ? p : "", size_t(n));
    };
    c.port.is_str = cfgs[i].port_is_name != 0;
    if (c.port.is_str) c.port.s = str(cfgs[i].port_name_ptr, cfgs[i].port_name_len, "port_name");
    else c.port.i = cfgs[i].port;
    c.proto = str(cfgs[i].protocol_ptr, cfgs[i].protocol_len, "protocol");
  }
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
  BytesMap ls_ids;   // label set id = its id here (0 = the empty map)
  BytesMap sel_ids;  // selector id = its id here
  std::unordered_map<std::string, uint32_t> cidr_ids;
  std::unordered_map<uint64_t, std::vector<uint32_t>> desc_ids;  // (name, protocol) -> descriptors by port
  std::unordered_map<int, uint32_t> pm_ids;
  const PolicyIR& ir;

  Flattener(Problem& p, const PolicyIR& i) : pb(p), ir(i) {
    pb.ls_off = {0};
    ls_ids.get("", 0);  // label set 0 == empty map (nil behaves the same for reads)
    pb.ls_off.push_back(0);
    pb.sel_off = {0};
  }

  // A label map as (key id, value id) pairs of the problem's dictionary, keys unique: sorted here,
  // then looked up by their raw bytes (every map with the same contents gets the same set)
  uint32_t label_set(std::vector<std::pair<uint32_t, uint32_t>>& kvs) {
    if (kvs.empty()) return 0;
    std::sort(kvs.begin(), kvs.end());
    bool added = false;
    const uint32_t id = ls_ids.get(reinterpret_cast<const char*>(kvs.data()), kvs.size() * sizeof(kvs[0]), &added);
    if (!added) return id;
    for (auto& kv : kvs) {
      pb.ls_key.push_back(kv.first);
      pb.ls_val.push_back(kv.second);
    }
    pb.ls_off.push_back(uint32_t(pb.ls_key.size()));
    return id;
  }
  uint32_t label_set(const std::map<std::string, std::string>& l) {
    std::vector<std::pair<uint32_t, uint32_t>> kvs;
    for (auto& kv : l) kvs.emplace_back(pb.intern(kv.first), pb.intern(kv.second));
    return label_set(kvs);
  }

  // a selector's identity: its matchLabels (sorted) and expressions, length-prefixed into one key
  std::string sel_key;
  void key_str(const std::string& x) {
    const uint32_t n = uint32_t(x.size());
    sel_key.append(reinterpret_cast<const char*>(&n), 4);
    sel_key.append(x);
  }
  uint32_t selector(const Selector& s) {
    sel_key.clear();
    for (auto& kv : s.labels) {
      key_str(kv.first);
      key_str(kv.second);
    }
    sel_key.push_back('\x01');
    for (auto& e : s.exprs) {
      key_str(e.key);
      key_str(e.op);
      const uint32_t nv = uint32_t(e.values.size());
      sel_key.append(reinterpret_cast<const char*>(&nv), 4);
      for (auto& v : e.values) key_str(v);
    }
    bool added = false;
    const uint32_t id = sel_ids.get(sel_key.data(), sel_key.size(), &added);
    if (!added) return id;
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
    pb.sel_off.push_back(uint32_t(pb.reqs.size()));
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

  // job descriptor (ResolvedPort, ResolvedPortName id, Protocol id)
  uint32_t desc(int32_t port, uint32_t n, uint32_t p) {
    const uint64_t k1 = (uint64_t(n) << 32) | p;
    auto it = desc_ids.find(k1);
    if (it != desc_ids.end())
      for (uint32_t id : it->second)
        if (pb.descs[id].port == port) return id;
    uint32_t id = uint32_t(pb.descs.size());
    pb.descs.push_back(DDesc{port, n, p, 0});
    desc_ids[k1].push_back(id);
    return id;
  }
  uint32_t desc(int32_t port, const std::string& name, const std::string& proto) { return desc(port, pb.intern(name), pb.intern(proto)); }
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
// Name groups of pods [q0, q1) — pods sharing their PodString "ns/name" share Items: grp[p] = the
// group's first pod.  Grouped by the (ns, name) pair of string ids (equal ids <=> equal strings in a
// Resources), which is the same relation as the joined string unless a namespace or name holds a '/'
// (then by the string itself).
static void name_groups(const Resources& res, uint32_t q0, uint32_t q1, std::vector<uint32_t>& grp) {
  grp.assign(q1, 0);
  bool slash = false;
  for (uint32_t p = q0; p < q1 && !slash; p++)
    slash = res.s(res.pod_ns[p]).find('/') != std::string::npos || res.s(res.pod_name[p]).find('/') != std::string::npos;
  if (slash) {
    std::unordered_map<std::string, uint32_t> first_of;
    for (uint32_t p = q0; p < q1; p++) grp[p] = first_of.emplace(res.pod_string(p), p).first->second;
    return;
  }
  U64Map first_of(q1 - q0);
  for (uint32_t p = q0; p < q1; p++) grp[p] = first_of.emplace((uint64_t(res.pod_ns[p]) << 32) | res.pod_name[p], p);
}

static std::string table_build_error(const Resources& res, const Problem& pb, const ProbeConfig& pc, uint32_t koff,
                                     uint32_t q0, uint32_t q1) {
  const uint32_t P = q1;
  if (q1 <= q0) return "";
  std::vector<uint32_t> grp;
  name_groups(res, q0, q1, grp);
  uint32_t s_b = P;  // the first pod that is not the first of its name group
  std::vector<uint8_t> multi(P, 0);  // the pod's name group has other pods
  for (uint32_t p = q0; p < P; p++)
    if (grp[p] != p) {
      if (s_b == P) s_b = p;
      multi[p] = multi[grp[p]] = 1;
    }
  // a job's key Protocol/ResolvedPort (job.go:23-25) as (protocol id, port)
  struct DJob {
    uint32_t d, i;  // destination pod, container index (AllAvailable) or 0
    uint32_t proto;
    int32_t port;
  };
  // PortProtocol jobs all carry the config's protocol: their keys differ by port only
  const uint32_t pc_proto = 0;
  std::vector<DJob> jobs[3];
  for (uint32_t d = q0; d < P; d++) {
    const size_t base = size_t(d) * pb.K + koff;
    if (pc.all_available) {
      for (uint32_t i = 0; i < res.n_conts(d); i++) jobs[0].push_back({d, i, res.cont(d, i).proto, res.cont(d, i).port});
      continue;
    }
    const uint8_t st = pb.slot_status[base];
    int port = -1;  // ResolvedPort: -1 for a named port that does not resolve (resources.go:303-308)
    if (st == CYC_JOB_VALID) port = pb.descs[size_t(pb.slot_desc[base])].port;
    else if (st == CYC_JOB_BAD_PORT_PROTOCOL) port = pc.port.i;
    const int cat = st == CYC_JOB_VALID ? 0 : st == CYC_JOB_BAD_PORT_PROTOCOL ? 1 : 2;
    jobs[cat].push_back({d, 0, pc_proto, port});
  }
  // (name group, key) pairs seen so far: a pod alone in its group can only repeat a key among its
  // own jobs (its containers, AllAvailable), checked in place; groups of several pods share a set
  struct GK {
    uint32_t g, proto;
    int32_t port;
    bool operator<(const GK& o) const { return std::tie(g, proto, port) < std::tie(o.g, o.proto, o.port); }
  };
  std::set<GK> seen;
  auto repeats = [&](const DJob& j, const std::vector<DJob>& js, size_t at) {
    if (multi[j.d]) return !seen.insert(GK{grp[j.d], j.proto, j.port}).second;
    // the pod's earlier jobs of this category are the entries just before it (same d)
    for (size_t x = at; x-- > 0 && js[x].d == j.d;)
      if (js[x].proto == j.proto && js[x].port == j.port) return true;
    return false;
  };
  auto key_text = [&](const DJob& j) {
    const std::string& proto = pc.all_available ? res.s(res.cont(j.d, j.i).proto) : pc.proto;
    return proto + "/" + std::to_string(j.port);
  };
  auto message = [&](const DJob& j, uint32_t from) {
    const std::string to_cont = pc.all_available ? res.s(res.cont(j.d, j.i).name) : "";
    return "unable to add job result: duplicate key " + key_text(j) + " (job {FromKey:" + res.pod_string(from) +
           " ToKey:" + res.pod_string(j.d) + " ToContainer:" + to_cont + "})";
  };
  for (int cat = 0; cat < 3; cat++) {
    const DJob* hit = nullptr;
    for (size_t x = 0; x < jobs[cat].size() && !hit; x++)
      if (repeats(jobs[cat][x], jobs[cat], x)) hit = &jobs[cat][x];
    if (!hit && s_b < P && !jobs[cat].empty()) return message(jobs[cat][0], s_b);
    if (hit) return message(*hit, q0);
  }
  return "";
}

// Problem dictionary ids of the resources' strings, interned on first use.
namespace {
struct ResIds {
  Problem& pb;
  const Resources& res;
  std::vector<uint32_t> sid;
  ResIds(Problem& p, const Resources& r) : pb(p), res(r), sid(r.str.size(), UINT32_MAX) {}
  uint32_t operator()(uint32_t r) {
    uint32_t& x = sid[r];
    if (x == UINT32_MAX) x = pb.intern(res.str[r]);
    return x;
  }
};
}  // namespace

Problem build_problem(const PolicyIR& ir, const Resources& res, const std::vector<ProbeConfig>& probes,
                      const std::vector<ProbeBlock>* blocks) {
  Problem pb;
  PhaseClock clk("build_problem");
  Flattener F(pb, ir);
  ResIds R(pb, res);
  pb.P = uint32_t(res.pods());
  pb.W = (pb.P + 63) / 64;
  if (blocks) {  // batched blocks: consecutive pod ranges covering the pods, namespaces private to a block
    pb.blocks = *blocks;
    pb.pod_blk.assign(pb.P, 0);
    uint32_t at = 0;
    std::unordered_map<uint32_t, uint32_t> ns_blk;
    for (uint32_t b = 0; b < blocks->size(); b++) {
      const ProbeBlock& bl = (*blocks)[b];
      if (bl.p0 != at || bl.p1 < bl.p0 || bl.p1 > pb.P || bl.cfg >= probes.size())
        throw Panic{CYC_ERR_ARG, "blocks must be consecutive pod ranges covering the pods, each with a probe config"};
      for (uint32_t q = bl.p0; q < bl.p1; q++) {
        pb.pod_blk[q] = b;
        // a namespace's targets apply to all its pods (TargetsApplyingToPod policy.go:68-82): a block's
        // problem is its own only if no other block has pods in its namespaces
        auto it = ns_blk.emplace(R(res.pod_ns[q]), b).first;
        if (it->second != b) throw Panic{CYC_ERR_ARG, "namespace " + res.s(res.pod_ns[q]) + " has pods in two blocks"};
      }
      at = bl.p1;
    }
    if (at != pb.P) throw Panic{CYC_ERR_ARG, "blocks must cover every pod"};
  }

  // ---- namespaces: r.Namespaces[ns] (nil when absent) as a label set, by namespace id
  std::unordered_map<uint32_t, uint32_t> ns_ls;
  std::vector<std::pair<uint32_t, uint32_t>> kvs;
  auto labels = [&](const std::vector<uint32_t>& key, const std::vector<uint32_t>& val, uint32_t lo, uint32_t hi) {
    // a Go map: each key once (a repeated key in the input: the last one wins)
    kvs.clear();
    for (uint32_t j = lo; j < hi; j++) kvs.emplace_back(R(key[j]), R(val[j]));
    if (kvs.size() > 1) {
      std::stable_sort(kvs.begin(), kvs.end(), [](auto& a, auto& b) { return a.first < b.first; });
      size_t w = 0;
      for (size_t j = 0; j < kvs.size(); j++) {
        if (w && kvs[w - 1].first == kvs[j].first) kvs[w - 1] = kvs[j];
        else kvs[w++] = kvs[j];
      }
      kvs.resize(w);
    }
    return F.label_set(kvs);
  };
  for (size_t i = 0; i < res.ns_name.size(); i++)
    ns_ls[R(res.ns_name[i])] = res.ns_nil[i] ? 0u : labels(res.ns_lab_key, res.ns_lab_val, res.ns_lab_off[i], res.ns_lab_off[i + 1]);

  // ---- pods
  bool any_bad_ip = false;
  pb.pod_ns.resize(pb.P);
  pb.pod_ls.resize(pb.P);
  pb.pod_nsls.resize(pb.P);
  pb.pod_ip.resize(pb.P);
  pb.pod_ip_str.assign(pb.P, std::string());
  std::vector<DIP> ip_of(res.str.size());  // an IP string parsed once
  std::vector<uint8_t> ip_done(res.str.size(), 0);
  for (uint32_t p = 0; p < pb.P; p++) {
    const uint32_t ns = R(res.pod_ns[p]);
    pb.pod_ns[p] = ns;
    pb.pod_ls[p] = labels(res.lab_key, res.lab_val, res.pod_lab_off[p], res.pod_lab_off[p + 1]);
    auto it = ns_ls.find(ns);
    pb.pod_nsls[p] = it == ns_ls.end() ? 0u : it->second;
    const uint32_t ips = res.pod_ip[p];
    if (!ip_done[ips]) {
      ip_of[ips] = parse_ip(res.s(ips));
      ip_done[ips] = 1;
    }
    pb.pod_ip[p] = ip_of[ips];
    if (!pb.pod_ip[p].valid) {
      any_bad_ip = true;
      pb.pod_ip_str[p] = res.s(ips);
    }
  }

  clk.lap("pods");
  bool any_ip_peer = flatten_targets(pb, F, ir);
  if (any_ip_peer && any_bad_ip) pb.may_err = true;
  clk.lap("targets");

  // ---- probe job slots (resources.go:274-364, resolved per destination pod)
  size_t maxc = 0;
  for (uint32_t p = 0; p < pb.P; p++) maxc = std::max<size_t>(maxc, res.n_conts(p));
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
    for (uint32_t p = 0; p < pb.P; p++) (res.n_conts(p) == 0 ? bare : any_cont) = true;
    for (size_t c = 0; c < probes.size(); c++)  // PortProtocol: every (from, to) pair builds a job;
      pb.expand_panic[c] = bare && (probes[c].all_available ? any_cont : true);  // AllAvailable: one per dst container
    pb.blk_expand_panic.assign(pb.blocks.size(), 0);
    for (size_t b = 0; b < pb.blocks.size(); b++) {  // the same, per block over its own pods
      bool bb = false, bc = false;
      for (uint32_t q = pb.blocks[b].p0; q < pb.blocks[b].p1; q++) (res.n_conts(q) == 0 ? bb : bc) = true;
      pb.blk_expand_panic[b] = bb && (probes[pb.blocks[b].cfg].all_available ? bc : true);
    }
  }
  for (size_t c = 0; c < probes.size(); c++) {
    const ProbeConfig& pc = probes[c];
    const uint32_t proto = pb.intern(pc.proto), pname = pc.port.is_str ? pb.intern(pc.port.s) : 0u;
    for (uint32_t d = 0; d < pb.P; d++) {
      if (!pb.blocks.empty() && pb.blocks[pb.pod_blk[d]].cfg != c) continue;  // a block answers its config only
      const size_t base = size_t(d) * pb.K + cfg_off[c];
      const uint32_t nc = res.n_conts(d);
      if (pc.all_available) {  // GetJobsAllAvailableServers :336-364
        for (uint32_t i = 0; i < nc; i++) {
          const Container& ct = res.cont(d, i);
          pb.slot_desc[base + i] = int32_t(F.desc(ct.port, R(ct.port_name), R(ct.proto)));
          pb.slot_status[base + i] = CYC_JOB_VALID;
        }
        continue;
      }
      // GetJobsForNamedPortProtocol :284-334 (every pair gets a job)
      const Container* hit = nullptr;
      for (uint32_t i = 0; i < nc && !hit; i++) {
        const Container& ct = res.cont(d, i);
        if (pc.port.is_str ? R(ct.port_name) == pname : ct.port == pc.port.i) hit = &ct;
      }
      if (pc.port.is_str) {  // ResolveNamedPort pod.go:132-139
        if (hit) {
          pb.slot_desc[base] = int32_t(F.desc(hit->port, pname, proto));
          pb.slot_status[base] = CYC_JOB_VALID;
        } else {
          pb.slot_status[base] = CYC_JOB_BAD_NAMED_PORT;
        }
      } else {  // ResolveNumberedPort pod.go:141-148 (protocol ignored)
        if (hit) {
          pb.slot_desc[base] = int32_t(F.desc(pc.port.i, R(hit->port_name), proto));
          pb.slot_status[base] = CYC_JOB_VALID;
        } else {
          pb.slot_status[base] = CYC_JOB_BAD_PORT_PROTOCOL;
        }
      }
    }
    clk.lap("job slots");
    if (pb.blocks.empty()) pb.dup_key_msg[c] = table_build_error(res, pb, pc, cfg_off[c], 0, pb.P);
    clk.lap("table build");
  }
  pb.blk_dup_msg.assign(pb.blocks.size(), "");
  for (size_t b = 0; b < pb.blocks.size(); b++) {
    const ProbeBlock& bl = pb.blocks[b];
    pb.blk_dup_msg[b] = table_build_error(res, pb, probes[bl.cfg], cfg_off[bl.cfg], bl.p0, bl.p1);
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

// The flat form of load_traffics (include/cyclonus_hip.h cyc_traffic_tables): every index and
// offset validated, CYC_ERR_ARG naming the first bad one.
std::vector<QueryTraffic> load_traffic_tables(const cyc_traffic_tables& t) {
  const FlatCheck ck{"cyc_traffic_tables"};
  if (t.n < 0 || t.n >= (int64_t(1) << 31)) ck.bad("n = " + std::to_string(t.n) + " out of range");
  if (t.str.n < 0) ck.bad("negative str.n");
  ck.offsets(t.str.off, t.str.n, "str.off");
  if (t.str.n && t.str.off[t.str.n] > t.str.off[0]) ck.need(t.str.bytes, "str.bytes");
  auto S = [&](int64_t i, const char* name, int64_t at) {
    ck.index(i, t.str.n, name, at);
    return std::string(t.str.bytes + t.str.off[i], size_t(t.str.off[i + 1] - t.str.off[i]));
  };
  std::vector<QueryTraffic> out(size_t(t.n));
  if (!t.n) return out;
  const int64_t ne = 2 * t.n;
  ck.need(t.internal, "internal");
  ck.need(t.ip, "ip");
  ck.need(t.port, "port");
  ck.need(t.port_name, "port_name");
  ck.need(t.protocol, "protocol");
  const int64_t nl = t.label_off ? ck.offsets(t.label_off, ne, "label_off") : 0;
  const int64_t nn = t.ns_label_off ? ck.offsets(t.ns_label_off, ne, "ns_label_off") : 0;
  if (t.label_off && nl > t.label_off[0]) {
    ck.need(t.label_key, "label_key");
    ck.need(t.label_val, "label_val");
  }
  if (t.ns_label_off && nn > t.ns_label_off[0]) {
    ck.need(t.ns_label_key, "ns_label_key");
    ck.need(t.ns_label_val, "ns_label_val");
  }
  for (int64_t e = 0; e < ne; e++) {
    QueryTraffic& q = out[size_t(e / 2)];
    QueryEnd& x = e % 2 ? q.dst : q.src;
    x.ip = S(t.ip[e], "ip", e);
    x.external = !t.internal[e];
    if (x.external) continue;
    ck.need(t.ns, "ns");
    x.ns = S(t.ns[e], "ns", e);
    if (t.label_off)  // a Go map: a repeated key, if given, keeps its last value
      for (int64_t j = t.label_off[e]; j < t.label_off[e + 1]; j++) x.labels[S(t.label_key[j], "label_key", j)] = S(t.label_val[j], "label_val", j);
    if (t.ns_label_off)
      for (int64_t j = t.ns_label_off[e]; j < t.ns_label_off[e + 1]; j++)
        x.ns_labels[S(t.ns_label_key[j], "ns_label_key", j)] = S(t.ns_label_val[j], "ns_label_val", j);
  }
  for (int64_t i = 0; i < t.n; i++) {
    out[size_t(i)].port = t.port[i];
    out[size_t(i)].port_name = S(t.port_name[i], "port_name", i);
    out[size_t(i)].proto = S(t.protocol[i], "protocol", i);
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
