// capi_driver.cpp — a C++ client of libcyclonus_hip's C ABI, standing in for the cgo binding a
// maintainer would add at the reference's JobRunner seam (pkg/connectivity/probe/jobrunner.go:60-62;
// INTEGRATION.md §1).  It drives exactly the calls that binding makes for RunProbeForConfig:
//   cyc_ctx_create -> cyc_policy_build_json -> cyc_policy_ir_json -> cyc_resources_load_json ->
//   cyc_probe_prepare -> cyc_table_run -> cyc_table_cells -> cyc_table_destroy -> cyc_ctx_destroy
// and prints every cell's (ingress, egress, combined) Connectivity as ShortString characters
// (connectivity.go:27-42), one line per (source, destination): "s d <in><eg><comb> per slot".
// With --flat it drives the binding's flat-table form instead (no JSON crosses the ABI):
//   cyc_ctx_create -> cyc_policy_load -> cyc_resources_load -> cyc_probe_prepare_configs -> ...
// reading the tables from field dumps (cyclonus_amd/flat.py dump_tables: "name kind count" lines,
// each followed by the raw array) and the probe configs from text lines ("all" / "int PORT PROTO" /
// "name NAME PROTO").
//
//   capi_driver POLICIES.json RESOURCES.json PROBES.json [--no-gpu]
//   capi_driver --flat POLICY.tab RESOURCES.tab PROBES.txt [--no-gpu]
// --no-gpu stops before the probe: the compiled (or loaded) policy in json.Marshal form, and with
// --flat also the loaded probe.Resources.
// Exit status: 0 ok, 2 usage / file error, 3 a library call failed (the status and
// cyc_last_error text are printed, e.g. the reference's panic message).
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "cyclonus_hip.h"

static std::string slurp(const char* path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) {
    std::fprintf(stderr, "cannot read %s\n", path);
    std::exit(2);
  }
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

static void check(cyc_ctx* ctx, int rc, const char* what) {
  if (rc == CYC_OK) return;
  std::printf("error %s rc=%d: %s\n", what, rc, cyc_last_error(ctx));
  std::exit(3);
}

static char short_string(uint8_t c) {  // connectivity.go:27-42; '-' = no job in the slot
  switch (c) {
    case CYC_CONN_UNKNOWN: return '?';
    case CYC_CONN_CHECK_FAILED: return '!';
    case CYC_CONN_BLOCKED: return 'X';
    case CYC_CONN_ALLOWED: return '.';
    case CYC_CONN_INVALID_NAMED_PORT: return 'P';
    case CYC_CONN_INVALID_PORT_PROTOCOL: return 'N';
    default: return '-';
  }
}

// A field dump of one tables struct: name -> raw bytes (absent = NULL).
struct Dump {
  std::map<std::string, std::string> f;
  explicit Dump(const std::string& text) {
    size_t at = 0;
    while (at < text.size()) {
      const size_t nl = text.find('\n', at);
      if (nl == std::string::npos) break;
      std::istringstream head(text.substr(at, nl - at));
      std::string name, kind;
      long long count = 0;
      head >> name >> kind >> count;
      at = nl + 1;
      if (count < 0) continue;
      const size_t bytes = size_t(count) * (kind == "i64" ? 8 : kind == "i32" ? 4 : 1);
      if (at + bytes > text.size()) {
        std::fprintf(stderr, "truncated table dump at %s\n", name.c_str());
        std::exit(2);
      }
      f[name] = text.substr(at, bytes);
      at += bytes;
    }
  }
  template <class T>
  const T* ptr(const char* name) const {
    const auto it = f.find(name);
    return it == f.end() ? nullptr : reinterpret_cast<const T*>(it->second.data());
  }
  int64_t i64(const char* name, int x = 0) const {
    const int64_t* p = ptr<int64_t>(name);
    return p ? p[x] : 0;
  }
  cyc_strings strings() const { return cyc_strings{i64("str.n"), ptr<char>("str.bytes"), ptr<int64_t>("str.off")}; }
};

#define I32(t, d, x) t.x = d.ptr<int32_t>(#x)
#define I64(t, d, x) t.x = d.ptr<int64_t>(#x)
#define U8(t, d, x) t.x = d.ptr<uint8_t>(#x)

static cyc_resource_tables resource_tables(const Dump& d) {
  cyc_resource_tables t{};
  t.str = d.strings();
  t.n_namespaces = d.i64("n_namespaces");
  I32(t, d, ns_name);
  U8(t, d, ns_nil);
  I64(t, d, ns_label_off);
  I32(t, d, ns_label_key);
  I32(t, d, ns_label_val);
  t.n_pods = d.i64("n_pods");
  I32(t, d, pod_ns);
  I32(t, d, pod_name);
  I32(t, d, pod_ip);
  I64(t, d, pod_label_off);
  I32(t, d, label_key);
  I32(t, d, label_val);
  I64(t, d, pod_cont_off);
  I32(t, d, cont_name);
  I32(t, d, cont_port);
  I32(t, d, cont_proto);
  I32(t, d, cont_port_name);
  U8(t, d, pod_nil);
  return t;
}

static cyc_policy_tables policy_tables(const Dump& d) {
  cyc_policy_tables t{};
  t.str = d.strings();
  t.n_selectors = d.i64("n_selectors");
  I64(t, d, sel_label_off);
  I32(t, d, sel_label_key);
  I32(t, d, sel_label_val);
  I64(t, d, sel_expr_off);
  I32(t, d, expr_key);
  I32(t, d, expr_op);
  I64(t, d, expr_value_off);
  I32(t, d, expr_value);
  t.n_port_matchers = d.i64("n_port_matchers");
  U8(t, d, pm_all);
  U8(t, d, pm_ports_nil);
  U8(t, d, pm_ranges_nil);
  I64(t, d, pm_port_off);
  U8(t, d, port_kind);
  I32(t, d, port_value);
  I32(t, d, port_proto);
  I64(t, d, pm_range_off);
  I32(t, d, range_from);
  I32(t, d, range_to);
  I32(t, d, range_proto);
  t.n_targets[0] = d.i64("n_targets", 0);
  t.n_targets[1] = d.i64("n_targets", 1);
  I32(t, d, target_ns);
  I32(t, d, target_sel);
  U8(t, d, target_peers_nil);
  I64(t, d, target_peer_off);
  I64(t, d, target_rule_off);
  I32(t, d, rule_name);
  U8(t, d, peer_kind);
  I32(t, d, peer_port);
  U8(t, d, peer_ns_kind);
  I32(t, d, peer_ns);
  I32(t, d, peer_pod_sel);
  I32(t, d, peer_cidr);
  I64(t, d, peer_except_off);
  U8(t, d, peer_except_nil);
  I32(t, d, except_cidr);
  return t;
}

// generator.ProbeConfig lines: "all" | "int PORT PROTO" | "name NAME PROTO" (PROTO may be absent = "")
struct Configs {
  std::vector<std::string> names, protos;
  std::vector<cyc_probe_config> c;
  explicit Configs(const std::string& text) {
    std::istringstream in(text);
    std::string line;
    std::vector<std::string> kinds, ports;
    while (std::getline(in, line)) {
      std::istringstream l(line);
      std::string kind, port, proto;
      if (!(l >> kind)) continue;
      l >> port >> proto;
      kinds.push_back(kind);
      ports.push_back(port);
      protos.push_back(proto);
    }
    names = ports;  // (stable storage for the c_str pointers below)
    c.resize(kinds.size());
    for (size_t i = 0; i < kinds.size(); i++) {
      c[i] = cyc_probe_config{};
      if (kinds[i] == "all") {
        c[i].all_available = 1;
        continue;
      }
      c[i].protocol_ptr = protos[i].data();
      c[i].protocol_len = int64_t(protos[i].size());
      if (kinds[i] == "name") {
        c[i].port_is_name = 1;
        c[i].port_name_ptr = names[i].data();
        c[i].port_name_len = int64_t(names[i].size());
      } else {
        c[i].port = int32_t(std::stol(ports[i]));
      }
    }
  }
};

static std::string ir_json(cyc_ctx* ctx) {
  const int64_t need = cyc_policy_ir_json(ctx, nullptr, 0);
  std::vector<char> ir(size_t(need > 0 ? need : 1));
  cyc_policy_ir_json(ctx, ir.data(), ir.size());
  return ir.data();
}

int main(int argc, char** argv) {
  const bool flat = argc > 1 && std::strcmp(argv[1], "--flat") == 0;
  if (flat) {
    argv++;
    argc--;
  }
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s [--flat] POLICIES RESOURCES PROBES [--no-gpu]\n", argv[0]);
    return 2;
  }
  const bool no_gpu = argc > 4 && std::strcmp(argv[4], "--no-gpu") == 0;
  const std::string pols = slurp(argv[1]), res = slurp(argv[2]), probes = slurp(argv[3]);
  cyc_ctx* ctx = nullptr;
  check(nullptr, cyc_ctx_create(0, &ctx), "cyc_ctx_create");
  cyc_probe_shape shape{};
  if (flat) {
    const Dump pd(pols), rd(res);
    const cyc_policy_tables pt = policy_tables(pd);
    check(ctx, cyc_policy_load(ctx, &pt), "cyc_policy_load");
    const cyc_resource_tables rt = resource_tables(rd);
    check(ctx, cyc_resources_load(ctx, &rt), "cyc_resources_load");
    if (no_gpu) {
      const int64_t need = cyc_resources_json(ctx, nullptr, 0);
      std::vector<char> rj(size_t(need > 0 ? need : 1));
      cyc_resources_json(ctx, rj.data(), rj.size());
      std::printf("ir %s\nresources %s\n", ir_json(ctx).c_str(), rj.data());
      cyc_ctx_destroy(ctx);
      return 0;
    }
    const Configs cf(probes);
    check(ctx, cyc_probe_prepare_configs(ctx, cf.c.data(), int64_t(cf.c.size()), &shape), "cyc_probe_prepare_configs");
  } else {
    check(ctx, cyc_policy_build_json(ctx, 1, pols.data(), pols.size()), "cyc_policy_build_json");
    if (no_gpu) {
      std::printf("ir %s\n", ir_json(ctx).c_str());
      cyc_ctx_destroy(ctx);
      return 0;
    }
    check(ctx, cyc_resources_load_json(ctx, res.data(), res.size()), "cyc_resources_load_json");
    check(ctx, cyc_probe_prepare(ctx, probes.data(), probes.size(), &shape), "cyc_probe_prepare");
  }
  const int64_t P = shape.pods, K = shape.slots;
  cyc_table* table = nullptr;
  check(ctx, cyc_table_run(ctx, 0, P, &table), "cyc_table_run");
  const size_t n = size_t(P) * size_t(P) * size_t(K);
  std::vector<uint8_t> in(n ? n : 1), eg(n ? n : 1), comb(n ? n : 1);
  const int rc = cyc_table_cells(table, 0, P, 0, P, 0, K, in.data(), eg.data(), comb.data());
  if (rc != CYC_OK) {
    std::printf("error cyc_table_cells rc=%d: %s\n", rc, cyc_table_error(table));
    return 3;
  }
  std::printf("shape %lld %lld\n", (long long)P, (long long)K);
  for (int64_t s = 0; s < P; s++)
    for (int64_t d = 0; d < P; d++) {
      std::printf("%lld %lld ", (long long)s, (long long)d);
      for (int64_t k = 0; k < K; k++) {
        const size_t x = (size_t(s) * P + d) * K + k;
        std::printf("%c%c%c", short_string(in[x]), short_string(eg[x]), short_string(comb[x]));
      }
      std::printf("\n");
    }
  cyc_table_destroy(table);
  cyc_ctx_destroy(ctx);
  return 0;
}
