// capi_driver.cpp — a C++ client of libcyclonus_hip's C ABI, standing in for the cgo binding a
// maintainer would add at the reference's JobRunner seam (pkg/connectivity/probe/jobrunner.go:60-62;
// INTEGRATION.md §1).  It drives exactly the calls that binding makes for RunProbeForConfig:
//   cyc_ctx_create -> cyc_policy_build_json -> cyc_policy_ir_json -> cyc_resources_load_json ->
//   cyc_probe_prepare -> cyc_table_run -> cyc_table_cells -> cyc_table_destroy -> cyc_ctx_destroy
// and prints every cell's (ingress, egress, combined) Connectivity as ShortString characters
// (connectivity.go:27-42), one line per (source, destination): "s d <in><eg><comb> per slot".
//
//   capi_driver POLICIES.json RESOURCES.json PROBES.json [--no-gpu]
// --no-gpu stops after the policy compile and prints the compiled policy (json.Marshal form).
// Exit status: 0 ok, 2 usage / file error, 3 a library call failed (the status and
// cyc_last_error text are printed, e.g. the reference's panic message).
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
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

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s POLICIES.json RESOURCES.json PROBES.json [--no-gpu]\n", argv[0]);
    return 2;
  }
  const bool no_gpu = argc > 4 && std::strcmp(argv[4], "--no-gpu") == 0;
  const std::string pols = slurp(argv[1]), res = slurp(argv[2]), probes = slurp(argv[3]);
  cyc_ctx* ctx = nullptr;
  check(nullptr, cyc_ctx_create(0, &ctx), "cyc_ctx_create");
  check(ctx, cyc_policy_build_json(ctx, 1, pols.data(), pols.size()), "cyc_policy_build_json");
  const int64_t need = cyc_policy_ir_json(ctx, nullptr, 0);
  std::vector<char> ir(size_t(need > 0 ? need : 1));
  cyc_policy_ir_json(ctx, ir.data(), ir.size());
  if (no_gpu) {
    std::printf("ir %s\n", ir.data());
    cyc_ctx_destroy(ctx);
    return 0;
  }
  check(ctx, cyc_resources_load_json(ctx, res.data(), res.size()), "cyc_resources_load_json");
  cyc_probe_shape shape{};
  check(ctx, cyc_probe_prepare(ctx, probes.data(), probes.size(), &shape), "cyc_probe_prepare");
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
