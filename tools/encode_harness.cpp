// encode_harness.cpp — host-only driver of the Solve encoder (encode.cpp)
// over gs_problem dumps written by gpusched.problem.Problem.dump().
// Built with g++ (no HIP) for two uses:
//  * sanitizers: tests/test_encode_sanitizers.py builds it with
//    -fsanitize=address,undefined and runs every dump once;
//  * profiling: build with -O2 -pg and run a dump many times (gprof).
// Usage: encode_harness [-n reps] dump...   prints "<status> <ms> <path>" per dump.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../karpenter-provider-ibm-cloud_amd/csrc/encode.hpp"

namespace {

struct Dump {
  std::vector<std::string> strs;
  std::vector<const char*> ptrs;
  std::vector<std::vector<char>> arrays;
  gs_problem p{};
};

bool read_exact(FILE* f, void* dst, size_t n) { return fread(dst, 1, n, f) == n; }

// layout: magic "GSPD", u32 version 4, u32 n_strings, per string u32 len +
// bytes, then 21 arrays in gs_problem order (value_ids .. namespaces),
// each u64 count + u64 element size + raw bytes
bool load(const char* path, Dump& d) {
  FILE* f = fopen(path, "rb");
  if (!f) return false;
  char magic[4];
  uint32_t ver = 0, ns = 0;
  bool ok = read_exact(f, magic, 4) && memcmp(magic, "GSPD", 4) == 0 && read_exact(f, &ver, 4) && ver == 4 &&
            read_exact(f, &ns, 4);
  for (uint32_t i = 0; ok && i < ns; i++) {
    uint32_t len = 0;
    ok = read_exact(f, &len, 4);
    std::string s(len, '\0');
    ok = ok && (len == 0 || read_exact(f, &s[0], len));
    d.strs.push_back(std::move(s));
  }
  for (int a = 0; ok && a < 21; a++) {
    uint64_t n = 0, es = 0;
    ok = read_exact(f, &n, 8) && read_exact(f, &es, 8);
    std::vector<char> buf(n * es);
    ok = ok && (buf.empty() || read_exact(f, buf.data(), buf.size()));
    d.arrays.push_back(std::move(buf));
  }
  fclose(f);
  if (!ok) return false;
  for (auto& s : d.strs) d.ptrs.push_back(s.c_str());
  auto A = [&](int i) -> const void* { return d.arrays[i].empty() ? nullptr : d.arrays[i].data(); };
  auto N = [&](int i, size_t es) { return (uint32_t)(d.arrays[i].size() / es); };
  gs_problem& p = d.p;
  p.strings = d.ptrs.data();
  p.n_strings = ns;
  p.value_ids = (const uint32_t*)A(0), p.n_value_ids = N(0, 4);
  p.reqs = (const gs_requirement*)A(1), p.n_reqs = N(1, sizeof(gs_requirement));
  p.quantities = (const gs_quantity*)A(2), p.n_quantities = N(2, sizeof(gs_quantity));
  p.labels = (const gs_label*)A(3), p.n_labels = N(3, sizeof(gs_label));
  p.taints = (const gs_taint*)A(4), p.n_taints = N(4, sizeof(gs_taint));
  p.tolerations = (const gs_toleration*)A(5), p.n_tolerations = N(5, sizeof(gs_toleration));
  p.terms = (const gs_term*)A(6), p.n_terms = N(6, sizeof(gs_term));
  p.it_refs = (const uint32_t*)A(7), p.n_it_refs = N(7, 4);
  p.offerings = (const gs_offering*)A(8), p.n_offerings = N(8, sizeof(gs_offering));
  p.instance_types = (const gs_instance_type*)A(9), p.n_instance_types = N(9, sizeof(gs_instance_type));
  p.nodepools = (const gs_nodepool*)A(10), p.n_nodepools = N(10, sizeof(gs_nodepool));
  p.pods = (const gs_pod*)A(11), p.n_pods = N(11, sizeof(gs_pod));
  p.nodes = (const gs_node*)A(12), p.n_nodes = N(12, sizeof(gs_node));
  p.spreads = (const gs_spread*)A(13), p.n_spreads = N(13, sizeof(gs_spread));
  p.bound_pods = (const gs_pod*)A(14), p.n_bound_pods = N(14, sizeof(gs_pod));
  p.bound_pod_node = (const uint32_t*)A(15);
  p.affinity_terms = (const gs_affinity_term*)A(16), p.n_affinity_terms = N(16, sizeof(gs_affinity_term));
  p.host_ports = (const gs_host_port*)A(17), p.n_host_ports = N(17, sizeof(gs_host_port));
  p.volumes = (const gs_volume*)A(18), p.n_volumes = N(18, sizeof(gs_volume));
  p.volume_limits = (const gs_volume_limit*)A(19), p.n_volume_limits = N(19, sizeof(gs_volume_limit));
  p.namespaces = (const gs_namespace*)A(20), p.n_namespaces = N(20, sizeof(gs_namespace));
  return true;
}

}  // namespace

int main(int argc, char** argv) {
  int reps = 1, i = 1;
  if (argc > 2 && strcmp(argv[1], "-n") == 0) {
    reps = atoi(argv[2]);
    i = 3;
  }
  int rc = 0;
  for (; i < argc; i++) {
    Dump d;
    if (!load(argv[i], d)) {
      fprintf(stderr, "cannot read %s\n", argv[i]);
      rc = 2;
      continue;
    }
    gsh::Err er;
    double best = 1e300;
    gsh::Encoded e;  // one per dump, reused across reps (as a context reuses its encoding)
    for (int r = 0; r < reps; r++) {
      auto t0 = std::chrono::steady_clock::now();
      er = gsh::encode(&d.p, e);
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (ms < best) best = ms;
    }
    printf("%d %.3f %s\n", (int)er.code, best, argv[i]);
  }
  return rc;
}
