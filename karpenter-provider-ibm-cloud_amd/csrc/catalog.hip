// catalog.hip — catalog ingest (gs_build_catalog): IBMInstanceTypeProvider
// .List over the VPC profile wire data, the product-side restatement of
//   List / listFromVPC                reference pkg/providers/common/instancetype/instancetype.go:221-246,433-537
//   convertVPCProfileToInstanceType   instancetype.go:659-790
//   calculateOverhead                 instancetype.go:792-858
//   getInstanceFamily/Size            instancetype.go:861-877
//   GetSupportedCapacityTypes         pkg/providers/common/capacitytype/capacitytype.go:48-85
//   UnavailableOfferings.IsUnavailable pkg/cache/unavailable_offerings.go:51-77
//
// The per-profile validation and string work runs on the host; the offering
// expansion (profiles x zones x capacity types: spot discount in float64 and
// the unavailable-offerings overlay, a binary search over the live keys)
// runs as one device pass.  Output is gs_problem-shaped (catalog.h strings).
#include "ctx.hpp"

#include <map>
#include <set>

namespace gscat {

// resource.ParseQuantity(s).MilliValue(): sign, digits with an optional
// fraction, then a binary-SI / decimal-SI suffix or a decimal exponent; the
// milli value is exact (128-bit rational) and rounds away from zero
bool parse_quantity_milli(const std::string& s, int64_t* out) {
  size_t i = 0;
  bool neg = false;
  if (i < s.size() && (s[i] == '+' || s[i] == '-')) neg = s[i++] == '-';
  __int128 num = 0, den = 1;
  bool any = false, frac = false;
  for (; i < s.size(); i++) {
    const char c = s[i];
    if (c == '.' && !frac) {
      frac = true;
      continue;
    }
    if (c < '0' || c > '9') break;
    if (num > ((__int128)1 << 100)) return false;
    num = num * 10 + (c - '0');
    if (frac) den *= 10;
    any = true;
  }
  if (!any) return false;
  const std::string suf = s.substr(i);
  int shift2 = 0, exp10 = 0;
  if (suf.size() == 2 && suf[1] == 'i') {
    const char* bins = "KMGTPE";
    const char* f = suf[0] ? std::strchr(bins, suf[0]) : nullptr;
    if (!f) return false;
    shift2 = 10 * (int)(f - bins + 1);
  } else if (suf.size() <= 1) {
    static const std::map<std::string, int> dec = {{"n", -9}, {"u", -6}, {"m", -3}, {"", 0}, {"k", 3},
                                                   {"M", 6},  {"G", 9},  {"T", 12}, {"P", 15}, {"E", 18}};
    auto f = dec.find(suf);
    if (f == dec.end()) return false;
    exp10 = f->second;
  } else if (suf[0] == 'e' || suf[0] == 'E') {
    size_t j = 1;
    bool eneg = false;
    if (suf[j] == '+' || suf[j] == '-') eneg = suf[j++] == '-';
    if (j >= suf.size()) return false;
    int e = 0;
    for (; j < suf.size(); j++) {
      if (suf[j] < '0' || suf[j] > '9' || e > 30) return false;
      e = e * 10 + (suf[j] - '0');
    }
    if (e > 30) return false;
    exp10 = eneg ? -e : e;
  } else {
    return false;
  }
  num <<= shift2;
  exp10 += 3;  // milli
  for (; exp10 > 0; exp10--) num *= 10;
  for (; exp10 < 0; exp10++) den *= 10;
  __int128 q = num / den + (num % den ? 1 : 0);
  if (q > (__int128)INT64_MAX) return false;
  *out = neg ? -(int64_t)q : (int64_t)q;
  return true;
}

// getInstanceFamily: the text before the first '-' ("balanced" when empty)
std::string family_of(const std::string& n) {
  const std::string f = n.substr(0, n.find('-'));
  return f.empty() ? "balanced" : f;
}
// getInstanceSize: the text after the first '-' that has one ("small" otherwise)
std::string size_of(const std::string& n) {
  for (size_t i = 0; i + 1 < n.size(); i++)
    if (n[i] == '-') return n.substr(i + 1);
  return "small";
}
// GetCapacityTypeFromAvailabilityClass
const char* ct_of_class(const char* cls) { return cls && std::strcmp(cls, "spot") == 0 ? "spot" : "on-demand"; }

struct OffDesc {
  uint32_t prof, zone, ct, pad;  // ct: 0 on-demand, 1 spot
};

// one lane per offering: price (spot discount as Go computes it, no
// contraction) and availability (live unavailable-offerings key)
__global__ __launch_bounds__(256) void catalog_offerings_kernel(const OffDesc* desc, uint32_t n, const double* base,
                                                                uint32_t Z, int32_t pct, const uint64_t* ukey,
                                                                const int64_t* uexp, uint32_t nu, int64_t now,
                                                                double* price, uint32_t* avail) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const OffDesc d = desc[i];
  double p = base[(size_t)d.prof * Z + d.zone];
  if (d.ct == 1) p = __ddiv_rn(__dmul_rn(p, (double)pct), 100.0);
  const uint64_t key = ((uint64_t)d.prof << 32) | ((uint64_t)d.zone << 1) | d.ct;
  uint32_t lo = 0, hi = nu;
  while (lo < hi) {
    const uint32_t m = (lo + hi) >> 1;
    if (ukey[m] < key) lo = m + 1;
    else hi = m;
  }
  // IsUnavailable: present and !now.After(expiry)
  const bool unav = lo < nu && ukey[lo] == key && !(now > uexp[lo]);
  price[i] = p;
  avail[i] = unav ? 0u : 1u;
}

}  // namespace gscat

using namespace gsc;
using namespace gscat;

extern "C" gs_status gs_build_catalog(gs_ctx* c, const gs_vpc_profile* prof, uint32_t n, const gs_catalog_env* env,
                                      gs_catalog* out) {
  if (!c || !env || !out || (n && !prof)) return GS_E_INVALID;
  std::memset(out, 0, sizeof(*out));
  auto& S = c->cat_strs;
  S.clear();
  std::unordered_map<std::string, uint32_t> sid;
  auto s = [&](const std::string& x) {
    auto f = sid.find(x);
    if (f != sid.end()) return f->second;
    const uint32_t id = (uint32_t)S.size();
    S.push_back(x);
    sid.emplace(x, id);
    return id;
  };
  s("");
  c->cat_vals.clear();
  c->cat_reqs.clear();
  c->cat_qty.clear();
  c->cat_offs.clear();
  c->cat_its.clear();
  c->cat_skipped.clear();
  c->cat_reasons.clear();
  auto req_in = [&](const std::string& key, const std::string& val) {
    gs_requirement r{};
    r.key = s(key);
    r.op = GS_OP_IN;
    r.values = gs_range{(uint32_t)c->cat_vals.size(), 1};
    r.min_values = -1;
    c->cat_vals.push_back(s(val));
    c->cat_reqs.push_back(r);
  };
  std::vector<std::string> zones;
  for (uint32_t z = 0; z < env->n_zones; z++) zones.push_back(env->zones && env->zones[z] ? env->zones[z] : "");
  const uint32_t Z = (uint32_t)zones.size();
  // calculateOverhead: defaults, each kubelet key replaced when it parses
  int64_t kc = 100, km = (int64_t)1 << 30, sc = 100, sm = (int64_t)1 << 30, ev = 500ll << 20;
  km *= 1000;
  sm *= 1000;
  ev *= 1000;
  if (env->has_kubelet) {
    int64_t v;
    auto take = [&](const char* q, int64_t* dst) {
      if (q && parse_quantity_milli(q, &v)) *dst = v;
    };
    take(env->kube_reserved_cpu, &kc);
    take(env->kube_reserved_memory, &km);
    take(env->system_reserved_cpu, &sc);
    take(env->system_reserved_memory, &sm);
    take(env->eviction_memory_available, &ev);
  }
  // pricing table: last matching entry wins
  std::map<std::string, std::vector<uint32_t>> price_rows;
  for (uint32_t k = 0; k < env->n_prices; k++)
    if (env->prices && env->prices[k].name) price_rows[env->prices[k].name].push_back(k);
  const int32_t pct = env->spot_discount_percent == 0 ? 60 : env->spot_discount_percent;
  // convert (host): validation, capacity, requirements, offering layout
  std::vector<OffDesc> desc;
  std::vector<double> base;
  std::vector<uint32_t> kept;  // profile index per converted type
  for (uint32_t i = 0; i < n; i++) {
    const gs_vpc_profile& p = prof[i];
    std::string err;
    const std::string name = p.name ? p.name : "";
    if (!p.name) err = "instance profile name is nil";
    else if (name.empty()) err = "instance profile has empty name";
    else if (p.vcpu_kind == GS_VPC_NIL) err = "instance profile " + name + " has no CPU count";
    else if (p.vcpu_kind != GS_VPC_VALUE) err = "instance profile " + name + " has unsupported CPU count type";
    else if (p.memory_kind == GS_VPC_NIL) err = "instance profile " + name + " has no memory";
    else if (p.memory_kind != GS_VPC_VALUE) err = "instance profile " + name + " has unsupported memory type";
    else if (Z == 0) err = std::string("no zones found for region ") + (env->region ? env->region : "");
    if (!err.empty()) {
      c->cat_skipped.push_back(i);
      c->cat_reasons.push_back(err);
      continue;
    }
    const int64_t cpu = p.vcpu, mem = p.memory_gib;
    const int64_t gpu = p.gpu_kind == GS_VPC_VALUE ? p.gpu : 0;
    const int64_t pods = cpu <= 2 ? 30 : (cpu <= 4 ? 60 : 110);
    gs_instance_type it{};
    it.name = s(name);
    it.requirements.begin = (uint32_t)c->cat_reqs.size();
    req_in("node.kubernetes.io/instance-type", name);
    req_in("kubernetes.io/arch", p.arch ? p.arch : "amd64");
    req_in("karpenter-ibm.sh/instance-family", family_of(name));
    req_in("karpenter-ibm.sh/instance-size", size_of(name));
    it.requirements.count = 4;
    it.capacity.begin = (uint32_t)c->cat_qty.size();
    c->cat_qty.push_back(gs_quantity{s("cpu"), cpu * 1000});
    c->cat_qty.push_back(gs_quantity{s("memory"), mem * ((int64_t)1 << 30) * 1000});
    c->cat_qty.push_back(gs_quantity{s("pods"), pods * 1000});
    c->cat_qty.push_back(gs_quantity{s("nvidia.com/gpu"), gpu * 1000});
    it.capacity.count = 4;
    it.overhead.begin = (uint32_t)c->cat_qty.size();
    c->cat_qty.push_back(gs_quantity{s("cpu"), kc + sc});
    c->cat_qty.push_back(gs_quantity{s("memory"), km + sm + ev});
    it.overhead.count = 2;
    // GetSupportedCapacityTypes (order kept, default on-demand)
    std::vector<uint32_t> cts;
    if (p.avail_kind == GS_AVAIL_ENUM)
      for (uint32_t k = 0; k < p.n_avail_values; k++)
        cts.push_back(std::strcmp(ct_of_class(p.avail_values[k]), "spot") == 0 ? 1u : 0u);
    if (p.avail_kind == GS_AVAIL_FIXED && p.n_avail_values > 0)
      cts.push_back(std::strcmp(ct_of_class(p.avail_values[0]), "spot") == 0 ? 1u : 0u);
    if (cts.empty()) cts.push_back(0);
    const uint32_t k = (uint32_t)kept.size();
    it.offerings = gs_range{(uint32_t)desc.size(), Z * (uint32_t)cts.size()};
    for (uint32_t z = 0; z < Z; z++) {
      double pz = 0.0;
      auto f = price_rows.find(name);
      if (f != price_rows.end())
        for (uint32_t r : f->second)
          if (!env->prices[r].zone || zones[z] == env->prices[r].zone) pz = env->prices[r].price;
      base.push_back(pz);
      for (uint32_t ct : cts) desc.push_back(OffDesc{k, z, ct, 0});
    }
    kept.push_back(i);
    c->cat_its.push_back(it);
  }
  if (kept.empty()) return fail(c, GS_E_INVALID, "no instance types found from VPC API");
  // live unavailable keys over the converted profiles
  std::unordered_map<std::string, std::vector<uint32_t>> kidx;
  for (uint32_t k = 0; k < kept.size(); k++) kidx[prof[kept[k]].name].push_back(k);
  std::vector<std::pair<uint64_t, int64_t>> uk;
  for (uint32_t u = 0; u < env->n_unavailable; u++) {
    if (!env->unavailable || !env->unavailable[u].key) continue;
    const std::string key = env->unavailable[u].key;
    // "<profile>:<zone>:<capacity type>": profile names hold no ':', zones may
    const size_t a = key.find(':'), b = key.rfind(':');
    if (a == std::string::npos || a == b) continue;
    auto f = kidx.find(key.substr(0, a));
    const std::string zone = key.substr(a + 1, b - a - 1), ct = key.substr(b + 1);
    if (f == kidx.end() || (ct != "spot" && ct != "on-demand")) continue;
    for (uint32_t k : f->second)
      for (uint32_t z = 0; z < Z; z++)
        if (zones[z] == zone)
          uk.push_back({((uint64_t)k << 32) | ((uint64_t)z << 1) | (ct == "spot" ? 1u : 0u),
                        env->unavailable[u].expiry_unix_ns});
  }
  // a repeated key keeps the last Add (map assignment)
  std::stable_sort(uk.begin(), uk.end(), [](auto& x, auto& y) { return x.first < y.first; });
  std::vector<uint64_t> ukey;
  std::vector<int64_t> uexp;
  for (size_t j = 0; j < uk.size(); j++) {
    if (!ukey.empty() && ukey.back() == uk[j].first) uexp.back() = uk[j].second;
    else {
      ukey.push_back(uk[j].first);
      uexp.push_back(uk[j].second);
    }
  }
  // device pass over every offering
  const uint32_t O = (uint32_t)desc.size();
  std::vector<double> price(O);
  std::vector<uint32_t> avail(O);
  try {
    HIPCHK(hipSetDevice(c->device));
    size_t off = 0;
    auto place = [&](size_t bytes) {
      const size_t o = off;
      off += (std::max<size_t>(bytes, 1) + 255) & ~(size_t)255;
      return o;
    };
    const size_t o_desc = place(O * sizeof(OffDesc)), o_base = place(base.size() * 8), o_uk = place(ukey.size() * 8),
                 o_ue = place(uexp.size() * 8), o_in = off, o_price = place((size_t)O * 8), o_av = place((size_t)O * 4);
    void* dbuf = nullptr;
    HIPCHK(hipMalloc(&dbuf, off));
    struct Free {
      void* p;
      ~Free() { (void)hipFree(p); }
    } guard{dbuf};
    char* b = (char*)dbuf;
    std::vector<char> h(o_in);
    std::memcpy(h.data() + o_desc, desc.data(), O * sizeof(OffDesc));
    std::memcpy(h.data() + o_base, base.data(), base.size() * 8);
    if (!ukey.empty()) {
      std::memcpy(h.data() + o_uk, ukey.data(), ukey.size() * 8);
      std::memcpy(h.data() + o_ue, uexp.data(), uexp.size() * 8);
    }
    HIPCHK(hipMemcpyAsync(b, h.data(), o_in, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(catalog_offerings_kernel, dim3((O + 255) / 256), dim3(256), 0, c->stream,
                       (const OffDesc*)(b + o_desc), O, (const double*)(b + o_base), Z, pct,
                       (const uint64_t*)(b + o_uk), (const int64_t*)(b + o_ue), (uint32_t)ukey.size(),
                       env->now_unix_ns, (double*)(b + o_price), (uint32_t*)(b + o_av));
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(price.data(), b + o_price, (size_t)O * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(avail.data(), b + o_av, (size_t)O * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
  } catch (const HipError& ex) {
    return fail(c, GS_E_HIP, ex.msg);
  }
  static const char* ctn[2] = {"on-demand", "spot"};
  for (uint32_t i = 0; i < O; i++) {
    gs_offering o{};
    o.requirements.begin = (uint32_t)c->cat_reqs.size();
    req_in("topology.kubernetes.io/zone", zones[desc[i].zone]);
    req_in("karpenter.sh/capacity-type", ctn[desc[i].ct]);
    o.requirements.count = 2;
    o.price = price[i];
    o.available = avail[i];
    c->cat_offs.push_back(o);
  }
  c->cat_ptrs.clear();
  for (auto& x : S) c->cat_ptrs.push_back(x.c_str());
  c->cat_reason_ptrs.clear();
  for (auto& x : c->cat_reasons) c->cat_reason_ptrs.push_back(x.c_str());
  out->strings = c->cat_ptrs.data();
  out->n_strings = (uint32_t)S.size();
  out->value_ids = c->cat_vals.data();
  out->n_value_ids = (uint32_t)c->cat_vals.size();
  out->reqs = c->cat_reqs.data();
  out->n_reqs = (uint32_t)c->cat_reqs.size();
  out->quantities = c->cat_qty.data();
  out->n_quantities = (uint32_t)c->cat_qty.size();
  out->offerings = c->cat_offs.data();
  out->n_offerings = (uint32_t)c->cat_offs.size();
  out->instance_types = c->cat_its.data();
  out->n_instance_types = (uint32_t)c->cat_its.size();
  out->n_skipped = (uint32_t)c->cat_skipped.size();
  out->skipped = c->cat_skipped.data();
  out->skip_reasons = c->cat_reason_ptrs.data();
  return GS_OK;
}
