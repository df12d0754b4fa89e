// catalog.cpp — TEST INFRASTRUCTURE ONLY (parity oracle; see oracle.h).
//
// Restatement of the IBM catalog builder that feeds Solve:
//   convertVPCProfileToInstanceType  reference pkg/providers/common/instancetype/instancetype.go:659-790
//   calculateOverhead                 instancetype.go:792-858
//   getInstanceFamily/getInstanceSize instancetype.go:861-877
//   calculateInstanceTypeScore        instancetype.go:90-110
//   GetSupportedCapacityTypes         pkg/providers/common/capacitytype/capacitytype.go:48-85
// Pinned by the reference's known-answer tests (tests/test_oracle_kats.py).
#include "oracle.h"
#include "gosort.h"

#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <vector>

namespace {

using std::string;
using std::vector;

// resource.ParseQuantity subset: <sign><digits>[.<digits>]<suffix>; returns
// the exact value as (num / den) with __int128, then MilliValue = ceil(x*1000).
bool parse_quantity_milli(const string& s, int64_t* out) {
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[i] == '+' || s[i] == '-') {
    neg = s[i] == '-';
    i++;
  }
  __int128 mant = 0;
  int frac = 0;
  bool digits = false, dot = false;
  for (; i < s.size(); i++) {
    char c = s[i];
    if (c >= '0' && c <= '9') {
      digits = true;
      if (mant > ((__int128)1 << 100)) return false;
      mant = mant * 10 + (c - '0');
      if (dot) frac++;
    } else if (c == '.' && !dot) {
      dot = true;
    } else {
      break;
    }
  }
  if (!digits) return false;
  string suf = s.substr(i);
  __int128 num = mant, den = 1;
  for (int k = 0; k < frac; k++) den *= 10;
  auto pow10 = [](int e) {
    __int128 v = 1;
    for (int k = 0; k < e; k++) v *= 10;
    return v;
  };
  static const std::map<string, int> bin = {{"Ki", 10}, {"Mi", 20}, {"Gi", 30}, {"Ti", 40}, {"Pi", 50}, {"Ei", 60}};
  static const std::map<string, int> dec = {{"n", -9}, {"u", -6}, {"m", -3}, {"", 0}, {"k", 3},
                                           {"M", 6},  {"G", 9},  {"T", 12}, {"P", 15}, {"E", 18}};
  int e10 = 0;
  if (bin.count(suf)) {
    num <<= bin.at(suf);
  } else if (dec.count(suf)) {
    e10 = dec.at(suf);
  } else if (!suf.empty() && (suf[0] == 'e' || suf[0] == 'E')) {
    int64_t e = 0;
    size_t j = 1;
    bool eneg = false;
    if (j < suf.size() && (suf[j] == '+' || suf[j] == '-')) {
      eneg = suf[j] == '-';
      j++;
    }
    if (j >= suf.size()) return false;
    for (; j < suf.size(); j++) {
      if (suf[j] < '0' || suf[j] > '9') return false;
      e = e * 10 + (suf[j] - '0');
      if (e > 30) return false;
    }
    e10 = (int)(eneg ? -e : e);
  } else {
    return false;
  }
  // milli: x * 1000
  e10 += 3;
  if (e10 >= 0) num *= pow10(e10);
  else den *= pow10(-e10);
  __int128 q = num / den;
  if (num % den) q += 1;  // MilliValue rounds up (toward +inf magnitude for positives)
  if (neg) q = -q;
  if (q > INT64_MAX || q < INT64_MIN) return false;
  *out = (int64_t)q;
  return true;
}

string family_of(const string& name) {
  // strings.SplitN(name, "-", 2)[0], "" -> "balanced"
  size_t d = name.find('-');
  string first = d == string::npos ? name : name.substr(0, d);
  return first.empty() ? "balanced" : first;
}
string size_of(const string& name) {
  // first '-' with at least one char after it
  for (size_t i = 0; i < name.size(); i++)
    if (name[i] == '-' && i + 1 < name.size()) return name.substr(i + 1);
  return "small";
}
string capacity_type_of(const string& cls) {
  if (cls == "spot") return "spot";
  return "on-demand";  // "standard", "" and unknown classes
}

string hexbits(double d) {
  uint64_t u;
  std::memcpy(&u, &d, 8);
  char buf[32];
  std::snprintf(buf, sizeof buf, "%016llx", (unsigned long long)u);
  return buf;
}

string g_text;
string g_tmp;

}  // namespace

extern "C" int oracle_parse_quantity_milli(const char* s, int64_t* milli_out) {
  return parse_quantity_milli(s ? s : "", milli_out) ? 0 : 1;
}

extern "C" const char* oracle_instance_family(const char* name) {
  g_tmp = family_of(name ? name : "");
  return g_tmp.c_str();
}
extern "C" const char* oracle_instance_size(const char* name) {
  g_tmp = size_of(name ? name : "");
  return g_tmp.c_str();
}
extern "C" const char* oracle_capacity_type(const char* cls) {
  g_tmp = capacity_type_of(cls ? cls : "");
  return g_tmp.c_str();
}

extern "C" double oracle_instance_score(int64_t cpu_milli, int64_t memory_bytes, double price) {
  // Capacity.Cpu().Value() rounds up; Memory().ScaledValue(Giga) rounds up
  double cpu = (double)((cpu_milli + 999) / 1000);
  double memGB = (double)((memory_bytes + 999999999) / 1000000000);
  if (price <= 0) return cpu + memGB;
  double a = price / cpu;
  double b = price / memGB;
  return (a + b) / 2;
}

// FilterInstanceTypes (instancetype.go:259-356): the four filters in List
// order (:319-344), then rankInstanceTypes (:358-379): sort.Slice over
// (type, score) records with Less = score[i] < score[j].
extern "C" gs_status oracle_rank_instance_types(uint32_t n, const int64_t* cpu_milli, const int64_t* memory_bytes,
                                                const double* price, const uint32_t* arch, uint32_t want_arch,
                                                int64_t min_cpu, int64_t min_memory_gb, double max_price,
                                                uint32_t* out_order, uint32_t* out_n, double* out_score) {
  if (!out_n || (n && (!cpu_milli || !memory_bytes || !price || !arch || !out_order || !out_score)))
    return GS_E_INVALID;
  if (n > GS_RANK_MAX) return GS_E_CAPACITY;
  for (uint32_t i = 0; i < n; i++)
    if (cpu_milli[i] < 0 || memory_bytes[i] < 0 || std::isnan(price[i])) return GS_E_INVALID;
  struct Rankings {
    std::vector<double> score;
    std::vector<uint32_t> idx;
    bool less(int i, int j) const { return score[i] < score[j]; }
    void swap(int i, int j) {
      std::swap(score[i], score[j]);
      std::swap(idx[i], idx[j]);
    }
  } r;
  for (uint32_t i = 0; i < n; i++) {
    if (want_arch != GS_ARCH_ANY && arch[i] != want_arch) continue;                  // :321
    if (min_cpu > 0 && (cpu_milli[i] + 999) / 1000 < min_cpu) continue;                // :326
    if (min_memory_gb > 0 && (double)memory_bytes[i] / (1024.0 * 1024 * 1024) < (double)min_memory_gb)
      continue;                                                                          // :331-335
    if (max_price > 0 && price[i] > max_price) continue;                                // :339
    r.score.push_back(oracle_instance_score(cpu_milli[i], memory_bytes[i], price[i]));
    r.idx.push_back(i);
  }
  gosort::slice(r, (int)r.idx.size());
  for (size_t k = 0; k < r.idx.size(); k++) {
    out_order[k] = r.idx[k];
    out_score[k] = r.score[k];
  }
  *out_n = (uint32_t)r.idx.size();
  return GS_OK;
}

extern "C" gs_status oracle_convert_profile(const oracle_profile* pr, const oracle_catalog_env* env,
                                            const char** text_out) {
  auto fail = [&](const string& m) {
    g_text = m;
    *text_out = g_text.c_str();
    return GS_E_INVALID;
  };
  if (!pr->name) return fail("instance profile name is nil");
  string name = pr->name;
  if (name.empty()) return fail("instance profile has empty name");
  if (pr->vcpu_kind == 0) return fail("instance profile " + name + " has no CPU count");
  if (pr->vcpu_kind != 1) return fail("instance profile " + name + " has unsupported CPU count type");
  int64_t cpu = pr->vcpu;
  if (pr->memory_kind == 0) return fail("instance profile " + name + " has no memory");
  if (pr->memory_kind != 1) return fail("instance profile " + name + " has unsupported memory type");
  int64_t memGiB = pr->memory_gib;
  string arch = pr->arch ? pr->arch : "amd64";
  int64_t gpu = pr->gpu_kind == 1 ? pr->gpu : 0;
  int64_t pods = 110;
  if (cpu <= 2) pods = 30;
  else if (cpu <= 4) pods = 60;
  if (!env->has_client) return fail("IBM client not initialized - cannot determine zones for instance offerings");
  if (env->n_zones == 0) return fail(string("no zones found for region ") + (env->region ? env->region : ""));  // instancetype.go:738-740
  // GetSupportedCapacityTypes
  vector<string> cts;
  if (pr->avail_kind == 1) {
    for (uint32_t i = 0; i < pr->n_avail_values; i++) cts.push_back(capacity_type_of(pr->avail_values[i]));
  } else if (pr->avail_kind == 2) {
    if (pr->n_avail_values > 0) cts.push_back(capacity_type_of(pr->avail_values[0]));
  }
  if (cts.empty()) cts.push_back("on-demand");
  int pct = env->spot_discount_percent;
  if (pct == 0) pct = 60;
  // UnavailableOfferings (pkg/cache/unavailable_offerings.go:36-77): Add is a
  // map assignment; IsUnavailable = present && !now.After(expiry)
  std::map<string, int64_t> unavailable;
  for (uint32_t i = 0; i < env->n_unavailable; i++)
    unavailable[env->unavailable[i]] = env->unavailable_expiry ? env->unavailable_expiry[i] : INT64_MAX;
  // calculateOverhead
  int64_t kc = 100, km = 1073741824000LL, sc = 100, sm = 1073741824000LL, ev = 524288000000LL;
  if (env->has_nodeclass && env->has_kubelet) {
    int64_t v;
    if (env->kube_reserved_cpu && parse_quantity_milli(env->kube_reserved_cpu, &v)) kc = v;
    if (env->kube_reserved_memory && parse_quantity_milli(env->kube_reserved_memory, &v)) km = v;
    if (env->system_reserved_cpu && parse_quantity_milli(env->system_reserved_cpu, &v)) sc = v;
    if (env->system_reserved_memory && parse_quantity_milli(env->system_reserved_memory, &v)) sm = v;
    if (env->eviction_memory_available && parse_quantity_milli(env->eviction_memory_available, &v)) ev = v;
  }
  string t;
  t += "name=" + name + "\n";
  t += "capacity=cpu:" + std::to_string(cpu * 1000) + ",memory:" + std::to_string(memGiB * 1073741824LL * 1000) +
       ",nvidia.com/gpu:" + std::to_string(gpu * 1000) + ",pods:" + std::to_string(pods * 1000) + "\n";
  t += "overhead=kube.cpu:" + std::to_string(kc) + ",kube.memory:" + std::to_string(km) +
       ",system.cpu:" + std::to_string(sc) + ",system.memory:" + std::to_string(sm) +
       ",eviction.memory:" + std::to_string(ev) + "\n";
  t += "requirements=karpenter-ibm.sh/instance-family|In|" + family_of(name) +
       ";karpenter-ibm.sh/instance-size|In|" + size_of(name) + ";kubernetes.io/arch|In|" + arch +
       ";node.kubernetes.io/instance-type|In|" + name + "\n";
  for (uint32_t z = 0; z < env->n_zones; z++) {
    string zone = env->zones[z];
    for (auto& ct : cts) {
      double price = 0.0;  // GetPrice error -> 0 (instancetype.go:753 discards the error)
      for (uint32_t k = 0; k < env->n_prices; k++)
        if (name == env->price_names[k] &&
            (!env->price_zones || !env->price_zones[k] || zone == env->price_zones[k]))
          price = env->prices[k];
      if (ct == "spot") price = price * (double)pct / 100.0;
      auto uf = unavailable.find(name + ":" + zone + ":" + ct);
      bool avail = !(uf != unavailable.end() && !(env->now_ns > uf->second));
      char pbuf[64];
      std::snprintf(pbuf, sizeof pbuf, "%.17g", price);
      t += "offering=" + zone + "|" + ct + "|" + hexbits(price) + "|" + pbuf + "|" + (avail ? "1" : "0") + "\n";
    }
  }
  g_text = t;
  *text_out = g_text.c_str();
  return GS_OK;
}
