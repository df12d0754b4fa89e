// solve.cpp — TEST INFRASTRUCTURE ONLY (parity oracle; see oracle.h).
//
// Literal CPU restatement of sigs.k8s.io/karpenter@v1.13.0 scheduling as the
// IBM provider drives it.  Representation is deliberately naive (string
// sets, string-keyed maps, copies on every CanAdd) so that it shares nothing
// with the product's bitset encoding.  Every <U> item is upstream behaviour
// restated from memory (the module is not in the container): "parity
// unpinned" for those.  Reference call sites are cited where they exist.
#include "oracle.h"
#include "gosort.h"

#include <arpa/inet.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <climits>
#include <cstdio>
#include <memory>
#include <cstring>
#include <map>
#include <optional>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

using std::optional;
using std::string;
using std::vector;

const char* kHostname = "kubernetes.io/hostname";
const char* kZone = "topology.kubernetes.io/zone";
const char* kCapacityType = "karpenter.sh/capacity-type";
const char* kNodePool = "karpenter.sh/nodepool";
const char* kEffectPreferNoSchedule = "PreferNoSchedule";

// <U> karpv1.WellKnownLabels + the 4 IBM keys inserted by
// reference pkg/apis/v1alpha1/labels.go:37-45.
const std::set<string>& well_known() {
  static const std::set<string> s = {
      "karpenter.sh/nodepool",
      "topology.kubernetes.io/zone",
      "topology.kubernetes.io/region",
      "node.kubernetes.io/instance-type",
      "kubernetes.io/arch",
      "kubernetes.io/os",
      "karpenter.sh/capacity-type",
      "node.kubernetes.io/windows-build",
      "karpenter-ibm.sh/instance-size",
      "karpenter-ibm.sh/instance-family",
      "karpenter-ibm.sh/instance-cpu",
      "karpenter-ibm.sh/instance-memory",
  };
  return s;
}

// <U> karpv1.NormalizedLabels
string normalize_key(const string& k) {
  static const std::map<string, string> m = {
      {"failure-domain.beta.kubernetes.io/zone", "topology.kubernetes.io/zone"},
      {"failure-domain.beta.kubernetes.io/region", "topology.kubernetes.io/region"},
      {"beta.kubernetes.io/arch", "kubernetes.io/arch"},
      {"beta.kubernetes.io/instance-type", "node.kubernetes.io/instance-type"},
      {"beta.kubernetes.io/os", "kubernetes.io/os"},
  };
  auto it = m.find(k);
  return it == m.end() ? k : it->second;
}

// Go strconv.Atoi (base 10, optional sign, int64 range)
bool go_atoi(const string& s, int64_t* out) {
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    i = 1;
  }
  if (i >= s.size()) return false;
  __int128 v = 0;
  for (; i < s.size(); i++) {
    if (s[i] < '0' || s[i] > '9') return false;
    v = v * 10 + (s[i] - '0');
    if (v > (__int128)INT64_MAX + 1) return false;
  }
  if (neg) v = -v;
  if (v > INT64_MAX || v < INT64_MIN) return false;
  *out = (int64_t)v;
  return true;
}

struct Status {
  gs_status code = GS_OK;
  string msg;
};

struct Unsupported {
  gs_status code;
  string msg;
};

// ---------------------------------------------------------------- Requirement
// <U> pkg/scheduling/requirement.go
struct Req {
  string key;
  bool complement = true;
  std::set<string> values;
  optional<int64_t> gt, lt;
  optional<int64_t> min_values;

  int64_t len() const {
    return complement ? INT64_MAX - (int64_t)values.size() : (int64_t)values.size();
  }
  int op() const {
    if (complement) return len() < INT64_MAX ? GS_OP_NOTIN : GS_OP_EXISTS;
    return len() > 0 ? GS_OP_IN : GS_OP_DOES_NOT_EXIST;
  }
  static bool within(const string& v, const optional<int64_t>& gt, const optional<int64_t>& lt) {
    if (!gt && !lt) return true;
    int64_t x;
    if (!go_atoi(v, &x)) return false;
    if (gt && *gt >= x) return false;
    if (lt && *lt <= x) return false;
    return true;
  }
  bool has(const string& v) const {
    if (complement) return !values.count(v) && within(v, gt, lt);
    return values.count(v) && within(v, gt, lt);
  }
  Req intersection(const Req& o) const {
    bool comp = complement && o.complement;
    optional<int64_t> g = gt, l = lt, mv = min_values;
    if (o.gt && (!g || *o.gt > *g)) g = o.gt;
    if (o.lt && (!l || *o.lt < *l)) l = o.lt;
    if (o.min_values && (!mv || *o.min_values > *mv)) mv = o.min_values;
    if (g && l && *g >= *l) {
      Req r;
      r.key = key;
      r.complement = false;  // DoesNotExist
      r.min_values = mv;
      return r;
    }
    std::set<string> vals;
    if (complement && o.complement) {
      vals = values;
      vals.insert(o.values.begin(), o.values.end());
    } else if (complement && !o.complement) {
      for (auto& v : o.values)
        if (!values.count(v)) vals.insert(v);
    } else if (!complement && o.complement) {
      for (auto& v : values)
        if (!o.values.count(v)) vals.insert(v);
    } else {
      for (auto& v : values)
        if (o.values.count(v)) vals.insert(v);
    }
    for (auto it = vals.begin(); it != vals.end();) {
      if (!within(*it, g, l)) it = vals.erase(it);
      else ++it;
    }
    if (!comp) {
      g.reset();
      l.reset();
    }
    Req r;
    r.key = key;
    r.complement = comp;
    r.values = std::move(vals);
    r.gt = g;
    r.lt = l;
    r.min_values = mv;
    return r;
  }
};

Req make_req(const string& key_in, int op, const vector<string>& values, optional<int64_t> mv) {
  Req r;
  r.key = normalize_key(key_in);
  r.complement = true;
  r.min_values = mv;
  if (op == GS_OP_IN || op == GS_OP_DOES_NOT_EXIST) r.complement = false;
  if (op == GS_OP_IN || op == GS_OP_NOTIN) r.values.insert(values.begin(), values.end());
  if (op >= GS_OP_GT && op <= GS_OP_LTE) {
    int64_t v = 0;
    if (values.empty() || !go_atoi(values[0], &v)) throw Unsupported{GS_E_INVALID, "Gt/Lt value is not an integer"};
    // <U> Gte x / Lte x over integer label values: greaterThan x-1 / lessThan x+1
    if ((op == GS_OP_GTE && v == INT64_MIN) || (op == GS_OP_LTE && v == INT64_MAX))
      throw Unsupported{GS_E_INVALID, "Gte/Lte bound out of range"};
    if (op == GS_OP_GT) r.gt = v;
    else if (op == GS_OP_LT) r.lt = v;
    else if (op == GS_OP_GTE) r.gt = v - 1;
    else r.lt = v + 1;
  }
  return r;
}

// <U> pkg/scheduling/requirements.go
struct Reqs {
  std::map<string, Req> m;

  void add(const Req& r) {
    auto it = m.find(r.key);
    if (it != m.end()) {
      Req x = r.intersection(it->second);
      it->second = std::move(x);
    } else {
      m.emplace(r.key, r);
    }
  }
  void add_all(const Reqs& o) {
    for (auto& kv : o.m) add(kv.second);
  }
  bool has_key(const string& k) const { return m.count(k) != 0; }
  Req get(const string& k) const {
    auto it = m.find(k);
    if (it != m.end()) return it->second;
    return make_req(k, GS_OP_EXISTS, {}, std::nullopt);
  }
  // Intersects: for shared keys there must be some value, unless both
  // operators are in {NotIn, DoesNotExist}
  bool intersects(const Reqs& in) const {
    for (auto& kv : m) {
      auto it = in.m.find(kv.first);
      if (it == in.m.end()) continue;
      const Req& existing = kv.second;
      const Req& incoming = it->second;
      if (existing.intersection(incoming).len() == 0) {
        int io = incoming.op(), eo = existing.op();
        if ((io == GS_OP_NOTIN || io == GS_OP_DOES_NOT_EXIST) && (eo == GS_OP_NOTIN || eo == GS_OP_DOES_NOT_EXIST))
          continue;
        return false;
      }
    }
    return true;
  }
  // Compatible(incoming, AllowUndefined = allow_wellknown ? WellKnownLabels : {})
  bool compatible(const Reqs& in, bool allow_wellknown) const {
    for (auto& kv : in.m) {
      if (allow_wellknown && well_known().count(kv.first)) continue;
      int o = kv.second.op();
      if (has_key(kv.first) || o == GS_OP_NOTIN || o == GS_OP_DOES_NOT_EXIST) continue;
      return false;
    }
    return intersects(in);
  }
};

// canonical text: keys ascending, "key|Op|v1,v2|gt|lt|minValues"
string canonical(const Reqs& r) {
  static const char* opn[] = {"In", "NotIn", "Exists", "DoesNotExist"};
  string s;
  for (auto& kv : r.m) {
    const Req& q = kv.second;
    if (!s.empty()) s += '\n';
    s += kv.first;
    s += '|';
    s += opn[q.op()];
    s += '|';
    bool first = true;
    for (auto& v : q.values) {
      if (!first) s += ',';
      s += v;
      first = false;
    }
    s += '|';
    s += q.gt ? std::to_string(*q.gt) : "-";
    s += '|';
    s += q.lt ? std::to_string(*q.lt) : "-";
    s += '|';
    s += q.min_values ? std::to_string(*q.min_values) : "-";
  }
  return s;
}

// ------------------------------------------------------------------ Resources
// <U> pkg/utils/resources
using Res = std::map<string, int64_t>;

Res merge(const Res& a, const Res& b) {
  Res r = a;
  for (auto& kv : b) r[kv.first] += kv.second;
  return r;
}
bool fits(const Res& cand, const Res& total) {
  for (auto& kv : total)
    if (kv.second < 0) return false;
  for (auto& kv : cand) {
    auto it = total.find(kv.first);
    int64_t t = it == total.end() ? 0 : it->second;
    if (kv.second > t) return false;
  }
  return true;
}
Res subtract(const Res& a, const Res& b) {
  Res r = a;
  for (auto& kv : a) {
    auto it = b.find(kv.first);
    if (it != b.end()) r[kv.first] = kv.second - it->second;
  }
  return r;
}
int64_t res_get(const Res& r, const string& k) {
  auto it = r.find(k);
  return it == r.end() ? 0 : it->second;
}

// --------------------------------------------------------------- Taints
struct Taint {
  string key, value, effect;
};
struct Toleration {
  string key, value, effect;
  int op;
};
// corev1 Toleration.ToleratesTaint
bool tolerates_taint(const Toleration& t, const Taint& taint) {
  if (!t.effect.empty() && t.effect != taint.effect) return false;
  if (!t.key.empty() && t.key != taint.key) return false;
  if (t.op == GS_TOL_EQUAL) return t.value == taint.value;
  if (t.op == GS_TOL_EXISTS) return true;
  return false;
}
// <U> scheduling.Taints.ToleratesPod: every taint tolerated by some toleration
bool tolerates_all(const vector<Taint>& taints, const vector<Toleration>& tols) {
  for (auto& tn : taints) {
    bool ok = false;
    for (auto& t : tols) ok = ok || tolerates_taint(t, tn);
    if (!ok) return false;
  }
  return true;
}

// ----------------------------------------------------------- model objects
struct Offering {
  Reqs reqs;
  double price;
  bool available;
};
struct InstanceType {
  uint32_t index;
  string name;
  Reqs reqs;
  Res capacity, overhead, allocatable;
  vector<Offering> offerings;
};

struct Term {
  vector<Req> reqs;  // raw NodeSelectorRequirements
  int32_t weight;
};

// corev1.TopologySpreadConstraint (zone / hostname keys)
struct Spread {
  string key;
  int32_t max_skew = 1;
  bool schedule_anyway = false;
  optional<int32_t> min_domains;
  bool has_selector = false;
  std::map<string, string> match_labels;
  struct Expr {
    string key;
    int op;
    std::set<string> values;
  };
  vector<Expr> exprs;
  bool ignore_affinity = false;
  bool honor_taints = false;  // nodeTaintsPolicy Honor
  // <U> TopologyNodeFilter (MakeTopologyNodeFilter): the owner's node selector
  // AND each required node-affinity term (OR over terms; the node selector
  // alone without terms), and the owner's tolerations
  vector<Reqs> filter;
  vector<Toleration> filter_tols;
  // the filter's part of TopologyGroup.Hash: hashstructure skips unexported
  // fields, so of each term's Requirements only the keys enter the hash (not
  // the values); Tolerations and both policies do (slices as sets: restated
  // as sorted lists)
  string filter_id;
  // metav1.LabelSelector over a pod's labels (nil selects nothing)
  bool matches(const std::map<string, string>& labels) const {
    if (!has_selector) return false;
    for (auto& kv : match_labels) {
      auto f = labels.find(kv.first);
      if (f == labels.end() || f->second != kv.second) return false;
    }
    for (auto& e : exprs) {
      auto f = labels.find(e.key);
      const bool present = f != labels.end();
      if (e.op == GS_OP_IN && !(present && e.values.count(f->second))) return false;
      if (e.op == GS_OP_NOTIN && present && e.values.count(f->second)) return false;
      if (e.op == GS_OP_EXISTS && !present) return false;
      if (e.op == GS_OP_DOES_NOT_EXIST && present) return false;
    }
    return true;
  }
  // <U> TopologyGroup.Hash: key, type, namespaces, selector, maxSkew and the
  // node filter; neither whenUnsatisfiable nor minDomains is part of it (a
  // group keeps its first owner's minDomains)
  string hash(const string& ns) const {
    string h = key + "|" + std::to_string(max_skew) + "|" + ns + "|" + (has_selector ? "1" : "0") + "|" +
               (ignore_affinity ? "I" : "H") + (honor_taints ? "H" : "I") + "|f:" + filter_id;
    for (auto& kv : match_labels) h += "|l:" + kv.first + "=" + kv.second;
    for (auto& e : exprs) {
      h += "|e:" + e.key + ":" + std::to_string(e.op);
      for (auto& v : e.values) h += "," + v;
    }
    return h;
  }
};

// corev1.PodAffinityTerm of podAffinity / podAntiAffinity (hostname key)
struct AffTerm {
  bool affinity = false;     // podAffinity (else podAntiAffinity)
  string key;
  bool required = false;
  int32_t weight = 0;
  Spread sel;                // has_selector / match_labels / exprs only
  std::set<string> nss;      // buildNamespaceList: the term's list, else the pod's namespace
  string hash() const {      // TopologyGroup.Hash: type, key, namespaces, selector
    string h = string(affinity ? "aff|" : "anti|") + key + "|" + (sel.has_selector ? "1" : "0");
    for (auto& n : nss) h += "|n:" + n;
    for (auto& kv : sel.match_labels) h += "|l:" + kv.first + "=" + kv.second;
    for (auto& e : sel.exprs) {
      h += "|e:" + e.key + ":" + std::to_string(e.op);
      for (auto& v : e.values) h += "," + v;
    }
    return h;
  }
};

// <U> scheduling.HostPort (GetHostPorts: nil hostIP parse -> 0.0.0.0, "" protocol -> TCP)
struct HostPort {
  string proto;
  bool unspecified = true;
  std::array<uint8_t, 16> ip{};  // IPv4 as ::ffff:a.b.c.d (net.IP.Equal)
  int32_t port = 0;
  bool matches(const HostPort& o) const {
    if (proto != o.proto || port != o.port) return false;
    if (unspecified || o.unspecified) return true;
    return ip == o.ip;
  }
};

bool ports_conflict(const vector<HostPort>& used, const vector<HostPort>& want) {
  for (auto& w : want)
    for (auto& u : used)
      if (w.matches(u)) return true;
  return false;
}

struct Pod {
  uint32_t index;
  string uid;
  int64_t ts;
  Res requests;
  std::map<string, string> node_selector;
  vector<Term> required;   // mutable (relaxation)
  vector<Term> preferred;  // mutable (relaxation)
  vector<Toleration> tolerations;
  Reqs reqs;    // cached PodData.Requirements
  Reqs strict;  // cached PodData.StrictRequirements (no preferred term)
  string ns;
  std::map<string, string> labels;
  vector<Spread> spreads;  // mutable (relaxation)
  vector<AffTerm> anti_required;
  vector<AffTerm> anti_preferred;  // mutable (relaxation)
  vector<AffTerm> aff_required;
  vector<AffTerm> aff_preferred;   // mutable (relaxation)
  vector<std::pair<string, string>> volumes;  // (CSI driver, volume id)
  vector<HostPort> ports;
};

struct Template {
  uint32_t np_index;
  string name;
  int32_t weight;
  Reqs reqs;
  vector<Taint> taints;
  vector<const InstanceType*> options;
  Res daemon;
  bool has_limits;
};

struct NodeClaim {
  const Template* tmpl;
  Reqs reqs;
  vector<const InstanceType*> options;
  Res requests;
  vector<const Pod*> pods;
  vector<HostPort> ports;  // hostPortUsage
};

struct ExistingNode {
  uint32_t index;
  string name;
  bool initialized;
  Reqs reqs;
  Reqs label_reqs;  // NewLabelRequirements(node.Labels) + hostname: countDomains reads the Node, not the Solve's state
  vector<Taint> taints;
  Res available, requests;
  vector<const Pod*> pods;
  vector<HostPort> ports;  // hostPortUsage of the bound pods
  std::map<string, std::set<string>> vols;  // VolumeUsage: driver -> volume ids
  std::map<string, int64_t> vol_limits;     // CSINode allocatable counts
};

// <U> NewPodRequirements: nodeSelector + heaviest preferred term (sort.Slice
// by weight desc, mutating the pod's slice) + first required term.
void update_pod_reqs(Pod& p) {
  Reqs r;
  for (auto& kv : p.node_selector) r.add(make_req(kv.first, GS_OP_IN, {kv.second}, std::nullopt));
  if (!p.preferred.empty()) {
    struct D {
      vector<Term>& t;
      bool less(int i, int j) { return t[i].weight > t[j].weight; }
      void swap(int i, int j) { std::swap(t[i], t[j]); }
    } d{p.preferred};
    gosort::slice(d, (int)p.preferred.size());
    for (auto& q : p.preferred[0].reqs) r.add(q);
  }
  Reqs strict;
  for (auto& kv : p.node_selector) strict.add(make_req(kv.first, GS_OP_IN, {kv.second}, std::nullopt));
  if (!p.required.empty()) {
    for (auto& q : p.required[0].reqs) r.add(q);
    for (auto& q : p.required[0].reqs) strict.add(q);
  }
  p.reqs = std::move(r);
  p.strict = std::move(strict);
}

// <U> Requirements.HasMinValues
bool has_min_values(const Reqs& reqs) {
  for (auto& kv : reqs.m)
    if (kv.second.min_values) return true;
  return false;
}

// <U> InstanceTypes.SatisfiesMinValues: for every requirement with minValues,
// the union of the instance types' values for its key (it.Requirements.Get(
// key).Values(): none when the type does not carry the key) is large enough
bool satisfies_min_values(const vector<const InstanceType*>& its, const Reqs& reqs) {
  for (auto& kv : reqs.m) {
    if (!kv.second.min_values) continue;
    std::set<string> vals;
    for (auto* it : its) {
      const Req r = it->reqs.get(kv.first);
      vals.insert(r.values.begin(), r.values.end());
    }
    if ((int64_t)vals.size() < *kv.second.min_values) return false;
  }
  return true;
}

// <U> filterInstanceTypesByRequirements (no short-circuit across ITs); a
// minValues miss (Strict policy) leaves nothing
vector<const InstanceType*> filter_its(const vector<const InstanceType*>& its, const Reqs& reqs, const Res& requests) {
  vector<const InstanceType*> out;
  for (auto* it : its) {
    bool compat = it->reqs.intersects(reqs);
    bool f = fits(requests, it->allocatable);
    bool has_off = false;
    for (auto& of : it->offerings) {
      if (of.available && reqs.compatible(of.reqs, true)) {
        has_off = true;
        break;
      }
    }
    if (compat && f && has_off) out.push_back(it);
  }
  if (has_min_values(reqs) && !satisfies_min_values(out, reqs)) out.clear();
  return out;
}

// <U> cloudprovider.InstanceTypes.OrderByPrice + Truncate(60)
vector<const InstanceType*> order_by_price(vector<const InstanceType*> its, const Reqs& reqs, size_t max_items) {
  auto cheapest = [&](const InstanceType* it) {
    double best = 0;
    bool any = false;
    for (auto& of : it->offerings) {
      if (!of.available || !reqs.compatible(of.reqs, true)) continue;
      if (!any || of.price < best) {
        best = of.price;
        any = true;
      }
    }
    return any ? best : __DBL_MAX__;
  };
  vector<std::pair<double, const InstanceType*>> keyed;
  for (auto* it : its) keyed.push_back({cheapest(it), it});
  // the comparator is a total order (names are unique) so any sort gives
  // sort.Slice's result
  std::sort(keyed.begin(), keyed.end(), [](const auto& a, const auto& b) {
    if (a.first == b.first) return a.second->name < b.second->name;
    return a.first < b.first;
  });
  vector<const InstanceType*> out;
  for (size_t i = 0; i < keyed.size() && i < max_items; i++) out.push_back(keyed[i].second);
  return out;
}

// <U> scheduling.TopologyGroup with an empty node filter:
// TopologyTypeSpread, TopologyTypePodAntiAffinity or TopologyTypePodAffinity
struct TGroup {
  bool anti = false;
  bool aff = false;
  string key;
  int32_t max_skew;
  optional<int32_t> min_domains;
  string ns;                          // spread: the owner's namespace
  std::set<string> nss;               // anti-affinity: the term's namespaces
  Spread sel;
  std::map<string, int64_t> domains;  // known domains and their counts
  std::set<uint32_t> owners;          // pod indices
  // <U> TopologyNodeFilter of a spread group (its first owner's; affinity
  // and anti-affinity groups have none and always match)
  bool spread = false;
  bool honor_affinity = false, honor_taints = false;
  vector<Reqs> filter;
  vector<Toleration> filter_tols;
  // <U> TopologyDomainGroup: the taints of every NodePool / node providing a
  // domain (ForEachDomain under TaintPolicy Honor)
  std::map<string, vector<vector<Taint>>> dom_taints;
  // TopologyNodeFilter.Matches(taints, requirements, compatibility options)
  bool filter_matches(const vector<Taint>& taints, const Reqs& reqs, bool allow_wellknown) const {
    if (!spread) return true;
    if (honor_affinity && !filter.empty()) {
      bool any = false;
      for (auto& f : filter) any = any || reqs.compatible(f, allow_wellknown);
      if (!any) return false;
    }
    return !honor_taints || tolerates_all(taints, filter_tols);
  }
  bool selects(const Pod& p) const {
    return (anti || aff ? nss.count(p.ns) > 0 : p.ns == ns) && sel.matches(p.labels);
  }
};

struct OracleState {
  vector<string> strings;
  vector<InstanceType> its;
  vector<Pod> pods;
  vector<Template> templates;  // filtered + ordered
  vector<ExistingNode> nodes;  // ordered
  vector<uint32_t> node_order;
  std::map<string, Res> remaining;  // nodepools with limits
  bool tolerate_pns = false;
  vector<string> resource_names;
  vector<TGroup> groups;            // creation order
  std::map<string, size_t> group_index;
  vector<TGroup> inverse;           // t.inverseTopologies (required anti-affinity)
  std::map<string, size_t> inverse_index;
  // NewTopology's inputs, kept for the groups Topology.Update creates
  // mid-Solve (a relaxation that changes a spread owner's node filter gives
  // it a new TopologyGroup.Hash): the domain universe and the bound pods
  vector<Reqs> np_reqs;
  vector<bool> np_has_its;
  vector<vector<Taint>> np_taints;
  vector<Pod> bound;
  vector<uint32_t> bound_node;
  vector<vector<Taint>> bound_node_taints;  // the Node's own taints (countDomains' filter)
};

// <U> a group's domains before any count: the In values of the requirements
// (+labels) of NodePools that have instance types, and of the existing
// nodes' labels, with the taints of each provider (TopologyDomainGroup)
void group_universe(const OracleState& st, TGroup& g) {
  for (size_t i = 0; i < st.np_reqs.size(); i++) {
    if (!st.np_has_its[i] || !st.np_reqs[i].has_key(g.key)) continue;
    const Req q = st.np_reqs[i].get(g.key);
    if (q.op() == GS_OP_IN)
      for (auto& v : q.values) {
        g.domains.emplace(v, 0);
        g.dom_taints[v].push_back(st.np_taints[i]);
      }
  }
  for (auto& n : st.nodes) {
    if (!n.label_reqs.has_key(g.key)) continue;
    const Req q = n.label_reqs.get(g.key);
    if (q.op() == GS_OP_IN)
      for (auto& v : q.values) {
        g.domains.emplace(v, 0);
        g.dom_taints[v].push_back(n.taints);
      }
  }
}

// <U> Topology.countDomains: selected bound pods on their nodes' domains,
// where the node passes the group's filter (the Node's own taints and
// labels, strict Compatible)
void count_domains(const OracleState& st, TGroup& g) {
  for (size_t b = 0; b < st.bound.size(); b++) {
    const Pod& bp = st.bound[b];
    const ExistingNode& n = st.nodes[st.bound_node[b]];
    if (!g.selects(bp) || !n.label_reqs.has_key(g.key)) continue;
    if (!g.filter_matches(st.bound_node_taints[b], n.label_reqs, false)) continue;
    const Req q = n.label_reqs.get(g.key);
    if (q.op() != GS_OP_IN) continue;
    if (g.anti)
      for (auto& v : q.values) g.domains[v]++;
    else if (q.values.size() == 1)
      g.domains[*q.values.begin()]++;
  }
}

// <U> NewTopologyGroup for a spread constraint of a pod in namespace ns
TGroup spread_group(const Spread& sp, const string& ns) {
  TGroup g;
  g.key = sp.key;
  g.max_skew = sp.max_skew;
  g.min_domains = sp.min_domains;
  g.ns = ns;
  g.sel = sp;
  g.spread = true;
  g.honor_affinity = !sp.ignore_affinity;
  g.honor_taints = sp.honor_taints;
  g.filter = sp.filter;
  g.filter_tols = sp.filter_tols;
  return g;
}

struct Builder {
  const gs_problem* p;
  OracleState& st;

  const string& str(uint32_t id) {
    if (id >= p->n_strings) throw Unsupported{GS_E_INVALID, "string id out of range"};
    return st.strings[id];
  }
  void check_range(gs_range r, uint32_t n, const char* what) {
    if ((uint64_t)r.begin + r.count > n) throw Unsupported{GS_E_INVALID, string("range out of bounds: ") + what};
  }
  bool allow_placeholder = false;  // launch-time filter: hostname values are plain labels
  // NodeSelectorRequirementWithMinValues appear in NodePool and NodeClaim
  // requirements; a pod's NodeSelectorRequirement has no minValues
  bool allow_min_values = false;
  Req req_of(const gs_requirement& q) {
    if (q.op > GS_OP_LTE) throw Unsupported{GS_E_INVALID, "unknown requirement operator"};
    if (!allow_placeholder && normalize_key(str(q.key)) == kHostname)
      for (uint32_t i = 0; i < q.values.count && q.values.begin + i < p->n_value_ids; i++)
        if (str(p->value_ids[q.values.begin + i]).rfind("hostname-placeholder-", 0) == 0)
          throw Unsupported{GS_E_UNSUPPORTED, "requirement names a hostname placeholder"};
    if (q.min_values >= 0 && !allow_min_values) throw Unsupported{GS_E_UNSUPPORTED, "minValues outside NodePool / NodeClaim requirements"};
    check_range(q.values, p->n_value_ids, "values");
    vector<string> vals;
    for (uint32_t i = 0; i < q.values.count; i++) vals.push_back(str(p->value_ids[q.values.begin + i]));
    return make_req(str(q.key), (int)q.op, vals,
                    q.min_values >= 0 ? optional<int64_t>(q.min_values) : std::nullopt);
  }
  vector<Req> raw_reqs(gs_range r) {
    check_range(r, p->n_reqs, "reqs");
    vector<Req> out;
    for (uint32_t i = 0; i < r.count; i++) out.push_back(req_of(p->reqs[r.begin + i]));
    return out;
  }
  Reqs reqs_of(gs_range r) {
    Reqs out;
    for (auto& q : raw_reqs(r)) out.add(q);
    return out;
  }
  Res res_of(gs_range r) {
    check_range(r, p->n_quantities, "quantities");
    Res out;
    for (uint32_t i = 0; i < r.count; i++) {
      auto& q = p->quantities[r.begin + i];
      out[str(q.resource)] += q.milli;
    }
    return out;
  }
  vector<Taint> taints_of(gs_range r) {
    check_range(r, p->n_taints, "taints");
    vector<Taint> out;
    for (uint32_t i = 0; i < r.count; i++) {
      auto& t = p->taints[r.begin + i];
      out.push_back({str(t.key), str(t.value), str(t.effect)});
    }
    return out;
  }
  // <U> StateNode.Taints() (karpenter pkg/controllers/state/statenode.go,
  // restated from upstream v1.x; the contract is spelled out at gs_node in
  // include/gpusched.h): reject KnownEphemeralTaints, and while a managed node
  // is not initialized also its NodeClaim's startup taints, from the
  // NodeClaim's taints (uninitialized managed node) or the node's; a rejected
  // taint matches by key and effect (corev1 Taint.MatchTaint)
  vector<Taint> state_taints(const gs_node& g) {
    const bool starting = g.managed != 0 && g.initialized == 0;
    vector<Taint> reject = {{"node.kubernetes.io/not-ready", "", "NoSchedule"},
                            {"node.kubernetes.io/unreachable", "", "NoSchedule"},
                            {"node.cloudprovider.kubernetes.io/uninitialized", "true", "NoSchedule"},
                            {"karpenter.sh/unregistered", "", "NoExecute"}};
    const vector<Taint> startup = taints_of(g.startup_taints);
    const vector<Taint> claim = taints_of(g.claim_taints);
    const vector<Taint> node = taints_of(g.taints);
    if (starting) reject.insert(reject.end(), startup.begin(), startup.end());
    vector<Taint> out;
    for (auto& t : starting ? claim : node) {
      bool matched = false;
      for (auto& r : reject)
        if (r.key == t.key && r.effect == t.effect) matched = true;
      if (!matched) out.push_back(t);
    }
    return out;
  }
  std::map<string, string> labels_of(gs_range r) {
    check_range(r, p->n_labels, "labels");
    std::map<string, string> out;
    for (uint32_t i = 0; i < r.count; i++) out[str(p->labels[r.begin + i].key)] = str(p->labels[r.begin + i].value);
    return out;
  }

  // <U> MakeTopologyNodeFilter over the pod's node selector, required
  // node-affinity terms and tolerations (set before pod_meta by build())
  static void node_filter(const Pod& pd, Spread& sp) {
    Reqs sel;
    for (auto& kv : pd.node_selector) sel.add(make_req(kv.first, GS_OP_IN, {kv.second}, std::nullopt));
    sp.filter.clear();
    if (pd.required.empty()) sp.filter.push_back(sel);
    for (auto& tm : pd.required) {
      Reqs r = sel;
      for (auto& q : tm.reqs) r.add(q);
      sp.filter.push_back(std::move(r));
    }
    sp.filter_tols = pd.tolerations;
    vector<string> terms, tols;
    for (auto& r : sp.filter) {
      string k;
      for (auto& kv : r.m) k += kv.first + ",";
      terms.push_back(k);
    }
    for (auto& t : pd.tolerations) tols.push_back(t.key + "=" + t.value + ":" + t.effect + "/" + std::to_string(t.op));
    std::sort(terms.begin(), terms.end());
    std::sort(tols.begin(), tols.end());
    sp.filter_id.clear();
    for (auto& t : terms) sp.filter_id += t + ";";
    sp.filter_id += "#";
    for (auto& t : tols) sp.filter_id += t + ";";
  }

  // namespace, labels and topology spread constraints of a pod
  void pod_meta(const gs_pod& g, Pod& pd, bool pending = true) {
    pd.ns = str(g.ns);
    pd.labels = labels_of(g.labels);
    check_range(g.spreads, p->n_spreads, "spreads");
    for (uint32_t k = 0; k < (pending ? g.spreads.count : 0); k++) {
      const gs_spread& q = p->spreads[g.spreads.begin + k];
      Spread sp;
      sp.key = normalize_key(str(q.topology_key));
      if (sp.key != kZone && sp.key != kHostname && sp.key != kCapacityType && sp.key != kNodePool)
        throw Unsupported{GS_E_UNSUPPORTED, "topology spread key other than zone / capacity type / NodePool / hostname"};
      if (q.max_skew < 1) throw Unsupported{GS_E_INVALID, "maxSkew < 1"};
      if (q.when_unsatisfiable > GS_SPREAD_SCHEDULE_ANYWAY || q.node_affinity_policy > GS_POLICY_IGNORE ||
          q.node_taints_policy > GS_POLICY_IGNORE)
        throw Unsupported{GS_E_INVALID, "bad topology spread enum"};
      sp.honor_taints = q.node_taints_policy == GS_POLICY_HONOR;
      sp.max_skew = q.max_skew;
      sp.schedule_anyway = q.when_unsatisfiable == GS_SPREAD_SCHEDULE_ANYWAY;
      if (q.min_domains > 0) sp.min_domains = q.min_domains;
      sp.has_selector = q.has_selector != 0;
      sp.match_labels = labels_of(q.match_labels);
      check_range(q.match_expressions, p->n_reqs, "reqs");
      for (uint32_t e = 0; e < q.match_expressions.count; e++) {
        const gs_requirement& r = p->reqs[q.match_expressions.begin + e];
        if (r.op > GS_OP_DOES_NOT_EXIST) throw Unsupported{GS_E_INVALID, "label selector operator"};
        check_range(r.values, p->n_value_ids, "values");
        Spread::Expr x{str(r.key), (int)r.op, {}};
        for (uint32_t v = 0; v < r.values.count; v++) x.values.insert(str(p->value_ids[r.values.begin + v]));
        sp.exprs.push_back(std::move(x));
      }
      // matchLabelKeys: key In [the pod's value] for every key the pod carries
      check_range(q.match_label_keys, p->n_value_ids, "values");
      for (uint32_t m = 0; m < q.match_label_keys.count; m++) {
        const string& k = str(p->value_ids[q.match_label_keys.begin + m]);
        auto f = pd.labels.find(k);
        if (f != pd.labels.end()) sp.exprs.push_back(Spread::Expr{k, GS_OP_IN, {f->second}});
      }
      sp.ignore_affinity = q.node_affinity_policy == GS_POLICY_IGNORE;
      node_filter(pd, sp);
      pd.spreads.push_back(std::move(sp));
    }
    auto terms = [&](gs_range rg, bool affinity) {
      check_range(rg, p->n_affinity_terms, "affinity_terms");
      for (uint32_t k = 0; k < rg.count; k++) {
        const gs_affinity_term& q = p->affinity_terms[rg.begin + k];
        AffTerm a;
        a.affinity = affinity;
        a.key = normalize_key(str(q.topology_key));
        // zone-key anti-affinity is deterministic (nextDomainAntiAffinity: every
        // empty domain); zone-key affinity bootstraps on a zone in Go map order
        if (a.key != kHostname && !(a.key == kZone && !affinity))
          throw Unsupported{GS_E_UNSUPPORTED, affinity ? "pod affinity topologyKey other than hostname"
                                                       : "pod anti-affinity topologyKey other than hostname / zone"};
        a.required = q.required != 0;
        a.weight = q.weight;
        a.sel.has_selector = q.has_selector != 0;
        a.sel.match_labels = labels_of(q.match_labels);
        check_range(q.match_expressions, p->n_reqs, "reqs");
        for (uint32_t e = 0; e < q.match_expressions.count; e++) {
          const gs_requirement& r = p->reqs[q.match_expressions.begin + e];
          if (r.op > GS_OP_DOES_NOT_EXIST) throw Unsupported{GS_E_INVALID, "label selector operator"};
          check_range(r.values, p->n_value_ids, "values");
          Spread::Expr x{str(r.key), (int)r.op, {}};
          for (uint32_t v = 0; v < r.values.count; v++) x.values.insert(str(p->value_ids[r.values.begin + v]));
          a.sel.exprs.push_back(std::move(x));
        }
        // <U> buildNamespaceList
        check_range(q.namespaces, p->n_value_ids, "values");
        for (uint32_t v = 0; v < q.namespaces.count; v++) a.nss.insert(str(p->value_ids[q.namespaces.begin + v]));
        if (q.has_ns_selector) {
          Spread nsel;
          nsel.has_selector = true;
          nsel.match_labels = labels_of(q.ns_match_labels);
          check_range(q.ns_match_expressions, p->n_reqs, "reqs");
          for (uint32_t e = 0; e < q.ns_match_expressions.count; e++) {
            const gs_requirement& r = p->reqs[q.ns_match_expressions.begin + e];
            if (r.op > GS_OP_DOES_NOT_EXIST) throw Unsupported{GS_E_INVALID, "label selector operator"};
            check_range(r.values, p->n_value_ids, "values");
            Spread::Expr x{str(r.key), (int)r.op, {}};
            for (uint32_t v = 0; v < r.values.count; v++) x.values.insert(str(p->value_ids[r.values.begin + v]));
            nsel.exprs.push_back(std::move(x));
          }
          check_range(gs_range{0, p->n_namespaces}, p->n_namespaces, "namespaces");
          for (uint32_t n = 0; n < p->n_namespaces; n++)
            if (nsel.matches(labels_of(p->namespaces[n].labels))) a.nss.insert(str(p->namespaces[n].name));
        } else if (a.nss.empty()) {
          a.nss.insert(pd.ns);
        }
        if (affinity) (a.required ? pd.aff_required : pd.aff_preferred).push_back(std::move(a));
        else (a.required ? pd.anti_required : pd.anti_preferred).push_back(std::move(a));
      }
    };
    terms(g.anti_affinity, false);
    if (pending) terms(g.affinity, true);  // pod affinity has no inverse: bound pods' terms do nothing
    if (pd.aff_preferred.size() > 12) throw Unsupported{GS_E_UNSUPPORTED, "more than 12 preferred pod affinity terms"};
    if (pd.anti_preferred.size() > 12) throw Unsupported{GS_E_UNSUPPORTED, "more than 12 preferred anti-affinity terms"};
    check_range(g.volumes, p->n_volumes, "volumes");
    for (uint32_t k = 0; k < g.volumes.count; k++)
      pd.volumes.push_back({str(p->volumes[g.volumes.begin + k].driver), str(p->volumes[g.volumes.begin + k].id)});
    check_range(g.host_ports, p->n_host_ports, "host_ports");
    for (uint32_t k = 0; k < g.host_ports.count; k++) {
      const gs_host_port& q = p->host_ports[g.host_ports.begin + k];
      if (q.port < 1 || q.port > 65535) throw Unsupported{GS_E_INVALID, "host port out of range"};
      HostPort hp;
      hp.proto = str(q.protocol).empty() ? "TCP" : str(q.protocol);
      hp.port = q.port;
      // net.ParseIP; nil -> 0.0.0.0
      const string& ip = str(q.ip);
      uint8_t b6[16];
      in_addr b4;
      if (inet_pton(AF_INET, ip.c_str(), &b4) == 1) {
        std::memset(hp.ip.data(), 0, 10);
        hp.ip[10] = hp.ip[11] = 0xff;
        std::memcpy(hp.ip.data() + 12, &b4, 4);
      } else if (inet_pton(AF_INET6, ip.c_str(), b6) == 1) {
        std::memcpy(hp.ip.data(), b6, 16);
      } else {
        hp.ip.fill(0);
        hp.ip[10] = hp.ip[11] = 0xff;  // 0.0.0.0
      }
      static const std::array<uint8_t, 16> z6{}, z4{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xff, 0xff, 0, 0, 0, 0};
      hp.unspecified = hp.ip == z6 || hp.ip == z4;  // IsUnspecified
      pd.ports.push_back(std::move(hp));
    }
  }

  TGroup anti_group(const AffTerm& a) {
    TGroup g;
    g.anti = !a.affinity;
    g.aff = a.affinity;
    g.key = a.key;
    g.max_skew = INT32_MAX;
    g.nss = a.nss;
    g.sel = a.sel;
    return g;
  }

  // <U> NewTopology: one group per distinct constraint of the pods being
  // scheduled; domain universe = In values of NodePool (+labels, + instance
  // type) requirements of NodePools that have instance types, plus existing
  // nodes' labels; counts = selected bound pods on existing nodes
  void build_topology() {
    for (auto& pd : st.pods)
      for (auto& sp : pd.spreads) {
        const string h = sp.hash(pd.ns);
        auto f = st.group_index.find(h);
        if (f == st.group_index.end()) {
          f = st.group_index.emplace(h, st.groups.size()).first;
          st.groups.push_back(spread_group(sp, pd.ns));
        }
        st.groups[f->second].owners.insert(pd.index);
      }
    // <U> newForTopologies: required and preferred anti-affinity terms
    for (auto& pd : st.pods)
      for (auto* terms : {&pd.anti_required, &pd.anti_preferred, &pd.aff_required, &pd.aff_preferred})
        for (auto& a : *terms) {
          const string h = a.hash();
          auto f = st.group_index.find(h);
          if (f == st.group_index.end()) {
            f = st.group_index.emplace(h, st.groups.size()).first;
            st.groups.push_back(anti_group(a));
          }
          st.groups[f->second].owners.insert(pd.index);
        }
    // <U> updateInverseAntiAffinity: one inverse group per required term,
    // owned by the pods that carry it (pending pods here, bound pods below)
    auto inverse_of = [&](const AffTerm& a) -> TGroup& {
      const string h = a.hash();
      auto f = st.inverse_index.find(h);
      if (f == st.inverse_index.end()) {
        f = st.inverse_index.emplace(h, st.inverse.size()).first;
        st.inverse.push_back(anti_group(a));
      }
      return st.inverse[f->second];
    };
    for (auto& pd : st.pods)
      for (auto& a : pd.anti_required) inverse_of(a).owners.insert(pd.index);
    st.bound.assign(p->n_bound_pods, Pod{});
    st.bound_node.assign(p->n_bound_pods, 0);
    st.bound_node_taints.assign(p->n_bound_pods, {});
    for (uint32_t b = 0; b < p->n_bound_pods; b++) {
      if (p->bound_pod_node[b] >= st.nodes.size()) throw Unsupported{GS_E_INVALID, "bound pod node out of range"};
      Pod& bp = st.bound[b];
      bp.index = UINT32_MAX;
      pod_meta(p->bound_pods[b], bp, false);
      st.bound_node[b] = p->bound_pod_node[b];
      st.bound_node_taints[b] = taints_of(p->nodes[p->bound_pod_node[b]].taints);
      for (auto& a : bp.anti_required) inverse_of(a);
      // ExistingNode hostPortUsage and VolumeUsage
      auto& n = st.nodes[p->bound_pod_node[b]];
      n.ports.insert(n.ports.end(), bp.ports.begin(), bp.ports.end());
      for (auto& v : bp.volumes) n.vols[v.first].insert(v.second);
    }
    if (st.groups.empty() && st.inverse.empty()) return;
    // <U> buildDomainGroups takes Requirement.Values() of NodePool x instance
    // type requirements: a NotIn's excluded values, an instance type's own
    // values.  The IBM instance types carry no zone / capacity type
    // (instancetype.go:719-724); the two ambiguous forms are refused
    for (auto* gs : {&st.groups, &st.inverse})
      for (auto& g : *gs) {
        if (g.key == kHostname) continue;
        for (size_t i = 0; i < st.np_reqs.size(); i++)
          if (st.np_has_its[i] && st.np_reqs[i].has_key(g.key) && st.np_reqs[i].get(g.key).op() == GS_OP_NOTIN)
            throw Unsupported{GS_E_UNSUPPORTED, "NodePool NotIn requirement on a topology key"};
        for (auto& it : st.its)
          if (it.reqs.has_key(g.key)) throw Unsupported{GS_E_UNSUPPORTED, "instance type requirement on a topology key"};
      }
    for (auto* gs : {&st.groups, &st.inverse})
      for (auto& g : *gs) group_universe(st, g);
    for (auto& g : st.groups) count_domains(st, g);
    // updateInverseAffinities: a bound carrier of a required term blocks its node
    for (uint32_t b = 0; b < p->n_bound_pods; b++) {
      const ExistingNode& n = st.nodes[st.bound_node[b]];
      for (auto& a : st.bound[b].anti_required) {
        TGroup& g = st.inverse[st.inverse_index.at(a.hash())];
        if (!n.label_reqs.has_key(g.key)) continue;
        const Req q = n.label_reqs.get(g.key);
        if (q.op() == GS_OP_IN)
          for (auto& v : q.values) g.domains[v]++;
      }
    }
  }

  void build() {
    st.strings.clear();
    for (uint32_t i = 0; i < p->n_strings; i++) st.strings.push_back(p->strings[i] ? p->strings[i] : "");
    // catalog
    st.its.resize(p->n_instance_types);
    for (uint32_t i = 0; i < p->n_instance_types; i++) {
      auto& g = p->instance_types[i];
      auto& it = st.its[i];
      it.index = i;
      it.name = str(g.name);
      it.reqs = reqs_of(g.requirements);
      it.capacity = res_of(g.capacity);
      it.overhead = res_of(g.overhead);
      it.allocatable = subtract(it.capacity, it.overhead);
      check_range(g.offerings, p->n_offerings, "offerings");
      for (uint32_t k = 0; k < g.offerings.count; k++) {
        auto& o = p->offerings[g.offerings.begin + k];
        it.offerings.push_back({reqs_of(o.requirements), o.price, o.available != 0});
      }
    }
    // templates: NodePools ordered by weight desc then name (<U> OrderByWeight)
    vector<uint32_t> order(p->n_nodepools);
    for (uint32_t i = 0; i < p->n_nodepools; i++) order[i] = i;
    std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
      auto& A = p->nodepools[a];
      auto& B = p->nodepools[b];
      if (A.weight == B.weight) return str(A.name) < str(B.name);
      return A.weight > B.weight;
    });
    auto& np_reqs = st.np_reqs;
    auto& np_has_its = st.np_has_its;
    auto& np_taints = st.np_taints;
    for (uint32_t npi : order) {
      auto& np = p->nodepools[npi];
      Template t;
      t.np_index = npi;
      t.name = str(np.name);
      t.weight = np.weight;
      allow_min_values = true;
      Reqs npreqs = reqs_of(np.requirements);
      allow_min_values = false;
      t.reqs = npreqs;
      auto labels = labels_of(np.labels);
      labels[kNodePool] = t.name;
      for (auto& kv : labels) t.reqs.add(make_req(kv.first, GS_OP_IN, {kv.second}, std::nullopt));
      t.taints = taints_of(np.taints);
      t.daemon = res_of(np.daemon_requests);
      t.has_limits = np.has_limits != 0;
      // CloudProvider.GetInstanceTypes filter (reference cloudprovider.go:573-577)
      check_range(np.instance_types, p->n_it_refs, "it_refs");
      vector<const InstanceType*> its;
      for (uint32_t k = 0; k < np.instance_types.count; k++) {
        uint32_t idx = p->it_refs[np.instance_types.begin + k];
        if (idx >= st.its.size()) throw Unsupported{GS_E_INVALID, "it_ref out of range"};
        const InstanceType* it = &st.its[idx];
        if (npreqs.compatible(it->reqs, true)) its.push_back(it);
      }
      np_reqs.push_back(t.reqs);
      np_has_its.push_back(!its.empty());
      np_taints.push_back(t.taints);
      // <U> NewScheduler: pre-filter instance types per template
      t.options = filter_its(its, t.reqs, Res{});
      if (t.has_limits) st.remaining[t.name] = res_of(np.limits);
      if (t.options.empty()) continue;
      st.templates.push_back(std::move(t));
    }
    for (auto& t : st.templates)
      for (auto& tn : t.taints)
        if (tn.effect == kEffectPreferNoSchedule) st.tolerate_pns = true;
    // pods
    st.pods.resize(p->n_pods);
    std::set<string> uids;
    for (uint32_t i = 0; i < p->n_pods; i++) {
      auto& g = p->pods[i];
      if (g.flags) throw Unsupported{GS_E_UNSUPPORTED, "pod topology/affinity/host ports/volumes"};
      auto& pd = st.pods[i];
      pd.index = i;
      pd.uid = str(g.uid);
      if (!uids.insert(pd.uid).second) throw Unsupported{GS_E_INVALID, "duplicate pod uid"};
      pd.ts = g.creation_ns;
      pd.requests = res_of(g.requests);
      pd.node_selector = labels_of(g.node_selector);
      check_range(g.required_terms, p->n_terms, "terms");
      for (uint32_t k = 0; k < g.required_terms.count; k++) {
        auto& tm = p->terms[g.required_terms.begin + k];
        pd.required.push_back({raw_reqs(tm.requirements), tm.weight});
      }
      check_range(g.preferred_terms, p->n_terms, "terms");
      for (uint32_t k = 0; k < g.preferred_terms.count; k++) {
        auto& tm = p->terms[g.preferred_terms.begin + k];
        pd.preferred.push_back({raw_reqs(tm.requirements), tm.weight});
      }
      check_range(g.tolerations, p->n_tolerations, "tolerations");
      for (uint32_t k = 0; k < g.tolerations.count; k++) {
        auto& t = p->tolerations[g.tolerations.begin + k];
        pd.tolerations.push_back({str(t.key), str(t.value), str(t.effect), (int)t.op});
      }
      pod_meta(g, pd);
      update_pod_reqs(pd);
    }
    // existing nodes: <U> initialized first, then by name (sort.SliceStable)
    st.nodes.resize(p->n_nodes);
    for (uint32_t i = 0; i < p->n_nodes; i++) {
      auto& g = p->nodes[i];
      auto& n = st.nodes[i];
      n.index = i;
      n.name = str(g.name);
      n.initialized = g.initialized != 0;
      for (auto& kv : labels_of(g.labels)) n.reqs.add(make_req(kv.first, GS_OP_IN, {kv.second}, std::nullopt));
      n.reqs.add(make_req(kHostname, GS_OP_IN, {n.name}, std::nullopt));
      n.label_reqs = n.reqs;
      n.taints = state_taints(g);
      n.available = res_of(g.available);
      n.requests = res_of(g.requests);
      check_range(g.volume_limits, p->n_volume_limits, "volume_limits");
      for (uint32_t k = 0; k < g.volume_limits.count; k++) {
        const gs_volume_limit& l = p->volume_limits[g.volume_limits.begin + k];
        n.vol_limits[str(l.driver)] = l.limit;
      }
    }
    st.node_order.resize(p->n_nodes);
    for (uint32_t i = 0; i < p->n_nodes; i++) st.node_order[i] = i;
    std::stable_sort(st.node_order.begin(), st.node_order.end(), [&](uint32_t a, uint32_t b) {
      auto& A = st.nodes[a];
      auto& B = st.nodes[b];
      if (A.initialized != B.initialized) return A.initialized;
      return A.name < B.name;
    });
    build_topology();
    // resource vocabulary (for dense claim requests)
    std::set<string> rn;
    for (uint32_t i = 0; i < p->n_quantities; i++) rn.insert(str(p->quantities[i].resource));
    st.resource_names.assign(rn.begin(), rn.end());
  }
};

// <U> Preferences.Relax: first applicable relaxation, in order
bool relax(Pod& p, bool tolerate_pns) {
  // removeRequiredNodeAffinityTerm
  if (p.required.size() > 1) {
    p.required.erase(p.required.begin());
    return true;
  }
  // removePreferredPodAffinityTerm: sort.Slice by weight desc, drop [0]
  if (!p.aff_preferred.empty()) {
    struct D {
      vector<AffTerm>& t;
      bool less(int i, int j) { return t[i].weight > t[j].weight; }
      void swap(int i, int j) { std::swap(t[i], t[j]); }
    } d{p.aff_preferred};
    gosort::slice(d, (int)p.aff_preferred.size());
    p.aff_preferred.erase(p.aff_preferred.begin());
    return true;
  }
  // removePreferredPodAntiAffinityTerm: sort.Slice by weight desc, drop [0]
  if (!p.anti_preferred.empty()) {
    struct D {
      vector<AffTerm>& t;
      bool less(int i, int j) { return t[i].weight > t[j].weight; }
      void swap(int i, int j) { std::swap(t[i], t[j]); }
    } d{p.anti_preferred};
    gosort::slice(d, (int)p.anti_preferred.size());
    p.anti_preferred.erase(p.anti_preferred.begin());
    return true;
  }
  // removePreferredNodeAffinityTerm: sort.SliceStable by weight desc, drop [0]
  if (!p.preferred.empty()) {
    std::stable_sort(p.preferred.begin(), p.preferred.end(),
                     [](const Term& a, const Term& b) { return a.weight > b.weight; });
    p.preferred.erase(p.preferred.begin());
    return true;
  }
  // removeTopologySpreadScheduleAnyway: swap-remove the first ScheduleAnyway
  for (size_t i = 0; i < p.spreads.size(); i++)
    if (p.spreads[i].schedule_anyway) {
      p.spreads[i] = p.spreads.back();
      p.spreads.pop_back();
      return true;
    }
  if (tolerate_pns) {
    for (auto& t : p.tolerations)
      if (t.key.empty() && t.op == GS_TOL_EXISTS && t.value.empty() && t.effect == kEffectPreferNoSchedule) return false;
    p.tolerations.push_back({"", "", kEffectPreferNoSchedule, GS_TOL_EXISTS});
    return true;
  }
  return false;
}

struct Scheduler {
  OracleState& st;

  // ---------------------------------------------------------- <U> Topology
  // <U> TopologyDomainGroup.ForEachDomain: under TaintPolicy Honor a domain
  // takes part only if some NodePool / node providing it has taints the pod
  // tolerates (a domain with no recorded provider is kept)
  static bool domain_tolerated(const TGroup& g, const string& d, const Pod& pod) {
    if (!g.honor_taints) return true;
    auto f = g.dom_taints.find(d);
    if (f == g.dom_taints.end() || f->second.empty()) return true;
    for (auto& ts : f->second)
      if (tolerates_all(ts, pod.tolerations)) return true;
    return false;
  }
  // TopologyGroup.domainMinCount
  int64_t domain_min_count(const TGroup& g, const Req& pod_domains, const Pod& pod) const {
    if (g.key == kHostname) return 0;
    int64_t mn = INT32_MAX;
    int32_t n = 0;
    for (auto& kv : g.domains)
      if (pod_domains.has(kv.first) && domain_tolerated(g, kv.first, pod)) {
        n++;
        mn = std::min(mn, kv.second);
      }
    if (g.min_domains && n < *g.min_domains) mn = 0;
    return mn;
  }
  // TopologyGroup.nextDomainTopologySpread: the minimum-count domain among
  // the node's domains within maxSkew.  Upstream iterates a Go map / an
  // unsorted set, so ties fall in random order; restated: smallest name.
  Req next_domain(const TGroup& g, const Pod& pod, const Req& pod_domains, const Req& node_domains) const {
    if (g.aff) {
      // nextDomainAffinity: the domains the pod allows that hold a selected
      // pod; while none does, a self-selecting pod bootstraps on one domain
      // both sides allow (upstream takes the first in map order: for the
      // hostname key the node side allows exactly one, its own)
      vector<string> opts;
      for (auto& kv : g.domains)
        if (kv.second > 0 && pod_domains.has(kv.first)) opts.push_back(kv.first);
      if (opts.empty() && g.selects(pod)) {
        for (auto& kv : g.domains)
          if (pod_domains.has(kv.first) && node_domains.has(kv.first)) {
            opts.push_back(kv.first);
            break;
          }
        if (opts.empty())
          for (auto& kv : g.domains)
            if (pod_domains.has(kv.first)) {
              opts.push_back(kv.first);
              break;
            }
      }
      if (opts.empty()) return make_req(g.key, GS_OP_DOES_NOT_EXIST, {}, std::nullopt);
      return make_req(g.key, GS_OP_IN, opts, std::nullopt);
    }
    if (g.anti) {
      // nextDomainAntiAffinity: the empty domains both sides allow
      vector<string> opts;
      for (auto& kv : g.domains)
        if (kv.second == 0 && node_domains.has(kv.first) && pod_domains.has(kv.first)) opts.push_back(kv.first);
      if (opts.empty()) return make_req(g.key, GS_OP_DOES_NOT_EXIST, {}, std::nullopt);
      return make_req(g.key, GS_OP_IN, opts, std::nullopt);
    }
    const int64_t mn = domain_min_count(g, pod_domains, pod);
    const int64_t self = g.selects(pod) ? 1 : 0;
    string best;
    int64_t best_count = INT32_MAX;
    auto consider = [&](const string& d, int64_t count) {
      count += self;
      if (count - mn <= g.max_skew && count < best_count) {
        best = d;
        best_count = count;
      }
    };
    if (node_domains.op() == GS_OP_IN) {
      for (auto& d : node_domains.values) {
        auto f = g.domains.find(d);
        if (f != g.domains.end()) consider(d, f->second);
      }
    } else {
      for (auto& kv : g.domains)
        if (node_domains.has(kv.first)) consider(kv.first, kv.second);
    }
    if (best_count == INT32_MAX) return make_req(g.key, GS_OP_DOES_NOT_EXIST, {}, std::nullopt);
    return make_req(g.key, GS_OP_IN, {best}, std::nullopt);
  }
  // Topology.AddRequirements over the groups the pod owns
  bool topology = true;  // off for the static (fresh NodeClaim) feasibility matrix
  bool topo_requirements(const Pod& pod, const Reqs& node_reqs, Reqs* out) const {
    if (!topology) return true;
    // getMatchingTopologies: owned groups, then inverse groups that select the pod
    vector<const TGroup*> match;
    for (auto& g : st.groups)
      if (g.owners.count(pod.index)) match.push_back(&g);
    for (auto& g : st.inverse)
      if (g.selects(pod)) match.push_back(&g);
    for (const TGroup* gp : match) {
      const TGroup& g = *gp;
      const Req pd = pod.strict.has_key(g.key) ? pod.strict.get(g.key) : make_req(g.key, GS_OP_EXISTS, {}, std::nullopt);
      const Req nd = node_reqs.has_key(g.key) ? node_reqs.get(g.key) : make_req(g.key, GS_OP_EXISTS, {}, std::nullopt);
      const Req d = next_domain(g, pod, pd, nd);
      if (d.len() == 0) return false;
      out->add(d);
    }
    return true;
  }
  // Topology.Record: every group that selects the pod counts the domain it
  // landed in, when that domain is known (a single value)
  // (TopologyGroup.Counts: the group selects the pod and its filter matches
  // the node / NodeClaim: taints, requirements; NodeClaims with
  // AllowUndefinedWellKnownLabels)
  void topo_record(const Pod& pod, const Reqs& reqs, const vector<Taint>& taints, bool allow_wellknown) {
    for (auto& g : st.groups) {
      if (!g.selects(pod) || !reqs.has_key(g.key)) continue;
      if (!g.filter_matches(taints, reqs, allow_wellknown)) continue;
      const Req d = reqs.get(g.key);
      if (d.complement) continue;
      if (g.anti) {
        for (auto& v : d.values) g.domains[v]++;  // every domain the pod could be in
      } else if (d.values.size() == 1) {
        g.domains[*d.values.begin()]++;
      }
    }
    // inverse groups the pod owns record where it landed
    for (auto& g : st.inverse) {
      if (!g.owners.count(pod.index) || !reqs.has_key(g.key)) continue;
      const Req d = reqs.get(g.key);
      if (!d.complement)
        for (auto& v : d.values) g.domains[v]++;
    }
  }
  // Topology.Register(hostname, placeholder)
  void topo_register_hostname(const string& h) {
    for (auto* gs : {&st.groups, &st.inverse})
      for (auto& g : *gs)
        if (g.key == kHostname) g.domains.emplace(h, 0);
  }
  // <U> Topology.Update after a relaxation: the pod leaves every group, then
  // owns the groups of its remaining constraints.  A spread's node filter
  // (MakeTopologyNodeFilter) is rebuilt from the relaxed pod: a dropped
  // required node-affinity term or the added PreferNoSchedule toleration
  // changes TopologyGroup.Hash, and a hash not seen yet is a group created
  // now, whose countDomains sees the cluster's bound pods only -- none of this
  // Solve's placements so far, and none of the hostname placeholders
  // registered before it
  uint64_t groups_created_in_solve = 0;
  void topo_update(Pod& pod) {
    for (auto& g : st.groups) g.owners.erase(pod.index);
    for (auto& sp : pod.spreads) {
      Builder::node_filter(pod, sp);
      auto f = st.group_index.find(sp.hash(pod.ns));
      if (f == st.group_index.end()) {
        f = st.group_index.emplace(sp.hash(pod.ns), st.groups.size()).first;
        st.groups.push_back(spread_group(sp, pod.ns));
        group_universe(st, st.groups.back());
        count_domains(st, st.groups.back());
        groups_created_in_solve++;
      }
      st.groups[f->second].owners.insert(pod.index);
    }
    for (auto* terms : {&pod.anti_required, &pod.anti_preferred, &pod.aff_required, &pod.aff_preferred})
      for (auto& a : *terms) {
        auto f = st.group_index.find(a.hash());
        if (f != st.group_index.end()) st.groups[f->second].owners.insert(pod.index);
      }
  }

  vector<NodeClaim*> claims;  // s.newNodeClaims (sorted in place per pod)
  vector<std::unique_ptr<NodeClaim>> owned;
  vector<NodeClaim*> creation_order;
  uint64_t pops = 0;
  uint64_t node_id = 0;  // <U> package-level nodeID counter, per solve here

  // <U> NodeClaim.CanAdd; returns true and fills the update on success
  bool claim_can_add(const NodeClaim& n, const Pod& pod, Reqs* reqs_out, vector<const InstanceType*>* its_out,
                     Res* req_out) {
    if (!tolerates_all(n.tmpl->taints, pod.tolerations)) return false;
    if (ports_conflict(n.ports, pod.ports)) return false;  // hostPortUsage.Conflicts
    Res requests = merge(n.requests, pod.requests);
    // Evaluation order only (same result): filterInstanceTypesByRequirements
    // keeps an instance type only if Fits(requests, allocatable), and every
    // step before it is side-effect free, so when no option fits the merged
    // requests CanAdd is false whatever the requirement checks would say.
    bool any_fit = false;
    for (auto* it : n.options)
      if (fits(requests, it->allocatable)) {
        any_fit = true;
        break;
      }
    if (!any_fit) return false;
    Reqs nr = n.reqs;  // NewRequirements(n.Requirements.Values()...)
    if (!nr.compatible(pod.reqs, true)) return false;
    nr.add_all(pod.reqs);
    Reqs topo;
    if (!topo_requirements(pod, nr, &topo)) return false;
    if (!nr.compatible(topo, true)) return false;
    nr.add_all(topo);
    auto remaining = filter_its(n.options, nr, requests);
    if (remaining.empty()) return false;
    *reqs_out = std::move(nr);
    *its_out = std::move(remaining);
    *req_out = std::move(requests);
    return true;
  }

  // <U> ExistingNode.CanAdd (strict Compatible: no AllowUndefined)
  bool node_can_add(const ExistingNode& n, const Pod& pod, Reqs* reqs_out, Res* req_out) {
    if (!tolerates_all(n.taints, pod.tolerations)) return false;
    if (ports_conflict(n.ports, pod.ports)) return false;  // hostPortUsage.Conflicts
    {
      // <U> VolumeUsage.ExceedsLimits: every driver of the union within its limit
      auto u = n.vols;
      for (auto& v : pod.volumes) u[v.first].insert(v.second);
      for (auto& kv : u) {
        auto f = n.vol_limits.find(kv.first);
        if (f != n.vol_limits.end() && (int64_t)kv.second.size() > f->second) return false;
      }
    }
    Res requests = merge(n.requests, pod.requests);
    if (!fits(requests, n.available)) return false;
    Reqs nr = n.reqs;
    if (!nr.compatible(pod.reqs, false)) return false;
    nr.add_all(pod.reqs);
    Reqs topo;
    if (!topo_requirements(pod, nr, &topo)) return false;
    if (!nr.compatible(topo, false)) return false;
    nr.add_all(topo);
    *reqs_out = std::move(nr);
    *req_out = std::move(requests);
    return true;
  }

  uint64_t claim_calls = 0, node_calls = 0;  // CanAdd calls (instrumentation)
  bool add(Pod& pod) {
    for (uint32_t ni : st.node_order) {
      auto& n = st.nodes[ni];
      Reqs r;
      Res q;
      node_calls++;
      if (node_can_add(n, pod, &r, &q)) {
        n.reqs = std::move(r);
        n.requests = std::move(q);
        n.pods.push_back(&pod);
        n.ports.insert(n.ports.end(), pod.ports.begin(), pod.ports.end());
        for (auto& v : pod.volumes) n.vols[v.first].insert(v.second);
        topo_record(pod, n.reqs, n.taints, false);
        return true;
      }
    }
    // sort.Slice(s.newNodeClaims, len(Pods) asc)
    struct D {
      vector<NodeClaim*>& c;
      bool less(int i, int j) { return c[i]->pods.size() < c[j]->pods.size(); }
      void swap(int i, int j) { std::swap(c[i], c[j]); }
    } d{claims};
    gosort::slice(d, (int)claims.size());
    for (auto* nc : claims) {
      Reqs r;
      vector<const InstanceType*> its;
      Res q;
      claim_calls++;
      if (claim_can_add(*nc, pod, &r, &its, &q)) {
        nc->reqs = std::move(r);
        nc->options = std::move(its);
        nc->requests = std::move(q);
        nc->pods.push_back(&pod);
        nc->ports.insert(nc->ports.end(), pod.ports.begin(), pod.ports.end());
        topo_record(pod, nc->reqs, nc->tmpl->taints, true);
        return true;
      }
    }
    for (auto& t : st.templates) {
      vector<const InstanceType*> its = t.options;
      auto rem = st.remaining.find(t.name);
      if (rem != st.remaining.end()) {
        // <U> filterByRemainingResources
        vector<const InstanceType*> f;
        for (auto* it : its) {
          bool viable = true;
          for (auto& kv : rem->second)
            if (res_get(it->capacity, kv.first) > kv.second) viable = false;
          if (viable) f.push_back(it);
        }
        its = std::move(f);
        if (its.empty()) continue;
      }
      // <U> NewNodeClaim: template reqs + hostname placeholder, requests = daemon
      auto nc = std::make_unique<NodeClaim>();
      nc->tmpl = &t;
      nc->reqs = t.reqs;
      char hn[48];
      std::snprintf(hn, sizeof hn, "hostname-placeholder-%04llu", (unsigned long long)++node_id);
      topo_register_hostname(hn);
      nc->reqs.add(make_req(kHostname, GS_OP_IN, {hn}, std::nullopt));
      nc->options = its;
      nc->requests = t.daemon;
      Reqs r;
      vector<const InstanceType*> its2;
      Res q;
      if (!claim_can_add(*nc, pod, &r, &its2, &q)) continue;
      nc->reqs = std::move(r);
      nc->options = std::move(its2);
      nc->requests = std::move(q);
      nc->pods.push_back(&pod);
      nc->ports.insert(nc->ports.end(), pod.ports.begin(), pod.ports.end());
      topo_record(pod, nc->reqs, nc->tmpl->taints, true);
      if (rem != st.remaining.end()) {
        // <U> subtractMax(remaining, nodeClaim.InstanceTypeOptions)
        Res mx;
        for (auto* it : nc->options)
          for (auto& kv : it->capacity) {
            auto f = mx.find(kv.first);
            if (f == mx.end() || kv.second > f->second) mx[kv.first] = kv.second;
          }
        for (auto& kv : rem->second) kv.second -= res_get(mx, kv.first);
      }
      claims.push_back(nc.get());
      creation_order.push_back(nc.get());
      owned.push_back(std::move(nc));
      return true;
    }
    return false;
  }

  // <U> Scheduler.Solve: queue + relax loop; returns error pods
  std::set<uint32_t> solve() {
    vector<Pod*> q;
    for (auto& p : st.pods) q.push_back(&p);
    // <U> NewQueue: byCPUAndMemoryDescending, then creationTimestamp, then UID
    // (a total order, so std::sort reproduces sort.Slice)
    std::sort(q.begin(), q.end(), [](const Pod* a, const Pod* b) {
      int64_t ac = res_get(a->requests, "cpu"), bc = res_get(b->requests, "cpu");
      if (ac != bc) return ac > bc;
      int64_t am = res_get(a->requests, "memory"), bm = res_get(b->requests, "memory");
      if (am != bm) return am > bm;
      if (a->ts != b->ts) return a->ts < b->ts;
      return a->uid < b->uid;
    });
    std::unordered_map<const Pod*, size_t> last_len;
    std::set<uint32_t> errors;
    size_t head = 0;
    std::vector<Pod*> queue = q;  // queue[head..]
    for (;;) {
      if (head >= queue.size()) break;
      Pod* p = queue[head];
      size_t len = queue.size() - head;
      auto ll = last_len.find(p);
      if (ll != last_len.end() && ll->second == len) break;
      head++;
      pops++;
      if (add(*p)) {
        errors.erase(p->index);
        continue;
      }
      errors.insert(p->index);
      bool relaxed = relax(*p, st.tolerate_pns);
      queue.push_back(p);
      if (relaxed) {
        last_len.clear();
        update_pod_reqs(*p);
        topo_update(*p);
      } else {
        last_len[p] = queue.size() - head;
      }
    }
    return errors;
  }
};

// ------------------------------------------------------------- result memory
struct ResultStore {
  vector<uint32_t> claim_nodepool, claim_pod_offsets, claim_pods, claim_it_offsets, claim_its;
  vector<string> req_text;
  vector<const char*> req_ptrs;
  vector<uint32_t> resource_names;
  vector<int64_t> claim_requests;
  vector<uint32_t> node_pod_offsets, node_pods, error_pods;
  // feasibility
  vector<uint64_t> rows;
  vector<int32_t> cheapest;
  vector<uint32_t> nfeas;
};
ResultStore g_res;
OracleState* g_state = nullptr;
uint64_t g_groups_created = 0;  // the last oracle_solve's groups created by Topology.Update

}  // namespace

extern "C" gs_status oracle_solve(const gs_problem* problem, gs_result* out) {
  auto t0 = std::chrono::steady_clock::now();
  delete g_state;
  g_state = new OracleState();
  OracleState& st = *g_state;
  try {
    Builder b{problem, st};
    b.build();
  } catch (const Unsupported& u) {
    return u.code;
  }
  const double build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  Scheduler s{st};
  auto errors = s.solve();
  ResultStore& r = g_res;
  r = ResultStore();
  r.claim_pod_offsets.push_back(0);
  r.claim_it_offsets.push_back(0);
  std::map<string, uint32_t> name_to_id;
  for (uint32_t i = 0; i < problem->n_strings; i++) name_to_id.emplace(st.strings[i], i);
  for (auto& rn : st.resource_names) r.resource_names.push_back(name_to_id[rn]);
  for (auto* nc : s.creation_order) {
    // FinalizeScheduling: drop hostname requirement
    nc->reqs.m.erase(kHostname);
    // <U> Results.TruncateInstanceTypes: a NodeClaim whose top 60 by price
    // miss minValues is dropped and its pods become pod errors
    auto top = order_by_price(nc->options, nc->reqs, 60);
    if (has_min_values(nc->reqs) && !satisfies_min_values(top, nc->reqs)) {
      for (auto* p : nc->pods) errors.insert(p->index);
      continue;
    }
    r.claim_nodepool.push_back(nc->tmpl->np_index);
    for (auto* p : nc->pods) r.claim_pods.push_back(p->index);
    r.claim_pod_offsets.push_back((uint32_t)r.claim_pods.size());
    for (auto* it : top) r.claim_its.push_back(it->index);
    r.claim_it_offsets.push_back((uint32_t)r.claim_its.size());
    r.req_text.push_back(canonical(nc->reqs));
    for (auto& rn : st.resource_names) r.claim_requests.push_back(res_get(nc->requests, rn));
  }
  for (auto& t : r.req_text) r.req_ptrs.push_back(t.c_str());
  r.node_pod_offsets.push_back(0);
  for (auto& n : st.nodes) {
    for (auto* p : n.pods) r.node_pods.push_back(p->index);
    r.node_pod_offsets.push_back((uint32_t)r.node_pods.size());
  }
  r.error_pods.assign(errors.begin(), errors.end());
  std::memset(out, 0, sizeof(*out));
  out->n_claims = (uint32_t)r.claim_nodepool.size();
  out->claim_nodepool = r.claim_nodepool.data();
  out->claim_pod_offsets = r.claim_pod_offsets.data();
  out->claim_pods = r.claim_pods.data();
  out->claim_it_offsets = r.claim_it_offsets.data();
  out->claim_its = r.claim_its.data();
  out->claim_requirements = r.req_ptrs.data();
  out->n_resources = (uint32_t)r.resource_names.size();
  out->resource_names = r.resource_names.data();
  out->claim_requests = r.claim_requests.data();
  out->n_nodes = (uint32_t)st.nodes.size();
  out->node_pod_offsets = r.node_pod_offsets.data();
  out->node_pods = r.node_pods.data();
  out->n_errors = (uint32_t)r.error_pods.size();
  out->error_pods = r.error_pods.data();
  out->pops = s.pops;
  out->claim_prefix = s.claim_calls;
  out->t_encode_ms = build_ms;  // the oracle's own input build (string sets)
  out->node_prefix = s.node_calls;
  g_groups_created = s.groups_created_in_solve;
  out->t_total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return GS_OK;
}

// instrumentation for the KATs: spread groups the last oracle_solve created
// mid-Solve (a relaxation re-keyed a spread owner)
extern "C" uint64_t oracle_last_groups_created(void) { return g_groups_created; }

extern "C" gs_status oracle_feasibility(const gs_problem* problem, gs_feas_result* out) {
  auto t0 = std::chrono::steady_clock::now();
  delete g_state;
  g_state = new OracleState();
  OracleState& st = *g_state;
  try {
    Builder b{problem, st};
    b.build();
  } catch (const Unsupported& u) {
    return u.code;
  }
  uint32_t P = problem->n_pods, T = problem->n_nodepools, N = problem->n_instance_types;
  uint32_t W = (N + 63) / 64;
  ResultStore& r = g_res;
  r = ResultStore();
  r.rows.assign((size_t)P * T * W, 0);
  r.cheapest.assign((size_t)P * T, -1);
  r.nfeas.assign((size_t)P * T, 0);
  uint64_t checks = 0;
  Scheduler s{st};
  s.topology = false;
  for (auto& t : st.templates) {
    for (auto* it : t.options) checks += (uint64_t)it->offerings.size() * P;
  }
  for (uint32_t pi = 0; pi < P; pi++) {
    const Pod& pod = st.pods[pi];
    for (auto& t : st.templates) {
      vector<const InstanceType*> its = t.options;
      auto rem = st.remaining.find(t.name);
      if (rem != st.remaining.end()) {
        vector<const InstanceType*> f;
        for (auto* it : its) {
          bool viable = true;
          for (auto& kv : rem->second)
            if (res_get(it->capacity, kv.first) > kv.second) viable = false;
          if (viable) f.push_back(it);
        }
        its = std::move(f);
      }
      NodeClaim nc;
      nc.tmpl = &t;
      nc.reqs = t.reqs;
      nc.reqs.add(make_req(kHostname, GS_OP_IN, {"hostname-placeholder-0001"}, std::nullopt));
      nc.options = its;
      nc.requests = t.daemon;
      Reqs rq;
      vector<const InstanceType*> rem_its;
      Res q;
      if (its.empty() || !s.claim_can_add(nc, pod, &rq, &rem_its, &q)) continue;
      size_t base = ((size_t)pi * T + t.np_index);
      uint32_t nf = 0;
      for (auto* it : rem_its) {
        r.rows[base * W + it->index / 64] |= 1ull << (it->index % 64);
        for (auto& of : it->offerings)
          if (of.available && rq.compatible(of.reqs, true)) nf++;
      }
      r.nfeas[base] = nf;
      rq.m.erase(kHostname);
      auto ordered = order_by_price(rem_its, rq, 1);
      r.cheapest[base] = ordered.empty() ? -1 : (int32_t)ordered[0]->index;
    }
  }
  std::memset(out, 0, sizeof(*out));
  out->n_pods = P;
  out->n_nodepools = T;
  out->n_its = N;
  out->words = W;
  out->rows = r.rows.data();
  out->cheapest_it = r.cheapest.data();
  out->n_feasible_offerings = r.nfeas.data();
  out->checks = checks;
  out->t_kernel_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return GS_OK;
}

extern "C" void oracle_go_sort_ints(int64_t* keys, uint32_t* perm, uint32_t n) {
  for (uint32_t i = 0; i < n; i++) perm[i] = i;
  struct D {
    int64_t* k;
    uint32_t* p;
    bool less(int i, int j) { return k[i] < k[j]; }
    void swap(int i, int j) {
      std::swap(k[i], k[j]);
      std::swap(p[i], p[j]);
    }
  } d{keys, perm};
  gosort::slice(d, (int)n);
}

// ===================================================================== consolidation
// <U> pkg/controllers/disruption (karpenter v1.13.0): SimulateScheduling,
// computeConsolidation, getCandidatePrices, filterByPrice,
// filterOutSameInstanceType, SingleNodeConsolidation.ComputeCommand (first
// non-NoOp in candidate order) and MultiNodeConsolidation
// .firstNConsolidationOption (binary search over candidates[0:mid+1]).
// SpotToSpotConsolidation is off (feature-gate default).  Each simulation is
// a fresh Builder + Scheduler over the reduced problem: deliberately naive.
namespace {

struct ConsStore {
  vector<gs_command> cmds;
  vector<uint32_t> opts;
  vector<double> prices;
};
ConsStore g_cons;

const char* kInstanceType = "node.kubernetes.io/instance-type";

struct Candidate {
  bool priced = false;  // getCandidatePrices found an offering
  double price = 0;
  string it_name;
  bool it_found = false;
  bool spot = false;
};

// <U> Candidate construction + getCandidatePrices for one state node:
// c.instanceType.Offerings.Compatible(NewLabelRequirements(labels)).Cheapest()
Candidate candidate_of(const gs_problem* p, const OracleState& st, uint32_t node) {
  Candidate c;
  Builder b{p, const_cast<OracleState&>(st)};
  auto labels = b.labels_of(p->nodes[node].labels);
  Reqs lr;
  for (auto& kv : labels) lr.add(make_req(kv.first, GS_OP_IN, {kv.second}, std::nullopt));
  auto ct = labels.find(kCapacityType);
  c.spot = ct != labels.end() && ct->second == "spot";
  auto itn = labels.find(kInstanceType);
  if (itn == labels.end()) return c;
  c.it_name = itn->second;
  for (auto& it : st.its) {
    if (it.name != c.it_name) continue;
    c.it_found = true;
    for (auto& of : it.offerings) {
      if (!lr.compatible(of.reqs, true)) continue;
      if (!c.priced || of.price < c.price) {
        c.price = of.price;
        c.priced = true;
      }
    }
    break;
  }
  return c;
}

// cheapest available offering compatible with reqs (OrderByPrice's key)
double cheapest_available(const InstanceType* it, const Reqs& reqs) {
  double best = __DBL_MAX__;
  bool any = false;
  for (auto& of : it->offerings) {
    if (!of.available || !reqs.compatible(of.reqs, true)) continue;
    if (!any || of.price < best) {
      best = of.price;
      any = true;
    }
  }
  return best;
}

// one computeConsolidation over a candidate set
gs_command simulate(const gs_consolidation* in, const vector<uint32_t>& cands, const OracleState& base,
                    vector<uint32_t>* opts_out, vector<double>* prices_out) {
  const gs_problem* cl = in->cluster;
  gs_command cmd;
  std::memset(&cmd, 0, sizeof cmd);
  cmd.n_candidates = (uint32_t)cands.size();
  std::set<uint32_t> cset(cands.begin(), cands.end());
  // SimulateScheduling: pending pods + the candidates' reschedulable pods,
  // state nodes minus the candidates
  vector<gs_pod> pods(cl->pods, cl->pods + cl->n_pods);
  const uint32_t n_pending = cl->n_pods;
  for (uint32_t c : cands)
    for (uint32_t b = 0; b < cl->n_bound_pods; b++)
      if (cl->bound_pod_node[b] == c) pods.push_back(cl->bound_pods[b]);
  vector<gs_node> nodes;
  vector<uint32_t> new_index(cl->n_nodes, UINT32_MAX);
  for (uint32_t n = 0; n < cl->n_nodes; n++)
    if (!cset.count(n)) {
      new_index[n] = (uint32_t)nodes.size();
      nodes.push_back(cl->nodes[n]);
    }
  // the other bound pods stay where they are (topology counts)
  vector<gs_pod> bound;
  vector<uint32_t> bound_node;
  for (uint32_t b = 0; b < cl->n_bound_pods; b++)
    if (!cset.count(cl->bound_pod_node[b])) {
      bound.push_back(cl->bound_pods[b]);
      bound_node.push_back(new_index[cl->bound_pod_node[b]]);
    }
  gs_problem sub = *cl;
  sub.pods = pods.data();
  sub.n_pods = (uint32_t)pods.size();
  sub.nodes = nodes.data();
  sub.n_nodes = (uint32_t)nodes.size();
  sub.bound_pods = bound.data();
  sub.n_bound_pods = (uint32_t)bound.size();
  sub.bound_pod_node = bound_node.data();
  OracleState st;
  Builder b{&sub, st};
  b.build();
  Scheduler s{st};
  auto errors = s.solve();
  // Results.TruncateInstanceTypes(MaxInstanceTypes): a NodeClaim whose top 60
  // by OrderByPrice miss a minValues requirement is dropped, its pods become
  // pod errors
  vector<NodeClaim*> kept;
  for (NodeClaim* nc : s.creation_order) {
    Reqs r = nc->reqs;
    r.m.erase(kHostname);
    if (has_min_values(r) && !satisfies_min_values(order_by_price(nc->options, r, 60), r)) {
      for (const Pod* p : nc->pods) errors.insert(p->index);
      continue;
    }
    kept.push_back(nc);
  }
  uint32_t failed = 0;
  for (uint32_t e : errors)
    if (e >= n_pending) failed++;
  // pods scheduled against an uninitialized node are errors too
  for (auto& n : st.nodes)
    if (!n.initialized)
      for (auto* p : n.pods)
        if (p->index >= n_pending) failed++;
  cmd.n_failed_pods = failed;
  cmd.n_new_claims = (uint32_t)kept.size();
  if (failed) {
    cmd.reason = GS_NOOP_UNSCHEDULABLE;
    return cmd;
  }
  if (cmd.n_new_claims == 0) {
    cmd.decision = GS_DECISION_DELETE;
    return cmd;
  }
  if (cmd.n_new_claims > 1) {
    cmd.reason = GS_NOOP_MULTIPLE_CLAIMS;
    return cmd;
  }
  double cp = 0;
  bool all_spot = true;
  for (uint32_t c : cands) {
    Candidate k = candidate_of(cl, base, c);
    if (!k.priced) {
      cmd.reason = GS_NOOP_PRICE_UNKNOWN;
      return cmd;
    }
    cp += k.price;
    all_spot = all_spot && k.spot;
  }
  cmd.candidate_price = cp;
  NodeClaim* nc = kept[0];
  nc->reqs.m.erase(kHostname);  // FinalizeScheduling
  auto ordered = order_by_price(nc->options, nc->reqs, 60);  // TruncateInstanceTypes + OrderByPrice
  Req ctr = nc->reqs.get(kCapacityType);
  if (all_spot && ctr.has("spot")) {
    cmd.reason = GS_NOOP_SPOT_TO_SPOT;
    return cmd;
  }
  // RemoveInstanceTypeOptionsByPriceAndMinValues: the options cheaper than the
  // candidates, then SatisfiesMinValues on what is left
  vector<const InstanceType*> keep;
  vector<double> kp;
  for (auto* it : ordered) {
    double pr = cheapest_available(it, nc->reqs);
    if (pr < cp) {
      keep.push_back(it);
      kp.push_back(pr);
    }
  }
  if (has_min_values(nc->reqs) && !satisfies_min_values(keep, nc->reqs)) {
    cmd.reason = GS_NOOP_MIN_VALUES;
    return cmd;
  }
  if (keep.empty()) {
    cmd.reason = GS_NOOP_NOT_CHEAPER;
    return cmd;
  }
  cmd.decision = GS_DECISION_REPLACE;
  cmd.nodepool = nc->tmpl->np_index;
  cmd.spot_only = ctr.has("spot") && ctr.has("on-demand") ? 1u : 0u;
  cmd.options.begin = (uint32_t)opts_out->size();
  cmd.options.count = (uint32_t)keep.size();
  for (size_t i = 0; i < keep.size(); i++) {
    opts_out->push_back(keep[i]->index);
    prices_out->push_back(kp[i]);
  }
  return cmd;
}

// <U> filterOutSameInstanceType on a Replace command's options
vector<uint32_t> filter_out_same_type(const gs_consolidation* in, const OracleState& base, const vector<uint32_t>& cands,
                                      const uint32_t* opts, const double* prices, uint32_t n) {
  std::set<string> existing;
  std::map<string, double> price_by_type;
  for (uint32_t c : cands) {
    Candidate k = candidate_of(in->cluster, base, c);
    existing.insert(k.it_name);
    if (!k.priced) continue;
    auto f = price_by_type.find(k.it_name);
    double ex = f == price_by_type.end() ? __DBL_MAX__ : f->second;
    if (k.price < ex) price_by_type[k.it_name] = k.price;
  }
  double max_price = __DBL_MAX__;
  for (uint32_t i = 0; i < n; i++) {
    const string& nm = base.its[opts[i]].name;
    if (!existing.count(nm)) continue;
    auto f = price_by_type.find(nm);
    double pr = f == price_by_type.end() ? 0.0 : f->second;  // Go map zero value
    if (pr < max_price) max_price = pr;
  }
  vector<uint32_t> out;
  for (uint32_t i = 0; i < n; i++)
    if (prices[i] < max_price) out.push_back(i);  // filterByPrice
  return out;
}

}  // namespace

extern "C" gs_status oracle_consolidate(const gs_consolidation* in, gs_consolidation_result* out, int32_t* chosen_out,
                                        uint32_t* multi_opts, uint32_t* n_multi_opts) {
  if (!in || !in->cluster || !out) return GS_E_INVALID;
  OracleState base;
  vector<vector<uint32_t>> sets;
  uint32_t mx = 0;
  try {
    Builder b{in->cluster, base};
    b.build();
    for (uint32_t i = 0; i < in->n_candidates; i++)
      if (in->candidates[i] >= in->cluster->n_nodes) return GS_E_INVALID;
    for (uint32_t i = 0; i < in->cluster->n_bound_pods; i++)
      if (in->cluster->bound_pod_node[i] >= in->cluster->n_nodes) return GS_E_INVALID;
    if (in->mode == GS_CONSOLIDATE_EVAL) {
      for (uint32_t s = 0; s < in->n_sets; s++) {
        if ((uint64_t)in->sets[s].begin + in->sets[s].count > in->n_candidates) return GS_E_INVALID;
        sets.emplace_back(in->candidates + in->sets[s].begin, in->candidates + in->sets[s].begin + in->sets[s].count);
      }
    } else if (in->mode == GS_CONSOLIDATE_SINGLE) {
      for (uint32_t i = 0; i < in->n_candidates; i++) sets.push_back({in->candidates[i]});
    } else if (in->mode == GS_CONSOLIDATE_MULTI) {
      const uint32_t n = in->n_candidates, cap = in->max_candidates ? in->max_candidates : 100;
      mx = n < cap ? n : cap;  // lo.Clamp(len, 0, 100)
      if (n >= 2) {
        if (n <= mx) mx = n - 1;
        for (uint32_t mid = 1; mid <= mx; mid++) sets.emplace_back(in->candidates, in->candidates + mid + 1);
      }
    } else {
      return GS_E_INVALID;
    }
    ConsStore& r = g_cons;
    r = ConsStore();
    for (auto& set : sets) r.cmds.push_back(simulate(in, set, base, &r.opts, &r.prices));
  } catch (const Unsupported& u) {
    return u.code;
  }
  ConsStore& r = g_cons;
  int32_t chosen = -1;
  if (n_multi_opts) *n_multi_opts = 0;
  if (in->mode == GS_CONSOLIDATE_SINGLE) {
    for (size_t i = 0; i < r.cmds.size(); i++)
      if (r.cmds[i].decision != GS_DECISION_NOOP) {
        chosen = (int32_t)i;
        break;
      }
  } else if (in->mode == GS_CONSOLIDATE_MULTI && !sets.empty()) {
    int lo = 1, hi = (int)mx;
    vector<uint32_t> saved;
    while (lo <= hi) {
      const int mid = (lo + hi) / 2;
      const gs_command& c = r.cmds[mid - 1];
      bool valid = false;
      vector<uint32_t> keep;
      if (c.decision == GS_DECISION_REPLACE) {
        auto idx = filter_out_same_type(in, base, sets[mid - 1], r.opts.data() + c.options.begin,
                                        r.prices.data() + c.options.begin, c.options.count);
        for (uint32_t i : idx) keep.push_back(r.opts[c.options.begin + i]);
        valid = !keep.empty();
        // RemoveInstanceTypeOptionsByPriceAndMinValues inside
        // filterOutSameInstanceType: a minValues miss invalidates the prefix
        for (auto& t : base.templates)
          if (t.np_index == c.nodepool && has_min_values(t.reqs)) {
            vector<const InstanceType*> its;
            for (uint32_t x : keep) its.push_back(&base.its[x]);
            if (!satisfies_min_values(its, t.reqs)) valid = false;
          }
      }
      if (valid || c.decision == GS_DECISION_DELETE) {
        chosen = mid - 1;
        saved = keep;
        lo = mid + 1;
      } else {
        hi = mid - 1;
      }
    }
    if (multi_opts && n_multi_opts) {
      for (size_t i = 0; i < saved.size() && i < 60; i++) multi_opts[i] = saved[i];
      *n_multi_opts = (uint32_t)std::min<size_t>(saved.size(), 60);
    }
  }
  if (chosen_out) *chosen_out = chosen;
  std::memset(out, 0, sizeof(*out));
  out->n_commands = (uint32_t)r.cmds.size();
  out->commands = r.cmds.data();
  out->options = r.opts.data();
  out->option_prices = r.prices.data();
  out->chosen = chosen;
  return GS_OK;
}

// ===================================================================== launch-time re-filter
// CloudProvider.Create (reference pkg/cloudprovider/cloudprovider.go:320-346):
//   reqs := NewNodeSelectorRequirementsWithMinValues(nodeClaim.Spec.Requirements...)
//   compatible := lo.Filter(instanceTypes, reqs.Compatible(i.Requirements, AllowUndefinedWellKnownLabels) == nil
//       && len(i.Offerings.Compatible(reqs).Available()) > 0 && resources.Fits(requests, i.Allocatable()))
// GetInstanceTypes (:574-577): the requirement clause alone.
// instance provider (vpc/instance/provider.go:215-221): instanceTypes[0].
// ResolveCapacityType (common/capacitytype/capacitytype.go:27-42).
namespace {

struct CatalogOracle {
  OracleState st;
  Builder b;
  explicit CatalogOracle(const gs_problem* p) : b{p, st} {
    b.allow_placeholder = true;
    b.allow_min_values = true;  // Compatible ignores minValues (cloudprovider.go:321-325)
    for (uint32_t i = 0; i < p->n_strings; i++) st.strings.push_back(p->strings[i] ? p->strings[i] : "");
    st.its.resize(p->n_instance_types);
    for (uint32_t i = 0; i < p->n_instance_types; i++) {
      auto& g = p->instance_types[i];
      auto& it = st.its[i];
      it.index = i;
      it.name = b.str(g.name);
      it.reqs = b.reqs_of(g.requirements);
      it.capacity = b.res_of(g.capacity);
      it.overhead = b.res_of(g.overhead);
      it.allocatable = subtract(it.capacity, it.overhead);
      b.check_range(g.offerings, p->n_offerings, "offerings");
      for (uint32_t k = 0; k < g.offerings.count; k++) {
        auto& o = p->offerings[g.offerings.begin + k];
        it.offerings.push_back({b.reqs_of(o.requirements), o.price, o.available != 0});
      }
    }
  }
  // Offerings.Compatible(reqs).Available(), in offering order
  static vector<const Offering*> available(const InstanceType& it, const Reqs& reqs) {
    vector<const Offering*> out;
    for (auto& o : it.offerings)
      if (reqs.compatible(o.reqs, true) && o.available) out.push_back(&o);
    return out;
  }
  static bool create_ok(const InstanceType& it, const Reqs& reqs, const Res& requests) {
    const bool req_ok = reqs.compatible(it.reqs, true);
    const bool off_ok = !available(it, reqs).empty();
    const bool fit = fits(requests, it.allocatable);
    return req_ok && off_ok && fit;
  }
  static uint32_t resolve_capacity_type(const Reqs& reqs, const vector<const InstanceType*>& its) {
    const Req allowed = reqs.get(kCapacityType);
    if (allowed.has("spot"))
      for (auto* it : its)
        for (auto* o : available(*it, reqs))
          if (o->reqs.get(kCapacityType).has("spot")) return GS_CAPACITY_SPOT;
    return GS_CAPACITY_ON_DEMAND;
  }
};

}  // namespace

extern "C" gs_status oracle_create_filter(const gs_problem* catalog, const gs_claim_query* qs, uint32_t nq,
                                          uint64_t* compatible, uint64_t* requirements, int32_t* selected,
                                          uint32_t* capacity_type) {
  try {
    CatalogOracle co(catalog);
    const uint32_t N = catalog->n_instance_types, W = (N + 63) / 64;
    for (uint32_t q = 0; q < nq; q++) {
      const Reqs reqs = co.b.reqs_of(qs[q].requirements);
      const Res requests = co.b.res_of(qs[q].requests);
      vector<const InstanceType*> list;
      for (uint32_t w = 0; w < W; w++) compatible[(size_t)q * W + w] = requirements[(size_t)q * W + w] = 0;
      for (auto& it : co.st.its) {
        if (reqs.compatible(it.reqs, true)) requirements[(size_t)q * W + it.index / 64] |= 1ull << (it.index % 64);
        if (!CatalogOracle::create_ok(it, reqs, requests)) continue;
        compatible[(size_t)q * W + it.index / 64] |= 1ull << (it.index % 64);
        list.push_back(&it);
      }
      selected[q] = list.empty() ? -1 : (int32_t)list[0]->index;
      capacity_type[q] = CatalogOracle::resolve_capacity_type(reqs, list);
    }
  } catch (const Unsupported& u) {
    return u.code;
  }
  return GS_OK;
}

extern "C" gs_status oracle_resolve_capacity_type(const gs_problem* catalog, const gs_claim_query* q,
                                                  const uint32_t* its, uint32_t n, uint32_t* out) {
  try {
    CatalogOracle co(catalog);
    vector<const InstanceType*> list;
    for (uint32_t i = 0; i < n; i++) {
      if (its[i] >= co.st.its.size()) return GS_E_INVALID;
      list.push_back(&co.st.its[its[i]]);
    }
    *out = CatalogOracle::resolve_capacity_type(co.b.reqs_of(q->requirements), list);
  } catch (const Unsupported& u) {
    return u.code;
  }
  return GS_OK;
}
