// encode.cpp — host encoder for the MI355X provisioning solve.
//
// Turns gs_problem (what Go's GetInstanceTypes + NewScheduler inputs carry,
// reference pkg/cloudprovider/cloudprovider.go:553-583) into the bitset/SoA
// layout of layout.hpp.  The requirement algebra here restates <U>
// sigs.k8s.io/karpenter pkg/scheduling (Requirement.Intersection/Has/Len/
// Operator, Requirements.Compatible/Intersects) on vocabulary bitsets; it is
// independent of the oracle's string-set restatement (oracle/solve.cpp).
#include "encode.hpp"

#include <arpa/inet.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <climits>
#include <cstdlib>
#include <exception>
#include <thread>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <sched.h>
#include <unistd.h>
#include <functional>
#include <tuple>
#include <cmath>
#include <cstring>
#include <numeric>
#include <set>
#include <stdexcept>
#include <system_error>
#include <string_view>

namespace gsh {
namespace {

const char* kZone = "topology.kubernetes.io/zone";
const char* kCapacityType = "karpenter.sh/capacity-type";
const char* kHostname = "kubernetes.io/hostname";
const char* kNodePool = "karpenter.sh/nodepool";
const char* kPNS = "PreferNoSchedule";
const char* kOmega = "\x01<unmentioned>";

// host threads of the encoder: GS_ENCODE_THREADS, else the CPUs this process
// may run on (sched_getaffinity) shared among LOCAL_WORLD_SIZE ranks of a
// torchrun job on the host, at most 16 (the GPU boxes give a process 16)
uint32_t enc_threads() {
  static const uint32_t n = [] {
    if (const char* s = std::getenv("GS_ENCODE_THREADS")) {
      const int v = std::atoi(s);
      if (v >= 1) return (uint32_t)std::min(v, 64);
    }
    unsigned cpus = 0;
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof set, &set) == 0) cpus = (unsigned)CPU_COUNT(&set);
    if (!cpus) cpus = std::thread::hardware_concurrency();
    if (const char* s = std::getenv("LOCAL_WORLD_SIZE")) {
      const int w = std::atoi(s);
      if (w > 1) cpus /= (unsigned)w;
    }
    return (uint32_t)std::max(1u, std::min(cpus ? cpus : 1u, 16u));
  }();
  return n;
}

// One process-wide pool of enc_threads() - 1 workers (started on first use,
// never torn down) serves every par_for: a call posts tokens for its job and
// works on it itself, so it completes even when every worker is busy (nested
// or concurrent calls from several contexts' threads).  A forked child has
// no workers and runs its loops serially.
struct PoolJob {
  std::function<void(uint32_t)> f;
  uint32_t n = 0, grain = 1;
  std::atomic<uint32_t> next{0}, done{0};
  std::mutex m;
  std::condition_variable cv;
  void work() {
    for (;;) {
      const uint32_t b = next.fetch_add(grain);
      if (b >= n) break;
      const uint32_t e = std::min(n, b + grain);
      for (uint32_t i = b; i < e; i++) f(i);
      if (done.fetch_add(e - b) + (e - b) == n) {
        std::lock_guard<std::mutex> g(m);
        cv.notify_all();
      }
    }
  }
};
struct Pool {
  pid_t pid = getpid();
  std::mutex m;
  std::condition_variable cv;
  std::deque<std::shared_ptr<PoolJob>> tokens;
  uint32_t workers = 0;
  explicit Pool(uint32_t n) {
    for (uint32_t t = 0; t < n; t++) {
      try {
        std::thread([this] { loop(); }).detach();
        workers++;
      } catch (const std::system_error&) {
        break;  // fewer workers: callers still finish their own jobs
      }
    }
  }
  void loop() {
    for (;;) {
      std::shared_ptr<PoolJob> j;
      {
        std::unique_lock<std::mutex> g(m);
        cv.wait(g, [&] { return !tokens.empty(); });
        j = std::move(tokens.front());
        tokens.pop_front();
      }
      j->work();
    }
  }
};
Pool* pool() {
  static Pool* p = new Pool(enc_threads() - 1);  // intentionally never destroyed (workers block on it)
  return p;
}

// f(i) for every i in [0, n), chunks of `grain` handed out to up to
// enc_threads() threads; f must not throw (callers keep per-item errors and
// raise the first by index afterwards, as the serial encoder would)
template <class F>
void par_for(uint32_t n, uint32_t grain, F&& f) {
  grain = std::max<uint32_t>(grain, 1);
  const uint32_t T = std::min<uint32_t>(enc_threads(), (n + grain - 1) / grain);
  Pool* pl = T > 1 ? pool() : nullptr;
  if (T <= 1 || !pl->workers || pl->pid != getpid()) {
    for (uint32_t i = 0; i < n; i++) f(i);
    return;
  }
  auto j = std::make_shared<PoolJob>();
  j->f = [&f](uint32_t i) { f(i); };
  j->n = n;
  j->grain = grain;
  {
    std::lock_guard<std::mutex> g(pl->m);
    for (uint32_t t = 1; t < T && t <= pl->workers; t++) pl->tokens.push_back(j);
  }
  pl->cv.notify_all();
  j->work();
  std::unique_lock<std::mutex> g(j->m);
  j->cv.wait(g, [&] { return j->done.load() == n; });
}

// g() on a pool worker, not waited for (the calling thread runs it itself
// when there are no workers, and under AddressSanitizer so that its leak
// check at exit sees no work in flight)
void run_detached(std::function<void()> g) {
#if defined(__SANITIZE_ADDRESS__)
  g();
#else
  Pool* pl = enc_threads() > 1 ? pool() : nullptr;
  if (!pl || !pl->workers || pl->pid != getpid()) {
    g();
    return;
  }
  auto j = std::make_shared<PoolJob>();
  j->f = [g = std::move(g)](uint32_t) { g(); };
  j->n = 1;
  {
    std::lock_guard<std::mutex> l(pl->m);
    pl->tokens.push_back(j);
  }
  pl->cv.notify_one();
#endif
}

// <U> v1.WellKnownLabels + IBM keys (reference pkg/apis/v1alpha1/labels.go:37-45)
bool is_wellknown(const std::string& k) {
  static const std::set<std::string> s = {
      "karpenter.sh/nodepool",           "topology.kubernetes.io/zone",      "topology.kubernetes.io/region",
      "node.kubernetes.io/instance-type", "kubernetes.io/arch",              "kubernetes.io/os",
      "karpenter.sh/capacity-type",       "node.kubernetes.io/windows-build", "karpenter-ibm.sh/instance-size",
      "karpenter-ibm.sh/instance-family", "karpenter-ibm.sh/instance-cpu",   "karpenter-ibm.sh/instance-memory"};
  return s.count(k) != 0;
}

std::string normalize(const std::string& k) {
  if (k == "failure-domain.beta.kubernetes.io/zone") return kZone;
  if (k == "failure-domain.beta.kubernetes.io/region") return "topology.kubernetes.io/region";
  if (k == "beta.kubernetes.io/arch") return "kubernetes.io/arch";
  if (k == "beta.kubernetes.io/instance-type") return "node.kubernetes.io/instance-type";
  if (k == "beta.kubernetes.io/os") return "kubernetes.io/os";
  return k;
}

// strconv.Atoi
bool atoi64(const std::string& s, int64_t* out) {
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    i = 1;
  }
  if (i == s.size()) return false;
  unsigned __int128 v = 0;
  for (; i < s.size(); i++) {
    if (s[i] < '0' || s[i] > '9') return false;
    v = v * 10 + (unsigned)(s[i] - '0');
    if (v > (unsigned __int128)INT64_MAX + 1) return false;
  }
  if (!neg && v > (unsigned __int128)INT64_MAX) return false;
  *out = neg ? (int64_t)(-(__int128)v) : (int64_t)v;
  return true;
}

struct Fail {
  gs_status code;
  std::string msg;
};

// values of a vocabulary within (gt, lt)
Bits within_mask(const Vocab& v, bool hg, int64_t gt, bool hl, int64_t lt) {
  Bits b(v.words());
  for (size_t i = 0; i < v.size(); i++) {
    if (!hg && !hl) {
      b.set(i);
      continue;
    }
    if (!v.isint[i]) continue;
    if (hg && gt >= v.ival[i]) continue;
    if (hl && lt <= v.ival[i]) continue;
    b.set(i);
  }
  return b;
}

Bits all_bits(const Vocab& v) { return within_mask(v, false, 0, false, 0); }

}  // namespace

KReq kreq_intersect(const Vocab& v, const KReq& a, const KReq& b) {
  KReq r;
  r.comp = a.comp && b.comp;
  r.hg = a.hg || b.hg;
  r.gt = a.hg && b.hg ? std::max(a.gt, b.gt) : (a.hg ? a.gt : b.gt);
  r.hl = a.hl || b.hl;
  r.lt = a.hl && b.hl ? std::min(a.lt, b.lt) : (a.hl ? a.lt : b.lt);
  r.mv = std::max(a.mv, b.mv);
  if (r.hg && r.hl && r.gt >= r.lt) {  // DoesNotExist
    KReq d;
    d.comp = false;
    d.has = Bits(v.words());
    d.excl = Bits(v.words());
    d.mv = r.mv;
    return d;
  }
  r.has = a.has;
  r.has &= b.has;
  r.excl = Bits(v.words());
  if (r.comp) {
    r.excl = a.excl;
    r.excl |= b.excl;
    r.excl &= within_mask(v, r.hg, r.gt, r.hl, r.lt);
  } else {
    r.hg = r.hl = false;
    r.gt = r.lt = 0;
  }
  return r;
}

namespace {

bool len_zero(const KReq& q) { return !q.comp && q.has.none(); }
int op_of(const KReq& q) {
  if (q.comp) return q.excl.none() ? GS_OP_EXISTS : GS_OP_NOTIN;
  return q.has.none() ? GS_OP_DOES_NOT_EXIST : GS_OP_IN;
}
bool exempt(const KReq& q) {
  int o = op_of(q);
  return o == GS_OP_NOTIN || o == GS_OP_DOES_NOT_EXIST;
}

KReq make_kreq(const Vocab& v, int op, const std::vector<uint32_t>& vals, int64_t bound) {
  KReq q;
  q.has = Bits(v.words());
  q.excl = Bits(v.words());
  switch (op) {
    case GS_OP_IN:
      q.comp = false;
      for (auto x : vals) q.has.set(x);
      break;
    case GS_OP_NOTIN:
      q.comp = true;
      for (auto x : vals) q.excl.set(x);
      q.has = all_bits(v);
      for (auto x : vals) q.has.reset(x);
      break;
    case GS_OP_EXISTS:
      q.comp = true;
      q.has = all_bits(v);
      break;
    case GS_OP_DOES_NOT_EXIST:
      q.comp = false;
      break;
    case GS_OP_GT:
      q.comp = true;
      q.hg = true;
      q.gt = bound;
      q.has = within_mask(v, true, bound, false, 0);
      break;
    case GS_OP_LT:
      q.comp = true;
      q.hl = true;
      q.lt = bound;
      q.has = within_mask(v, false, 0, true, bound);
      break;
  }
  return q;
}

}  // namespace

void reqs_add(const Encoded& e, Reqs& r, uint32_t key, const KReq& q) {
  auto it = r.find(key);
  if (it == r.end()) r.emplace(key, q);
  else it->second = kreq_intersect(e.keys[key].vocab, q, it->second);
}

namespace {

void reqs_add_all(const Encoded& e, Reqs& r, const Reqs& o) {
  for (auto& kv : o) reqs_add(e, r, kv.first, kv.second);
}

// <U> Requirements.Compatible(incoming, AllowUndefinedWellKnownLabels if allow_wk)
bool reqs_compatible(const Encoded& e, const Reqs& r, const Reqs& in, bool allow_wk) {
  for (auto& kv : in) {
    if (allow_wk && e.keys[kv.first].wellknown) continue;
    if (r.count(kv.first)) continue;
    if (exempt(kv.second)) continue;
    return false;
  }
  for (auto& kv : in) {
    auto it = r.find(kv.first);
    if (it == r.end()) continue;
    KReq x = kreq_intersect(e.keys[kv.first].vocab, it->second, kv.second);
    if (len_zero(x) && !(exempt(it->second) && exempt(kv.second))) return false;
  }
  return true;
}

struct Ctx {
  const gs_problem* p;
  Encoded& e;
  std::vector<std::string> strs;
  // GS_ENCODE_PROFILE: sub-phase wall clock on stderr (diagnostics)
  bool pprof = std::getenv("GS_ENCODE_PROFILE") != nullptr;
  std::chrono::steady_clock::time_point pt_last = std::chrono::steady_clock::now();
  void ph(const char* name) {
    if (!pprof) return;
    const auto t = std::chrono::steady_clock::now();
    std::fprintf(stderr, "  pods.%-18s %8.3f ms\n", name, std::chrono::duration<double, std::milli>(t - pt_last).count());
    pt_last = t;
  }

  const std::string& S(uint32_t id) const {
    if (id >= strs.size()) throw Fail{GS_E_INVALID, "string id out of range"};
    return strs[id];
  }
  void chk(gs_range r, uint32_t n, const char* what) const {
    if ((uint64_t)r.begin + r.count > n) throw Fail{GS_E_INVALID, std::string("range out of bounds: ") + what};
  }

  // canonical string ids: the first id carrying each distinct text (callers
  // may repeat a string under several ids)
  std::vector<uint32_t> canon;
  void build_canon() {
    const uint32_t n = (uint32_t)strs.size();
    canon.resize(n);
    // strings hashed in parallel, then each shard's first-id map built by its
    // own thread over its ids in ascending order
    const uint32_t SH = 64;
    std::vector<uint64_t> hs(n);
    par_for(n, 4096, [&](uint32_t i) { hs[i] = std::hash<std::string_view>{}(std::string_view(strs[i])); });
    std::vector<uint32_t> cnt(SH + 1, 0), ids(n);
    for (uint32_t i = 0; i < n; i++) cnt[hs[i] % SH + 1]++;
    for (uint32_t k = 0; k < SH; k++) cnt[k + 1] += cnt[k];
    {
      std::vector<uint32_t> fill(cnt.begin(), cnt.end() - 1);
      for (uint32_t i = 0; i < n; i++) ids[fill[hs[i] % SH]++] = i;
    }
    par_for(SH, 1, [&](uint32_t k) {
      std::unordered_map<std::string_view, uint32_t> first;
      first.reserve((cnt[k + 1] - cnt[k]) * 2);
      for (uint32_t x = cnt[k]; x < cnt[k + 1]; x++) {
        const uint32_t i = ids[x];
        canon[i] = first.emplace(std::string_view(strs[i]), i).first->second;
      }
    });
  }
  uint32_t C(uint32_t id) const {
    if (id >= canon.size()) throw Fail{GS_E_INVALID, "string id out of range"};
    return canon[id];
  }

  // ---------------------------------------------------------- vocabulary
  std::map<std::string, std::set<std::string>> mentions;

  void mention(const std::string& key, const std::string& val) { mentions[normalize(key)].insert(val); }
  void mention_key(const std::string& key) { mentions[normalize(key)]; }
  void mention_reqs(gs_range r) {
    chk(r, p->n_reqs, "reqs");
    for (uint32_t i = 0; i < r.count; i++) {
      auto& q = p->reqs[r.begin + i];
      if (q.op > GS_OP_LTE) throw Fail{GS_E_INVALID, "unknown requirement operator"};
      chk(q.values, p->n_value_ids, "values");
      mention_key(S(q.key));
      if (q.op == GS_OP_IN || q.op == GS_OP_NOTIN)
        for (uint32_t k = 0; k < q.values.count; k++) {
          const std::string& v = S(p->value_ids[q.values.begin + k]);
          if (normalize(S(q.key)) == kHostname && v.rfind("hostname-placeholder-", 0) == 0)
            throw Fail{GS_E_UNSUPPORTED, "requirement names a hostname placeholder"};
          mention(S(q.key), v);
        }
      if (q.op >= GS_OP_GT) {
        int64_t x;
        if (q.values.count < 1 || !atoi64(S(p->value_ids[q.values.begin]), &x))
          throw Fail{GS_E_INVALID, "Gt/Lt/Gte/Lte value is not an integer"};
        if ((q.op == GS_OP_GTE && x == INT64_MIN) || (q.op == GS_OP_LTE && x == INT64_MAX))
          throw Fail{GS_E_INVALID, "Gte/Lte bound out of range"};
      }
    }
  }
  void mention_labels(gs_range r) {
    chk(r, p->n_labels, "labels");
    for (uint32_t i = 0; i < r.count; i++) mention(S(p->labels[r.begin + i].key), S(p->labels[r.begin + i].value));
  }

  void build_vocab() {
    mention_key(kZone);
    mention_key(kCapacityType);
    mention_key(kHostname);
    mention_key(kNodePool);
    for (uint32_t i = 0; i < p->n_instance_types; i++) {
      auto& it = p->instance_types[i];
      mention_reqs(it.requirements);
      chk(it.offerings, p->n_offerings, "offerings");
      for (uint32_t k = 0; k < it.offerings.count; k++) mention_reqs(p->offerings[it.offerings.begin + k].requirements);
    }
    for (uint32_t i = 0; i < p->n_nodepools; i++) {
      auto& np = p->nodepools[i];
      mention_reqs(np.requirements);
      mention_labels(np.labels);
      mention(kNodePool, S(np.name));
    }
    // node label values matter only where a requirement can tell them apart:
    // on instance-type / offering keys, or as integers under Gt/Lt bounds.
    // Any other value behaves exactly like the unmentioned value omega.
    std::set<std::string> label_keys = {kZone, kCapacityType}, bounded;
    // a NodePool-key spread tells nodes of unknown NodePools apart (domains)
    for (uint32_t i = 0; i < p->n_spreads; i++)
      if (normalize(S(p->spreads[i].topology_key)) == kNodePool) label_keys.insert(kNodePool);
    if (p->n_instance_types) {
      auto& it0 = p->instance_types[0];
      chk(it0.requirements, p->n_reqs, "reqs");
      for (uint32_t k = 0; k < it0.requirements.count; k++)
        label_keys.insert(normalize(S(p->reqs[it0.requirements.begin + k].key)));
    }
    for (uint32_t i = 0; i < p->n_reqs; i++)
      if (p->reqs[i].op >= GS_OP_GT && p->reqs[i].op <= GS_OP_LTE) bounded.insert(normalize(S(p->reqs[i].key)));
    auto node_mention = [&](const std::string& key, const std::string& val) {
      const std::string k = normalize(key);
      int64_t x;
      if (label_keys.count(k) || (bounded.count(k) && atoi64(val, &x))) mention(k, val);
      else mention_key(k);
    };
    for (uint32_t i = 0; i < p->n_nodes; i++) {
      chk(p->nodes[i].labels, p->n_labels, "labels");
      for (uint32_t k = 0; k < p->nodes[i].labels.count; k++)
        node_mention(S(p->labels[p->nodes[i].labels.begin + k].key), S(p->labels[p->nodes[i].labels.begin + k].value));
      node_mention(kHostname, S(p->nodes[i].name));
    }
    for (uint32_t i = 0; i < p->n_pods; i++) {
      auto& pd = p->pods[i];
      mention_labels(pd.node_selector);
      chk(pd.required_terms, p->n_terms, "terms");
      chk(pd.preferred_terms, p->n_terms, "terms");
      for (uint32_t k = 0; k < pd.required_terms.count; k++) mention_reqs(p->terms[pd.required_terms.begin + k].requirements);
      for (uint32_t k = 0; k < pd.preferred_terms.count; k++)
        mention_reqs(p->terms[pd.preferred_terms.begin + k].requirements);
    }
    for (auto& kv : mentions) {
      Key k;
      k.name = kv.first;
      k.wellknown = is_wellknown(kv.first);
      for (auto& v : kv.second) {
        k.vocab.id[v] = (uint32_t)k.vocab.vals.size();
        k.vocab.vals.push_back(v);
      }
      k.vocab.omega = (uint32_t)k.vocab.vals.size();
      k.vocab.vals.push_back(kOmega);
      for (auto& v : k.vocab.vals) {
        int64_t x = 0;
        bool ok = v != kOmega && atoi64(v, &x);
        k.vocab.isint.push_back(ok);
        k.vocab.ival.push_back(x);
      }
      e.key_id[k.name] = (uint32_t)e.keys.size();
      e.keys.push_back(std::move(k));
    }
    e.k_zone = e.key_id[kZone];
    e.k_ct = e.key_id[kCapacityType];
    e.k_hostname = e.key_id[kHostname];
    e.k_nodepool = e.key_id[kNodePool];
    // spreads on the capacity-type key move the domain machinery onto it
    // (build_nodes / build_pods swap the zone and capacity-type fields)
    e.dom_ct = e.dom_np = false;
    for (uint32_t i = 0; i < p->n_spreads; i++) {
      const std::string k = normalize(S(p->spreads[i].topology_key));
      e.dom_ct = e.dom_ct || k == kCapacityType;
      e.dom_np = e.dom_np || k == kNodePool;
    }
    e.k_dom = e.dom_np ? e.k_nodepool : e.dom_ct ? e.k_ct : e.k_zone;
  }

  uint32_t key_of(uint32_t sid) const { return e.key_id.at(normalize(S(sid))); }

  KReq kreq_of(const gs_requirement& q) const {
    uint32_t k = key_of(q.key);
    const Vocab& v = e.keys[k].vocab;
    std::vector<uint32_t> vals;
    int64_t bound = 0;
    if (q.op == GS_OP_IN || q.op == GS_OP_NOTIN)
      for (uint32_t i = 0; i < q.values.count; i++) vals.push_back(v.id.at(S(p->value_ids[q.values.begin + i])));
    int op = (int)q.op;
    if (op >= GS_OP_GT) atoi64(S(p->value_ids[q.values.begin]), &bound);
    // over integer label values Gte x is Gt x-1 and Lte x is Lt x+1
    if (op == GS_OP_GTE) {
      op = GS_OP_GT;
      bound -= 1;
    } else if (op == GS_OP_LTE) {
      op = GS_OP_LT;
      bound += 1;
    }
    KReq r = make_kreq(v, op, vals, bound);
    r.mv = q.min_values >= 0 ? q.min_values : -1;
    return r;
  }
  // a pod's NodeSelectorRequirement carries no minValues
  void no_min_values(gs_range r) const {
    chk(r, p->n_reqs, "reqs");
    for (uint32_t i = 0; i < r.count; i++)
      if (p->reqs[r.begin + i].min_values >= 0)
        throw Fail{GS_E_UNSUPPORTED, "minValues outside NodePool / NodeClaim requirements"};
  }
  Reqs reqs_of(gs_range r) const {
    Reqs out;
    for (uint32_t i = 0; i < r.count; i++) {
      auto& q = p->reqs[r.begin + i];
      reqs_add(e, out, key_of(q.key), kreq_of(q));
    }
    return out;
  }
  KReq in_one(uint32_t key, const std::string& val) const {
    const Vocab& v = e.keys[key].vocab;
    return make_kreq(v, GS_OP_IN, {v.id.at(val)}, 0);
  }
  KReq in_one_or_omega(uint32_t key, const std::string& val) const {
    const Vocab& v = e.keys[key].vocab;
    auto f = v.id.find(val);
    return make_kreq(v, GS_OP_IN, {f == v.id.end() ? v.omega : f->second}, 0);
  }
  Reqs node_labels_reqs(gs_range r) const {
    Reqs out;
    for (uint32_t i = 0; i < r.count; i++) {
      uint32_t k = key_of(p->labels[r.begin + i].key);
      reqs_add(e, out, k, in_one_or_omega(k, S(p->labels[r.begin + i].value)));
    }
    return out;
  }
  Reqs labels_reqs(gs_range r) const {
    Reqs out;
    for (uint32_t i = 0; i < r.count; i++) {
      uint32_t k = key_of(p->labels[r.begin + i].key);
      reqs_add(e, out, k, in_one(k, S(p->labels[r.begin + i].value)));
    }
    return out;
  }

  // ----------------------------------------------------------- catalog
  void build_catalog() {
    e.N = p->n_instance_types;
    e.W = (e.N + 63) / 64;
    if (e.N == 0) throw Fail{GS_E_INVALID, "empty catalog"};
    // IT keys: the key set of IT 0; every IT must carry exactly those keys,
    // each single-valued In (reference instancetype.go:721-726)
    std::vector<uint32_t> k0;
    for (uint32_t i = 0; i < e.N; i++) {
      auto& it = p->instance_types[i];
      std::vector<uint32_t> ks;
      for (uint32_t k = 0; k < it.requirements.count; k++) {
        auto& q = p->reqs[it.requirements.begin + k];
        if (q.op != GS_OP_IN || q.values.count != 1)
          throw Fail{GS_E_UNSUPPORTED, "instance type requirement is not single-valued In"};
        ks.push_back(key_of(q.key));
      }
      std::sort(ks.begin(), ks.end());
      if (std::adjacent_find(ks.begin(), ks.end()) != ks.end())
        throw Fail{GS_E_UNSUPPORTED, "instance type repeats a requirement key"};
      if (i == 0) k0 = ks;
      else if (ks != k0) throw Fail{GS_E_UNSUPPORTED, "instance types carry different requirement keys"};
    }
    for (auto k : k0) {
      if (k == e.k_zone || k == e.k_ct || k == e.k_hostname)
        throw Fail{GS_E_UNSUPPORTED, "instance type requirement on zone/capacity-type/hostname"};
      e.keys[k].cls = KEY_IT;
      e.keys[k].slot = (int)e.it_keys.size();
      e.it_keys.push_back(k);
    }
    e.K = (uint32_t)e.it_keys.size();
    if (e.K > (uint32_t)gsd::KMAX_IT) throw Fail{GS_E_UNSUPPORTED, "too many instance-type keys"};
    e.keys[e.k_zone].cls = KEY_ZONE;
    e.keys[e.k_ct].cls = KEY_CT;
    // catalog zones / capacity types in first-appearance order
    std::map<uint32_t, uint32_t> zmap, cmap;
    struct Off {
      uint32_t z, c;
      double price;
      bool avail;
    };
    std::vector<std::vector<Off>> offs(e.N);
    for (uint32_t i = 0; i < e.N; i++) {
      auto& it = p->instance_types[i];
      if (it.offerings.count > (uint32_t)gsd::SMAX) throw Fail{GS_E_UNSUPPORTED, "too many offerings per instance type"};
      for (uint32_t s = 0; s < it.offerings.count; s++) {
        auto& o = p->offerings[it.offerings.begin + s];
        uint32_t zv = gsd::NONE, cv = gsd::NONE;
        for (uint32_t k = 0; k < o.requirements.count; k++) {
          auto& q = p->reqs[o.requirements.begin + k];
          uint32_t key = key_of(q.key);
          if (q.op != GS_OP_IN || q.values.count != 1) throw Fail{GS_E_UNSUPPORTED, "offering requirement not single In"};
          uint32_t vid = e.keys[key].vocab.id.at(S(p->value_ids[q.values.begin]));
          if (key == e.k_zone && zv == gsd::NONE) zv = vid;
          else if (key == e.k_ct && cv == gsd::NONE) cv = vid;
          else throw Fail{GS_E_UNSUPPORTED, "offering requirements other than one zone and one capacity type"};
        }
        if (zv == gsd::NONE || cv == gsd::NONE) throw Fail{GS_E_UNSUPPORTED, "offering without zone or capacity type"};
        if (std::isnan(o.price)) throw Fail{GS_E_UNSUPPORTED, "NaN offering price"};
        if (!zmap.count(zv)) {
          uint32_t n = (uint32_t)zmap.size();
          zmap[zv] = n;
          e.cat_zone.push_back(zv);
        }
        if (!cmap.count(cv)) {
          uint32_t n = (uint32_t)cmap.size();
          cmap[cv] = n;
          e.cat_ct.push_back(cv);
        }
        offs[i].push_back({zmap[zv], cmap[cv], o.price, o.available != 0});
      }
    }
    e.Z = (uint32_t)e.cat_zone.size();
    e.C = (uint32_t)e.cat_ct.size();
    if (e.Z * e.C > 64) throw Fail{GS_E_UNSUPPORTED, "zones x capacity types > 64"};
    // resources
    // (canonical string ids of the resource names: the first id carrying
    // each text, so a resource's lowest string id is its canonical id)
    std::set<std::string> rn;
    std::vector<uint32_t> res_cids;
    {
      std::vector<uint8_t> seen(strs.size(), 0);
      for (uint32_t i = 0; i < p->n_quantities; i++) {
        const uint32_t c = C(p->quantities[i].resource);
        if (!seen[c]) {
          seen[c] = 1;
          rn.insert(strs[c]);
          res_cids.push_back(c);
        }
      }
    }
    e.res_names.assign(rn.begin(), rn.end());
    e.R = (uint32_t)e.res_names.size();
    if (e.R > (uint32_t)gsd::RMAX) throw Fail{GS_E_UNSUPPORTED, "more than 8 distinct resources"};
    std::unordered_map<std::string, uint32_t> rid;
    for (uint32_t r = 0; r < e.R; r++) rid[e.res_names[r]] = r;
    e.res_name_ids.assign(e.R, 0);
    std::vector<uint32_t> rid_of_cid(res_cids.size());
    for (size_t k = 0; k < res_cids.size(); k++) {
      const uint32_t r = rid.at(strs[res_cids[k]]);
      e.res_name_ids[r] = res_cids[k];
      rid_of_cid[k] = r;
    }
    rid_map = rid;
    // string id -> resource index for every string a quantity names (the
    // only ids resvec_fn looks up)
    rid_of_sid.assign(strs.size(), gsd::NONE);
    {
      std::unordered_map<uint32_t, uint32_t> by_cid;
      for (size_t k = 0; k < res_cids.size(); k++) by_cid[res_cids[k]] = rid_of_cid[k];
      for (uint32_t i = 0; i < p->n_quantities; i++) {
        const uint32_t sid = p->quantities[i].resource;
        if (rid_of_sid[sid] == gsd::NONE) rid_of_sid[sid] = by_cid.at(C(sid));
      }
    }
    auto resvec = [this](gs_range r, int64_t* out, bool* present) { resvec_fn(r, out, present); };
    // per IT arrays
    e.it_vid.assign((size_t)e.K * e.N, 0);
    e.it_alloc.assign((size_t)e.R * e.N, 0);
    e.it_cap.assign((size_t)e.R * e.N, 0);
    e.it_pair.assign(e.N, 0);
    e.it_prank.assign((size_t)e.N * 64, gsd::NONE);
    // price ranks
    std::vector<double> prices;
    for (auto& v : offs)
      for (auto& o : v) prices.push_back(o.price);
    std::sort(prices.begin(), prices.end());
    prices.erase(std::unique(prices.begin(), prices.end(), [](double a, double b) { return a == b; }), prices.end());
    e.prices = prices;
    auto prank = [&](double x) {
      return (uint32_t)(std::lower_bound(prices.begin(), prices.end(), x) - prices.begin());
    };
    std::vector<uint8_t> ok(e.N, 1);
    for (uint32_t i = 0; i < e.N; i++) {
      auto& it = p->instance_types[i];
      for (uint32_t k = 0; k < it.requirements.count; k++) {
        auto& q = p->reqs[it.requirements.begin + k];
        uint32_t key = key_of(q.key);
        e.it_vid[(size_t)e.keys[key].slot * e.N + i] = e.keys[key].vocab.id.at(S(p->value_ids[q.values.begin]));
      }
      int64_t cap[gsd::RMAX] = {0}, ovh[gsd::RMAX] = {0};
      bool capp[gsd::RMAX] = {false}, ovhp[gsd::RMAX] = {false};
      resvec(it.capacity, cap, capp);
      resvec(it.overhead, ovh, ovhp);
      for (uint32_t r = 0; r < e.R; r++) {
        // Allocatable = Subtract(Capacity, Overhead.Total()) over capacity keys
        int64_t a = capp[r] ? cap[r] - (ovhp[r] ? ovh[r] : 0) : 0;
        e.it_alloc[(size_t)r * e.N + i] = a;
        e.it_cap[(size_t)r * e.N + i] = cap[r];
        if (capp[r] && a < 0) ok[i] = 0;  // <U> Fits: any negative total never fits
      }
      uint64_t seen = 0;
      for (auto& o : offs[i]) {
        uint32_t g = o.z * e.C + o.c;
        if (seen >> g & 1) throw Fail{GS_E_UNSUPPORTED, "instance type repeats a (zone, capacity type) offering"};
        seen |= 1ull << g;
        if (o.avail) {
          e.it_pair[i] |= 1ull << g;
          e.it_prank[(size_t)i * 64 + g] = prank(o.price);
        }
      }
      if (!ok[i]) e.it_pair[i] = 0;  // never selectable
    }
    it_ok.assign(e.W, 0);
    for (uint32_t i = 0; i < e.N; i++)
      if (ok[i]) it_ok[i / 64] |= 1ull << (i % 64);
    // name ranks (Go string order = bytewise)
    std::vector<uint32_t> order(e.N);
    std::iota(order.begin(), order.end(), 0);
    std::vector<std::string> names(e.N);
    for (uint32_t i = 0; i < e.N; i++) names[i] = S(p->instance_types[i].name);
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return names[a] < names[b]; });
    for (uint32_t i = 0; i + 1 < e.N; i++)
      if (names[order[i]] == names[order[i + 1]]) throw Fail{GS_E_INVALID, "duplicate instance type name"};
    e.it_namerank.assign(e.N, 0);
    e.rank_to_it = order;
    for (uint32_t r = 0; r < e.N; r++) e.it_namerank[order[r]] = r;
    // slot sets
    e.slot_set.assign((size_t)64 * e.W, 0);
    for (uint32_t i = 0; i < e.N; i++)
      for (uint32_t g = 0; g < 64; g++)
        if (e.it_pair[i] >> g & 1) e.slot_set[(size_t)g * e.W + i / 64] |= 1ull << (i % 64);
    // fit thresholds per resource over selectable ITs
    e.thr_off.assign(e.R + 1, 0);
    std::vector<std::vector<int64_t>> vals(e.R);
    for (uint32_t r = 0; r < e.R; r++) {
      for (uint32_t i = 0; i < e.N; i++)
        if (ok[i]) vals[r].push_back(e.it_alloc[(size_t)r * e.N + i]);
      std::sort(vals[r].begin(), vals[r].end());
      vals[r].erase(std::unique(vals[r].begin(), vals[r].end()), vals[r].end());
      e.thr_off[r + 1] = e.thr_off[r] + (uint32_t)vals[r].size();
    }
    e.thr_val.clear();
    for (uint32_t r = 0; r < e.R; r++) e.thr_val.insert(e.thr_val.end(), vals[r].begin(), vals[r].end());
    // thr_set: for resource r, m in [0, n_r]: rows at (thr_off[r] + r + m)
    e.thr_set.assign((size_t)(e.thr_off[e.R] + e.R) * e.W, 0);
    for (uint32_t r = 0; r < e.R; r++)
      for (uint32_t m = 0; m < vals[r].size(); m++) {
        uint64_t* row = &e.thr_set[(size_t)(e.thr_off[r] + r + m) * e.W];
        for (uint32_t i = 0; i < e.N; i++)
          if (ok[i] && e.it_alloc[(size_t)r * e.N + i] >= vals[r][m]) row[i / 64] |= 1ull << (i % 64);
      }
  }
  std::vector<uint64_t> it_ok;
  std::unordered_map<std::string, uint32_t> rid_map;
  std::vector<uint32_t> rid_of_sid;  // string id -> resource index (NONE: not a resource)
  void resvec_fn(gs_range r, int64_t* out, bool* present) const {
    chk(r, p->n_quantities, "quantities");
    for (uint32_t k = 0; k < r.count; k++) {
      auto& q = p->quantities[r.begin + k];
      if (q.resource >= rid_of_sid.size() || rid_of_sid[q.resource] == gsd::NONE)
        throw Fail{GS_E_INVALID, "unknown resource"};
      const uint32_t x = rid_of_sid[q.resource];
      out[x] += q.milli;
      if (present) present[x] = true;
    }
  }

  // ----------------------------------------------------- helpers on Reqs
  uint64_t zone_has(const Reqs& r) const {
    auto it = r.find(e.k_zone);
    uint64_t m = 0;
    for (uint32_t z = 0; z < e.Z; z++)
      if (it == r.end() || it->second.has.test(e.cat_zone[z])) m |= 1ull << z;
    return m;
  }
  uint64_t ct_has(const Reqs& r) const {
    auto it = r.find(e.k_ct);
    uint64_t m = 0;
    for (uint32_t c = 0; c < e.C; c++)
      if (it == r.end() || it->second.has.test(e.cat_ct[c])) m |= 1ull << c;
    return m;
  }
  // zone Has over the zone vocabulary (first word; topology needs <= 64
  // values) and the complement flag of the zone requirement
  uint64_t zone_full(const Reqs& r) const {
    auto f = r.find(e.k_dom);
    return f == r.end() ? ~0ull : f->second.has.w[0];
  }
  uint32_t zone_flags(const Reqs& r) const {
    auto f = r.find(e.k_dom);
    return f == r.end() || f->second.comp ? gsd::ZF_COMP : 0u;
  }

  // ------------------------------------------------ topology spread (<U>)
  struct SpreadEnc {
    std::string key;
    int32_t skew = 1, mind = 0;
    bool sa = false, has_sel = false, ignore_aff = false, honor_taints = false;
    // <U> TopologyGroup.Hash's node-filter part (oracle/solve.cpp
    // node_filter): taint policy, the filter terms' keys (not their values)
    // and the owner's tolerations; ftext: the terms with their values (a
    // group's owners under AffinityPolicy Honor must agree on it)
    std::string fid, ftext;
    // AffinityPolicy Honor with a filter on more than the zone key: the first
    // owner's filter terms (build_topology applies them to the bound pods'
    // nodes and requires every counted pending spec to carry the same terms)
    bool strict_aff = false;
    std::vector<Reqs> filter;
    std::map<std::string, std::string> ml;
    std::vector<std::tuple<std::string, uint32_t, std::set<std::string>>> ex;
    // metav1.LabelSelector (nil selects nothing)
    bool matches(const std::map<std::string, std::string>& labels) const {
      if (!has_sel) return false;
      for (auto& kv : ml) {
        auto f = labels.find(kv.first);
        if (f == labels.end() || f->second != kv.second) return false;
      }
      for (auto& x : ex) {
        auto f = labels.find(std::get<0>(x));
        const bool present = f != labels.end();
        const uint32_t op = std::get<1>(x);
        const auto& vals = std::get<2>(x);
        if (op == GS_OP_IN && !(present && vals.count(f->second))) return false;
        if (op == GS_OP_NOTIN && present && vals.count(f->second)) return false;
        if (op == GS_OP_EXISTS && !present) return false;
        if (op == GS_OP_DOES_NOT_EXIST && present) return false;
      }
      return true;
    }
    // (minDomains is not part of it: a group keeps its first owner's)
    std::string hash(const std::string& ns) const {
      std::string h = key + "|" + std::to_string(skew) + "|" + ns + "|" + (has_sel ? "1" : "0") +
                      (ignore_aff ? "I" : "H") + (honor_taints ? "H" : "I") + "|f:" + fid;
      for (auto& kv : ml) h += "|l:" + kv.first + "=" + kv.second;
      for (auto& x : ex) {
        h += "|e:" + std::get<0>(x) + ":" + std::to_string(std::get<1>(x));
        for (auto& v : std::get<2>(x)) h += "," + v;
      }
      return h;
    }
  };
  // <U> corev1.PodAffinityTerm of pod (anti-)affinity (hostname or zone key)
  struct AntiEnc {
    SpreadEnc sel;              // key / has_sel / ml / ex
    std::set<std::string> nss;  // the term's namespaces, else the pod's
    bool required = false;
    int32_t weight = 0;
    bool selects(const std::string& ns, const std::map<std::string, std::string>& labels) const {
      return nss.count(ns) && sel.matches(labels);
    }
    std::string hash() const {
      std::string h = "anti|" + sel.key + "|" + std::string(sel.has_sel ? "1" : "0");
      for (auto& n : nss) h += "|n:" + n;
      for (auto& kv : sel.ml) h += "|l:" + kv.first + "=" + kv.second;
      for (auto& x : sel.ex) {
        h += "|e:" + std::get<0>(x) + ":" + std::to_string(std::get<1>(x));
        for (auto& v : std::get<2>(x)) h += "," + v;
      }
      return h;
    }
  };
  // <U> scheduling.HostPort: Matches = same protocol and port, and either IP
  // unspecified or equal (net.ParseIP; unparsable -> 0.0.0.0)
  struct PortEnc {
    std::string proto;
    bool unspec = true;
    std::array<uint8_t, 16> ip{};
    int32_t port = 0;
    bool matches(const PortEnc& o) const {
      return proto == o.proto && port == o.port && (unspec || o.unspec || ip == o.ip);
    }
    std::string key() const {
      std::string k = proto + "|" + std::to_string(port) + "|";
      if (!unspec) k.append((const char*)ip.data(), 16);
      return k;
    }
  };
  // what makes a pod counted by a group
  struct PodSel {
    std::string ns;
    std::map<std::string, std::string> labels;
    std::set<std::string> carried;  // hashes of its required anti-affinity terms
    std::vector<PortEnc> ports;
  };
  // A topology group as the device sees it.  kind 0: a spread constraint
  // (counts the pods its selector selects in the owner's namespace).  The
  // anti-affinity and host-port constraints are hostname groups whose owner
  // may join only a domain with count + self <= skew, self = the owner is
  // counted itself; with skew = self that is "count == 0":
  //  kind 1 TopologyTypePodAntiAffinity (counts the pods the term selects),
  //  kind 2 its inverse for a required term (owners = the pods the term
  //         selects; counts the pods carrying the term),
  //  kind 3 HostPortUsage (owners = pods with port entry e; counts the pods
  //         with an entry that Matches e).
  // kind 4 (TopologyTypePodAffinity) counts the pods its term selects and
  // admits an owner where count > 0, or, while the total is 0, anywhere if
  // the owner is counted itself (tg_aff; the kernel keeps the total).
  struct GroupEnc {
    SpreadEnc sp;
    std::string ns;
    int kind = 0;
    AntiEnc anti;
    std::string inv_hash;
    PortEnc port;
    uint32_t owner_spec = gsd::NONE;  // spread groups: the first owner's spec
    // a spread group no pod's first variant keys: Topology.Update creates it
    // when a relaxation first moves a pod to this hash (lazy index; the
    // kernels record into it only once some pod has relaxed into it)
    bool lazy = false;
    uint32_t lazy_idx = 0;
    uint32_t owner_state = 0;         // the first owner's relaxation state (PodWork filter states)
    uint32_t owner_sv = gsd::NONE;    // the first owner's spec variant in that state
  };
  std::vector<GroupEnc> groups;
  std::map<std::string, uint32_t> group_idx;
  // spread groups whose node filter cannot matter (both policies Ignore, or
  // affinity Honor over an empty filter with taints Ignore) and that agree on
  // everything else, minDomains included, count the same pods in the same
  // domains: upstream keeps one group per filter (TopologyGroup.Hash), the
  // product shares one (pod_phase_b)
  std::map<std::string, uint32_t> merge_idx;
  std::vector<PodSel> pod_sel;  // per pod spec (spec_of)
  std::vector<std::pair<Reqs, bool>> np_universe;  // NodePool requirements (+labels), has instance types
  uint32_t bound_alias = gsd::NONE;  // bound pod b is also pod bound_alias + b (consolidation)

  std::map<std::string, std::string> label_map(gs_range r) const {
    chk(r, p->n_labels, "labels");
    std::map<std::string, std::string> m;
    for (uint32_t i = 0; i < r.count; i++) m[S(p->labels[r.begin + i].key)] = S(p->labels[r.begin + i].value);
    return m;
  }
  std::vector<SpreadEnc> spreads_of(const gs_pod& pd) const {
    chk(pd.spreads, p->n_spreads, "spreads");
    std::vector<SpreadEnc> out;
    for (uint32_t k = 0; k < pd.spreads.count; k++) {
      const gs_spread& q = p->spreads[pd.spreads.begin + k];
      SpreadEnc sp;
      sp.key = normalize(S(q.topology_key));
      if (sp.key != kZone && sp.key != kHostname && sp.key != kCapacityType && sp.key != kNodePool)
        throw Fail{GS_E_UNSUPPORTED, "topology spread key other than zone / capacity type / NodePool / hostname"};
      if (sp.key != kHostname && sp.key != e.keys[e.k_dom].name)
        throw Fail{GS_E_UNSUPPORTED, "topology spreads on more than one of the zone, capacity-type and NodePool keys"};
      if (q.max_skew < 1) throw Fail{GS_E_INVALID, "maxSkew < 1"};
      if (q.when_unsatisfiable > GS_SPREAD_SCHEDULE_ANYWAY || q.node_affinity_policy > GS_POLICY_IGNORE ||
          q.node_taints_policy > GS_POLICY_IGNORE)
        throw Fail{GS_E_INVALID, "bad topology spread enum"};
      // nodeTaintsPolicy Honor (TopologyNodeFilter.Matches: the owner's
      // tolerations must tolerate a node's / NodeClaim's taints for it to
      // count and for its domain to enter the minimum) is accepted when the
      // owner tolerates every taint of the problem, where it equals Ignore;
      // checked in build_nodes once every taint is known
      sp.honor_taints = q.node_taints_policy == GS_POLICY_HONOR;
      sp.skew = q.max_skew;
      sp.mind = q.min_domains > 0 ? q.min_domains : 0;
      sp.sa = q.when_unsatisfiable == GS_SPREAD_SCHEDULE_ANYWAY;
      sp.has_sel = q.has_selector != 0;
      sp.ignore_aff = q.node_affinity_policy == GS_POLICY_IGNORE;
      sp.ml = label_map(q.match_labels);
      chk(q.match_expressions, p->n_reqs, "reqs");
      for (uint32_t x = 0; x < q.match_expressions.count; x++) {
        const gs_requirement& r = p->reqs[q.match_expressions.begin + x];
        if (r.op > GS_OP_DOES_NOT_EXIST) throw Fail{GS_E_INVALID, "label selector operator"};
        chk(r.values, p->n_value_ids, "values");
        std::set<std::string> vals;
        for (uint32_t v = 0; v < r.values.count; v++) vals.insert(S(p->value_ids[r.values.begin + v]));
        sp.ex.emplace_back(S(r.key), r.op, std::move(vals));
      }
      // matchLabelKeys: key In [the pod's value] for every key the pod carries
      chk(q.match_label_keys, p->n_value_ids, "values");
      if (q.match_label_keys.count) {
        const auto labels = label_map(pd.labels);
        for (uint32_t m = 0; m < q.match_label_keys.count; m++) {
          const std::string& k = S(p->value_ids[q.match_label_keys.begin + m]);
          auto f = labels.find(k);
          if (f != labels.end()) sp.ex.emplace_back(k, (uint32_t)GS_OP_IN, std::set<std::string>{f->second});
        }
      }
      out.push_back(std::move(sp));
    }
    return out;
  }
  std::vector<AntiEnc> antis_of(const gs_pod& pd) const { return terms_of(pd, pd.anti_affinity, false); }
  // zone-key anti-affinity is deterministic (every empty zone both sides
  // allow); zone-key pod affinity bootstraps on a zone picked in Go map order
  std::vector<AntiEnc> terms_of(const gs_pod& pd, gs_range rg, bool affinity) const {
    chk(rg, p->n_affinity_terms, "affinity_terms");
    std::vector<AntiEnc> out;
    for (uint32_t k = 0; k < rg.count; k++) {
      const gs_affinity_term& q = p->affinity_terms[rg.begin + k];
      const std::string tk = normalize(S(q.topology_key));
      if (tk != kHostname && !(tk == kZone && !affinity))
        throw Fail{GS_E_UNSUPPORTED, affinity ? "pod affinity topologyKey other than hostname"
                                              : "pod anti-affinity topologyKey other than hostname / zone"};
      if (e.k_dom != e.k_zone && tk == kZone)
        throw Fail{GS_E_UNSUPPORTED, "zone-key pod anti-affinity beside capacity-type / NodePool topology spreads"};
      AntiEnc a;
      a.required = q.required != 0;
      a.weight = q.weight;
      a.sel.key = tk;
      a.sel.has_sel = q.has_selector != 0;
      a.sel.ml = label_map(q.match_labels);
      chk(q.match_expressions, p->n_reqs, "reqs");
      for (uint32_t x = 0; x < q.match_expressions.count; x++) {
        const gs_requirement& r = p->reqs[q.match_expressions.begin + x];
        if (r.op > GS_OP_DOES_NOT_EXIST) throw Fail{GS_E_INVALID, "label selector operator"};
        chk(r.values, p->n_value_ids, "values");
        std::set<std::string> vals;
        for (uint32_t v = 0; v < r.values.count; v++) vals.insert(S(p->value_ids[r.values.begin + v]));
        a.sel.ex.emplace_back(S(r.key), r.op, std::move(vals));
      }
      // <U> buildNamespaceList: the listed namespaces plus those the
      // namespaceSelector matches; neither = the pod's namespace
      chk(q.namespaces, p->n_value_ids, "values");
      for (uint32_t v = 0; v < q.namespaces.count; v++) a.nss.insert(S(p->value_ids[q.namespaces.begin + v]));
      if (q.has_ns_selector) {
        SpreadEnc nsel;
        nsel.has_sel = true;
        nsel.ml = label_map(q.ns_match_labels);
        chk(q.ns_match_expressions, p->n_reqs, "reqs");
        for (uint32_t x = 0; x < q.ns_match_expressions.count; x++) {
          const gs_requirement& r = p->reqs[q.ns_match_expressions.begin + x];
          if (r.op > GS_OP_DOES_NOT_EXIST) throw Fail{GS_E_INVALID, "label selector operator"};
          chk(r.values, p->n_value_ids, "values");
          std::set<std::string> vals;
          for (uint32_t v = 0; v < r.values.count; v++) vals.insert(S(p->value_ids[r.values.begin + v]));
          nsel.ex.emplace_back(S(r.key), r.op, std::move(vals));
        }
        chk(gs_range{0, p->n_namespaces}, p->n_namespaces, "namespaces");
        for (uint32_t n = 0; n < p->n_namespaces; n++)
          if (nsel.matches(label_map(p->namespaces[n].labels))) a.nss.insert(S(p->namespaces[n].name));
      } else if (a.nss.empty()) {
        a.nss.insert(S(pd.ns));
      }
      out.push_back(std::move(a));
    }
    return out;
  }
  std::vector<PortEnc> ports_of(const gs_pod& pd) const {
    chk(pd.host_ports, p->n_host_ports, "host_ports");
    std::vector<PortEnc> out;
    static const std::array<uint8_t, 16> z6{}, z4{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xff, 0xff, 0, 0, 0, 0};
    for (uint32_t k = 0; k < pd.host_ports.count; k++) {
      const gs_host_port& q = p->host_ports[pd.host_ports.begin + k];
      if (q.port < 1 || q.port > 65535) throw Fail{GS_E_INVALID, "host port out of range"};
      PortEnc e;
      e.proto = S(q.protocol).empty() ? std::string("TCP") : S(q.protocol);
      e.port = q.port;
      const std::string& ip = S(q.ip);
      in_addr b4;
      std::array<uint8_t, 16> b6;
      e.ip = z4;  // unparsable: 0.0.0.0
      if (inet_pton(AF_INET, ip.c_str(), &b4) == 1) std::memcpy(e.ip.data() + 12, &b4, 4);
      else if (inet_pton(AF_INET6, ip.c_str(), b6.data()) == 1) e.ip = b6;
      e.unspec = e.ip == z6 || e.ip == z4;
      out.push_back(e);
    }
    return out;
  }
  PodSel sel_of(const gs_pod& pd) const {
    PodSel ps;
    ps.ns = S(pd.ns);
    ps.labels = label_map(pd.labels);
    for (auto& a : antis_of(pd))
      if (a.required) ps.carried.insert(a.hash());
    ps.ports = ports_of(pd);
    return ps;
  }
  bool group_counts(const GroupEnc& g, const PodSel& ps) const {
    switch (g.kind) {
      case 0: return ps.ns == g.ns && g.sp.matches(ps.labels);
      case 1:
      case 4: return g.anti.selects(ps.ns, ps.labels);
      case 2: return ps.carried.count(g.inv_hash) != 0;
      default:
        for (auto& e : ps.ports)
          if (e.matches(g.port)) return true;
        return false;
    }
  }
  uint32_t group_id(const std::string& h, GroupEnc&& g) {
    auto f = group_idx.find(h);
    if (f == group_idx.end()) {
      if (groups.size() >= (size_t)gsd::TGMAX) throw Fail{GS_E_UNSUPPORTED, "more than 4096 topology groups"};
      f = group_idx.emplace(h, (uint32_t)groups.size()).first;
      groups.push_back(std::move(g));
    }
    return f->second;
  }
  // a group admitting an owner only where the count is 0: on the hostname key
  // through count + self <= skew = self; on the zone key (anti-affinity and
  // its inverse) the domains with count 0 (TK_ANTI)
  GroupEnc host_group(int kind, bool self, const std::string& key = kHostname) const {
    GroupEnc g;
    g.kind = kind;
    g.sp.key = key;
    g.sp.skew = self ? 1 : 0;
    return g;
  }

  // Candidate groups of a pod for group_counts: each group is filed under
  // one thing a counted pod must carry (a matchLabels pair, a carried term,
  // a host port's protocol and number); groups with no such anchor are
  // checked for every pod, and nil selectors select nothing
  struct SelIndex {
    std::unordered_map<std::string, std::vector<uint32_t>> by;
    std::vector<uint32_t> generic;
    explicit SelIndex(const std::vector<GroupEnc>& gs) {
      for (uint32_t g = 0; g < gs.size(); g++) {
        const GroupEnc& x = gs[g];
        if (x.kind == 2) {
          by["C" + x.inv_hash].push_back(g);
        } else if (x.kind == 3) {
          by["P" + x.port.proto + "|" + std::to_string(x.port.port)].push_back(g);
        } else {
          const SpreadEnc& sel = x.kind == 0 ? x.sp : x.anti.sel;
          if (!sel.has_sel) continue;
          if (!sel.ml.empty()) by["L" + sel.ml.begin()->first + "=" + sel.ml.begin()->second].push_back(g);
          else generic.push_back(g);
        }
      }
    }
    void candidates(const PodSel& ps, std::vector<uint32_t>* out) const {
      *out = generic;
      auto add = [&](const std::string& k) {
        auto f = by.find(k);
        if (f != by.end()) out->insert(out->end(), f->second.begin(), f->second.end());
      };
      if (!by.empty()) {
        for (auto& kv : ps.labels) add("L" + kv.first + "=" + kv.second);
        for (auto& h : ps.carried) add("C" + h);
        for (auto& pe : ps.ports) add("P" + pe.proto + "|" + std::to_string(pe.port));
      }
      std::sort(out->begin(), out->end());
      out->erase(std::unique(out->begin(), out->end()), out->end());
    }
  };

  // <U> VolumeUsage (ExistingNode.CanAdd's ExceedsLimits): per node the
  // distinct volumes of its bound pods per driver and the CSINode limits; a
  // node already over a limit takes no pod at all (the union check fails
  // whatever the pod mounts)
  // A volume only one pod mounts (pods and bound pods, a bound pod that is
  // also in the pod list -- consolidation -- counting once) can never be on a
  // node the pod is placed on: it is a per-driver count of "fresh" volumes.
  // The others (<= 64 distinct) are bits a node may already hold.
  void build_volumes() {
    std::map<std::string, uint32_t> drv;
    std::map<std::pair<std::string, std::string>, uint32_t> vol;
    std::map<std::pair<std::string, std::string>, std::set<uint32_t>> users;
    auto volkey = [&](const gs_volume& v) { return std::make_pair(S(v.driver), S(v.id)); };
    for (uint32_t i = 0; i < e.P; i++) {
      const gs_pod& pd = p->pods[i];
      chk(pd.volumes, p->n_volumes, "volumes");
      for (uint32_t k = 0; k < pd.volumes.count; k++) users[volkey(p->volumes[pd.volumes.begin + k])].insert(i);
    }
    if (p->n_bound_pods && !p->bound_pod_node) throw Fail{GS_E_INVALID, "bound pods without their nodes"};
    for (uint32_t b = 0; b < p->n_bound_pods; b++) {
      const gs_pod& bp = p->bound_pods[b];
      chk(bp.volumes, p->n_volumes, "volumes");
      const uint32_t who = bound_alias != gsd::NONE ? bound_alias + b : e.P + b;
      for (uint32_t k = 0; k < bp.volumes.count; k++) {
        auto f = users.find(volkey(p->volumes[bp.volumes.begin + k]));
        if (f != users.end()) f->second.insert(who);  // only volumes pods in the list mount matter
      }
    }
    // without pending volumes the kernels never read these (any_vol)
    const size_t PV = users.empty() ? 1 : std::max<uint32_t>(e.P, 1);
    e.pod_vol.assign(PV * gsd::VDMAX, 0);
    e.pod_vfresh.assign(PV * gsd::VDMAX, 0);
    for (uint32_t i = 0; i < e.P; i++) {
      const gs_pod& pd = p->pods[i];
      if (!pd.volumes.count) continue;
      std::set<std::pair<std::string, std::string>> mine;
      for (uint32_t k = 0; k < pd.volumes.count; k++) mine.insert(volkey(p->volumes[pd.volumes.begin + k]));
      for (auto& vk : mine) {
        const uint32_t d = drv.emplace(vk.first, (uint32_t)drv.size()).first->second;
        if (d >= (uint32_t)gsd::VDMAX) throw Fail{GS_E_UNSUPPORTED, "pending pods mount volumes of more than 4 CSI drivers"};
        if (users[vk].size() < 2) {
          e.pod_vfresh[(size_t)i * gsd::VDMAX + d]++;
          continue;
        }
        const uint32_t b = vol.emplace(vk, (uint32_t)vol.size()).first->second;
        if (b >= 64) throw Fail{GS_E_UNSUPPORTED, "pods share more than 64 distinct volumes"};
        e.pod_vol[(size_t)i * gsd::VDMAX + d] |= 1ull << b;
      }
    }
    std::vector<uint32_t> pos_of(e.NN);
    for (uint32_t i = 0; i < e.NN; i++) pos_of[e.node_order[i]] = i;
    std::vector<std::map<std::string, std::set<std::string>>> used(e.NN);
    if (p->n_bound_pods && !p->bound_pod_node) throw Fail{GS_E_INVALID, "bound pods without their nodes"};
    for (uint32_t b = 0; b < p->n_bound_pods; b++) {
      const gs_pod& bp = p->bound_pods[b];
      if (p->bound_pod_node[b] >= e.NN) throw Fail{GS_E_INVALID, "bound pod node out of range"};
      chk(bp.volumes, p->n_volumes, "volumes");
      for (uint32_t k = 0; k < bp.volumes.count; k++) {
        const gs_volume& v = p->volumes[bp.volumes.begin + k];
        used[pos_of[p->bound_pod_node[b]]][S(v.driver)].insert(S(v.id));
      }
    }
    e.n_vol.assign(std::max<uint32_t>(e.NN, 1), gsd::NodeVol{});
    for (uint32_t pos = 0; pos < e.NN; pos++) {
      const gs_node& g = p->nodes[e.node_order[pos]];
      chk(g.volume_limits, p->n_volume_limits, "volume_limits");
      std::map<std::string, int64_t> lim;
      for (uint32_t k = 0; k < g.volume_limits.count; k++)
        lim[S(p->volume_limits[g.volume_limits.begin + k].driver)] = p->volume_limits[g.volume_limits.begin + k].limit;
      gsd::NodeVol& nv = e.n_vol[pos];
      for (int d = 0; d < gsd::VDMAX; d++) nv.lim[d] = INT32_MAX;
      for (auto& kv : used[pos]) {
        auto f = lim.find(kv.first);
        if (f != lim.end() && (int64_t)kv.second.size() > f->second) e.nodes[pos].ok = 0;  // already over
      }
      for (auto& dv : drv) {
        auto f = lim.find(dv.first);
        if (f != lim.end()) nv.lim[dv.second] = (int32_t)std::max<int64_t>(f->second, -1);
        auto u = used[pos].find(dv.first);
        nv.cnt[dv.second] = u == used[pos].end() ? 0 : (int32_t)u->second.size();
      }
      for (auto& vv : vol) {
        auto u = used[pos].find(vv.first.first);
        if (u != used[pos].end() && u->second.count(vv.first.second)) nv.present |= 1ull << vv.second;
      }
    }
    e.any_vol = !drv.empty() && e.NN > 0;
  }

  // <U> NewTopology: domain universe (In values of NodePool requirements of
  // NodePools that have instance types, existing nodes' labels) and the
  // counts of the selected bound pods; per variant the owned-group list, per
  // pod the selection list (layout.hpp VarRec own_off / sel_off)
  void build_topology() {
    e.TG = (uint32_t)groups.size();
    e.lazy_slot.assign(1, 0);
    e.var_lz_off.assign(2, 0);
    e.lz_idx.assign(1, 0);
    e.lz_mind.assign(1, 0);
    if (!e.TG) return;
    const Vocab& zv = e.keys[e.k_dom].vocab;
    bool any_zone = false;
    for (auto& g : groups) any_zone = any_zone || g.sp.key != kHostname;
    if (any_zone && zv.size() > (size_t)gsd::ZVMAX)
      throw Fail{GS_E_UNSUPPORTED, "zone / capacity-type topology groups over more than 63 domain values"};
    e.NZV = (uint32_t)std::min<size_t>(zv.size() - 1, gsd::ZVMAX);
    e.ZS = std::max<uint32_t>(e.NZV, 1);
    e.zone_order.resize(e.NZV);
    std::iota(e.zone_order.begin(), e.zone_order.end(), 0);
    std::sort(e.zone_order.begin(), e.zone_order.end(), [&](uint32_t a, uint32_t b) { return zv.vals[a] < zv.vals[b]; });
    e.zone_cat.assign(gsd::ZVMAX, gsd::NONE);
    if (e.dom_np) {
      // a NodePool domain narrows no catalog zone or capacity type
    } else if (e.dom_ct) {
      for (uint32_t c = 0; c < e.C; c++)
        if (e.cat_ct[c] < (uint32_t)gsd::ZVMAX) e.zone_cat[e.cat_ct[c]] = c;
    } else {
      for (uint32_t z = 0; z < e.Z; z++)
        if (e.cat_zone[z] < (uint32_t)gsd::ZVMAX) e.zone_cat[e.cat_zone[z]] = z;
    }
    // <U> buildDomainGroups inserts Requirement.Values() of each NodePool's
    // requirements combined with each of its instance types': for a NotIn
    // those are the excluded values (this restatement takes In values only),
    // and an instance type's own requirement on the key would add its values.
    // The IBM catalog's instance types carry neither a zone nor a capacity
    // type (instancetype.go:719-724), so an unconstrained NodePool provides
    // no domain either way; the two ambiguous forms are refused, not guessed
    if (any_zone) {
      for (auto& u : np_universe) {
        if (!u.second) continue;
        auto f = u.first.find(e.k_dom);
        if (f != u.first.end() && f->second.comp && !f->second.excl.none())
          throw Fail{GS_E_UNSUPPORTED, "a NodePool NotIn requirement on the topology spread key " + e.keys[e.k_dom].name};
      }
      for (uint32_t k : e.it_keys)
        if (k == e.k_dom)
          throw Fail{GS_E_UNSUPPORTED, "instance types with a requirement on the topology spread key " + e.keys[e.k_dom].name};
    }
    uint64_t known_zone = 0;
    for (auto& u : np_universe) {
      if (!u.second) continue;
      auto f = u.first.find(e.k_dom);
      if (f != u.first.end() && !f->second.comp) known_zone |= f->second.has.w[0];  // operator In
    }
    e.known_np = known_zone;
    e.zone_nodes.assign(gsd::ZVMAX, 0);
    for (auto& nr : e.nodes)
      if (nr.dvid < e.ZS) {
        known_zone |= 1ull << nr.dvid;
        e.zone_nodes[nr.dvid]++;
      }
    e.zknown0 = known_zone;
    e.tgroups.assign(e.TG, gsd::TGroupRec{});
    for (uint32_t g = 0; g < e.TG; g++) {
      gsd::TGroupRec& t = e.tgroups[g];
      t.skew = groups[g].sp.skew;
      // a lazy group's minDomains is its creator's, known at the Relax that
      // creates it: -(lazy index + 1) reads the kernels' lazy minDomains
      t.mind = groups[g].lazy ? -(int32_t)groups[g].lazy_idx - 1 : groups[g].sp.mind;
      const int kind = groups[g].kind;
      if (groups[g].sp.key == kHostname) {
        t.kind = gsd::TK_HOST | (kind == 4 ? gsd::TK_AFF : 0u);
        t.slot = e.TGH++;
      } else {
        t.kind = kind == 1 || kind == 2 ? gsd::TK_ANTI : 0u;
        t.slot = e.TGZ++;
        t.known0 = known_zone;
      }
    }
    // <U> TopologyDomainGroup.ForEachDomain under TaintPolicy Honor: a domain
    // enters domainMinCount only if a NodePool (with instance types) or a node
    // providing it has taints the pod (this relaxation) tolerates.  Folded into
    // the variant's strict domains, which only the minimum reads (topo_tmin)
    {
      bool any_honor = false;
      for (auto& g : groups) any_honor = any_honor || (g.kind == 0 && g.sp.honor_taints && g.sp.key != kHostname);
      if (any_honor) {
        std::vector<std::pair<uint64_t, uint64_t>> prov;  // (taint classes, domains)
        for (size_t i = 0; i < np_universe.size(); i++) {
          if (!np_universe[i].second) continue;
          auto f = np_universe[i].first.find(e.k_dom);
          if (f == np_universe[i].first.end() || f->second.comp) continue;
          uint64_t cm = 0;
          for (uint32_t id : np_universe_taints[i]) cm |= 1ull << taint_cls[id];
          prov.emplace_back(cm, f->second.has.w[0]);
        }
        for (auto& nr : e.nodes)
          if (nr.dvid < e.ZS) prov.emplace_back(nr.taints, 1ull << nr.dvid);
        for (uint32_t v = 0; v < e.V; v++) {
          const uint32_t sv = e.var_sv[v];
          uint32_t nh = 0, ni = 0;
          for (uint32_t g : e.variants[sv].own)
            if (groups[g].kind == 0 && groups[g].sp.key != kHostname) (groups[g].sp.honor_taints ? nh : ni)++;
          if (!nh) continue;
          if (ni)
            throw Fail{GS_E_UNSUPPORTED, "a pod owning zone-key spreads with both nodeTaintsPolicy Honor and Ignore"};
          // a domain no NodePool or node provides (one a Record adds during
          // the Solve) has no taints to tolerate: it stays
          uint64_t dm = 0, provided = 0;
          for (auto& pr : prov) {
            provided |= pr.second;
            if ((pr.first & ~final_sv_tol[sv]) == 0) dm |= pr.second;
          }
          e.vars[v].zs &= dm | ~provided;
        }
      }
    }
    // <U> Topology.AddRequirements intersects every owned group's domains: two
    // groups that pick different domains leave an empty requirement, which a
    // node lacking the domain label passes (strict Compatible: DoesNotExist).
    // The kernels test each group against the node's own domain instead, so
    // such a node beside a pod owning two or more zone-count groups is refused
    if (e.TGZ) {
      bool lacking = false;
      for (auto& nr : e.nodes) lacking = lacking || nr.dvid == gsd::DVID_NONE;
      if (lacking)
        for (auto& pv : e.variants) {
          uint32_t nz = 0;
          for (uint32_t g : pv.own) nz += groups[g].sp.key != kHostname;
          if (nz >= 2)
            throw Fail{GS_E_UNSUPPORTED, "an existing node lacking the " + e.keys[e.k_dom].name +
                                             " label beside a pod owning several topology groups on that key"};
        }
    }
    if (gsd::topo_lds_bytes(e.TGZ, e.ZS, e.TGH, n_lazy) > 64u * 1024u)
      throw Fail{GS_E_UNSUPPORTED, "topology group state exceeds 64 KiB of LDS (zone groups x zones)"};
    e.zcnt0.assign((size_t)std::max<uint32_t>(e.TGZ, 1) * e.ZS, 0);
    e.htot0.assign(std::max<uint32_t>(e.TGH, 1), 0);
    e.hn0.assign((size_t)std::max<uint32_t>(e.TGH, 1) * std::max<uint32_t>(e.NN, 1), 0);
    e.zn_cnt.assign((size_t)std::max<uint32_t>(e.TGZ, 1) * std::max<uint32_t>(e.NN, 1), 0);
    std::vector<uint32_t> pos_of(e.NN);
    for (uint32_t i = 0; i < e.NN; i++) pos_of[e.node_order[i]] = i;
    if (p->n_bound_pods && !p->bound_pod_node) throw Fail{GS_E_INVALID, "bound pods without their nodes"};
    SelIndex six(groups);
    std::vector<uint32_t> cand;
    // <U> countDomains under AffinityPolicy Honor: a bound pod counts only on
    // a node whose labels (+ hostname) are strictly Compatible with one of the
    // group's filter terms (oracle/solve.cpp TGroup::filter_matches)
    std::vector<std::unique_ptr<Reqs>> nreqs(e.NN);
    auto node_matches = [&](const SpreadEnc& sp, uint32_t raw) {
      if (!nreqs[raw]) {
        const gs_node& g = p->nodes[raw];
        nreqs[raw].reset(new Reqs(node_labels_reqs(g.labels)));
        reqs_add(e, *nreqs[raw], e.k_hostname, in_one_or_omega(e.k_hostname, S(g.name)));
      }
      for (auto& f : sp.filter)
        if (reqs_compatible(e, *nreqs[raw], f, false)) return true;
      return false;
    };
    // nodeTaintsPolicy Honor: the group's first owner's tolerations (before
    // Relax) against a bound pod's Node taints in countDomains, and its
    // tolerated taint classes for the counted specs below
    std::vector<uint64_t> g_otol(e.TG, ~0ull);
    for (uint32_t g = 0; g < e.TG; g++)
      if (groups[g].kind == 0 && groups[g].sp.honor_taints) g_otol[g] = final_sv_tol[groups[g].owner_sv];
    auto node_tolerated = [&](uint32_t g, uint32_t raw) {
      const std::vector<Tol>& tols = variant_tols[groups[g].owner_sv];
      const gs_range r = p->nodes[raw].taints;
      chk(r, p->n_taints, "taints");
      for (uint32_t k = 0; k < r.count; k++) {
        const gs_taint& t = p->taints[r.begin + k];
        if (!tolerated(tols, TaintKey{S(t.key), S(t.value), S(t.effect)})) return false;
      }
      return true;
    };
    for (uint32_t b = 0; b < p->n_bound_pods; b++) {
      const gs_pod& bp = p->bound_pods[b];
      if (p->bound_pod_node[b] >= e.NN) throw Fail{GS_E_INVALID, "bound pod node out of range"};
      const uint32_t pos = pos_of[p->bound_pod_node[b]];
      const PodSel ps = sel_of(bp);
      six.candidates(ps, &cand);
      for (uint32_t g : cand) {
        if (!group_counts(groups[g], ps)) continue;
        if (groups[g].kind == 0 && groups[g].sp.strict_aff && !node_matches(groups[g].sp, p->bound_pod_node[b]))
          continue;
        if (groups[g].kind == 0 && groups[g].sp.honor_taints && !node_tolerated(g, p->bound_pod_node[b])) continue;
        gsd::TGroupRec& t = e.tgroups[g];
        if (t.kind & gsd::TK_HOST) {
          e.hn0[(size_t)t.slot * e.NN + pos]++;
          e.htot0[t.slot]++;  // the total over domains (affinity bootstrap)
        } else {
          const uint32_t z = e.nodes[pos].dvid;
          if (z == gsd::NONE || z >= e.ZS) continue;
          e.zcnt0[(size_t)t.slot * e.ZS + z]++;
          e.zn_cnt[(size_t)t.slot * e.NN + pos]++;
          t.known0 |= 1ull << z;
        }
      }
    }
    // per spec: the selection list (shared by its pods' variants), then each
    // spec variant's own list with the self flag; a pod's variants point at
    // its spec's lists
    e.tg_list.clear();
    std::vector<uint8_t> selected(e.TG, 0);
    std::vector<uint32_t> mine;
    const uint32_t NS = (uint32_t)spec_rep.size();
    std::vector<uint32_t> sel_off(NS), sel_n(NS), own_off(e.variants.size()), own_n(e.variants.size());
    for (uint32_t s = 0; s < NS; s++) {
      six.candidates(pod_sel[s], &cand);
      mine.clear();
      for (uint32_t g : cand)
        if (group_counts(groups[g], pod_sel[s])) mine.push_back(g);
      for (uint32_t g : mine) {
        // taint Honor: every NodeClaim / node a counted pod can land on (it
        // tolerates the taints) must be one the owner tolerates, in every
        // relaxation of the pod (Relax may add the PreferNoSchedule toleration)
        if (groups[g].kind == 0 && groups[g].sp.honor_taints)
          for (uint32_t sv = sv_begin[s]; sv < sv_begin[s] + sv_count[s]; sv++)
            if (final_sv_tol[sv] & ~g_otol[g])
              throw Fail{GS_E_UNSUPPORTED, "a pod counted by a topology spread (nodeTaintsPolicy Honor) tolerating a "
                                           "taint its owner does not"};
      }
      for (uint32_t g : mine) {
        const SpreadEnc& sp = groups[g].sp;
        if (groups[g].kind != 0 || !sp.strict_aff) continue;
        // the NodeClaims / nodes this spec lands on match the owner's filter
        // only if it carries the same terms and no preference narrows them
        if (spec_aff_text[s] != sp.ftext)
          throw Fail{GS_E_UNSUPPORTED,
                     "a pod counted by a topology spread (nodeAffinityPolicy Honor) without its owner's node affinity"};
        for (uint32_t k : spec_pref_keys[s])
          for (auto& f : sp.filter)
            if (f.count(k))
              throw Fail{GS_E_UNSUPPORTED,
                         "a pod counted by a topology spread (nodeAffinityPolicy Honor) with preferred node affinity "
                         "on a key of the spread's filter"};
      }
      sel_off[s] = (uint32_t)e.tg_list.size();
      sel_n[s] = (uint32_t)mine.size();
      for (uint32_t g : mine) {
        selected[g] = 1;
        if (groups[g].lazy)  // slots and lazy indices < 4096: slot in bits 0..11, lazy index in 12..23
          e.tg_list.push_back(e.tgroups[g].slot | (groups[g].lazy_idx << 12) | ((e.tgroups[g].kind | gsd::TK_LAZY) << 24));
        else
          e.tg_list.push_back(e.tgroups[g].slot | (e.tgroups[g].kind << 24));
      }
      for (uint32_t sv = sv_begin[s]; sv < sv_begin[s] + sv_count[s]; sv++) {
        own_off[sv] = (uint32_t)e.tg_list.size();
        for (uint32_t g : e.variants[sv].own) e.tg_list.push_back(g | (selected[g] ? gsd::TL_SELF : 0u));
        own_n[sv] = (uint32_t)e.variants[sv].own.size();
      }
      for (uint32_t g : mine) selected[g] = 0;
    }
    for (uint32_t i = 0; i < e.P; i++) {
      const uint32_t s = spec_of[i];
      for (uint32_t v = e.var_begin[i]; v < e.var_begin[i] + e.var_count[i]; v++) {
        gsd::VarRec& vr = e.vars[v];
        vr.sel_off = sel_off[s];
        vr.sel_n = sel_n[s];
        vr.own_off = own_off[e.var_sv[v]];
        vr.own_n = own_n[e.var_sv[v]];
      }
    }
    if (e.tg_list.empty()) e.tg_list.push_back(0);
    // per device variant: the lazy groups a pod owns once it relaxes into it
    // (the kernels activate them at that Relax)
    e.n_lazy = n_lazy;
    e.lazy_slot.assign(std::max<uint32_t>(n_lazy, 1), 0);
    for (uint32_t g = 0; g < e.TG; g++)
      if (groups[g].lazy)
        e.lazy_slot[groups[g].lazy_idx] = e.tgroups[g].slot | ((e.tgroups[g].kind & gsd::TK_HOST) ? gsd::LZ_HOST : 0u);
    if (n_lazy) {
      // per spec variant its lazy groups (ascending, unique) with its
      // minDomains for each; device variants share their spec variant's run
      std::vector<uint32_t> sv_off(e.variants.size() + 1, 0);
      e.lz_idx.clear();
      e.lz_mind.clear();
      for (size_t sv = 0; sv < e.variants.size(); sv++) {
        auto lm = e.variants[sv].lazy_mind;
        std::sort(lm.begin(), lm.end());
        lm.erase(std::unique(lm.begin(), lm.end(), [](auto& x, auto& y) { return x.first == y.first; }), lm.end());
        sv_off[sv] = (uint32_t)e.lz_idx.size();
        for (auto& x : lm) {
          e.lz_idx.push_back(x.first);
          e.lz_mind.push_back(x.second);
        }
        sv_off[sv + 1] = (uint32_t)e.lz_idx.size();
      }
      // device variant v: [var_lz_off[2v], var_lz_off[2v + 1])
      e.var_lz_off.assign(2 * (size_t)e.V, 0);
      for (uint32_t v = 0; v < e.V; v++) {
        e.var_lz_off[2 * (size_t)v] = sv_off[e.var_sv[v]];
        e.var_lz_off[2 * (size_t)v + 1] = sv_off[e.var_sv[v] + 1];
      }
      if (e.lz_idx.empty()) {
        e.lz_idx.assign(1, 0);
        e.lz_mind.assign(1, 0);
      }
    }
  }

  // CT_SPOT | CT_OD: Requirement.Has("spot") / Has("on-demand") of the
  // capacity-type key (an absent key is Exists: both); values nobody
  // mentions behave like omega
  uint32_t ct_bits(const Reqs& r) {
    auto f = r.find(e.k_ct);
    if (f == r.end()) return gsd::CT_SPOT | gsd::CT_OD;
    const Vocab& v = e.keys[e.k_ct].vocab;
    auto vid = [&](const char* x) {
      auto g = v.id.find(x);
      return g == v.id.end() ? v.omega : g->second;
    };
    return (f->second.has.test(vid("spot")) ? gsd::CT_SPOT : 0u) | (f->second.has.test(vid("on-demand")) ? gsd::CT_OD : 0u);
  }

  uint64_t grid(uint64_t zm, uint64_t cm) const {
    uint64_t g = 0;
    for (uint32_t z = 0; z < e.Z; z++)
      if (zm >> z & 1) g |= (cm & ((1ull << e.C) - 1)) << (z * e.C);
    return g;
  }
  // compat(IT, reqs) over IT keys: <U> it.Requirements.Intersects(reqs)
  bool it_compat(uint32_t i, const Reqs& r) const {
    for (uint32_t k = 0; k < e.K; k++) {
      auto f = r.find(e.it_keys[k]);
      if (f == r.end()) continue;
      if (!f->second.has.test(e.it_vid[(size_t)k * e.N + i])) return false;
    }
    return true;
  }
  gsd::FK to_fk(const KReq& q) const {
    gsd::FK f{};
    for (int i = 0; i < gsd::FKW; i++) {
      f.has[i] = i < (int)q.has.w.size() ? q.has.w[i] : 0;
      f.excl[i] = i < (int)q.excl.w.size() ? q.excl.w[i] : 0;
    }
    f.gt = q.gt;
    f.lt = q.lt;
    f.flags = gsd::FK_PRESENT | (q.comp ? gsd::FK_COMP : 0) | (q.hg ? gsd::FK_GT : 0) | (q.hl ? gsd::FK_LT : 0);
    return f;
  }

  // ----------------------------------------------------------- taints
  struct TaintKey {
    std::string k, v, eff;
    bool operator<(const TaintKey& o) const { return std::tie(k, v, eff) < std::tie(o.k, o.v, o.eff); }
  };
  std::map<TaintKey, uint32_t> taint_id;
  std::vector<TaintKey> taint_list;
  // the distinct taints of a NodePool / node (raw ids); the device masks are
  // over taint classes (build_taint_classes), so the raw vocabulary may
  // exceed 64
  std::vector<uint32_t> taint_ids(gs_range r, const std::vector<std::pair<std::string, std::string>>* reject = nullptr) {
    chk(r, p->n_taints, "taints");
    std::vector<uint32_t> ids;
    for (uint32_t i = 0; i < r.count; i++) {
      auto& t = p->taints[r.begin + i];
      TaintKey tk{S(t.key), S(t.value), S(t.effect)};
      bool drop = false;
      if (reject)
        for (auto& kr : *reject) drop = drop || (kr.first == tk.k && kr.second == tk.eff);  // Taint.MatchTaint
      if (drop) continue;
      auto f = taint_id.find(tk);
      uint32_t id;
      if (f == taint_id.end()) {
        id = (uint32_t)taint_list.size();
        if (id >= (1u << 16)) throw Fail{GS_E_UNSUPPORTED, "more than 65536 distinct taints"};
        taint_id[tk] = id;
        taint_list.push_back(tk);
      } else {
        id = f->second;
      }
      ids.push_back(id);
    }
    return ids;
  }
  std::vector<std::vector<uint32_t>> tmpl_taints, node_taints;  // raw ids per template / node position
  // <U> StateNode.Taints() (include/gpusched.h gs_node): while a managed node
  // initializes its NodeClaim's taints stand for the node's, and its startup
  // taints are ignored like the known ephemeral ones; matched by key + effect
  std::vector<uint32_t> state_taint_ids(const gs_node& g) {
    chk(g.taints, p->n_taints, "taints");
    chk(g.claim_taints, p->n_taints, "taints");
    chk(g.startup_taints, p->n_taints, "taints");
    const bool starting = g.managed && !g.initialized;
    std::vector<std::pair<std::string, std::string>> reject = {{"node.kubernetes.io/not-ready", "NoSchedule"},
                                                               {"node.kubernetes.io/unreachable", "NoSchedule"},
                                                               {"node.cloudprovider.kubernetes.io/uninitialized", "NoSchedule"},
                                                               {"karpenter.sh/unregistered", "NoExecute"}};
    if (starting)
      for (uint32_t i = 0; i < g.startup_taints.count; i++) {
        auto& t = p->taints[g.startup_taints.begin + i];
        reject.emplace_back(S(t.key), S(t.effect));
      }
    return taint_ids(starting ? g.claim_taints : g.taints, &reject);
  }
  struct Tol {
    std::string k, v, eff;
    uint32_t op;
  };
  // corev1 Toleration.ToleratesTaint by some toleration of the list
  static bool tolerated(const std::vector<Tol>& tols, const TaintKey& tn) {
    for (auto& t : tols) {
      if (!t.eff.empty() && t.eff != tn.eff) continue;
      if (!t.k.empty() && t.k != tn.k) continue;
      if (t.op == GS_TOL_EQUAL ? t.v == tn.v : t.op == GS_TOL_EXISTS) return true;
    }
    return false;
  }
  // Taint classes: two taints that exactly the same spec variants tolerate are
  // interchangeable in every Taints.ToleratesPod (a NodePool / node is
  // tolerated iff each of its taints is), so the device masks carry one bit
  // per class of equal toleration pattern; more than 64 classes is refused.
  // Sets the templates' and nodes' taint masks and every variant's tol / tolt.
  void build_taint_classes() {
    const size_t NSV = variant_tols.size(), NW = (NSV + 63) / 64;
    std::map<std::vector<uint64_t>, uint32_t> cls_of;
    std::vector<uint32_t> cls(taint_list.size());
    std::vector<uint64_t> sv_tol(NSV, 0);
    std::vector<uint64_t> sig(NW);
    for (size_t id = 0; id < taint_list.size(); id++) {
      std::fill(sig.begin(), sig.end(), 0ull);
      for (size_t sv = 0; sv < NSV; sv++)
        if (tolerated(variant_tols[sv], taint_list[id])) sig[sv / 64] |= 1ull << (sv % 64);
      auto f = cls_of.find(sig);
      if (f == cls_of.end()) {
        if (cls_of.size() >= 64) throw Fail{GS_E_UNSUPPORTED, "more than 64 taint classes (distinct toleration patterns over the taints)"};
        const uint32_t c = (uint32_t)cls_of.size();
        f = cls_of.emplace(sig, c).first;
        for (size_t sv = 0; sv < NSV; sv++)
          if (sig[sv / 64] >> (sv % 64) & 1) sv_tol[sv] |= 1ull << c;
      }
      cls[id] = f->second;
    }
    n_taint_classes = (uint32_t)cls_of.size();
    auto mask = [&](const std::vector<uint32_t>& ids) {
      uint64_t m = 0;
      for (uint32_t id : ids) m |= 1ull << cls[id];
      return m;
    };
    for (uint32_t t = 0; t < e.T; t++) e.tmpl[t].taints = mask(tmpl_taints[t]);
    for (uint32_t pos = 0; pos < e.NN; pos++) e.nodes[pos].taints = mask(node_taints[pos]);
    for (uint32_t v = 0; v < e.V; v++) {
      gsd::VarRec& vr = e.vars[v];
      vr.tol = sv_tol[e.var_sv[v]];
      vr.tolt = 0;
      for (uint32_t t = 0; t < e.T; t++)
        if ((e.tmpl[t].taints & ~vr.tol) == 0) vr.tolt |= 1ull << t;
    }
    for (size_t sv = 0; sv < NSV; sv++) e.variants[sv].tol = sv_tol[sv];
    final_sv_tol = std::move(sv_tol);
    taint_cls = cls;
  }
  uint32_t n_taint_classes = 0;
  std::vector<uint64_t> final_sv_tol;
  std::vector<uint32_t> taint_cls;                        // taint id -> class (build_taint_classes)
  std::vector<std::vector<uint32_t>> np_universe_taints;  // per np_universe entry: its taint ids

  // --------------------------------------------------------- templates
  bool tolerate_pns = false;
  std::vector<std::vector<Tol>> variant_tols;
  std::vector<uint32_t> honor_specs;  // specs owning a nodeTaintsPolicy Honor spread
  void build_templates() {
    // dense per-key value ids of the catalog (minValues counting)
    e.it_dvid.assign((size_t)e.K * e.N, 0);
    e.it_ndv.assign(e.K, 0);
    for (uint32_t k = 0; k < e.K; k++) {
      std::map<uint32_t, uint16_t> dense;
      for (uint32_t i = 0; i < e.N; i++) {
        auto f = dense.emplace(e.it_vid[(size_t)k * e.N + i], (uint16_t)std::min<size_t>(dense.size(), 65535)).first;
        e.it_dvid[(size_t)k * e.N + i] = f->second;
      }
      e.it_ndv[k] = (uint32_t)dense.size();
      if (dense.size() == e.N) e.it_key_unique |= 1u << k;
    }
    std::vector<uint32_t> order(p->n_nodepools);
    std::iota(order.begin(), order.end(), 0);
    std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
      auto& A = p->nodepools[a];
      auto& B = p->nodepools[b];
      if (A.weight == B.weight) return S(A.name) < S(B.name);
      return A.weight > B.weight;
    });
    for (uint32_t npi : order) {
      auto& np = p->nodepools[npi];
      Reqs npreqs = reqs_of(np.requirements);
      // NewNodeClaimTemplate: spec requirements + labels + nodepool label
      Reqs tr = npreqs;
      std::map<std::string, std::string> labels;
      for (uint32_t i = 0; i < np.labels.count; i++)
        labels[S(p->labels[np.labels.begin + i].key)] = S(p->labels[np.labels.begin + i].value);
      labels[kNodePool] = S(np.name);
      for (auto& kv : labels) {
        uint32_t k = e.key_id.at(normalize(kv.first));
        reqs_add(e, tr, k, in_one(k, kv.second));
      }
      uint64_t zm = zone_has(tr), cm = ct_has(tr), G = grid(zm, cm);
      // GetInstanceTypes filter + NewScheduler pre-filter (compat, fits({}), offering)
      chk(np.instance_types, p->n_it_refs, "it_refs");
      for (uint32_t k = 0; k < np.instance_types.count; k++) {
        uint32_t i = p->it_refs[np.instance_types.begin + k];
        if (i < e.N) e.checks_per_pod += p->instance_types[i].offerings.count;
      }
      std::vector<uint64_t> opts(e.W, 0);
      bool any = false, has_its = false;
      for (uint32_t k = 0; k < np.instance_types.count; k++) {
        uint32_t i = p->it_refs[np.instance_types.begin + k];
        if (i >= e.N) throw Fail{GS_E_INVALID, "it_ref out of range"};
        Reqs itr;
        for (uint32_t kk = 0; kk < e.K; kk++)
          itr.emplace(e.it_keys[kk], in_one(e.it_keys[kk], e.keys[e.it_keys[kk]].vocab.vals[e.it_vid[(size_t)kk * e.N + i]]));
        if (!reqs_compatible(e, npreqs, itr, true)) continue;
        has_its = true;  // CloudProvider.GetInstanceTypes keeps it (topology universe)
        if (!(it_ok[i / 64] >> (i % 64) & 1)) continue;
        if (!it_compat(i, tr)) continue;
        if (!(e.it_pair[i] & G)) continue;
        opts[i / 64] |= 1ull << (i % 64);
        any = true;
      }
      std::vector<uint32_t> tm = taint_ids(np.taints);
      np_universe.emplace_back(tr, has_its);
      np_universe_taints.push_back(tm);
      // <U> minValues (Strict): NewScheduler's filterInstanceTypesByRequirements
      // drops the NodePool when its options miss a minimum.  Instance types
      // carry no value for a key outside the IT keys (Values() is empty).
      uint32_t mv_mask = 0;
      uint16_t mvk[gsd::KMAX_IT] = {0};
      for (auto& kv : tr) {
        if (kv.second.mv <= 0) continue;
        if (e.keys[kv.first].cls != KEY_IT) {
          any = false;
          continue;
        }
        const int ks = e.keys[kv.first].slot;
        if (!((e.it_key_unique >> ks) & 1) && e.it_ndv[ks] > 256)
          throw Fail{GS_E_UNSUPPORTED, "minValues on a key with more than 256 instance-type values"};
        mv_mask |= 1u << ks;
        mvk[ks] = (uint16_t)std::min<int64_t>(kv.second.mv, 65535);
        std::set<uint32_t> vals;
        for (uint32_t i = 0; i < e.N; i++)
          if ((opts[i / 64] >> (i % 64)) & 1) vals.insert(e.it_vid[(size_t)ks * e.N + i]);
        if ((int64_t)vals.size() < kv.second.mv) any = false;
      }
      if (!any) continue;
      if (e.T >= (uint32_t)gsd::TMAX) throw Fail{GS_E_UNSUPPORTED, "more than 64 NodePools"};
      gsd::TmplRec t{};
      t.np_index = npi;
      t.zm = zm;
      t.cm = cm;
      t.taints = 0;  // build_taint_classes
      bool present[gsd::RMAX] = {false};
      resvec_fn(np.daemon_requests, t.daemon, nullptr);
      if (np.has_limits) {
        t.has_limits = 1;
        resvec_fn(np.limits, t.limits, present);
        for (uint32_t r = 0; r < e.R; r++)
          if (present[r]) t.limit_rmask |= 1u << r;
      }
      for (uint32_t i = 0; i < np.taints.count; i++)
        if (S(p->taints[np.taints.begin + i].effect) == kPNS) tolerate_pns = true;
      // NewNodeClaim adds hostname In[placeholder]
      reqs_add(e, tr, e.k_hostname, make_kreq(e.keys[e.k_hostname].vocab, GS_OP_IN, {e.keys[e.k_hostname].vocab.omega}, 0));
      t.ctb = ct_bits(tr);
      {
        // the static matrix folds NodePool limits in: filterByRemainingResources
        std::vector<uint64_t> lim = opts;
        if (t.has_limits)
          for (uint32_t i = 0; i < e.N; i++) {
            if (!(lim[i / 64] >> (i % 64) & 1)) continue;
            for (uint32_t r = 0; r < e.R; r++)
              if ((t.limit_rmask >> r & 1) && e.it_cap[(size_t)r * e.N + i] > t.limits[r]) lim[i / 64] &= ~(1ull << (i % 64));
          }
        e.t_limopts.insert(e.t_limopts.end(), lim.begin(), lim.end());
      }
      t.zfull = zone_full(tr);
      t.zflags = zone_flags(tr);
      t.mv_mask = mv_mask;
      for (int k = 0; k < gsd::KMAX_IT; k++) t.mv[k] = mvk[k];
      if (mv_mask) e.any_mv = true;
      e.tmpl.push_back(t);
      tmpl_taints.push_back(std::move(tm));
      e.t_opts.insert(e.t_opts.end(), opts.begin(), opts.end());
      e.tmpl_reqs.push_back(tr);
      e.T++;
    }
  }

  // --------------------------------------------------------------- pods
  // <U> ExistingNode.CanAdd: a node lacking a label satisfies a pod's
  // NotIn / DoesNotExist on it (Requirements.Compatible), and Add then gives
  // the node a requirement on that key, which later pods meet by intersection.
  // Instance-type, zone and capacity-type keys hold a node's label as one
  // value id; where some node lacks such a key that some pod term constrains
  // with NotIn / DoesNotExist, the key also gets a free slot ("shadow") that
  // carries the nodes' full requirement state, and the node check runs on it
  // instead of the value id.  Claims keep their own checks (the shadow entry
  // is a redundant, well-known free key there).  Not for a zone key that
  // topology counts on (a node's zone domain comes from its label).
  void choose_shadow_keys() {
    if (!p->n_nodes) return;
    std::set<uint32_t> constrained;
    // every key a pod's node selector or terms mention: a variant's
    // requirement can come out NotIn / DoesNotExist from In / Gt / Lt terms
    // too (an empty intersection is DoesNotExist)
    auto scan = [&](const gs_pod* pods, uint32_t n) {
      for (uint32_t i = 0; i < n; i++) {
        const gs_range sr = pods[i].node_selector;
        chk(sr, p->n_labels, "labels");
        for (uint32_t j = 0; j < sr.count; j++) constrained.insert(key_of(p->labels[sr.begin + j].key));
        for (gs_range tr : {pods[i].required_terms, pods[i].preferred_terms}) {
          chk(tr, p->n_terms, "terms");
          for (uint32_t t = 0; t < tr.count; t++) {
            const gs_range rr = p->terms[tr.begin + t].requirements;
            chk(rr, p->n_reqs, "reqs");
            for (uint32_t q = 0; q < rr.count; q++) constrained.insert(key_of(p->reqs[rr.begin + q].key));
          }
        }
      }
    };
    scan(p->pods, p->n_pods);
    if (p->bound_pods) scan(p->bound_pods, p->n_bound_pods);
    bool zone_topology = false;
    for (uint32_t i = 0; i < p->n_spreads; i++) zone_topology = zone_topology || normalize(S(p->spreads[i].topology_key)) == kZone;
    for (uint32_t i = 0; i < p->n_affinity_terms; i++)
      zone_topology = zone_topology || normalize(S(p->affinity_terms[i].topology_key)) == kZone;
    for (uint32_t k : constrained) {
      Key& key = e.keys[k];
      if (key.cls == KEY_FREE || !key.wellknown || key.vocab.size() > (size_t)gsd::FKV) continue;
      if (key.cls == KEY_ZONE && zone_topology) continue;
      if (key.cls == KEY_CT && e.dom_ct) continue;
      bool lacking = false;
      for (uint32_t i = 0; i < p->n_nodes && !lacking; i++) {
        const gs_range lr = p->nodes[i].labels;
        chk(lr, p->n_labels, "labels");
        bool has = false;
        for (uint32_t j = 0; j < lr.count && !has; j++) has = key_of(p->labels[lr.begin + j].key) == k;
        lacking = !has;
      }
      if (lacking) shadow_keys.push_back(k);
    }
  }
  std::vector<uint32_t> shadow_keys;

  void build_free_slots() {
    for (uint32_t k = 0; k < e.keys.size(); k++) {
      if (e.keys[k].cls != KEY_FREE) continue;
      if (e.keys[k].vocab.size() > (size_t)gsd::FKV)
        throw Fail{GS_E_UNSUPPORTED, "free key vocabulary > 255 values: " + e.keys[k].name};
      if (e.free_keys.size() >= (size_t)gsd::FMAX) throw Fail{GS_E_UNSUPPORTED, "more than 16 free requirement keys"};
      e.keys[k].slot = (int)e.free_keys.size();
      if (e.keys[k].wellknown) e.wk_slots |= 1ull << e.free_keys.size();
      e.free_keys.push_back(k);
    }
    choose_shadow_keys();
    for (uint32_t k : shadow_keys) {
      if (e.free_keys.size() >= (size_t)gsd::FMAX) break;  // build_nodes refuses what stays unshadowed
      e.keys[k].shadow = (int)e.free_keys.size();
      e.wk_slots |= 1ull << e.free_keys.size();
      e.free_keys.push_back(k);
    }
    e.F = (uint32_t)e.free_keys.size();
    e.fk_ival.assign((size_t)std::max<uint32_t>(e.F, 1) * gsd::FKV, 0);
    e.fk_isint.assign((size_t)std::max<uint32_t>(e.F, 1) * gsd::FKW, 0);
    for (uint32_t s = 0; s < e.F; s++) {
      auto& v = e.keys[e.free_keys[s]].vocab;
      for (uint32_t i = 0; i < v.size(); i++) {
        e.fk_ival[(size_t)s * gsd::FKV + i] = v.ival[i];
        if (v.isint[i]) e.fk_isint[(size_t)s * gsd::FKW + i / 64] |= 1ull << (i % 64);
      }
    }
    e.t_fk.assign((size_t)e.T * std::max<uint32_t>(e.F, 1), gsd::FK{});
    for (uint32_t t = 0; t < e.T; t++)
      for (auto& kv : e.tmpl_reqs[t]) {
        const Key& key = e.keys[kv.first];
        if (key.cls == KEY_FREE || key.shadow >= 0)
          e.t_fk[(size_t)t * e.F + (key.cls == KEY_FREE ? key.slot : key.shadow)] = to_fk(kv.second);
      }
  }

  // A pod's spec as bytes: everything but its uid, creation time, requests
  // and volumes (canonical string ids, so equal text is equal bytes).  Pods
  // with equal bytes have the same variants, groups and selection lists
  // (Deployments: thousands of replicas, one spec).  false: a range or id is
  // out of bounds (the pod is its own spec; its encode raises the error).
  bool pod_sig(const gs_pod& pd, std::vector<uint32_t>& out) const {
    auto u32 = [&](uint32_t x) { out.push_back(x); };
    auto sid = [&](uint32_t id) {
      if (id >= canon.size()) return false;
      u32(canon[id]);
      return true;
    };
    auto rng = [&](gs_range r, uint32_t n) { return (uint64_t)r.begin + r.count <= n; };
    auto labels = [&](gs_range r) {
      if (!rng(r, p->n_labels)) return false;
      u32(r.count);
      for (uint32_t k = 0; k < r.count; k++)
        if (!sid(p->labels[r.begin + k].key) || !sid(p->labels[r.begin + k].value)) return false;
      return true;
    };
    auto vids = [&](gs_range r) {
      if (!rng(r, p->n_value_ids)) return false;
      u32(r.count);
      for (uint32_t k = 0; k < r.count; k++)
        if (!sid(p->value_ids[r.begin + k])) return false;
      return true;
    };
    auto reqs = [&](gs_range r) {
      if (!rng(r, p->n_reqs)) return false;
      u32(r.count);
      for (uint32_t k = 0; k < r.count; k++) {
        const gs_requirement& q = p->reqs[r.begin + k];
        if (!sid(q.key)) return false;
        u32(q.op);
        u32((uint32_t)q.min_values);
        if (!vids(q.values)) return false;
      }
      return true;
    };
    auto terms = [&](gs_range r) {
      if (!rng(r, p->n_terms)) return false;
      u32(r.count);
      for (uint32_t k = 0; k < r.count; k++) {
        u32((uint32_t)p->terms[r.begin + k].weight);
        if (!reqs(p->terms[r.begin + k].requirements)) return false;
      }
      return true;
    };
    auto aff = [&](gs_range r) {
      if (!rng(r, p->n_affinity_terms)) return false;
      u32(r.count);
      for (uint32_t k = 0; k < r.count; k++) {
        const gs_affinity_term& q = p->affinity_terms[r.begin + k];
        if (!sid(q.topology_key)) return false;
        u32(q.required);
        u32((uint32_t)q.weight);
        u32(q.has_selector);
        u32(q.has_ns_selector);
        if (!labels(q.match_labels) || !reqs(q.match_expressions) || !vids(q.namespaces) ||
            !labels(q.ns_match_labels) || !reqs(q.ns_match_expressions))
          return false;
      }
      return true;
    };
    out.clear();
    u32(pd.flags);
    if (!sid(pd.ns) || !labels(pd.node_selector) || !terms(pd.required_terms) || !terms(pd.preferred_terms) ||
        !labels(pd.labels) || !rng(pd.tolerations, p->n_tolerations) || !rng(pd.spreads, p->n_spreads) ||
        !rng(pd.host_ports, p->n_host_ports))
      return false;
    u32(pd.tolerations.count);
    for (uint32_t k = 0; k < pd.tolerations.count; k++) {
      const gs_toleration& t = p->tolerations[pd.tolerations.begin + k];
      u32(t.op);
      if (!sid(t.key) || !sid(t.value) || !sid(t.effect)) return false;
    }
    u32(pd.spreads.count);
    for (uint32_t k = 0; k < pd.spreads.count; k++) {
      const gs_spread& q = p->spreads[pd.spreads.begin + k];
      if (!sid(q.topology_key)) return false;
      u32((uint32_t)q.max_skew);
      u32(q.when_unsatisfiable);
      u32((uint32_t)q.min_domains);
      u32(q.has_selector);
      u32(q.node_affinity_policy);
      u32(q.node_taints_policy);
      if (!labels(q.match_labels) || !reqs(q.match_expressions) || !vids(q.match_label_keys)) return false;
    }
    if (!aff(pd.anti_affinity) || !aff(pd.affinity)) return false;
    u32(pd.host_ports.count);
    for (uint32_t k = 0; k < pd.host_ports.count; k++) {
      const gs_host_port& h = p->host_ports[pd.host_ports.begin + k];
      u32((uint32_t)h.port);
      if (!sid(h.protocol) || !sid(h.ip)) return false;
    }
    return true;
  }

  // Per-spec encode work.  Phase A (parallel over specs) builds everything
  // the spec determines; phase B (serial, in the order pods first carry each
  // spec) assigns topology group ids, numbered in the order pods first name
  // them; phase C (parallel) builds the Relax variants.  An error is the
  // serial encoder's: the first failing pod's.
  struct GroupKey {
    std::string key;
    GroupEnc g;
    bool required = false;
    int32_t weight = 0;
  };
  struct PodWork {
    std::exception_ptr err;
    Reqs ns;
    std::vector<Reqs> req_terms;
    std::vector<std::pair<int32_t, Reqs>> pref;
    std::vector<SpreadEnc> sps;
    std::vector<std::string> sp_hash, sp_merge;
    std::vector<GroupKey> g_anti, g_aff, g_inv, g_port;  // in the order the pod names them
    std::vector<Tol> tols;
    std::vector<uint32_t> sgid, own_static;
    std::vector<std::pair<int32_t, uint32_t>> anti_pref, aff_pref;  // (weight, group)
    std::vector<PodVariant> vars;
    std::vector<std::vector<Tol>> var_tols;
    bool honor_taints = false;  // a spread with nodeTaintsPolicy Honor
    std::string aff_text;             // the node filter's terms with their values
    std::vector<uint32_t> pref_keys;  // keys of the preferred node-affinity terms
    // relaxation states of the spreads' node filter (<U> MakeTopologyNodeFilter
    // of the relaxed pod): state r < nT keeps the required terms from r on,
    // state nT adds the PreferNoSchedule toleration; per state the spreads
    // as that pod would key them, their hashes and group ids
    uint32_t n_states = 1;
    std::vector<std::vector<SpreadEnc>> st_sps;
    std::vector<std::vector<std::string>> st_hash;
    std::vector<std::vector<uint32_t>> st_gid;
    std::vector<uint32_t> var_state;  // per variant
  };
  // <U> MakeTopologyNodeFilter of one relaxation state: node selector AND
  // each required term from ri on (the selector alone without terms), the
  // tolerations; fid = TopologyGroup.Hash's part (term keys, tolerations),
  // text = the terms with their values, zone_only = no key past the zone
  struct FilterState {
    std::vector<Reqs> fr;
    std::string fid, text;
    bool zone_only = true, empty = true;
  };
  FilterState filter_state(const PodWork& w, size_t ri, const std::vector<Tol>& tols) const {
    FilterState f;
    if (w.req_terms.empty()) f.fr.push_back(w.ns);
    for (size_t t = ri; t < w.req_terms.size(); t++) {
      Reqs r = w.ns;
      for (auto& kv : w.req_terms[t]) reqs_add(e, r, kv.first, kv.second);
      f.fr.push_back(std::move(r));
    }
    std::vector<std::string> texts, terms, tl;
    for (auto& r : f.fr) {
      texts.push_back(canonical(e, r));
      std::vector<std::string> ks;
      for (auto& kv : r) ks.push_back(e.keys[kv.first].name);
      std::sort(ks.begin(), ks.end());
      std::string k;
      for (auto& x : ks) k += x + ",";
      terms.push_back(std::move(k));
      f.empty = f.empty && r.empty();
    }
    std::sort(texts.begin(), texts.end());
    for (auto& t : texts) f.text += t + "\x1e";
    for (auto& t : tols) tl.push_back(t.k + "=" + t.v + ":" + t.eff + "/" + std::to_string(t.op));
    std::sort(terms.begin(), terms.end());
    std::sort(tl.begin(), tl.end());
    for (auto& t : terms) f.fid += t + ";";
    f.fid += "#";
    for (auto& t : tl) f.fid += t + ";";
    for (auto& kv : w.ns) f.zone_only = f.zone_only && kv.first == e.k_zone;
    for (size_t t = ri; t < w.req_terms.size(); t++)
      for (auto& kv : w.req_terms[t]) f.zone_only = f.zone_only && kv.first == e.k_zone;
    return f;
  }
  // the spreads keyed under one filter state.  nodeAffinityPolicy Honor
  // equals Ignore when the filter constrains the zone key alone
  // (oracle/solve.cpp: it then drops only nodes / NodeClaims outside the
  // owner's zones); other filters are applied exactly where they can differ:
  // a bound pod counts only on a node the filter matches, and the pending
  // pods the group counts must carry the owner's filter terms
  // (build_topology), so every NodeClaim / node they land on matches it
  static void key_spreads(std::vector<SpreadEnc>& sps, const FilterState& f) {
    for (auto& sp : sps) {
      sp.fid = f.fid;
      sp.ftext = sp.ignore_aff ? std::string() : f.text;
      sp.strict_aff = !f.zone_only && !sp.ignore_aff;
      sp.filter = sp.strict_aff ? f.fr : std::vector<Reqs>();
    }
  }
  // pods -> specs: spec_of[pod], spec_rep[spec] (its first pod), and per spec
  // its variants' range in e.variants (sv_begin / sv_count)
  std::vector<uint32_t> spec_of, spec_rep, sv_begin, sv_count;
  std::vector<std::string> spec_aff_text;               // PodWork::aff_text per spec
  std::vector<std::vector<uint32_t>> spec_pref_keys;    // PodWork::pref_keys per spec

  void pod_phase_a(uint32_t i, PodWork& w, const std::map<std::string, AntiEnc>& inv_terms, bool topo_inputs) {
    auto& pd = p->pods[i];
    w.ns = labels_reqs(pd.node_selector);
    for (uint32_t k = 0; k < pd.required_terms.count; k++) {
      no_min_values(p->terms[pd.required_terms.begin + k].requirements);
      w.req_terms.push_back(reqs_of(p->terms[pd.required_terms.begin + k].requirements));
    }
    for (uint32_t k = 0; k < pd.preferred_terms.count; k++) {
      auto& tm = p->terms[pd.preferred_terms.begin + k];
      no_min_values(tm.requirements);
      w.pref.push_back({tm.weight, reqs_of(tm.requirements)});
    }
    if (w.pref.size() > 12) throw Fail{GS_E_UNSUPPORTED, "more than 12 preferred node-affinity terms"};
    // sort.Slice by weight desc on <= 12 elements is insertion sort: stable
    std::stable_sort(w.pref.begin(), w.pref.end(), [](auto& a, auto& b) { return a.first > b.first; });
    // topology spread constraints -> groups (owners); namespace / labels for selectors
    const std::string& pns = S(pd.ns);
    chk(pd.labels, p->n_labels, "labels");
    w.sps = spreads_of(pd);
    for (auto& sp : w.sps) w.honor_taints = w.honor_taints || sp.honor_taints;
    chk(pd.tolerations, p->n_tolerations, "tolerations");
    for (uint32_t k = 0; k < pd.tolerations.count; k++) {
      auto& t = p->tolerations[pd.tolerations.begin + k];
      w.tols.push_back({S(t.key), S(t.value), S(t.effect), t.op});
    }
    // <U> MakeTopologyNodeFilter: node selector AND each required term.  Its
    // text (terms with values) is kept for every spec of a problem with
    // topology inputs: a spec counted by a group whose Honor filter reaches
    // past the zone key must carry that same filter (build_topology)
    FilterState f0;
    if (topo_inputs || !w.sps.empty()) f0 = filter_state(w, 0, w.tols);
    if (topo_inputs) {
      w.aff_text = f0.text;
      for (auto& pr : w.pref)
        for (auto& kv : pr.second) w.pref_keys.push_back(kv.first);
    }
    if (!w.sps.empty()) {
      key_spreads(w.sps, f0);
      // the states Relax moves the filter through: each dropped required
      // term, then the PreferNoSchedule toleration (pod_phase_c's order)
      const size_t nT = std::max<size_t>(w.req_terms.size(), 1);
      bool has_pns = false;
      for (auto& t : w.tols) has_pns = has_pns || (t.k.empty() && t.op == GS_TOL_EXISTS && t.v.empty() && t.eff == kPNS);
      w.n_states = (uint32_t)nT + (tolerate_pns && !has_pns ? 1u : 0u);
      w.st_sps.resize(w.n_states);
      w.st_hash.resize(w.n_states);
      w.st_gid.resize(w.n_states);
      for (uint32_t st = 1; st < w.n_states; st++) {
        std::vector<Tol> tols = w.tols;
        if (st == nT) tols.push_back({"", "", kPNS, GS_TOL_EXISTS});
        w.st_sps[st] = w.sps;
        key_spreads(w.st_sps[st], filter_state(w, std::min<size_t>(st, nT - 1), tols));
        for (auto& sp : w.st_sps[st]) w.st_hash[st].push_back(sp.hash(pns));
      }
    }
    const bool filter_empty = f0.empty;
    for (auto& sp : w.sps) {
      w.sp_hash.push_back(sp.hash(pns));
      std::string mk;
      // GS_GROUP_MERGE=0: one group per upstream group (A/B knob)
      static const bool merge_on = !std::getenv("GS_GROUP_MERGE") || std::atoi(std::getenv("GS_GROUP_MERGE")) != 0;
      if (merge_on && !sp.honor_taints && (sp.ignore_aff || filter_empty)) {
        SpreadEnc x = sp;
        x.fid = "-";
        mk = x.hash(pns) + "|m:" + std::to_string(sp.mind);
      }
      w.sp_merge.push_back(std::move(mk));
    }
    // anti-affinity, inverse anti-affinity and host-port groups
    if (topo_inputs) {
      const PodSel& me = pod_sel[spec_of[i]];
      for (auto& a : antis_of(pd)) {
        const bool self = a.selects(me.ns, me.labels);
        GroupEnc g = host_group(1, self, a.sel.key);
        g.anti = a;
        w.g_anti.push_back(GroupKey{"A|" + a.hash() + (self ? "|s" : "|n"), std::move(g), a.required, a.weight});
      }
      for (auto& a : terms_of(pd, pd.affinity, true)) {
        GroupEnc g = host_group(4, false);
        g.anti = a;
        w.g_aff.push_back(GroupKey{"F|" + a.hash(), std::move(g), a.required, a.weight});
      }
      for (auto& kv : inv_terms) {
        if (!kv.second.selects(me.ns, me.labels)) continue;
        const bool self = me.carried.count(kv.first) != 0;
        GroupEnc g = host_group(2, self, kv.second.sel.key);
        g.inv_hash = kv.first;
        w.g_inv.push_back(GroupKey{"I|" + kv.first + (self ? "|s" : "|n"), std::move(g)});
      }
      for (auto& pe : me.ports) {
        GroupEnc g = host_group(3, true);
        g.port = pe;
        w.g_port.push_back(GroupKey{"P|" + pe.key(), std::move(g)});
      }
    }
  }

  void pod_phase_b(uint32_t i, PodWork& w) {
    const std::string pns = S(p->pods[i].ns);
    for (size_t k = 0; k < w.sps.size(); k++) {
      auto f = group_idx.find(w.sp_hash[k]);
      if (f == group_idx.end()) {
        auto m = w.sp_merge[k].empty() ? merge_idx.end() : merge_idx.find(w.sp_merge[k]);
        if (m != merge_idx.end()) {
          f = group_idx.emplace(w.sp_hash[k], m->second).first;
        } else {
          if (groups.size() >= (size_t)gsd::TGMAX) throw Fail{GS_E_UNSUPPORTED, "more than 4096 topology groups"};
          f = group_idx.emplace(w.sp_hash[k], (uint32_t)groups.size()).first;
          if (!w.sp_merge[k].empty()) merge_idx.emplace(w.sp_merge[k], (uint32_t)groups.size());
          groups.push_back(GroupEnc{w.sps[k], pns});
          groups.back().owner_spec = spec_of[i];
        }
      } else if (!w.sps[k].ignore_aff && groups[f->second].sp.ftext != w.sps[k].ftext) {
        // upstream keys the group by the filter's keys and keeps its first
        // owner's filter: later owners with other values would see counts
        // filtered by someone else's node affinity
        throw Fail{GS_E_UNSUPPORTED,
                   "pods sharing a topology spread (nodeAffinityPolicy Honor) with different node affinity values"};
      }
      w.sgid.push_back(f->second);
    }
    for (auto& gk : w.g_anti) {
      const uint32_t gid = group_id(gk.key, std::move(gk.g));
      if (gk.required) w.own_static.push_back(gid);
      else w.anti_pref.push_back({gk.weight, gid});
    }
    if (w.anti_pref.size() > 12) throw Fail{GS_E_UNSUPPORTED, "more than 12 preferred anti-affinity terms"};
    for (auto& gk : w.g_aff) {
      const uint32_t gid = group_id(gk.key, std::move(gk.g));
      if (gk.required) w.own_static.push_back(gid);
      else w.aff_pref.push_back({gk.weight, gid});
    }
    if (w.aff_pref.size() > 12) throw Fail{GS_E_UNSUPPORTED, "more than 12 preferred pod affinity terms"};
    // sort.Slice by weight desc on <= 12 elements is insertion sort: stable
    std::stable_sort(w.aff_pref.begin(), w.aff_pref.end(), [](auto& a, auto& b) { return a.first > b.first; });
    std::stable_sort(w.anti_pref.begin(), w.anti_pref.end(), [](auto& a, auto& b) { return a.first > b.first; });
    for (auto& gk : w.g_inv) w.own_static.push_back(group_id(gk.key, std::move(gk.g)));
    for (auto& gk : w.g_port) w.own_static.push_back(group_id(gk.key, std::move(gk.g)));
    // the first variant owns every group (later ones only drop groups)
    std::vector<uint32_t> own = w.sgid;
    own.insert(own.end(), w.own_static.begin(), w.own_static.end());
    for (auto& x : w.anti_pref) own.push_back(x.second);
    for (auto& x : w.aff_pref) own.push_back(x.second);
    std::sort(own.begin(), own.end());
    if (std::unique(own.begin(), own.end()) - own.begin() > (ptrdiff_t)gsd::OWNMAX)
      throw Fail{GS_E_UNSUPPORTED, "a pod owns more than 64 topology groups"};
    w.g_anti.clear();
    w.g_aff.clear();
    w.g_inv.clear();
    w.g_port.clear();
  }

  uint32_t n_lazy = 0;
  void pod_phase_b2(uint32_t s, PodWork& w) {
    const std::string pns = S(p->pods[spec_rep[s]].ns);
    for (uint32_t st = 1; st < w.n_states; st++) {
      w.st_gid[st].clear();
      for (size_t k = 0; k < w.st_sps[st].size(); k++) {
        const SpreadEnc& sp = w.st_sps[st][k];
        auto f = group_idx.find(w.st_hash[st][k]);
        if (f == group_idx.end()) {
          // Topology.Update's new group counts the cluster's bound pods only
          // (a hostname group also lacks the in-flight NodeClaims registered
          // before it: the kernels mark those HC_UNKNOWN when it is created)
          if (groups.size() >= (size_t)gsd::TGMAX) throw Fail{GS_E_UNSUPPORTED, "more than 4096 topology groups"};
          if (n_lazy >= (uint32_t)gsd::TGMAX)
            throw Fail{GS_E_UNSUPPORTED, "more than 4096 topology spread groups created by relaxation"};
          f = group_idx.emplace(w.st_hash[st][k], (uint32_t)groups.size()).first;
          groups.push_back(GroupEnc{sp, pns});
          GroupEnc& g = groups.back();
          g.owner_spec = s;
          g.lazy = true;
          g.lazy_idx = n_lazy++;
          g.owner_state = st;
        } else {
          const GroupEnc& g = groups[f->second];
          if (!sp.ignore_aff && g.sp.ftext != sp.ftext)
            throw Fail{GS_E_UNSUPPORTED,
                       "pods sharing a topology spread (nodeAffinityPolicy Honor) with different node affinity values"};
        }
        w.st_gid[st].push_back(f->second);
      }
    }
  }

  // <U> NewPodRequirements + Preferences.Relax: every variant of one spec
  void pod_phase_c(PodWork& w) {
    std::vector<uint32_t> cur(w.sps.size());  // current constraints (swap-remove order)
    std::iota(cur.begin(), cur.end(), 0);
    std::vector<Tol> tols = w.tols;
    size_t ri = 0, pi = 0, ai = 0, fi = 0;
    uint32_t state = 0;  // the spreads' filter state (pod_phase_a)
    if (!w.sps.empty()) w.st_gid[0] = w.sgid;
    for (;;) {
      // <U> NewPodRequirements: nodeSelector + heaviest preferred + first required
      PodVariant v;
      v.reqs = w.ns;
      v.strict = w.ns;
      if (pi < w.pref.size()) reqs_add_all(e, v.reqs, w.pref[pi].second);
      if (ri < w.req_terms.size()) {
        reqs_add_all(e, v.reqs, w.req_terms[ri]);
        reqs_add_all(e, v.strict, w.req_terms[ri]);
      }
      v.tol = 0;  // build_taint_classes
      for (uint32_t k : cur) {
        const uint32_t g = w.st_gid[state][k];
        v.own.push_back(g);
        // the pod that relaxes first creates a lazy group with its own
        // minDomains (the kernels set it at that Relax)
        if (groups[g].lazy) v.lazy_mind.emplace_back(groups[g].lazy_idx, w.st_sps[state][k].mind);
      }
      w.var_state.push_back(state);
      v.own.insert(v.own.end(), w.own_static.begin(), w.own_static.end());
      for (size_t k = ai; k < w.anti_pref.size(); k++) v.own.push_back(w.anti_pref[k].second);
      for (size_t k = fi; k < w.aff_pref.size(); k++) v.own.push_back(w.aff_pref[k].second);
      std::sort(v.own.begin(), v.own.end());
      v.own.erase(std::unique(v.own.begin(), v.own.end()), v.own.end());
      w.vars.push_back(std::move(v));
      w.var_tols.push_back(tols);
      // <U> Preferences.Relax
      if (w.req_terms.size() - ri > 1) {
        ri++;
        state = (uint32_t)ri;
        continue;
      }
      // removePreferredPodAffinityTerm, then ...AntiAffinityTerm (the heaviest)
      if (fi < w.aff_pref.size()) {
        fi++;
        continue;
      }
      if (ai < w.anti_pref.size()) {
        ai++;
        continue;
      }
      if (pi < w.pref.size()) {
        pi++;
        continue;
      }
      // removeTopologySpreadScheduleAnyway: swap-remove the first one
      bool removed = false;
      for (size_t k = 0; k < cur.size() && !removed; k++)
        if (w.sps[cur[k]].sa) {
          cur[k] = cur.back();
          cur.pop_back();
          removed = true;
        }
      if (removed) continue;
      if (tolerate_pns) {
        bool has = false;
        for (auto& t : tols)
          if (t.k.empty() && t.op == GS_TOL_EXISTS && t.v.empty() && t.eff == kPNS) has = true;
        if (!has) {
          tols.push_back({"", "", kPNS, GS_TOL_EXISTS});
          state = w.n_states - 1;
          continue;
        }
      }
      break;
    }
  }

  void build_pods() {
    pt_last = std::chrono::steady_clock::now();
    e.P = p->n_pods;
    e.pod_req.assign((size_t)e.P * e.R, 0);
    // pods -> specs (first-carrier order): a 64-bit hash of each pod's spec
    // bytes in parallel, specs numbered by first hash occurrence, then every
    // pod's bytes compared with its spec's first pod's (a hash collision
    // falls back to an exact map over the bytes)
    spec_of.assign(e.P, 0);
    spec_rep.clear();
    {
      auto mix = [](const std::vector<uint32_t>& v) {
        uint64_t h = 0x9E3779B97F4A7C15ull ^ v.size();
        for (uint32_t x : v) {
          h ^= x;
          h *= 0xFF51AFD7ED558CCDull;
          h ^= h >> 32;
        }
        return h;
      };
      std::vector<uint64_t> hs(e.P);
      std::vector<uint8_t> ok(e.P, 0);
      par_for(e.P, 1024, [&](uint32_t i) {
        thread_local std::vector<uint32_t> buf;
        buf.clear();
        ok[i] = pod_sig(p->pods[i], buf);
        hs[i] = mix(buf);
      });
      std::unordered_map<uint64_t, uint32_t> first;
      first.reserve(256);
      for (uint32_t i = 0; i < e.P; i++) {
        if (!ok[i]) {
          spec_of[i] = (uint32_t)spec_rep.size();
          spec_rep.push_back(i);
          continue;
        }
        auto f = first.emplace(hs[i], (uint32_t)spec_rep.size());
        if (f.second) spec_rep.push_back(i);
        spec_of[i] = f.first->second;
      }
      std::vector<uint8_t> clash(e.P, 0);
      par_for(e.P, 1024, [&](uint32_t i) {
        const uint32_t r = spec_rep[spec_of[i]];
        if (r == i) return;
        thread_local std::vector<uint32_t> a, b;
        a.clear();
        b.clear();
        pod_sig(p->pods[i], a);
        pod_sig(p->pods[r], b);
        clash[i] = a != b;
      });
      std::map<std::vector<uint32_t>, uint32_t> exact;  // specs a collision split off
      for (uint32_t i = 0; i < e.P; i++) {
        if (!clash[i]) continue;
        std::vector<uint32_t> a;
        pod_sig(p->pods[i], a);
        auto f = exact.emplace(std::move(a), (uint32_t)spec_rep.size());
        if (f.second) spec_rep.push_back(i);
        spec_of[i] = f.first->second;
      }
      // specs numbered in first-carrier order (a collision's spec was appended)
      std::vector<uint32_t> order(spec_rep.size());
      std::iota(order.begin(), order.end(), 0);
      std::sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return spec_rep[x] < spec_rep[y]; });
      std::vector<uint32_t> rank(spec_rep.size());
      for (uint32_t k = 0; k < order.size(); k++) rank[order[k]] = k;
      std::vector<uint32_t> rep2(spec_rep.size());
      for (uint32_t k = 0; k < order.size(); k++) rep2[k] = spec_rep[order[k]];
      spec_rep.swap(rep2);
      for (uint32_t i = 0; i < e.P; i++) spec_of[i] = rank[spec_of[i]];
    }
    const uint32_t NS = (uint32_t)spec_rep.size();
    ph("specs");
    // <U> the inverse anti-affinity groups: required terms of pending and
    // bound pods (Topology.updateInverseAntiAffinity / updateInverseAffinities)
    // a problem without spreads, affinity terms or host ports builds no
    // group: the per-spec selection state (labels, carried terms) is skipped
    const bool topo_inputs = p->n_spreads || p->n_affinity_terms || p->n_host_ports;
    std::map<std::string, AntiEnc> inv_terms;
    if (topo_inputs) {
      pod_sel.assign(NS, PodSel{});
      std::vector<std::vector<AntiEnc>> req_antis(NS);
      std::vector<std::exception_ptr> serr(NS);
      par_for(NS, 8, [&](uint32_t s) {
        try {
          pod_sel[s] = sel_of(p->pods[spec_rep[s]]);
          for (auto& a : antis_of(p->pods[spec_rep[s]]))
            if (a.required) req_antis[s].push_back(std::move(a));
        } catch (...) {
          serr[s] = std::current_exception();
        }
      });
      // specs in first-carrier order: the first error and the first-inserted
      // term are the serial encoder's
      for (uint32_t s = 0; s < NS; s++) {
        if (serr[s]) std::rethrow_exception(serr[s]);
        for (auto& a : req_antis[s]) inv_terms.emplace(a.hash(), a);
      }
      chk(gs_range{0, p->n_bound_pods}, p->n_bound_pods, "bound pods");
      for (uint32_t b = 0; b < p->n_bound_pods; b++)
        for (auto& a : antis_of(p->bound_pods[b]))
          if (a.required) inv_terms.emplace(a.hash(), a);
    } else {
      for (uint32_t i = 0; i < e.P; i++) {
        chk(p->pods[i].anti_affinity, p->n_affinity_terms, "affinity_terms");
        chk(p->pods[i].affinity, p->n_affinity_terms, "affinity_terms");
        chk(p->pods[i].host_ports, p->n_host_ports, "host_ports");
      }
    }
    ph("groups");
    // the first pod whose uid an earlier pod carries (or names no string)
    uint32_t dup_at = e.P;
    bool dup_bad_id = false;
    {
      std::vector<uint8_t> uid_seen(strs.size(), 0);
      for (uint32_t i = 0; i < e.P && dup_at == e.P; i++) {
        if (p->pods[i].uid >= canon.size()) {
          dup_at = i;
          dup_bad_id = true;
          break;
        }
        const uint32_t cu = canon[p->pods[i].uid];
        if (uid_seen[cu]) dup_at = i;
        uid_seen[cu] = 1;
      }
    }
    ph("uids");
    // requests per pod, the spec's work per spec
    std::vector<std::exception_ptr> rerr(e.P);
    par_for(e.P, 1024, [&](uint32_t i) {
      try {
        resvec_fn(p->pods[i].requests, &e.pod_req[(size_t)i * e.R], nullptr);
      } catch (...) {
        rerr[i] = std::current_exception();
      }
    });
    std::vector<PodWork> work(NS);
    par_for(NS, 8, [&](uint32_t s) {
      const uint32_t i = spec_rep[s];
      if (p->pods[i].flags || i >= dup_at) return;
      try {
        pod_phase_a(i, work[s], inv_terms, topo_inputs);
      } catch (...) {
        work[s].err = std::current_exception();
      }
    });
    for (uint32_t i = 0; i < e.P; i++) {
      if (p->pods[i].flags) throw Fail{GS_E_UNSUPPORTED, "pod topology spread / pod affinity / host ports / volumes"};
      if (i == dup_at) throw Fail{GS_E_INVALID, dup_bad_id ? "string id out of range" : "duplicate pod uid"};
      if (rerr[i]) std::rethrow_exception(rerr[i]);
      const uint32_t s = spec_of[i];
      if (spec_rep[s] != i) continue;
      if (work[s].err) std::rethrow_exception(work[s].err);
      pod_phase_b(i, work[s]);
    }
    // <U> Topology.Update after a relaxation: every spread keyed under the
    // relaxed filter joins the group of that hash; a hash no pod's first
    // variant keys is a group created at that moment (lazy), in spec order
    for (uint32_t s = 0; s < NS; s++) pod_phase_b2(s, work[s]);
    par_for(NS, 8, [&](uint32_t s) {
      try {
        pod_phase_c(work[s]);
      } catch (...) {
        work[s].err = std::current_exception();
      }
    });
    for (uint32_t s = 0; s < NS; s++)
      if (work[s].err) std::rethrow_exception(work[s].err);
    spec_aff_text.assign(NS, std::string());
    spec_pref_keys.assign(NS, {});
    for (uint32_t s = 0; s < NS; s++) {
      spec_aff_text[s] = std::move(work[s].aff_text);
      spec_pref_keys[s] = std::move(work[s].pref_keys);
    }
    ph("spec_work");
    // spec variants (e.variants), then the device variants: each pod's
    // spec's variants in order (e.var_sv: device variant -> spec variant)
    sv_begin.assign(NS, 0);
    sv_count.assign(NS, 0);
    std::vector<std::vector<uint32_t>> spec_var_state(NS);
    for (uint32_t s = 0; s < NS; s++) {
      spec_var_state[s] = std::move(work[s].var_state);
      sv_begin[s] = (uint32_t)e.variants.size();
      sv_count[s] = (uint32_t)work[s].vars.size();
      for (auto& v : work[s].vars) e.variants.push_back(std::move(v));
      for (auto& t : work[s].var_tols) variant_tols.push_back(std::move(t));
      if (work[s].honor_taints) honor_specs.push_back(s);
    }
    // a group's first owner variant: the first variant of its first owner
    // spec (lazy groups: the first in the state that keys them)
    for (auto& g : groups) {
      if (g.owner_spec == gsd::NONE) continue;
      g.owner_sv = sv_begin[g.owner_spec];
      if (!g.lazy) continue;
      const auto& vs = spec_var_state[g.owner_spec];
      uint32_t k = 0;
      while (k < vs.size() && vs[k] != g.owner_state) k++;
      if (k == vs.size()) throw Fail{GS_E_INVALID, "internal: lazy topology group without its relaxation state"};
      g.owner_sv += k;
    }
    e.var_begin.resize(e.P);
    e.var_count.resize(e.P);
    uint32_t nv = 0;
    for (uint32_t i = 0; i < e.P; i++) {
      e.var_begin[i] = nv;
      e.var_count[i] = sv_count[spec_of[i]];
      nv += e.var_count[i];
    }
    e.var_sv.resize(nv);
    par_for(e.P, 2048, [&](uint32_t i) {
      const uint32_t b = sv_begin[spec_of[i]];
      for (uint32_t k = 0; k < e.var_count[i]; k++) e.var_sv[e.var_begin[i] + k] = b + k;
    });
    std::vector<int64_t> cpu(e.P, 0), mem(e.P, 0);
    auto rc = rid_map.find("cpu"), rmm = rid_map.find("memory");
    for (uint32_t i = 0; i < e.P; i++) {
      if (rc != rid_map.end()) cpu[i] = e.pod_req[(size_t)i * e.R + rc->second];
      if (rmm != rid_map.end()) mem[i] = e.pod_req[(size_t)i * e.R + rmm->second];
    }
    { std::vector<PodWork>().swap(work); }
    e.V = nv;
    ph("variants");
    // device variant records; identical has-bitsets share one arena slot and
    // identical IT-key requirement sets one class
    e.vars.resize(e.V);
    e.var_itclass.assign(e.V, gsd::NONE);
    std::map<std::vector<uint64_t>, uint32_t> arena_slot, itclass_of;
    std::vector<std::vector<uint32_t>> class_offs;  // per class: arena offset per IT key (NONE: unconstrained)
    auto arena = [&](const std::vector<uint64_t>& words) {
      auto f = arena_slot.find(words);
      if (f != arena_slot.end()) return f->second;
      const uint32_t off = (uint32_t)e.itmask.size();
      e.itmask.insert(e.itmask.end(), words.begin(), words.end());
      arena_slot.emplace(words, off);
      return off;
    };
    // one record per spec variant (serial: arena slots, classes and free-key
    // entries in first-use order), then every device variant a copy of its
    // spec variant's with its pod and index
    const uint32_t SV = (uint32_t)e.variants.size();
    std::vector<gsd::VarRec> sv_rec(SV);
    std::vector<uint32_t> sv_itclass(SV, gsd::NONE);
    for (uint32_t sv = 0; sv < SV; sv++) {
      auto& pv = e.variants[sv];
      gsd::VarRec& vr = sv_rec[sv];
      std::memset(&vr, 0, sizeof vr);
      for (int k = 0; k < gsd::KMAX_IT; k++) vr.itmask_off[k] = gsd::NONE;
      bool itk = false;
      for (uint32_t k = 0; k < e.K; k++) {
        auto f = pv.reqs.find(e.it_keys[k]);
        if (f == pv.reqs.end()) continue;
        vr.itmask_off[k] = arena(f->second.has.w);
        itk = true;
      }
      if (itk) {
        // the class key: the arena slots of the constrained keys
        std::vector<uint64_t> sig(vr.itmask_off, vr.itmask_off + e.K);
        auto f = itclass_of.find(sig);
        if (f == itclass_of.end()) {
          f = itclass_of.emplace(sig, (uint32_t)class_offs.size()).first;
          class_offs.emplace_back(vr.itmask_off, vr.itmask_off + e.K);
        }
        sv_itclass[sv] = f->second;
      }
      vr.zfull_off = vr.cfull_off = gsd::NONE;
      for (int kk = 0; kk < 2; kk++) {
        auto f = pv.reqs.find(kk ? e.k_ct : e.k_zone);
        if (f == pv.reqs.end()) continue;
        (kk ? vr.cfull_off : vr.zfull_off) = arena(f->second.has.w);
      }
      vr.zm = zone_has(pv.reqs);
      vr.cm = ct_has(pv.reqs);
      vr.ctb = ct_bits(pv.reqs) | (pv.reqs.empty() && pv.own.empty() ? gsd::VF_SIMPLE : 0u);
      // owns a zone spread group: only those read the per-pod minimum counts
      for (uint32_t g : pv.own)
        if (groups[g].sp.key != kHostname && groups[g].kind == 0) vr.ctb |= gsd::VF_ZSPREAD;
      // hostname-only topology (spread, anti-affinity, inverse, host ports;
      // not pod affinity): the wave kernel's fast accept reads the counts
      if (pv.reqs.empty() && !pv.own.empty() && pv.own.size() <= 4) {
        bool host = true;
        for (uint32_t g : pv.own) host = host && groups[g].sp.key == kHostname && groups[g].kind != 4;
        if (host) vr.ctb |= gsd::VF_HOSTFA;
      }
      vr.zs = zone_full(pv.strict);
      vr.zn = zone_full(pv.reqs);
      vr.zflags = zone_flags(pv.reqs);
      vr.tol = vr.tolt = 0;  // build_taint_classes
      vr.fk_begin = (uint32_t)e.fk_entries.size();
      for (auto& kv : pv.reqs) {
        const Key& key = e.keys[kv.first];
        if (key.cls != KEY_FREE && key.shadow < 0) continue;
        gsd::FKEntry fe{};
        fe.slot = (uint32_t)(key.cls == KEY_FREE ? key.slot : key.shadow);
        fe.st = to_fk(kv.second);
        e.fk_entries.push_back(fe);
        // the existing-node check of a shadowed key runs on its free slot
        // (the IT-key class above already has this key's mask)
        if (key.cls == KEY_IT) vr.itmask_off[key.slot] = gsd::NONE;
        else if (key.cls == KEY_ZONE) vr.zfull_off = gsd::NONE;
        else vr.cfull_off = gsd::NONE;
      }
      vr.fk_count = (uint32_t)e.fk_entries.size() - vr.fk_begin;

    }
    par_for(e.P, 1024, [&](uint32_t i) {
      for (uint32_t v = e.var_begin[i]; v < e.var_begin[i] + e.var_count[i]; v++) {
        e.vars[v] = sv_rec[e.var_sv[v]];
        e.vars[v].pod = i;
        e.vars[v].vix = v;
        e.var_itclass[v] = sv_itclass[e.var_sv[v]];
      }
    });
    if (e.itmask.empty()) e.itmask.push_back(0);
    e.itclass_mask.assign(std::max<size_t>(class_offs.size(), 1) * e.W, 0);
    for (size_t c = 0; c < class_offs.size(); c++)
      for (uint32_t it = 0; it < e.N; it++) {
        bool ok = true;
        for (uint32_t k = 0; k < e.K && ok; k++) {
          const uint32_t off = class_offs[c][k];
          if (off == gsd::NONE) continue;
          const uint32_t vid = e.it_vid[(size_t)k * e.N + it];
          ok = (e.itmask[off + (vid >> 6)] >> (vid & 63)) & 1;
        }
        if (ok) e.itclass_mask[c * e.W + it / 64] |= 1ull << (it % 64);
      }
    if (e.fk_entries.empty()) e.fk_entries.push_back(gsd::FKEntry{});
    ph("var_records");
    // <U> NewQueue: cpu desc, memory desc, creationTimestamp asc, UID asc (total order)
    // sorted on packed keys: the UID's first 8 bytes (big-endian, so integer
    // order is byte order) decide most ties without touching the strings
    // the fields as order-preserving unsigned integers (cpu and memory
    // descending, creation time ascending; signed -> unsigned by flipping the
    // sign bit) and the UID's first 8 bytes, in two 128-bit words: the sort
    // compares integers; keys that tie (UIDs sharing 8 bytes) are put in full
    // order afterwards
    struct QK {
      unsigned __int128 k, k2;
      uint32_t i;
    };
    std::vector<QK> qk(e.P);
    par_for(e.P, 4096, [&](uint32_t i) {
      const std::string& u = strs[p->pods[i].uid];  // checked by the uid pass
      uint64_t x = 0;
      for (size_t b = 0; b < 8; b++) x = (x << 8) | (b < u.size() ? (uint8_t)u[b] : 0u);
      auto bias = [](int64_t v) { return (uint64_t)v ^ (1ull << 63); };
      qk[i] = QK{((unsigned __int128)~bias(cpu[i]) << 64) | ~bias(mem[i]),
                 ((unsigned __int128)bias(p->pods[i].creation_ns) << 64) | x, i};
    });
    ph("queue_keys");
    auto kless = [](const QK& a, const QK& b) { return a.k != b.k ? a.k < b.k : a.k2 < b.k2; };
    auto qless = [&](const QK& a, const QK& b) {
      if (a.k != b.k) return a.k < b.k;
      if (a.k2 != b.k2) return a.k2 < b.k2;
      return strs[p->pods[a.i].uid] < strs[p->pods[b.i].uid];
    };
    // a total order (uids are unique): chunks sorted in parallel, then merged
    // pairwise; the result is the one order whatever the split
    {
      const uint32_t T = std::max<uint32_t>(1, std::min<uint32_t>(enc_threads(), e.P / 8192));
      std::vector<uint32_t> cut(T + 1);
      for (uint32_t t = 0; t <= T; t++) cut[t] = (uint32_t)((uint64_t)e.P * t / T);
      par_for(T, 1, [&](uint32_t t) { std::sort(qk.begin() + cut[t], qk.begin() + cut[t + 1], kless); });
      ph("queue_sort_chunks");
      // pairwise merge rounds between two buffers; each merge is split into
      // T output pieces by co-rank (merge path) so every round runs on all
      // threads
      std::vector<QK> tmp(e.P);
      std::vector<QK>* src = &qk;
      std::vector<QK>* dst = &tmp;
      for (uint32_t w = 1; w < T; w *= 2) {
        struct Piece {
          uint32_t a, m, b, k0, k1;
        };
        std::vector<Piece> pieces;
        for (uint32_t t = 0; t < T; t += 2 * w) {
          const uint32_t a = cut[t], m = cut[std::min(T, t + w)], b = cut[std::min(T, t + 2 * w)];
          for (uint32_t q = 0; q < T; q++)
            pieces.push_back({a, m, b, (uint32_t)((uint64_t)(b - a) * q / T), (uint32_t)((uint64_t)(b - a) * (q + 1) / T)});
        }
        const std::vector<QK>& S = *src;
        std::vector<QK>& D = *dst;
        // co-rank: how many of the output's first k come from the left run
        auto corank = [&](uint32_t a, uint32_t m, uint32_t b, uint32_t k) {
          uint32_t lo = k > b - m ? k - (b - m) : 0u, hi = std::min(k, m - a);
          while (lo < hi) {
            const uint32_t i = (lo + hi) / 2, j = k - i;  // i from the left, j from the right
            if (kless(S[m + j - 1], S[a + i])) hi = i;   // right[j-1] < left[i]: take fewer from the left
            else lo = i + 1;
          }
          return lo;
        };
        par_for((uint32_t)pieces.size(), 1, [&](uint32_t x) {
          const Piece& pc = pieces[x];
          const uint32_t i0 = corank(pc.a, pc.m, pc.b, pc.k0), i1 = corank(pc.a, pc.m, pc.b, pc.k1);
          std::merge(S.begin() + pc.a + i0, S.begin() + pc.a + i1, S.begin() + pc.m + (pc.k0 - i0),
                     S.begin() + pc.m + (pc.k1 - i1), D.begin() + pc.a + pc.k0, kless);
        });
        std::swap(src, dst);
      }
      if (src != &qk) qk.swap(tmp);
      ph("queue_sort_merge");
      // runs of equal keys (UIDs that share their first 8 bytes): full order
      for (uint32_t a = 0; a < e.P;) {
        uint32_t b = a + 1;
        while (b < e.P && qk[b].k == qk[a].k && qk[b].k2 == qk[a].k2) b++;
        if (b - a > 1) std::sort(qk.begin() + a, qk.begin() + b, qless);
        a = b;
      }
    }
    ph("queue_sort");
    e.queue0.resize(e.P);
    for (uint32_t k = 0; k < e.P; k++) e.queue0[k] = qk[k].i;
    e.checks = (uint64_t)e.P * e.checks_per_pod;
  }

  // <U> ExistingNode: labels + hostname In[name]; initialized first, then name
  void build_nodes() {
    e.NN = p->n_nodes;
    std::vector<uint32_t> order(e.NN);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
      const bool ia = p->nodes[a].initialized != 0, ib = p->nodes[b].initialized != 0;
      if (ia != ib) return ia;
      return S(p->nodes[a].name) < S(p->nodes[b].name);
    });
    e.node_order = order;
    e.nodes.assign(e.NN, gsd::NodeRec{});
    node_taints.assign(e.NN, {});
    e.n_fk.assign((size_t)std::max<uint32_t>(e.NN, 1) * std::max<uint32_t>(e.F, 1), gsd::FK{});
    // keys some pod variant constrains with NotIn/DoesNotExist: a node lacking
    // such a non-free key would gain dynamic state there (refused below)
    std::set<uint32_t> exempt_keys;
    for (auto& pv : e.variants)
      for (auto& kv : pv.reqs)
        if (e.keys[kv.first].cls != KEY_FREE && e.keys[kv.first].shadow < 0 && exempt(kv.second))
          exempt_keys.insert(kv.first);
    for (uint32_t pos = 0; pos < e.NN; pos++) {
      const gs_node& g = p->nodes[order[pos]];
      gsd::NodeRec& nr = e.nodes[pos];
      for (int k = 0; k < gsd::KMAX_IT; k++) nr.vid[k] = gsd::NONE;
      nr.zvid = nr.cvid = gsd::NONE;
      nr.dvid = gsd::DVID_NONE;
      Reqs reqs = node_labels_reqs(g.labels);
      uint32_t hk = e.k_hostname;
      reqs_add(e, reqs, hk, in_one_or_omega(hk, S(g.name)));
      for (auto& kv : reqs) {
        const Key& key = e.keys[kv.first];
        if (key.cls == KEY_FREE) {
          e.n_fk[(size_t)pos * e.F + key.slot] = to_fk(kv.second);
          continue;
        }
        if (key.shadow >= 0) e.n_fk[(size_t)pos * e.F + key.shadow] = to_fk(kv.second);
        // a label is In[v]: exactly one has-bit
        uint32_t vid = gsd::NONE;
        for (size_t i = 0; i < key.vocab.size(); i++)
          if (kv.second.has.test(i)) vid = (uint32_t)i;
        if (key.cls == KEY_IT) nr.vid[key.slot] = vid;
        else if (key.cls == KEY_ZONE) nr.zvid = vid;
        else nr.cvid = vid;
      }
      {
        // the topology domain key's value (zone, capacity type or NodePool)
        auto fd = reqs.find(e.k_dom);
        if (fd != reqs.end())
          for (size_t i = 0; i < e.keys[e.k_dom].vocab.size(); i++)
            if (fd->second.has.test(i)) nr.dvid = (uint16_t)i;
      }
      for (uint32_t k : exempt_keys) {
        bool has = reqs.count(k) != 0;
        if (!has)
          throw Fail{GS_E_UNSUPPORTED, "existing node lacks a label that a pod constrains with NotIn/DoesNotExist (" +
                                           e.keys[k].name + ": no free slot left, or its vocabulary exceeds 255 values)"};
      }
      bool present[gsd::RMAX] = {false};
      resvec_fn(g.available, nr.avail, present);
      nr.ok = 1;
      for (uint32_t r = 0; r < e.R; r++)
        if (present[r] && nr.avail[r] < 0) nr.ok = 0;  // <U> Fits: negative total never fits
      resvec_fn(g.requests, nr.req, nullptr);
      nr.taints = 0;  // build_taint_classes
      node_taints[pos] = state_taint_ids(g);
      nr.init = g.initialized ? 1u : 0u;
    }
    // every taint is known now (NodePools', then nodes'): the class masks
    build_taint_classes();
    const std::vector<uint64_t>& sv_tol = final_sv_tol;
    // nodeTaintsPolicy Honor: the group's filter holds the owner's own
    // tolerations (before Relax adds PreferNoSchedule); tolerating every
    // NodePool and node taint makes TopologyNodeFilter.Matches always true
    (void)sv_tol;  // nodeTaintsPolicy Honor: applied in build_topology
  }
};

}  // namespace

namespace {
}  // namespace

std::string canonical(const Encoded& e, const Reqs& r) {
  std::vector<std::pair<std::string, const KReq*>> items;
  for (auto& kv : r) items.push_back({e.keys[kv.first].name, &kv.second});
  std::sort(items.begin(), items.end(), [](auto& a, auto& b) { return a.first < b.first; });
  static const char* opn[] = {"In", "NotIn", "Exists", "DoesNotExist"};
  std::string s;
  for (auto& it : items) {
    const KReq& q = *it.second;
    const Vocab& v = e.keys[e.key_id.at(it.first)].vocab;
    if (!s.empty()) s += '\n';
    s += it.first;
    s += '|';
    s += opn[op_of(q)];
    s += '|';
    std::vector<std::string> vals;
    const Bits& b = q.comp ? q.excl : q.has;
    for (size_t i = 0; i < v.size(); i++)
      if (b.test(i)) vals.push_back(v.vals[i]);
    std::sort(vals.begin(), vals.end());
    for (size_t i = 0; i < vals.size(); i++) {
      if (i) s += ',';
      s += vals[i];
    }
    s += '|';
    s += q.comp && q.hg ? std::to_string(q.gt) : "-";
    s += '|';
    s += q.comp && q.hl ? std::to_string(q.lt) : "-";
    s += '|';
    s += q.mv >= 0 ? std::to_string(q.mv) : "-";
  }
  return s;
}

Err encode(const gs_problem* p, Encoded& e, uint32_t bound_alias) {
  // GS_ENCODE_PROFILE: per-phase wall clock on stderr (diagnostics)
  static const bool prof = std::getenv("GS_ENCODE_PROFILE") != nullptr;
  auto t_last = std::chrono::steady_clock::now();
  auto phase = [&](const char* name) {
    if (!prof) return;
    const auto t = std::chrono::steady_clock::now();
    std::fprintf(stderr, "encode %-12s %8.3f ms\n", name, std::chrono::duration<double, std::milli>(t - t_last).count());
    t_last = t;
  };
  // the per-pod arrays keep their capacity across the prepares of one
  // context: a repeated Solve of a similar batch refills mapped memory
  // instead of faulting in fresh pages (~13 MB of variant records at CM)
  auto vars = std::move(e.vars);
  auto pod_req = std::move(e.pod_req);
  auto var_begin = std::move(e.var_begin), var_count = std::move(e.var_count), var_sv = std::move(e.var_sv),
       var_itclass = std::move(e.var_itclass), queue0 = std::move(e.queue0);
  e = Encoded();
  for (auto* v : {&var_begin, &var_count, &var_sv, &var_itclass, &queue0}) v->clear();
  vars.clear();
  pod_req.clear();
  e.vars = std::move(vars);
  e.pod_req = std::move(pod_req);
  e.var_begin = std::move(var_begin);
  e.var_count = std::move(var_count);
  e.var_sv = std::move(var_sv);
  e.var_itclass = std::move(var_itclass);
  e.queue0 = std::move(queue0);
  phase("reset");
  Err r{};
  // the encoder's scratch (strings, maps, per-spec tables: ~10^5 heap blocks
  // at CM) is freed on a pool worker after encode returns, off the Solve's
  // critical path
  std::shared_ptr<Ctx> cp(new Ctx{p, e, {}});
  {
    Ctx& c = *cp;
    c.bound_alias = bound_alias;
    try {
      c.strs.resize(p->n_strings);
      par_for(p->n_strings, 4096, [&](uint32_t i) {
        if (p->strings[i]) c.strs[i] = p->strings[i];
      });
      phase("strings");
      c.build_canon();
      phase("canon");
      c.build_vocab();
      phase("vocab");
      c.build_catalog();
      phase("catalog");
      c.build_templates();
      phase("templates");
      c.build_free_slots();
      phase("free_slots");
      c.build_pods();
      phase("pods");
      c.build_nodes();
      phase("nodes");
      c.build_topology();
      phase("topology");
      c.build_volumes();
      phase("volumes");
    } catch (const Fail& f) {
      r = Err{f.code, f.msg};
    } catch (const std::out_of_range& ex) {
      r = Err{GS_E_INVALID, std::string("unknown vocabulary value: ") + ex.what()};
    }
  }
  run_detached([cp]() mutable { cp.reset(); });
  cp.reset();
  phase("teardown");
  return r;
}

void host_copy_parallel(void* dst_base, const HostCopy* copies, size_t n) {
  // pieces of at most 1 MiB, handed out to the encoder's threads
  constexpr size_t kPiece = 1u << 20;
  std::vector<HostCopy> pieces;
  size_t total = 0;
  for (size_t i = 0; i < n; i++)
    for (size_t o = 0; o < copies[i].bytes; o += kPiece)
      pieces.push_back({(const char*)copies[i].src + o, copies[i].off + o, std::min(kPiece, copies[i].bytes - o)});
  for (auto& p : pieces) total += p.bytes;
  char* dst = (char*)dst_base;
  par_for((uint32_t)pieces.size(), total >= (8u << 20) ? 1u : (uint32_t)pieces.size() + 1,
          [&](uint32_t i) { std::memcpy(dst + pieces[i].off, pieces[i].src, pieces[i].bytes); });
}

// label helpers shared with the launch-time re-filter (filter.hip)
bool label_is_wellknown(const std::string& k) { return is_wellknown(k); }
std::string label_normalize(const std::string& k) { return normalize(k); }
bool go_atoi64(const std::string& s, int64_t* out) { return atoi64(s, out); }

}  // namespace gsh
