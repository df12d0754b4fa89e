// filter.hip — launch-time re-filter of emitted NodeClaims (gs_create_filter):
// CloudProvider.Create's instance-type filter (reference
// pkg/cloudprovider/cloudprovider.go:322-346), GetInstanceTypes' NodePool
// filter (:574-577), the instance provider's instanceTypes[0] pick
// (pkg/providers/vpc/instance/provider.go:215-221) and ResolveCapacityType
// (pkg/providers/common/capacitytype/capacitytype.go:27-42), for a batch of
// NodeClaims in one device pass.
//
// Unlike the Solve encoder (encode.cpp), which folds requirements into
// per-key vocabulary bitsets under the restrictions the FFD kernels need,
// this path keeps the general <U> scheduling.Requirement algebra: every
// requirement list is reduced on the host to one entry per (normalised) key
// — complement flag, Gt/Lt bounds and a sorted list of dense value ids — and
// the kernel evaluates Requirements.Compatible for each (claim, instance
// type) pair by merging the two key-sorted lists (one lane per pair).
//
// HBM layout (one arena per call):
//   reqs[]  FReq (32 B) — all requirement lists, key-sorted within a list
//   vals[]  u32 dense value ids, sorted within a requirement
//   vint[]  i64 parsed value (strconv.Atoi) per dense value, vok[] u8 parse ok
//   its[]   FIt: requirement list, offering range, Allocatable() < 0 flag
//   offs[]  FOff: requirement list, Available, Requirements.Get(ct).Has(spot)
//   alloc[] i64 [N][R]: Allocatable() over the resources the claims request
//   qs[]    FQuery: requirement list + request range into qty[]
//   out     u64 bitsets [Q][W] x3 (Create filter, requirements-only, spot)
#include "ctx.hpp"

#include <map>
#include <set>

namespace gsf {

enum : uint32_t { F_COMP = 1, F_GT = 2, F_LT = 4, F_WK = 8 };

struct FReq {
  uint32_t key, flags, vb, vn;
  int64_t gt, lt;
};
struct FList {
  uint32_t b, n;
};
struct FIt {
  FList reqs;
  uint32_t ob, on;
  uint32_t alloc_neg, pad;
};
struct FOff {
  FList reqs;
  uint32_t available, spot;
};
struct FQty {
  uint32_t r, pad;
  int64_t v;
};
struct FQuery {
  FList reqs;
  uint32_t qb, qn;
};
static_assert(sizeof(FReq) == 32 && sizeof(FIt) == 24 && sizeof(FOff) == 16 && sizeof(FQty) == 16, "filter layout");

struct DevFilter {
  const FReq* reqs;
  const uint32_t* vals;
  const int64_t* vint;
  const uint8_t* vok;
  const FIt* its;
  const FOff* offs;
  const int64_t* alloc;
  const FQuery* qs;
  const FQty* qty;
  uint32_t N, Q, R, W;
  uint64_t* out_create;
  uint64_t* out_reqs;
  uint64_t* out_spot;
};

// ----------------------------------------------------------------- device
__device__ __forceinline__ bool exempt(const FReq& q) {
  // Operator() in {NotIn, DoesNotExist}
  return (q.flags & F_COMP) ? q.vn != 0 : q.vn == 0;
}

__device__ __forceinline__ bool contains(const uint32_t* v, uint32_t n, uint32_t x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    uint32_t m = (lo + hi) >> 1;
    if (v[m] < x) lo = m + 1;
    else hi = m;
  }
  return lo < n && v[lo] == x;
}

// <U> Requirement.Intersection(a, b).Len() == 0
__device__ bool len_zero(const DevFilter& d, const FReq& a, const FReq& b) {
  const bool hg = (a.flags | b.flags) & F_GT, hl = (a.flags | b.flags) & F_LT;
  int64_t gt = (a.flags & F_GT) ? a.gt : b.gt;
  if ((a.flags & F_GT) && (b.flags & F_GT)) gt = a.gt > b.gt ? a.gt : b.gt;
  int64_t lt = (a.flags & F_LT) ? a.lt : b.lt;
  if ((a.flags & F_LT) && (b.flags & F_LT)) lt = a.lt < b.lt ? a.lt : b.lt;
  if (hg && hl && gt >= lt) return true;  // DoesNotExist
  const bool ac = a.flags & F_COMP, bc = b.flags & F_COMP;
  if (ac && bc) return false;  // MaxInt64 - |union| > 0
  // walk the concrete side (the smaller one when both are concrete)
  const FReq* s = &a;
  const FReq* o = &b;
  if (ac || (!bc && b.vn < a.vn)) {
    s = &b;
    o = &a;
  }
  const bool want = !(o->flags & F_COMP);  // concrete other: intersection; complement: difference
  for (uint32_t i = 0; i < s->vn; i++) {
    const uint32_t v = d.vals[s->vb + i];
    if (contains(d.vals + o->vb, o->vn, v) != want) continue;
    if (hg || hl) {
      if (!d.vok[v]) continue;
      const int64_t x = d.vint[v];
      if ((hg && gt >= x) || (hl && lt <= x)) continue;
    }
    return false;
  }
  return true;
}

// <U> Requirements.Compatible(incoming, AllowUndefinedWellKnownLabels):
// incoming keys the existing list lacks must be well known or NotIn /
// DoesNotExist; shared keys must intersect unless both are NotIn/DoesNotExist
__device__ bool compatible(const DevFilter& d, FList ex, FList in) {
  uint32_t i = ex.b;
  const uint32_t ie = ex.b + ex.n;
  for (uint32_t j = in.b; j < in.b + in.n; j++) {
    const FReq b = d.reqs[j];
    while (i < ie && d.reqs[i].key < b.key) i++;
    if (i < ie && d.reqs[i].key == b.key) {
      const FReq a = d.reqs[i];
      if (len_zero(d, a, b) && !(exempt(a) && exempt(b))) return false;
    } else if (!(b.flags & F_WK) && !exempt(b)) {
      return false;
    }
  }
  return true;
}

// one lane per (claim, instance type); blockIdx.y = claim, 256 types per block
__global__ __launch_bounds__(256) void claim_filter_kernel(DevFilter d) {
  const uint32_t q = blockIdx.y;
  const uint32_t it = blockIdx.x * 256 + threadIdx.x;
  bool ok_req = false, ok_create = false, ok_spot = false;
  if (it < d.N) {
    const FQuery Q = d.qs[q];
    const FIt I = d.its[it];
    ok_req = compatible(d, Q.reqs, I.reqs);
    bool fits = !I.alloc_neg;
    for (uint32_t k = 0; fits && k < Q.qn; k++) {
      const FQty x = d.qty[Q.qb + k];
      fits = x.v <= d.alloc[(size_t)it * d.R + x.r];
    }
    bool any = false;
    for (uint32_t o = 0; ok_req && fits && o < I.on; o++) {
      const FOff f = d.offs[I.ob + o];
      if (!f.available || !compatible(d, Q.reqs, f.reqs)) continue;
      any = true;
      if (f.spot) {
        ok_spot = true;
        break;
      }
    }
    ok_create = ok_req && fits && any;
    ok_spot = ok_spot && ok_create;
  }
  const uint64_t b_req = __ballot(ok_req), b_create = __ballot(ok_create), b_spot = __ballot(ok_spot);
  const uint32_t w = it >> 6;
  if ((threadIdx.x & 63) == 0 && w < d.W) {
    const size_t o = (size_t)q * d.W + w;
    d.out_reqs[o] = b_req;
    d.out_create[o] = b_create;
    d.out_spot[o] = b_spot;
  }
}

// ------------------------------------------------------------------- host
struct Fail {
  gs_status code;
  std::string msg;
};

// one requirement on one key during host reduction
struct HReq {
  uint32_t key;
  bool comp = true;
  std::vector<uint32_t> vals;  // sorted dense value ids
  bool hg = false, hl = false;
  int64_t gt = 0, lt = 0;
};

struct Enc {
  const gs_problem* p;
  std::vector<std::string> strs;
  std::map<std::string, uint32_t> key_id;
  std::vector<std::string> key_name;
  std::unordered_map<std::string, uint32_t> val_id;
  std::vector<int64_t> vint;
  std::vector<uint8_t> vok;
  std::vector<FReq> reqs;
  std::vector<uint32_t> vals;

  const std::string& S(uint32_t id) const {
    if (id >= strs.size()) throw Fail{GS_E_INVALID, "string id out of range"};
    return strs[id];
  }
  void chk(gs_range r, uint32_t n, const char* what) const {
    if ((uint64_t)r.begin + r.count > n) throw Fail{GS_E_INVALID, std::string("range out of bounds: ") + what};
  }
  uint32_t value(const std::string& v) {
    auto f = val_id.find(v);
    if (f != val_id.end()) return f->second;
    const uint32_t id = (uint32_t)vint.size();
    val_id.emplace(v, id);
    int64_t x = 0;
    vok.push_back(gsh::go_atoi64(v, &x) ? 1 : 0);
    vint.push_back(x);
    return id;
  }
  bool within(uint32_t v, bool hg, int64_t gt, bool hl, int64_t lt) const {
    if (!hg && !hl) return true;
    if (!vok[v]) return false;
    return !(hg && gt >= vint[v]) && !(hl && lt <= vint[v]);
  }
  // <U> NewRequirement (keys normalised, In/NotIn values, Gt/Lt bounds)
  HReq make(const gs_requirement& q) {
    if (q.op > GS_OP_LTE) throw Fail{GS_E_INVALID, "unknown requirement operator"};
    // minValues: Compatible ignores it (reference cloudprovider.go:321-325)
    chk(q.values, p->n_value_ids, "values");
    const std::string k = gsh::label_normalize(S(q.key));
    auto f = key_id.find(k);
    HReq r;
    if (f == key_id.end()) {
      r.key = (uint32_t)key_name.size();
      key_id.emplace(k, r.key);
      key_name.push_back(k);
    } else {
      r.key = f->second;
    }
    r.comp = !(q.op == GS_OP_IN || q.op == GS_OP_DOES_NOT_EXIST);
    if (q.op == GS_OP_IN || q.op == GS_OP_NOTIN) {
      for (uint32_t i = 0; i < q.values.count; i++) r.vals.push_back(value(S(p->value_ids[q.values.begin + i])));
      std::sort(r.vals.begin(), r.vals.end());
      r.vals.erase(std::unique(r.vals.begin(), r.vals.end()), r.vals.end());
    }
    if (q.op >= GS_OP_GT) {
      int64_t x = 0;
      if (q.values.count < 1 || !gsh::go_atoi64(S(p->value_ids[q.values.begin]), &x))
        throw Fail{GS_E_INVALID, "Gt/Lt/Gte/Lte value is not an integer"};
      if ((q.op == GS_OP_GTE && x == INT64_MIN) || (q.op == GS_OP_LTE && x == INT64_MAX))
        throw Fail{GS_E_INVALID, "Gte/Lte bound out of range"};
      // over integer label values Gte x is Gt x-1 and Lte x is Lt x+1
      const bool lower = q.op == GS_OP_GT || q.op == GS_OP_GTE;
      const int64_t b = q.op == GS_OP_GTE ? x - 1 : q.op == GS_OP_LTE ? x + 1 : x;
      (lower ? r.hg : r.hl) = true;
      (lower ? r.gt : r.lt) = b;
    }
    return r;
  }
  // <U> Requirement.Intersection (Requirements.Add on a repeated key)
  HReq intersect(const HReq& a, const HReq& b) const {
    HReq r;
    r.key = a.key;
    r.hg = a.hg || b.hg;
    r.gt = a.hg && b.hg ? std::max(a.gt, b.gt) : (a.hg ? a.gt : b.gt);
    r.hl = a.hl || b.hl;
    r.lt = a.hl && b.hl ? std::min(a.lt, b.lt) : (a.hl ? a.lt : b.lt);
    if (r.hg && r.hl && r.gt >= r.lt) {  // DoesNotExist
      r.comp = false;
      r.hg = r.hl = false;
      return r;
    }
    r.comp = a.comp && b.comp;
    std::vector<uint32_t> v;
    if (a.comp && b.comp)
      std::set_union(a.vals.begin(), a.vals.end(), b.vals.begin(), b.vals.end(), std::back_inserter(v));
    else if (a.comp)
      std::set_difference(b.vals.begin(), b.vals.end(), a.vals.begin(), a.vals.end(), std::back_inserter(v));
    else if (b.comp)
      std::set_difference(a.vals.begin(), a.vals.end(), b.vals.begin(), b.vals.end(), std::back_inserter(v));
    else
      std::set_intersection(a.vals.begin(), a.vals.end(), b.vals.begin(), b.vals.end(), std::back_inserter(v));
    for (uint32_t x : v)
      if (within(x, r.hg, r.gt, r.hl, r.lt)) r.vals.push_back(x);
    if (!r.comp) r.hg = r.hl = false;
    return r;
  }
  // NewNodeSelectorRequirementsWithMinValues: one entry per key
  std::map<uint32_t, HReq> reduce(gs_range rg) {
    chk(rg, p->n_reqs, "reqs");
    std::map<uint32_t, HReq> m;
    for (uint32_t i = 0; i < rg.count; i++) {
      HReq r = make(p->reqs[rg.begin + i]);
      auto f = m.find(r.key);
      if (f == m.end()) m.emplace(r.key, std::move(r));
      else f->second = intersect(r, f->second);
    }
    return m;
  }
  FList emit(const std::map<uint32_t, HReq>& m) {
    FList l{(uint32_t)reqs.size(), (uint32_t)m.size()};
    for (auto& kv : m) {
      const HReq& r = kv.second;
      FReq f{};
      f.key = r.key;
      f.flags = (r.comp ? F_COMP : 0) | (r.hg ? F_GT : 0) | (r.hl ? F_LT : 0) |
                (gsh::label_is_wellknown(key_name[r.key]) ? F_WK : 0);
      f.vb = (uint32_t)vals.size();
      f.vn = (uint32_t)r.vals.size();
      f.gt = r.gt;
      f.lt = r.lt;
      vals.insert(vals.end(), r.vals.begin(), r.vals.end());
      reqs.push_back(f);
    }
    return l;
  }
  // Requirements.Get(capacity-type).Has("spot") (absent key: Exists)
  bool has_spot(const std::map<uint32_t, HReq>& m) {
    auto k = key_id.find("karpenter.sh/capacity-type");
    if (k == key_id.end()) return true;
    auto f = m.find(k->second);
    if (f == m.end()) return true;
    const HReq& r = f->second;
    const uint32_t v = value("spot");
    const bool in = std::binary_search(r.vals.begin(), r.vals.end(), v);
    return (r.comp ? !in : in) && within(v, r.hg, r.gt, r.hl, r.lt);
  }
};

}  // namespace gsf

using namespace gsc;
using namespace gsf;

extern "C" gs_status gs_create_filter(gs_ctx* c, const gs_problem* p, const gs_claim_query* qs, uint32_t nq,
                                      gs_claim_filter_result* out) {
  if (!c || !p || !out || (nq && !qs)) return GS_E_INVALID;
  std::memset(out, 0, sizeof(*out));
  // reject before any allocation: the grid's y dimension, and every array the
  // host pass reads that is null while its count is not
  if (nq > 65535u) return fail(c, GS_E_INVALID, "more than 65535 claims in one gs_create_filter call");
  if ((p->n_instance_types && !p->instance_types) || (p->n_offerings && !p->offerings) ||
      (p->n_quantities && !p->quantities) || (p->n_reqs && !p->reqs) || (p->n_value_ids && !p->value_ids) ||
      (p->n_strings && !p->strings))
    return fail(c, GS_E_INVALID, "null array with a non-zero count");
  Enc e;
  e.p = p;
  std::vector<FIt> its;
  std::vector<FOff> offs;
  std::vector<FQuery> fq;
  std::vector<FQty> qty;
  std::vector<int64_t> alloc;
  std::vector<uint8_t> q_spot;  // the claim's capacity-type requirement allows spot
  uint32_t R = 0;
  const uint32_t N = p->n_instance_types;
  try {
    if (p->n_strings && !p->strings) throw Fail{GS_E_INVALID, "strings"};
    e.strs.reserve(p->n_strings);
    for (uint32_t i = 0; i < p->n_strings; i++) e.strs.push_back(p->strings[i] ? p->strings[i] : "");
    // claims first: their requested resources form the Fits vocabulary
    std::map<std::string, uint32_t> res_id;
    for (uint32_t q = 0; q < nq; q++) {
      auto m = e.reduce(qs[q].requirements);
      FQuery x{};
      x.reqs = e.emit(m);
      q_spot.push_back(e.has_spot(m) ? 1 : 0);
      e.chk(qs[q].requests, p->n_quantities, "requests");
      std::map<uint32_t, int64_t> sum;  // resource lists are maps: repeated names add
      for (uint32_t k = 0; k < qs[q].requests.count; k++) {
        const gs_quantity& g = p->quantities[qs[q].requests.begin + k];
        auto f = res_id.emplace(e.S(g.resource), (uint32_t)res_id.size()).first;
        sum[f->second] += g.milli;
      }
      x.qb = (uint32_t)qty.size();
      x.qn = (uint32_t)sum.size();
      for (auto& kv : sum) qty.push_back(FQty{kv.first, 0, kv.second});
      fq.push_back(x);
    }
    R = std::max<uint32_t>(1, (uint32_t)res_id.size());
    alloc.assign((size_t)N * R, 0);
    e.chk(gs_range{0, N}, N, "instance_types");
    for (uint32_t i = 0; i < N; i++) {
      const gs_instance_type& g = p->instance_types[i];
      FIt x{};
      x.reqs = e.emit(e.reduce(g.requirements));
      // Allocatable() = capacity - overhead over the capacity's resources
      e.chk(g.capacity, p->n_quantities, "capacity");
      e.chk(g.overhead, p->n_quantities, "overhead");
      std::map<std::string, int64_t> cap, ovh;
      for (uint32_t k = 0; k < g.capacity.count; k++)
        cap[e.S(p->quantities[g.capacity.begin + k].resource)] += p->quantities[g.capacity.begin + k].milli;
      for (uint32_t k = 0; k < g.overhead.count; k++)
        ovh[e.S(p->quantities[g.overhead.begin + k].resource)] += p->quantities[g.overhead.begin + k].milli;
      for (auto& kv : cap) {
        auto o = ovh.find(kv.first);
        const int64_t a = kv.second - (o == ovh.end() ? 0 : o->second);
        if (a < 0) x.alloc_neg = 1;
        auto r = res_id.find(kv.first);
        if (r != res_id.end()) alloc[(size_t)i * R + r->second] = a;
      }
      e.chk(g.offerings, p->n_offerings, "offerings");
      x.ob = (uint32_t)offs.size();
      x.on = g.offerings.count;
      for (uint32_t k = 0; k < g.offerings.count; k++) {
        const gs_offering& o = p->offerings[g.offerings.begin + k];
        auto m = e.reduce(o.requirements);
        FOff f{};
        f.reqs = e.emit(m);
        f.available = o.available ? 1 : 0;
        f.spot = e.has_spot(m) ? 1 : 0;
        offs.push_back(f);
      }
      its.push_back(x);
    }
  } catch (const Fail& f) {
    return fail(c, f.code, f.msg);
  }
  const uint32_t W = (N + 63) / 64;
  c->cf_create.assign((size_t)nq * W, 0);
  c->cf_reqs.assign((size_t)nq * W, 0);
  c->cf_spot.assign((size_t)nq * W, 0);
  if (nq && N) {
    try {
      HIPCHK(hipSetDevice(c->device));
      // one arena: inputs then the three output bitsets
      size_t off = 0;
      auto place = [&](size_t bytes) {
        const size_t o = off;
        off += (std::max<size_t>(bytes, 1) + 255) & ~(size_t)255;
        return o;
      };
      const size_t o_reqs = place(e.reqs.size() * sizeof(FReq)), o_vals = place(e.vals.size() * 4),
                   o_vint = place(e.vint.size() * 8), o_vok = place(e.vok.size()), o_its = place(its.size() * sizeof(FIt)),
                   o_offs = place(offs.size() * sizeof(FOff)), o_alloc = place(alloc.size() * 8),
                   o_qs = place(fq.size() * sizeof(FQuery)), o_qty = place(qty.size() * sizeof(FQty)),
                   o_out = place((size_t)3 * nq * W * 8);
      if (off > c->cf_bytes) {
        if (c->cf_dev) HIPCHK(hipFree(c->cf_dev));
        c->cf_dev = nullptr;
        c->cf_bytes = 0;
        HIPCHK(hipMalloc(&c->cf_dev, off));
        c->cf_bytes = off;
      }
      char* base = (char*)c->cf_dev;
      // pinned staging: one host copy, one H2D transfer
      std::vector<char> h(o_out);
      auto put = [&](size_t o, const void* src, size_t bytes) {
        if (bytes) std::memcpy(h.data() + o, src, bytes);
      };
      put(o_reqs, e.reqs.data(), e.reqs.size() * sizeof(FReq));
      put(o_vals, e.vals.data(), e.vals.size() * 4);
      put(o_vint, e.vint.data(), e.vint.size() * 8);
      put(o_vok, e.vok.data(), e.vok.size());
      put(o_its, its.data(), its.size() * sizeof(FIt));
      put(o_offs, offs.data(), offs.size() * sizeof(FOff));
      put(o_alloc, alloc.data(), alloc.size() * 8);
      put(o_qs, fq.data(), fq.size() * sizeof(FQuery));
      put(o_qty, qty.data(), qty.size() * sizeof(FQty));
      HIPCHK(hipMemcpyAsync(base, h.data(), o_out, hipMemcpyHostToDevice, c->stream));
      DevFilter d{};
      d.reqs = (const FReq*)(base + o_reqs);
      d.vals = (const uint32_t*)(base + o_vals);
      d.vint = (const int64_t*)(base + o_vint);
      d.vok = (const uint8_t*)(base + o_vok);
      d.its = (const FIt*)(base + o_its);
      d.offs = (const FOff*)(base + o_offs);
      d.alloc = (const int64_t*)(base + o_alloc);
      d.qs = (const FQuery*)(base + o_qs);
      d.qty = (const FQty*)(base + o_qty);
      d.N = N;
      d.Q = nq;
      d.R = R;
      d.W = W;
      d.out_create = (uint64_t*)(base + o_out);
      d.out_reqs = d.out_create + (size_t)nq * W;
      d.out_spot = d.out_reqs + (size_t)nq * W;
      HIPCHK(hipEventRecord(c->ev[6], c->stream));
      hipLaunchKernelGGL(claim_filter_kernel, dim3((N + 255) / 256, nq), dim3(256), 0, c->stream, d);
      HIPCHK(hipGetLastError());
      HIPCHK(hipEventRecord(c->ev[7], c->stream));
      const size_t ob = (size_t)nq * W * 8;
      HIPCHK(hipMemcpyAsync(c->cf_create.data(), d.out_create, ob, hipMemcpyDeviceToHost, c->stream));
      HIPCHK(hipMemcpyAsync(c->cf_reqs.data(), d.out_reqs, ob, hipMemcpyDeviceToHost, c->stream));
      HIPCHK(hipMemcpyAsync(c->cf_spot.data(), d.out_spot, ob, hipMemcpyDeviceToHost, c->stream));
      HIPCHK(hipStreamSynchronize(c->stream));
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, c->ev[6], c->ev[7]));
      c->t_filter = ms;
    } catch (const HipError& ex) {
      return fail(c, GS_E_HIP, ex.msg);
    }
  }
  c->cf_n.assign(nq, 0);
  c->cf_sel.assign(nq, -1);
  c->cf_ct.assign(nq, GS_CAPACITY_ON_DEMAND);
  for (uint32_t q = 0; q < nq; q++) {
    bool spot = false;
    for (uint32_t w = 0; w < W; w++) {
      const uint64_t x = c->cf_create[(size_t)q * W + w];
      if (x && c->cf_sel[q] < 0) c->cf_sel[q] = (int32_t)(64 * w + __builtin_ctzll(x));
      c->cf_n[q] += (uint32_t)__builtin_popcountll(x);
      spot |= c->cf_spot[(size_t)q * W + w] != 0;
    }
    if (q_spot[q] && spot) c->cf_ct[q] = GS_CAPACITY_SPOT;
  }
  out->n_queries = nq;
  out->words = W;
  out->compatible = c->cf_create.data();
  out->requirements = c->cf_reqs.data();
  out->n_compatible = c->cf_n.data();
  out->selected = c->cf_sel.data();
  out->capacity_type = c->cf_ct.data();
  return GS_OK;
}
