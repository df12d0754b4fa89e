// encode.hpp — host-side encoder: gs_problem (strings) -> label-vocabulary
// bitsets + int64 SoA (layout.hpp), and the bitset requirement algebra used
// to build templates / pod variants and to decode NodeClaim requirements.
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/gpusched.h"
#include "layout.hpp"

namespace gsh {

// ------------------------------------------------------------------ bitsets
struct Bits {
  std::vector<uint64_t> w;
  Bits() = default;
  explicit Bits(size_t words) : w(words, 0) {}
  bool test(size_t i) const { return (w[i >> 6] >> (i & 63)) & 1; }
  void set(size_t i) { w[i >> 6] |= 1ull << (i & 63); }
  void reset(size_t i) { w[i >> 6] &= ~(1ull << (i & 63)); }
  bool none() const {
    for (auto x : w)
      if (x) return false;
    return true;
  }
  size_t count() const {
    size_t c = 0;
    for (auto x : w) c += __builtin_popcountll(x);
    return c;
  }
  Bits& operator&=(const Bits& o) {
    for (size_t i = 0; i < w.size(); i++) w[i] &= o.w[i];
    return *this;
  }
  Bits& operator|=(const Bits& o) {
    for (size_t i = 0; i < w.size(); i++) w[i] |= o.w[i];
    return *this;
  }
};

// value vocabulary of one requirement key; the last entry is omega, a value
// no requirement mentions (stands for hostname placeholders)
struct Vocab {
  std::vector<std::string> vals;
  std::unordered_map<std::string, uint32_t> id;
  std::vector<uint8_t> isint;
  std::vector<int64_t> ival;
  uint32_t omega = 0;
  size_t words() const { return (vals.size() + 63) / 64; }
  size_t size() const { return vals.size(); }
};

// Requirement on one key, as bitsets over the key's vocabulary.
// Semantics follow <U> scheduling.Requirement: complement / values / bounds.
struct KReq {
  bool comp = true;
  Bits has;   // Has(v) for every vocabulary value
  Bits excl;  // complement sets: excluded values (after bound filtering)
  bool hg = false, hl = false;
  int64_t gt = 0, lt = 0;
  int64_t mv = -1;  // minValues (-1: unset); Add keeps the larger
};

enum KeyClass : uint8_t { KEY_IT = 0, KEY_ZONE = 1, KEY_CT = 2, KEY_FREE = 3 };

struct Key {
  std::string name;
  Vocab vocab;
  KeyClass cls = KEY_FREE;
  bool wellknown = false;
  int slot = -1;  // IT-key index or free slot
  // instance-type / zone / capacity-type key that an existing node lacks while
  // a pod constrains it (possibly NotIn / DoesNotExist): the nodes' requirement on it
  // lives in this free slot (the node gains state there, <U> ExistingNode.Add)
  int shadow = -1;
};

using Reqs = std::map<uint32_t, KReq>;  // key id -> requirement

struct PodVariant {
  Reqs reqs;
  Reqs strict;      // PodData.StrictRequirements: no preferred term (topology podDomains)
  uint64_t tol = 0;
  std::vector<uint32_t> own;  // topology groups owned (after relaxations), ascending ids
  std::vector<std::pair<uint32_t, int32_t>> lazy_mind;  // (lazy group, this variant's minDomains for it)
};

struct Encoded {
  // vocabulary
  std::vector<Key> keys;
  std::unordered_map<std::string, uint32_t> key_id;
  uint32_t k_zone = gsd::NONE, k_ct = gsd::NONE, k_hostname = gsd::NONE, k_nodepool = gsd::NONE;
  // the topology domain key of the zone-count machinery: the zone, or the
  // capacity type when the problem's spreads use that key (dom_ct; the
  // kernels then narrow a NodeClaim's catalog capacity types, not zones)
  uint32_t k_dom = gsd::NONE;
  bool dom_ct = false, dom_np = false;
  std::vector<uint32_t> it_keys;    // key ids, IT key order
  std::vector<uint32_t> free_keys;  // key ids, free slot order
  std::vector<uint32_t> cat_zone;   // catalog zone id -> vocab id
  std::vector<uint32_t> cat_ct;
  std::vector<std::string> res_names;  // sorted
  std::vector<uint32_t> res_name_ids;  // string ids
  // sizes
  uint32_t N = 0, W = 0, R = 0, Z = 0, C = 0, T = 0, F = 0, V = 0, P = 0, K = 0, NT = 0;
  uint64_t wk_slots = 0;
  uint64_t checks = 0;
  uint64_t checks_per_pod = 0;
  // device arrays (host copies)
  std::vector<uint32_t> it_vid, it_prank, it_namerank, rank_to_it, thr_off;
  std::vector<uint16_t> it_dvid;    // [K][N] dense value ids for minValues counting
  uint32_t it_key_unique = 0;       // IT keys with a distinct value per type
  std::vector<uint32_t> it_ndv;     // [K] distinct values per IT key
  bool any_mv = false;              // some template carries minValues
  bool any_vol = false;             // pending pods mount CSI volumes and nodes exist
  std::vector<gsd::NodeVol> n_vol;  // [NN] in node order
  std::vector<uint64_t> pod_vol;    // [P][VDMAX] shared-volume bits
  std::vector<uint32_t> pod_vfresh; // [P][VDMAX] volumes only this pod mounts
  std::vector<int64_t> it_alloc, it_cap, thr_val, fk_ival;
  std::vector<uint64_t> it_pair, slot_set, thr_set, fk_isint;
  std::vector<double> prices;  // distinct offering prices ascending: price rank -> price
  std::vector<uint64_t> t_limopts;   // [T][W] template options within the NodePool limits (static matrix)
  std::vector<gsd::TmplRec> tmpl;
  std::vector<uint64_t> t_opts;
  std::vector<gsd::FK> t_fk;
  std::vector<int64_t> pod_req;
  std::vector<uint32_t> var_begin, var_count, queue0;
  std::vector<uint32_t> var_sv;  // [V] device variant -> its spec variant (index into `variants`)
  std::vector<gsd::VarRec> vars;
  std::vector<uint64_t> itmask;
  // variants with IT-key requirements, deduplicated by those requirements:
  // class c allows instance type i iff every constrained key's Has covers
  // i's value (<U> it.Requirements.Intersects on IT keys)
  std::vector<uint32_t> var_itclass;
  std::vector<uint64_t> itclass_mask;
  std::vector<gsd::FKEntry> fk_entries;
  uint32_t NN = 0;
  std::vector<uint32_t> node_order;  // device position -> gs_problem node index
  std::vector<gsd::NodeRec> nodes;
  std::vector<gsd::FK> n_fk;
  // topology groups (layout.hpp DevProblem topology fields)
  uint32_t TG = 0, TGH = 0, TGZ = 0, NZV = 0, ZS = 1;
  std::vector<gsd::TGroupRec> tgroups;
  std::vector<uint32_t> tg_list;     // own / selection list arena
  std::vector<int32_t> zcnt0;        // [TGZ][ZS]
  std::vector<int32_t> htot0;        // [TGH]
  uint32_t n_lazy = 0;               // spread groups Topology.Update creates on a relaxation (<= TGMAX)
  std::vector<uint32_t> lazy_slot;   // [n_lazy] slot | LZ_HOST for hostname groups
  std::vector<uint32_t> var_lz_off;  // [V + 1] (or [2]): CSR of the lazy groups each variant owns
  std::vector<uint32_t> lz_idx;      // their lazy indices
  std::vector<int32_t> lz_mind;      // and this variant's minDomains for each (the creator's, at the Relax)
  std::vector<uint32_t> zone_order;  // zone vocabulary ids by name
  std::vector<uint32_t> zone_cat;    // [64]
  std::vector<int32_t> hn0;          // [TGH][NN]
  // consolidation: per zone group, the counted bound pods on each node
  // [TGZ][NN] (a simulation subtracts its candidates' pods), the domains the
  // NodePools contribute, and the number of nodes per zone value
  std::vector<int32_t> zn_cnt;
  uint64_t known_np = 0;
  uint64_t zknown0 = 0;              // layout.hpp DevProblem::zknown0
  std::vector<int32_t> zone_nodes;   // [64]
  // host-only, for decode
  std::vector<Reqs> tmpl_reqs;  // incl. hostname In[omega]
  std::vector<PodVariant> variants;  // per spec variant: pods with equal specs share them (var_sv)
};

// status + message
struct Err {
  gs_status code = GS_OK;
  std::string msg;
};

// bound_alias != NONE: bound pod b is also pod bound_alias + b of the pod
// list (consolidation encodes the bound pods both as counted and as
// schedulable pods)
Err encode(const gs_problem* p, Encoded& e, uint32_t bound_alias = gsd::NONE);

// <U> v1.WellKnownLabels (+ IBM keys), v1.NormalizedLabels, strconv.Atoi
bool label_is_wellknown(const std::string& k);
std::string label_normalize(const std::string& k);
bool go_atoi64(const std::string& s, int64_t* out);

// algebra (exposed for decode)
KReq kreq_intersect(const Vocab& v, const KReq& a, const KReq& b);
void reqs_add(const Encoded& e, Reqs& r, uint32_t key, const KReq& q);
std::string canonical(const Encoded& e, const Reqs& r);

// host -> host copies of an upload image (gs_ctx::commit), split over the
// encoder's threads when large
struct HostCopy {
  const void* src;
  size_t off, bytes;
};
void host_copy_parallel(void* dst_base, const HostCopy* copies, size_t n);

}  // namespace gsh
