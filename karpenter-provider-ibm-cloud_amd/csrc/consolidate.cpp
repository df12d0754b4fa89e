// consolidate.cpp — consolidation entry points of libgpusched.so
// (gs_consolidate, gs_consolidate_rerun, gs_consolidation_choose).
//
// <U> sigs.k8s.io/karpenter@v1.13.0 pkg/controllers/disruption:
//   SimulateScheduling      every simulation is an independent Solve of the
//                           pending pods + the candidates' reschedulable pods
//                           against the state nodes minus the candidates; the
//                           device runs one workgroup per simulation
//                           (ffd_kernel<R, SIM=true>, then trunc_kernel)
//   computeConsolidation    host decision per simulation (below)
//   SingleNodeConsolidation first non-NoOp command in candidate order
//   MultiNodeConsolidation  firstNConsolidationOption's binary search, replayed
//                           over the evaluated prefixes candidates[0:mid+1]
// Reached in the reference through karpenter-core's disruption controller
// (reference cmd/controller/main.go:76-86); pricing inputs come from the
// provider's catalog (reference instancetype.go:749-773).
#include <map>
#include <numeric>
#include <set>
#include <unordered_map>

#include "ctx.hpp"

#include <cstdio>
#include <cstdlib>

namespace gsc {
namespace {

const char* kZoneKey = "topology.kubernetes.io/zone";
const char* kCtKey = "karpenter.sh/capacity-type";
const char* kItKey = "node.kubernetes.io/instance-type";

// <U> karpv1.NormalizedLabels for the keys read here
std::string norm_key(const std::string& k) {
  if (k == "failure-domain.beta.kubernetes.io/zone") return kZoneKey;
  if (k == "beta.kubernetes.io/instance-type") return kItKey;
  return k;
}

const char* str(const gs_problem* p, uint32_t id) { return id < p->n_strings && p->strings[id] ? p->strings[id] : ""; }


CandInfo candidate_info(const gs_problem* p, uint32_t node) {
  CandInfo ci;
  const gs_node& n = p->nodes[node];
  std::string zone, ct;
  bool has_zone = false, has_ct = false, has_it = false;
  for (uint32_t i = 0; i < n.labels.count; i++) {
    const gs_label& l = p->labels[n.labels.begin + i];
    const std::string k = norm_key(str(p, l.key));
    if (k == kZoneKey) {
      zone = str(p, l.value);
      has_zone = true;
    } else if (k == kCtKey) {
      ct = str(p, l.value);
      has_ct = true;
    } else if (k == kItKey) {
      ci.it_name = str(p, l.value);
      has_it = true;
    }
  }
  ci.spot = has_ct && ct == "spot";
  if (!has_it) return ci;
  for (uint32_t i = 0; i < p->n_instance_types; i++) {
    const gs_instance_type& it = p->instance_types[i];
    if (ci.it_name != str(p, it.name)) continue;
    for (uint32_t s = 0; s < it.offerings.count; s++) {
      const gs_offering& o = p->offerings[it.offerings.begin + s];
      // offering requirements are zone In[z], capacity-type In[ct] (the
      // encoder refuses anything else); well-known keys the node lacks are
      // allowed (AllowUndefinedWellKnownLabels)
      bool ok = true;
      for (uint32_t k = 0; k < o.requirements.count; k++) {
        const gs_requirement& q = p->reqs[o.requirements.begin + k];
        const std::string key = norm_key(str(p, q.key));
        const std::string val = q.values.count ? str(p, p->value_ids[q.values.begin]) : "";
        if (key == kZoneKey && has_zone && val != zone) ok = false;
        if (key == kCtKey && has_ct && val != ct) ok = false;
      }
      if (!ok) continue;
      if (!ci.priced || o.price < ci.price) {  // lo.MinBy: first minimum
        ci.price = o.price;
        ci.priced = true;
      }
    }
    break;
  }
  return ci;
}

}  // namespace

// What the decisions read from the caller's cluster, copied at
// gs_consolidate time (gs_consolidate_rerun must not touch caller memory:
// the ABI only borrows it for the duration of a call)
CandTable build_cand_table(const gs_problem* p, const uint32_t* cands, uint32_t n) {
  CandTable t;
  for (uint32_t i = 0; i < n; i++)
    if (cands[i] < p->n_nodes && !t.node.count(cands[i])) t.node.emplace(cands[i], candidate_info(p, cands[i]));
  t.it_name.reserve(p->n_instance_types);
  for (uint32_t i = 0; i < p->n_instance_types; i++) t.it_name.push_back(str(p, p->instance_types[i].name));
  // NodePool minValues: the keys and minimums, and the instance types' values of those keys
  std::set<std::string> keys;
  t.np_mv.assign(p->n_nodepools, {});
  for (uint32_t np = 0; np < p->n_nodepools; np++) {
    const gs_range r = p->nodepools[np].requirements;
    for (uint32_t k = 0; k < r.count && (uint64_t)r.begin + k < p->n_reqs; k++) {
      const gs_requirement& q = p->reqs[r.begin + k];
      if (q.min_values < 0) continue;
      t.np_mv[np].push_back({norm_key(str(p, q.key)), q.min_values});
      keys.insert(t.np_mv[np].back().first);
    }
  }
  if (!keys.empty()) {
    t.it_vals.assign(p->n_instance_types, {});
    for (uint32_t i = 0; i < p->n_instance_types; i++) {
      const gs_range r = p->instance_types[i].requirements;
      for (uint32_t k = 0; k < r.count && (uint64_t)r.begin + k < p->n_reqs; k++) {
        const gs_requirement& q = p->reqs[r.begin + k];
        const std::string key = norm_key(str(p, q.key));
        if (!keys.count(key) || q.op != GS_OP_IN) continue;
        auto& vals = t.it_vals[i][key];
        for (uint32_t v = 0; v < q.values.count && (uint64_t)q.values.begin + v < p->n_value_ids; v++)
          vals.push_back(str(p, p->value_ids[q.values.begin + v]));
      }
    }
  }
  return t;
}

// <U> InstanceTypes.SatisfiesMinValues(NodeClaim requirements) on an option
// list: the NodeClaim's minimums are its NodePool's
bool mv_satisfied(const CandTable& t, uint32_t nodepool, const uint32_t* its, size_t n) {
  if (nodepool >= t.np_mv.size()) return true;
  for (auto& km : t.np_mv[nodepool]) {
    std::set<std::string> vals;
    for (size_t i = 0; i < n; i++) {
      if (its[i] >= t.it_vals.size()) continue;
      auto f = t.it_vals[its[i]].find(km.first);
      if (f != t.it_vals[its[i]].end()) vals.insert(f->second.begin(), f->second.end());
    }
    if ((int64_t)vals.size() < km.second) return false;
  }
  return true;
}

namespace {

// the simulations a mode evaluates (candidate node indices per simulation)
gs_status build_sets(const gs_consolidation* in, SimPlan& sp, std::string* err) {
  sp.sets.clear();
  sp.multi_max = 0;
  const uint32_t n = in->n_candidates;
  if (in->mode == GS_CONSOLIDATE_EVAL) {
    for (uint32_t s = 0; s < in->n_sets; s++) {
      const gs_range r = in->sets[s];
      if ((uint64_t)r.begin + r.count > n) {
        *err = "candidate set out of range";
        return GS_E_INVALID;
      }
      sp.sets.emplace_back(in->candidates + r.begin, in->candidates + r.begin + r.count);
    }
  } else if (in->mode == GS_CONSOLIDATE_SINGLE) {
    for (uint32_t i = 0; i < n; i++) sp.sets.push_back({in->candidates[i]});
  } else if (in->mode == GS_CONSOLIDATE_MULTI) {
    // maxParallel := lo.Clamp(len(candidates), 0, 100); if len <= max { max = len - 1 }
    const uint32_t cap = in->max_candidates ? in->max_candidates : 100;
    uint32_t mx = std::min(n, cap);
    if (n >= 2) {
      if (n <= mx) mx = n - 1;
      for (uint32_t mid = 1; mid <= mx; mid++) sp.sets.emplace_back(in->candidates, in->candidates + mid + 1);
      sp.multi_max = mx;
    }
  } else {
    *err = "unknown consolidation mode";
    return GS_E_INVALID;
  }
  return GS_OK;
}

uint64_t grid_of(uint64_t zm, uint64_t cm, uint32_t Z, uint32_t C) {
  const uint64_t cmask = C >= 64 ? ~0ull : ((1ull << C) - 1);
  uint64_t g = 0;
  for (uint32_t z = 0; z < Z; z++)
    if ((zm >> z) & 1) g |= (cm & cmask) << (z * C);
  return g;
}

// <U> filterOutSameInstanceType: indices of the options that survive
std::vector<uint32_t> filter_out_same_type(const CandTable& t, const std::vector<uint32_t>& cands,
                                           const uint32_t* opts, const double* prices, uint32_t n) {
  std::set<std::string> existing;
  std::map<std::string, double> price_by_type;
  for (uint32_t c : cands) {
    const CandInfo& ci = t.node.at(c);
    existing.insert(ci.it_name);
    if (!ci.priced) continue;
    auto f = price_by_type.find(ci.it_name);
    const double ex = f == price_by_type.end() ? __DBL_MAX__ : f->second;
    if (ci.price < ex) price_by_type[ci.it_name] = ci.price;
  }
  double max_price = __DBL_MAX__;
  for (uint32_t i = 0; i < n; i++) {
    const std::string& nm = t.it_name[opts[i]];
    if (!existing.count(nm)) continue;
    auto f = price_by_type.find(nm);
    const double pr = f == price_by_type.end() ? 0.0 : f->second;  // Go map zero value
    if (pr < max_price) max_price = pr;
  }
  std::vector<uint32_t> out;
  for (uint32_t i = 0; i < n; i++)
    if (prices[i] < max_price) out.push_back(i);  // filterByPrice
  return out;
}

// policy replay over a complete command table
int32_t choose(const CandTable& t, uint32_t mode, const std::vector<std::vector<uint32_t>>& sets, uint32_t multi_max,
               const gs_command* cmds, const uint32_t* opts, const double* prices, std::vector<uint32_t>* multi_opts) {
  multi_opts->clear();
  if (mode == GS_CONSOLIDATE_SINGLE) {
    for (size_t i = 0; i < sets.size(); i++)
      if (cmds[i].decision == GS_DECISION_DELETE || cmds[i].decision == GS_DECISION_REPLACE) return (int32_t)i;
    return -1;
  }
  if (mode != GS_CONSOLIDATE_MULTI || sets.empty()) return -1;
  int32_t chosen = -1;
  int lo = 1, hi = (int)multi_max;
  while (lo <= hi) {
    const int mid = (lo + hi) / 2;
    const gs_command& c = cmds[mid - 1];
    bool valid = false;
    std::vector<uint32_t> keep;
    if (c.decision == GS_DECISION_REPLACE) {
      for (uint32_t i : filter_out_same_type(t, sets[mid - 1], opts + c.options.begin, prices + c.options.begin,
                                             c.options.count))
        keep.push_back(opts[c.options.begin + i]);
      // filterOutSameInstanceType ends in RemoveInstanceTypeOptionsByPriceAndMinValues
      valid = !keep.empty() && mv_satisfied(t, c.nodepool, keep.data(), keep.size());
    }
    if (valid || c.decision == GS_DECISION_DELETE) {
      chosen = mid - 1;
      *multi_opts = keep;
      lo = mid + 1;
    } else {
      hi = mid - 1;
    }
  }
  return chosen;
}

// pods of each evaluated simulation in queue order, node positions removed
gs_status plan_sims(gs_ctx* c, const gs_consolidation* in, std::string* err) {
  SimPlan& sp = c->sims;
  const gsh::Encoded& e = c->enc;
  gs_status st = build_sets(in, sp, err);
  if (st != GS_OK) return st;
  sp.evaluated.clear();
  const uint32_t sc = in->shard_count;
  for (uint32_t s = 0; s < sp.sets.size(); s++)
    if (sc == 0 || s % sc == in->shard_index) sp.evaluated.push_back(s);
  std::vector<uint32_t> rank(e.P), pos_of(e.NN);
  for (uint32_t i = 0; i < e.P; i++) rank[e.queue0[i]] = i;
  for (uint32_t i = 0; i < e.NN; i++) pos_of[e.node_order[i]] = i;
  const uint32_t np = c->n_pending;
  std::vector<uint32_t> pend(np);
  std::iota(pend.begin(), pend.end(), 0);
  std::sort(pend.begin(), pend.end(), [&](uint32_t a, uint32_t b) { return rank[a] < rank[b]; });
  std::vector<std::vector<uint32_t>> bound_by_node(e.NN);
  const gs_problem* cl = in->cluster;
  for (uint32_t b = 0; b < cl->n_bound_pods; b++) bound_by_node[cl->bound_pod_node[b]].push_back(np + b);
  sp.pod_off.assign(1, 0);
  sp.pods.clear();
  sp.cand_off.assign(1, 0);
  sp.cands.clear();
  sp.known.clear();
  sp.max_pods = 0;
  sp.ov_cap = 0;
  std::vector<uint32_t> mine, merged;
  std::vector<int32_t> zn(64);
  for (uint32_t s : sp.evaluated) {
    mine.clear();
    for (uint32_t n : sp.sets[s]) {
      mine.insert(mine.end(), bound_by_node[n].begin(), bound_by_node[n].end());
      sp.cands.push_back(pos_of[n]);
    }
    if (e.TGZ) {
      // <U> NewTopology over the state nodes the simulation keeps: the
      // NodePools' zones plus the zones of the remaining nodes
      std::copy(e.zone_nodes.begin(), e.zone_nodes.end(), zn.begin());
      for (uint32_t n : sp.sets[s]) {
        const uint32_t z = e.nodes[pos_of[n]].dvid;
        if (z < 64) zn[z]--;
      }
      uint64_t k = e.known_np;
      for (uint32_t z = 0; z < 64; z++)
        if (zn[z] > 0) k |= 1ull << z;
      sp.known.push_back(k);
    }
    std::sort(mine.begin(), mine.end(), [&](uint32_t a, uint32_t b) { return rank[a] < rank[b]; });
    merged.resize(pend.size() + mine.size());
    std::merge(pend.begin(), pend.end(), mine.begin(), mine.end(), merged.begin(),
               [&](uint32_t a, uint32_t b) { return rank[a] < rank[b]; });
    sp.pods.insert(sp.pods.end(), merged.begin(), merged.end());
    sp.pod_off.push_back((uint32_t)sp.pods.size());
    sp.cand_off.push_back((uint32_t)sp.cands.size());
    sp.max_pods = std::max<uint32_t>(sp.max_pods, (uint32_t)merged.size());
    sp.ov_cap = std::max<uint32_t>(sp.ov_cap, (uint32_t)(merged.size() + sp.sets[s].size()));
  }
  if (sp.evaluated.size() >= (1u << 20) - 1u) {
    *err = "more than 1,048,574 simulations in one call";
    return GS_E_CAPACITY;
  }
  if (sp.max_pods > 0xFFFFu) {
    *err = "a simulation holds more than 65535 pods";
    return GS_E_CAPACITY;
  }
  const uint32_t lds = gsk_ffd_lds_bytes(std::max<uint32_t>(sp.max_pods, 1), (uint32_t)e.thr_val.size(),
                                         (e.NN + 31) / 32, gsd::topo_lds_bytes(e.TGZ, e.ZS, e.TGH, e.n_lazy)) +
                       8u * gsd::ovh_slots_for(sp.ov_cap);
  if (lds > gsk_ffd_dyn_lds_max()) {
    *err = "simulation exceeds the workgroup LDS (pods per simulation or state nodes)";
    return GS_E_CAPACITY;
  }
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device);
  // persistent workgroups draining the simulation counter: as many as stay
  // resident (occupancy of the simulation kernel at this LDS size)
  // many simulations: the narrow workgroup (throughput); few: the wide one
  // (each simulation's latency) -- ffd.hip FB_SIM / FB_SIM_NARROW
  sp.nt = sp.evaluated.size() >= 4 * (size_t)std::max(cus, 1) ? 128u : 256u;
  const bool general = e.TG || e.any_mv || e.any_vol;
  uint32_t per_cu = gsk_ffd_sim_blocks_per_cu(e.R, lds, sp.nt, general ? 1u : 0u);
  // the simulations' queue arrays and add logs in LDS when that costs no
  // resident workgroup (ffd.hip s_simq / s_simlog)
  const uint32_t lds_q = lds + 32u * std::max<uint32_t>(sp.max_pods, 1);
  sp.sim_lds = false;
  if (lds_q <= gsk_ffd_dyn_lds_max() && gsk_ffd_sim_blocks_per_cu(e.R, lds_q, sp.nt, general ? 1u : 0u) >= per_cu) {
    sp.sim_lds = true;
  }
  if (const char* x = std::getenv("GS_SIM_LDS"))  // A/B experiments: 0 off, 1 on whenever it fits
    sp.sim_lds = std::atoi(x) != 0 && lds_q <= gsk_ffd_dyn_lds_max();
  if (std::getenv("GS_SIM_DEBUG"))
    std::fprintf(stderr, "gpusched sim plan: sims %zu max_pods %u nt %u lds %u per_cu %u lds_q per_cu %u sim_lds %d\n",
                 sp.evaluated.size(), sp.max_pods, sp.nt, lds, per_cu,
                 gsk_ffd_sim_blocks_per_cu(e.R, lds_q, sp.nt, general ? 1u : 0u), (int)sp.sim_lds);
  if (const char* x = std::getenv("GS_SIM_PER_CU"))  // experiments: fewer persistent workgroups per CU
    per_cu = std::max<uint32_t>(1, std::min<uint32_t>(per_cu, (uint32_t)std::atoi(x)));
  sp.blocks = (uint32_t)std::min<size_t>(sp.evaluated.size(), (size_t)std::max(cus, 1) * per_cu);
  // per-block overlays of hostname counts: at most 1 GiB (fewer persistent blocks otherwise)
  const size_t ov_row = (size_t)std::max<uint32_t>(sp.ov_cap, 1) * e.TGH * sizeof(uint64_t);
  if (ov_row) sp.blocks = (uint32_t)std::max<size_t>(1, std::min<size_t>(sp.blocks, (size_t)(1u << 30) / ov_row));
  return GS_OK;
}

// launch the device part and decide every evaluated simulation
// A simulation clears the NodeClaim hostname-count cells it recorded at its
// own end (ffd.hip: the rows stay zero at rest).  A launch that failed, or a
// simulation that stopped early, may leave cells set: clear the rows so a
// gs_consolidate_rerun on this upload starts from zero, or, when even that
// fails, require a fresh gs_consolidate.
void reset_sim_counts(gs_ctx* c) {
  if (!c->hc_bytes || !c->dp.hc) return;
  if (hipMemsetAsync(c->dp.hc, 0, c->hc_bytes, c->stream) != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess)
    c->cons_ready = false;
}

gs_status run_and_decide(gs_ctx* c, gs_consolidation_result* out) {
  const gsh::Encoded& e = c->enc;
  const SimPlan& sp = c->sims;
  const gs_consolidation* in = &c->cons_in;
  auto& d = c->dp;
  const size_t NS = sp.evaluated.size();
  const gsd::SimCtrl* ctrl = c->h_ctrl;
  const gsd::ClaimRec* hdr = c->h_hdr;
  const uint32_t* its = c->h_its;
  const uint32_t* nits = c->h_nits;
  float a = 0, b = 0, x = 0;
  try {
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipEventRecord(c->ev[0], c->stream));
    HIPCHK(gsk_feas(&d, 0, 0, ~0u, c->stream));
    HIPCHK(hipEventRecord(c->ev[1], c->stream));
    if (NS) {
      HIPCHK(hipMemsetAsync(d.sim_next, 0, sizeof(uint32_t), c->stream));
      // a fresh overlay stamp prefix per launch; cells of 4,095 launches ago
      // could match again, so the cells are cleared when the prefix wraps
      d.ov_epoch = (d.ov_epoch + 1u) & 0xFFFu;
      if (!d.ov_epoch) {
        if (c->ov_hn_bytes) HIPCHK(hipMemsetAsync(d.ov_hn, 0, c->ov_hn_bytes, c->stream));
        d.ov_epoch = 1;
      }
      HIPCHK(gsk_ffd(&d, sp.blocks, c->stream));
    }
    HIPCHK(hipEventRecord(c->ev[2], c->stream));
    if (NS) HIPCHK(gsk_trunc(&d, trunc_lds_bytes(d.N), (uint32_t)sp.pods.size(), c->stream));
    HIPCHK(hipEventRecord(c->ev[3], c->stream));
    HIPCHK(hipEventSynchronize(c->ev[3]));
    HIPCHK(hipEventElapsedTime(&a, c->ev[0], c->ev[1]));
    HIPCHK(hipEventElapsedTime(&b, c->ev[1], c->ev[2]));
    HIPCHK(hipEventElapsedTime(&x, c->ev[2], c->ev[3]));
  } catch (const HipError& ex) {
    reset_sim_counts(c);
    return fail(c, GS_E_HIP, ex.msg);
  }
  c->t_feas = a;
  c->t_sim = b;
  c->t_trunc = x;
  auto t0 = Clock::now();
  try {
    if (NS) {
      // per simulation: control block (NodeClaim count, failed pods), the
      // single NodeClaim's header and its OrderByPrice/Truncate(60) list
      HIPCHK(hipMemcpyAsync(c->h_ctrl, d.sim_ctrl, NS * sizeof(gsd::SimCtrl), hipMemcpyDeviceToHost, c->stream));
      c->h_blk.resize(sp.blocks);
      HIPCHK(hipMemcpyAsync(c->h_blk.data(), d.sim_blk, sp.blocks * sizeof(gsd::Ctrl), hipMemcpyDeviceToHost,
                            c->stream));
      HIPCHK(hipMemcpyAsync(c->h_hdr, d.sim_hdr, NS * sizeof(gsd::ClaimRec), hipMemcpyDeviceToHost, c->stream));
      HIPCHK(hipMemcpyAsync(c->h_its, d.c_its, NS * 60 * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
      HIPCHK(hipMemcpyAsync(c->h_nits, d.c_nits, NS * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
      HIPCHK(hipStreamSynchronize(c->stream));
    }
  } catch (const HipError& ex) {
    return fail(c, GS_E_HIP, ex.msg);
  }
  c->commands.assign(sp.sets.size(), gs_command{});
  c->cmd_options.clear();
  c->cmd_prices.clear();
  for (size_t s = 0; s < sp.sets.size(); s++) {
    c->commands[s].decision = GS_DECISION_SKIPPED;
    c->commands[s].n_candidates = (uint32_t)sp.sets[s].size();
  }
  uint64_t checks = 0, node_evals = 0, pops = 0, node_prefix = 0;
  if (NS)
    for (const gsd::Ctrl& b : c->h_blk) {
      node_evals += b.node_evals;
      node_prefix += b.node_prefix;
      pops += b.pops;
    }
  for (size_t k = 0; k < NS; k++) {
    const uint32_t s = sp.evaluated[k];
    const gsd::SimCtrl& ct = ctrl[k];
    if (ct.status != 0) reset_sim_counts(c);
    if (ct.status == gsd::ST_POD_COUNT)
      return fail(c, GS_E_CAPACITY, "a simulated NodeClaim would hold more than 65535 pods (16-bit pod count)");
    if (ct.status != 0) return fail(c, GS_E_HIP, "simulation kernel reported an internal error");
    const uint32_t q0 = sp.pod_off[k], P = sp.pod_off[k + 1] - q0;
    checks += (uint64_t)P * (e.NN - sp.sets[s].size() + e.checks_per_pod);
    gs_command& cmd = c->commands[s];
    cmd.decision = GS_DECISION_NOOP;
    cmd.n_new_claims = ct.n_claims;
    // !AllNonPendingPodsScheduled: unplaced non-pending pods, and non-pending
    // pods placed on uninitialized nodes (SimulateScheduling; counted on device)
    const uint32_t failed = ct.failed;
    cmd.n_failed_pods = failed;
    if (failed) {
      cmd.reason = GS_NOOP_UNSCHEDULABLE;
      continue;
    }
    if (ct.n_claims == 0) {
      cmd.decision = GS_DECISION_DELETE;
      continue;
    }
    if (ct.n_claims > 1) {
      cmd.reason = GS_NOOP_MULTIPLE_CLAIMS;
      continue;
    }
    double cp = 0;
    bool all_spot = true, priced = true;
    for (uint32_t n : sp.sets[s]) {
      const CandInfo& ci = c->cand_table.node.at(n);
      priced = priced && ci.priced;
      cp += ci.price;
      all_spot = all_spot && ci.spot;
    }
    if (!priced) {
      cmd.reason = GS_NOOP_PRICE_UNKNOWN;
      continue;
    }
    cmd.candidate_price = cp;
    // the NodeClaim's capacity-type requirement: template AND every added pod
    const gsd::ClaimRec& h = hdr[k];
    bool has_spot = (h.ctb & gsd::CT_SPOT) != 0;
    bool has_od = (h.ctb & gsd::CT_OD) != 0;
    if (e.dom_ct && !(h.zflags & gsd::ZF_COMP)) {
      // capacity-type topology domains: the In set after the spreads'
      // narrowing is the claim's domain Has (as the decoder writes it)
      const auto& v = e.keys[e.k_ct].vocab;
      auto in = [&](const char* x) {
        auto g = v.id.find(x);
        const uint32_t id = g == v.id.end() ? v.omega : g->second;
        return id < 64 && ((h.zfull >> id) & 1);
      };
      has_spot = has_spot && in("spot");
      has_od = has_od && in("on-demand");
    }
    if (all_spot && has_spot) {  // SpotToSpotConsolidation disabled
      cmd.reason = GS_NOOP_SPOT_TO_SPOT;
      continue;
    }
    // RemoveInstanceTypeOptionsByPriceAndMinValues over the OrderByPrice list
    // (the price filter, then SatisfiesMinValues on what is left)
    const uint64_t G = grid_of(h.zm, h.cm, e.Z, e.C);
    const uint32_t ob = (uint32_t)c->cmd_options.size();
    for (uint32_t i = 0; i < nits[k]; i++) {
      const uint32_t it = its[k * 60 + i];
      uint32_t minp = gsd::NONE;
      uint64_t m = e.it_pair[it] & G;
      while (m) {
        const uint32_t g = (uint32_t)__builtin_ctzll(m);
        m &= m - 1;
        minp = std::min(minp, e.it_prank[(size_t)it * 64 + g]);
      }
      const double pr = minp == gsd::NONE ? __DBL_MAX__ : e.prices[minp];
      if (pr < cp) {
        c->cmd_options.push_back(it);
        c->cmd_prices.push_back(pr);
      }
    }
    const uint32_t n_opt = (uint32_t)c->cmd_options.size() - ob;
    const uint32_t np = e.tmpl[h.tmpl].np_index;
    if (e.tmpl[h.tmpl].mv_mask && !mv_satisfied(c->cand_table, np, c->cmd_options.data() + ob, n_opt)) {
      c->cmd_options.resize(ob);
      c->cmd_prices.resize(ob);
      cmd.reason = GS_NOOP_MIN_VALUES;
      continue;
    }
    if (n_opt == 0) {
      cmd.reason = GS_NOOP_NOT_CHEAPER;
      continue;
    }
    cmd.decision = GS_DECISION_REPLACE;
    cmd.nodepool = np;
    cmd.spot_only = has_spot && has_od ? 1u : 0u;
    cmd.options = gs_range{ob, n_opt};
  }
  int32_t chosen = -1;
  c->multi_opts.clear();
  if (NS == sp.sets.size())
    chosen = choose(c->cand_table, in->mode, sp.sets, sp.multi_max, c->commands.data(), c->cmd_options.data(),
                    c->cmd_prices.data(), &c->multi_opts);
  c->t_fetch = ms_since(t0);
  std::memset(out, 0, sizeof(*out));
  out->n_commands = (uint32_t)c->commands.size();
  out->commands = c->commands.data();
  out->options = c->cmd_options.data();
  out->option_prices = c->cmd_prices.data();
  out->chosen = chosen;
  out->n_multi_options = (uint32_t)c->multi_opts.size();
  out->multi_options = c->multi_opts.data();
  out->pods_simulated = (uint32_t)sp.pods.size();
  out->checks = checks;
  out->node_evals = node_evals;
  out->node_prefix = node_prefix;
  out->pops = pops;
  out->t_encode_ms = c->t_encode;
  out->t_upload_ms = c->t_upload;
  out->t_feas_ms = c->t_feas;
  out->t_sim_ms = c->t_sim;
  out->t_truncate_ms = c->t_trunc;
  out->t_fetch_ms = c->t_fetch;
  return GS_OK;
}

gs_status check_input(const gs_consolidation* in, std::string* err) {
  if (!in || !in->cluster) {
    *err = "null input";
    return GS_E_INVALID;
  }
  const gs_problem* p = in->cluster;
  for (uint32_t i = 0; i < in->n_candidates; i++)
    if (in->candidates[i] >= p->n_nodes) {
      *err = "candidate node index out of range";
      return GS_E_INVALID;
    }
  if (p->n_bound_pods && !p->bound_pod_node) {
    *err = "bound pods without their nodes";
    return GS_E_INVALID;
  }
  for (uint32_t i = 0; i < p->n_bound_pods; i++)
    if (p->bound_pod_node[i] >= p->n_nodes) {
      *err = "bound pod node index out of range";
      return GS_E_INVALID;
    }
  if (in->shard_count && in->shard_index >= in->shard_count) {
    *err = "shard index out of range";
    return GS_E_INVALID;
  }
  return GS_OK;
}

}  // namespace

// the host policy replay over a complete command table (gs_consolidation_choose
// and the sharded context's merge)
int32_t choose_commands(const CandTable& t, const gs_consolidation* in, const gs_command* commands,
                        const uint32_t* options, const double* prices, std::vector<uint32_t>* multi) {
  SimPlan sp;
  std::string err;
  if (build_sets(in, sp, &err) != GS_OK) return -1;
  return choose(t, in->mode, sp.sets, sp.multi_max, commands, options, prices, multi);
}
}  // namespace gsc

using namespace gsc;

extern "C" {

gs_status gs_consolidate(gs_ctx* c, const gs_consolidation* in, gs_consolidation_result* out) {
  if (!c || !out) return GS_E_INVALID;
  std::string err;
  gs_status st = check_input(in, &err);
  if (st != GS_OK) return fail(c, st, err);
  if (!c->shards.empty()) return sharded_consolidate(c, in, out);
  c->prepared = c->ran = false;
  // own copies of the caller's candidate arrays (gs_consolidate_rerun)
  c->cons_cands.assign(in->candidates, in->candidates + in->n_candidates);
  c->cons_sets.assign(in->sets, in->sets + (in->mode == GS_CONSOLIDATE_EVAL ? in->n_sets : 0));
  c->cons_in = *in;
  c->cons_in.candidates = c->cons_cands.data();
  c->cons_in.sets = c->cons_sets.data();
  c->cand_table = build_cand_table(in->cluster, in->candidates, in->n_candidates);
  // the combined pod list: pending pods, then every bound pod
  const gs_problem* cl = in->cluster;
  c->n_pending = cl->n_pods;
  c->cons_pods.assign(cl->pods, cl->pods + cl->n_pods);
  c->cons_pods.insert(c->cons_pods.end(), cl->bound_pods, cl->bound_pods + cl->n_bound_pods);
  // every bound pod is in the combined pod list (a simulation reschedules the
  // candidates' pods) and stays a bound pod (the topology counts, host ports
  // and volumes of the nodes a simulation keeps): bound pod b is pod n_pending + b
  c->cons_problem = *cl;
  c->cons_problem.pods = c->cons_pods.data();
  c->cons_problem.n_pods = (uint32_t)c->cons_pods.size();
  c->n_nodepools = c->cons_problem.n_nodepools;
  auto t0 = Clock::now();
  gsh::Err er = gsh::encode(&c->cons_problem, c->enc, c->n_pending);
  c->t_encode = ms_since(t0);
  if (er.code != GS_OK) return fail(c, er.code, er.msg);
  er = capacity_check(c->enc);
  if (er.code != GS_OK) return fail(c, er.code, er.msg);
  st = plan_sims(c, &c->cons_in, &err);
  if (st != GS_OK) return fail(c, st, err);
  try {
    HIPCHK(hipSetDevice(c->device));
    auto t1 = Clock::now();
    upload_problem(c, &c->sims);
    c->t_upload = ms_since(t1);
  } catch (const HipError& ex) {
    return fail(c, GS_E_HIP, ex.msg);
  }
  c->cons_ready = true;
  return run_and_decide(c, out);
}

gs_status gs_consolidate_rerun(gs_ctx* c, gs_consolidation_result* out) {
  if (!c || !out || !c->cons_ready) return GS_E_INVALID;
  if (!c->shards.empty()) return sharded_consolidate(c, nullptr, out);
  return run_and_decide(c, out);
}

gs_status gs_consolidation_choose(const gs_consolidation* in, const gs_command* commands, uint32_t n_commands,
                                  const uint32_t* options, const double* option_prices, int32_t* chosen,
                                  uint32_t* multi_options, uint32_t* n_multi_options) {
  std::string err;
  if (!chosen || check_input(in, &err) != GS_OK) return GS_E_INVALID;
  SimPlan sp;
  if (build_sets(in, sp, &err) != GS_OK) return GS_E_INVALID;
  if (n_commands != sp.sets.size()) return GS_E_INVALID;
  for (uint32_t s = 0; s < n_commands; s++)
    if (commands[s].decision == GS_DECISION_SKIPPED) return GS_E_INVALID;
  std::vector<uint32_t> mo;
  const CandTable t = build_cand_table(in->cluster, in->candidates, in->n_candidates);
  *chosen = choose(t, in->mode, sp.sets, sp.multi_max, commands, options, option_prices, &mo);
  if (multi_options && n_multi_options) {
    const uint32_t n = (uint32_t)std::min<size_t>(mo.size(), 60);
    std::copy(mo.begin(), mo.begin() + n, multi_options);
    *n_multi_options = n;
  }
  return GS_OK;
}

}  // extern "C"
