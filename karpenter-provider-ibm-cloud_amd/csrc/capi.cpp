// capi.cpp — C-ABI of libgpusched.so (include/gpusched.h): context, HBM
// buffers, kernel launches on one HIP stream, result decode.
#include "ctx.hpp"

#include <set>

namespace gsc {

gs_status fail(gs_ctx* c, gs_status s, const std::string& m) {
  c->err = m;
  return s;
}

void upload_problem(gs_ctx* c, const SimPlan* sims) {
  auto& e = c->enc;
  auto& d = c->dp;
  c->plan.clear();
  c->plan_bytes = 0;
  c->free_all();
  std::memset(&d, 0, sizeof d);
  d.N = e.N;
  d.W = e.W;
  d.R = e.R;
  d.Z = e.Z;
  d.C = e.C;
  d.T = e.T;
  d.F = e.F;
  d.V = e.V;
  d.P = e.P;
  d.K = e.K;
  d.NT = e.NT;
  d.wk_slots = e.wk_slots;
  d.RQ = std::min<uint32_t>(e.R, 4);
  d.n_thr = (uint32_t)e.thr_val.size();
  if (sims) {
    d.max_claims = std::max<uint32_t>(sims->max_pods, 1);
  } else {
    // NodeClaims the LDS holds next to the thresholds, topology state and
    // (single-wave kernel) the existing nodes' slack codes
    // (the block kernel's capacity; the single-wave kernel's is smaller by the
    // node codes -- a Solve that outgrows it reruns on the block kernel)
    const uint32_t other = gsk_ffd_lds_bytes(0, (uint32_t)e.thr_val.size(), 0, gsd::topo_lds_bytes(e.TGZ, e.ZS, e.TGH, e.n_lazy)) + 8;
    const uint32_t dyn = std::min(gsk_ffd_dyn_lds_max(), gsk_ffdw_dyn_lds_max());
    auto claims_fit = [&](uint32_t extra) {
      const uint32_t fit = dyn > other + extra ? (dyn - other - extra) / 23 : 0;
      return std::min<uint32_t>(std::min<uint32_t>(std::max<uint32_t>(e.P, 1), kMaxClaimsLds), fit);
    };
    d.max_claims = claims_fit(0);
    if (!d.max_claims) throw HipError{"topology / threshold state leaves no LDS for NodeClaims"};
    const bool wave_ok = !(c->cfg_flags & GS_CFG_BLOCK_SOLVE) && e.NN <= kWaveSolveMaxNodes;
    d.max_claims_wave = wave_ok ? claims_fit(gsd::wave_node_lds_bytes(e.NN)) : 0u;
    c->wave = d.max_claims_wave > 0;
  }
  c->upload(d.it_vid, e.it_vid);
  c->upload(d.it_dvid, e.it_dvid);
  d.it_key_unique = e.it_key_unique;
  d.any_mv = e.any_mv ? 1u : 0u;
  d.any_vol = e.any_vol ? 1u : 0u;
  c->upload(d.n_vol0, e.n_vol);
  c->alloc(d.n_vol, e.n_vol.size());
  c->upload(d.pod_vol, e.pod_vol);
  c->upload(d.pod_vfresh, e.pod_vfresh);
  c->upload(d.it_alloc, e.it_alloc);
  c->upload(d.it_cap, e.it_cap);
  c->upload(d.it_pair, e.it_pair);
  c->upload(d.it_prank, e.it_prank);
  c->upload(d.it_namerank, e.it_namerank);
  c->upload(d.rank_to_it, e.rank_to_it);
  c->upload(d.slot_set, e.slot_set);
  {
    std::vector<int64_t> tv = e.thr_val;  // 4 sentinels: the device reads a 4-wide window past each range
    tv.insert(tv.end(), 4, INT64_MAX);
    c->upload(d.thr_val, std::move(tv));
  }
  c->upload(d.thr_off, e.thr_off);
  {
    // threshold rows re-strided to OW words (16-B aligned rows for the scan)
    const uint32_t OW = std::max<uint32_t>(4, (e.W + 3) & ~3u);
    const size_t nrows = e.W ? e.thr_set.size() / e.W : 0;
    std::vector<uint64_t> ts(std::max<size_t>(nrows, 1) * OW, 0);
    for (size_t q = 0; q < nrows; q++)
      std::copy(e.thr_set.begin() + q * e.W, e.thr_set.begin() + (q + 1) * e.W, ts.begin() + q * OW);
    c->upload(d.thr_set, std::move(ts));
  }
  c->upload(d.fk_ival, e.fk_ival);
  c->upload(d.fk_isint, e.fk_isint);
  c->upload(d.tmpl, e.tmpl);
  c->upload(d.t_opts, e.t_opts);
  c->upload(d.t_limopts, e.t_limopts);
  c->upload(d.t_fk, e.t_fk);
  c->upload(d.pod_req, e.pod_req);
  c->upload(d.var_begin, e.var_begin);
  c->upload(d.var_count, e.var_count);
  c->upload(d.vars, e.vars);
  c->upload(d.itmask, e.itmask);
  c->upload(d.var_itclass, e.var_itclass);
  {
    std::vector<uint32_t> vp(std::max<uint32_t>(e.V, 1), 0);
    for (uint32_t v = 0; v < e.V; v++) vp[v] = e.vars[v].pod;
    c->upload(d.var_pod, std::move(vp));
  }
  c->upload(d.itclass_mask, e.itclass_mask);
  c->upload(d.fk_entries, e.fk_entries);
  c->upload(d.queue0, e.queue0);
  if (!sims) {
    // the first pass over the queue pops pods in queue0 order with their first
    // variant: records laid out in that order let the kernel prefetch the next
    // pod in one round trip (gathered on the device after the upload)
    c->alloc(d.qvars, std::max<uint32_t>(e.P, 1));
    c->alloc(d.qreqs, (size_t)std::max<uint32_t>(e.P, 1) * std::max<uint32_t>(e.R, 1));
    c->alloc(d.qcodes, (size_t)std::max<uint32_t>(e.P, 1) * 4);
    c->alloc(d.qrun, std::max<uint32_t>(e.P, 1));
  }
  d.NN = e.NN;
  // topology spread groups
  d.TG = e.TG;
  d.TGH = e.TGH;
  d.TGZ = e.TGZ;
  d.ZS = e.ZS;
  d.NZV = e.NZV;
  d.dom_ct = e.dom_ct ? 1u : 0u;
  d.dom_np = e.dom_np ? 1u : 0u;
  d.zknown0 = e.zknown0;
  c->upload(d.tgroups, e.tgroups);
  c->upload(d.tg_list, e.tg_list);
  d.n_lazy = e.n_lazy;
  c->upload(d.lazy_slot, e.lazy_slot);
  c->upload(d.var_lz_off, e.var_lz_off);
  c->upload(d.lz_idx, e.lz_idx);
  c->upload(d.lz_mind, e.lz_mind);
  c->upload(d.zcnt0, e.zcnt0);
  c->upload(d.htot0, e.htot0);
  c->upload(d.zone_order, e.zone_order);
  c->upload(d.zone_cat, e.zone_cat);
  c->upload(d.hn0, e.hn0);
  if (sims && (e.TGH || e.TGZ) && e.NN) {
    // each node's nonzero counts, node-major sparse: a simulation excludes its
    // candidates' pods by reading their few entries (the dense
    // node row was ~TGH x 4 B per simulation on the e2e shape)
    std::vector<uint32_t> off(e.NN + 1, 0);
    for (uint32_t g = 0; g < e.TGZ; g++)
      for (uint32_t n = 0; n < e.NN; n++) off[n + 1] += e.zn_cnt[(size_t)g * e.NN + n] != 0;
    for (uint32_t g = 0; g < e.TGH; g++)
      for (uint32_t n = 0; n < e.NN; n++) off[n + 1] += e.hn0[(size_t)g * e.NN + n] != 0;
    for (uint32_t n = 0; n < e.NN; n++) off[n + 1] += off[n];
    std::vector<uint64_t> sp(std::max<uint32_t>(off[e.NN], 1));
    std::vector<uint32_t> fill(off.begin(), off.end() - 1);
    auto put = [&](uint32_t g, int32_t c, uint32_t n) { sp[fill[n]++] = (uint64_t)g << 32 | (uint32_t)c; };
    for (uint32_t g = 0; g < e.TGZ; g++)
      for (uint32_t n = 0; n < e.NN; n++)
        if (int32_t c = e.zn_cnt[(size_t)g * e.NN + n]) put(g, c, n);
    for (uint32_t g = 0; g < e.TGH; g++)
      for (uint32_t n = 0; n < e.NN; n++)
        if (int32_t c = e.hn0[(size_t)g * e.NN + n]) put(e.TGZ + g, c, n);
    c->upload(d.nsp_off, std::move(off));
    c->upload(d.nsp, std::move(sp));
  } else {
    d.nsp_off = nullptr;
    d.nsp = nullptr;
  }
  c->alloc(d.hn, e.hn0.size());
  c->upload(d.nodes0, e.nodes);
  c->upload(d.n_fk0, e.n_fk);
  // the provisioning Solve works on a global copy of the nodes; simulations
  // share nodes0 read-only and keep per-block overlays
  c->alloc(d.nodes, sims ? 1 : std::max<uint32_t>(e.NN, 1));
  c->alloc(d.n_fk, sims ? 1 : e.n_fk.size());
  const size_t VT = (size_t)e.V * e.T, F1 = std::max<uint32_t>(e.F, 1), R1 = std::max<uint32_t>(e.R, 1);
  // pod arenas (queue, log) and claim arenas: the whole problem, or the sum
  // over simulations (a simulation opens at most one NodeClaim per pod)
  const size_t PA = sims ? sims->pods.size() : e.P;
  const size_t CA = sims ? sims->pods.size() : d.max_claims;
  const size_t NS = sims ? sims->evaluated.size() : 0;
  d.claim_cap = (uint32_t)CA;
  c->ch = false;
  d.OW = std::max<uint32_t>(4, (e.W + 3) & ~3u);
  c->alloc(d.rows, VT * d.OW);
  c->alloc(d.cheapest, VT);
  c->alloc(d.cheapest_key, VT);
  c->alloc(d.nfo, VT);
  c->alloc(d.fk_ok, VT);
  c->alloc(d.pair_cur, VT * R1);
  c->alloc(d.queue, PA);
  c->alloc(d.last_len, PA);
  c->alloc(d.last_epoch, PA);
  c->alloc(d.cur_var, PA);
  c->alloc(d.c_rec, CA);
  c->alloc(d.c_opts, CA * d.OW);
  c->alloc(d.c_fk, CA * F1);
  c->alloc(d.t_rem, (sims ? NS : 1) * e.T * R1);
  c->alloc(d.log, PA);
  c->alloc(d.c_sorted, sims ? 1 : CA);
  c->alloc(d.ctrl, 1);
  c->alloc(d.c_its, (sims ? NS : CA) * 60);
  c->alloc(d.c_nits, sims ? NS : CA);
  // simulations keep the NodeClaims' hostname counts zero at rest (ffd.hip):
  // zeroed once per upload
  c->hc_bytes = 0;
  if (sims) {
    c->alloc_zero(d.hc, (size_t)std::max<uint32_t>(e.TGH, 1) * CA);
    c->hc_bytes = (size_t)std::max<uint32_t>(e.TGH, 1) * CA * sizeof(int32_t);
  } else {
    c->alloc(d.hc, (size_t)std::max<uint32_t>(e.TGH, 1) * CA);
  }
  if (sims) {
    d.n_sims = (uint32_t)NS;
    d.sim_nt = sims->nt;
    d.ov_cap = std::max<uint32_t>(sims->ov_cap, 1);
    d.nb_words = (e.NN + 31) / 32;
    c->upload(d.sim_pod_off, sims->pod_off);
    c->upload(d.sim_pods, sims->pods);
    c->upload(d.sim_cand_off, sims->cand_off);
    c->upload(d.sim_cands, sims->cands);
    c->alloc(d.ov_req, (size_t)sims->blocks * d.ov_cap * gsd::RMAX);
    c->alloc(d.ov_fk, (size_t)sims->blocks * d.ov_cap * F1);
    // the general (topology / volumes / minValues) simulation variant
    c->alloc_zero(d.ov_hn, (size_t)sims->blocks * d.ov_cap * std::max<uint32_t>(e.TGH, 1));
    c->ov_hn_bytes = (size_t)sims->blocks * d.ov_cap * std::max<uint32_t>(e.TGH, 1) * sizeof(uint64_t);
    d.ov_epoch = 0;
    c->alloc(d.ov_vol, e.any_vol ? (size_t)sims->blocks * d.ov_cap : 1);
    d.ovh_slots = gsd::ovh_slots_for(d.ov_cap);
    d.sim_lds = sims->sim_lds ? 1u : 0u;
    c->alloc(d.ov_map, d.ovh_slots ? 1 : (size_t)sims->blocks * std::max<uint32_t>(e.NN, 1));
    {
      std::vector<uint64_t> known = sims->known;
      known.resize(std::max<size_t>(NS, 1), 0);
      c->upload(d.sim_known, std::move(known));
    }
    c->alloc(d.slot_its, e.any_mv ? CA * 60 : 1);
    c->alloc(d.slot_nits, e.any_mv ? CA : 1);
    c->alloc(d.slot_drop, e.any_mv ? CA : 1);
    c->alloc(d.sim_ctrl, NS);
    c->alloc(d.sim_blk, sims->blocks);
    c->alloc(d.sim_hdr, NS);
    c->alloc(d.sim_next, 1);
    d.n_pending = c->n_pending;
    auto pinned = [&](auto*& dst, size_t n) {
      void* h = nullptr;
      HIPCHK(hipHostMalloc(&h, std::max<size_t>(n, 1) * sizeof(*dst), hipHostMallocDefault));
      c->host_allocs.push_back(h);
      dst = (std::remove_reference_t<decltype(dst)>)h;
    };
    pinned(c->h_ctrl, NS);
    pinned(c->h_hdr, NS);
    pinned(c->h_its, NS * 60);
    pinned(c->h_nits, NS);
  }
  c->commit();
  if (!sims) {
    HIPCHK(gsk_queue_records(&d, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
  }
}

uint32_t trunc_lds_bytes(uint32_t N) {
  uint32_t np2 = 1;
  while (np2 < N) np2 <<= 1;
  return np2 * 8;
}

// <U> OrderByPrice(...)[0] tables for the static matrix: for every distinct
// offering grid G = grid(template AND pod zones, template AND pod capacity
// types), the instance types with an available offering in G, keyed and
// sorted by (min price rank over G, name rank).  Built once per prepared
// problem, on the first gs_feasibility.
uint64_t host_grid_of(uint64_t zm, uint64_t cm, uint32_t Z, uint32_t C) {
  const uint64_t cmask = C >= 64 ? ~0ull : ((1ull << C) - 1);
  uint64_t g = 0;
  for (uint32_t z = 0; z < Z; z++)
    if ((zm >> z) & 1) g |= (cm & cmask) << (z * C);
  return g;
}

void build_grid_orders(gs_ctx* c) {
  auto& e = c->enc;
  auto& d = c->dp;
  if (d.grid_list) return;
  std::set<std::pair<uint64_t, uint64_t>> zc;
  for (uint32_t v = 0; v < e.V; v++) zc.insert({e.vars[v].zm, e.vars[v].cm});
  std::set<uint64_t> gs;
  for (uint32_t t = 0; t < e.T; t++)
    for (auto& m : zc) gs.insert(host_grid_of(e.tmpl[t].zm & m.first, e.tmpl[t].cm & m.second, e.Z, e.C));
  std::vector<uint64_t> list(gs.begin(), gs.end()), keys;
  std::vector<uint32_t> off{0}, its;
  uint32_t max_cnt = 0;
  for (uint64_t G : list) max_cnt = std::max<uint32_t>(max_cnt, (uint32_t)__builtin_popcountll(G));
  uint32_t NPL = 1;
  while ((1u << NPL) <= max_cnt) NPL++;
  std::vector<uint64_t> planes(std::max<size_t>(list.size(), 1) * NPL * e.W, 0);
  for (size_t g = 0; g < list.size(); g++) {
    const uint64_t G = list[g];
    const size_t b = keys.size();
    std::vector<std::pair<uint64_t, uint32_t>> ki;
    for (uint32_t i = 0; i < e.N; i++) {
      uint32_t mp = gsd::NONE;
      for (uint64_t m = e.it_pair[i] & G; m; m &= m - 1) mp = std::min(mp, e.it_prank[(size_t)i * 64 + __builtin_ctzll(m)]);
      if (mp != gsd::NONE) ki.push_back({((uint64_t)mp << 32) | e.it_namerank[i], i});
      const uint32_t cnt = (uint32_t)__builtin_popcountll(e.it_pair[i] & G);
      for (uint32_t pb = 0; pb < NPL; pb++)
        if ((cnt >> pb) & 1) planes[(g * NPL + pb) * e.W + i / 64] |= 1ull << (i % 64);
    }
    std::sort(ki.begin(), ki.end());
    for (auto& x : ki) {
      keys.push_back(x.first);
      its.push_back(x.second);
    }
    (void)b;
    off.push_back((uint32_t)keys.size());
  }
  if (keys.empty()) {
    keys.push_back(0);
    its.push_back(0);
  }
  // rank blocks: grid g's list positions [64k, 64k + 64) as an instance-type
  // bitset, so the cheapest-offering search tests 64 list entries per AND
  // instead of walking the list (at most 64 MiB; the list walk otherwise)
  uint32_t NB = 0;
  for (size_t g = 0; g + 1 < off.size(); g++) NB = std::max<uint32_t>(NB, (off[g + 1] - off[g] + 63) / 64);
  std::vector<uint64_t> blocks;
  if (!list.empty() && NB && list.size() * NB * (size_t)e.W * 8 <= ((size_t)64 << 20)) {
    blocks.assign(list.size() * NB * (size_t)e.W, 0);
    for (size_t g = 0; g + 1 < off.size(); g++)
      for (uint32_t q = off[g]; q < off[g + 1]; q++) {
        const uint32_t k = (q - off[g]) / 64, it = its[q];
        blocks[((size_t)g * NB + k) * e.W + it / 64] |= 1ull << (it % 64);
      }
  }
  const size_t bl = list.size() * 8, bo = off.size() * 4, bk = keys.size() * 8, bi = its.size() * 4,
               bp = planes.size() * 8, bb = blocks.size() * 8;
  auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
  char* p = nullptr;
  HIPCHK(hipMalloc((void**)&p, up(bl) + up(bo) + up(bk) + up(bi) + up(bp) + up(bb)));
  c->allocs.push_back(p);
  char* po = p + up(bl);
  char* pk = po + up(bo);
  char* pi = pk + up(bk);
  char* pp = pi + up(bi);
  char* pb = pp + up(bp);
  HIPCHK(hipMemcpyAsync(p, list.data(), bl, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(po, off.data(), bo, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(pk, keys.data(), bk, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(pi, its.data(), bi, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(pp, planes.data(), bp, hipMemcpyHostToDevice, c->stream));
  if (bb) HIPCHK(hipMemcpyAsync(pb, blocks.data(), bb, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  d.grid_list = (const uint64_t*)p;
  d.grid_off = (const uint32_t*)po;
  d.grid_keys = (const uint64_t*)pk;
  d.grid_its = (const uint32_t*)pi;
  d.grid_planes = (const uint64_t*)pp;
  d.grid_blocks = bb ? (const uint64_t*)pb : nullptr;
  d.grid_nb = bb ? NB : 0u;
  d.n_grids = (uint32_t)list.size();
  d.n_planes = NPL;
}

void launch_feas(gs_ctx* c, uint32_t apply_limits, uint32_t w_lo, uint32_t w_hi, bool mv_rows) {
  if (apply_limits) build_grid_orders(c);
  HIPCHK(gsk_feas(&c->dp, apply_limits, w_lo, w_hi, c->stream));
  // the static matrix's rows answer CanAdd on a fresh NodeClaim, minValues
  // included (whole rows only: callers refuse column shards with minValues;
  // a sharded context applies it after the merge)
  if (apply_limits && mv_rows && c->enc.any_mv) HIPCHK(gsk_mv_rows(&c->dp, c->stream));
}

// device capacity of the encoded problem (the FFD kernel keeps these in LDS)
gsh::Err capacity_check(const gsh::Encoded& e) {
  if (e.N > 8192) return gsh::Err{GS_E_CAPACITY, "more than 8192 instance types"};
  if (e.thr_val.size() + 4 > gsd::THR_LDS_MAX)
    return gsh::Err{GS_E_CAPACITY, "more than 2044 distinct allocatable values over the resources"};
  if ((size_t)e.Z * e.C * e.W > gsd::SLOT_LDS_MAX)
    return gsh::Err{GS_E_CAPACITY, "zones x capacity types x instance-type words exceeds 1024"};
  return gsh::Err{GS_OK, ""};
}

gs_status prepare_one(gs_ctx* c, const gs_problem* p) {
  c->prepared = c->ran = false;
  c->cons_ready = false;
  auto t0 = Clock::now();
  gsh::Err er = gsh::encode(p, c->enc);
  c->t_encode = ms_since(t0);
  if (er.code != GS_OK) return fail(c, er.code, er.msg);
  er = capacity_check(c->enc);
  if (er.code != GS_OK) return fail(c, er.code, er.msg);
  c->n_nodepools = p->n_nodepools;
  try {
    HIPCHK(hipSetDevice(c->device));
    auto t1 = Clock::now();
    upload_problem(c, nullptr);
    c->t_upload = ms_since(t1);
  } catch (const HipError& e) {
    return fail(c, GS_E_HIP, e.msg);
  }
  c->prepared = true;
  return GS_OK;
}

gs_status prepare_from(gs_ctx* c, const gs_ctx* src) {
  c->prepared = c->ran = false;
  c->cons_ready = false;
  c->enc = src->enc;
  c->n_nodepools = src->n_nodepools;
  c->t_encode = 0;
  try {
    HIPCHK(hipSetDevice(c->device));
    auto t1 = Clock::now();
    upload_problem(c, nullptr);
    c->t_upload = ms_since(t1);
  } catch (const HipError& e) {
    return fail(c, GS_E_HIP, e.msg);
  }
  c->prepared = true;
  return GS_OK;
}

}  // namespace gsc

using namespace gsc;

extern "C" {

const char* gs_version(void) { return "gpusched 0.1 (gfx950)"; }

uint32_t gs_abi_sizes(uint32_t* out, uint32_t n) {
  const uint32_t s[31] = {sizeof(gs_range),        sizeof(gs_requirement),         sizeof(gs_quantity),
                          sizeof(gs_label),        sizeof(gs_taint),               sizeof(gs_toleration),
                          sizeof(gs_term),         sizeof(gs_offering),            sizeof(gs_instance_type),
                          sizeof(gs_nodepool),     sizeof(gs_pod),                 sizeof(gs_node),
                          sizeof(gs_problem),      sizeof(gs_result),              sizeof(gs_feas_result),
                          sizeof(gs_config),       sizeof(gs_consolidation),       sizeof(gs_command),
                          sizeof(gs_consolidation_result), sizeof(gs_claim_query),
                          sizeof(gs_claim_filter_result), sizeof(gs_vpc_profile), sizeof(gs_price),
                          sizeof(gs_unavailable), sizeof(gs_catalog_env), sizeof(gs_catalog),
                          sizeof(gs_affinity_term), sizeof(gs_host_port), sizeof(gs_volume),
                          sizeof(gs_volume_limit), sizeof(gs_namespace)};
  for (uint32_t i = 0; i < n && i < 31; i++) out[i] = s[i];
  return 31;
}

gs_status gs_validate(const gs_problem* p, char* err, size_t len) {
  if (!p) return GS_E_INVALID;
  gsh::Encoded enc;
  gsh::Err er = gsh::encode(p, enc);
  if (er.code == GS_OK) er = capacity_check(enc);
  if (err && len) {
    size_t n = std::min(len - 1, er.msg.size());
    std::memcpy(err, er.msg.data(), n);
    err[n] = 0;
  }
  return er.code;
}

size_t gs_last_error(const gs_ctx* ctx, char* buf, size_t len) {
  if (!ctx) return 0;
  if (buf && len) {
    size_t n = std::min(len - 1, ctx->err.size());
    std::memcpy(buf, ctx->err.data(), n);
    buf[n] = 0;
  }
  return ctx->err.size();
}

gs_status gs_create(const gs_config* cfg, gs_ctx** out) {
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return GS_E_NO_DEVICE;
  auto* c = new gs_ctx();
  c->device = cfg ? cfg->device : 0;
  c->cfg_flags = cfg ? cfg->flags : 0;
  try {
    HIPCHK(hipSetDevice(c->device));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, c->device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
      delete c;
      return GS_E_NO_DEVICE;
    }
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    for (auto& e : c->ev) HIPCHK(hipEventCreate(&e));
    HIPCHK(gsk_init_ffd(kLdsBytes));
    HIPCHK(gsk_init_ffdw(kLdsBytes));
    HIPCHK(gsk_init_trunc(65536));
  } catch (const HipError& e) {
    delete c;
    return GS_E_HIP;
  }
  if (cfg && cfg->n_shards > 1) {
    for (uint32_t k = 0; k < cfg->n_shards; k++) {
      gs_config sc = *cfg;
      sc.device = cfg->shard_devices ? cfg->shard_devices[k] : cfg->device;
      sc.n_shards = 0;
      sc.shard_devices = nullptr;
      gs_ctx* child = nullptr;
      const gs_status st = gs_create(&sc, &child);
      if (st != GS_OK) {
        gs_destroy(c);
        return st;
      }
      c->shards.push_back(child);
    }
    // the merge kernel on `device` reads every shard's slice: peer access to
    // each other device (xGMI)
    for (gs_ctx* s : c->shards) {
      if (s->device == c->device) continue;
      (void)hipSetDevice(c->device);
      const hipError_t pe = hipDeviceEnablePeerAccess(s->device, 0);
      if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled) {
        c->err = std::string("peer access to shard device ") + std::to_string(s->device) + ": " + hipGetErrorString(pe);
        gs_destroy(c);
        return GS_E_HIP;
      }
    }
    if (cfg->flags & GS_CFG_RCCL) {
      std::vector<int> devs;
      for (gs_ctx* s : c->shards) devs.push_back(s->device);
      c->comms.assign(devs.size(), nullptr);
      const ncclResult_t r = ncclCommInitAll(c->comms.data(), (int)devs.size(), devs.data());
      if (r != ncclSuccess) {
        c->comms.clear();
        gs_destroy(c);
        return GS_E_RCCL;
      }
    }
    (void)hipSetDevice(c->device);
  }
  *out = c;
  return GS_OK;
}

void gs_destroy(gs_ctx* c) {
  if (!c) return;
  for (ncclComm_t m : c->comms)
    if (m) (void)ncclCommDestroy(m);
  c->comms.clear();
  for (gs_ctx* s : c->shards) gs_destroy(s);
  c->shards.clear();
  (void)hipSetDevice(c->device);
  c->free_all();
  if (c->arena) (void)hipFree(c->arena);
  if (c->stage) (void)hipHostFree(c->stage);
  if (c->cf_dev) (void)hipFree(c->cf_dev);
  for (auto& e : c->ev)
    if (e) (void)hipEventDestroy(e);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

gs_status gs_prepare(gs_ctx* c, const gs_problem* p) {
  if (!c || !p) return GS_E_INVALID;
  if (!c->shards.empty()) return sharded_prepare(c, p);
  return prepare_one(c, p);
}

// claim arrays for up to min(P, 65,535) NodeClaims (the packed sort order
// keeps 16-bit claim ids), hostname counts within 2 GiB; false if that is no
// more than the LDS already held
static bool grow_claims(gs_ctx* c, bool force = false) {
  auto& d = c->dp;
  const auto& e = c->enc;
  size_t cap = std::min<size_t>(std::max<uint32_t>(d.P, 1), 65535);
  const size_t per_h = (size_t)std::max<uint32_t>(e.TGH, 1) * sizeof(int32_t);
  cap = std::min<size_t>(cap, ((size_t)2 << 30) / per_h);
  if (cap <= d.max_claims_wave && !force) return false;
  const size_t F1 = std::max<uint32_t>(e.F, 1);
  auto get = [&](auto*& dst, size_t n) {
    void* p = nullptr;
    HIPCHK(hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(*dst)));
    c->allocs.push_back(p);
    dst = (std::remove_reference_t<decltype(dst)>)p;
  };
  get(d.c_rec, cap);
  get(d.c_opts, cap * d.OW);
  get(d.c_fk, cap * F1);
  get(d.c_sorted, cap);
  get(d.c_its, cap * 60);
  get(d.c_nits, cap);
  get(d.hc, cap * std::max<uint32_t>(e.TGH, 1));
  get(d.ch_slk, cap);
  get(d.ch_rm, cap);
  get(d.ch_so, cap);
  get(d.ch_scr, cap);
  get(d.ch_tmpl, cap);
  d.claim_cap = (uint32_t)cap;
  c->ch = true;
  return true;
}

gs_status gs_run(gs_ctx* c) {
  if (!c || !c->prepared) return GS_E_INVALID;
  const auto tw = Clock::now();
  try {
    HIPCHK(hipSetDevice(c->device));
    auto& d = c->dp;
    HIPCHK(hipEventRecord(c->ev[0], c->stream));
    launch_feas(c, 0);
    HIPCHK(hipEventRecord(c->ev[1], c->stream));
    if (c->wave && !c->ch && (c->cfg_flags & GS_CFG_CLAIMS_HBM) && !grow_claims(c, true))
      throw HipError{"claim arrays for the HBM claim mode"};
    if (c->wave)
      HIPCHK(gsk_ffdw(&d, c->ch ? 1u : 0u, c->stream));
    else
      HIPCHK(gsk_ffd(&d, 1, c->stream));
    HIPCHK(hipEventRecord(c->ev[2], c->stream));
    HIPCHK(gsk_trunc(&d, trunc_lds_bytes(d.N), 0, c->stream));
    HIPCHK(hipEventRecord(c->ev[3], c->stream));
    HIPCHK(hipEventSynchronize(c->ev[3]));
    if (c->wave && !c->ch && d.P > d.max_claims_wave) {
      // the single-wave kernel ran out of LDS NodeClaims: grow the claim
      // arrays and rerun it with the claim scan state in HBM (later runs of
      // this prepared problem start there)
      uint32_t st = 0;
      HIPCHK(hipMemcpy(&st, &d.ctrl->status, sizeof st, hipMemcpyDeviceToHost));
      if (st == gsd::ST_CLAIMS && grow_claims(c)) {
        HIPCHK(hipEventRecord(c->ev[1], c->stream));
        HIPCHK(gsk_ffdw(&d, 1, c->stream));
        HIPCHK(hipEventRecord(c->ev[2], c->stream));
        HIPCHK(gsk_trunc(&d, trunc_lds_bytes(d.N), 0, c->stream));
        HIPCHK(hipEventRecord(c->ev[3], c->stream));
        HIPCHK(hipEventSynchronize(c->ev[3]));
      }
    }
    float a = 0, b = 0, x = 0;
    HIPCHK(hipEventElapsedTime(&a, c->ev[0], c->ev[1]));
    HIPCHK(hipEventElapsedTime(&b, c->ev[1], c->ev[2]));
    HIPCHK(hipEventElapsedTime(&x, c->ev[2], c->ev[3]));
    c->t_feas = a;
    c->t_ffd = b;
    c->t_trunc = x;
  } catch (const HipError& e) {
    return fail(c, GS_E_HIP, e.msg);
  }
  c->t_run_wall = ms_since(tw);
  c->ran = true;
  return GS_OK;
}

// diagnostic (not in the public header): FFD control block counters
extern "C" gs_status gs_debug_ctrl(gs_ctx* c, uint64_t* out, uint32_t n) {
  if (!c || !c->ran) return GS_E_INVALID;
  gsd::Ctrl ctl;
  if (hipMemcpy(&ctl, c->dp.ctrl, sizeof ctl, hipMemcpyDeviceToHost) != hipSuccess) return GS_E_HIP;
  for (uint32_t i = 0; i < n && i < 16; i++) out[i] = ctl.dbg[i];
  return GS_OK;
}

gs_status gs_last_run_ms(const gs_ctx* c, double out[3]) {
  if (!c || !c->ran || !out) return GS_E_INVALID;
  out[0] = c->t_feas;
  out[1] = c->t_ffd;
  out[2] = c->t_trunc;
  return GS_OK;
}

gs_status gs_fetch(gs_ctx* c, gs_result* out) {
  if (!c || !c->ran || !out) return GS_E_INVALID;
  auto t0 = Clock::now();
  auto& e = c->enc;
  auto& d = c->dp;
  std::vector<gsd::LogRec> log;
  std::vector<gsd::ClaimRec> hdr;
  std::vector<uint32_t> its, nits, queue;
  try {
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpy(&c->ctrl, d.ctrl, sizeof(gsd::Ctrl), hipMemcpyDeviceToHost));
    const uint32_t M = c->ctrl.n_claims;
    log.resize(c->ctrl.n_log);
    hdr.resize(M);
    its.resize((size_t)M * 60);
    nits.resize(M);
    queue.resize(e.P);
    if (!log.empty()) HIPCHK(hipMemcpy(log.data(), d.log, log.size() * sizeof(gsd::LogRec), hipMemcpyDeviceToHost));
    if (M) {
      HIPCHK(hipMemcpy(hdr.data(), d.c_rec, M * sizeof(gsd::ClaimRec), hipMemcpyDeviceToHost));
      HIPCHK(hipMemcpy(its.data(), d.c_its, its.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
      HIPCHK(hipMemcpy(nits.data(), d.c_nits, M * sizeof(uint32_t), hipMemcpyDeviceToHost));
    }
    if (e.P) HIPCHK(hipMemcpy(queue.data(), d.queue, e.P * sizeof(uint32_t), hipMemcpyDeviceToHost));
  } catch (const HipError& ex) {
    return fail(c, GS_E_HIP, ex.msg);
  }
  if (c->ctrl.status == gsd::ST_CLAIMS)
    return fail(c, GS_E_CAPACITY, "NodeClaim count exceeded the device capacity (" +
                                      std::to_string(c->ch ? std::min<uint32_t>(c->dp.claim_cap, 65535) : c->dp.max_claims) +
                                      " in-flight NodeClaims)");
  if (c->ctrl.status == gsd::ST_POD_COUNT)
    return fail(c, GS_E_CAPACITY, "a NodeClaim would hold more than 65535 pods (16-bit pod count in LDS)");
  if (c->ctrl.status == gsd::ST_INTERNAL) return fail(c, GS_E_HIP, "ffd kernel reported an internal error (queue / channel bound)");
  if (c->ctrl.status != 0) return fail(c, GS_E_HIP, "ffd kernel reported an unknown status");
  const uint32_t M = c->ctrl.n_claims;
  // pods per claim in add order, and each claim's requirement set
  std::vector<std::vector<uint32_t>> cp(M);
  std::vector<gsh::Reqs> creq(M);
  for (uint32_t j = 0; j < M; j++) creq[j] = e.tmpl_reqs[hdr[j].tmpl];
  c->node_pod_offsets.assign(1, 0);
  c->node_pods.clear();
  std::vector<std::vector<uint32_t>> np_(e.NN);
  for (auto& l : log) {
    if (l.target & 0x80000000u) {
      const uint32_t pos = l.target & 0x7FFFFFFFu;
      if (pos >= e.NN) return fail(c, GS_E_HIP, "corrupt add log");
      np_[e.node_order[pos]].push_back(l.pod);
      continue;
    }
    if (l.target >= M) return fail(c, GS_E_HIP, "corrupt add log");
    cp[l.target].push_back(l.pod);
    for (auto& kv : e.variants[e.var_sv[l.var]].reqs) gsh::reqs_add(e, creq[l.target], kv.first, kv.second);
  }
  c->claim_nodepool.assign(M, 0);
  c->claim_pod_offsets.assign(1, 0);
  c->claim_pods.clear();
  c->claim_it_offsets.assign(1, 0);
  c->claim_its.clear();
  c->req_text.assign(M, "");
  c->claim_requests.assign((size_t)M * e.R, 0);
  // <U> Results.TruncateInstanceTypes: a NodeClaim whose top 60 by price miss
  // its template's minValues is dropped, its pods become pod errors
  std::vector<uint32_t> dropped_pods;
  uint32_t kept = 0;
  for (uint32_t j = 0; j < M; j++) {
    const gsd::TmplRec& tr = e.tmpl[hdr[j].tmpl];
    bool drop = false;
    for (uint32_t mm = tr.mv_mask; mm && !drop; mm &= mm - 1) {
      const uint32_t k = (uint32_t)__builtin_ctz(mm);
      std::set<uint32_t> vals;
      for (uint32_t q = 0; q < nits[j]; q++) vals.insert(e.it_vid[(size_t)k * e.N + its[(size_t)j * 60 + q]]);
      drop = vals.size() < tr.mv[k];
    }
    if (drop) {
      dropped_pods.insert(dropped_pods.end(), cp[j].begin(), cp[j].end());
      continue;
    }
    c->claim_nodepool[kept] = tr.np_index;
    c->claim_pods.insert(c->claim_pods.end(), cp[j].begin(), cp[j].end());
    c->claim_pod_offsets.push_back((uint32_t)c->claim_pods.size());
    c->claim_its.insert(c->claim_its.end(), its.begin() + (size_t)j * 60, its.begin() + (size_t)j * 60 + nits[j]);
    c->claim_it_offsets.push_back((uint32_t)c->claim_its.size());
    if (e.TG && e.keys[e.k_dom].vocab.size() <= (size_t)gsd::ZVMAX && !(hdr[j].zflags & gsd::ZF_COMP)) {
      // topology spread narrowed the zone to In[domain]: the device's zone
      // Has already includes it (template AND pods AND topology)
      gsh::KReq q;
      q.comp = false;
      q.has = gsh::Bits(e.keys[e.k_dom].vocab.words());
      q.excl = gsh::Bits(e.keys[e.k_dom].vocab.words());
      q.has.w[0] = hdr[j].zfull;
      gsh::reqs_add(e, creq[j], e.k_dom, q);
    }
    creq[j].erase(e.k_hostname);  // FinalizeScheduling
    c->req_text[kept] = gsh::canonical(e, creq[j]);
    for (uint32_t r = 0; r < e.R; r++) c->claim_requests[(size_t)kept * e.R + r] = hdr[j].tot(r);
    kept++;
  }
  c->claim_nodepool.resize(kept);
  c->req_text.resize(kept);
  c->claim_requests.resize((size_t)kept * e.R);
  c->req_ptrs.clear();
  for (auto& s : c->req_text) c->req_ptrs.push_back(s.c_str());
  c->error_pods.clear();
  for (uint32_t i = 0; i < c->ctrl.qlen; i++) c->error_pods.push_back(queue[(c->ctrl.qhead + i) % e.P]);
  c->error_pods.insert(c->error_pods.end(), dropped_pods.begin(), dropped_pods.end());
  std::sort(c->error_pods.begin(), c->error_pods.end());
  for (auto& v : np_) {
    c->node_pods.insert(c->node_pods.end(), v.begin(), v.end());
    c->node_pod_offsets.push_back((uint32_t)c->node_pods.size());
  }
  c->t_fetch = ms_since(t0);
  std::memset(out, 0, sizeof(*out));
  out->n_claims = kept;
  out->claim_nodepool = c->claim_nodepool.data();
  out->claim_pod_offsets = c->claim_pod_offsets.data();
  out->claim_pods = c->claim_pods.data();
  out->claim_it_offsets = c->claim_it_offsets.data();
  out->claim_its = c->claim_its.data();
  out->claim_requirements = c->req_ptrs.data();
  out->n_resources = e.R;
  out->resource_names = e.res_name_ids.data();
  out->claim_requests = c->claim_requests.data();
  out->n_nodes = e.NN;
  out->node_pod_offsets = c->node_pod_offsets.data();
  out->node_pods = c->node_pods.data();
  out->n_errors = (uint32_t)c->error_pods.size();
  out->error_pods = c->error_pods.data();
  out->checks = e.checks;
  out->pops = c->ctrl.pops;
  out->cand_evals = c->ctrl.cand_evals;
  out->cand_full = c->ctrl.cand_full;
  out->claim_prefix = c->ctrl.claim_prefix;
  out->node_prefix = c->ctrl.node_prefix;
  // wall_clock64 runs at 100 MHz; ~0: the phase timers are not built in (-1)
  auto phase_ms = [](uint64_t t) { return t == ~0ull ? -1.0 : (double)t * 1e-5; };
  out->t_ffd_sort_ms = phase_ms(c->ctrl.t_sort);
  out->t_ffd_scan_ms = phase_ms(c->ctrl.t_scan);
  out->t_ffd_template_ms = phase_ms(c->ctrl.t_tmpl);
  out->sorts_fast = c->ctrl.fast_sorts;
  out->sorts_generic = c->ctrl.generic_sorts;
  out->words = e.W;
  out->n_templates = e.T;
  out->n_variants = e.V;
  out->t_encode_ms = c->t_encode;
  out->t_upload_ms = c->t_upload;
  out->t_feas_ms = c->t_feas;
  out->t_ffd_ms = c->t_ffd;
  out->t_truncate_ms = c->t_trunc;
  out->t_fetch_ms = c->t_fetch;
  out->t_total_ms = c->t_encode + c->t_upload + c->t_feas + c->t_ffd + c->t_trunc + c->t_fetch;
  out->t_run_wall_ms = c->t_run_wall;
  out->t_wall_ms = 0;
  return GS_OK;
}

gs_status gs_solve(gs_ctx* c, const gs_problem* p, gs_result* out) {
  const auto tw = Clock::now();
  gs_status s = gs_prepare(c, p);
  if (s != GS_OK) return s;
  s = gs_run(c);
  if (s != GS_OK) return s;
  s = gs_fetch(c, out);
  if (s == GS_OK) out->t_wall_ms = ms_since(tw);
  return s;
}

gs_status gs_feasibility_shard(gs_ctx* c, uint32_t word_begin, uint32_t word_end, gs_feas_result* out) {
  if (!c || !c->prepared || !out) return GS_E_INVALID;
  auto& e = c->enc;
  const uint32_t P = e.P, NP = c->n_nodepools, W = e.W;
  word_end = std::min(word_end, W);
  if (e.any_mv && (word_begin > 0 || word_end < W))
    return fail(c, GS_E_UNSUPPORTED, "minValues needs whole static-matrix rows (no instance-type column shards)");
  if (word_begin > word_end) return fail(c, GS_E_INVALID, "empty or inverted word range");
  double ms = 0, merge_ms = 0;
  const uint32_t OW = c->dp.OW;
  std::vector<uint64_t> rows((size_t)e.V * e.T * OW), key((size_t)e.V * e.T);
  std::vector<uint32_t> ch((size_t)e.V * e.T), nfo((size_t)e.V * e.T);
  if (!c->shards.empty()) {
    // the shards compute, the parent's device merges: the result is in c->dp
    const gs_status st = sharded_compute(c, word_begin, word_end, &ms, &merge_ms);
    if (st != GS_OK) return st;
  }
  try {
    HIPCHK(hipSetDevice(c->device));
    if (c->shards.empty()) {
      float f = 0;
      HIPCHK(hipEventRecord(c->ev[4], c->stream));
      launch_feas(c, 1, word_begin, word_end);
      HIPCHK(hipEventRecord(c->ev[5], c->stream));
      HIPCHK(hipEventSynchronize(c->ev[5]));
      HIPCHK(hipEventElapsedTime(&f, c->ev[4], c->ev[5]));
      ms = f;
    }
    if (!rows.empty()) HIPCHK(hipMemcpy(rows.data(), c->dp.rows, rows.size() * 8, hipMemcpyDeviceToHost));
    if (!ch.empty()) {
      HIPCHK(hipMemcpy(ch.data(), c->dp.cheapest, ch.size() * 4, hipMemcpyDeviceToHost));
      HIPCHK(hipMemcpy(nfo.data(), c->dp.nfo, nfo.size() * 4, hipMemcpyDeviceToHost));
      HIPCHK(hipMemcpy(key.data(), c->dp.cheapest_key, key.size() * 8, hipMemcpyDeviceToHost));
    }
  } catch (const HipError& ex) {
    return fail(c, GS_E_HIP, ex.msg);
  }
  c->f_rows.assign((size_t)P * NP * W, 0);
  c->f_cheapest.assign((size_t)P * NP, -1);
  c->f_nfo.assign((size_t)P * NP, 0);
  c->f_key.assign((size_t)P * NP, 0x7FFFFFFFFFFFFFFFull);
  for (uint32_t p = 0; p < P; p++) {
    const uint32_t v = e.var_begin[p];  // the pod as given (no relaxation)
    for (uint32_t t = 0; t < e.T; t++) {
      const uint32_t np = e.tmpl[t].np_index;
      const size_t src = (size_t)v * e.T + t, dst = (size_t)p * NP + np;
      // words outside [word_begin, word_end) stay zero
      std::memcpy(&c->f_rows[dst * W + word_begin], &rows[src * OW + word_begin], (size_t)(word_end - word_begin) * 8);
      c->f_cheapest[dst] = ch[src] == gsd::NONE ? -1 : (int32_t)ch[src];
      c->f_nfo[dst] = nfo[src];
      c->f_key[dst] = key[src];
    }
  }
  std::memset(out, 0, sizeof(*out));
  out->n_pods = P;
  out->n_nodepools = NP;
  out->n_its = e.N;
  out->words = W;
  out->rows = c->f_rows.data();
  out->cheapest_it = c->f_cheapest.data();
  out->n_feasible_offerings = c->f_nfo.data();
  out->checks = e.checks;
  out->t_kernel_ms = ms;
  out->cheapest_key = c->f_key.data();
  out->it_name_rank = e.it_namerank.data();
  out->word_begin = word_begin;
  out->word_end = word_end;
  return GS_OK;
}

gs_status gs_feasibility(gs_ctx* c, gs_feas_result* out) { return gs_feasibility_shard(c, 0, ~0u, out); }

gs_status gs_feasibility_shard_device(gs_ctx* c, uint32_t word_begin, uint32_t word_end, gs_feas_device* out) {
  if (!c || !c->prepared || !out) return GS_E_INVALID;
  auto& e = c->enc;
  word_end = std::min(word_end, e.W);
  if (e.any_mv && (word_begin > 0 || word_end < e.W))
    return fail(c, GS_E_UNSUPPORTED, "minValues needs whole static-matrix rows (no instance-type column shards)");
  if (word_begin > word_end) return fail(c, GS_E_INVALID, "empty or inverted word range");
  double ms = 0, merge_ms = 0;
  if (!c->shards.empty()) {
    const gs_status st = sharded_compute(c, word_begin, word_end, &ms, &merge_ms);
    if (st != GS_OK) return st;
  } else {
    float f = 0;
    try {
      HIPCHK(hipSetDevice(c->device));
      HIPCHK(hipEventRecord(c->ev[4], c->stream));
      launch_feas(c, 1, word_begin, word_end);
      HIPCHK(hipEventRecord(c->ev[5], c->stream));
      HIPCHK(hipEventSynchronize(c->ev[5]));
      HIPCHK(hipEventElapsedTime(&f, c->ev[4], c->ev[5]));
    } catch (const HipError& ex) {
      return fail(c, GS_E_HIP, ex.msg);
    }
    ms = f;
  }
  c->f_tmpl_np.resize(e.T);
  for (uint32_t t = 0; t < e.T; t++) c->f_tmpl_np[t] = e.tmpl[t].np_index;
  c->f_var_of_pod.resize(e.P);
  for (uint32_t p = 0; p < e.P; p++) c->f_var_of_pod[p] = e.var_begin[p];
  std::memset(out, 0, sizeof(*out));
  out->n_variants = e.V;
  out->n_templates = e.T;
  out->words = e.W;
  out->row_stride = c->dp.OW;
  out->word_begin = word_begin;
  out->word_end = word_end;
  out->rows = c->dp.rows;
  out->n_feasible_offerings = c->dp.nfo;
  out->cheapest_key = reinterpret_cast<int64_t*>(c->dp.cheapest_key);
  out->variant_of_pod = c->f_var_of_pod.data();
  out->template_nodepool = c->f_tmpl_np.data();
  out->it_name_rank = e.it_namerank.data();
  out->n_pods = e.P;
  out->n_its = e.N;
  out->checks = e.checks;
  out->t_kernel_ms = ms;
  out->t_merge_ms = merge_ms;
  return GS_OK;
}

}  // extern "C"
