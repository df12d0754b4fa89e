// multi.cpp — one context, several devices (gs_config.n_shards > 1): the
// library-owned multi-GPU path for a single controller process.
//
// Consolidation simulations are independent units: simulation s runs on
// shard s % n (each shard a child gs_ctx on its own device and stream, driven
// from its own host thread); the parent merges the command tables and replays
// the SingleNode / MultiNode selection on the host exactly as
// gs_consolidation_choose does, so the result equals the single-device call.
// The static feasibility matrix shards by instance-type words: each shard
// computes a disjoint word range on its device; a merge kernel on the parent's
// device gathers the rows (peer reads over xGMI), adds the offering counts
// and keeps the minimum OrderByPrice key (RCCL all-reduces the counts and keys
// first with GS_CFG_RCCL).  The provisioning Solve is sequential in pod order
// and stays on the parent's device.
#include <thread>

#include "ctx.hpp"

namespace gsc {

namespace {

// run f(k) for every shard on its own host thread
template <class F>
std::vector<gs_status> on_shards(gs_ctx* c, F f) {
  const size_t K = c->shards.size();
  std::vector<gs_status> st(K, GS_OK);
  std::vector<std::thread> th;
  for (size_t k = 0; k < K; k++) th.emplace_back([&, k] { st[k] = f(k); });
  for (auto& t : th) t.join();
  return st;
}

gs_status first_error(gs_ctx* c, const std::vector<gs_status>& st) {
  for (size_t k = 0; k < st.size(); k++)
    if (st[k] != GS_OK) {
      char buf[512];
      gs_last_error(c->shards[k], buf, sizeof buf);
      return fail(c, st[k], "shard " + std::to_string(k) + ": " + buf);
    }
  return GS_OK;
}

}  // namespace

// encode once on the parent, upload that encoding to every shard in parallel
gs_status sharded_prepare(gs_ctx* c, const gs_problem* p) {
  const gs_status mine = prepare_one(c, p);
  if (mine != GS_OK) return mine;
  auto st = on_shards(c, [&](size_t k) { return prepare_from(c->shards[k], c); });
  return first_error(c, st);
}

// The static matrix of words [wb, we): shard k computes its even slice on its
// own device (no minValues pass: rows are partial), then -- with RCCL -- the
// offering counts (SUM) and cheapest keys (MIN) are all-reduced across the
// shards' buffers in place, and one kernel on the parent's device gathers
// every word from its owner and finishes the counts / keys (merge_shards_kernel).
// The merged matrix is the parent's own device buffers; minValues runs on it.
gs_status sharded_compute(gs_ctx* c, uint32_t wb, uint32_t we, double* kernel_ms, double* merge_ms) {
  const uint32_t K = (uint32_t)c->shards.size();
  if (K > (uint32_t)gsd::SHARDS_MAX) return fail(c, GS_E_INVALID, "more than 16 shards");
  const uint32_t n = we - wb;
  auto lo_of = [&](uint32_t k) { return wb + (uint32_t)((uint64_t)n * k / K); };
  std::vector<float> t(K, 0.f);
  auto st = on_shards(c, [&](size_t k) -> gs_status {
    gs_ctx* s = c->shards[k];
    try {
      HIPCHK(hipSetDevice(s->device));
      HIPCHK(hipEventRecord(s->ev[4], s->stream));
      launch_feas(s, 1, lo_of((uint32_t)k), lo_of((uint32_t)k + 1), false);
      HIPCHK(hipEventRecord(s->ev[5], s->stream));
      HIPCHK(hipEventSynchronize(s->ev[5]));
      HIPCHK(hipEventElapsedTime(&t[k], s->ev[4], s->ev[5]));
    } catch (const HipError& ex) {
      return fail(s, GS_E_HIP, ex.msg);
    }
    return GS_OK;
  });
  gs_status es = first_error(c, st);
  if (es != GS_OK) return es;
  *kernel_ms = 0;
  for (float x : t) *kernel_ms = std::max(*kernel_ms, (double)x);
  const size_t VT = (size_t)c->enc.V * c->enc.T;
  auto t0 = Clock::now();
  if (!c->comms.empty()) {
    ncclResult_t r = ncclGroupStart();
    for (uint32_t k = 0; k < K && r == ncclSuccess; k++) {
      gs_ctx* s = c->shards[k];
      r = ncclAllReduce(s->dp.cheapest_key, s->dp.cheapest_key, VT, ncclUint64, ncclMin, c->comms[k], s->stream);
      if (r == ncclSuccess) r = ncclAllReduce(s->dp.nfo, s->dp.nfo, VT, ncclUint32, ncclSum, c->comms[k], s->stream);
    }
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess)
      return fail(c, GS_E_RCCL, std::string("RCCL all-reduce of the shard keys / counts: ") +
                                    ncclGetErrorString(r != ncclSuccess ? r : r2));
    for (gs_ctx* s : c->shards) {
      (void)hipSetDevice(s->device);
      if (hipStreamSynchronize(s->stream) != hipSuccess) return fail(c, GS_E_RCCL, "RCCL stream");
    }
  }
  gsd::ShardMerge m{};
  for (uint32_t k = 0; k < K; k++) {
    const gsd::DevProblem& sd = c->shards[k]->dp;
    m.src[k] = gsd::ShardSrc{sd.rows, sd.nfo, sd.cheapest_key, lo_of(k), lo_of(k + 1)};
  }
  m.K = K;
  m.K_red = c->comms.empty() ? K : 1u;
  m.VT = (uint32_t)VT;
  m.OW = c->dp.OW;
  m.wb = wb;
  m.we = we;
  m.rows = c->dp.rows;
  m.nfo = c->dp.nfo;
  m.key = c->dp.cheapest_key;
  m.cheapest = c->dp.cheapest;
  m.rank_to_it = c->dp.rank_to_it;
  float mk = 0;
  try {
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipEventRecord(c->ev[6], c->stream));
    HIPCHK(gsk_merge_shards(&m, c->stream));
    HIPCHK(hipEventRecord(c->ev[7], c->stream));
    if (c->enc.any_mv) HIPCHK(gsk_mv_rows(&c->dp, c->stream));  // whole rows now
    HIPCHK(hipEventSynchronize(c->ev[7]));
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipEventElapsedTime(&mk, c->ev[6], c->ev[7]));
  } catch (const HipError& ex) {
    return fail(c, GS_E_HIP, ex.msg);
  }
  // the gather kernel; with RCCL the host wall clock over all-reduce + gather
  *merge_ms = c->comms.empty() ? (double)mk : ms_since(t0);
  return GS_OK;
}

// in != nullptr: gs_consolidate (keeps the copies the reruns need);
// in == nullptr: gs_consolidate_rerun
gs_status sharded_consolidate(gs_ctx* c, const gs_consolidation* in, gs_consolidation_result* out) {
  const uint32_t K = (uint32_t)c->shards.size();
  if (in) {
    if (in->shard_count > 1) return fail(c, GS_E_INVALID, "a sharded context shards itself: leave shard_index/count zero");
    c->cons_ready = false;
    c->cons_cands.assign(in->candidates, in->candidates + in->n_candidates);
    c->cons_sets.assign(in->sets, in->sets + (in->mode == GS_CONSOLIDATE_EVAL ? in->n_sets : 0));
    c->cons_in = *in;
    c->cons_in.cluster = nullptr;  // not kept past the call
    c->cons_in.candidates = c->cons_cands.data();
    c->cons_in.sets = c->cons_sets.data();
    c->cand_table = build_cand_table(in->cluster, in->candidates, in->n_candidates);
  }
  std::vector<gs_consolidation_result> r(K);
  auto st = on_shards(c, [&](size_t k) {
    if (!in) return gs_consolidate_rerun(c->shards[k], &r[k]);
    gs_consolidation sk = *in;
    sk.shard_index = (uint32_t)k;
    sk.shard_count = K;
    return gs_consolidate(c->shards[k], &sk, &r[k]);
  });
  const gs_status es = first_error(c, st);
  if (es != GS_OK) return es;
  const uint32_t n = r[0].n_commands;
  for (uint32_t k = 1; k < K; k++)
    if (r[k].n_commands != n) return fail(c, GS_E_HIP, "shards disagree on the simulation count");
  c->commands.assign(n, gs_command{});
  c->cmd_options.clear();
  c->cmd_prices.clear();
  for (uint32_t s = 0; s < n; s++) {
    const gs_consolidation_result& rk = r[s % K];
    gs_command cmd = rk.commands[s];
    const uint32_t ob = (uint32_t)c->cmd_options.size();
    c->cmd_options.insert(c->cmd_options.end(), rk.options + cmd.options.begin,
                          rk.options + cmd.options.begin + cmd.options.count);
    c->cmd_prices.insert(c->cmd_prices.end(), rk.option_prices + cmd.options.begin,
                         rk.option_prices + cmd.options.begin + cmd.options.count);
    cmd.options.begin = ob;
    c->commands[s] = cmd;
  }
  c->multi_opts.clear();
  const int32_t chosen = choose_commands(c->cand_table, &c->cons_in, c->commands.data(), c->cmd_options.data(),
                                         c->cmd_prices.data(), &c->multi_opts);
  std::memset(out, 0, sizeof(*out));
  out->n_commands = n;
  out->commands = c->commands.data();
  out->options = c->cmd_options.data();
  out->option_prices = c->cmd_prices.data();
  out->chosen = chosen;
  out->n_multi_options = (uint32_t)c->multi_opts.size();
  out->multi_options = c->multi_opts.data();
  for (uint32_t k = 0; k < K; k++) {
    out->pods_simulated += r[k].pods_simulated;
    out->checks += r[k].checks;
    out->node_evals += r[k].node_evals;
    out->node_prefix += r[k].node_prefix;
    out->pops += r[k].pops;
    out->t_encode_ms = std::max(out->t_encode_ms, r[k].t_encode_ms);
    out->t_upload_ms = std::max(out->t_upload_ms, r[k].t_upload_ms);
    out->t_feas_ms = std::max(out->t_feas_ms, r[k].t_feas_ms);
    out->t_sim_ms = std::max(out->t_sim_ms, r[k].t_sim_ms);
    out->t_truncate_ms = std::max(out->t_truncate_ms, r[k].t_truncate_ms);
    out->t_fetch_ms = std::max(out->t_fetch_ms, r[k].t_fetch_ms);
  }
  c->cons_ready = true;
  return GS_OK;
}

}  // namespace gsc
