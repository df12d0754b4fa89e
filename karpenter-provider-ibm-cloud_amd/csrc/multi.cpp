// multi.cpp — one context, several devices (gs_config.n_shards > 1): the
// library-owned multi-GPU path for a single controller process.
//
// Consolidation simulations are independent units: simulation s runs on
// shard s % n (each shard a child gs_ctx on its own device and stream, driven
// from its own host thread); the parent merges the command tables and replays
// the SingleNode / MultiNode selection on the host exactly as
// gs_consolidation_choose does, so the result equals the single-device call.
// The static feasibility matrix shards by instance-type words: each shard
// computes a disjoint word range, the parent copies the rows, adds the
// offering counts and keeps the minimum OrderByPrice key.  The provisioning
// Solve is sequential in pod order and stays on the parent's device.
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

gs_status sharded_prepare(gs_ctx* c, const gs_problem* p) {
  gs_status mine = GS_OK;
  std::thread self([&] { mine = prepare_one(c, p); });
  auto st = on_shards(c, [&](size_t k) { return gs_prepare(c->shards[k], p); });
  self.join();
  if (mine != GS_OK) return mine;
  return first_error(c, st);
}

gs_status sharded_feasibility(gs_ctx* c, uint32_t word_begin, uint32_t word_end, gs_feas_result* out) {
  auto& e = c->enc;
  const uint32_t W = e.W, P = e.P, NP = c->n_nodepools, K = (uint32_t)c->shards.size();
  word_end = std::min(word_end, W);
  if (word_begin > word_end) return fail(c, GS_E_INVALID, "empty or inverted word range");
  std::vector<gs_feas_result> r(K);
  auto st = on_shards(c, [&](size_t k) {
    const uint32_t n = word_end - word_begin;
    const uint32_t lo = word_begin + (uint32_t)((uint64_t)n * k / K), hi = word_begin + (uint32_t)((uint64_t)n * (k + 1) / K);
    return gs_feasibility_shard(c->shards[k], lo, hi, &r[k]);
  });
  const gs_status es = first_error(c, st);
  if (es != GS_OK) return es;
  const size_t PN = (size_t)P * NP;
  c->f_rows.assign(PN * W, 0);
  c->f_nfo.assign(PN, 0);
  c->f_key.assign(PN, 0x7FFFFFFFFFFFFFFFull);
  c->f_cheapest.assign(PN, -1);
  double ms = 0;
  for (uint32_t k = 0; k < K; k++) {
    // rows: each shard's words are its own (zero elsewhere)
    for (uint32_t w = r[k].word_begin; w < r[k].word_end; w++)
      for (size_t q = 0; q < PN; q++) c->f_rows[q * W + w] = r[k].rows[q * W + w];
    for (size_t q = 0; q < PN; q++) {
      c->f_nfo[q] += r[k].n_feasible_offerings[q];
      if (r[k].cheapest_key[q] < c->f_key[q]) {
        c->f_key[q] = r[k].cheapest_key[q];
        c->f_cheapest[q] = r[k].cheapest_it[q];
      }
    }
    ms = std::max(ms, r[k].t_kernel_ms);
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
