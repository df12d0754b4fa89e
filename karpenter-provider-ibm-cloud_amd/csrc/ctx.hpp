// ctx.hpp — gs_ctx (one device context of libgpusched.so) and the host
// helpers shared by the Solve (capi.cpp) and consolidation (consolidate.cpp)
// entry points.
#pragma once
#include <cstdio>
#include <cstdlib>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <string>
#include <map>
#include <memory>
#include <unordered_map>
#include <vector>

#include "../../include/gpusched.h"
#include "encode.hpp"
#include "layout.hpp"

extern "C" hipError_t gsk_init_trunc(uint32_t trunc_lds_bytes);
extern "C" hipError_t gsk_init_ffd(uint32_t lds_total);
extern "C" uint32_t gsk_ffd_dyn_lds_max(void);
extern "C" uint32_t gsk_ffd_sim_blocks_per_cu(uint32_t R, uint32_t lds, uint32_t nt, uint32_t general);
extern "C" uint32_t gsk_ffd_lds_bytes(uint32_t max_claims, uint32_t nthr, uint32_t nb_words,
                                      uint32_t topo_bytes);
extern "C" hipError_t gsk_feas(const gsd::DevProblem* d, uint32_t apply_limits, uint32_t w_lo, uint32_t w_hi,
                               hipStream_t s);
extern "C" hipError_t gsk_ffd(const gsd::DevProblem* d, uint32_t blocks, hipStream_t s);
extern "C" hipError_t gsk_init_ffdw(uint32_t lds_total);
extern "C" uint32_t gsk_ffdw_dyn_lds_max(void);
extern "C" hipError_t gsk_ffdw(const gsd::DevProblem* d, uint32_t ch, hipStream_t s);
extern "C" hipError_t gsk_trunc(const gsd::DevProblem* d, uint32_t lds_bytes, uint32_t n_slots, hipStream_t s);
extern "C" hipError_t gsk_mv_rows(const gsd::DevProblem* d, hipStream_t s);
extern "C" hipError_t gsk_queue_records(const gsd::DevProblem* d, hipStream_t s);
extern "C" hipError_t gsk_merge_shards(const gsd::ShardMerge* m, hipStream_t s);

namespace gsc {

constexpr uint32_t kMaxClaimsLds = 8192;  // LDS: 4x u16 slack + room, ord/sc/scratch u16, tmpl u8, thresholds
constexpr uint32_t kLdsBytes = 160 * 1024; // gfx950 LDS per workgroup
// the single-wave Solve (ffd_wave.hip) keeps 17 B of slack codes per existing
// node in LDS (layout.hpp wave_node_lds_bytes) beside the NodeClaims; larger
// clusters run the block kernel (ffd.hip)
constexpr uint32_t kWaveSolveMaxNodes = 6144;

using Clock = std::chrono::steady_clock;
inline double ms_since(Clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
}

struct HipError {
  std::string msg;
};
#define HIPCHK(x)                                                                        \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) throw HipError{std::string(#x) + ": " + hipGetErrorString(e_)}; \
  } while (0)

// one disruption candidate: <U> Candidate.instanceType / capacityType and
// getCandidatePrices' c.instanceType.Offerings.Compatible(labels).Cheapest()
struct CandInfo {
  bool priced = false;
  double price = 0;
  std::string it_name;
  bool spot = false;
};
struct CandTable {
  std::unordered_map<uint32_t, CandInfo> node;  // candidate node index -> info
  std::vector<std::string> it_name;              // catalog index -> instance-type name
  // NodePool minValues (<U> SatisfiesMinValues in
  // RemoveInstanceTypeOptionsByPriceAndMinValues): per NodePool the (key,
  // minimum) pairs, per instance type its values of those keys
  std::vector<std::vector<std::pair<std::string, int64_t>>> np_mv;
  std::vector<std::map<std::string, std::vector<std::string>>> it_vals;
};
bool mv_satisfied(const CandTable& t, uint32_t nodepool, const uint32_t* its, size_t n);

// The simulations of one gs_consolidate call (device-side layout: layout.hpp
// DevProblem consolidation fields).
struct SimPlan {
  std::vector<std::vector<uint32_t>> sets;  // candidate node indices (gs_problem order) per simulation
  std::vector<uint32_t> evaluated;          // simulations of this shard, in order
  std::vector<uint32_t> pod_off, pods;      // per evaluated simulation: pod ids in queue order
  std::vector<uint32_t> cand_off, cands;    // per evaluated simulation: device node positions removed
  uint32_t max_pods = 0, ov_cap = 0, blocks = 0, nt = 256;
  bool sim_lds = false;                     // per-simulation queue arrays and add log in LDS
  std::vector<uint64_t> known;              // per evaluated simulation: zone domains known without its candidates
  uint32_t multi_max = 0;                   // MULTI: firstNConsolidationOption's max
};

}  // namespace gsc

struct gs_ctx {
  int device = 0;
  uint32_t cfg_flags = 0;  // gs_config.flags
  std::vector<gs_ctx*> shards;  // gs_config.n_shards > 1: one child context per shard (multi.cpp)
  std::vector<ncclComm_t> comms;  // GS_CFG_RCCL: one communicator rank per shard (ncclCommInitAll)
  std::string err;
  hipStream_t stream = nullptr;
  hipEvent_t ev[8] = {};
  std::vector<void*> allocs;
  gsh::Encoded enc;
  gsd::DevProblem dp{};
  bool prepared = false, ran = false;
  bool wave = false;  // the prepared Solve runs the single-wave kernel
  bool ch = false;    // ... with its claim scan state in HBM (grown past the LDS NodeClaims)
  uint32_t n_nodepools = 0;  // of the prepared problem (the caller's arrays are not kept)
  double t_encode = 0, t_upload = 0, t_feas = 0, t_ffd = 0, t_trunc = 0, t_fetch = 0, t_run_wall = 0;
  // result storage
  std::vector<uint32_t> claim_nodepool, claim_pod_offsets, claim_pods, claim_it_offsets, claim_its;
  std::vector<std::string> req_text;
  std::vector<const char*> req_ptrs;
  std::vector<int64_t> claim_requests;
  std::vector<uint32_t> node_pod_offsets, node_pods, error_pods;
  std::vector<uint64_t> f_rows;
  std::vector<int32_t> f_cheapest;
  std::vector<uint32_t> f_nfo;
  std::vector<uint64_t> f_key;
  std::vector<uint32_t> f_var_of_pod, f_tmpl_np;
  gsd::Ctrl ctrl{};
  // consolidation: the combined problem (pending ++ bound pods), the plan,
  // the input copy (rerun) and result storage
  std::vector<gs_pod> cons_pods;
  gs_problem cons_problem{};
  gs_consolidation cons_in{};
  std::vector<uint32_t> cons_cands;
  std::vector<gs_range> cons_sets;
  uint32_t n_pending = 0;
  gsc::SimPlan sims;
  gsc::CandTable cand_table;
  std::vector<gs_command> commands;
  std::vector<uint32_t> cmd_options;
  std::vector<double> cmd_prices;
  std::vector<uint32_t> multi_opts;
  bool cons_ready = false;
  // pinned per-simulation result staging (allocated with the plan)
  gsd::SimCtrl* h_ctrl = nullptr;
  std::vector<gsd::Ctrl> h_blk;  // the simulation workgroups' counter sums
  gsd::ClaimRec* h_hdr = nullptr;
  uint32_t* h_its = nullptr;
  uint32_t* h_nits = nullptr;
  double t_sim = 0;

  // gs_create_filter: grow-once device arena and result storage
  void* cf_dev = nullptr;
  size_t cf_bytes = 0;
  std::vector<uint64_t> cf_create, cf_reqs, cf_spot;
  std::vector<uint32_t> cf_n, cf_ct;
  std::vector<int32_t> cf_sel;
  double t_filter = 0;
  // gs_build_catalog result storage
  std::vector<std::string> cat_strs, cat_reasons;
  std::vector<const char*> cat_ptrs, cat_reason_ptrs;
  std::vector<uint32_t> cat_vals, cat_skipped;
  std::vector<gs_requirement> cat_reqs;
  std::vector<gs_quantity> cat_qty;
  std::vector<gs_offering> cat_offs;
  std::vector<gs_instance_type> cat_its;

  std::vector<void*> host_allocs;  // pinned staging buffers (consolidation results)
  void free_all() {
    for (void* p : allocs) (void)hipFree(p);
    allocs.clear();
    for (void* p : host_allocs) (void)hipHostFree(p);
    host_allocs.clear();
  }
  // Device buffers of one prepared problem come from ONE allocation (an arena
  // of 256-B aligned sub-buffers): large pages, few TLB entries for the
  // single-workgroup FFD kernel's gathers.  plan() records, commit() places.
  // The arena and a pinned staging image of the uploaded buffers persist
  // across prepares and only grow: commit() lays the
  // uploaded buffers out first, copies their host arrays once into the
  // pinned image and issues one H2D copy, without re-hipMalloc per prepare.
  struct Planned {
    void** dst;
    size_t bytes;
    const void* src;  // uploaded host bytes (nullptr: device-only buffer)
    bool zero;
  };
  std::vector<Planned> plan;
  std::vector<std::shared_ptr<void>> keep;  // host arrays built for one upload (live until commit)
  size_t plan_bytes = 0;
  size_t ov_hn_bytes = 0;  // the simulation overlay cells (cleared when the stamp prefix wraps)
  size_t hc_bytes = 0;     // simulations: the NodeClaim hostname-count rows (zero at rest)
  void* arena = nullptr;
  size_t arena_bytes = 0;
  void* stage = nullptr;  // pinned
  size_t stage_bytes = 0;
  template <class P>
  void alloc(P*& dst, size_t n) {
    const size_t b = std::max<size_t>(n, 1) * sizeof(P);
    plan.push_back(Planned{(void**)&dst, b, nullptr, false});
    plan_bytes += (b + 255) & ~(size_t)255;
  }
  template <class P>
  void alloc_zero(P*& dst, size_t n) {
    alloc(dst, n);
    plan.back().zero = true;
  }
  // v must live until commit(): the encoder's arrays (c->enc) or, through
  // the rvalue overload, a temporary kept here
  template <class P, class T>
  void upload(P*& dst, const std::vector<T>& v) {
    static_assert(sizeof(P) == sizeof(T), "upload type");
    alloc(dst, v.size());
    if (!v.empty()) plan.back().src = v.data();
  }
  template <class P, class T>
  void upload(P*& dst, std::vector<T>&& v) {
    auto h = std::make_shared<std::vector<T>>(std::move(v));
    keep.push_back(h);
    upload(dst, *h);
  }
  double t_stage_ms = 0, t_h2d_ms = 0;  // commit's split: host copy into the pinned image, H2D + memsets
  void commit();
};

namespace gsc {

gs_status fail(gs_ctx* c, gs_status s, const std::string& m);
gs_status prepare_one(gs_ctx* c, const gs_problem* p);  // gs_prepare on one device
gs_status prepare_from(gs_ctx* c, const gs_ctx* src);    // upload another context's encoding (shards)
void launch_feas(gs_ctx* c, uint32_t apply_limits, uint32_t w_lo = 0, uint32_t w_hi = ~0u, bool mv_rows = true);
// the static matrix of words [wb, we) on every shard, merged into the parent's device buffers
gs_status sharded_compute(gs_ctx* c, uint32_t wb, uint32_t we, double* kernel_ms, double* merge_ms);
// multi.cpp: contexts with shards
gs_status sharded_prepare(gs_ctx* c, const gs_problem* p);
gs_status sharded_consolidate(gs_ctx* c, const gs_consolidation* in, gs_consolidation_result* out);
CandTable build_cand_table(const gs_problem* p, const uint32_t* cands, uint32_t n);
int32_t choose_commands(const CandTable& t, const gs_consolidation* in, const gs_command* commands,
                        const uint32_t* options, const double* prices, std::vector<uint32_t>* multi);
gsh::Err capacity_check(const gsh::Encoded& e);
uint32_t trunc_lds_bytes(uint32_t N);
// encode output -> device arena; `sims` non-null: consolidation arenas
void upload_problem(gs_ctx* c, const SimPlan* sims);

}  // namespace gsc

inline void gs_ctx::commit() {
  using gsc::HipError;
  auto up = [](size_t b) { return (b + 255) & ~(size_t)255; };
  // uploaded buffers first (one contiguous image), then zeroed, then the rest
  size_t off_up = 0, off_zero = 0, off_rest = 0;
  for (auto& q : plan)
    if (q.src) off_up += up(q.bytes);
    else if (q.zero) off_zero += up(q.bytes);
    else off_rest += up(q.bytes);
  const size_t n_up = off_up, n_zero = off_zero, total = std::max<size_t>(n_up + n_zero + off_rest, 256);
  if (total > arena_bytes) {
    if (arena) HIPCHK(hipFree(arena));
    arena = nullptr;
    arena_bytes = 0;
    const size_t want = total + total / 4;  // headroom: a slightly larger problem reuses it
    HIPCHK(hipMalloc(&arena, want));
    arena_bytes = want;
  }
  if (n_up > stage_bytes) {
    if (stage) HIPCHK(hipHostFree(stage));
    stage = nullptr;
    stage_bytes = 0;
    const size_t want = n_up + n_up / 4;
    HIPCHK(hipHostMalloc(&stage, want, hipHostMallocDefault));
    stage_bytes = want;
  }
  char* base = (char*)arena;
  std::vector<gsh::HostCopy> copies;
  size_t a = 0, z = n_up, r = n_up + n_zero;
  for (auto& q : plan) {
    if (q.src) {
      *q.dst = base + a;
      copies.push_back({q.src, a, q.bytes});
      a += up(q.bytes);
    } else if (q.zero) {
      *q.dst = base + z;
      z += up(q.bytes);
    } else {
      *q.dst = base + r;
      r += up(q.bytes);
    }
  }
  const auto t0 = gsc::Clock::now();
  gsh::host_copy_parallel(stage, copies.data(), copies.size());
  t_stage_ms = gsc::ms_since(t0);
  const auto t1 = gsc::Clock::now();
  if (n_up) HIPCHK(hipMemcpyAsync(base, stage, n_up, hipMemcpyHostToDevice, stream));
  if (n_zero) HIPCHK(hipMemsetAsync(base + n_up, 0, n_zero, stream));
  HIPCHK(hipStreamSynchronize(stream));
  t_h2d_ms = gsc::ms_since(t1);
  static const bool prof = std::getenv("GS_ENCODE_PROFILE") != nullptr;
  if (prof)
    std::fprintf(stderr, "upload.stage %.3f ms  upload.h2d %.3f ms  (%zu B uploaded, %zu B zeroed, %zu B total)\n",
                 t_stage_ms, t_h2d_ms, n_up, n_zero, total);
  plan.clear();
  keep.clear();
  plan_bytes = 0;
}
