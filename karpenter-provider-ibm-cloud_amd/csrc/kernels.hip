// kernels.hip — gfx950 (CDNA4, wave64) kernels of the provisioning solve.
//
//  K1/K2 feas_kernel   pod-variant x template x instance-type feasibility rows
//                      (one wave per (variant, template); lane = instance type;
//                      __ballot packs 64 ITs per word) + wave argmin of the
//                      cheapest compatible offering, key (price_rank<<32|name_rank)
//  K4    ffd_kernel    (ffd.hip) the sequential Scheduler.Solve queue loop as
//                      ONE persistent workgroup, or one workgroup per
//                      consolidation simulation
//  K3    trunc_kernel  per NodeClaim: OrderByPrice + Truncate(60)
//
// All integer/bitset work: no MFMA.  Semantics cited as <U> restate
// sigs.k8s.io/karpenter@v1.13.0 ("parity").
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "devutil.hpp"
#include "layout.hpp"

using namespace gsd;

namespace {

constexpr int BLOCK = 256;

}  // namespace

// ===================================================================== K1/K2
// A wave evaluates PP = 64/LP (variant v, template t) pairs at once: lane
// group s (LP lanes, LP = the row's word count rounded up to a power of two,
// at most 64) holds pair s's row, lane wl of the group row word wl (+64 per
// extra pass when W > 64).  The row is word-parallel bitset algebra over
// instance types:
//   row = template options (static: within NodePool limits)
//       AND_r  thr_set[r][lower_bound(thr_val_r, daemon_r + pod_r)]   (Fits)
//       AND    OR_{pair g in grid(template, pod)} slot_set[g]          (offering)
//       AND    the IT-key requirement class mask (variants with IT-key
//              requirements; one mask per distinct requirement set)
// The threshold searches of all PP pairs run first, one lane per (pair,
// resource), so the dependent binary-search chains overlap instead of
// serialising per pair.  nfo = sum_g popcount(row AND slot_set[g]); the
// cheapest instance type (= OrderByPrice(...)[0]) is the first instance type
// of the pair's grid order (capi.cpp build_grid_orders) that is in the row.
// static_mode = 1 (gs_feasibility): a NodeClaim opened for the pod alone, with
// the free-key Compatible check and the NodePool limits folded into the row.
// static_mode = 0 (FFD): rows carry only the monotone predicates; the
// free-key check against the fresh template goes to fk_ok[] because an
// in-flight NodeClaim can gain keys that make a later pod compatible.
namespace {

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace

// <U> resources.Fits(Merge(daemon, pod), allocatable) cursors, one lane per
// (variant, template, resource): the first threshold >= the demand.  A pass of
// its own so that the dependent binary-search loads of all pairs overlap.
__global__ __launch_bounds__(BLOCK) void feas_cursor_kernel(DevProblem d) {
  const uint32_t R = d.R, T = d.T;
  const uint64_t id = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (id >= (uint64_t)d.V * T * R) return;
  const uint32_t r = (uint32_t)(id % R);
  const uint64_t pair = id / R;
  const uint32_t v = (uint32_t)(pair / T), t = (uint32_t)(pair % T);
  const int64_t dem = d.tmpl[t].daemon[r] + d.pod_req[(size_t)d.var_pod[v] * R + r];
  const uint32_t o = d.thr_off[r];
  d.pair_cur[id] = o + r + lower_bound_i64(d.thr_val + o, d.thr_off[r + 1] - o, dem);
}

template <uint32_t LP>
__global__ __launch_bounds__(BLOCK) void feas_kernel(DevProblem d, uint32_t static_mode, uint32_t w_lo,
                                                     uint32_t w_hi) {
  constexpr uint32_t PP = 64 / LP;
  __shared__ uint64_t s_row[BLOCK / 64][256];  // the wave's rows (PP x W words, or the first 256 when LP = 64)
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t sub = lane / LP, wl = lane % LP;
  const uint32_t VT = d.V * d.T;
  const uint32_t pair0 = __builtin_amdgcn_readfirstlane((blockIdx.x * (BLOCK / 64) + wv) * PP);
  if (pair0 >= VT) return;  // wave-uniform
  const uint32_t W = d.W, OW = d.OW, R = d.R, T = d.T;

  const uint32_t pair = pair0 + sub;
  const bool valid = pair < VT;
  const uint32_t v = valid ? pair / T : 0, t = valid ? pair % T : 0;
  const VarRec& vr = d.vars[v];
  const TmplRec& tr = d.tmpl[t];
  // per-pair parts of NodeClaim.CanAdd on a fresh NodeClaim (uniform in the group)
  bool ok_all = valid && (tr.taints & ~vr.tol) == 0;  // <U> Taints.ToleratesPod
  const bool fk_ok = valid && var_fk_ok(d, vr, d.t_fk + (size_t)t * d.F);
  if (static_mode) ok_all = ok_all && fk_ok;
  const uint64_t G = grid_of(tr.zm & vr.zm, tr.cm & vr.cm, d.Z, d.C), Gt = grid_of(tr.zm, tr.cm, d.Z, d.C);
  if (!G) ok_all = false;
  // <U> compatible(it, reqs): it.Requirements.Intersects(reqs) on IT keys,
  // precomputed per distinct IT-key requirement set (encoder classes)
  const uint32_t itc = valid ? d.var_itclass[v] : NONE;
  const uint64_t* itmask = itc != NONE ? d.itclass_mask + (size_t)itc * W : nullptr;
  const uint64_t* topts = (static_mode && tr.has_limits ? d.t_limopts : d.t_opts) + (size_t)t * W;
  uint64_t* rowout = d.rows + (size_t)pair * OW;
  uint32_t cur[RMAX];
#pragma unroll
  for (uint32_t r = 0; r < RMAX; r++) cur[r] = valid && r < R ? d.pair_cur[(size_t)pair * R + r] : 0u;
  // static matrix: the pair's grid in the OrderByPrice tables (capi.cpp build_grid_orders)
  uint32_t gi = 0;
  if (static_mode) {
    uint32_t lo = 0, hi = d.n_grids;
    while (lo < hi) {
      const uint32_t m = (lo + hi) >> 1;
      if (d.grid_list[m] < G) lo = m + 1;
      else hi = m;
    }
    gi = lo;
  }
  const uint64_t* planes = d.grid_planes + (size_t)gi * d.n_planes * W;

  uint32_t nf = 0;
  uint64_t any = 0;
  uint64_t xr[2] = {0, 0};  // this lane's row words wl and wl + LP (W <= 2 LP)
  for (uint32_t w0 = 0; w0 < W; w0 += LP) {
    const uint32_t w = w0 + wl;
    uint64_t x = 0;
    if (ok_all && w < W && w >= w_lo && w < w_hi) {  // this instance-type column shard
      x = topts[w];
#pragma unroll
      for (uint32_t r = 0; r < RMAX; r++)
        if (r < R) x &= d.thr_set[(size_t)cur[r] * OW + w];
      if (G != Gt) {  // template options already have an offering on the template's grid
        uint64_t off = 0;
        for (uint64_t m = G; m; m &= m - 1) off |= d.slot_set[(size_t)(__ffsll((long long)m) - 1) * W + w];
        x &= off;
      }
      if (itmask) x &= itmask[w];
    }
    if (valid && w < W) {
      rowout[w] = x;
      // the pair's row words in LDS for the cheapest-offering scan (PP x W <= 256)
      if (LP < 64) s_row[wv][sub * W + w] = x;
      else if (w < 256) s_row[wv][w] = x;
      // offerings: sum over grid pairs of row AND slot_set[g]
      // (the Solve's rows need neither the offering count nor the cheapest type)
      if (static_mode && G)
        for (uint32_t b = 0; b < d.n_planes; b++) nf += (uint32_t)__popcll(x & planes[(size_t)b * W + w]) << b;
    }
    if (w0 == 0) xr[0] = x;
    else if (w0 == LP) xr[1] = x;
    any |= x;
  }
  // group reductions (LP lanes, xor partners stay inside the group)
#pragma unroll
  for (uint32_t m = LP / 2; m >= 1; m >>= 1) nf += (uint32_t)__shfl_xor((int)nf, (int)m);
  const uint64_t nonempty = __ballot(any != 0);
  wave_lds_sync();
  uint32_t cheapest = NONE;
  uint64_t ckey = 0x7FFFFFFFFFFFFFFFull;  // INT64_MAX: none
  if (static_mode) {
    // <U> OrderByPrice(...)[0]: the pair's grid G indexes a list of the
    // instance types with an available offering in G, sorted by (min price
    // rank over G, name rank); the first one in the row is the cheapest.
    // Every lane group scans its own pair's list, KS x LP keys per step.
#ifndef GS_K1_KS
#define GS_K1_KS 2
#endif
    constexpr uint32_t KS = LP >= 16 ? GS_K1_KS : (64 / LP > 8 ? 8 : 64 / LP);
    const uint64_t gmask = (LP == 64 ? ~0ull : ((1ull << LP) - 1)) << (sub * LP);
    const uint32_t kb = d.grid_off[gi], ke = d.grid_off[gi + 1];
    const uint64_t* srow = s_row[wv] + (LP < 64 ? sub * W : 0);
    bool active = valid && ((nonempty & gmask) != 0);
#ifndef GS_K1_BLOCKS
#define GS_K1_BLOCKS 1
#endif
    if (GS_K1_BLOCKS && d.grid_blocks) {
      // rank blocks: the first block of the grid's list the row intersects
      // (8 blocks per step, every block one AND per row word), then the first
      // list entry of that block in the row
      const uint32_t NB = d.grid_nb;
      const uint64_t* Bg = d.grid_blocks + (size_t)gi * NB * W;
      const uint32_t nbg = (ke - kb + 63) / 64;
      uint32_t fk = NONE;
      for (uint32_t k0 = 0; __ballot(active); k0 += 8) {
        uint32_t hm = 0;
        if (active) {
#pragma unroll
          for (uint32_t q = 0; q < 8; q++) {
            const uint32_t k = k0 + q;
            if (k < nbg) {
              const uint64_t* bk = Bg + (size_t)k * W;
              bool h = wl < W && (xr[0] & bk[wl]) != 0;
              if (wl + LP < W) h = h || (xr[1] & bk[wl + LP]) != 0;
              hm |= h ? 1u << q : 0u;
            }
          }
        }
#pragma unroll
        for (uint32_t m = LP / 2; m >= 1; m >>= 1) hm |= (uint32_t)__shfl_xor((int)hm, (int)m);
        if (active && hm) {
          fk = k0 + (uint32_t)__ffs((int)hm) - 1;
          active = false;
        }
        if (k0 + 8 >= nbg) active = false;
      }
      const uint32_t p0 = kb + 64 * (fk != NONE ? fk : 0u);
      uint32_t best = NONE;
#pragma unroll
      for (uint32_t e = 0; e < 64; e += LP) {
        const uint32_t j = p0 + e + wl;
        if (fk != NONE && e + wl < 64 && j < ke) {
          const uint32_t it = d.grid_its[j];
          if (((srow[it >> 6] >> (it & 63)) & 1) && e + wl < best) best = e + wl;
        }
      }
#pragma unroll
      for (uint32_t m = LP / 2; m >= 1; m >>= 1) {
        const uint32_t y = (uint32_t)__shfl_xor((int)best, (int)m);
        best = y < best ? y : best;
      }
      if (fk != NONE && best != NONE) {
        cheapest = d.grid_its[p0 + best];
        ckey = d.grid_keys[p0 + best];
      }
      active = false;
    }
    for (uint32_t base = kb; __ballot(active); base += KS * LP) {
      uint32_t it[KS];
      bool hit[KS];
#pragma unroll
      for (uint32_t k = 0; k < KS; k++) {
        const uint32_t j = base + k * LP + wl;
        it[k] = active && j < ke ? d.grid_its[j] : NONE;
      }
#pragma unroll
      for (uint32_t k = 0; k < KS; k++) hit[k] = it[k] != NONE && ((srow[it[k] >> 6] >> (it[k] & 63)) & 1);
      uint32_t first = NONE;
#pragma unroll
      for (uint32_t k = 0; k < KS; k++) {
        const uint64_t bk = __ballot(hit[k]) & gmask;
        if (first == NONE && bk) first = k * LP + ((uint32_t)__ffsll((long long)bk) - 1 - sub * LP);
      }
      if (active && first != NONE) {
        const uint32_t j = base + first;
        cheapest = d.grid_its[j];
        ckey = d.grid_keys[j];
        active = false;
      }
      if (base + KS * LP >= ke) active = false;
    }
  }
  if (valid && wl == 0) {
    d.fk_ok[pair] = fk_ok ? 1u : 0u;
    d.nfo[pair] = nf;
    d.cheapest[pair] = cheapest;
    if (static_mode) d.cheapest_key[pair] = ckey;
  }
}

// ========================================================================= K3
// <U> InstanceTypes.OrderByPrice(reqs) + Truncate(60): key per option IT =
// (rank of its cheapest available compatible offering price, name rank)
// Consolidation simulations (n_sims > 0): block s truncates the NodeClaim of
// simulation s when it opened exactly one (the only case computeConsolidation
// prices); output slot s.  With minValues (all_slots): block j truncates
// NodeClaim arena slot j of whichever simulation holds it and flags a top 60
// that misses a minimum (<U> Results.TruncateInstanceTypes drops it); the
// sim_fix kernel then settles each simulation.
extern "C" __global__ __launch_bounds__(BLOCK) void trunc_kernel(DevProblem d, uint32_t all_slots) {
  extern __shared__ uint64_t keys[];
  __shared__ uint32_t cnt;
  uint32_t j = blockIdx.x;  // claim
  const uint32_t o = blockIdx.x;  // output slot
  if (all_slots) {
    // the simulation whose arena holds slot j: last s with sim_pod_off[s] <= j
    uint32_t lo = 0, hi = d.n_sims;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (d.sim_pod_off[mid] <= j) lo = mid;
      else hi = mid;
    }
    if (j >= d.sim_pod_off[d.n_sims] || d.sim_ctrl[lo].status != 0 || j - d.sim_pod_off[lo] >= d.sim_ctrl[lo].n_claims)
      return;
  } else if (d.n_sims) {
    if (o >= d.n_sims || d.sim_ctrl[o].status != 0 || d.sim_ctrl[o].n_claims != 1) return;
    j = d.sim_pod_off[o];
  } else if (j >= d.ctrl->n_claims) {
    return;
  }
  const uint32_t tid = threadIdx.x;
  const ClaimRec& h = d.c_rec[j];
  const uint64_t G = grid_of(h.zm, h.cm, d.Z, d.C);
  if (tid == 0) cnt = 0;
  __syncthreads();
  for (uint32_t i = tid; i < d.N; i += BLOCK) {
    if (!((d.c_opts[(size_t)j * d.OW + (i >> 6)] >> (i & 63)) & 1)) continue;
    uint32_t minp = NONE;
    uint64_t m = d.it_pair[i] & G;
    while (m) {
      const uint32_t g = __ffsll((long long)m) - 1;
      m &= m - 1;
      const uint32_t pr = d.it_prank[(size_t)i * 64 + g];
      minp = pr < minp ? pr : minp;
    }
    const uint32_t slot = atomicAdd(&cnt, 1u);
    keys[slot] = ((uint64_t)minp << 32) | d.it_namerank[i];
  }
  __syncthreads();
  const uint32_t n = cnt;
  uint32_t np2 = 1;
  while (np2 < n) np2 <<= 1;
  for (uint32_t i = n + tid; i < np2; i += BLOCK) keys[i] = ~0ull;
  __syncthreads();
  // bitonic sort of np2 keys
  for (uint32_t k = 2; k <= np2; k <<= 1) {
    for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
      for (uint32_t i = tid; i < np2; i += BLOCK) {
        const uint32_t ixj = i ^ jj;
        if (ixj > i) {
          const uint64_t a = keys[i], b = keys[ixj];
          const bool up = (i & k) == 0;
          if ((a > b) == up) {
            keys[i] = b;
            keys[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  const uint32_t take = n < 60 ? n : 60;
  if (all_slots) {
    for (uint32_t i = tid; i < take; i += BLOCK) d.slot_its[(size_t)j * 60 + i] = d.rank_to_it[(uint32_t)keys[i]];
    if (tid == 0) {
      d.slot_nits[j] = take;
      // SatisfiesMinValues on the top 60: distinct values per minimum key
      const TmplRec& tr = d.tmpl[h.tmpl];
      bool ok = true;
      for (uint32_t mm = tr.mv_mask; mm && ok; mm &= mm - 1) {
        const uint32_t k = (uint32_t)__builtin_ctz(mm);
        uint32_t nd = take;
        if (!((d.it_key_unique >> k) & 1)) {
          uint64_t sv[4] = {0, 0, 0, 0};
          nd = 0;
          for (uint32_t i = 0; i < take; i++) {
            const uint32_t x = d.it_dvid[(size_t)k * d.N + d.rank_to_it[(uint32_t)keys[i]]];
            const uint64_t bit = 1ull << (x & 63);
            if (!(sv[x >> 6] & bit)) {
              sv[x >> 6] |= bit;
              nd++;
            }
          }
        }
        ok = nd >= tr.mv[k];
      }
      d.slot_drop[j] = ok ? 0u : 1u;
    }
    return;
  }
  if (d.n_sims && tid < sizeof(ClaimRec) / 4) ((uint32_t*)(d.sim_hdr + o))[tid] = ((const uint32_t*)&h)[tid];
  for (uint32_t i = tid; i < take; i += BLOCK) d.c_its[(size_t)o * 60 + i] = d.rank_to_it[(uint32_t)keys[i]];
  if (tid == 0) d.c_nits[o] = take;
}

// Simulations with minValues: <U> Results.TruncateInstanceTypes drops every
// NodeClaim flagged by trunc_kernel (all_slots); their pods become pod errors,
// which count against the simulation when not pending
// (AllNonPendingPodsScheduled).  One thread per simulation: the surviving
// count, the failed pods, and the single survivor's header and top 60 in the
// per-simulation output slot.
extern "C" __global__ __launch_bounds__(BLOCK) void sim_fix_kernel(DevProblem d) {
  const uint32_t s = blockIdx.x * BLOCK + threadIdx.x;
  if (s >= d.n_sims) return;
  SimCtrl& c = d.sim_ctrl[s];
  if (c.status) return;
  const uint32_t off = d.sim_pod_off[s], nc = c.n_claims;
  uint32_t surv = 0, sj = NONE;
  bool drop = false;
  for (uint32_t j = 0; j < nc; j++) {
    if (d.slot_drop[off + j]) {
      drop = true;
    } else {
      if (!surv) sj = j;
      surv++;
    }
  }
  if (drop) {
    uint32_t extra = 0;
    for (uint32_t i = 0; i < c.n_log; i++) {
      const LogRec l = d.log[off + i];
      if (!(l.target & 0x80000000u) && d.slot_drop[off + l.target] && l.pod >= d.n_pending) extra++;
    }
    c.failed += extra;
  }
  c.n_claims = surv;
  if (surv == 1) {
    const uint32_t* src = (const uint32_t*)(d.c_rec + off + sj);
    uint32_t* dst = (uint32_t*)(d.sim_hdr + s);
    for (uint32_t q = 0; q < sizeof(ClaimRec) / 4; q++) dst[q] = src[q];
    const uint32_t nt = d.slot_nits[off + sj];
    for (uint32_t i = 0; i < nt; i++) d.c_its[(size_t)s * 60 + i] = d.slot_its[(size_t)(off + sj) * 60 + i];
    d.c_nits[s] = nt;
  }
}

// ------------------------------------------------------------ host launchers
extern "C" hipError_t gsk_init_trunc(uint32_t trunc_lds_bytes) {
  return hipFuncSetAttribute((const void*)trunc_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)trunc_lds_bytes);
}

template <uint32_t LP>
static void launch_feas_lp(const DevProblem* d, uint32_t static_mode, uint32_t w_lo, uint32_t w_hi, hipStream_t s) {
  const uint64_t pairs = (uint64_t)d->V * d->T;
  const uint64_t per_block = (BLOCK / 64) * (64 / LP);
  const uint32_t blocks = (uint32_t)((pairs + per_block - 1) / per_block);
  hipLaunchKernelGGL(feas_kernel<LP>, dim3(blocks), dim3(BLOCK), 0, s, *d, static_mode, w_lo, w_hi);
}

extern "C" hipError_t gsk_feas(const DevProblem* d, uint32_t static_mode, uint32_t w_lo, uint32_t w_hi,
                               hipStream_t s) {
  if (!d->V || !d->T) return hipSuccess;
  const uint64_t nc = (uint64_t)d->V * d->T * d->R;
  if (nc) hipLaunchKernelGGL(feas_cursor_kernel, dim3((uint32_t)((nc + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s, *d);
  // lanes per pair: the row's word count rounded up to a power of two, at
  // most GS_K1_LPMAX (a lane then takes W / LP words; PP x W <= 256 keeps the
  // pairs' rows in the wave's LDS slice).  The kernel is a chain of dependent
  // loads per wave: more pairs per wave is fewer chains.  C5 (W = 32), same
  // session: LP 32 0.1268 ms, 16 0.1200, 8 0.1354 (profiles/r5/k1_lanes_ab.txt)
#ifndef GS_K1_LPMAX
#define GS_K1_LPMAX 16
#endif
  uint32_t W = d->W;
  if (GS_K1_LPMAX < 64 && W > GS_K1_LPMAX && W <= 32 && W * (64 / GS_K1_LPMAX) <= 256) W = GS_K1_LPMAX;
  if (W <= 1) launch_feas_lp<1>(d, static_mode, w_lo, w_hi, s);
  else if (W <= 2) launch_feas_lp<2>(d, static_mode, w_lo, w_hi, s);
  else if (W <= 4) launch_feas_lp<4>(d, static_mode, w_lo, w_hi, s);
  else if (W <= 8) launch_feas_lp<8>(d, static_mode, w_lo, w_hi, s);
  else if (W <= 16) launch_feas_lp<16>(d, static_mode, w_lo, w_hi, s);
  else if (W <= 32) launch_feas_lp<32>(d, static_mode, w_lo, w_hi, s);
  else launch_feas_lp<64>(d, static_mode, w_lo, w_hi, s);
  return hipGetLastError();
}

// <U> minValues (Strict) on the static matrix: a fresh NodeClaim whose
// options miss a template minimum is not addable, so its row is empty (no
// cheapest type, no offering).  One wave per (variant, template) pair whose
// template carries minValues; lane w holds words w, w + 64, ...
__global__ __launch_bounds__(BLOCK) void mv_rows_kernel(DevProblem d) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t pair = __builtin_amdgcn_readfirstlane(blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6));
  if (pair >= d.V * d.T) return;  // wave-uniform
  const TmplRec& tr = d.tmpl[pair % d.T];
  if (!tr.mv_mask) return;
  uint64_t* row = d.rows + (size_t)pair * d.OW;
  bool ok = true;
  for (uint32_t mm = tr.mv_mask; mm && ok; mm &= mm - 1) {
    const uint32_t k = (uint32_t)__builtin_ctz(mm);
    uint32_t n = 0;
    if ((d.it_key_unique >> k) & 1) {
      for (uint32_t w = lane; w < d.W; w += 64) n += (uint32_t)__popcll(row[w]);
      n = wave_sum_u32(n);
    } else {
      const uint16_t* dv = d.it_dvid + (size_t)k * d.N;
      uint64_t sv[4] = {0, 0, 0, 0};
      for (uint32_t w = lane; w < d.W; w += 64)
        for (uint64_t m = row[w]; m; m &= m - 1) {
          const uint32_t x = dv[w * 64 + (uint32_t)__builtin_ctzll(m)];
#pragma unroll
          for (uint32_t q = 0; q < 4; q++) sv[q] |= (x >> 6) == q ? 1ull << (x & 63) : 0ull;
        }
#pragma unroll
      for (uint32_t q = 0; q < 4; q++) {
        for (int o = 32; o >= 1; o >>= 1) sv[q] |= shfl_xor_u64(sv[q], o);
        n += (uint32_t)__popcll(sv[q]);
      }
    }
    ok = n >= tr.mv[k];
  }
  if (ok) return;
  for (uint32_t w = lane; w < d.W; w += 64) row[w] = 0;
  if (lane == 0) {
    d.nfo[pair] = 0;
    d.cheapest[pair] = NONE;
    d.cheapest_key[pair] = 0x7FFFFFFFFFFFFFFFull;
  }
}

extern "C" hipError_t gsk_mv_rows(const DevProblem* d, hipStream_t s) {
  const uint64_t pairs = (uint64_t)d->V * d->T;
  if (!pairs) return hipSuccess;
  hipLaunchKernelGGL(mv_rows_kernel, dim3((uint32_t)((pairs + BLOCK / 64 - 1) / (BLOCK / 64))), dim3(BLOCK), 0, s, *d);
  return hipGetLastError();
}

// ==================================================== shard merge (multi-GPU)
// A sharded context's static matrix: shard k computed instance-type words
// [lo_k, hi_k) of every (variant, template) row on its own device.  One
// kernel on the parent's device gathers each word from the shard that owns
// it (peer loads over xGMI, or local memory when a device repeats), adds the
// per-shard offering counts and keeps the minimum OrderByPrice key (the
// cheapest offering's instance type is the key's name rank).  With RCCL the
// counts and keys were all-reduced already: shard 0's are final (K_red = 1).
extern "C" __global__ __launch_bounds__(BLOCK) void merge_shards_kernel(ShardMerge m) {
  const size_t stride = (size_t)gridDim.x * BLOCK, i0 = (size_t)blockIdx.x * BLOCK + threadIdx.x;
  const uint32_t nw = m.we - m.wb;
  for (size_t i = i0; i < (size_t)m.VT * nw; i += stride) {
    const size_t vt = i / nw;
    const uint32_t w = m.wb + (uint32_t)(i % nw);
    uint32_t k = 0;
    while (k + 1 < m.K && w >= m.src[k].hi) k++;
    m.rows[vt * m.OW + w] = m.src[k].rows[vt * m.OW + w];
  }
  for (size_t vt = i0; vt < m.VT; vt += stride) {
    uint32_t n = 0;
    uint64_t key = 0x7FFFFFFFFFFFFFFFull;
    for (uint32_t k = 0; k < m.K_red; k++) {
      n += m.src[k].nfo[vt];
      const uint64_t x = m.src[k].key[vt];
      key = x < key ? x : key;
    }
    m.nfo[vt] = n;
    m.key[vt] = key;
    m.cheapest[vt] = key == 0x7FFFFFFFFFFFFFFFull ? NONE : m.rank_to_it[(uint32_t)key];
  }
}

extern "C" hipError_t gsk_merge_shards(const ShardMerge* m, hipStream_t s) {
  const size_t work = (size_t)m->VT * (m->we - m->wb > 0 ? m->we - m->wb : 1);
  const uint32_t grid = (uint32_t)std::min<size_t>((work + BLOCK - 1) / BLOCK, 8192);
  hipLaunchKernelGGL(merge_shards_kernel, dim3(grid ? grid : 1), dim3(BLOCK), 0, s, *m);
  return hipGetLastError();
}

// simulations with minValues (any_mv): every NodeClaim arena slot, then the
// per-simulation settlement; otherwise one block per simulation / NodeClaim
extern "C" hipError_t gsk_trunc(const DevProblem* d, uint32_t lds_bytes, uint32_t n_slots, hipStream_t s) {
  if (d->n_sims && d->any_mv) {
    if (!n_slots) return hipSuccess;
    hipLaunchKernelGGL(trunc_kernel, dim3(n_slots), dim3(BLOCK), lds_bytes, s, *d, 1u);
    hipLaunchKernelGGL(sim_fix_kernel, dim3((d->n_sims + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, *d);
    return hipGetLastError();
  }
  const uint32_t grid = d->n_sims ? d->n_sims : d->claim_cap;
  if (!grid) return hipSuccess;
  hipLaunchKernelGGL(trunc_kernel, dim3(grid), dim3(BLOCK), lds_bytes, s, *d, 0u);
  return hipGetLastError();
}
