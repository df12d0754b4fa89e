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

#include "devutil.hpp"
#include "layout.hpp"

using namespace gsd;

namespace {

constexpr int BLOCK = 256;

}  // namespace

// ===================================================================== K1/K2
// one wave per (variant v, template t); lane i of step w = instance type w*64+i
// static_mode = 1 (gs_feasibility): a NodeClaim opened for the pod alone, with
// the free-key Compatible check and the NodePool limits folded into the row.
// static_mode = 0 (FFD): rows carry only the monotone predicates (taints, IT
// requirements, fits, offerings); the free-key check against the fresh
// template goes to fk_ok[] because an in-flight NodeClaim can gain keys that
// make a later pod compatible.
extern "C" __global__ __launch_bounds__(BLOCK) void feas_kernel(DevProblem d, uint32_t static_mode) {
  const uint32_t lane = threadIdx.x & 63;
  // wave-uniform in SGPRs: the variant record is read in place (scalar
  // loads), never copied into a dynamically indexed private array (scratch)
  const uint32_t pair = __builtin_amdgcn_readfirstlane(blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6));
  if (pair >= d.V * d.T) return;  // wave-uniform
  const uint32_t v = pair / d.T, t = pair % d.T;
  const VarRec& vr = d.vars[v];
  const TmplRec& tr = d.tmpl[t];
  uint64_t* rowout = d.rows + (size_t)pair * d.OW;

  // wave-uniform parts of NodeClaim.CanAdd on a fresh NodeClaim
  bool ok_all = (tr.taints & ~vr.tol) == 0;  // <U> Taints.ToleratesPod
  const bool fk_ok = var_fk_ok(d, vr, d.t_fk + (size_t)t * d.F);
  if (static_mode) ok_all = ok_all && fk_ok;
  int64_t dem[RMAX];
  const int64_t* preq = d.pod_req + (size_t)vr.pod * d.R;
#pragma unroll
  for (uint32_t r = 0; r < RMAX; r++) dem[r] = r < d.R ? tr.daemon[r] + preq[r] : 0;  // Merge(daemon, pod)
  const uint64_t G = grid_of(tr.zm & vr.zm, tr.cm & vr.cm, d.Z, d.C);
  const bool lim = static_mode && tr.has_limits;

  uint64_t best = ~0ull;
  uint32_t nf = 0;
  for (uint32_t w = 0; w < d.W; w++) {
    const uint32_t i = w * 64 + lane;
    bool ok = ok_all && i < d.N && ((d.t_opts[(size_t)t * d.W + w] >> lane) & 1);
    if (ok) {
      // <U> compatible(it, reqs): it.Requirements.Intersects(reqs) on IT keys
      for (uint32_t k = 0; k < d.K; k++) {
        const uint32_t off = vr.itmask_off[k];
        if (off == NONE) continue;
        const uint32_t vid = d.it_vid[(size_t)k * d.N + i];
        ok = ok && ((d.itmask[off + (vid >> 6)] >> (vid & 63)) & 1);
      }
    }
    if (ok) {
      // <U> resources.Fits(requests, it.Allocatable())
#pragma unroll
      for (uint32_t r = 0; r < RMAX; r++) ok = ok && (r >= d.R || d.it_alloc[(size_t)r * d.N + i] >= dem[r]);
    }
    if (ok && lim) {
      // <U> filterByRemainingResources
      for (uint32_t r = 0; r < d.R; r++)
        if ((tr.limit_rmask >> r) & 1) ok = ok && d.it_cap[(size_t)r * d.N + i] <= tr.limits[r];
    }
    // <U> offering.Available && reqs.IsCompatible(offering.Requirements)
    const uint64_t pm = ok ? (d.it_pair[i] & G) : 0;
    ok = pm != 0;
    const uint64_t word = __ballot(ok);
    if (lane == 0) rowout[w] = word;
    if (ok) {
      nf += __popcll(pm);
      uint32_t minp = NONE;
      uint64_t m = pm;
      while (m) {
        const uint32_t g = __ffsll((long long)m) - 1;
        m &= m - 1;
        const uint32_t pr = d.it_prank[(size_t)i * 64 + g];
        minp = pr < minp ? pr : minp;
      }
      const uint64_t key = ((uint64_t)minp << 32) | d.it_namerank[i];
      best = key < best ? key : best;
    }
  }
  best = wave_min_u64(best);
  nf = wave_sum_u32(nf);
  if (lane == 0) {
    d.fk_ok[pair] = fk_ok ? 1u : 0u;
    d.nfo[pair] = nf;
    d.cheapest[pair] = best == ~0ull ? NONE : d.rank_to_it[(uint32_t)best];
  }
}

// ========================================================================= K3
// <U> InstanceTypes.OrderByPrice(reqs) + Truncate(60): key per option IT =
// (rank of its cheapest available compatible offering price, name rank)
// Consolidation simulations (n_sims > 0): block s truncates the NodeClaim of
// simulation s when it opened exactly one (the only case computeConsolidation
// prices); output slot s.
extern "C" __global__ __launch_bounds__(BLOCK) void trunc_kernel(DevProblem d) {
  extern __shared__ uint64_t keys[];
  __shared__ uint32_t cnt;
  uint32_t j = blockIdx.x;  // claim
  const uint32_t o = blockIdx.x;  // output slot
  if (d.n_sims) {
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
  if (d.n_sims && tid < sizeof(ClaimRec) / 4) ((uint32_t*)(d.sim_hdr + o))[tid] = ((const uint32_t*)&h)[tid];
  for (uint32_t i = tid; i < take; i += BLOCK) d.c_its[(size_t)o * 60 + i] = d.rank_to_it[(uint32_t)keys[i]];
  if (tid == 0) d.c_nits[o] = take;
}

// ------------------------------------------------------------ host launchers
extern "C" hipError_t gsk_init_trunc(uint32_t trunc_lds_bytes) {
  return hipFuncSetAttribute((const void*)trunc_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)trunc_lds_bytes);
}

extern "C" hipError_t gsk_feas(const DevProblem* d, uint32_t static_mode, hipStream_t s) {
  const uint64_t pairs = (uint64_t)d->V * d->T;
  if (!pairs) return hipSuccess;
  const uint32_t blocks = (uint32_t)((pairs + (BLOCK / 64) - 1) / (BLOCK / 64));
  hipLaunchKernelGGL(feas_kernel, dim3(blocks), dim3(BLOCK), 0, s, *d, static_mode);
  return hipGetLastError();
}


extern "C" hipError_t gsk_trunc(const DevProblem* d, uint32_t lds_bytes, hipStream_t s) {
  const uint32_t grid = d->n_sims ? d->n_sims : d->max_claims;
  if (!grid) return hipSuccess;
  hipLaunchKernelGGL(trunc_kernel, dim3(grid), dim3(BLOCK), lds_bytes, s, *d);
  return hipGetLastError();
}
