// ffd_wave.hip — K4 provisioning Solve as ONE wave: the state reset kernel,
// the launcher (the kernel template is in ffd_wave.hpp, its instantiations
// in ffd_wave_r.hip) and the autoplacement ranking sort.
#include "ffd_wave.hpp"

using namespace gsd;

// Grid-wide reset of the Solve's working state (queue, per-pod counters,
// NodePool remaining limits, existing-node copies, hostname counts): the
// single-wave kernel starts from it.
extern "C" __global__ __launch_bounds__(256) void ffd_init_kernel(DevProblem d) {
  const uint32_t stride = gridDim.x * blockDim.x;
  const uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x;
  for (uint32_t i = i0; i < d.P; i += stride) {
    d.queue[i] = d.queue0[i];
    d.last_epoch[i] = 0;
    d.last_len[i] = 0;
    d.cur_var[i] = d.var_begin[i];
  }
  for (uint32_t i = i0; i < d.T * d.R; i += stride) d.t_rem[i] = d.tmpl[i / d.R].limits[i % d.R];
  for (uint32_t i = i0; i < d.NN; i += stride) d.nodes[i] = d.nodes0[i];
  for (uint32_t i = i0; i < d.NN * d.F; i += stride) d.n_fk[i] = d.n_fk0[i];
  for (uint32_t i = i0; i < d.TGH * d.NN; i += stride) d.hn[i] = d.hn0[i];
  if (d.any_vol)
    for (uint32_t i = i0; i < d.NN; i += stride) d.n_vol[i] = d.n_vol0[i];
}


// ---------------------------------------------------------------- launchers
// The kernel instantiations live in ffd_wave_r.hip, one translation unit per
// (R, TOPO): each exports its launcher and its LDS attribute setter.
extern "C" uint32_t gsk_ffd_lds_bytes(uint32_t max_claims, uint32_t nthr, uint32_t nb_words,
                                      uint32_t topo_bytes);
#define GSK_DECL(n, t)                                                                                  \
  extern "C" hipError_t gsk_ffdw_launch_r##n##_t##t(const DevProblem* d, uint32_t mode, uint32_t lds, hipStream_t s); \
  extern "C" hipError_t gsk_ffdw_attr_r##n##_t##t(uint32_t lds_total, uint32_t* dyn_min);
#define GSK_DECL2(n) GSK_DECL(n, 0) GSK_DECL(n, 1)
GSK_DECL2(1) GSK_DECL2(2) GSK_DECL2(3) GSK_DECL2(4) GSK_DECL2(5) GSK_DECL2(6) GSK_DECL2(7) GSK_DECL2(8)
#undef GSK_DECL2
#undef GSK_DECL
static uint32_t g_ffdw_dyn_max = 0;

extern "C" hipError_t gsk_init_ffdw(uint32_t lds_total) {
  hipError_t e = hipSuccess;
  uint32_t dmin = 0;
#define GSK_ATTR(n, t) \
  if (hipError_t x = gsk_ffdw_attr_r##n##_t##t(lds_total, &dmin); x != hipSuccess) e = x;
#define GSK_ATTR2(n) GSK_ATTR(n, 0) GSK_ATTR(n, 1)
  GSK_ATTR2(1) GSK_ATTR2(2) GSK_ATTR2(3) GSK_ATTR2(4) GSK_ATTR2(5) GSK_ATTR2(6) GSK_ATTR2(7) GSK_ATTR2(8)
#undef GSK_ATTR2
#undef GSK_ATTR
  g_ffdw_dyn_max = dmin;
  return e;
}

extern "C" uint32_t gsk_ffdw_dyn_lds_max(void) { return g_ffdw_dyn_max; }

// the single-wave provisioning Solve: grid-wide state reset, then one wave;
// ch: the claim scan state in HBM (d->ch_* allocated, claim_cap slots)
extern "C" hipError_t gsk_ffdw(const DevProblem* d, uint32_t ch, hipStream_t s) {
  const uint32_t lds = gsk_ffd_lds_bytes(ch ? 0u : d->max_claims_wave, d->n_thr, 0, topo_lds_bytes(d->TGZ, d->ZS, d->TGH, d->n_lazy)) +
                       wave_node_lds_bytes(d->NN);
  if (lds > g_ffdw_dyn_max) return hipErrorInvalidConfiguration;
  if (d->n_sims) return hipErrorInvalidValue;
  if (ch && !(d->ch_slk && d->ch_rm && d->ch_so && d->ch_scr && d->ch_tmpl)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ffd_init_kernel, dim3(256), dim3(256), 0, s, *d);
  const bool topo = d->TG || d->any_mv || d->any_vol;
  const uint32_t mode = (ch ? 1u : 0u) | (d->W > WREG ? 2u : 0u);
  switch (d->R * 2 + (topo ? 1 : 0)) {
#define GSK_CASE(n)                                                     \
  case 2 * n: return gsk_ffdw_launch_r##n##_t0(d, mode, lds, s);        \
  case 2 * n + 1: return gsk_ffdw_launch_r##n##_t1(d, mode, lds, s);
    GSK_CASE(1) GSK_CASE(2) GSK_CASE(3) GSK_CASE(4) GSK_CASE(5) GSK_CASE(6) GSK_CASE(7) GSK_CASE(8)
#undef GSK_CASE
    default:
      return hipErrorInvalidValue;
  }
}

// ------------------------------------------------ autoplacement ranking sort
// gs_rank_instance_types (rank.hip) sorts its kept instance types with the
// single-wave sort.Slice restatement above (WaveSort: every partition step a
// ballot, no workgroup barrier).  keys[k] = how many kept scores are strictly
// below score k: the same Less outcomes as the float64 compare (NaN refused
// on the host), so the permutation is the reference's.  pos[k] = compacted
// position; both sorted in place.  *np = the kept count (written by
// rank_kernel on the same stream); cap bounds it (<= GS_RANK_MAX).
extern "C" __global__ __launch_bounds__(64) void rank_sort_kernel(uint16_t* keys, uint16_t* pos, const uint32_t* np,
                                                                  uint32_t cap, int x) {
  extern __shared__ uint32_t rs_lds[];  // so[cap] (key | position << 16) | scr u16[cap + 2]
  __shared__ Frame rs_stk[64];
  const uint32_t n = __builtin_amdgcn_readfirstlane(*np <= cap ? *np : 0u);
  const uint32_t lane = threadIdx.x;
  lds_u32* so = (lds_u32*)rs_lds;
  lds_u16* scr = (lds_u16*)(rs_lds + cap);
  for (uint32_t k = lane; k < n; k += 64) so[k] = (uint32_t)keys[k] | ((uint32_t)pos[k] << 16);
  wsync();
  wave_pdqsort<GS_WAVE_SEQ, lds_u32, lds_u16, false, true>(so, scr, (lds_frame*)rs_stk, lane, (n + 1) / 2, (int)n,
                                                          x < (int)n ? x : -1);
  for (uint32_t k = lane; k < n; k += 64) {
    const uint32_t x = so[k];
    keys[k] = (uint16_t)(x & 0xFFFFu);
    pos[k] = (uint16_t)(x >> 16);
  }
}

// x: a position known to be the only one out of order (the test hook's
// one-change inputs take WaveSort::partition_known whatever the Solve's
// GS_KNOWN_PARTITION), or -1 (the ranking)
extern "C" hipError_t gsk_rank_sort(uint16_t* keys, uint16_t* pos, const uint32_t* np, uint32_t cap, int x, hipStream_t s) {
  const size_t lds = (size_t)cap * sizeof(uint32_t) + (size_t)(cap + 2) * sizeof(uint16_t);
  hipLaunchKernelGGL(rank_sort_kernel, dim3(1), dim3(64), lds, s, keys, pos, np, cap, x);
  return hipGetLastError();
}

