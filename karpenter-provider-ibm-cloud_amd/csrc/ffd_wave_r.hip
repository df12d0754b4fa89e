// ffd_wave_r.hip — the instantiations of ffdw_kernel (ffd_wave.hpp) for one
// resource count GS_WAVE_R and one variant GS_WAVE_TOPO (0: the plain
// variant, 1: the general one), with the claim scan state in LDS (register
// mode) or in HBM (ch), for narrow and wide option rows: compiled once per (R, TOPO) so the large register-
// mode bodies build in parallel (Makefile ffd_wave_r<R>_t<T>.o).
#include "ffd_wave.hpp"

#ifndef GS_WAVE_R
#error "GS_WAVE_R (1..8) and GS_WAVE_TOPO (0/1) select the instantiation"
#endif

using namespace gsd;

#define GSK_CAT2(a, b, c, d) a##b##c##d
#define GSK_CAT(a, b, c, d) GSK_CAT2(a, b, c, d)
#define GSK_LAUNCH GSK_CAT(gsk_ffdw_launch_r, GS_WAVE_R, _t, GS_WAVE_TOPO)
#define GSK_ATTR GSK_CAT(gsk_ffdw_attr_r, GS_WAVE_R, _t, GS_WAVE_TOPO)

template <bool CH, bool WIDE>
static hipError_t ffdw_attr_one(uint32_t lds_total, uint32_t* dyn_min) {
  const void* fn = (const void*)ffdw_kernel<GS_WAVE_R, GS_WAVE_TOPO != 0, CH, WIDE>;
  hipFuncAttributes a;
  hipError_t e = hipFuncGetAttributes(&a, fn);
  if (e != hipSuccess) return e;
  const uint32_t dyn = lds_total > a.sharedSizeBytes ? lds_total - (uint32_t)a.sharedSizeBytes : 0;
  if (!*dyn_min || dyn < *dyn_min) *dyn_min = dyn;
  return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn);
}

extern "C" hipError_t GSK_ATTR(uint32_t lds_total, uint32_t* dyn_min) {
  const hipError_t e[4] = {ffdw_attr_one<false, false>(lds_total, dyn_min), ffdw_attr_one<true, false>(lds_total, dyn_min),
                           ffdw_attr_one<false, true>(lds_total, dyn_min), ffdw_attr_one<true, true>(lds_total, dyn_min)};
  for (hipError_t x : e)
    if (x != hipSuccess) return x;
  return hipSuccess;
}

// mode: bit 0 = claim scan state in HBM, bit 1 = wide option rows (W > WREG)
extern "C" hipError_t GSK_LAUNCH(const DevProblem* d, uint32_t mode, uint32_t lds, hipStream_t s) {
  constexpr bool T = GS_WAVE_TOPO != 0;
  switch (mode & 3u) {
    case 0: hipLaunchKernelGGL((ffdw_kernel<GS_WAVE_R, T, false, false>), dim3(1), dim3(128), lds, s, *d); break;
    case 1: hipLaunchKernelGGL((ffdw_kernel<GS_WAVE_R, T, true, false>), dim3(1), dim3(128), lds, s, *d); break;
    case 2: hipLaunchKernelGGL((ffdw_kernel<GS_WAVE_R, T, false, true>), dim3(1), dim3(128), lds, s, *d); break;
    default: hipLaunchKernelGGL((ffdw_kernel<GS_WAVE_R, T, true, true>), dim3(1), dim3(128), lds, s, *d); break;
  }
  return hipGetLastError();
}
