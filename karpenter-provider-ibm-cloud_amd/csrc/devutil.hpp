// devutil.hpp — device helpers shared by the gfx950 kernels: wave64
// reductions, (zone x capacity-type) grid masks and the free-key requirement
// algebra (<U> scheduling.Requirement on <= 256-value vocabularies).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "layout.hpp"

namespace gsd {
constexpr uint32_t INF = 0xFFFFFFFFu;

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t x, int m) {
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  lo = __shfl_xor((int)lo, m);
  hi = __shfl_xor((int)hi, m);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t x) {
  for (int m = 32; m >= 1; m >>= 1) {
    uint64_t y = shfl_xor_u64(x, m);
    x = y < x ? y : x;
  }
  return x;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t x) {
  for (int m = 32; m >= 1; m >>= 1) x += (uint32_t)__shfl_xor((int)x, m);
  return x;
}

// (zone mask x capacity-type mask) -> pair grid mask, pair g = z*C + c
__device__ __forceinline__ uint64_t grid_of(uint64_t zm, uint64_t cm, uint32_t Z, uint32_t C) {
  uint64_t cmask = cm & ((C >= 64) ? ~0ull : ((1ull << C) - 1));
  uint64_t g = 0;
  for (uint32_t z = 0; z < Z; z++)
    if ((zm >> z) & 1) g |= cmask << (z * C);
  return g;
}

// ------------------------------------------------- free-key requirement ops
__device__ __forceinline__ bool fk_any(const uint64_t* w) {
  uint64_t x = 0;
#pragma unroll
  for (int i = 0; i < FKW; i++) x |= w[i];
  return x != 0;
}
__device__ __forceinline__ bool fk_exempt(const FK& q) {
  // Operator() in {NotIn, DoesNotExist}
  return (q.flags & FK_COMP) ? fk_any(q.excl) : !fk_any(q.has);
}

// <U> Requirements.Compatible for one free key (AllowUndefinedWellKnownLabels)
__device__ __forceinline__ bool fk_compatible(const FK& c, const FK& p, bool wellknown) {
  if (!(c.flags & FK_PRESENT)) return wellknown || fk_exempt(p);
  bool len0;
  if ((c.flags & FK_COMP) && (p.flags & FK_COMP)) {
    bool hg = (c.flags | p.flags) & FK_GT, hl = (c.flags | p.flags) & FK_LT;
    int64_t gt = (c.flags & FK_GT) ? c.gt : p.gt;
    if ((c.flags & FK_GT) && (p.flags & FK_GT)) gt = c.gt > p.gt ? c.gt : p.gt;
    int64_t lt = (c.flags & FK_LT) ? c.lt : p.lt;
    if ((c.flags & FK_LT) && (p.flags & FK_LT)) lt = c.lt < p.lt ? c.lt : p.lt;
    len0 = hg && hl && gt >= lt;
  } else {
    uint64_t x = 0;
#pragma unroll
    for (int i = 0; i < FKW; i++) x |= c.has[i] & p.has[i];
    len0 = x == 0;
  }
  return !len0 || (fk_exempt(c) && fk_exempt(p));
}

// <U> Requirement.Intersection for one free key; ival [FKV], isint [FKW]
// (the key's vocabulary: integer values and which entries are integers)
__device__ FK fk_intersect(const FK& a, const FK& b, const int64_t* ival, const uint64_t* isint) {
  FK r;
  r.pad = 0;
  bool comp = (a.flags & FK_COMP) && (b.flags & FK_COMP);
  bool hg = (a.flags | b.flags) & FK_GT, hl = (a.flags | b.flags) & FK_LT;
  int64_t gt = (a.flags & FK_GT) ? a.gt : b.gt;
  if ((a.flags & FK_GT) && (b.flags & FK_GT)) gt = a.gt > b.gt ? a.gt : b.gt;
  int64_t lt = (a.flags & FK_LT) ? a.lt : b.lt;
  if ((a.flags & FK_LT) && (b.flags & FK_LT)) lt = a.lt < b.lt ? a.lt : b.lt;
  if (hg && hl && gt >= lt) {
    for (int i = 0; i < FKW; i++) r.has[i] = r.excl[i] = 0;
    r.gt = r.lt = 0;
    r.flags = FK_PRESENT;
    return r;
  }
  for (int i = 0; i < FKW; i++) r.has[i] = a.has[i] & b.has[i];
  if (comp) {
    for (int k = 0; k < FKW; k++) {
      uint64_t w = ~0ull;
      if (hg || hl) {
        w = 0;
        for (int i = 0; i < 64; i++) {
          if (!((isint[k] >> i) & 1)) continue;
          int64_t x = ival[k * 64 + i];
          if (hg && gt >= x) continue;
          if (hl && lt <= x) continue;
          w |= 1ull << i;
        }
      }
      r.excl[k] = (a.excl[k] | b.excl[k]) & w;
    }
    r.gt = hg ? gt : 0;
    r.lt = hl ? lt : 0;
    r.flags = FK_PRESENT | FK_COMP | (hg ? FK_GT : 0) | (hl ? FK_LT : 0);
  } else {
    for (int i = 0; i < FKW; i++) r.excl[i] = 0;
    r.gt = r.lt = 0;
    r.flags = FK_PRESENT;
  }
  return r;
}

template <class DP>
__device__ __forceinline__ bool var_fk_ok(const DP& d, const VarRec& vr, const FK* claim_fk) {
  for (uint32_t k = 0; k < vr.fk_count; k++) {
    const FKEntry& e = d.fk_entries[vr.fk_begin + k];
    if (!fk_compatible(claim_fk[e.slot], e.st, (d.wk_slots >> e.slot) & 1)) return false;
  }
  return true;
}

// <U> strict Requirements.Compatible (ExistingNode: no AllowUndefined)
template <class DP>
__device__ __forceinline__ bool var_fk_ok_strict(const DP& d, const VarRec& vr, const FK* node_fk) {
  for (uint32_t k = 0; k < vr.fk_count; k++) {
    const FKEntry& e = d.fk_entries[vr.fk_begin + k];
    if (!fk_compatible(node_fk[e.slot], e.st, false)) return false;
  }
  return true;
}

// first index m in [0,n) with vals[m] >= x (n if none)
__device__ __forceinline__ uint32_t lower_bound_i64(const int64_t* vals, uint32_t n, int64_t x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (vals[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}


}  // namespace gsd
