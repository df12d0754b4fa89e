// ffd_wave.hpp — the single-wave provisioning Solve kernel template
// (ffdw_kernel), shared by the per-(R, TOPO) translation units
// ffd_wave_r.hip compiles (one per resource count and variant, built in
// parallel).
#pragma once
//
// The <U> Scheduler.Solve queue loop is sequential in pod order; its cost
// per pod is a chain of dependent steps (pop, sort.Slice emulation, first-fit
// scan of the in-flight NodeClaims, NodeClaim.Add).  A multi-wave workgroup
// pays a workgroup barrier and an LDS round trip of shared loop state for
// every step of that chain; one wave pays neither:
//  * the loop state (queue head/length, epoch, claim count, pending sort
//    modification) lives in scalar registers;
//  * the sorted NodeClaim order is one packed u32 per position (count in the
//    low 16 bits, claim id in the high 16): one LDS access reads or moves
//    both, and the scan reads a position's claim id and count together;
//  * every cross-lane LDS hand-off is ordered by the wave's in-order LDS
//    queue (wsync() only stops the compiler from reordering);
//  * the next pod's variant record and requests are prefetched into lanes
//    during the current pod (first pass: records laid out in queue order);
//  * a fast-accepted NodeClaim.Add (requests only) is LDS updates plus
//    no-return atomic adds of the requests at L2, issued by the solver
//    itself: no round trip (the agent wave only stages first-pass records);
//  * the one-claim sort.Slice rotation moves a 64-position window in one
//    LDS round trip (whole-wave DPP shift).
// Results are bit-identical to ffd.hip's block kernel (same restatement of
// Go's sort.Slice, same candidate order, same Add), which still serves the
// consolidation simulations and Solves with many existing nodes.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "devutil.hpp"
#include "ffd_common.hpp"
#include "layout.hpp"

using namespace gsd;

namespace {

constexpr uint32_t VR_DW = sizeof(VarRec) / 4;
static_assert(VR_DW == 32, "VarRec is one dword per lane of a half wave");
static_assert(offsetof(VarRec, fk_begin) == 4 && offsetof(VarRec, fk_count) == 8 && offsetof(VarRec, ctb) == 12 &&
                  offsetof(VarRec, itmask_off) == 16 && offsetof(VarRec, zfull_off) == 48 &&
                  offsetof(VarRec, cfull_off) == 52 && offsetof(VarRec, zm) == 56 && offsetof(VarRec, cm) == 64 &&
                  offsetof(VarRec, tol) == 72 && offsetof(VarRec, tolt) == 80 && offsetof(VarRec, own_off) == 88 &&
                  offsetof(VarRec, own_n) == 92 && offsetof(VarRec, sel_off) == 96 && offsetof(VarRec, sel_n) == 100 &&
                  offsetof(VarRec, zs) == 104 && offsetof(VarRec, zn) == 112 &&
                  offsetof(VarRec, zflags) == 120 && offsetof(VarRec, vix) == 124,
              "VarRec dword map used by ffdw_kernel");
static_assert(offsetof(ClaimRec, maxa) == 128, "ClaimRec maxa after two 64-B lines");

constexpr uint32_t WREG = 4;  // option words a scoring lane keeps in registers
#ifndef GS_ADD_LANES  // experiment builds: 0 = the winner lane updates every option word
#define GS_ADD_LANES 1
#endif
// solver <-> memory-agent wave channels (LDS)
#ifndef GS_RING
#define GS_RING 16
#endif
constexpr uint32_t RING = GS_RING;  // first-pass pod records staged ahead of the solver
constexpr uint32_t RING_DW = 53; // VarRec (32 dwords) + requests (<= 16 dwords) + request codes (4 dwords) + qrun
constexpr uint32_t RING_CODES = 48;  // lanes 48..51: floor codes lo/hi dword, ceil codes lo/hi dword
constexpr uint32_t RING_QRUN = 52;   // lane 52: qrun (records from here on with this one's spec, <= 16)
constexpr uint32_t WQ = 32;      // global-memory write requests in flight
constexpr uint32_t WQ_DW = 16;
enum : uint32_t { WQ_LOG = 1, WQ_FA = 2, WQ_STOP = 3, WQ_NFA = 4 };
constexpr uint32_t SPIN_MAX = 1u << 26;  // bounded waits: a stuck partner ends the kernel, not the GPU
constexpr uint64_t SWAR_HI = 0x8000800080008000ull;  // top bit of each 16-bit code field
enum : uint32_t { MOD_NONE = 0, MOD_INC = 1, MOD_APPEND = 2 };
#ifndef GS_WAVE_SEQ
#define GS_WAVE_SEQ 32
#endif
// GS_KNOWN_PARTITION: the first partition of a one-change sort searches the
// boundary (known_partition, out of line) instead of counting every key; 0
// never, 1 every instantiation, 2 the topology ones.  Bit-exact (the GPU
// suite; tests/test_wave_sort.py's one-change inputs through the rank
// kernel's instantiation, which always has it).  Inlined into the sort it
// changed the CM kernel's code shape (59.5 -> 60.7 KB) and CM got slower
// (268.7 -> 273.5 ms); out of line the kernel keeps its shape: same session
// CM 268.7 -> 264.6, E2E 243.4 -> 238.4, C3 383.3 -> 381.6 ms
// (profiles/r6/known_partition_ab.txt)
#ifndef GS_KNOWN_PARTITION
#define GS_KNOWN_PARTITION 1
#endif
#ifndef GS_REG_SORT  // 1: sort frames of <= 64 NodeClaims in registers (RegSort); 0: lane 0 over LDS (<= SEQ)
#define GS_REG_SORT 1
#endif

// GS_FFD_TL (diagnostic build): shader cycles per pod-loop segment into Ctrl.dbg
#if defined(GS_FFD_TL) && defined(GS_CAT_SEG)
// with GS_CAT_TL: the segments of the pods of category GS_CAT_SEG only
#define TLW(k)                                         \
  do {                                                 \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();  \
    ptl[k] += t_ - tl_last;                            \
    tl_last = t_;                                      \
  } while (0)
#elif defined(GS_FFD_TL)
#define TLW(k)                                         \
  do {                                                 \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();  \
    tl[k] += t_ - tl_last;                             \
    tl_last = t_;                                      \
  } while (0)
#else
#define TLW(k) \
  do {         \
  } while (0)
#endif

// channel words are polled: volatile LDS accesses.  The pointer is cast to
// the LDS address space explicitly (a volatile access through a generic
// pointer compiles to a flat, system-coherent load that also waits on every
// outstanding global memory operation).
typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ uint32_t vld(const uint32_t* p) { return *(const volatile lds_u32*)(const lds_u32*)p; }
__device__ __forceinline__ void vst(uint32_t* p, uint32_t x) { *(volatile lds_u32*)(lds_u32*)p = x; }

// The Solve loop keeps only its own state in scalar registers; its cold
// paths re-read the kernel arguments through the kernarg pointer (scalar
// loads from the constant cache) and the pod's variant fields from the
// record lane (readlane) where they use them, instead of holding ~100
// scalar values across the loop (which spills them into VGPR lanes).
__device__ __forceinline__ KArg karg() {
  KArg p = (KArg)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return p;
}
// an opaque copy: readlanes of it are not merged with earlier ones
__device__ __forceinline__ uint32_t fresh(uint32_t x) {
  asm volatile("" : "+v"(x));
  return x;
}

__device__ __forceinline__ uint64_t shfl_u64(uint64_t x, uint32_t src) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)x, (int)src), hi = (uint32_t)__shfl((int)(uint32_t)(x >> 32), (int)src);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t x) {
  for (int m = 32; m >= 1; m >>= 1) {
    const uint64_t y = shfl_xor_u64(x, m);
    x = y > x ? y : x;
  }
  return x;
}

// ------------------------------------------------ 16-bit code fields (SWAR)
// a request / slack / room is four 15-bit codes in one u64 (layout.hpp
// qcode); SWAR_HI keeps the borrow of each field inside the field
__device__ __forceinline__ bool swar_ge(uint64_t a, uint64_t b) {  // every field a >= b
  return (((a | SWAR_HI) - b) & SWAR_HI) == SWAR_HI;
}
__device__ __forceinline__ uint64_t swar_max(uint64_t a, uint64_t b) {  // field-wise max
  const uint64_t m = ((((a | SWAR_HI) - b) & SWAR_HI) >> 15) * 0xFFFFull;
  return (a & m) | (b & ~m);
}
__device__ __forceinline__ uint64_t wave_swar_max(uint64_t x) {
  for (int m = 32; m >= 1; m >>= 1) x = swar_max(x, shfl_xor_u64(x, m));
  return x;
}

// wave maximum of an unsigned value, uniform result: row prefix maxima and
// row broadcasts in DPP, lane 63 read out (no LDS round trip)
__device__ __forceinline__ uint32_t dpp_max_step(uint32_t x, uint32_t y) { return x > y ? x : y; }
__device__ __forceinline__ uint32_t wave_max_dpp(uint32_t x) {
  x = dpp_max_step(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true));  // row_shr:1
  x = dpp_max_step(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true));  // row_shr:2
  x = dpp_max_step(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true));  // row_shr:4
  x = dpp_max_step(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true));  // row_shr:8
  x = dpp_max_step(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false));  // row_bcast:15
  x = dpp_max_step(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false));  // row_bcast:31
  return rlane(x, 63u);
}

// -------------------------------------------------------- wave-parallel sort
// sort.Slice(newNodeClaims, len(Pods) asc) over the packed order: the block
// restatement of pdqsort_func (ffd.hip Blk) with one wave, so every block
// reduction is a ballot and every barrier an in-order LDS queue.  Ranges up
// to SEQ elements run the sequential port on lane 0.
// partition of the whole array [0, n) when the caller knows its shape:
// every position but x (the NodeClaim the last Add raised, or the appended
// one) holds a non-decreasing sequence.  After swap(0, pivot) the positions
// of (0, n) outside E = {x, pivot} still do, so the keys below the pivot's
// are those before a boundary t (a 64-ary search, two LDS round trips)
// plus E's, and each misplaced list has at most |E| + |E| entries near t /
// mid and at E.  Same permutation as partition(): the k-th misplaced
// position of the left side (ascending) trades with the k-th of the right
// side (descending).  n > 64.
struct KnownPart {
  int mid;
  int flags;  // 1 already partitioned, 2 left side uniform, 4 right side uniform
};
template <class U32, bool G>
__device__ __noinline__ KnownPart known_partition(U32* so, int n, int pivot, int x) {
  n = __builtin_amdgcn_readfirstlane(n);
  pivot = __builtin_amdgcn_readfirstlane(pivot);
  x = __builtin_amdgcn_readfirstlane(x);
  const uint32_t lane = threadIdx.x & 63u;
  auto key = [&](int i) { return (uint32_t)so[i] & 0xFFFFu; };
  auto swap = [&](int i, int j) {
    const uint32_t a = so[i];
    so[i] = so[j];
    so[j] = a;
  };
  bool already_, luni_, runi_;
  bool* already = &already_;
  bool* luni = &luni_;
  bool* runi = &runi_;
  if (lane == 0) swap(0, pivot);
  wsyncT<G>();
  const uint32_t p = key(0);
  const int e0 = x >= 1 && x < n ? x : -1;
  const int e1 = pivot != x && pivot >= 1 && pivot < n ? pivot : -1;
  auto in_e = [&](int k) { return k == e0 || k == e1; };
  auto skip_e = [&](int k) {  // the first position >= k outside E
    k += in_e(k) ? 1 : 0;
    k += in_e(k) ? 1 : 0;
    return k;
  };
  // t: the first position of [1, n) outside E with key >= p (n if none)
  const int step = (n - 1 + 63) / 64;
  const int q = skip_e(1 + (int)lane * step);
  const bool qv = 1 + (int)lane * step < n && q < n;
  const uint64_t m1 = __ballot(qv && key(qv ? q : 0) >= p);
  int lo, hi;  // t is in [lo, hi]
  if (m1) {
    const int l = (int)ffs64(m1);
    lo = l == 0 ? 1 : (int)rlane((uint32_t)q, (uint32_t)(l - 1)) + 1;
    hi = (int)rlane((uint32_t)q, (uint32_t)l);
  } else {
    const int lv = 63 - (int)__clzll((long long)__ballot(qv));
    lo = (int)rlane((uint32_t)q, (uint32_t)lv) + 1;
    hi = n;
  }
  int t = hi;
  for (int base = lo; base < hi; base += 64) {
    const int k = base + (int)lane;
    const bool ok = k < hi && k < n && !in_e(k);
    const uint64_t m2 = __ballot(ok && key(ok ? k : 0) >= p);
    if (m2) {
      t = base + (int)ffs64(m2);
      break;
    }
  }
  // E's keys, read by every lane (uniform)
  const uint32_t k0 = e0 >= 0 ? key(e0) : 0u, k1 = e1 >= 0 ? key(e1) : 0u;
  const int e_lt = (e0 >= 0 && k0 < p ? 1 : 0) + (e1 >= 0 && k1 < p ? 1 : 0);
  const int e_before_t = (e0 >= 1 && e0 < t ? 1 : 0) + (e1 >= 1 && e1 < t ? 1 : 0);
  const int mid = (t - 1) - e_before_t + e_lt;
  // side uniformity (before any swap): the sorted part's first and last
  // keys on each side, and E's keys
  {
    auto prev_out = [&](int k) {
      k -= in_e(k) ? 1 : 0;
      k -= in_e(k) ? 1 : 0;
      return k;
    };
    uint32_t amin = 0xFFFFu, amax = 0, bmin = 0xFFFFu, bmax = 0;
    const int f1 = skip_e(1), l1 = prev_out(t - 1);
    if (f1 < t && l1 >= 1 && f1 <= l1) {
      amin = key(f1);
      amax = key(l1);
    }
    const int l2 = prev_out(n - 1);
    if (t < n && l2 >= t) {
      bmin = key(t);
      bmax = key(l2);
    }
    if (e0 >= 0) {
      if (k0 < p) {
        amin = k0 < amin ? k0 : amin;
        amax = k0 > amax ? k0 : amax;
      } else {
        bmin = k0 < bmin ? k0 : bmin;
        bmax = k0 > bmax ? k0 : bmax;
      }
    }
    if (e1 >= 0) {
      if (k1 < p) {
        amin = k1 < amin ? k1 : amin;
        amax = k1 > amax ? k1 : amax;
      } else {
        bmin = k1 < bmin ? k1 : bmin;
        bmax = k1 > bmax ? k1 : bmax;
      }
    }
    *luni = amin >= amax;  // empty or one key value
    *runi = bmin >= bmax;
  }
  // candidates: lanes 0..3 positions from t (left side past the boundary),
  // lanes 4..7 positions from mid + 1 (right side before it), lanes 8, 9 E
  int pos = -1;
  bool left = false, right = false;
  if (lane < 4) {
    pos = t + (int)lane;
    left = pos <= mid && pos < n && !in_e(pos);
  } else if (lane < 8) {
    pos = mid + 1 + (int)(lane - 4);
    right = pos < t && pos < n && !in_e(pos);
  } else if (lane == 8 || lane == 9) {
    pos = lane == 8 ? e0 : e1;
    if (pos >= 1) {
      const uint32_t ke = lane == 8 ? k0 : k1;
      left = pos <= mid && ke >= p;
      right = pos > mid && ke < p;
    }
  }
  const uint64_t lm = __ballot(left), rm = __ballot(right);
  const uint32_t s = (uint32_t)__popcll(lm);
  if (s) {
    // ranks (left ascending, right descending by position) and partners
    // (the other side's lane of the same rank): uniform loops over the
    // flagged lanes
    const uint64_t fl = lm | rm;
    int r = 0;
    for (uint64_t mm = fl; mm; mm &= mm - 1) {
      const uint32_t j = ffs64(mm);
      const int pj = (int)rlane((uint32_t)pos, j);
      const bool lj = (lm >> j) & 1ull;
      r += (left && lj && pj < pos) || (right && !lj && pj > pos) ? 1 : 0;
    }
    int partner = (int)lane;
    for (uint64_t mm = fl; mm; mm &= mm - 1) {
      const uint32_t j = ffs64(mm);
      const int rj = (int)rlane((uint32_t)r, j);
      const bool lj = (lm >> j) & 1ull;
      if (((left && !lj) || (right && lj)) && rj == r) partner = (int)j;
    }
    const uint32_t wv = (left || right) ? (uint32_t)so[pos] : 0u;
    const uint32_t pv = (uint32_t)__shfl((int)wv, partner);
    wsyncT<G>();
    if (left || right) so[pos] = pv;
    wsyncT<G>();
  }
  if (lane == 0) swap(mid, 0);
  wsyncT<G>();
  *already = s == 0;
  return KnownPart{mid, (already_ ? 1 : 0) | (luni_ ? 2 : 0) | (runi_ ? 4 : 0)};
}

template <int SEQ, class U32 = lds_u32, class U16 = lds_u16, bool G = false, bool KNOWN = false>
struct WaveSort {
  static_assert(SEQ >= 12, "ranges <= 12 must reach Go's insertion sort");
  U32* so;
  U16* scr;  // compaction scratch: [0, half) left list, [half, 2 half) right list
  lds_frame* stk;
  uint32_t lane, half;

  __device__ __forceinline__ uint32_t key(int i) const { return so[i] & 0xFFFFu; }
  __device__ __forceinline__ void swap(int i, int j) const {
    const uint32_t a = so[i];
    so[i] = so[j];
    so[j] = a;
  }
  // the passes below test RW x 64 positions per step: every lane issues its
  // RW LDS reads before the first ballot (one round trip per step)
#ifndef GS_SORT_RW
#define GS_SORT_RW 4
#endif
  static constexpr int RW = GS_SORT_RW;
  template <class Pred>
  __device__ uint32_t count(int lo, int hi, Pred pred) const {
    uint32_t c = 0;
    for (int base = lo; base < hi; base += 64 * RW) {
      bool in[RW];
#pragma unroll
      for (int u = 0; u < RW; u++) {
        const int k = base + u * 64 + (int)lane;
        in[u] = k < hi && pred(k);
      }
#pragma unroll
      for (int u = 0; u < RW; u++) c += (uint32_t)__popcll(__ballot(in[u]));
    }
    return c;
  }
  // positions k in [lo,hi) with pred(k), ascending or descending, to out[]
  template <class Pred>
  __device__ uint32_t compact(int lo, int hi, bool desc, U16* out, Pred pred) const {
    uint32_t total = 0;
    const int n = hi - lo;
    for (int base = 0; base < n; base += 64 * RW) {
      bool in[RW];
#pragma unroll
      for (int u = 0; u < RW; u++) {
        const int idx = base + u * 64 + (int)lane;
        in[u] = idx < n && pred(desc ? hi - 1 - idx : lo + idx);
      }
#pragma unroll
      for (int u = 0; u < RW; u++) {
        const int idx = base + u * 64 + (int)lane;
        const uint64_t m = __ballot(in[u]);
        if (in[u]) out[total + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = (uint16_t)(desc ? hi - 1 - idx : lo + idx);
        total += (uint32_t)__popcll(m);
      }
    }
    wsyncT<G>();
    return total;
  }
  // swap the k-th left-list position with the k-th right-list position
  __device__ void swap_lists(uint32_t s) const {
    for (uint32_t k = lane; k < s; k += 64) {
      const int x = scr[k], y = scr[half + k];
      const uint32_t a = so[x], b = so[y];
      wsyncT<G>();
      so[x] = b;
      so[y] = a;
    }
    wsyncT<G>();
  }
  // the count pass of a partition: how many keys in [lo, hi) are below the
  // pivot (<= it with LE), and whether the keys on each side are all equal
  // (the sides become the child frames: a side of equal keys is sorted by a
  // few swaps, see pdqsort_body)
  // *mk: lane c keeps the predicate's ballot of chunk c (positions
  // lo + 64c ...): with hi - lo <= 4096 the misplaced lists come from these
  // masks (lists_from_masks) instead of two more passes over the keys
  template <bool LE>
  __device__ uint32_t count_split(int lo, int hi, uint32_t p, bool* lo_uni, bool* hi_uni, uint64_t* mk) const {
    // branch-free: every lane keeps the side maxima of keys and of
    // complemented keys (VALU), reduced once per partition in DPP
    constexpr int RC = 2 * RW;  // positions read per lane before the first wait
    uint32_t c = 0, amax = 0, anot = 0, bmax = 0, bnot = 0;
    uint64_t mine = 0;
    for (int base = lo; base < hi; base += 64 * RC) {
      uint32_t kk[RC];
#pragma unroll
      for (int u = 0; u < RC; u++) {
        const int k = base + u * 64 + (int)lane;
        kk[u] = key(k < hi ? k : hi - 1);  // unconditional read: no exec-masked load
      }
#pragma unroll
      for (int u = 0; u < RC; u++) {
        const int k = base + u * 64 + (int)lane;
        const bool valid = k < hi;
        const bool in = valid && (LE ? kk[u] <= p : kk[u] < p);
        const bool out = valid && !in;
        const uint64_t bi = __ballot(in);
        c += (uint32_t)__popcll(bi);
        mine = lane == (uint32_t)((base - lo) / 64 + u) ? bi : mine;
        const uint32_t nk = 0xFFFFu - kk[u];
        amax = in && kk[u] > amax ? kk[u] : amax;
        anot = in && nk > anot ? nk : anot;
        bmax = out && kk[u] > bmax ? kk[u] : bmax;
        bnot = out && nk > bnot ? nk : bnot;
      }
    }
    *mk = mine;
    amax = wave_max_dpp(amax);
    anot = wave_max_dpp(anot);
    bmax = wave_max_dpp(bmax);
    bnot = wave_max_dpp(bnot);
    *lo_uni = c == 0 || amax == 0xFFFFu - anot;  // empty or one key value
    *hi_uni = c == (uint32_t)(hi - lo) || bmax == 0xFFFFu - bnot;
    return c;
  }
  static constexpr int MASK_MAX = 64 * 64;  // positions the lanes' chunk masks cover
#ifndef GS_MASK_LISTS  // experiment builds: 0 = the two compaction passes instead
#define GS_MASK_LISTS 1
#endif
  // a partition's two misplaced lists from the lanes' masks of [lo, lo + n):
  // x < nl is the left side, misplaced where the predicate fails (ascending
  // positions to scr[0 ..]); x >= nl the right side, misplaced where it holds
  // (descending positions to scr[half ..]); returns the left list's length
  __device__ uint32_t lists_from_masks(int lo, uint32_t nl, uint32_t n, uint64_t mk) const {
    const uint32_t x0 = lane * 64u;
    const uint64_t valid = x0 >= n ? 0ull : (n - x0 >= 64u ? ~0ull : ((1ull << (n - x0)) - 1ull));
    const uint64_t left = x0 >= nl ? 0ull : (nl - x0 >= 64u ? ~0ull : ((1ull << (nl - x0)) - 1ull));
    const uint64_t lm = ~mk & left & valid, rm = mk & ~left & valid;
    const uint32_t lc = (uint32_t)__popcll(lm), rc = (uint32_t)__popcll(rm);
    // inclusive prefix over lanes of (lc | rc << 16), row scans and row
    // broadcasts in DPP (no LDS round trip)
    uint32_t x = lc | rc << 16;
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
    const uint32_t tot = rlane(x, 63u);
    const uint32_t lpre = x & 0xFFFFu;                          // lanes <= this one
    const uint32_t rsuf = (tot >> 16) - (x >> 16) + rc;         // lanes >= this one
    const uint32_t total = tot & 0xFFFFu;
    uint32_t k = lpre - lc;
    for (uint64_t m = lm; m; m &= m - 1) scr[k++] = (uint16_t)(lo + (int)(x0 + ffs64(m)));
    k = rsuf - rc;
    for (uint64_t m = rm; m;) {
      const uint32_t bit = 63u - (uint32_t)__clzll((long long)m);
      scr[half + k++] = (uint16_t)(lo + (int)(x0 + bit));
      m &= ~(1ull << bit);
    }
    wsyncT<G>();
    return total;
  }
#ifdef GS_SORT_TL2
#define PTL(k)                                                                  \
  do {                                                                          \
    const uint64_t n_ = __builtin_amdgcn_s_memtime();                           \
    if (lane == 0 && stl) stl[8 + (k)] += n_ - p_last;                          \
    p_last = n_;                                                                \
  } while (0)
#else
#define PTL(k) \
  do {         \
  } while (0)
#endif
  __device__ int partition(int a, int b, int pivot, bool* already, bool* luni, bool* runi) const {
#ifdef GS_SORT_TL2
    uint64_t p_last = __builtin_amdgcn_s_memtime();
#endif
    if (lane == 0) swap(a, pivot);
    wsyncT<G>();
    const uint32_t p = key(a);
    PTL(0);
    uint64_t mk;
    const int mid = a + (int)count_split<false>(a + 1, b, p, luni, runi, &mk);
    PTL(1);
    uint32_t s;
    if (GS_MASK_LISTS && b - a - 1 <= MASK_MAX) {
      s = lists_from_masks(a + 1, (uint32_t)(mid - a), (uint32_t)(b - a - 1), mk);
    } else {
      s = compact(a + 1, mid + 1, false, scr, [&](int k) { return key(k) >= p; });
      compact(mid + 1, b, true, scr + half, [&](int k) { return key(k) < p; });
    }
    PTL(2);
    swap_lists(s);
    if (lane == 0) swap(mid, a);
    wsyncT<G>();
    PTL(3);
    *already = s == 0;
    return mid;
  }
  // partition of the whole array [0, n) when the caller knows its shape
  // (known_partition below, out of line)
  __device__ int partition_known(int n, int pivot, int x, bool* already, bool* luni, bool* runi) const;
  __device__ int partition_equal(int a, int b, int pivot, bool* runi) const {
    if (lane == 0) swap(a, pivot);
    wsyncT<G>();
    const uint32_t p = key(a);
    bool luni;
    uint64_t mk;
    const int mid = a + (int)count_split<true>(a + 1, b, p, &luni, runi, &mk);
    uint32_t s;
    if (GS_MASK_LISTS && b - a - 1 <= MASK_MAX) {
      s = lists_from_masks(a + 1, (uint32_t)(mid - a), (uint32_t)(b - a - 1), mk);
    } else {
      s = compact(a + 1, mid + 1, false, scr, [&](int k) { return key(k) > p; });
      compact(mid + 1, b, true, scr + half, [&](int k) { return key(k) <= p; });
    }
    swap_lists(s);
    return mid + 1;
  }
  // one rotation: left = the element at lo lands at hi, (lo, hi] shift left;
  // otherwise the element at hi lands at lo, [lo, hi) shift right.  Passes of
  // 64 positions read before they write, in the order that never overwrites
  // a position a later pass still reads.
  __device__ void rotate(int lo, int hi, bool left) const {
    if (hi <= lo) return;
    const uint32_t x = so[left ? lo : hi];
    wsyncT<G>();
    // RU x 64 positions per pass: every lane loads its RU values (one LDS
    // round trip), then stores them one position over
    constexpr int RU = 4;
    if (left) {
      for (int base = lo; base < hi; base += 64 * RU) {
        uint32_t v[RU];
#pragma unroll
        for (int u = 0; u < RU; u++) {
          const int k = base + u * 64 + (int)lane;
          v[u] = k < hi ? so[k + 1] : 0u;
        }
        wsyncT<G>();
#pragma unroll
        for (int u = 0; u < RU; u++) {
          const int k = base + u * 64 + (int)lane;
          if (k < hi) so[k] = v[u];
        }
        wsyncT<G>();
      }
      if (lane == 0) so[hi] = x;
    } else {
      for (int top = hi - 1; top >= lo; top -= 64 * RU) {
        uint32_t v[RU];
#pragma unroll
        for (int u = 0; u < RU; u++) {
          const int k = top - u * 64 - (int)lane;
          v[u] = k >= lo ? so[k] : 0u;
        }
        wsyncT<G>();
#pragma unroll
        for (int u = 0; u < RU; u++) {
          const int k = top - u * 64 - (int)lane;
          if (k >= lo) so[k + 1] = v[u];
        }
        wsyncT<G>();
      }
      if (lane == 0) so[lo] = x;
    }
    wsyncT<G>();
  }
  // first k in [from, b) with key(k) < key(k-1); b if none
  __device__ int first_inversion(int from, int b) const {
    for (int base = from; base < b; base += 64 * RW) {
      bool hit[RW];
      uint32_t kc[RW], kp[RW];
#pragma unroll
      for (int u = 0; u < RW; u++) {
        const int k = base + u * 64 + (int)lane, kk = k < b ? k : b - 1;  // unconditional reads
        kc[u] = key(kk);
        kp[u] = key(kk - 1);
      }
#pragma unroll
      for (int u = 0; u < RW; u++) hit[u] = base + u * 64 + (int)lane < b && kc[u] < kp[u];
#pragma unroll
      for (int u = 0; u < RW; u++) {
        const uint64_t m = __ballot(hit[u]);
        if (m) return base + u * 64 + (int)ffs64(m);
      }
    }
    return b;
  }
  __device__ bool partial_insertion_sort(int a, int b) const {
    int i = a + 1;
    for (int j = 0; j < 5; j++) {
      i = first_inversion(i, b);
      if (i == b) return true;
      if (b - a < 50) return false;
      if (lane == 0) swap(i, i - 1);
      wsyncT<G>();
      if (i - a >= 2) {
        // the smaller element (now at i-1) moves left past larger elements,
        // down to absolute index 0 (Go's loop runs to j >= 1)
        const uint32_t x = key(i - 1);
        int q = -1;
        for (int top = i - 2; top >= 0; top -= 64) {
          const int k = top - (int)lane;
          const uint64_t m = __ballot(k >= 0 && key(k) <= x);
          if (m) {
            q = top - (int)ffs64(m);  // lowest lane = highest position
            break;
          }
        }
        rotate(q + 1, i - 1, false);
      }
      if (b - i >= 2) {
        const uint32_t y = key(i);
        int q = b;
        for (int base = i + 1; base < b; base += 64) {
          const int k = base + (int)lane;
          const uint64_t m = __ballot(k < b && key(k) >= y);
          if (m) {
            q = base + (int)ffs64(m);
            break;
          }
        }
        rotate(i, q - 1, true);
      }
    }
    return false;
  }
  __device__ void reverse_range(int a, int b) const {
    const int n = (b - a) / 2;
    for (int k = (int)lane; k < n; k += 64) {
      const uint32_t x = so[a + k], y = so[b - 1 - k];
      wsyncT<G>();
      so[a + k] = y;
      so[b - 1 - k] = x;
    }
    wsyncT<G>();
  }
#ifndef GS_UNIFORM  // experiment builds: 0 = no equal-key frame shortcut
#define GS_UNIFORM 1
#endif
#ifdef GS_SORT_TL
  // diagnostic: shader cycles per part of the generic sort (lane 0 sums into stl[])
  uint64_t* stl = nullptr;
#define STL(k)                                                     \
  do {                                                             \
    const uint64_t now_ = __builtin_amdgcn_s_memtime();            \
    if (lane == 0 && stl) stl[k] += now_ - t_last_;                \
    t_last_ = now_;                                                \
  } while (0)
#else
#define STL(k) \
  do {         \
  } while (0)
#endif
  // x: the one position known to break the order (GS_KNOWN_PARTITION: the
  // first partition then runs partition_known), or -1
  __device__ __forceinline__ void pdqsort_body(int n, int x = -1) const {
#ifdef GS_SORT_TL
    uint64_t t_last_ = __builtin_amdgcn_s_memtime();
#endif
    const SeqSortT<PackedAccT<U32>> seq{{so}};
    if (GS_REG_SORT ? n <= 64 : n <= SEQ) {
      if (GS_REG_SORT) {
        reg_pdq_frame(PackedArr<U32, G>{so}, 0, n, bits_len((uint64_t)n), 1, 1);
      } else {
        if (lane == 0) seq.pdq_frame(Frame{0, n, bits_len((uint64_t)n), 1, 1});
        wsyncT<G>();
      }
      return;
    }
    int sp = 0;
    uint32_t stk_ab = 0, stk_fl = 0;
    Frame f{0, n, bits_len((uint64_t)n), 1, 1};
    bool pristine = KNOWN && x >= 0;  // the array is still sorted but for x
    for (;;) {
      for (;;) {
        // wave-uniform frame state: scalar registers and branches
        f.a = __builtin_amdgcn_readfirstlane(f.a);
        f.b = __builtin_amdgcn_readfirstlane(f.b);
        f.limit = __builtin_amdgcn_readfirstlane(f.limit);
        f.wb = __builtin_amdgcn_readfirstlane(f.wb);
        f.wp = __builtin_amdgcn_readfirstlane(f.wp);
        f.uni = __builtin_amdgcn_readfirstlane(f.uni);
        const int length = f.b - f.a;
        STL(6);  // frame bookkeeping
        if (GS_REG_SORT ? length <= 64 : length <= SEQ) {
          if (GS_REG_SORT) {
            reg_pdq_frame(PackedArr<U32, G>{so}, f.a, f.b, f.limit, f.wb, f.wp);
          } else {
            if (lane == 0) seq.pdq_frame(f);
            wsyncT<G>();
          }
          STL(0);
          break;
        }
        if (f.limit == 0) {
          if (lane == 0) seq.heap_sort(f.a, f.b);
          wsyncT<G>();
          STL(0);
          break;
        }
        if (!f.wb) {
          if (lane == 0) seq.break_patterns(f.a, f.b);
          wsyncT<G>();
          f.limit--;
          STL(0);
        }
        if (GS_UNIFORM && f.uni) {
          // every key in [a, b) is equal (swaps keep it so): choosePivot makes
          // no swap (hint increasing, pivot the middle sample), a partial
          // insertion sort finds no inversion, partitionEqual takes the whole
          // range and partition none of it; only their first swap remains
          const int pivot = f.a + length / 4 * 2;
          if (f.wb && f.wp) break;
          const bool eq = f.a > 0 && !(key(f.a - 1) < key(pivot));
          if (lane == 0) swap(f.a, pivot);
          wsyncT<G>();
          if (eq) {
            f.a = f.b;
            STL(1);
            continue;
          }
          // partition: mid = a, already partitioned; the empty left side is
          // the smaller child, so the frame continues with [a + 1, b)
          f.wp = 1;
          f.wb = 0 >= length / 8;
          f.a = f.a + 1;
          STL(1);
          continue;
        }
        int hint = 0;
        int pivot = seq.choose_pivot_fast(f.a, f.b, &hint);  // every lane, same keys
        pivot = __builtin_amdgcn_readfirstlane(pivot);
        hint = __builtin_amdgcn_readfirstlane(hint);
        if (hint == 2) {
          reverse_range(f.a, f.b);
          pivot = (f.b - 1) - (pivot - f.a);
          hint = 1;
          pristine = false;
        }
        STL(2);
        if (f.wb && f.wp && hint == 1) {
          const bool done = partial_insertion_sort(f.a, f.b);
          STL(3);
          if (done) break;
          pristine = false;
        }
        if (f.a > 0 && !(key(f.a - 1) < key(pivot))) {
          bool runi;
          f.a = partition_equal(f.a, f.b, pivot, &runi);
          f.uni = runi;
          STL(4);
          continue;
        }
        bool already, luni, runi;
        const int mid = pristine && f.a == 0 && f.b == n ? partition_known(n, pivot, x, &already, &luni, &runi)
                                                         : partition(f.a, f.b, pivot, &already, &luni, &runi);
        pristine = false;
        STL(5);
        f.wp = already;
        const int leftLen = mid - f.a, rightLen = f.b - mid;
        const int bal = length / 8;
        Frame child;
        if (leftLen < rightLen) {
          f.wb = leftLen >= bal;
          child = Frame{f.a, mid, f.limit, 1, 1, luni};
          f.a = mid + 1;
          f.uni = runi;
        } else {
          f.wb = rightLen >= bal;
          child = Frame{mid + 1, f.b, f.limit, 1, 1, runi};
          f.b = mid;
          f.uni = luni;
        }
        // the continuing frame waits in lane sp of two VGPRs (depth <= 12
        // for 4,096 NodeClaims)
        stk_ab = wlane(stk_ab, sp, (uint32_t)f.a | (uint32_t)f.b << 16);
        stk_fl = wlane(stk_fl, sp, (uint32_t)f.limit | (uint32_t)f.wb << 8 | (uint32_t)f.wp << 9 | (uint32_t)f.uni << 10);
        sp++;
        f = child;
      }
      sp = __builtin_amdgcn_readfirstlane(sp);
      if (sp == 0) break;
      sp--;
      const uint32_t ab = rlane(stk_ab, (uint32_t)sp), fl = rlane(stk_fl, (uint32_t)sp);
      f.a = (int)(ab & 0xFFFFu);
      f.b = (int)(ab >> 16);
      f.limit = (int)(fl & 0xFFu);
      f.wb = (int)((fl >> 8) & 1u);
      f.wp = (int)((fl >> 9) & 1u);
      f.uni = (int)((fl >> 10) & 1u);
    }
    wsyncT<G>();
  }
};

template <int SEQ, class U32, class U16, bool G, bool KNOWN>
__device__ int WaveSort<SEQ, U32, U16, G, KNOWN>::partition_known(int n, int pivot, int x, bool* already, bool* luni,
                                                                 bool* runi) const {
  const KnownPart kp = known_partition<U32, G>(so, n, pivot, x);
  *already = (kp.flags & 1) != 0;
  *luni = (kp.flags & 2) != 0;
  *runi = (kp.flags & 4) != 0;
  return kp.mid;
}

// The run batch's placement (GS_RUN_BATCH, the pod loop below): out of line,
// so its registers do not weigh on the rest of the loop.  Pods 2..k of the
// batch (lane j < k: pod bp / variant bv) join the claims U_1..U_{k-1} at
// lanes fl + 1..; returns the window after the k - 1 rotations
struct RunWin {
  uint32_t ow, wtok;
  uint64_t wsl, wrm;
};
template <uint32_t RR>
__device__ __noinline__ RunWin run_batch_place(RunWin w, uint64_t rq, uint32_t bp, uint32_t bv, uint32_t fl, uint32_t m,
                                               uint32_t k, uint32_t nlog, uint32_t rqn, LogRec* log, ClaimRec* c_rec) {
  const uint32_t lane = threadIdx.x & 63u;
  fl = __builtin_amdgcn_readfirstlane(fl);
  m = __builtin_amdgcn_readfirstlane(m);
  k = __builtin_amdgcn_readfirstlane(k);
  nlog = __builtin_amdgcn_readfirstlane(nlog);
  rqn = __builtin_amdgcn_readfirstlane(rqn);
  // lane j < k: its pod's log entry (claim U_j); lanes 4i + r:
  // pod i + 2's request r into U_{i+1}'s totals
  const uint32_t cj = (uint32_t)__shfl((int)w.ow, (int)((fl + lane) & 63u)) >> 16;
  if (lane >= 1 && lane < k) log[nlog + lane - 1] = LogRec{bp, bv, cj, 0};
  {
    const uint32_t j = 1u + (lane >> 2), r = lane & 3u;
    const uint32_t ci = (uint32_t)__shfl((int)w.ow, (int)((fl + j) & 63u)) >> 16;
    const int64_t rqr = (int64_t)shfl_u64(rq, r);
    if (j < k && r < RR && rqr != 0)
      atomicAdd((unsigned long long*)&c_rec[ci].tot_lo[r], (unsigned long long)rqr);
  }
  // lanes 4i + r re-quantize resource r of U_{i+1} (as this
  // pod's lanes r did for U_0), packed across the quad with
  // DPP and moved back to U_{i+1}'s lane
  {
    const uint32_t i = lane >> 2, r = lane & 3u, src_l = (fl + 1u + i) & 63u;
    const uint64_t rm_i = shfl_u64(w.wrm, src_l), sl_i = shfl_u64(w.wsl, src_l);
    uint32_t q_rm = 0, q_sl = 0;
    if (r < rqn) {
      const int64_t rqr = (int64_t)shfl_u64(rq, r);
      q_rm = qcode_floor(qcode_value((uint32_t)(rm_i >> (16 * r)) & 0xFFFFu) - rqr);
      q_sl = qcode_ceil(qcode_value((uint32_t)(sl_i >> (16 * r)) & 0xFFFFu) - rqr);
    }
    uint32_t prm2 = (lane & 1u) ? q_rm << 16 : q_rm, psl2 = (lane & 1u) ? q_sl << 16 : q_sl;
    prm2 |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)prm2, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    psl2 |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)psl2, 0xB1, 0xF, 0xF, false);
    const uint32_t hrm2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)prm2, 0x102, 0xF, 0xF, false);  // row_shl:2
    const uint32_t hsl2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)psl2, 0x102, 0xF, 0xF, false);
    // lane 4i now holds U_{i+1}'s packed codes (lo dword, hi dword)
    const uint32_t back = 4u * ((lane - fl - 1u) & 15u);
    const uint32_t rm_lo = (uint32_t)__shfl((int)prm2, (int)back), rm_hi = (uint32_t)__shfl((int)hrm2, (int)back);
    const uint32_t sl_lo = (uint32_t)__shfl((int)psl2, (int)back), sl_hi = (uint32_t)__shfl((int)hsl2, (int)back);
    if (lane > fl && lane < fl + k) {
      w.wrm = ((uint64_t)rm_hi << 32) | rm_lo;
      w.wsl = ((uint64_t)sl_hi << 32) | sl_lo;
      w.ow = w.ow + 1u;
    }
  }
  // the window after k - 1 rotations with the k-th pending:
  // lane fl holds U_{k-1}, then U_k..U_{m-1} (count c), then
  // U_{k-2}..U_0 (count c + 1, each placed in front of the last)
  const uint32_t rel = lane - fl;
  uint32_t src = lane;
  if (lane >= fl && lane < fl + m) src = fl + (rel == 0 ? k - 1 : (rel <= m - k ? k - 1 + rel : m - 1 - rel));
  w.ow = (uint32_t)__shfl((int)w.ow, (int)src);
  w.wsl = shfl_u64(w.wsl, src);
  w.wrm = shfl_u64(w.wrm, src);
  w.wtok = (uint32_t)__shfl((int)w.wtok, (int)src);
  return w;
}

// The generic sort's one out-of-line body: the members arrive as scalar
// arguments and the sorter is rebuilt locally, so they stay in registers (a
// member function would reload them through a `this` pointer in scratch
// after every LDS store)
template <int SEQ, class U32 = lds_u32, class U16 = lds_u16, bool G = false, bool KNOWN = false>
__device__ __noinline__ void wave_pdqsort(U32* so, U16* scr, lds_frame* stk, uint32_t lane, uint32_t half, int n, int x
#ifdef GS_SORT_TL
                                          , uint64_t* stl = nullptr
#endif
) {
  n = __builtin_amdgcn_readfirstlane(n);
  x = __builtin_amdgcn_readfirstlane(x);
  half = __builtin_amdgcn_readfirstlane(half);
#ifdef GS_SORT_TL
  WaveSort<SEQ, U32, U16, G, KNOWN> w{so, scr, stk, lane, half};
  w.stl = stl;
#else
  const WaveSort<SEQ, U32, U16, G, KNOWN> w{so, scr, stk, lane, half};
#endif
  w.pdqsort_body(n, x);
}

// <U> Requirements.Compatible over the variant's free-key entries
__device__ __forceinline__ bool fk_ok_range(const DevProblem& d, uint32_t fb, uint32_t fc, const FK* cfk, bool strict) {
  for (uint32_t k = 0; k < fc; k++) {
    const FKEntry& e = d.fk_entries[fb + k];
    if (!fk_compatible(cfk[e.slot], e.st, strict ? false : ((d.wk_slots >> e.slot) & 1))) return false;
  }
  return true;
}

}  // namespace

// Go's choosePivot on n >= 50 elements samples the adjacent triples around
// n/4, n/2 and 3n/4 (medianAdjacent) and reports "increasing" iff no
// comparison swaps.  The array was sorted before this pod's Add, which
// changed one key: INC raised key(modpos), so the only inversion is
// (modpos, modpos + 1) and a swap needs both inside one triple (t-1, t, t+1),
// i.e. modpos in {t-1, t}; otherwise the triple medians stay ordered.  APPEND
// put the only out-of-order key at n-1, past every sampled position.  Only a
// touched sample needs the LDS reads of pivot_hint_wave.
__device__ __forceinline__ bool pivot_touched(uint32_t modkind, uint32_t modpos, uint32_t n) {
  if (modkind != MOD_INC) return false;
  const uint32_t q = n / 4;
  const uint32_t t[3] = {q, 2 * q, 3 * q};
  bool hit = false;
#pragma unroll
  for (int k = 0; k < 3; k++) hit = hit || modpos + 1 == t[k] || modpos == t[k];
  return hit;
}

// CH: the claim scan state (slack, room, sorted order, sort scratch,
// template) lives in HBM instead of LDS -- a Solve with more NodeClaims than
// the LDS holds (capi gs_run reruns it so)
// WIDE: option rows of more than WREG words (the launcher picks it from d.W):
// the narrow instantiation keeps a candidate's words in registers and
// carries none of the wide rows' lane-split code, and the other way round
template <uint32_t RR, bool TOPO, bool CH = false, bool WIDE = false>
__global__ __launch_bounds__(128, 1) void ffdw_kernel(DevProblem d) {
  constexpr bool KNOWN_PART = GS_KNOWN_PARTITION == 1 || (GS_KNOWN_PARTITION == 2 && TOPO);
  extern __shared__ uint64_t lds64[];
  __shared__ Frame s_stk[64];
#ifdef GS_SORT_TL
  __shared__ uint64_t s_stl[12];
  if (threadIdx.x < 12) s_stl[threadIdx.x] = 0;
#endif
  __shared__ uint64_t s_slot[SLOT_LDS_MAX];
  __shared__ uint64_t s_tzm[TMAX], s_tcm[TMAX];
  __shared__ uint32_t s_thoff[RMAX + 1];
  __shared__ uint32_t s_exl[64];  // exact-check batch: position | claim << 16
  // channels between the solver (wave 0) and the memory agent (wave 1)
  __shared__ uint32_t s_ring[RING][RING_DW];  // first-pass pod records
  __shared__ uint32_t s_ring_seq[RING];       // queue position + 1 held by each slot
  __shared__ uint32_t s_wq[WQ][WQ_DW];        // write requests
  __shared__ uint32_t s_ctl[4];               // [0] first-pass pops, [1] requests posted, [2] requests completed,
                                              // [3] solver heartbeat (pops)
  constexpr uint32_t R = RR;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t MC = CH ? (d.claim_cap < 65535u ? d.claim_cap : 65535u) : d.max_claims_wave;
  const uint32_t MCL = CH ? 0u : MC;  // NodeClaims in LDS
  // dynamic LDS, per claim 23 B (the block kernel's layout, ffd.hip):
  // slack u64 | room u64 | packed order u32 | sort scratch u16 | template u8
  uint64_t* s_slk = CH ? d.ch_slk : lds64;
  uint64_t* s_rm = CH ? d.ch_rm : s_slk + MC;
  uint32_t* s_so = CH ? d.ch_so : (uint32_t*)(s_rm + MC);
  uint16_t* s_scr = CH ? d.ch_scr : (uint16_t*)(s_so + MC);
  uint8_t* s_tmpl = CH ? d.ch_tmpl : (uint8_t*)(s_scr + MC);
  const uint32_t thr_base = (23u * MCL + 7u) & ~7u;
  int64_t* s_thr = (int64_t*)((char*)lds64 + thr_base);
  const uint32_t W = d.W, F = d.F, T = d.T, OW = d.OW, P = d.P;
  if (WIDE)
    __builtin_assume(W > WREG);
  else
    __builtin_assume(W <= WREG);
  const uint32_t nthr = d.thr_off[R];
  const uint32_t tg_off = (thr_base + (nthr + 4u) * 8u + 7u) & ~7u;
  const TopoS ts = topo_lds((char*)lds64 + tg_off, d.TGZ, d.ZS, d.TGH, d.n_lazy);
  // existing nodes (wave_node_lds_bytes): slack codes (upper bound), room
  // codes (lower bound) of available - requests per resource 0..3, and a
  // flag byte: bit 0 = plain (ok, no taints, resources 4.. not over)
  const uint32_t nd_off = (tg_off + topo_lds_bytes(d.TGZ, d.ZS, d.TGH, d.n_lazy) + 7u) & ~7u;
  uint64_t* s_nslk = (uint64_t*)((char*)lds64 + nd_off);
  uint64_t* s_nrm = (uint64_t*)((char*)lds64 + nd_off + d.NN * 8u);
  uint8_t* s_nflag = (uint8_t*)((char*)lds64 + nd_off + d.NN * 16u);
  const int64_t* thr = s_thr;
  const uint64_t* slot = s_slot;

  for (uint32_t i = tid; i < nthr + 4; i += 128) s_thr[i] = i < nthr ? d.thr_val[i] : INT64_MAX;
  for (uint32_t i = tid; i < d.Z * d.C * W; i += 128) s_slot[i] = d.slot_set[i];
  if (tid <= R) s_thoff[tid] = d.thr_off[tid];
  for (uint32_t t = tid; t < T; t += 128) {
    s_tzm[t] = d.tmpl[t].zm;
    s_tcm[t] = d.tmpl[t].cm;
  }
  if (TOPO) topo_init(d, ts, d.zknown0, tid, 128);
  for (uint32_t n = tid; n < d.NN; n += 128) {
    const NodeRec& nr = d.nodes0[n];
    int64_t sl[RR];
#pragma unroll
    for (uint32_t r = 0; r < RR; r++) sl[r] = nr.avail[r] - nr.req[r];
    uint64_t a = 0, b = 0;
    bool plain = nr.ok && nr.taints == 0;
#pragma unroll
    for (uint32_t r = 0; r < RR; r++) {
      if (r < 4 && r < d.RQ) {
        a |= (uint64_t)qcode_ceil(sl[r]) << (16 * r);
        b |= (uint64_t)qcode_floor(sl[r]) << (16 * r);
      }
      if (r >= 4) plain = plain && sl[r] >= 0;
    }
    s_nslk[n] = a;
    s_nrm[n] = b;
    s_nflag[n] = plain ? 1u : 0u;
  }
  if (tid < RING) s_ring_seq[tid] = 0;
  if (tid < 4) s_ctl[tid] = 0;
  __syncthreads();  // the only workgroup barrier: the waves split here

  if (wave == 1) {
    // ================================================== memory agent wave
    // (1) stages the next first-pass pod records (queue order) into the LDS
    //     ring ahead of the solver; (2) with GS_AGENT_WRITES=1 only (the
    //     round-2 design), performs the solver's posted global writes (add
    //     log, fast-accept request totals) and reports their completion; by
    //     default the solver issues them itself (fire-and-forget) and only
    //     the final WQ_STOP is posted.
    const uint32_t* qv_dw = (const uint32_t*)d.qvars;
    const uint32_t* qr_dw = (const uint32_t*)d.qreqs;
    uint32_t k_fill = 0, head = 0, idle = 0, beat = 0;
    for (;;) {
      bool busy = false, stop = false;
      const uint32_t tail = __builtin_amdgcn_readfirstlane(vld(&s_ctl[1]));
      while (head != tail) {
        const uint32_t x = lane < WQ_DW ? vld(&s_wq[head % WQ][lane]) : 0u;
        const uint32_t type = rlane(x, 0), idx = rlane(x, 1), tgt = rlane(x, 4);
        const uint32_t rlo = (uint32_t)__shfl((int)x, (int)(5 + 2 * (lane & 3))),
                       rhi = (uint32_t)__shfl((int)x, (int)(6 + 2 * (lane & 3)));
        if (type == WQ_STOP) {
          stop = true;
        } else {
          if (lane == 0) d.log[idx] = LogRec{rlane(x, 2), rlane(x, 3), type == WQ_NFA ? tgt | 0x80000000u : tgt, 0};
          const uint64_t a = (uint64_t)rlo | ((uint64_t)rhi << 32);
          if (type == WQ_FA && lane < R && lane < 4 && a)
            atomicAdd((unsigned long long*)&d.c_rec[tgt].tot_lo[lane], (unsigned long long)a);
          if (type == WQ_NFA && lane < R && lane < 4 && a)
            atomicAdd((unsigned long long*)&d.nodes[tgt].req[lane], (unsigned long long)a);
        }
        head++;
        busy = true;
      }
      if (busy) {
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the writes are done
        wsyncT<CH>();
        if (lane == 0) vst(&s_ctl[2], head);
      }
      if (stop) break;
      const uint32_t sq = __builtin_amdgcn_readfirstlane(vld(&s_ctl[0]));
      const uint32_t lim = P < sq + RING ? P : sq + RING;
      if (k_fill < lim) {
        constexpr uint32_t KB = 8;
        const uint32_t n = lim - k_fill < KB ? lim - k_fill : KB;
        uint32_t val[KB];
#pragma unroll
        for (uint32_t i = 0; i < KB; i++) {
          const size_t k = k_fill + i;
          val[i] = 0;
          if (i < n) {
            if (lane < VR_DW) val[i] = qv_dw[k * VR_DW + lane];
            else if (lane < 32 + 2 * R) val[i] = qr_dw[k * 2 * R + (lane - 32)];
            else if (lane >= RING_CODES && lane < RING_CODES + 4) val[i] = d.qcodes[k * 4 + (lane - RING_CODES)];
            else if (lane == RING_QRUN) val[i] = d.qrun[k];
          }
        }
#pragma unroll
        for (uint32_t i = 0; i < KB; i++)
          if (i < n && lane < RING_DW) s_ring[(k_fill + i) % RING][lane] = val[i];
        wsyncT<CH>();
#pragma unroll
        for (uint32_t i = 0; i < KB; i++)
          if (i < n && lane == 0) vst(&s_ring_seq[(k_fill + i) % RING], k_fill + i + 1);
        k_fill += n;
        busy = true;
      }
      // the agent leaves on WQ_STOP only; its bounded wait (a stuck solver
      // ends the kernel, not the GPU) restarts whenever the solver pops a pod,
      // so a long tail of pods that post nothing (failures, relaxations)
      // cannot outlast it
      const uint32_t hb = __builtin_amdgcn_readfirstlane(vld(&s_ctl[3]));
      if (busy || hb != beat) {
        idle = 0;
        beat = hb;
      } else {
#ifdef GS_AGENT_SLEEP
        __builtin_amdgcn_s_sleep(GS_AGENT_SLEEP);
#else
        __builtin_amdgcn_s_sleep(1);
#endif
        if (++idle > SPIN_MAX) break;
      }
    }
    return;
  }

  // ======================================================== solver wave
  using U32 = std::conditional_t<CH, uint32_t, lds_u32>;
  using U16 = std::conditional_t<CH, uint16_t, lds_u16>;
  const WaveSort<GS_WAVE_SEQ, U32, U16, CH> ws{(U32*)s_so, (U16*)s_scr, (lds_frame*)s_stk, lane, MC / 2};
  const PackedAccT<U32> acc{(U32*)s_so};
  uint32_t wq_tail = 0;  // write requests posted
  uint32_t wq_seen = 0;  // completions last read from s_ctl[2] (posting waits only when that looks full)
  // Infeasible-prefix hint: sorted positions [0, hint) hold NodeClaims that
  // cannot take a pod with requests >= hint_rq (resources 0..3) that
  // tolerates no template outside hint_tolt.  NodeClaims only fill up
  // (requests grow, options shrink), so the prefix stays infeasible; every
  // reorder of the sorted order moves the bound exactly (or drops it).
  // Pods come sorted by cpu, then memory, descending: runs of equal
  // requests skip the prefix their predecessors already ruled out.
  uint32_t hint = 0;
  bool hint_ok = false;
  uint64_t hint_tolt = 0;
  int64_t hint_rq = 0;  // lane r < 4: that pod's request r
  // Existing nodes: positions [0, nhint) cannot take a pod whose requests are
  // all >= hint_nrq and that tolerates no taint outside nhint_tol (nodes
  // only fill up; a pod with requirements, topology or volumes is only more
  // constrained).  Set by plain pods (no requirements, topology, volumes).
  uint32_t nhint = 0;
  bool nhint_ok = false;
  uint64_t nhint_tol = 0;
  int64_t hint_nrq = 0;  // lane r < R: that pod's request r
  bool chan_err = false;  // a channel wait exceeded SPIN_MAX
  // post one write request (uniform control flow: every lane takes part):
  // lanes 0..4 the header, lanes 32.. (the record's request dwords) dwords 5..
  auto post = [&](uint32_t type, uint32_t idx, uint32_t pod, uint32_t var, uint32_t tgt, uint32_t rqd_) {
    if (wq_tail - wq_seen >= WQ) {
      for (uint32_t spin = 0;; spin++) {
        wq_seen = __builtin_amdgcn_readfirstlane(vld(&s_ctl[2]));
        if (wq_tail - wq_seen < WQ) break;
        __builtin_amdgcn_s_sleep(1);
        if (spin > SPIN_MAX) {
          chan_err = true;
          break;
        }
      }
    }
    const uint32_t x = lane == 0 ? type : lane == 1 ? idx : lane == 2 ? pod : lane == 3 ? var : lane == 4 ? tgt : rqd_;
    const bool rqw = (type == WQ_FA || type == WQ_NFA) && lane >= 32 && lane < 40;
    if (lane < 5 || rqw) s_wq[wq_tail % WQ][lane < 5 ? lane : lane - 27] = x;
    wsyncT<CH>();
    if (lane == 0) vst(&s_ctl[1], wq_tail + 1);
    wq_tail++;
  };
  // wait until every posted write has completed (before reading claim state)
  auto drain = [&]() {
    for (uint32_t spin = 0; __builtin_amdgcn_readfirstlane(vld(&s_ctl[2])) != wq_tail; spin++) {
      __builtin_amdgcn_s_sleep(1);
      if (spin > SPIN_MAX) {
        chan_err = true;
        break;
      }
    }
  };

  // Solver-side global writes (GS_AGENT_WRITES=0, the default): the add log
  // entry (lane 0) and, for a requests-only Add, the no-return atomic adds
  // of the requests (lanes r < min(R, 4)).  They are fire-and-forget: the
  // next exact check's loads wait on the vector memory counter, which the
  // wave's earlier stores and atomics precede, instead of draining the
  // agent's channel.
#ifndef GS_AGENT_WRITES
#define GS_AGENT_WRITES 0
#endif
  auto emit = [&](uint32_t type, uint32_t idx, uint32_t pod, uint32_t var, uint32_t tgt, uint32_t rqd_, int64_t rql) {
    if (GS_AGENT_WRITES) {
      post(type, idx, pod, var, tgt, rqd_);
      return;
    }
    const auto& KD = *karg();
    if (lane == 0) KD.log[idx] = LogRec{pod, var, type == WQ_NFA ? tgt | 0x80000000u : tgt, 0};
    if ((type == WQ_FA || type == WQ_NFA) && lane < R && lane < 4 && rql != 0) {
      unsigned long long* a = type == WQ_FA ? (unsigned long long*)&KD.c_rec[tgt].tot_lo[lane]
                                            : (unsigned long long*)&KD.nodes[tgt].req[lane];
      atomicAdd(a, (unsigned long long)rql);
    }
  };

  // uniform loop state (scalar registers)
  uint32_t qhead = 0, qlen = P, epoch = 1, M = 0, modkind = MOD_NONE, modpos = 0, nlog = 0, status = 0;
  bool wrapped = false;
  uint64_t pops = 0;
  // instrumentation counters, lane k = counter k (no scalar registers)
  enum { C_GEN = 0, C_FAST, C_CAND, C_FULL, C_NEV, C_NPRE, C_FA, C_ALG,
         // run mode (diagnostics, Ctrl.dbg[8..13] outside the timeline build)
         C_RPODS, C_RENTER, C_RX_PIVOT, C_RX_WIN, C_RX_SPEC, C_RX_SCAN, C_RX_XC, C_RBATCH, C_RBPODS, C_RBT0, C_RBT1 };
  uint64_t ctr = 0;
#ifdef GS_NO_CTR  // experiment builds: the counters' cost
#define CTR(k, x) ((void)0)
#elif defined(GS_CTR_LDS)  // experiment: counters as no-return LDS atomic adds by lane 0
  __shared__ unsigned long long s_ctr[8];
  if (lane < 8) s_ctr[lane] = 0;
  wsync();
#define CTR(k, x)                                                        \
  do {                                                                   \
    if (lane == 0) atomicAdd(&s_ctr[(k)], (unsigned long long)(x));     \
  } while (0)
#else
#define CTR(k, x) (ctr += lane == (k) ? (uint64_t)(x) : 0ull)
#endif
  const uint64_t max_pops = ((uint64_t)(d.V - d.P) + 2) * (uint64_t)P + P + 16;

#ifdef GS_FFD_TL
#ifdef GS_CAT_SEG
  uint64_t ptl[8] = {0, 0, 0, 0, 0, 0, 0, 0}, n_cat = 0;
#endif
  uint64_t tl[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tl_last = __builtin_amdgcn_s_memtime();
  uint64_t n_fsum = 0, n_xns = 0, n_xb = 0, n_xwin = 0, n_nonsimple = 0, n_rot = 0, n_rotlen = 0, n_gen_cyc = 0;
#endif
  uint32_t pf_x = 0, pf_seq = 0;  // prefetched ring record and its sequence word
  // Runs of identical simple pods (GS_RUNS).  Queue order puts equal
  // requests together (cpu, memory descending), so most first-pass pods
  // repeat the previous pod's spec (CM: 88 % of pods, runs of 8 on average).
  // For such a pod the whole NodeClaim.CanAdd chain -- the pending one-claim
  // sort.Slice rotation, the scan from the infeasible-prefix bound, the fast
  // accept -- only reads and writes the 64 sorted positions from the last
  // Add on: the run keeps that window (order word, slack and room codes,
  // template tolerated) in registers and places pod after pod there, with the
  // same rotation, ballots and code arithmetic as the LDS path, so the result
  // is bit-identical.  Anything else (a pivot sample touched, a run of equal
  // keys leaving the window, a candidate needing the exact check, no
  // candidate in the window, another spec) writes the window back and hands
  // the pod to the general path below.
#ifndef GS_RUNS
#define GS_RUNS 1
#endif
#ifndef GS_RUN_EXACT
#define GS_RUN_EXACT 1
#endif
#ifndef GS_RUN_REBASE
#define GS_RUN_REBASE 1
#endif
#ifndef GS_RUN_NODES
#define GS_RUN_NODES 1
#endif
// GS_RUN_BATCH=1: up to 16 pods of a run placed in one step (round 6,
// bit-exact).  Off by default: it cuts run-mode cycles per pod 4,225 -> 3,914
// on CM, but the pod loop's register allocation around the added code costs
// the general path as much (same session, FFD ms: CM 283.2 -> 282.9, C2
// 36.4 -> 37.7, C1 3.18 -> 3.51; profiles/r6/run_batch_*.txt)
#ifndef GS_RUN_BATCH
#define GS_RUN_BATCH 0
#endif
#ifndef GS_RUN_WIDE  // the wide-row instantiation in run mode
#define GS_RUN_WIDE 0
#endif
#ifndef GS_RUN_WIDE_EXACT  // ... with the window's exact checks, one candidate at a time over all lanes
#define GS_RUN_WIDE_EXACT 1
#endif
#ifdef GS_RUN_TL
  uint64_t run_cyc = 0;  // s_memtime ticks inside run mode
#endif
#ifdef GS_CAT_TL
  // diagnostic build: shader cycles per pod category (lane k = category k):
  // 0 run mode, 1 simple pod on an in-flight claim, 3 other pod on an
  // in-flight claim, 4 new NodeClaim, 5 failed (relax / push), 6 on an
  // existing node
  uint64_t cat_cyc = 0, cat_n = 0, cat_t = __builtin_amdgcn_s_memtime();
  uint32_t cat_k = 7;
#define CAT(k) (cat_k = (k))
#else
#define CAT(k) ((void)0)
#endif
  bool run_prev = false;  // the last pod was a first-pass simple pod placed on an in-flight NodeClaim
  uint32_t run_rec = 0;   // its ring record (lanes: VarRec dwords, requests, request codes)
  for (;;) {
    // ---------------------------------------------------------- Queue.Pop
    TLW(7);  // previous pod's tail (continue paths)
#ifdef GS_CAT_TL
    {
      const uint64_t t_ = __builtin_amdgcn_s_memtime();
      cat_cyc += lane == cat_k ? t_ - cat_t : 0ull;
      cat_n += lane == cat_k && cat_k != 0 ? 1ull : 0ull;
      cat_t = t_;
#if defined(GS_FFD_TL) && defined(GS_CAT_SEG)
      if (cat_k == GS_CAT_SEG) {
        n_cat++;
#pragma unroll
        for (int q = 0; q < 8; q++) tl[q] += ptl[q];
      }
#pragma unroll
      for (int q = 0; q < 8; q++) ptl[q] = 0;
#endif
      cat_k = 7;
    }
#endif
    if (status) break;
    if (pops > max_pops) {
      status = 2;
      break;
    }
    if (qlen == 0) break;
    // (the narrow non-topology instantiation only: the topology and wide-row
    // instantiations measured slower with the run code in them, C3 398 -> 420,
    // e2e 273 -> 283, C5 1,245 -> 1,292 ms, profiles/r5/runs_ab.txt)
    // (existing nodes: only once the run's spec is known to fit none of them --
    // its last general pod, a plain pod, set the node hint past the last node;
    // nodes only fill up and no run pod is placed on one)
    if (GS_RUNS && !TOPO && (!WIDE || GS_RUN_WIDE) && run_prev && !wrapped && modkind == MOD_INC && M >= 50 &&
        (d.NN == 0 || (GS_RUN_NODES && nhint_ok && nhint >= d.NN))) {
      run_prev = false;
      auto same_spec = [&](uint32_t x) {
        return __ballot(lane >= 1 && lane < RING_QRUN && lane != VR_DW - 1 && x != run_rec) == 0;
      };
      if (__builtin_amdgcn_readfirstlane(pf_seq) == qhead + 1 && same_spec(pf_x)) {
        // the run's spec: tolerated templates, request codes and requests
        const uint64_t r_tolt = (uint64_t)rlane(run_rec, 20) | ((uint64_t)rlane(run_rec, 21) << 32);
        const uint64_t r_rqq = (uint64_t)rlane(run_rec, RING_CODES) | ((uint64_t)rlane(run_rec, RING_CODES + 1) << 32);
        const uint64_t r_rqc = (uint64_t)rlane(run_rec, RING_CODES + 2) | ((uint64_t)rlane(run_rec, RING_CODES + 3) << 32);
        int64_t r_rq = 0;  // lane r < R: request r
        {
          const uint32_t lo = (uint32_t)__shfl((int)run_rec, (int)(32 + 2 * (lane & 7))),
                         hi = (uint32_t)__shfl((int)run_rec, (int)(33 + 2 * (lane & 7)));
          if (lane < RR) r_rq = (int64_t)(((uint64_t)hi << 32) | lo);
        }
        // the window: sorted positions [base, base + 64), the last Add's claim at lane 0
        uint32_t base = modpos;
        uint32_t wpos = base + lane;
        bool valid = wpos < M;
        uint32_t ow = 0;
        uint64_t wsl = 0, wrm = 0;
        uint32_t wtok = 0;
        auto load_window = [&]() {
          wpos = base + lane;
          valid = wpos < M;
          ow = valid ? (uint32_t)s_so[wpos] : 0xFFFFu;  // past M: key 0xFFFF ends every run of equal keys
          wsl = wrm = 0;
          wtok = 0;
          if (valid) {
            const uint32_t je = ow >> 16;
            wsl = s_slk[je];
            wrm = s_rm[je];
            wtok = (uint32_t)((r_tolt >> (T > 1 ? (uint32_t)s_tmpl[je] : 0u)) & 1u);
          }
        };
        load_window();
        uint32_t lf = 0;  // lane of the claim the last Add raised
        bool dirty = false;
        CTR(C_RENTER, 1);
        CAT(0);
#ifdef GS_RUN_TL
        const uint64_t rt0 = __builtin_amdgcn_s_memtime();
#endif
        for (;;) {
          // sort.Slice: the raised claim moves to the end of its run of equal keys
          const uint32_t x = rlane(ow, lf) & 0xFFFFu;
          const bool ptouch = pivot_touched(MOD_INC, modpos, M);
          const uint64_t b = ptouch ? 0ull : __ballot(lane > lf && (ow & 0xFFFFu) >= x);
          const uint32_t eo = b ? ffs64(b) : 64u;
          if (!b) {
            // a pivot sample touched, or the raised claim's run of equal keys
            // leaves the window (GS_RUN_REBASE): the window goes back to LDS,
            // the general path's sort step runs there (one rotation past the
            // run; with a touched sample only when choosePivot still reports
            // "increasing", else the pod leaves for the general sort), and
            // the window is re-read at the infeasible-prefix bound (modpos:
            // the claims after it moved one position left)
            CTR(ptouch ? C_RX_PIVOT : C_RX_WIN, 1);
            if (!GS_RUN_REBASE) break;
            wsyncT<CH>();
            if (dirty && valid) {
              s_so[wpos] = ow;
              s_slk[ow >> 16] = wsl;
              s_rm[ow >> 16] = wrm;
            }
            wsyncT<CH>();
            dirty = false;
            const uint32_t e2 = wave_first(modpos + 1, M, lane, [&](uint32_t k) { return acc.key(k) >= x; });
            if (e2 > modpos + 1) {
              if (ptouch && pivot_hint_wave(acc, (int)M, lane) != 1) break;  // Go's full pdqsort: the general path
              CTR(C_FAST, 1);
              ws.rotate((int)modpos, (int)e2 - 1, true);
              if (modpos < hint && e2 - 1 >= hint) hint--;
            }
            base = modpos;
            load_window();
            lf = 0;
          } else if (eo > lf + 1) {
            CTR(C_FAST, 1);
            auto rot = [&](uint32_t y) -> uint32_t {
              const uint32_t sh = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)y, 0x130, 0xF, 0xF, false);  // lane i <- i + 1
              const uint32_t y0 = rlane(y, lf);
              return lane + 1 == eo ? y0 : (lane >= lf && lane + 1 < eo) ? sh : y;
            };
            ow = rot(ow);
            wsl = ((uint64_t)rot((uint32_t)(wsl >> 32)) << 32) | rot((uint32_t)wsl);
            wrm = ((uint64_t)rot((uint32_t)(wrm >> 32)) << 32) | rot((uint32_t)wrm);
            wtok = rot(wtok);
            dirty = true;
          }
          modkind = MOD_NONE;
          // the next pod: the same spec, staged in the ring?
          if (!(__builtin_amdgcn_readfirstlane(pf_seq) == qhead + 1 && same_spec(pf_x))) {
            CTR(C_RX_SPEC, 1);
            break;
          }
          if (pops + 1 > max_pops || qhead + 1 == P) break;
          // the scan from the infeasible-prefix bound (the last Add's
          // position): the first candidate must be a fast accept
          const uint32_t lo = modpos - base;
          const bool lp = (lane >= lo) & valid & (wtok != 0) & swar_ge(wsl, r_rqq);
          const uint64_t lpb = __ballot(lp), fab = __ballot(lp & swar_ge(wrm, r_rqc));
          if (!lpb) {
            CTR(C_RX_SCAN, 1);
            break;
          }
          uint32_t fl = ffs64(lpb);
          // The exact NodeClaim.CanAdd inside the run (GS_RUN_EXACT): the
          // window's candidates before its first fast accept that need it (a
          // threshold cursor would move) are checked one lane each, as the
          // general path's phase B checks the same batch; the first feasible
          // one wins, else the fast accept; with neither in the window the pod
          // leaves the run (the general path scans on past it)
          bool xwin = false;
          uint64_t x_nx[WREG] = {0, 0, 0, 0};
          uint64_t x_w[2] = {0, 0};  // wide rows: this lane's option words (lane, lane + 64) after the Add
          int64_t x_tot[RR], x_ma[RR];
          uint32_t x_mrow[RR];
          uint64_t x_zm = 0;
#pragma unroll
          for (uint32_t r = 0; r < RR; r++) {
            x_tot[r] = 0;
            x_ma[r] = 0;
            x_mrow[r] = 0;
          }
          const uint64_t vzm = (uint64_t)rlane(run_rec, 14) | ((uint64_t)rlane(run_rec, 15) << 32);
          const uint64_t vcm = (uint64_t)rlane(run_rec, 16) | ((uint64_t)rlane(run_rec, 17) << 32);
          auto RQV = [&](uint32_t r) -> int64_t {
            return (int64_t)((uint64_t)rlane(run_rec, 32 + 2 * r) | ((uint64_t)rlane(run_rec, 33 + 2 * r) << 32));
          };
          if (!(fab & 1ull << fl)) {
            if (!GS_RUN_EXACT || (WIDE && !GS_RUN_WIDE_EXACT) || rlane(run_rec, 2) != 0) {  // free-key entries: the general path
              CTR(C_RX_SCAN, 1);
              break;
            }
            const uint32_t mfl = fab ? ffs64(fab) : 64u;
            const uint64_t ex = lpb & ~fab & (mfl == 64 ? ~0ull : ((1ull << mfl) - 1ull));
            const auto& KD = *karg();
            const uint32_t pvx = rlane(pf_x, VR_DW - 1);  // the next pod's variant (its K1 rows)
            bool feas = false;
            uint64_t fm = 0;
            if (WIDE) {
              // wide rows: the candidates one after another in window order,
              // every lane one option word (and the word 64 on); the first
              // feasible one wins, as in the general path's batch
              for (uint64_t exw = ex; exw; exw &= exw - 1) {
                const uint32_t c = ffs64(exw);
                const uint32_t j = rlane(ow, c) >> 16;
                const uint32_t t = T > 1 ? (uint32_t)s_tmpl[j] : 0u;
                const ClaimRec* cr = KD.c_rec + j;
                uint32_t cur[RR];
#pragma unroll
                for (uint32_t r = 0; r < RR; r++) x_ma[r] = cr->maxa[r];
                uint64_t x_cm;
                {
                  const uint4* q = (const uint4*)cr;
                  const uint4 h0 = q[0], h1 = q[1], h2 = q[2], h3 = q[3];
                  const int64_t tl4[4] = {(int64_t)(((uint64_t)h0.y << 32) | h0.x), (int64_t)(((uint64_t)h0.w << 32) | h0.z),
                                          (int64_t)(((uint64_t)h1.y << 32) | h1.x), (int64_t)(((uint64_t)h1.w << 32) | h1.z)};
                  const uint32_t cl[4] = {h2.x & 0xFFFFu, h2.x >> 16, h2.y & 0xFFFFu, h2.y >> 16};
                  x_zm = ((uint64_t)h2.w << 32) | h2.z;
                  x_cm = ((uint64_t)h3.y << 32) | h3.x;
#pragma unroll
                  for (uint32_t r = 0; r < RR; r++) {
                    x_tot[r] = r < 4 ? tl4[r] : cr->tot_hi[r - 4];
                    cur[r] = r < 4 ? cl[r] : cr->thr_hi[r - 4];
                  }
                }
                const uint64_t G = grid_of(x_zm & vzm, x_cm & vcm, KD.Z, KD.C);
                const uint64_t Gt = grid_of(s_tzm[t] & vzm, s_tcm[t] & vcm, KD.Z, KD.C);
                uint32_t mm[RR];
#pragma unroll
                for (uint32_t r = 0; r < RR; r++) {
                  const uint32_t o = s_thoff[r], n = s_thoff[r + 1] - o;
                  mm[r] = thr_window(thr + o, n, cur[r], x_tot[r] + RQV(r));
                  if (mm[r] == cur[r] + 4 && mm[r] < n) mm[r] = thr_search(thr + o, n, mm[r], x_tot[r] + RQV(r));
                  x_mrow[r] = o + r + mm[r];
                }
                const uint64_t* row = KD.rows + ((size_t)pvx * T + t) * OW;
                const uint64_t* opts = KD.c_opts + (size_t)j * OW;
                bool anyw = false;
#pragma unroll
                for (uint32_t h = 0; h < 2; h++) {
                  const uint32_t w = lane + 64 * h;
                  uint64_t x = 0;
                  if (w < W) {
                    x = opts[w] & row[w];
#pragma unroll
                    for (uint32_t r = 0; r < RR; r++)
                      if (mm[r] != cur[r]) x &= KD.thr_set[(size_t)x_mrow[r] * OW + w];
                    if (G != Gt) {
                      uint64_t off = 0;
                      for (uint64_t gm = G; gm; gm &= gm - 1) off |= slot[(size_t)ffs64(gm) * W + w];
                      x &= off;
                    }
                  }
                  x_w[h] = x;
                  anyw = anyw || x != 0;
                }
                if (__ballot(anyw)) {
                  fm = 1ull << c;
                  break;
                }
              }
            } else if ((ex >> lane) & 1) {
              const uint32_t j = ow >> 16;
              const uint32_t t = T > 1 ? (uint32_t)s_tmpl[j] : 0u;
              const ClaimRec* cr = KD.c_rec + j;
              uint32_t cur[RR];
#pragma unroll
              for (uint32_t r = 0; r < RR; r++) x_ma[r] = cr->maxa[r];
              uint64_t x_cm;
              {
                const uint4* q = (const uint4*)cr;
                const uint4 h0 = q[0], h1 = q[1], h2 = q[2], h3 = q[3];
                const int64_t tl4[4] = {(int64_t)(((uint64_t)h0.y << 32) | h0.x), (int64_t)(((uint64_t)h0.w << 32) | h0.z),
                                        (int64_t)(((uint64_t)h1.y << 32) | h1.x), (int64_t)(((uint64_t)h1.w << 32) | h1.z)};
                const uint32_t cl[4] = {h2.x & 0xFFFFu, h2.x >> 16, h2.y & 0xFFFFu, h2.y >> 16};
                x_zm = ((uint64_t)h2.w << 32) | h2.z;
                x_cm = ((uint64_t)h3.y << 32) | h3.x;
#pragma unroll
                for (uint32_t r = 0; r < RR; r++) {
                  x_tot[r] = r < 4 ? tl4[r] : cr->tot_hi[r - 4];
                  cur[r] = r < 4 ? cl[r] : cr->thr_hi[r - 4];
                }
              }
              const uint64_t* row = KD.rows + ((size_t)pvx * T + t) * OW;
              const uint64_t* opts = KD.c_opts + (size_t)j * OW;
              {
                const uint4* oq = (const uint4*)opts;
                const uint4* rq4 = (const uint4*)row;
                const uint4 o0 = oq[0], o1 = oq[1], r0 = rq4[0], r1 = rq4[1];
                const uint64_t a[4] = {(((uint64_t)o0.y << 32) | o0.x) & (((uint64_t)r0.y << 32) | r0.x),
                                       (((uint64_t)o0.w << 32) | o0.z) & (((uint64_t)r0.w << 32) | r0.z),
                                       (((uint64_t)o1.y << 32) | o1.x) & (((uint64_t)r1.y << 32) | r1.x),
                                       (((uint64_t)o1.w << 32) | o1.z) & (((uint64_t)r1.w << 32) | r1.z)};
#pragma unroll
                for (uint32_t w = 0; w < WREG; w++) x_nx[w] = w < W ? a[w] : 0;
              }
              const uint64_t G = grid_of(x_zm & vzm, x_cm & vcm, KD.Z, KD.C);
              const uint64_t Gt = grid_of(s_tzm[t] & vzm, s_tcm[t] & vcm, KD.Z, KD.C);
              uint32_t mm[RR];
#pragma unroll
              for (uint32_t r = 0; r < RR; r++) {
                const uint32_t o = s_thoff[r], n = s_thoff[r + 1] - o;
                mm[r] = thr_window(thr + o, n, cur[r], x_tot[r] + RQV(r));
              }
#pragma unroll
              for (uint32_t r = 0; r < RR; r++) {
                const uint32_t o = s_thoff[r], n = s_thoff[r + 1] - o;
                if (mm[r] == cur[r] + 4 && mm[r] < n) mm[r] = thr_search(thr + o, n, mm[r], x_tot[r] + RQV(r));
                x_mrow[r] = o + r + mm[r];
              }
#pragma unroll
              for (uint32_t r = 0; r < RR; r++) {
                if (mm[r] != cur[r]) {
                  const uint4* tq = (const uint4*)(KD.thr_set + (size_t)x_mrow[r] * OW);
                  const uint4 t0 = tq[0], t1 = tq[1];
                  x_nx[0] &= ((uint64_t)t0.y << 32) | t0.x;
                  x_nx[1] &= ((uint64_t)t0.w << 32) | t0.z;
                  x_nx[2] &= ((uint64_t)t1.y << 32) | t1.x;
                  x_nx[3] &= ((uint64_t)t1.w << 32) | t1.z;
                }
              }
              if (G != Gt) {
                uint64_t off[WREG] = {};
                for (uint64_t gm = G; gm; gm &= gm - 1) {
                  const uint32_t g = ffs64(gm);
#pragma unroll
                  for (uint32_t w = 0; w < WREG; w++)
                    if (w < W) off[w] |= slot[g * W + w];
                }
#pragma unroll
                for (uint32_t w = 0; w < WREG; w++) x_nx[w] &= off[w];
              }
              uint64_t accw = 0;
#pragma unroll
              for (uint32_t w = 0; w < WREG; w++) accw |= x_nx[w];
              feas = accw != 0;
            }
            CTR(C_FULL, __popcll(ex));
            CTR(C_RX_XC, 1);
            if (!WIDE) fm = __ballot(feas);
            if (fm) {
              fl = ffs64(fm);
              xwin = true;
            } else if (fab) {
              fl = mfl;
            } else {
              CTR(C_RX_SCAN, 1);
              break;
            }
          }
          const uint32_t e = rlane(ow, fl);
          if ((e & 0xFFFFu) == 0xFFFFu) {
            status = 3;  // the u16 pod count would overflow
            break;
          }
          // Queue.Pop of the pod (first pass: the ring record at qhead)
          const uint32_t x_rec = pf_x;
          const uint32_t pp = rlane(x_rec, 0), pv = rlane(x_rec, VR_DW - 1);
          wsyncT<CH>();
          if (lane == 0) vst(&s_ctl[0], qhead + 1);  // the slot may be refilled
          qhead++;
          qlen--;
          pops++;
          if ((pops & 15) == 0 && lane == 0) vst(&s_ctl[3], (uint32_t)pops);
          pf_seq = vld(&s_ring_seq[qhead % RING]);
          pf_x = lane < RING_DW ? vld(&s_ring[qhead % RING][lane]) : 0u;
          if (xwin) {
            // NodeClaim.Add after the exact check, by the winning lane (as
            // the general path's): options, requests, cursors, the exact
            // slack / room codes, requirements; the window takes the codes
            const auto& KD = *karg();
            const uint32_t vctb = rlane(run_rec, 3);
            if (WIDE) {
              // the winner's option words, one lane per word
              uint64_t* wopts = KD.c_opts + (size_t)(e >> 16) * OW;
#pragma unroll
              for (uint32_t h = 0; h < 2; h++)
                if (lane + 64 * h < W) wopts[lane + 64 * h] = x_w[h];
            }
            if (lane == fl) {
              const uint32_t j = ow >> 16;
              ClaimRec* cr = KD.c_rec + j;
              uint64_t* opts = KD.c_opts + (size_t)j * OW;
              if (!WIDE) {
#pragma unroll
                for (uint32_t w = 0; w < WREG; w++)
                  if (w < W) opts[w] = x_nx[w];
              }
              int64_t nt[RR];
              uint32_t cu[RR];
#pragma unroll
              for (uint32_t r = 0; r < RR; r++) {
                nt[r] = x_tot[r] + RQV(r);
                cu[r] = x_mrow[r] - s_thoff[r] - r;
                cr->tot(r) = nt[r];
                cr->thr(r) = (uint16_t)cu[r];
              }
              wsl = pack_slack(d, x_ma, nt);
              wrm = pack_room(thr, s_thoff, cu, nt, KD.RQ);
              s_slk[j] = wsl;
              s_rm[j] = wrm;
              cr->zm = x_zm & vzm;
              cr->cm &= vcm;
              cr->ctb &= vctb;
              ow = e + 1u;
            }
            dirty = true;
            const uint32_t f = base + fl;
            wsyncT<CH>();
            emit(WQ_LOG, nlog, pp, pv, e >> 16, 0, 0);
            nlog++;
            CTR(C_CAND, M - modpos < 64 ? M - modpos : 64);
            CTR(C_ALG, f + 1);
            CTR(C_NPRE, d.NN);  // every existing node was tried first
            CTR(C_RPODS, 1);
#ifdef GS_CAT_TL
            cat_n += lane == 0 ? 1ull : 0ull;
#endif
            hint = f;
            modkind = MOD_INC;
            modpos = f;
            lf = fl;
            continue;
          }
          // fast accept: NodeClaim.Add changes the requests only; room and
          // slack of lane fl shrink by the request (lanes r < RQ re-quantize
          // resource r, packed across lanes 0..3 as in the general path)
          const uint64_t rm = ((uint64_t)rlane((uint32_t)(wrm >> 32), fl) << 32) | rlane((uint32_t)wrm, fl);
          const uint64_t sl = ((uint64_t)rlane((uint32_t)(wsl >> 32), fl) << 32) | rlane((uint32_t)wsl, fl);
          uint32_t c_rm = 0, c_sl = 0;
          if (lane < d.RQ) {
            const uint32_t sh = 16 * lane;
            c_rm = qcode_floor(qcode_value((uint32_t)(rm >> sh) & 0xFFFFu) - r_rq);
            c_sl = qcode_ceil(qcode_value((uint32_t)(sl >> sh) & 0xFFFFu) - r_rq);
          }
          uint32_t prm = (lane & 1u) ? c_rm << 16 : c_rm, psl = (lane & 1u) ? c_sl << 16 : c_sl;
          prm |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)prm, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
          psl |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)psl, 0xB1, 0xF, 0xF, false);
          const uint32_t hrm = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)prm, 0x102, 0xF, 0xF, false);  // row_shl:2
          const uint32_t hsl = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)psl, 0x102, 0xF, 0xF, false);
          const uint64_t nrm = (uint64_t)rlane(prm, 0) | ((uint64_t)rlane(hrm, 0) << 32);
          const uint64_t nsl = (uint64_t)rlane(psl, 0) | ((uint64_t)rlane(hsl, 0) << 32);
          if (lane == fl) {
            wrm = nrm;
            wsl = nsl;
            ow = e + 1u;
          }
          dirty = true;
          const uint32_t f = base + fl;
          emit(WQ_FA, nlog, pp, pv, e >> 16, run_rec, r_rq);  // the requests into the claim totals, and the log
          nlog++;
          CTR(C_CAND, M - modpos < 64 ? M - modpos : 64);
          CTR(C_FA, 1);
          CTR(C_ALG, f + 1);
          CTR(C_NPRE, d.NN);  // every existing node was tried first
          CTR(C_RPODS, 1);
#ifdef GS_CAT_TL
          cat_n += lane == 0 ? 1ull : 0ull;
#endif
          hint = f;
          modkind = MOD_INC;
          modpos = f;
          lf = fl;
#if GS_RUN_BATCH
          // A batch of the run's next pods.  This pod
          // joined U_0, the claim at lane fl (count c -> c + 1); U_1.. at
          // lanes fl + 1.. are the other count-c claims (up to lane e2).
          // sort.Slice moves U_0 behind them, so the next pod's scan (from
          // position f: the prefix before it stays infeasible) finds U_1 at f;
          // if U_1 is a fast accept (its bit in this scan's fab) the pod joins
          // it, its sort.Slice is the same one rotation from the same position
          // f (one choosePivot check for all), and so on: pod j joins U_j.
          // While U_j is a fast accept and the ring holds the next record of
          // the run's spec (qrun), up to 16 pods are placed here at once --
          // log entries and request atomics lane-parallel, U_j's codes
          // re-quantized on its own lane, the window permuted once -- and the
          // last pod's rotation stays pending as after a single Add.
          // Bit-identical to placing them one by one.
          {
#ifdef GS_RUN_TL
            const uint64_t tb0 = __builtin_amdgcn_s_memtime();
#endif
            const uint32_t c = e & 0xFFFFu;
            const uint64_t after = __ballot(lane > fl && (ow & 0xFFFFu) > c);
            uint32_t k = 1;
            if (after && c + 2u < 0xFFFFu && !pivot_touched(MOD_INC, f, M)) {
              const uint32_t m = ffs64(after) - fl;  // U_0..U_{m-1} at lanes fl..fl + m - 1
              k = 1u + (uint32_t)__builtin_ctzll(~(fab >> (fl + 1)));
              k = k < m ? k : m;
              const uint32_t nrun = rlane(x_rec, RING_QRUN);
              k = k < nrun ? k : nrun;
              const uint32_t q1 = qhead - 1;  // this pod's queue position
              if (q1 + k > P - 1) k = P - 1 - q1;
              if (pops + k > max_pops) k = 1;
              if (k >= 2) {
                // pods 2..k (lanes j = 1..k-1, queue position q1 + j): the
                // sequence word, pod and variant in one LDS round trip
                const bool jl = lane >= 1 && lane < k;
                const uint32_t slot = (q1 + lane) % RING;
                const uint32_t sq = jl ? vld(&s_ring_seq[slot]) : 0u;
                const uint32_t bp = jl ? vld(&s_ring[slot][0]) : 0u;
                const uint32_t bv = jl ? vld(&s_ring[slot][VR_DW - 1]) : 0u;
                k = 1u + (uint32_t)__builtin_ctzll(~(__ballot(jl && sq == q1 + lane + 1) >> 1));
#ifdef GS_RUN_TL
                const uint64_t tb1 = __builtin_amdgcn_s_memtime();
#endif
                if (k >= 2) {
                  const auto& KD = *karg();
                  RunWin rw{ow, wtok, wsl, wrm};
                  rw = run_batch_place<RR>(rw, (uint64_t)r_rq, bp, bv, fl, m, k, nlog, d.RQ, KD.log, KD.c_rec);
                  ow = rw.ow;
                  wtok = rw.wtok;
                  wsl = rw.wsl;
                  wrm = rw.wrm;
                  // Queue.Pop of pods 2..k: their ring slots may be refilled
                  wsyncT<CH>();
                  if (lane == 0) {
                    vst(&s_ctl[0], q1 + k);
                    vst(&s_ctl[3], (uint32_t)(pops + k - 1));
                  }
                  qhead = q1 + k;
                  qlen -= k - 1;
                  pops += k - 1;
                  nlog += k - 1;
                  pf_seq = vld(&s_ring_seq[qhead % RING]);
                  pf_x = lane < RING_DW ? vld(&s_ring[qhead % RING][lane]) : 0u;
                  CTR(C_FAST, k - 1);
                  CTR(C_CAND, (uint64_t)(k - 1) * (M - f < 64 ? M - f : 64));
                  CTR(C_FA, k - 1);
                  CTR(C_ALG, (uint64_t)(k - 1) * (f + 1));
                  CTR(C_NPRE, (uint64_t)(k - 1) * d.NN);
                  CTR(C_RPODS, k - 1);
                  CTR(C_RBATCH, 1);
                  CTR(C_RBPODS, k - 1);
#ifdef GS_RUN_TL
                  CTR(C_RBT1, __builtin_amdgcn_s_memtime() - tb1);
#endif
                }
              }
            }
#ifdef GS_RUN_TL
            CTR(C_RBT0, __builtin_amdgcn_s_memtime() - tb0);
#endif
          }
#endif
        }
        if (dirty) {
          // the window back to LDS: positions, and the codes of its claims
          wsyncT<CH>();
          if (valid) {
            s_so[wpos] = ow;
            s_slk[ow >> 16] = wsl;
            s_rm[ow >> 16] = wrm;
          }
          wsyncT<CH>();
        }
#ifdef GS_RUN_TL
        run_cyc += __builtin_amdgcn_s_memtime() - rt0;
#endif
        continue;
      }
    }
    uint32_t vrd, rqd, p, v;
    uint64_t rqq_p = 0, rqc_p = 0;  // request codes (floor / ceil) of resources 0..3, 16 bits each
    const bool from_ring = !wrapped;
    if (from_ring) {
      // first pass: the pod at qhead is queue0[qhead] with its first
      // variant and was never pushed (no staleness stop); the agent staged
      // its record in ring slot qhead % RING.  The sequence word and the
      // record are read in one round trip: the LDS serves a wave's reads in
      // order and the agent wrote the record before the sequence word.
      const uint32_t rs = qhead % RING;
      uint32_t x = pf_x;  // read during the previous pop
      if (__builtin_amdgcn_readfirstlane(pf_seq) != qhead + 1) {
        for (uint32_t spin = 0;; spin++) {
          const uint32_t sq = vld(&s_ring_seq[rs]);
          x = lane < RING_DW ? vld(&s_ring[rs][lane]) : 0u;
          if (__builtin_amdgcn_readfirstlane(sq) == qhead + 1) break;
          __builtin_amdgcn_s_sleep(0);
          if (spin > SPIN_MAX) {
            chan_err = true;
            break;
          }
        }
      }
      if (chan_err) {
        status = 2;
        break;
      }
      wsyncT<CH>();
      if (lane == 0) vst(&s_ctl[0], qhead + 1);  // the slot may be refilled
      vrd = x;
      rqd = x;
      p = rlane(vrd, 0);
      v = rlane(vrd, VR_DW - 1);
      rqq_p = (uint64_t)rlane(x, RING_CODES) | ((uint64_t)rlane(x, RING_CODES + 1) << 32);
      rqc_p = (uint64_t)rlane(x, RING_CODES + 2) | ((uint64_t)rlane(x, RING_CODES + 3) << 32);
    } else {
      p = __builtin_amdgcn_readfirstlane(d.queue[qhead]);
      const uint32_t le = __builtin_amdgcn_readfirstlane(d.last_epoch[p]);
      const uint32_t ll = __builtin_amdgcn_readfirstlane(d.last_len[p]);
      v = __builtin_amdgcn_readfirstlane(d.cur_var[p]);
      if (le == epoch && ll == qlen) break;
      vrd = lane < VR_DW ? ((const uint32_t*)(d.vars + v))[lane] : 0u;
      rqd = lane >= 32 && lane < 32 + 2 * R ? ((const uint32_t*)(d.pod_req + (size_t)p * R))[lane - 32] : 0u;
    }
    if (qhead + 1 == P) wrapped = true;
    qhead = qhead + 1 == P ? 0 : qhead + 1;
    qlen--;
    pops++;
    if ((pops & 15) == 0 && lane == 0) vst(&s_ctl[3], (uint32_t)pops);  // heartbeat for the agent's bounded wait
    if (!wrapped) {
      // the next first-pass record, read now: its round trip overlaps this
      // pod (a slot the agent has not filled yet is re-read at the pop)
      pf_seq = vld(&s_ring_seq[qhead % RING]);
      pf_x = lane < RING_DW ? vld(&s_ring[qhead % RING][lane]) : 0u;
    }
    const uint32_t gp = p;
    auto VD = [&](uint32_t i) -> uint32_t { return rlane(vrd, i); };
    auto VD64 = [&](uint32_t i) -> uint64_t { return (uint64_t)VD(i) | ((uint64_t)VD(i + 1) << 32); };
    const uint32_t vctb = VD(3);
    const uint64_t vtolt = VD64(20);
    // topology: own list (groups the variant owns), selection list (groups counting the pod)
    const uint32_t own_off = TOPO ? VD(22) : 0u, own_n = TOPO ? VD(23) : 0u;
    const uint32_t sel_off = TOPO ? VD(24) : 0u, sel_n = TOPO ? VD(25) : 0u;
    // the owned groups staged in lanes 0..own_n-1 now (own_n <= OWNMAX = 64):
    // the topology checks of the node scan, the exact batch and the fresh
    // NodeClaim read them by readlane instead of two dependent HBM loads each
    uint32_t og_e = 0, og_skew = 0, og_slot = 0, og_kind = 0;
    if (TOPO && own_n) {
      const auto& KD = *karg();
      if (lane < own_n) {
        og_e = KD.tg_list[own_off + lane];
        const TGroupRec& tg = KD.tgroups[og_e & TL_GID];
        og_skew = (uint32_t)tg.skew;
        og_slot = tg.slot;
        og_kind = tg.kind;
      }
    }
    auto OWN = [&](uint32_t k) -> OwnG {
      return OwnG{rlane(og_e, k), (int32_t)rlane(og_skew, k), rlane(og_slot, k), rlane(og_kind, k)};
    };
    // the requests stay in the record's lanes 32.. (rqd): every use site
    // reads them with its own readlanes (RQ), so no 64-bit request is held
    // in scalar registers across the pod (they spilled into VGPR lanes)
// (GS_RQ_AT copies the record: use it in uniform control flow only)
#define GS_RQ_AT(name)                                                                                \
  const uint32_t name##_x = fresh(rqd);                                                               \
  auto name = [&](uint32_t r) -> int64_t {                                                            \
    return (int64_t)((uint64_t)rlane(name##_x, 32 + 2 * r) | ((uint64_t)rlane(name##_x, 33 + 2 * r) << 32)); \
  }
    // lane r < R: resource r's request (lanes 2r + 32, 2r + 33 of the record)
    int64_t rq_lane = 0;
    {
      const uint32_t lo = (uint32_t)__shfl((int)rqd, (int)(32 + 2 * (lane & 7))),
                     hi = (uint32_t)__shfl((int)rqd, (int)(33 + 2 * (lane & 7)));
      if (lane < RR) rq_lane = (int64_t)(((uint64_t)hi << 32) | lo);
    }
    // resources 4.. requested at all (the LDS codes cover resources 0..3)
    const bool rq_hi = RR > 4 && __ballot(lane >= 4 && lane < RR && rq_lane != 0) != 0;
    if (!from_ring) {
      // a wrapped pop read its record itself: the request codes too
      GS_RQ_AT(RQ);
#pragma unroll
      for (uint32_t r = 0; r < 4; r++)
        if (r < d.RQ && r < RR) {
          rqq_p |= (uint64_t)qcode_floor(RQ(r)) << (16 * r);
          rqc_p |= (uint64_t)qcode_ceil(RQ(r)) << (16 * r);
        }
    }

    TLW(0);  // pop + record
    // <U> Topology.AddRequirements: each owned zone group's minimum domain
    // count over the pod's strict zone domains (domainMinCount); only a pod
    // owning a zone spread group reads them
    if (TOPO && own_n && (vctb & VF_ZSPREAD)) {
      const auto& KD = *karg();
      const uint64_t vzs = rlane(vrd, 26) | ((uint64_t)rlane(vrd, 27) << 32);
      topo_tmin(KD, ts, own_off, own_n, vzs, lane);
      wsyncT<CH>();
    }

    // ----------------- existing nodes in order: first ExistingNode.CanAdd wins
    if (d.NN) {
      const auto& KD = *karg();
      const uint32_t vx = fresh(vrd);
      auto VX = [&](uint32_t i) -> uint32_t { return rlane(vx, i); };
      auto VX64 = [&](uint32_t i) -> uint64_t { return (uint64_t)VX(i) | ((uint64_t)VX(i + 1) << 32); };
      const uint32_t fk_begin = VX(1), fk_count = VX(2), zfull_off = VX(12), cfull_off = VX(13);
      const uint64_t vtol = VX64(18);
      // <U> VolumeUsage: the pod's pending-volume bits per CSI driver
      uint64_t pvol[VDMAX] = {0, 0, 0, 0};
      uint32_t pfresh[VDMAX] = {0, 0, 0, 0};
      if (TOPO && KD.any_vol)
#pragma unroll
        for (uint32_t q = 0; q < VDMAX; q++) {
          pvol[q] = KD.pod_vol[(size_t)gp * VDMAX + q];
          pfresh[q] = KD.pod_vfresh[(size_t)gp * VDMAX + q];
        }
      // LDS prefilter (per resource 0..3: request code <= slack code) and,
      // for a plain pod (no requirements, topology or volumes) on a plain
      // node, the sufficient test (request code <= room code: CanAdd holds
      // without reading the node); the exact ExistingNode.CanAdd runs on the
      // prefilter's survivors before the chunk's first fast accept
      bool pvany = false;
#pragma unroll
      for (uint32_t q = 0; q < VDMAX; q++) pvany = pvany || pvol[q] || pfresh[q];
      bool nplain = (vctb & VF_SIMPLE) && !pvany;
      nplain = nplain && !rq_hi;
      const uint64_t nrqq = rqq_p, nrqc = rqc_p;
      uint32_t nlo = 0;
      if (nhint_ok && (vtol & ~nhint_tol) == 0) {
        const bool ge = lane >= R || rq_lane >= hint_nrq;
        if (__ballot(!ge) == 0) nlo = nhint;
      }
      uint32_t fn = INF;
      bool nfa_win = false;
      GS_RQ_AT(RQ);  // in uniform control flow: the copy must hold every lane
      for (uint32_t base = nlo & ~63u; base < KD.NN; base += 64) {
        const uint32_t n = base + lane;
        const bool in = (n < KD.NN) & (n >= nlo);
        const uint32_t nc = in ? n : 0u;
        const uint64_t nsl = s_nslk[nc], nrm = s_nrm[nc];
        const uint32_t nfl = s_nflag[nc];
        const bool lp = in & swar_ge(nsl, nrqq);
        const bool fa = lp & nplain & (bool)(nfl & 1u) & swar_ge(nrm, nrqc);
        const uint64_t lpb = __ballot(lp);
        CTR(C_NEV, KD.NN - base < 64 ? KD.NN - base : 64);
        if (!lpb) continue;
        const uint64_t fab = __ballot(fa);
        const uint32_t mfl = fab ? ffs64(fab) : 64u;
        const bool need = lp & !fa & (lane < mfl);
        bool feas = fa;
        if (__ballot(need)) {
          if (GS_AGENT_WRITES) drain();  // node requests the agent still adds (fast accepts)
          if (need) {
            const NodeRec& nr = KD.nodes[n];
            const FK* nfk = KD.n_fk + (size_t)n * F;
            feas = nr.ok && (nr.taints & ~vtol) == 0;  // Taints.ToleratesPod
#pragma unroll
            for (uint32_t r = 0; r < RR; r++) feas = feas && nr.req[r] + RQ(r) <= nr.avail[r];  // Fits
#pragma unroll
            for (uint32_t k = 0; k < KMAX_IT; k++) {
              const uint32_t off = VX(4 + k);
              if (k >= KD.K || !feas || off == NONE) continue;
              const uint32_t vid = nr.vid[k];
              feas = vid != NONE && ((KD.itmask[off + (vid >> 6)] >> (vid & 63)) & 1);
            }
            if (feas && zfull_off != NONE)
              feas = nr.zvid != NONE && ((KD.itmask[zfull_off + (nr.zvid >> 6)] >> (nr.zvid & 63)) & 1);
            if (feas && cfull_off != NONE)
              feas = nr.cvid != NONE && ((KD.itmask[cfull_off + (nr.cvid >> 6)] >> (nr.cvid & 63)) & 1);
            if (feas && fk_count) feas = fk_ok_range(d, fk_begin, fk_count, nfk, true);
            if (TOPO && feas && own_n)
              feas = topo_node_ok_g(KD, ts, own_n, nr.dvid,
                                    [&](uint32_t hs) -> int64_t { return KD.hn[(size_t)hs * KD.NN + n]; }, OWN);
            if (TOPO && feas && KD.any_vol) {
              // ExceedsLimits: distinct volumes per driver after the union
              const NodeVol& nv = KD.n_vol[n];
#pragma unroll
              for (uint32_t q = 0; q < VDMAX; q++)
                if (pvol[q] | pfresh[q]) feas = feas && nv.cnt[q] + (int32_t)pfresh[q] + __popcll(pvol[q] & ~nv.present) <= nv.lim[q];
            }
          }
        }
        const uint64_t b = __ballot(feas);
        if (b) {
          fn = base + ffs64(b);
          nfa_win = ((fab >> ffs64(b)) & 1) != 0;
          break;
        }
      }
      CTR(C_NPRE, fn != INF ? fn + 1 : KD.NN);
      if (nplain) {
        // [nlo, fn) (or all) cannot take these requests; nodes only fill up
        nhint = fn != INF ? fn : KD.NN;
        nhint_ok = true;
        nhint_tol = vtol;
        hint_nrq = rq_lane;
      }
      if (fn != INF && nfa_win) {
        // ExistingNode.Add of a plain pod: requests only.  The LDS codes
        // shrink by the request (still an upper / lower bound); the agent adds
        // the requests to the node (an exact check drains the channel first)
        const uint64_t sl = s_nslk[fn], rm = s_nrm[fn];
        uint32_t c_sl = 0, c_rm = 0;
        if (lane < KD.RQ) {
          const uint32_t sh = 16 * lane;
          c_sl = qcode_ceil(qcode_value((uint32_t)(sl >> sh) & 0xFFFFu) - rq_lane);
          c_rm = qcode_floor(qcode_value((uint32_t)(rm >> sh) & 0xFFFFu) - rq_lane);
        }
        uint64_t sl2 = 0, rm2 = 0;
#pragma unroll
        for (uint32_t r = 0; r < 4; r++)
          if (r < KD.RQ) {
            sl2 |= (uint64_t)rlane(c_sl, r) << (16 * r);
            rm2 |= (uint64_t)rlane(c_rm, r) << (16 * r);
          }
        if (lane == 0) {
          s_nslk[fn] = sl2;
          s_nrm[fn] = rm2;
          // <U> Topology.Record in the groups that select the pod
          if (TOPO && sel_n) {
            const uint32_t z = KD.nodes0[fn].dvid;
            topo_record(KD, ts, sel_off, sel_n, z < 64u ? 1ull << z : 0ull, 0u,
                        [&](uint32_t hs) { KD.hn[(size_t)hs * KD.NN + fn]++; });
          }
        }
        wsyncT<CH>();
        emit(WQ_NFA, nlog, gp, v, fn, rqd, rq_lane);
        nlog++;
        CAT(6);
        continue;
      }
      if (fn != INF) {
        // ExistingNode.Add: requests and requirements
        int64_t* areq = KD.nodes[fn].req;
        FK* afk = KD.n_fk + (size_t)fn * F;
        int64_t nreq = 0, navl = 0;
        if (lane < R) {
          nreq = areq[lane] + rq_lane;
          navl = KD.nodes[fn].avail[lane];
          areq[lane] = nreq;
        }
        if (lane < fk_count) {
          const FKEntry& e = KD.fk_entries[fk_begin + lane];
          FK* nf = afk + e.slot;
          const FK cur = *nf;
          *nf = (cur.flags & FK_PRESENT) ? fk_intersect(cur, e.st, KD.fk_ival + (size_t)e.slot * FKV, KD.fk_isint + (size_t)e.slot * FKW)
                                         : e.st;
        }
        {
          // the node's LDS codes from its exact remainder
          const int64_t sl = navl - nreq;
          const uint32_t c_sl = lane < KD.RQ ? qcode_ceil(sl) : 0u, c_rm = lane < KD.RQ ? qcode_floor(sl) : 0u;
          const bool over = lane >= 4 && lane < R && sl < 0;
          uint64_t sl2 = 0, rm2 = 0;
#pragma unroll
          for (uint32_t r = 0; r < 4; r++) {
            sl2 |= (uint64_t)rlane(c_sl, r) << (16 * r);
            rm2 |= (uint64_t)rlane(c_rm, r) << (16 * r);
          }
          const bool anyover = __ballot(over) != 0;
          if (lane == 0) {
            s_nslk[fn] = sl2;
            s_nrm[fn] = rm2;
            if (anyover) s_nflag[fn] = 0;
          }
        }
        if (lane == 0) {
          if (TOPO && KD.any_vol) {
            // VolumeUsage.Add
            NodeVol& nv = KD.n_vol[fn];
            uint64_t all = 0;
#pragma unroll
            for (uint32_t q = 0; q < VDMAX; q++) {
              nv.cnt[q] += (int32_t)pfresh[q] + __popcll(pvol[q] & ~nv.present);
              all |= pvol[q];
            }
            nv.present |= all;
          }
          // <U> Topology.Record: the node's labels are single domains
          if (TOPO && sel_n) {
            const uint32_t z = KD.nodes0[fn].dvid;
            topo_record(KD, ts, sel_off, sel_n, z < 64u ? 1ull << z : 0ull, 0u,
                        [&](uint32_t hs) { KD.hn[(size_t)hs * KD.NN + fn]++; });
          }
        }
        wsyncT<CH>();
        emit(WQ_LOG, nlog, gp, v, fn | 0x80000000u, 0, 0);
        nlog++;
        CAT(6);
        continue;
      }
    }

    TLW(1);  // topology minimum + existing nodes
    // ------------------------------- sort.Slice(newNodeClaims, len(Pods) asc)
    uint32_t win_base = INF, win_v = 0;  // positions [win_base, +64) after the rotation (the scan may start there)
    if (M >= 50 && modkind == MOD_INC && !pivot_touched(modkind, modpos, M)) {
      // the common case in one LDS round trip: read the 64 positions from
      // modpos, find the end e of the raised key's run inside them, and
      // rotate [modpos, e) left there (whole-wave DPP shift); a run that
      // leaves the window takes the general path below
      const uint32_t k = modpos + lane;
      const uint32_t w = k < M ? (uint32_t)acc.so[k] : 0xFFFFu;
      const uint32_t w0 = rlane(w, 0), x = w0 & 0xFFFFu;
      const uint64_t b = __ballot(lane >= 1 && (w & 0xFFFFu) >= x);
      if (b) {
        const uint32_t eo = ffs64(b);  // e = modpos + eo
        if (eo > 1) {
          CTR(C_FAST, 1);
          const uint32_t sh = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x130, 0xF, 0xF, false);  // lane i <- i + 1
          const uint32_t nw = lane + 1 == eo ? w0 : sh;
          wsyncT<CH>();
          if (lane < eo) acc.so[k] = nw;
          wsyncT<CH>();
          win_v = lane < eo ? nw : w;
#ifdef GS_FFD_TL
          n_rot++;
          n_rotlen += eo - 1;
#endif
          // (modpos, e-1] shift left, the changed claim lands at e-1
          if (modpos < hint && modpos + eo - 1 >= hint) hint--;
        } else {
          win_v = w;
        }
        win_base = modpos;
        modkind = MOD_NONE;
      }
    }
    if (M > 1 && modkind != MOD_NONE) {
      // at most one NodeClaim changed since the last sort: one pod added at
      // modpos (INC) or one NodeClaim appended (APPEND)
      bool inversion = false;
      if (modkind == MOD_INC) inversion = modpos + 1 < M && acc.key(modpos + 1) < acc.key(modpos);
      else if (modkind == MOD_APPEND) inversion = acc.key(M - 2) > acc.key(M - 1);
      inversion = __builtin_amdgcn_readfirstlane(inversion ? 1u : 0u) != 0;
      if (inversion) {
        if (M <= 12) {
          if (GS_REG_SORT) {
            reg_pdq_frame(PackedArr<U32, CH>{(U32*)s_so}, 0, (int)M, bits_len((uint64_t)M), 1, 1);  // insertionSort
          } else {
            if (lane == 0) SeqSortT<PackedAccT<U32>>{{(U32*)s_so}}.insertion_sort(0, (int)M);
            wsyncT<CH>();
          }
          hint_ok = false;
        } else if (M >= 50 && (!pivot_touched(modkind, modpos, M) || pivot_hint_wave(acc, (int)M, lane) == 1)) {
          // partialInsertionSort fixes the single inversion: one rotation
          CTR(C_FAST, 1);
          if (modkind == MOD_INC) {
            const uint32_t x = acc.key(modpos);
            const uint32_t e = wave_first(modpos + 1, M, lane, [&](uint32_t k) { return acc.key(k) >= x; });
            ws.rotate((int)modpos, (int)e - 1, true);
#ifdef GS_FFD_TL
            n_rot++;
            n_rotlen += e - 1 - modpos;
#endif
            // (modpos, e-1] shift left, the changed claim lands at e-1
            if (modpos < hint && e - 1 >= hint) hint--;
          } else {
            const uint32_t x = acc.key(M - 1);
            const uint32_t lo = wave_first(0, M - 1, lane, [&](uint32_t k) { return acc.key(k) > x; });
            ws.rotate((int)lo, (int)M - 1, false);
#ifdef GS_FFD_TL
            n_rot++;
            n_rotlen += M - 1 - lo;
#endif
            if (lo < hint) hint = lo;  // the new claim lands at lo
          }
        } else {
          CTR(C_GEN, 1);
          // the one position the last Add moved out of order
          const int known_x = modkind == MOD_INC ? (int)modpos : (int)M - 1;
#ifdef GS_FFD_TL
          const uint64_t g0_ = __builtin_amdgcn_s_memtime();
#endif
#ifdef GS_SORT_TL
          wave_pdqsort<GS_WAVE_SEQ, U32, U16, CH, KNOWN_PART>(ws.so, ws.scr, ws.stk, ws.lane, ws.half, (int)M, known_x, s_stl);
#else
          wave_pdqsort<GS_WAVE_SEQ, U32, U16, CH, KNOWN_PART>(ws.so, ws.scr, ws.stk, ws.lane, ws.half, (int)M, known_x);
#endif
#ifdef GS_FFD_TL
          n_gen_cyc += __builtin_amdgcn_s_memtime() - g0_;
#endif
          hint_ok = false;
        }
      }
      modkind = MOD_NONE;
    }

    TLW(2);  // sort
    // rqq_p / rqc_p: the request codes for the LDS slack / room tests, packed
    // 16 bits per resource (codes < 2^15, so a SWAR subtract compares all four
    // at once)
#ifdef GS_NO_FAST
    bool simple = false;
#else
    // a pod with no requirements and no owned topology group (VF_SIMPLE):
    // its CanAdd is resources and taints only, in either variant
    bool simple = (vctb & VF_SIMPLE) != 0;
#endif
    simple = simple && !rq_hi;  // room covers resources 0..3
    // hostname-only topology (VF_HOSTFA): the scan reads each candidate's
    // counts of the owned groups; a candidate over a skew is infeasible
    // (dropped), one within them that passes the room test is a fast accept
#ifndef GS_HOSTFA
#define GS_HOSTFA 1
#endif
    const bool hostfa = GS_HOSTFA && TOPO && !rq_hi && (vctb & VF_HOSTFA) != 0;
#ifdef GS_FFD_TL
    n_nonsimple += simple ? 0u : 1u;
#endif

    // --------------------------- in-flight NodeClaims, first that CanAdd wins
    // Phase A walks the sorted positions in LDS, one 64-position chunk per
    // step (2 or 4 chunks per step measured slower:
    // profiles/r2/ffd_scan_width_ab.txt), with the necessary test (template
    // tolerated, request code <= slack code per resource) and, for simple
    // pods, the sufficient test
    // (request code <= room code: CanAdd holds without reading the claim).
    // It stops at the first fast accept, collecting every candidate before it
    // that needs the exact check (at most 64 per batch).  Phase B runs the
    // exact NodeClaim.CanAdd on the batch, one lane per candidate: the first
    // feasible candidate wins, else the fast accept, else the scan resumes.
    uint32_t f = INF;
    bool ovf = false;  // the winner lane's u16 pod count overflowed
    uint32_t lo_bound = 0;
    if (hint_ok && (vtolt & ~hint_tolt) == 0) {
      const bool ge = lane >= 4 || lane >= R || rq_lane >= hint_rq;
      if (__ballot(!ge) == 0) lo_bound = hint;
    }
    uint32_t scan_from = lo_bound;  // chunks start at the bound (no dead lanes below it)
    for (;;) {
      uint32_t nex = 0, fa_pos = INF, fa_j = 0, resume = INF;
      // the fast accept's chunk, kept in lanes: its order words, slack and
      // room codes (the Add reads the winner's lane, no LDS round trip)
      uint32_t fa_ev = 0, fa_l = 0;  // fa_l: the fast accept's lane (chunks start at the bound, unaligned)
      uint64_t fa_sq = 0, fa_rv = 0;
      // the next chunk's order words are read with this chunk's codes, one
      // LDS round trip less per further chunk (C5 1,266 -> 1,241 ms, CM 325 ->
      // 322); the general narrow variant measured no better (e2e, C3) and
      // keeps the plain loop; gathering the next chunk's codes too measured
      // slower (C5 1,245 -> 1,270; profiles/r4/scan_prefetch_ab.txt)
#ifndef GS_SCAN_PF
#define GS_SCAN_PF 1
#endif
      constexpr bool SPF = GS_SCAN_PF && (WIDE || !TOPO);
      uint32_t ev_next = 0;
      bool have_next = false;
      for (uint32_t cb = scan_from; cb < M; cb += 64) {
        const uint32_t pos = cb + lane;
        // the sort's window is this chunk when the scan starts where the last
        // Add landed (runs of equal pods): no LDS read of the order words
        const uint32_t ev = cb == win_base ? win_v : (SPF && have_next) ? ev_next : s_so[pos < M ? pos : M - 1], je = ev >> 16;
        if (SPF) {
          const uint32_t pn = pos + 64u;
          ev_next = s_so[pn < M ? pn : M - 1];
          have_next = true;
        }
        const uint64_t sq = s_slk[je], rmv = s_rm[je];
        const uint32_t tt = T > 1 ? (uint32_t)s_tmpl[je] : 0u;
        // bitwise (not short-circuit) predicates: no branches
        bool lp = (pos >= lo_bound) & (pos < M) & (bool)((vtolt >> tt) & 1) & swar_ge(sq, rqq_p);
        if (TOPO && hostfa && lp) {
          const auto& KD = *karg();
          const int32_t* hrow = KD.hc + (size_t)je * KD.TGH;
#ifdef GS_HOSTFA_UNROLL
#pragma unroll
          for (uint32_t k = 0; k < 4; k++) {
            if (k < own_n) {
              const int64_t c = hrow[rlane(og_slot, k)] + ((rlane(og_e, k) & TL_SELF) ? 1 : 0);
              lp = lp && c <= (int64_t)(int32_t)rlane(og_skew, k);
            }
          }
#else
          for (uint32_t k = 0; k < own_n; k++) {
            const int64_t c = hrow[rlane(og_slot, k)] + ((rlane(og_e, k) & TL_SELF) ? 1 : 0);
            lp = lp && c <= (int64_t)(int32_t)rlane(og_skew, k);
          }
#endif
        }
        const bool fa = lp & (simple | hostfa) & swar_ge(rmv, rqc_p);
        const uint64_t fab = __ballot(fa), exb = __ballot(lp & !fa);
        const uint32_t mfl = fab ? ffs64(fab) : 64u;
        const uint64_t ex = exb & (mfl == 64 ? ~0ull : ((1ull << mfl) - 1ull));
        const uint32_t cnt = (uint32_t)__popcll(ex);
        if (nex + cnt > 64) {
          resume = cb;  // batch full: check it, then rescan from this chunk
          break;
        }
        CTR(C_CAND, M - cb < 64 ? M - cb : 64);
        if (ex) {
          if ((ex >> lane) & 1) s_exl[nex + (uint32_t)__popcll(ex & ((1ull << lane) - 1ull))] = (pos & 0xFFFFu) | (je << 16);
          nex += cnt;
        }
        if (fab) {
          fa_pos = cb + mfl;
          fa_j = rlane(je, mfl);
          fa_ev = ev;
          fa_l = mfl;
          fa_sq = sq;
          fa_rv = rmv;
          break;
        }
      }
      wsyncT<CH>();
      TLW(5);  // phase A: LDS prefilter
      if (nex) {
        if (GS_AGENT_WRITES) drain();  // the agent's request totals must be in the claim records
        const auto& KD = *karg();
        const uint32_t vx = fresh(vrd);
        auto VX = [&](uint32_t i) -> uint32_t { return rlane(vx, i); };
        auto VX64 = [&](uint32_t i) -> uint64_t { return (uint64_t)VX(i) | ((uint64_t)VX(i + 1) << 32); };
        const uint32_t fk_begin = VX(1), fk_count = VX(2), vzflags = VX(30);
        const uint64_t vzm = VX64(14), vcm = VX64(16), vzn = VX64(28);
        // --- exact NodeClaim.CanAdd, lane i = i-th candidate (ascending
        // positions): one 64-B header read, option words and the (variant,
        // template) row, threshold cursors, offering grid
        CTR(C_FULL, nex);
#ifdef GS_FFD_TL
        n_xns += simple ? 0u : nex;
        n_xb++;
#endif
        // wide option rows (W > WREG words): a small batch spreads each
        // candidate over L lanes, each testing every L-th 4-word chunk, so a
        // candidate takes W / 4L dependent round trips instead of W / 4
#ifdef GS_NO_EXACT_LANES  // experiment builds: one lane per candidate at every width
        const uint32_t lgL = 0u;
#else
        const uint32_t lgL = !WIDE ? 0u : nex <= 8 ? 3u : nex <= 16 ? 2u : nex <= 32 ? 1u : 0u;
#endif
        const uint32_t lgW = W <= 4 ? 0u : W <= 8 ? 1u : W <= 16 ? 2u : 3u;  // no more lanes than 4-word chunks
        const uint32_t lg = lgL < lgW ? lgL : lgW;
        const uint32_t cx = lane >> lg, sub = lane & ((1u << lg) - 1u);
        const uint32_t xe = cx < nex ? s_exl[cx] : 0u;
        const uint32_t j = xe >> 16, xpos = xe & 0xFFFFu;
        const uint32_t t = cx < nex ? (uint32_t)s_tmpl[j] : 0u;
        GS_RQ_AT(RQ);
      bool feas = false;
      uint64_t zset = ~0ull;  // zone domains topology allows on this NodeClaim (~0: unconstrained)
      uint64_t zm = 0, cm = 0, czf = 0;
      uint32_t czfl = 0;
      uint32_t mrow[RR];
      int64_t tot[RR];
      // GS_MAXA_PF: each candidate lane also loads its claim's maxa (the
      // slack bound the Add re-quantizes with) with the header, so the
      // winner's Add does not wait on a load of its own
#ifndef GS_MAXA_PF
#define GS_MAXA_PF 1
#endif
      int64_t maxa_pre[RR];
#pragma unroll
      for (uint32_t r = 0; r < RR; r++) maxa_pre[r] = 0;
      uint64_t nx[WREG] = {0, 0, 0, 0};
      uint64_t G = 0, Gt = 0;
      if (cx < nex) {
        const ClaimRec* cr = KD.c_rec + j;
        uint32_t cur[RR];
        if (GS_MAXA_PF) {
#pragma unroll
          for (uint32_t r = 0; r < RR; r++) maxa_pre[r] = cr->maxa[r];
        }
        {
          const uint4* q = (const uint4*)cr;
          const uint4 h0 = q[0], h1 = q[1], h2 = q[2], h3 = q[3];
          const int64_t lo[4] = {(int64_t)(((uint64_t)h0.y << 32) | h0.x), (int64_t)(((uint64_t)h0.w << 32) | h0.z),
                                 (int64_t)(((uint64_t)h1.y << 32) | h1.x), (int64_t)(((uint64_t)h1.w << 32) | h1.z)};
          const uint32_t cl[4] = {h2.x & 0xFFFFu, h2.x >> 16, h2.y & 0xFFFFu, h2.y >> 16};
          zm = ((uint64_t)h2.w << 32) | h2.z;
          cm = ((uint64_t)h3.y << 32) | h3.x;
#pragma unroll
          for (uint32_t r = 0; r < RR; r++) {
            tot[r] = r < 4 ? lo[r] : cr->tot_hi[r - 4];
            cur[r] = r < 4 ? cl[r] : cr->thr_hi[r - 4];
          }
        }
        const uint64_t* row = KD.rows + ((size_t)v * T + t) * OW;
        const uint64_t* opts = KD.c_opts + (size_t)j * OW;
        if (!WIDE) {
          const uint4* oq = (const uint4*)opts;
          const uint4* rq4 = (const uint4*)row;
          const uint4 o0 = oq[0], o1 = oq[1], r0 = rq4[0], r1 = rq4[1];
          const uint64_t a[4] = {(((uint64_t)o0.y << 32) | o0.x) & (((uint64_t)r0.y << 32) | r0.x),
                                 (((uint64_t)o0.w << 32) | o0.z) & (((uint64_t)r0.w << 32) | r0.z),
                                 (((uint64_t)o1.y << 32) | o1.x) & (((uint64_t)r1.y << 32) | r1.x),
                                 (((uint64_t)o1.w << 32) | o1.z) & (((uint64_t)r1.w << 32) | r1.z)};
#pragma unroll
          for (uint32_t w = 0; w < WREG; w++) nx[w] = w < W ? a[w] : 0;
        }
        bool pre = true;
        if (fk_count) pre = fk_ok_range(d, fk_begin, fk_count, KD.c_fk + (size_t)j * F, false);
        if (TOPO && pre && own_n) {
          // <U> Topology.AddRequirements on the NodeClaim over its (claim AND
          // pod) zone domains; hostname groups: this NodeClaim's counts
          czf = cr->zfull;
          czfl = cr->zflags;
          const int32_t* hrow = KD.hc + (size_t)j * KD.TGH;
          zset = topo_claim_g(KD, ts, own_n, czf & vzn, [&](uint32_t hs) -> int64_t { return hrow[hs]; }, OWN);
          pre = zset != 0;
          if (pre && zset != ~0ull) {
            // the domains narrow the catalog zones, or (dom_ct) capacity types
            const uint64_t dcat = topo_catmask(KD, zset);
            if (KD.dom_ct) cm &= dcat;
            else if (!KD.dom_np) zm &= dcat;
          }
        }
        if (pre) {
          G = grid_of(zm & vzm, cm & vcm, KD.Z, KD.C);
          Gt = grid_of(s_tzm[t] & vzm, s_tcm[t] & vcm, KD.Z, KD.C);
          uint32_t mm[RR];
#pragma unroll
          for (uint32_t r = 0; r < RR; r++) {
            const uint32_t o = s_thoff[r], n = s_thoff[r + 1] - o;
            mm[r] = thr_window(thr + o, n, cur[r], tot[r] + RQ(r));
          }
#pragma unroll
          for (uint32_t r = 0; r < RR; r++) {
            const uint32_t o = s_thoff[r], n = s_thoff[r + 1] - o;
            if (mm[r] == cur[r] + 4 && mm[r] < n) mm[r] = thr_search(thr + o, n, mm[r], tot[r] + RQ(r));
            mrow[r] = o + r + mm[r];
          }
          uint64_t accw = 0;
          if (!WIDE) {
            // opts ⊆ thr_set[cur] (invariant of every Add): only a resource
            // whose cursor moves narrows the options further
#pragma unroll
            for (uint32_t r = 0; r < RR; r++) {
              if (mm[r] != cur[r]) {
                const uint4* tq = (const uint4*)(KD.thr_set + (size_t)mrow[r] * OW);
                const uint4 t0 = tq[0], t1 = tq[1];
                nx[0] &= ((uint64_t)t0.y << 32) | t0.x;
                nx[1] &= ((uint64_t)t0.w << 32) | t0.z;
                nx[2] &= ((uint64_t)t1.y << 32) | t1.x;
                nx[3] &= ((uint64_t)t1.w << 32) | t1.z;
              }
            }
            if (G != Gt) {
              uint64_t off[WREG] = {};
              for (uint64_t gm = G; gm; gm &= gm - 1) {
                const uint32_t g = ffs64(gm);
#pragma unroll
                for (uint32_t w = 0; w < WREG; w++)
                  if (w < W) off[w] |= slot[g * W + w];
              }
#pragma unroll
              for (uint32_t w = 0; w < WREG; w++) nx[w] &= off[w];
            }
#pragma unroll
            for (uint32_t w = 0; w < WREG; w++) accw |= nx[w];
          } else {
            // GS_XC chunks of 4 words per round trip (the loads of all of them
            // issued before any is used), stop at the first batch with a survivor
#ifndef GS_XC
#define GS_XC 2
#endif
            for (uint32_t w0 = sub * 4; w0 < W && !accw; w0 += (4u * GS_XC) << lg) {
              uint4 o[GS_XC][2], rw[GS_XC][2], tt[GS_XC][RR][2];
#pragma unroll
              for (uint32_t c = 0; c < GS_XC; c++) {
                const uint32_t wc = w0 + (c * 4u << lg);
                if (wc < W) {
                  const uint4* oq = (const uint4*)(opts + wc);
                  const uint4* rq4 = (const uint4*)(row + wc);
                  o[c][0] = oq[0];
                  o[c][1] = oq[1];
                  rw[c][0] = rq4[0];
                  rw[c][1] = rq4[1];
#pragma unroll
                  for (uint32_t r = 0; r < RR; r++) {
                    if (mm[r] == cur[r]) continue;
                    const uint4* tq = (const uint4*)(KD.thr_set + (size_t)mrow[r] * OW + wc);
                    tt[c][r][0] = tq[0];
                    tt[c][r][1] = tq[1];
                  }
                }
              }
#pragma unroll
              for (uint32_t c = 0; c < GS_XC; c++) {
                const uint32_t wc = w0 + (c * 4u << lg);
                if (wc >= W) continue;
                uint64_t x[4] = {(((uint64_t)o[c][0].y << 32) | o[c][0].x) & (((uint64_t)rw[c][0].y << 32) | rw[c][0].x),
                                 (((uint64_t)o[c][0].w << 32) | o[c][0].z) & (((uint64_t)rw[c][0].w << 32) | rw[c][0].z),
                                 (((uint64_t)o[c][1].y << 32) | o[c][1].x) & (((uint64_t)rw[c][1].y << 32) | rw[c][1].x),
                                 (((uint64_t)o[c][1].w << 32) | o[c][1].z) & (((uint64_t)rw[c][1].w << 32) | rw[c][1].z)};
#pragma unroll
                for (uint32_t r = 0; r < RR; r++) {
                  if (mm[r] == cur[r]) continue;
                  x[0] &= ((uint64_t)tt[c][r][0].y << 32) | tt[c][r][0].x;
                  x[1] &= ((uint64_t)tt[c][r][0].w << 32) | tt[c][r][0].z;
                  x[2] &= ((uint64_t)tt[c][r][1].y << 32) | tt[c][r][1].x;
                  x[3] &= ((uint64_t)tt[c][r][1].w << 32) | tt[c][r][1].z;
                }
#pragma unroll
                for (uint32_t w = 0; w < 4; w++) {
                  if (wc + w >= W) x[w] = 0;
                  if (x[w] && G != Gt) {
                    uint64_t off = 0;
                    for (uint64_t gm = G; gm; gm &= gm - 1) off |= slot[(size_t)ffs64(gm) * W + wc + w];
                    x[w] &= off;
                  }
                  accw |= x[w];
                }
              }
            }
          }
          // the candidate's lanes (all active: pre is per candidate)
          const uint64_t gb = __ballot(accw != 0);
          feas = ((gb >> (lane & ~((1u << lg) - 1u))) & ((1ull << (1u << lg)) - 1ull)) != 0;
          if (TOPO && feas && KD.tmpl[t].mv_mask) {
            // minValues over the NodeClaim's options after Add (per lane)
            feas = mv_ok(KD, KD.tmpl[t], [&](uint32_t w) -> uint64_t {
              if (!WIDE) return w == 0 ? nx[0] : w == 1 ? nx[1] : w == 2 ? nx[2] : nx[3];
              uint64_t x = opts[w] & row[w];
#pragma unroll
              for (uint32_t r = 0; r < RR; r++) x &= KD.thr_set[(size_t)mrow[r] * OW + w];
              if (G != Gt) {
                uint64_t off = 0;
                for (uint64_t gm = G; gm; gm &= gm - 1) off |= slot[(size_t)ffs64(gm) * W + w];
                x &= off;
              }
              return x;
            });
          }
        }
      }
        const uint64_t fm = __ballot(feas);
        TLW(6);  // phase B: exact checks
        if (fm) {
          const uint32_t wl = ffs64(fm);
          f = rlane(xpos, wl);
#ifdef GS_FFD_TL
          n_xwin++;
#endif
        if (GS_ADD_LANES && WIDE) {
          // the winner's option words after Add, one lane per word (one
          // round trip per 64 words instead of one per word): its threshold
          // rows and offering grid come from its lane
          const uint32_t jw = rlane(j, wl), tw = rlane(t, wl);
          uint32_t mw[RR];
  #pragma unroll
          for (uint32_t r = 0; r < RR; r++) mw[r] = rlane(mrow[r], wl);
          const uint64_t Gw = ((uint64_t)rlane((uint32_t)(G >> 32), wl) << 32) | rlane((uint32_t)G, wl);
          const uint64_t Gtw = ((uint64_t)rlane((uint32_t)(Gt >> 32), wl) << 32) | rlane((uint32_t)Gt, wl);
          uint64_t* wopts = KD.c_opts + (size_t)jw * OW;
          const uint64_t* row = KD.rows + ((size_t)v * T + tw) * OW;
          for (uint32_t w = lane; w < W; w += 64) {
            uint64_t x = wopts[w] & row[w];
  #pragma unroll
            for (uint32_t r = 0; r < RR; r++) x &= KD.thr_set[(size_t)mw[r] * OW + w];
            if (Gw != Gtw) {
              uint64_t off = 0;
              for (uint64_t gm = Gw; gm; gm &= gm - 1) off |= slot[(size_t)ffs64(gm) * W + w];
              x &= off;
            }
            wopts[w] = x;
          }
        }
        if (lane == wl) {
          // NodeClaim.Add by the winning lane: options (wide rows: above),
          // requests, requirements
          ClaimRec* cr = KD.c_rec + j;
          uint64_t* opts = KD.c_opts + (size_t)j * OW;
          if (!WIDE) {
  #pragma unroll
            for (uint32_t w = 0; w < WREG; w++)
              if (w < W) opts[w] = nx[w];  // already narrowed to the grid
          } else if (WIDE && !GS_ADD_LANES) {
            const uint64_t* row = KD.rows + ((size_t)v * T + t) * OW;
            for (uint32_t w = 0; w < W; w++) {
              uint64_t x = opts[w] & row[w];
  #pragma unroll
              for (uint32_t r = 0; r < RR; r++) x &= KD.thr_set[(size_t)mrow[r] * OW + w];
              if (G != Gt) {
                uint64_t off = 0;
                for (uint64_t gm = G; gm; gm &= gm - 1) off |= slot[(size_t)ffs64(gm) * W + w];
                x &= off;
              }
              opts[w] = x;
            }
          }
          int64_t nt[RR], ma[RR];
          uint32_t cu[RR];
  #pragma unroll
          for (uint32_t r = 0; r < RR; r++) {
            nt[r] = tot[r] + RQ(r);
            ma[r] = GS_MAXA_PF ? maxa_pre[r] : cr->maxa[r];
            cu[r] = mrow[r] - s_thoff[r] - r;
            cr->tot(r) = nt[r];
            cr->thr(r) = (uint16_t)cu[r];
          }
          s_slk[j] = pack_slack(d, ma, nt);  // exact re-quantization: no drift
          s_rm[j] = pack_room(thr, s_thoff, cu, nt, KD.RQ);
          cr->zm = zm & vzm;  // zm (dom_ct: cm) carries the topology narrowing
          cr->cm = cm & vcm;
          cr->ctb &= vctb;
          if (TOPO) {
            // zone requirement after Add (+ the topology domain), then
            // <U> Topology.Record for every group selecting the pod
            if (!own_n) {
              czf = cr->zfull;
              czfl = cr->zflags;
            }
            const uint64_t zf = czf & vzn & zset;
            const uint32_t zl = zset != ~0ull ? 0u : (czfl & vzflags);
            cr->zfull = zf;
            cr->zflags = zl;
            int32_t* hrow = KD.hc + (size_t)j * KD.TGH;
            topo_record(KD, ts, sel_off, sel_n, zf, zl, [&](uint32_t hs) { hrow[hs] = (hrow[hs] & HC_COUNT) + 1; });
          }
          FK* cf = KD.c_fk + (size_t)j * F;
          for (uint32_t k = 0; k < fk_count; k++) {
            const FKEntry& e = KD.fk_entries[fk_begin + k];
            const FK cur = cf[e.slot];
            cf[e.slot] = (cur.flags & FK_PRESENT)
                             ? fk_intersect(cur, e.st, KD.fk_ival + (size_t)e.slot * FKV, KD.fk_isint + (size_t)e.slot * FKW)
                             : e.st;
          }
          const uint32_t e = s_so[f];
          if ((e & 0xFFFFu) == 0xFFFFu) ovf = true;
          s_so[f] = e + 1u;
        }
          wsyncT<CH>();
          emit(WQ_LOG, nlog, gp, v, rlane(j, wl), 0, 0);
          break;
        }
      }
      if (fa_pos != INF) {
        // --- fast accept (simple pod): NodeClaim.Add changes the requests
        // only; options, cursors and requirements stay.  LDS room and slack
        // shrink by the request (still a lower / upper bound); the agent wave
        // adds the requests to the claim's totals (an exact check drains the
        // channel before it reads them).
        f = fa_pos;
        const uint32_t j = fa_j;
        {
          // lane r < RQ re-quantizes resource r: room (lower bound) and
          // slack (upper bound) shrink by the request.  The old codes and
          // order word come from the scan's lanes; the new codes are packed
          // across lanes 0..3 with DPP (no scalar round trip) and lane 0
          // stores them
          const uint32_t fl = fa_l;
          const uint64_t rm = ((uint64_t)rlane((uint32_t)(fa_rv >> 32), fl) << 32) | rlane((uint32_t)fa_rv, fl);
          const uint64_t sl = ((uint64_t)rlane((uint32_t)(fa_sq >> 32), fl) << 32) | rlane((uint32_t)fa_sq, fl);
          const uint32_t e = rlane(fa_ev, fl);
          uint32_t c_rm = 0, c_sl = 0;
          if (lane < d.RQ) {
            const uint32_t sh = 16 * lane;
            c_rm = qcode_floor(qcode_value((uint32_t)(rm >> sh) & 0xFFFFu) - rq_lane);
            c_sl = qcode_ceil(qcode_value((uint32_t)(sl >> sh) & 0xFFFFu) - rq_lane);
          }
          uint32_t prm = (lane & 1u) ? c_rm << 16 : c_rm, psl = (lane & 1u) ? c_sl << 16 : c_sl;
          prm |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)prm, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
          psl |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)psl, 0xB1, 0xF, 0xF, false);
          const uint32_t hrm = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)prm, 0x102, 0xF, 0xF, false);  // row_shl:2
          const uint32_t hsl = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)psl, 0x102, 0xF, 0xF, false);
          if ((e & 0xFFFFu) == 0xFFFFu) ovf = true;
          if (lane == 0) {
            s_rm[j] = (uint64_t)prm | ((uint64_t)hrm << 32);
            s_slk[j] = (uint64_t)psl | ((uint64_t)hsl << 32);
            s_so[f] = e + 1u;
            if (TOPO && sel_n) {
              // <U> Topology.Record in the groups that select the pod: the
              // NodeClaim's requirements are unchanged by this Add
              const auto& KD = *karg();
              const ClaimRec* cr = KD.c_rec + j;
              int32_t* hrow = KD.hc + (size_t)j * KD.TGH;
              topo_record(KD, ts, sel_off, sel_n, cr->zfull, cr->zflags, [&](uint32_t hs) { hrow[hs] = (hrow[hs] & HC_COUNT) + 1; });
            }
          }
        }
        wsyncT<CH>();
        emit(WQ_FA, nlog, gp, v, j, rqd, rq_lane);  // the requests into the claim totals, and the log
        CTR(C_FA, 1);
        break;
      }
      if (resume == INF) break;
      scan_from = resume;
    }
    if (__ballot(ovf)) status = 3;
    CTR(C_ALG, f != INF ? f + 1 : M);  // the reference's NodeClaim.CanAdd calls
    TLW(3);  // scan + Add
#ifdef GS_FFD_TL
    n_fsum += f != INF ? f : 0;
#endif
    if (simple) {
      // [0, f) (or all positions) are infeasible for these requests
      hint = f != INF ? f : M;
      hint_ok = true;
      hint_tolt = vtolt;
      hint_rq = rq_lane;
    }
    if (f != INF) {
      wsyncT<CH>();
      modkind = MOD_INC;
      modpos = f;
      nlog++;
      // the next pod may repeat this one's spec (runs, above)
      run_prev = GS_RUNS && !TOPO && (!WIDE || GS_RUN_WIDE) && from_ring && simple && !__ballot(ovf);
      CAT(simple ? 1 : 3);
      run_rec = vrd;
      continue;
    }

    // ------------------------------- new NodeClaim from templates, in order
    bool opened = false;
    {
      const auto& KD = *karg();
      const uint32_t vx = fresh(vrd);
      auto VX = [&](uint32_t i) -> uint32_t { return rlane(vx, i); };
      auto VX64 = [&](uint32_t i) -> uint64_t { return (uint64_t)VX(i) | ((uint64_t)VX(i + 1) << 32); };
      const uint32_t fk_begin = VX(1), fk_count = VX(2), vzflags = VX(30);
      const uint64_t vzm = VX64(14), vcm = VX64(16), vzn = VX64(28);
    for (uint32_t t = 0; t < T; t++) {
      const TmplRec& tr = KD.tmpl[t];
      const uint64_t* row = KD.rows + ((size_t)v * T + t) * OW;
      // <U> Topology on the fresh NodeClaim (template AND pod zone domains;
      // a new hostname domain has count 0, always within maxSkew >= 1):
      // the picked zone narrows the K1 row to that zone's offerings
      // (pod affinity on the fresh hostname domain, count 0: only the
      // bootstrap of a self-selecting pod while no selected pod runs)
      uint64_t tzs = ~0ull, tzcat = ~0ull;  // allowed zone domains / their catalog zones
      if (TOPO && own_n) {
        tzs = topo_claim_g(KD, ts, own_n, tr.zfull & vzn, [](uint32_t) -> int64_t { return 0; }, OWN);
        if (tzs != 0 && tzs != ~0ull && !KD.dom_np) tzcat = topo_catmask(KD, tzs);
        tzs = (uint64_t)uniform_i64((int64_t)tzs);
        tzcat = (uint64_t)uniform_i64((int64_t)tzcat);
        if (tzs == 0 || tzcat == 0) continue;
      }
      // dom_ct: the picked domains are capacity types of the template's zones
      const bool dct = KD.dom_ct != 0;
      const uint64_t tcm = tr.cm & vcm & (dct ? tzcat : ~0ull), tzsel = dct ? tr.zm & vzm : tzcat;
      const bool dnp = KD.dom_np != 0;  // a NodePool domain narrows no offering
      auto rowx = [&](uint32_t w) -> uint64_t {
        uint64_t x = row[w];
        if (tzs != ~0ull && !dnp) {
          uint64_t off = 0;
          for (uint64_t zm_ = tzsel; zm_; zm_ &= zm_ - 1) {
            const uint32_t zc = ffs64(zm_);
            for (uint32_t c = 0; c < KD.C; c++)
              if ((tcm >> c) & 1) off |= slot[(zc * KD.C + c) * W + w];
          }
          x &= off;
        }
        return x;
      };
      bool anyl = false;
      if (KD.fk_ok[(size_t)v * T + t])
        for (uint32_t w = lane; w < W; w += 64) anyl = anyl || rowx(w) != 0;
      if (!__ballot(anyl)) continue;
      if (tr.has_limits) {
        // <U> filterByRemainingResources on the template's options
        bool hit = false;
        for (uint32_t i = lane; i < KD.N; i += 64) {
          if (!((rowx(i >> 6) >> (i & 63)) & 1)) continue;
          bool ok = true;
          for (uint32_t r = 0; r < R; r++)
            if ((tr.limit_rmask >> r) & 1) ok = ok && KD.it_cap[(size_t)r * KD.N + i] <= KD.t_rem[(size_t)t * R + r];
          hit = hit || ok;
        }
        if (!__ballot(hit)) continue;
      }
      // threshold cursors of the fresh claim: lane r < R
      int64_t tot_l = 0;
      uint32_t c0_l = 0;
      if (lane < R) {
        tot_l = tr.daemon[lane] + rq_lane;
        const uint32_t o = s_thoff[lane], n = s_thoff[lane + 1] - o;
        c0_l = thr_search(thr + o, n, 0, tot_l);
      }
      uint32_t c0[RR];
#pragma unroll
      for (uint32_t r = 0; r < RR; r++) c0[r] = (uint32_t)__shfl((int)c0_l, (int)r);
      // option words (lane w holds word w, and w + 64)
      uint64_t xw[2] = {0, 0};
#pragma unroll
      for (uint32_t h = 0; h < 2; h++) {
        const uint32_t w = lane + 64 * h;
        if (w >= W) continue;
        uint64_t x = rowx(w);
        // establish opts ⊆ thr_set[cursor] for the candidate scan
#pragma unroll
        for (uint32_t r = 0; r < RR; r++) x &= KD.thr_set[(size_t)(s_thoff[r] + r + c0[r]) * OW + w];
        if (tr.has_limits) {
          uint64_t y = 0;
          for (uint64_t m = x; m; m &= m - 1) {
            const uint32_t b = ffs64(m);
            const uint32_t i = w * 64 + b;
            bool ok = true;
            for (uint32_t r = 0; r < R; r++)
              if ((tr.limit_rmask >> r) & 1) ok = ok && KD.it_cap[(size_t)r * KD.N + i] <= KD.t_rem[(size_t)t * R + r];
            if (ok) y |= 1ull << b;
          }
          x = y;
        }
        xw[h] = x;
      }
      // minValues over the fresh NodeClaim's options (uniform: every lane
      // evaluates the same words)
      if (TOPO && tr.mv_mask && !mv_ok(KD, tr, [&](uint32_t w) { return shfl_u64(xw[w >> 6], w & 63); })) continue;
      if (M >= MC) {
        status = 1;
        break;
      }
      const uint32_t j = M;
      ClaimRec* cr = KD.c_rec + j;
#pragma unroll
      for (uint32_t h = 0; h < 2; h++)
        if (lane + 64 * h < W) KD.c_opts[(size_t)j * OW + lane + 64 * h] = xw[h];
      if (lane < RR) {
        cr->tot(lane) = tot_l;
        cr->thr(lane) = (uint16_t)c0_l;
      }
      // max allocatable over the new claim's options (the slack bound), and
      // (limits) the max capacity for subtractMax: lane = instance type
      uint64_t mxa[RR], mxc[RR];
#pragma unroll
      for (uint32_t r = 0; r < RR; r++) mxa[r] = mxc[r] = 0;
      for (uint32_t w = 0; w < W; w++) {
        const uint64_t word = shfl_u64(xw[w >> 6], w & 63);
        if (!((word >> lane) & 1)) continue;
        const uint32_t i = w * 64 + lane;
#pragma unroll
        for (uint32_t r = 0; r < RR; r++) {
          const uint64_t a = (uint64_t)KD.it_alloc[(size_t)r * KD.N + i];
          mxa[r] = a > mxa[r] ? a : mxa[r];
          if (tr.has_limits && ((tr.limit_rmask >> r) & 1)) {
            const uint64_t c = (uint64_t)(KD.it_cap[(size_t)r * KD.N + i] + (1ll << 62));
            mxc[r] = c > mxc[r] ? c : mxc[r];
          }
        }
      }
      int64_t ma[RR], nt[RR];
      GS_RQ_AT(RQ);
#pragma unroll
      for (uint32_t r = 0; r < RR; r++) {
        ma[r] = (int64_t)wave_max_u64(mxa[r]);
        if (tr.has_limits) mxc[r] = wave_max_u64(mxc[r]);
        nt[r] = tr.daemon[r] + RQ(r);
      }
      // <U> Topology.Register(hostname placeholder): the claim's counts start at 0
      if (TOPO)
        for (uint32_t h = lane; h < KD.TGH; h += 64) KD.hc[(size_t)j * KD.TGH + h] = 0;
      const uint64_t n_sl = pack_slack(d, ma, nt), n_rm = pack_room(thr, s_thoff, c0, nt, KD.RQ);
      wsyncT<CH>();
      if (lane == 0) {
        cr->tmpl = t;
        cr->count = 1;
        cr->zm = tr.zm & vzm & (dct ? ~0ull : tzcat);
        cr->cm = tcm;
        cr->ctb = tr.ctb & vctb;
        cr->zfull = tr.zfull & vzn & tzs;
        cr->zflags = tzs != ~0ull ? 0u : (tr.zflags & vzflags);
#pragma unroll
        for (uint32_t r = 0; r < RR; r++) cr->maxa[r] = ma[r];
        if (TOPO && sel_n) {
          // <U> Topology.Record
          int32_t* hrow = KD.hc + (size_t)j * KD.TGH;
          topo_record(KD, ts, sel_off, sel_n, cr->zfull, cr->zflags, [&](uint32_t hs) { hrow[hs] = (hrow[hs] & HC_COUNT) + 1; });
        }
        FK* cf = KD.c_fk + (size_t)j * F;
        for (uint32_t s = 0; s < F; s++) cf[s] = KD.t_fk[(size_t)t * F + s];
        for (uint32_t k = 0; k < fk_count; k++) {
          const FKEntry& e = KD.fk_entries[fk_begin + k];
          const FK cur = cf[e.slot];
          cf[e.slot] = (cur.flags & FK_PRESENT)
                           ? fk_intersect(cur, e.st, KD.fk_ival + (size_t)e.slot * FKV, KD.fk_isint + (size_t)e.slot * FKW)
                           : e.st;
        }
        s_so[M] = 1u | (M << 16);
        s_tmpl[M] = (uint8_t)t;
        s_slk[j] = n_sl;
        s_rm[j] = n_rm;
        if (tr.has_limits) {
          // <U> subtractMax(remaining, nodeClaim.InstanceTypeOptions)
          for (uint32_t r = 0; r < R; r++)
            if (((tr.limit_rmask >> r) & 1) && mxc[r] != 0) KD.t_rem[(size_t)t * R + r] -= (int64_t)(mxc[r] - (1ull << 62));
        }
      }
      wsyncT<CH>();
      emit(WQ_LOG, nlog, gp, v, j, 0, 0);
      M++;
      modkind = MOD_APPEND;
      nlog++;
      opened = true;
      break;
    }
    }
    TLW(4);  // new NodeClaim
    if (status) break;
    if (opened) {
      CAT(4);
      continue;
    }
    CAT(5);

    // -------------------------------------- failed: Relax, then Queue.Push
    {
      const auto& KD = *karg();
      const uint32_t vb = __builtin_amdgcn_readfirstlane(KD.var_begin[gp]);
      const uint32_t vc = __builtin_amdgcn_readfirstlane(KD.var_count[gp]);
      const bool relaxed = v + 1 < vb + vc;
      uint32_t tail = qhead + qlen;
      if (tail >= P) tail -= P;
      qlen++;
      if (TOPO && relaxed && KD.n_lazy) topo_relaxed(KD, ts, v + 1, KD.hc, M, lane, 64u);
      if (lane == 0) {
        if (relaxed) KD.cur_var[p] = v + 1;
        KD.queue[tail] = p;
        if (!relaxed) {
          KD.last_epoch[p] = epoch;
          KD.last_len[p] = qlen;
        }
      }
      if (relaxed) epoch++;
    }
  }
  // stop the agent once every posted write is done
  post(WQ_STOP, 0, 0, 0, 0, 0);
  drain();
  if (chan_err) status = 2;
  wsyncT<CH>();
  for (uint32_t i = lane; i < M; i += 64) {
    const uint32_t e = s_so[i];
    d.c_sorted[i] = e >> 16;
    d.c_rec[e >> 16].count = e & 0xFFFFu;
  }
#ifdef GS_CTR_LDS
  wsync();
  auto ctr_at = [&](uint32_t k) -> uint64_t { return (uint64_t)s_ctr[k]; };
#else
  auto ctr_at = [&](uint32_t k) -> uint64_t { return (uint64_t)rlane((uint32_t)ctr, k) | ((uint64_t)rlane((uint32_t)(ctr >> 32), k) << 32); };
#endif
  const uint64_t ctr_gen = ctr_at(C_GEN), ctr_fast = ctr_at(C_FAST), ctr_cand = ctr_at(C_CAND), ctr_full = ctr_at(C_FULL),
                 ctr_nev = ctr_at(C_NEV), ctr_npre = ctr_at(C_NPRE), ctr_fa = ctr_at(C_FA), ctr_alg = ctr_at(C_ALG);
#ifdef GS_CAT_TL
  uint64_t cat_cyc_l[8], cat_n_l[8];
#pragma unroll
  for (uint32_t q = 0; q < 8; q++) {
    cat_cyc_l[q] = (uint64_t)rlane((uint32_t)cat_cyc, q) | ((uint64_t)rlane((uint32_t)(cat_cyc >> 32), q) << 32);
    cat_n_l[q] = (uint64_t)rlane((uint32_t)cat_n, q) | ((uint64_t)rlane((uint32_t)(cat_n >> 32), q) << 32);
  }
#endif
  uint64_t ctr_run[7];
#pragma unroll
  for (uint32_t q = 0; q < 7; q++) ctr_run[q] = ctr_at(C_RPODS + q);
  if (lane == 0) {
    Ctrl c = {};
    c.status = status;
    c.n_claims = M;
    c.n_log = nlog;
    c.qhead = qhead;
    c.qlen = qlen;
    c.epoch = epoch;
    c.pops = pops;
    c.generic_sorts = ctr_gen;
    c.fast_sorts = ctr_fast;
    c.cand_evals = ctr_cand;
    c.cand_full = ctr_full;
    c.node_evals = ctr_nev;
    c.node_prefix = ctr_npre;
    c.claim_prefix = ctr_alg;
    c.dbg[15] = ctr_fa;
#ifdef GS_CAT_TL
    for (uint32_t q = 0; q < 8; q++) {
      c.dbg[q] = cat_cyc_l[q];
      c.dbg[8 + q] = cat_n_l[q];
    }
#elif !defined(GS_FFD_TL)
    for (uint32_t q = 0; q < 6; q++) c.dbg[8 + q] = ctr_run[q];
#ifdef GS_RUN_TL
    c.dbg[14] = run_cyc;
#else
    c.dbg[14] = ctr_run[6];  // run-mode exact batches
#endif
    c.dbg[5] = ctr_at(C_RBPODS);  // pods placed in run batches (GS_RUN_BATCH)
    c.dbg[6] = ctr_at(C_RBATCH);  // run batches
#ifdef GS_RUN_TL
    c.dbg[3] = ctr_at(C_RBT0);  // ticks in the batch step, check included
    c.dbg[4] = ctr_at(C_RBT1);  // ticks in the batches' placement
#endif
#endif
    c.t_sort = c.t_scan = c.t_tmpl = ~0ull;  // not measured: gs_result reports -1
#ifdef GS_FFD_TL
    for (int q = 0; q < 8; q++) c.dbg[q] = tl[q];
    c.dbg[8] = n_gen_cyc;  // shader cycles in Go's full pdqsort (generic sorts)
#ifdef GS_SORT_TL
    for (int q = 0; q < 7; q++) c.dbg[9 + q] = s_stl[q];  // generic sort: seq, uniform, pivot, partial, peq, part, frames
#ifdef GS_SORT_TL2
    for (int q = 0; q < 4; q++) c.dbg[q] = s_stl[8 + q];  // partition: swap in, count, lists, swaps out
#endif
#else
    c.dbg[9] = n_xns;
    c.dbg[10] = n_xb;
    c.dbg[11] = n_xwin;
#ifdef GS_CAT_SEG
    c.dbg[12] = n_cat;
#else
    c.dbg[12] = n_nonsimple;
#endif
    c.dbg[13] = n_rot;
    c.dbg[14] = n_rotlen;
#endif
#endif
    *d.ctrl = c;
  }
}
