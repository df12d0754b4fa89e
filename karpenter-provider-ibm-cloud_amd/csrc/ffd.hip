// ffd.hip — K4: the <U> Scheduler.Solve queue loop (first-fit decreasing over
// existing/in-flight/new NodeClaims) as ONE persistent 1024-thread workgroup.
//
// Per popped pod:
//  1. sort.Slice(newNodeClaims, len(Pods) asc) is reproduced EXACTLY (Go's
//     pdqsort_func permutes ties; which NodeClaim a pod lands on depends on
//     it).  Between two sorts at most one NodeClaim changed (one pod added,
//     or one NodeClaim appended), so the common case is resolved in O(1)
//     decisions + one parallel rotation (see DESIGN.md "sort emulation");
//     every other case runs a block-parallel restatement of pdqsort_func
//     whose partition / partitionEqual / partialInsertionSort passes are
//     ballot-prefix compactions over LDS.
//  2. in-flight NodeClaims are scored 1024 at a time in sorted order; a cheap
//     necessary test (tolerated template, per-resource slack upper bound)
//     gates the exact NodeClaim.CanAdd (free-key Compatible, instance-type
//     bitset AND, fits via per-resource threshold bitsets, offering grid);
//     the first feasible position wins (block min).
//  3. otherwise templates in weight order open a new NodeClaim from the
//     precomputed K1 row (limits applied dynamically); else Relax + requeue.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "devutil.hpp"
#include "ffd_common.hpp"
#include "layout.hpp"

using namespace gsd;

namespace {

// GS_FFD_TL (diagnostic build): tid 0 accumulates shader cycles per segment
// of the pod loop into S.tl[k], reported through Ctrl.dbg
#ifdef GS_FFD_TL
#define TL(k)                                              \
  do {                                                     \
    if (tid == 0) {                                        \
      const uint64_t tl_t_ = __builtin_amdgcn_s_memtime(); \
      S.tl[k] += tl_t_ - S.tl_last;                        \
      S.tl_last = tl_t_;                                   \
    }                                                      \
  } while (0)
#else
#define TL(k) \
  do {        \
  } while (0)
#endif
#ifndef GS_FB_MAX
#define GS_FB_MAX 512
#endif
constexpr int FB_MAX = GS_FB_MAX;  // workgroup size of the provisioning Solve (512: 256 VGPRs, no spills)
// Workgroup sizes of one consolidation simulation.  Many small simulations
// (SingleNode: thousands, ~20 pods each) are throughput-bound: 128 threads at
// 3 waves per SIMD compile spill-free and keep 6 workgroups per CU resident.
// Few large ones (MultiNode prefixes: up to 100 nodes' pods) are latency-bound
// and use 256 threads (gs_consolidate picks, DevProblem::sim_nt).
constexpr int FB_SIM = 256;
constexpr int FB_SIM_NARROW = 128;
constexpr int NWAVE_MAX = FB_MAX / 64;
#ifndef GS_SEQ_SORT
#define GS_SEQ_SORT 32  // measured on CM: 32 -> 789 ms, 64 -> 815, 128 -> 819 (same box)
#endif
constexpr int SEQ_SORT = GS_SEQ_SORT;  // subranges up to this length sort on thread 0

constexpr uint32_t WREG = 4;  // option words a scoring lane keeps in registers
enum : uint32_t { MOD_NONE = 0, MOD_INC = 1, MOD_APPEND = 2 };


// Block-uniform state of the pod loop.  Every wave reads it once per pod
// right after the loop-top barrier and then keeps its own register copy,
// computing the pop, the sort decision and the scan's bookkeeping
// identically; thread 0 writes every change to the other buffer (read by the
// next pod, and by the paths that still share state through LDS: existing
// nodes, new NodeClaims, Relax/Push), so no wave can see a half-updated copy.
struct alignas(16) Hot {
  uint32_t qhead, qlen, epoch, M;
  uint32_t modkind, modpos, nlog, cb;  // cb: which vrb/reqb buffer holds the current pod
  uint32_t wrapped, status, nx_valid, nx_pod;  // wrapped: pods now come back from Push
  uint32_t nx_gp, nx_le, nx_ll, nx_cv;         // next-pod pipeline (published by wave 1)
  uint64_t pops, pad;
};

struct Shared {
  Hot hb[2];  // the pod loop's block-uniform state, double-buffered per pod
  uint32_t found;
  uint32_t fast_path, modpos_sorted;
  uint32_t rot_lo, rot_hi;  // fast path: the one rotation partialInsertionSort performs
  int piv, hint;
  uint64_t generic, fast, cand, cand_full, node_evals, node_prefix, claim_prefix;
  uint32_t failed;
  uint64_t t_sort, t_scan, t_tmpl, t0;
  uint64_t dbg[16];
  uint64_t tl[16], tl_last;  // GS_FFD_TL: shader cycles per loop segment (tid 0)
  uint64_t tl_arr[NWAVE_MAX];  // GS_FFD_TL: per-wave arrival at the loop-top barrier
  uint32_t c0[RMAX];  // threshold cursors of a NodeClaim being opened
  uint32_t mvok;      // minValues verdict on the NodeClaim being opened
  uint32_t red[2][NWAVE_MAX];
  alignas(16) uint32_t red2[2][NWAVE_MAX];  // Wg reductions (own double buffer: never adjacent to a Blk one)
  unsigned long long red64[RMAX];
  Frame stk[48];
  // next-pod pipeline: wave 1 prefetches the next pop during the current pod
  uint32_t use_pf;
  // solve in this block: simulation id, pod/claim arena offset, global pod id,
  // overlay entry count / the entry being written (and whether it is new)
  uint32_t sim, qoff, gpod, nov, ove, ov_new, ov_fk;
  alignas(16) uint32_t vrb[2][(sizeof(VarRec) / 4 + 3) & ~3u];
  alignas(16) int64_t reqb[2][RMAX];
};
constexpr uint32_t VR_DW = sizeof(VarRec) / 4;
static_assert(VR_DW <= 32, "VarRec prefetch uses one lane per dword");


// ------------------------------------------------------- hot block helpers
// The per-pod reductions and the one-step rotation.  Only force-inlined
// methods and never passed by address, so the object stays in registers and
// every pointer keeps its LDS address space (ds_* instructions; Blk below is
// materialized in scratch by its out-of-line sort methods, which costs
// scratch + flat round trips per call).
template <uint32_t NT>
struct Wg {
  static constexpr int NWAVE = (int)NT / 64;
  static constexpr int KR = 8;  // rotate1 handles up to KR * NT elements
  uint32_t* red;                // [2][NWAVE_MAX]
  uint16_t* sc;
  uint16_t* ord;
  uint32_t tid, lane, wave;
  uint32_t tog;
  // Reductions over lane-ordered positions: thread t stands for position
  // base + t, so a wave's first flagged position is one ballot (no lane
  // shuffles: ds_bpermute chains cost ~60 cycles per step); one LDS slot per
  // wave, one barrier, one vector read of all slots.
  __device__ __forceinline__ uint32_t wave_first(bool flag, uint32_t base) const {
    const uint64_t b = __ballot(flag);
    return b ? base + wave * 64u + (uint32_t)__ffsll((long long)b) - 1u : INF;
  }
  __device__ __forceinline__ uint32_t cross_min(uint32_t v) {
    uint32_t* r = red + tog * NWAVE_MAX;
    if (lane == 0) r[wave] = v;
    __syncthreads();
    uint32_t x = INF;
#pragma unroll
    for (int w = 0; w < NWAVE; w += 4) {
      const uint4 q = *(const uint4*)(r + w);
      x = q.x < x ? q.x : x;
      if (w + 1 < NWAVE) x = q.y < x ? q.y : x;
      if (w + 2 < NWAVE) x = q.z < x ? q.z : x;
      if (w + 3 < NWAVE) x = q.w < x ? q.w : x;
    }
    tog ^= 1u;
    return x;
  }
  // first position base + t whose flag is set (INF if none)
  __device__ __forceinline__ uint32_t first(bool flag, uint32_t base) { return cross_min(wave_first(flag, base)); }
  // the first positions of two flags (16-bit positions) in one barrier
  __device__ __forceinline__ uint2 first2(bool fa, bool fb, uint32_t base) {
    const uint32_t a = wave_first(fa, base), b = wave_first(fb, base);
    const uint32_t v = ((a < 0xFFFFu ? a : 0xFFFFu) << 16) | (b < 0xFFFFu ? b : 0xFFFFu);
    uint32_t* r = red + tog * NWAVE_MAX;
    if (lane == 0) r[wave] = v;
    __syncthreads();
    uint32_t ra = 0xFFFFu, rb = 0xFFFFu;
#pragma unroll
    for (int w = 0; w < NWAVE; w += 4) {
      const uint4 q = *(const uint4*)(r + w);
      const uint32_t xs[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int k = 0; k < 4; k++) {
        if (w + k >= NWAVE) break;
        ra = (xs[k] >> 16) < ra ? (xs[k] >> 16) : ra;
        rb = (xs[k] & 0xFFFFu) < rb ? (xs[k] & 0xFFFFu) : rb;
      }
    }
    tog ^= 1u;
    return make_uint2(ra == 0xFFFFu ? INF : ra, rb == 0xFFFFu ? INF : rb);
  }
  // rotate [lo, hi] by one (left: lo's element lands at hi; right: hi's at lo)
  // in one staged read / barrier / write; false if the range is too long
  __device__ __forceinline__ bool rotate1(int lo, int hi, bool left) {
    if (hi - lo + 1 > KR * (int)NT) return false;
    uint16_t vs[KR], vo[KR];
#pragma unroll
    for (int i = 0; i < KR; i++) {
      const int k = lo + (int)tid + i * (int)NT;
      if (k <= hi) {
        const int src = left ? (k == hi ? lo : k + 1) : (k == lo ? hi : k - 1);
        vs[i] = sc[src];
        vo[i] = ord[src];
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < KR; i++) {
      const int k = lo + (int)tid + i * (int)NT;
      if (k <= hi) {
        sc[k] = vs[i];
        ord[k] = vo[i];
      }
    }
    return true;
  }
};

// ------------------------------------------------------------ block-parallel
// SEQ: subranges up to this length run on thread 0 (any SEQ >= 12 gives the
// same permutation: both paths restate pdqsort_func)
template <uint32_t NT, int SEQ = SEQ_SORT>
struct Blk {
  static_assert(SEQ >= 12, "block pdqsort must hand ranges <= 12 (Go's insertion-sort cutoff) to SeqSort");
  static constexpr int FB = (int)NT;
  static constexpr int NWAVE = (int)NT / 64;
  uint16_t* sc;
  uint16_t* ord;
  uint16_t* scr;  // >= max_claims entries
  Shared& S;
  uint32_t tid, lane, wave;
  uint32_t tog;  // reduction double-buffer toggle (uniform)
  uint32_t half; // scr split point

  __device__ void sync() { __syncthreads(); }
  __device__ void swap(int i, int j) const {
    uint16_t a = sc[i];
    sc[i] = sc[j];
    sc[j] = a;
    a = ord[i];
    ord[i] = ord[j];
    ord[j] = a;
  }
  // block reductions: one barrier each (double-buffered slots)
  __device__ uint32_t bmin(uint32_t v) {
    for (int m = 32; m >= 1; m >>= 1) {
      uint32_t y = (uint32_t)__shfl_xor((int)v, m);
      v = y < v ? y : v;
    }
    if (lane == 0) S.red[tog][wave] = v;
    sync();
    uint32_t r = S.red[tog][0];
    for (int w = 1; w < NWAVE; w++) r = S.red[tog][w] < r ? S.red[tog][w] : r;
    tog ^= 1;
    return r;
  }
  // two independent minima of 16-bit positions (INF = none) in one barrier
  __device__ uint2 bmin2(uint32_t a, uint32_t b) {
    a = a < 0xFFFFu ? a : 0xFFFFu;
    b = b < 0xFFFFu ? b : 0xFFFFu;
    for (int m = 32; m >= 1; m >>= 1) {
      const uint32_t ya = (uint32_t)__shfl_xor((int)a, m), yb = (uint32_t)__shfl_xor((int)b, m);
      a = ya < a ? ya : a;
      b = yb < b ? yb : b;
    }
    if (lane == 0) S.red[tog][wave] = (a << 16) | b;
    sync();
    uint32_t ra = 0xFFFFu, rb = 0xFFFFu;
    for (int w = 0; w < NWAVE; w++) {
      const uint32_t x = S.red[tog][w];
      ra = (x >> 16) < ra ? (x >> 16) : ra;
      rb = (x & 0xFFFFu) < rb ? (x & 0xFFFFu) : rb;
    }
    tog ^= 1;
    return make_uint2(ra == 0xFFFFu ? INF : ra, rb == 0xFFFFu ? INF : rb);
  }
  __device__ int32_t bmax(int32_t v) {
    for (int m = 32; m >= 1; m >>= 1) {
      int32_t y = __shfl_xor(v, m);
      v = y > v ? y : v;
    }
    if (lane == 0) S.red[tog][wave] = (uint32_t)v;
    sync();
    int32_t r = (int32_t)S.red[tog][0];
    for (int w = 1; w < NWAVE; w++) r = (int32_t)S.red[tog][w] > r ? (int32_t)S.red[tog][w] : r;
    tog ^= 1;
    return r;
  }
  // positions k in [lo,hi) with pred(k), in ascending (desc=false) or
  // descending order, written to out[]; returns the count
  template <class Pred>
  __device__ uint32_t compact(int lo, int hi, bool desc, uint16_t* out, Pred pred) {
    uint32_t total = 0;
    const int n = hi - lo;
    for (int base = 0; base < n; base += FB) {
      const int idx = base + (int)tid;
      const int k = desc ? hi - 1 - idx : lo + idx;
      const bool in = idx < n && pred(k);
      const uint64_t mask = __ballot(in);
      const uint32_t rank = __popcll(mask & ((1ull << lane) - 1));
      if (lane == 0) S.red[tog][wave] = __popcll(mask);
      sync();
      uint32_t off = 0, all = 0;
      for (uint32_t w = 0; w < NWAVE; w++) {
        const uint32_t c = S.red[tog][w];
        off += w < wave ? c : 0;
        all += c;
      }
      if (in) out[total + off + rank] = (uint16_t)k;
      total += all;
      tog ^= 1;
    }
    sync();
    return total;
  }
  // One rotation of [lo, hi] staged through registers across a single
  // barrier: left = the element at lo moves to hi (the rest shift left),
  // otherwise the element at hi moves to lo.  Each thread owns destinations
  // lo + tid + i*FB (i < KR); returns false when the range is too long.
  static constexpr int KR = 8;
  __device__ bool rotate1(int lo, int hi, bool left) {
    if (hi - lo + 1 > KR * FB) return false;
    uint16_t vs[KR], vo[KR];
#pragma unroll
    for (int i = 0; i < KR; i++) {
      const int k = lo + (int)tid + i * FB;
      if (k <= hi) {
        const int src = left ? (k == hi ? lo : k + 1) : (k == lo ? hi : k - 1);
        vs[i] = sc[src];
        vo[i] = ord[src];
      }
    }
    sync();
#pragma unroll
    for (int i = 0; i < KR; i++) {
      const int k = lo + (int)tid + i * FB;
      if (k <= hi) {
        sc[k] = vs[i];
        ord[k] = vo[i];
      }
    }
    return true;
  }
  // shift [lo,hi) right by one; the element at hi lands at lo
  __device__ void rotate_right(int lo, int hi) {
    if (hi <= lo) return;
    const uint16_t xs = sc[hi], xo = ord[hi];
    sync();
    for (int done = 0; done < hi - lo; done += FB) {
      const int k = hi - 1 - done - (int)tid;
      const bool act = k >= lo;
      uint16_t s = 0, o = 0;
      if (act) {
        s = sc[k];
        o = ord[k];
      }
      sync();
      if (act) {
        sc[k + 1] = s;
        ord[k + 1] = o;
      }
      sync();
    }
    if (tid == 0) {
      sc[lo] = xs;
      ord[lo] = xo;
    }
    sync();
  }
  // shift (lo,hi] left by one; the element at lo lands at hi
  __device__ void rotate_left(int lo, int hi) {
    if (hi <= lo) return;
    const uint16_t xs = sc[lo], xo = ord[lo];
    sync();
    for (int base = lo; base < hi; base += FB) {
      const int k = base + (int)tid;
      const bool act = k < hi;
      uint16_t s = 0, o = 0;
      if (act) {
        s = sc[k + 1];
        o = ord[k + 1];
      }
      sync();
      if (act) {
        sc[k] = s;
        ord[k] = o;
      }
      sync();
    }
    if (tid == 0) {
      sc[hi] = xs;
      ord[hi] = xo;
    }
    sync();
  }
  // partition_func: pair the k-th misplaced element of the left region
  // (ascending) with the k-th of the right region (descending), exactly the
  // swaps the sequential two-pointer loop performs
  __device__ int partition(int a, int b, int pivot, bool* already) {
    if (tid == 0) swap(a, pivot);
    sync();
    const uint16_t p = sc[a];
    uint32_t cnt = 0;
    for (int k = a + 1 + (int)tid; k < b; k += FB) cnt += sc[k] < p;
    // block sum via compact-style slots
    for (int m = 32; m >= 1; m >>= 1) cnt += (uint32_t)__shfl_xor((int)cnt, m);
    if (lane == 0) S.red[tog][wave] = cnt;
    sync();
    uint32_t nless = 0;
    for (int w = 0; w < NWAVE; w++) nless += S.red[tog][w];
    tog ^= 1;
    const int mid = a + (int)nless;
    const uint32_t s = compact(a + 1, mid + 1, false, scr, [&](int k) { return sc[k] >= p; });
    compact(mid + 1, b, true, scr + half, [&](int k) { return sc[k] < p; });
    for (uint32_t k = tid; k < s; k += FB) swap(scr[k], scr[half + k]);
    sync();
    if (tid == 0) swap(mid, a);
    sync();
    *already = s == 0;
    return mid;
  }
  __device__ int partition_equal(int a, int b, int pivot) {
    if (tid == 0) swap(a, pivot);
    sync();
    const uint16_t p = sc[a];
    uint32_t cnt = 0;
    for (int k = a + 1 + (int)tid; k < b; k += FB) cnt += sc[k] <= p;
    for (int m = 32; m >= 1; m >>= 1) cnt += (uint32_t)__shfl_xor((int)cnt, m);
    if (lane == 0) S.red[tog][wave] = cnt;
    sync();
    uint32_t neq = 0;
    for (int w = 0; w < NWAVE; w++) neq += S.red[tog][w];
    tog ^= 1;
    const int mid = a + (int)neq;
    const uint32_t s = compact(a + 1, mid + 1, false, scr, [&](int k) { return sc[k] > p; });
    compact(mid + 1, b, true, scr + half, [&](int k) { return sc[k] <= p; });
    for (uint32_t k = tid; k < s; k += FB) swap(scr[k], scr[half + k]);
    sync();
    return mid + 1;
  }
  // first k in [from,b) with sc[k] < sc[k-1]; b if none
  __device__ int first_inversion(int from, int b) {
    for (int base = from; base < b; base += FB) {
      const int k = base + (int)tid;
      const uint32_t hit = (k < b && sc[k] < sc[k - 1]) ? (uint32_t)k : INF;
      const uint32_t m = bmin(hit);
      if (m != INF) return (int)m;
    }
    return b;
  }
  __device__ bool partial_insertion_sort(int a, int b) {
    int i = a + 1;
    for (int j = 0; j < 5; j++) {
      i = first_inversion(i, b);
      if (i == b) return true;
      if (b - a < 50) return false;
      sync();
      if (tid == 0) swap(i, i - 1);
      sync();
      if (i - a >= 2) {
        // the smaller element (now at i-1) moves left past larger elements,
        // down to absolute index 0 (Go's loop runs to j >= 1)
        const uint16_t x = sc[i - 1];
        int q = -1;
        for (int top = i - 2; top >= 0; top -= FB) {
          const int k = top - (int)tid;
          const int32_t hit = (k >= 0 && sc[k] <= x) ? k : -1;
          const int32_t m = bmax(hit);
          if (m >= 0) {
            q = m;
            break;
          }
          if (top - FB < 0) break;
        }
        rotate_right(q + 1, i - 1);
      }
      if (b - i >= 2) {
        const uint16_t y = sc[i];
        int q = b;
        for (int base = i + 1; base < b; base += FB) {
          const int k = base + (int)tid;
          const uint32_t hit = (k < b && sc[k] >= y) ? (uint32_t)k : INF;
          const uint32_t m = bmin(hit);
          if (m != INF) {
            q = (int)m;
            break;
          }
        }
        rotate_left(i, q - 1);
      }
    }
    return false;
  }
  __device__ void reverse_range(int a, int b) {
    const int n = (b - a) / 2;
    for (int k = (int)tid; k < n; k += FB) swap(a + k, b - 1 - k);
    sync();
  }
  __device__ __forceinline__ void pdqsort_body(int n) {
    SeqSort seq{{sc, ord}};
    if (n <= SEQ) {
      if (tid == 0) seq.pdq_frame(Frame{0, n, bits_len((uint64_t)n), 1, 1});
      sync();
      return;
    }
    int sp = 0;
    Frame f{0, n, bits_len((uint64_t)n), 1, 1};
    for (;;) {
      for (;;) {
        const int length = f.b - f.a;
        if (length <= SEQ) {
          if (tid == 0) seq.pdq_frame(f);
          sync();
          break;
        }
        if (f.limit == 0) {
          if (tid == 0) seq.heap_sort(f.a, f.b);
          sync();
          break;
        }
        if (!f.wb) {
          if (tid == 0) seq.break_patterns(f.a, f.b);
          sync();
          f.limit--;
        }
        if (tid == 0) {
          int h;
          S.piv = seq.choose_pivot_fast(f.a, f.b, &h);
          S.hint = h;
        }
        sync();
        int pivot = S.piv, hint = S.hint;
        if (hint == 2) {
          reverse_range(f.a, f.b);
          pivot = (f.b - 1) - (pivot - f.a);
          hint = 1;
        }
        if (f.wb && f.wp && hint == 1) {
          if (partial_insertion_sort(f.a, f.b)) break;
        }
        sync();
        if (f.a > 0 && !(sc[f.a - 1] < sc[pivot])) {
          f.a = partition_equal(f.a, f.b, pivot);
          continue;
        }
        bool already;
        const int mid = partition(f.a, f.b, pivot, &already);
        f.wp = already;
        const int leftLen = mid - f.a, rightLen = f.b - mid;
        const int bal = length / 8;
        Frame child;
        if (leftLen < rightLen) {
          f.wb = leftLen >= bal;
          child = Frame{f.a, mid, f.limit, 1, 1};
          f.a = mid + 1;
        } else {
          f.wb = rightLen >= bal;
          child = Frame{mid + 1, f.b, f.limit, 1, 1};
          f.b = mid;
        }
        if (tid == 0) S.stk[sp] = f;
        sp++;
        f = child;
      }
      if (sp == 0) break;
      sync();
      sp--;
      f = S.stk[sp];
    }
    sync();
  }
};

// The generic sort's one out-of-line body (ROUND 6): the
// helper's fields arrive as scalar arguments with the LDS pointers
// LDS-qualified and the helper is rebuilt locally.  As a member function its
// `this` pointed at a per-lane copy in scratch: every workgroup stored the
// helper at start-up (~7 KB of the ~11.9 KB per-workgroup prologue writes of
// the simulation kernel, profiles/r5/sim_writes_per_wg.txt) and the sort's
// LDS accesses compiled to flat_* instructions.  Returns the reduction toggle.
template <uint32_t NT, int SEQ>
__device__ __noinline__ uint32_t blk_pdqsort(lds_u16* sc, lds_u16* ord, lds_u16* scr, __attribute__((address_space(3))) Shared* S,
                                             uint32_t tid, uint32_t tog, uint32_t half, int n) {
  Blk<NT, SEQ> b{(uint16_t*)sc, (uint16_t*)ord, (uint16_t*)scr, *(Shared*)S, tid, tid & 63u, tid >> 6, tog, half};
  b.pdqsort_body(n);
  return b.tog;
}


}  // namespace

// The kernel serves two launch shapes:
//  * SIM = false: ONE workgroup runs the provisioning Solve over all P pods;
//    existing nodes live in a global working copy (nodes / n_fk).
//  * SIM = true: a persistent grid, one consolidation simulation per
//    workgroup at a time (work counter d.sim_next).  A simulation re-Solves
//    its pod subset (pending pods + the candidates' pods, queue order) against
//    the existing nodes minus its candidates: the shared read-only base
//    nodes0 / n_fk0 plus an overlay of the nodes this simulation touched (LDS
//    bitmap + overlay ids, global req/FK copies per block).
// Waves per SIMD the SIM shapes are compiled for.  At 4 the register budget
// is 128 and the simulation loop spills (scratch traffic was 2/3 of the
// kernel's HBM bytes on C4); at 3 (168 registers) the narrow shape is
// spill-free.  The wide shape (few long simulations: MultiNode prefixes)
// runs at 2 (256 registers, no VGPR spills): round 5, same session, c4_multi
// 9.73 -> 8.03 ms at 2 (8.11 at 3, 4 before), c4_e2e_multi 2.06 -> 2.01
// (profiles/r5/sim_wide_wpe_ab.txt).
#ifndef GS_SIM_NARROW_WPE  // experiment builds: the narrow shape's waves per SIMD
#define GS_SIM_NARROW_WPE 3
#endif
#ifndef GS_SIM_WIDE_WPE  // experiment builds: the wide shape's waves per SIMD
#define GS_SIM_WIDE_WPE 2
#endif
constexpr int sim_waves_per_eu(uint32_t nt) { return nt <= (uint32_t)FB_SIM_NARROW ? GS_SIM_NARROW_WPE : GS_SIM_WIDE_WPE; }
constexpr uint32_t OV_EXCL = 0x80000000u;  // overlay entry of a removed (candidate) node
constexpr uint32_t OV_FK = 0x40000000u;    // the entry holds its own free-key state (copied on the first Add that needs it)

template <uint32_t RR, bool SIM, uint32_t NT, bool TOPO>
__global__ __launch_bounds__(NT, SIM ? sim_waves_per_eu(NT) : 1) void ffd_kernel(DevProblem d) {
  constexpr uint32_t FB = NT;  // threads of this workgroup
  extern __shared__ uint64_t lds64[];
  __shared__ Shared S;
  const uint32_t MC = d.max_claims;  // LDS claim capacity (SIM: the largest simulation's pod count)
  uint64_t* s_slk = lds64;      // 4x u16 quantized slack per claim (upper bound)
  uint64_t* s_rm = s_slk + MC;  // 4x u16 quantized room before a cursor moves (lower bound)
  uint16_t* s_ord = (uint16_t*)(s_rm + MC);
  uint16_t* s_sc = s_ord + MC;
  uint16_t* s_scr = s_sc + MC;
  uint8_t* s_tmpl = (uint8_t*)(s_scr + MC);
  // byte offset arithmetic keeps the pointer in the LDS address space (ds_read, not flat)
  int64_t* s_thr = (int64_t*)((char*)lds64 + ((23u * MC + 7u) & ~7u));
  __shared__ uint64_t s_tzm[TMAX], s_tcm[TMAX];
  __shared__ uint32_t s_thoff[RMAX + 1];
  const uint32_t tid = threadIdx.x;
  constexpr uint32_t R = RR;  // resource dimensions (= d.R), compile-time
  const uint32_t W = d.W, F = d.F, T = d.T;
  const uint32_t OW = d.OW;  // claim option stride (words, 16-B multiple)
  const uint32_t nthr = d.thr_off[R];
  const int64_t* thr = s_thr;  // gs_prepare refuses nthr > THR_LDS_MAX
  uint32_t* s_nb = (uint32_t*)((char*)lds64 + ((23u * MC + 7u) & ~7u) + (nthr + 4u) * 8u);  // SIM: touched nodes
  // SIM: a touched node's overlay entry (| OV_EXCL: a removed candidate), valid where its s_nb bit is set
  uint32_t* const ov_map = SIM ? d.ov_map + (size_t)blockIdx.x * d.NN : nullptr;
  // topology: known domains, per-pod minimum counts, zone counts, hostname totals
  const uint32_t tg_off = (((23u * MC + 7u) & ~7u) + (nthr + 4u) * 8u + d.nb_words * 4u + 7u) & ~7u;
  const TopoS ts = topo_lds((char*)lds64 + tg_off, d.TGZ, d.ZS, d.TGH, d.n_lazy);
  // SIM, small simulations: node -> overlay entry in an LDS hash (keys node + 1,
  // open addressing), after the topology state
  const uint32_t ovh = SIM ? d.ovh_slots : 0u, ovh_mask = ovh - 1u;
  uint32_t* const s_ovk = (uint32_t*)((char*)lds64 + ((tg_off + topo_lds_bytes(d.TGZ, d.ZS, d.TGH, d.n_lazy) + 7u) & ~7u));
  uint32_t* const s_ovv = s_ovk + ovh;
  // SIM with d.sim_lds: each simulation's queue, staleness (last epoch /
  // length), current variant and add log in LDS after the hash (4 x u32 +
  // 16 B per pod): none of them leaves the workgroup, so they cost no HBM
  // writes (those partial-line stores were most of a
  // simulation's write traffic)
  uint32_t* const s_simq = s_ovv + ovh;
  LogRec* const s_simlog = (LogRec*)(s_simq + 4u * MC);
  auto ovm_get = [&](uint32_t n) -> uint32_t {
    if (!ovh) return ov_map[n];
    uint32_t h = (n * 2654435761u) & ovh_mask;
    for (uint32_t i = 0; i < ovh; i++, h = (h + 1u) & ovh_mask)
      if (s_ovk[h] == n + 1u) return s_ovv[h];
    return OV_EXCL;  // unreachable: callers ask only for nodes the bitmap marks
  };
  auto ovm_put = [&](uint32_t n, uint32_t v) {  // one thread per node at a time
    if (!ovh) {
      ov_map[n] = v;
      return;
    }
    uint32_t h = (n * 2654435761u) & ovh_mask;
    for (uint32_t i = 0; i < ovh; i++, h = (h + 1u) & ovh_mask) {
      const uint32_t k = atomicCAS(&s_ovk[h], 0u, n + 1u);
      if (k == 0u || k == n + 1u) {
        s_ovv[h] = v;
        return;
      }
    }
  };
  Blk<NT> blk{s_sc, s_ord, s_scr, S, tid, tid & 63, tid >> 6, 0, MC / 2};
  Wg<NT> wg{&S.red2[0][0], s_sc, s_ord, tid, tid & 63, tid >> 6, 0};

  for (uint32_t i = tid; i < nthr + 4; i += FB) s_thr[i] = i < nthr ? d.thr_val[i] : INT64_MAX;
  __shared__ uint64_t s_slot[SLOT_LDS_MAX];
  const uint32_t nslot = d.Z * d.C * W;
  const uint64_t* slot = s_slot;  // gs_prepare refuses Z*C*W > SLOT_LDS_MAX
  for (uint32_t i = tid; i < nslot; i += FB) s_slot[i] = d.slot_set[i];
  if (!SIM) {
    for (uint32_t i = tid; i < d.NN; i += FB) d.nodes[i] = d.nodes0[i];
    for (uint32_t i = tid; i < d.NN * F; i += FB) d.n_fk[i] = d.n_fk0[i];
    if (d.any_vol)
      for (uint32_t i = tid; i < d.NN; i += FB) d.n_vol[i] = d.n_vol0[i];
  }
  if (tid <= R) s_thoff[tid] = d.thr_off[tid];
  for (uint32_t t = tid; t < T; t += FB) {
    s_tzm[t] = d.tmpl[t].zm;
    s_tcm[t] = d.tmpl[t].cm;
  }
  const uint32_t wave = tid >> 6, lane = tid & 63;

  // SIM, thread 0: this workgroup's sums of its simulations' counters
  uint64_t b_pops = 0, b_gen = 0, b_fast = 0, b_cand = 0, b_full = 0, b_nev = 0, b_npre = 0, b_cpre = 0;
  for (uint32_t iter = 0;; iter++) {
    // ------------------------------------------------ next simulation (SIM)
    if (tid == 0) S.sim = SIM ? atomicAdd(d.sim_next, 1u) : iter;
    __syncthreads();
    const uint32_t sim = S.sim;
    if (sim >= (SIM ? d.n_sims : 1u)) break;  // block-uniform: every wave leaves
    const uint32_t qoff = SIM ? d.sim_pod_off[sim] : 0u;
    // SIM: this simulation's overlay stamp (launch epoch, simulation)
    const uint32_t ov_stamp = (d.ov_epoch << 20) | (sim + 1u);
    const uint32_t P = SIM ? d.sim_pod_off[sim + 1] - qoff : d.P;
    const uint32_t MCs = SIM ? P : MC;  // claim arena of this solve (one claim per pod at most)
    const bool qlds = SIM && d.sim_lds;
    uint32_t* const queue = qlds ? s_simq : d.queue + qoff;
    uint32_t* const last_len = qlds ? s_simq + MC : d.last_len + qoff;
    uint32_t* const last_epoch = qlds ? s_simq + 2u * MC : d.last_epoch + qoff;
    uint32_t* const cur_var = qlds ? s_simq + 3u * MC : d.cur_var + qoff;
    LogRec* const logp = qlds ? s_simlog : d.log + qoff;
    int64_t* const t_rem = d.t_rem + (SIM ? (size_t)sim * T * R : 0);
    auto gpod = [&](uint32_t local) -> uint32_t { return SIM ? d.sim_pods[qoff + local] : local; };

    for (uint32_t i = tid; i < P; i += FB) {
      queue[i] = SIM ? i : d.queue0[i];  // simulation pods are listed in queue order
      last_epoch[i] = 0;
      last_len[i] = 0;
      cur_var[i] = d.var_begin[gpod(i)];
    }
    for (uint32_t i = tid; i < T * R; i += FB) t_rem[i] = d.tmpl[i / R].limits[i % R];
    if (TOPO) {
      // <U> Topology: counts before the Solve (selected bound pods); a
      // simulation knows the zones of the nodes it keeps (and the NodePools')
      topo_init(d, ts, SIM ? d.sim_known[sim] : d.zknown0, tid, FB);
      if (!SIM)
        for (uint32_t i = tid; i < d.TGH * d.NN; i += FB) d.hn[i] = d.hn0[i];
    }
    uint32_t ncand = 0;
    if (SIM) {
      const uint32_t c0 = d.sim_cand_off[sim];
      ncand = d.sim_cand_off[sim + 1] - c0;
      for (uint32_t i = tid; i < d.nb_words; i += FB) s_nb[i] = 0;
      for (uint32_t i = tid; i < ovh; i += FB) s_ovk[i] = 0;
      __syncthreads();
      for (uint32_t k = tid; k < ncand; k += FB) {
        const uint32_t n = d.sim_cands[c0 + k];
        ovm_put(n, k | OV_EXCL);
        atomicOr(&s_nb[n >> 5], 1u << (n & 31));
      }
      if (TOPO) {
        // SimulateScheduling reschedules the candidates' pods: Topology
        // excludes them from the counts (excludedPods)
        for (uint32_t k = 0; k < ncand && d.nsp_off; k++) {
          const uint32_t n = d.sim_cands[c0 + k], e0 = d.nsp_off[n], e1 = d.nsp_off[n + 1];
          for (uint32_t x = e0 + tid; x < e1; x += FB) {
            const uint64_t en = d.nsp[x];
            const uint32_t g = (uint32_t)(en >> 32);
            const int32_t c = (int32_t)(uint32_t)en;
            if (g < d.TGZ) {
              const uint32_t z = d.nodes0[n].dvid;
              if (z < d.ZS) atomicSub(&ts.zcnt[g * d.ZS + z], c);
            } else {
              atomicSub(&ts.htot[g - d.TGZ], c);
            }
          }
        }
      }
    }
    if (tid == 0) {
      S.hb[0].M = 0;
      S.hb[0].qhead = 0;
      S.hb[0].qlen = P;
      S.hb[0].epoch = 1;
      S.hb[0].modkind = MOD_NONE;
      S.hb[0].nlog = 0;
      S.nov = ncand;
      S.qoff = qoff;
      S.hb[0].pops = S.generic = S.fast = S.cand = S.cand_full = S.node_evals = S.node_prefix = S.claim_prefix = 0;
      S.failed = 0;
      S.t_sort = S.t_scan = S.t_tmpl = 0;
      for (int q = 0; q < 16; q++) S.dbg[q] = S.tl[q] = 0;
      S.tl_last = __builtin_amdgcn_s_memtime();
      S.t0 = wall_clock64();
      S.dbg[7] = __builtin_amdgcn_s_memtime();
      S.hb[0].status = 0;
      S.hb[0].nx_valid = 0;
      S.hb[0].cb = 0;
      S.hb[0].wrapped = 0;
    }
    __syncthreads();
    const uint64_t max_pops = ((uint64_t)(d.V - d.P) + 2) * (uint64_t)P + P + 16;
    // per-wave copy of the uniform state; par: the buffer this pod reads
    Hot h = S.hb[0];
    uint32_t par = 1;

    uint64_t tLoop = 0;
    // wave-1 prefetch registers: stage 0 none, 1 pod id, 2 counters+variant, 3 records
    uint32_t pf_state = 0, pf_pod = 0, pf_gp = 0, pf_le = 0, pf_ll = 0, pf_cv = 0, pf_vr = 0, pf_rq = 0;
    auto pf_stage2 = [&]() {
      if (wave == 1 && lane == 0 && pf_state == 1) {
        pf_le = last_epoch[pf_pod];
        pf_ll = last_len[pf_pod];
        pf_cv = cur_var[pf_pod];
        pf_gp = gpod(pf_pod);
        pf_state = 2;
      }
    };
    auto pf_stage3 = [&]() {
      if (wave == 1) {
        const uint32_t st = __builtin_amdgcn_readfirstlane(pf_state);
        if (st == 2) {
          const uint32_t cv = __builtin_amdgcn_readfirstlane(pf_cv), gp = __builtin_amdgcn_readfirstlane(pf_gp);
          if (lane < VR_DW) pf_vr = ((const uint32_t*)(d.vars + cv))[lane];
          if (lane >= 32 && lane < 32 + 2 * RR) pf_rq = ((const uint32_t*)(d.pod_req + (size_t)gp * R))[lane - 32];
          pf_state = 3;
        }
      }
    };
    for (;;) {
      TL(0);  // end of the previous pod -> loop top
      par ^= 1u;
      Hot& HN = S.hb[par ^ 1u];  // thread 0 writes this pod's changes here
      // publish last iteration's prefetch into the spare buffer
      if (wave == 1) {
        const uint32_t st = __builtin_amdgcn_readfirstlane(pf_state);
        if (st == 3 || st == 4) {
          const uint32_t nb = h.cb ^ 1u;  // the buffer the current pod does not use
          if (lane < VR_DW) S.vrb[nb][lane] = pf_vr;
          if (lane >= 32 && lane < 32 + 2 * RR) ((uint32_t*)S.reqb[nb])[lane - 32] = pf_rq;
          // first-pass records carry their pod and variant ids; such a pod
          // was never pushed (last epoch / length 0)
          const uint32_t rpod = __builtin_amdgcn_readfirstlane(pf_vr), rvix = __builtin_amdgcn_readlane(pf_vr, VR_DW - 1);
          if (lane == 0) {
            S.hb[par].nx_valid = 1;
            S.hb[par].nx_pod = st == 4 ? rpod : pf_pod;
            S.hb[par].nx_gp = st == 4 ? rpod : pf_gp;
            S.hb[par].nx_le = st == 4 ? 0u : pf_le;
            S.hb[par].nx_ll = st == 4 ? 0u : pf_ll;
            S.hb[par].nx_cv = st == 4 ? rvix : pf_cv;
          }
        } else if (lane == 0) {
          S.hb[par].nx_valid = 0;
        }
        pf_state = 0;
      }
#ifdef GS_FFD_TL
      if (lane == 0) S.tl_arr[wave] = __builtin_amdgcn_s_memtime();
#endif
      __syncthreads();
#ifdef GS_FFD_TL
      if (tid == 0) {
        // the last wave to arrive and how much later than wave 0 it came
        uint64_t last = S.tl_arr[0];
        uint32_t lw = 0;
        for (uint32_t w = 1; w < (uint32_t)(FB / 64); w++)
          if (S.tl_arr[w] > last) {
            last = S.tl_arr[w];
            lw = w;
          }
        S.tl[11] += last - S.tl_arr[0];
        S.tl[12 + (lw < 3 ? lw : 3)]++;
      }
#endif
      TL(1);  // publish + barrier
      // ------------------------------------------------------------ Queue.Pop
      // computed identically by every wave from one read of the uniform state
      if (tid == 0) {
        tLoop = phase_clock();
        if (S.dbg[14]) S.dbg[5] += tLoop - S.dbg[14];  // iteration end -> pop (prefetch publish)
      }
      h = S.hb[par];
      h.qhead = __builtin_amdgcn_readfirstlane(h.qhead);
      h.qlen = __builtin_amdgcn_readfirstlane(h.qlen);
      h.epoch = __builtin_amdgcn_readfirstlane(h.epoch);
      h.M = __builtin_amdgcn_readfirstlane(h.M);
      h.modkind = __builtin_amdgcn_readfirstlane(h.modkind);
      h.modpos = __builtin_amdgcn_readfirstlane(h.modpos);
      h.nlog = __builtin_amdgcn_readfirstlane(h.nlog);
      h.cb = __builtin_amdgcn_readfirstlane(h.cb);
      h.wrapped = __builtin_amdgcn_readfirstlane(h.wrapped);
      h.status = __builtin_amdgcn_readfirstlane(h.status);
      h.pops = (uint64_t)uniform_i64((int64_t)h.pops);
      bool stop = false, pf = false;
      uint32_t p = 0, gp = 0, v = 0;
      if (h.status) {
        stop = true;  // set by a NodeClaim update of the previous pod
      } else if (h.pops > max_pops) {
        h.status = 2;
        stop = true;
      } else if (h.qlen == 0) {
        stop = true;
      } else {
        uint32_t le, ll;
        pf = __builtin_amdgcn_readfirstlane(h.nx_valid) != 0;
        if (pf) {
          p = __builtin_amdgcn_readfirstlane(h.nx_pod);
          gp = __builtin_amdgcn_readfirstlane(h.nx_gp);
          le = __builtin_amdgcn_readfirstlane(h.nx_le);
          ll = __builtin_amdgcn_readfirstlane(h.nx_ll);
          v = __builtin_amdgcn_readfirstlane(h.nx_cv);
        } else {
          p = __builtin_amdgcn_readfirstlane(queue[h.qhead]);
          gp = __builtin_amdgcn_readfirstlane(gpod(p));
          le = __builtin_amdgcn_readfirstlane(last_epoch[p]);
          ll = __builtin_amdgcn_readfirstlane(last_len[p]);
          v = __builtin_amdgcn_readfirstlane(cur_var[p]);
        }
        if (le == h.epoch && ll == h.qlen) {
          stop = true;
        } else {
          if (h.qhead + 1 == P) h.wrapped = 1;
          h.qhead = h.qhead + 1 == P ? 0 : h.qhead + 1;
          h.qlen--;
          h.pops++;
          if (pf) h.cb ^= 1u;
        }
      }
      if (tid == 0) {
        HN.qhead = h.qhead;
        HN.qlen = h.qlen;
        HN.epoch = h.epoch;
        HN.M = h.M;
        HN.modkind = h.modkind;
        HN.modpos = h.modpos;
        HN.nlog = h.nlog;
        HN.cb = h.cb;
        HN.wrapped = h.wrapped;
        HN.status = h.status;
        HN.pops = h.pops;
        S.found = 0;
      }
      TL(2);  // pop
      if (stop) break;
      if (!pf) {
        // not prefetched: wave 0 stages the variant record and requests in LDS
        if (wave == 0) {
          if (lane < VR_DW) S.vrb[h.cb][lane] = ((const uint32_t*)(d.vars + v))[lane];
          if (lane >= 32 && lane < 32 + 2 * RR)
            ((uint32_t*)S.reqb[h.cb])[lane - 32] = ((const uint32_t*)(d.pod_req + (size_t)gp * R))[lane - 32];
        }
        __syncthreads();
      }
      const VarRec& vr = *(const VarRec*)S.vrb[h.cb];
      const int64_t* preq = S.reqb[h.cb];
      // stage 1: the next pod id (its queue slot cannot change during this pod
      // unless the queue is empty now, when this pod itself may come back)
      if (wave == 1 && h.qlen > 0) {
        if (!SIM && !h.wrapped) {
          // first pass: the next pod is queue0[qhead] with its first variant,
          // its records are contiguous in queue order: one round trip
          const uint32_t k = h.qhead;
          if (lane < VR_DW) pf_vr = ((const uint32_t*)(d.qvars + k))[lane];
          if (lane >= 32 && lane < 32 + 2 * RR) pf_rq = ((const uint32_t*)(d.qreqs + (size_t)k * R))[lane - 32];
          pf_state = 4;
        } else if (lane == 0) {
          pf_pod = queue[h.qhead];
          pf_state = 1;
        }
      }
      const uint32_t M = h.M;
      uint64_t tA = 0;
      if (tid == 0) {
        tA = phase_clock();
        S.dbg[4] += tA - tLoop;  // pop + variant load
      }

      int64_t rq[RR];
#pragma unroll
      for (uint32_t r = 0; r < RR; r++) rq[r] = r < R ? uniform_i64(preq[r]) : 0;

      // <U> Topology.AddRequirements, per pod: the minimum domain count of every
      // zone group the pod owns over its strict zone domains (domainMinCount)
      // topology: the groups the pod owns (own list) and that count it (selection list)
      const uint32_t own_n = TOPO ? vr.own_n : 0u, own_off = TOPO ? vr.own_off : 0u;
      const uint32_t sel_n = TOPO ? vr.sel_n : 0u, sel_off = TOPO ? vr.sel_off : 0u;
      // the owned groups staged in LDS (the topology checks of every node /
      // NodeClaim candidate read them there instead of two dependent loads)
      __shared__ OwnG s_own[OWNMAX];
      if (TOPO && own_n) {
        if (tid < own_n) s_own[tid] = OwnMem<DevProblem>{d, own_off}(tid);
        if (tid < 64 && (vr.ctb & VF_ZSPREAD)) topo_tmin(d, ts, own_off, own_n, vr.zs, tid);
        __syncthreads();
      }
      auto OWN = [&](uint32_t k) -> OwnG { return s_own[k]; };

      // --------------- existing nodes in order: first ExistingNode.CanAdd wins
      if (d.NN) {
        // first-fit: a 64-node window first (the common hit), then full-width
        // chunks; every chunk ends in one block min over node positions
        // <U> VolumeUsage: the pod's pending-volume bits per CSI driver
        uint64_t pvol[VDMAX] = {0, 0, 0, 0};
        uint32_t pfresh[VDMAX] = {0, 0, 0, 0};
        if (TOPO && d.any_vol)
#pragma unroll
          for (uint32_t q = 0; q < VDMAX; q++) {
          pvol[q] = d.pod_vol[(size_t)gp * VDMAX + q];
          pfresh[q] = d.pod_vfresh[(size_t)gp * VDMAX + q];
        }
        uint32_t fn = INF;
        for (uint32_t base = 0, width = 64; base < d.NN; base += width, width = FB) {
          const uint32_t n = base + tid;
          bool feas = false;
          if (tid < width && n < d.NN) {
            const NodeRec& nr = SIM ? d.nodes0[n] : d.nodes[n];
            const int64_t* nreq = nr.req;
            const FK* nfk = (SIM ? d.n_fk0 : d.n_fk) + (size_t)n * F;
            feas = nr.ok && (nr.taints & ~vr.tol) == 0;  // Taints.ToleratesPod
            size_t oe = ~(size_t)0;  // SIM: the node's overlay entry (hostname counts, volume usage)
            if (SIM && feas && ((s_nb[n >> 5] >> (n & 31)) & 1)) {
              // touched by this simulation: removed candidate, or overlay copy
              const uint32_t e = ovm_get(n);
              if (e & OV_EXCL) {
                feas = false;
              } else {
                oe = (size_t)blockIdx.x * d.ov_cap + (e & ~OV_FK);
                nreq = d.ov_req + oe * RMAX;
                if (e & OV_FK) nfk = d.ov_fk + oe * F;  // else the node's base free-key state still holds
              }
            }
#pragma unroll
            for (uint32_t r = 0; r < RR; r++)
              feas = feas && (r >= R || nreq[r] + rq[r] <= nr.avail[r]);  // Fits(requests, available)
            // strict Compatible on label keys: the node's label value must be Has()
            for (uint32_t k = 0; k < d.K && feas; k++) {
              const uint32_t off = vr.itmask_off[k];
              if (off == NONE) continue;
              const uint32_t vid = nr.vid[k];
              feas = vid != NONE && ((d.itmask[off + (vid >> 6)] >> (vid & 63)) & 1);
            }
            if (feas && vr.zfull_off != NONE)
              feas = nr.zvid != NONE && ((d.itmask[vr.zfull_off + (nr.zvid >> 6)] >> (nr.zvid & 63)) & 1);
            if (feas && vr.cfull_off != NONE)
              feas = nr.cvid != NONE && ((d.itmask[vr.cfull_off + (nr.cvid >> 6)] >> (nr.cvid & 63)) & 1);
            if (feas && vr.fk_count) feas = var_fk_ok_strict(d, vr, nfk);
            if (TOPO && feas && own_n)
              feas = topo_node_ok_g(d, ts, own_n, nr.dvid, [&](uint32_t hs) -> int64_t {
                if (!SIM) return d.hn[(size_t)hs * d.NN + n];
                // an overlay cell counts only where this simulation wrote it
                // (its stamp); other groups keep the node's base count
                if (oe != ~(size_t)0) {
                  const uint64_t x = d.ov_hn[oe * d.TGH + hs];
                  if ((uint32_t)(x >> 32) == ov_stamp) return (int32_t)(uint32_t)x;
                }
                return d.hn0[(size_t)hs * d.NN + n];
              }, OWN);
            if (TOPO && feas && d.any_vol) {
              // ExceedsLimits: distinct volumes per driver after the union
              const NodeVol& nv = !SIM ? d.n_vol[n] : oe != ~(size_t)0 ? d.ov_vol[oe] : d.n_vol0[n];
#pragma unroll
              for (uint32_t q = 0; q < VDMAX; q++)
                if (pvol[q] | pfresh[q]) feas = feas && nv.cnt[q] + (int32_t)pfresh[q] + __popcll(pvol[q] & ~nv.present) <= nv.lim[q];
            }
          }
          fn = wg.first(feas, base);
          if (tid == 0) S.node_evals += d.NN - base < width ? d.NN - base : width;
          if (fn != INF) break;
        }
        if (tid == 0) S.node_prefix += fn != INF ? fn + 1 : d.NN;
        if (fn != INF) {
          // ExistingNode.Add: requests and requirements
          int64_t* areq;
          FK* afk;
          int32_t* ahn = nullptr;   // the node's hostname counts (row stride ahs)
          size_t ahs = 0;
          NodeVol* avol = nullptr;  // the node's volume usage
          size_t ovx = 0;           // SIM: the node's overlay entry
          if (SIM) {
            // copy-on-write overlay entry for the node
            if (tid == 0) {
              uint32_t e = INF;
              if ((s_nb[fn >> 5] >> (fn & 31)) & 1) {
                e = ovm_get(fn);  // a kept node (the scan rejects removed ones)
                S.ov_new = 0;
              } else {
                e = S.nov++;
                ovm_put(fn, e);
                s_nb[fn >> 5] |= 1u << (fn & 31);
                S.ov_new = 1;
              }
              S.ove = e & ~OV_FK;
              S.ov_fk = (e & OV_FK) != 0;
              // a pod with free-key requirements narrows the node's state: the
              // entry takes its own copy now (below) and keeps it
              if (vr.fk_count && !(e & OV_FK)) ovm_put(fn, e | OV_FK);
            }
            __syncthreads();
            const size_t oe = (size_t)blockIdx.x * d.ov_cap + S.ove;
            ovx = oe;
            areq = d.ov_req + oe * RMAX;
            afk = d.ov_fk + oe * F;
            if (TOPO) avol = d.ov_vol + oe;
            if (S.ov_new) {
              if (tid < R) areq[tid] = d.nodes0[fn].req[tid];
              if (TOPO && d.any_vol && tid == FB - 1) *avol = d.n_vol0[fn];
            }
            if (vr.fk_count && !S.ov_fk && tid >= 64 && tid < 64 + F) afk[tid - 64] = d.n_fk0[(size_t)fn * F + (tid - 64)];
            __syncthreads();
          } else {
            areq = d.nodes[fn].req;
            afk = d.n_fk + (size_t)fn * F;
            ahn = d.hn + fn;
            ahs = d.NN;
            avol = d.n_vol + fn;
          }
          if (tid < R) areq[tid] += preq[tid];
          if (tid >= 64 && tid < 64 + vr.fk_count) {
            const FKEntry& e = d.fk_entries[vr.fk_begin + (tid - 64)];
            FK* nf = afk + e.slot;
            const FK cur = *nf;
            *nf = (cur.flags & FK_PRESENT) ? fk_intersect(cur, e.st, d.fk_ival + (size_t)e.slot * FKV, d.fk_isint + (size_t)e.slot * FKW)
                                           : e.st;
          }
          if (tid == 0) {
            if (TOPO && d.any_vol) {
              // VolumeUsage.Add
              NodeVol& nv = *avol;
              uint64_t all = 0;
#pragma unroll
              for (uint32_t q = 0; q < VDMAX; q++) {
                nv.cnt[q] += (int32_t)pfresh[q] + __popcll(pvol[q] & ~nv.present);
                all |= pvol[q];
              }
              nv.present |= all;
            }
            logp[HN.nlog++] = LogRec{gp, v, fn | 0x80000000u, 0};
            S.found = 1;
            // <U> Topology.Record: the node's labels are single domains
            if (TOPO && sel_n) {
              const uint32_t z = d.nodes0[fn].dvid;
              topo_record(d, ts, sel_off, sel_n, z < 64u ? 1ull << z : 0ull, 0u, [&](uint32_t hs) {
                if (SIM) {
                  // copy-on-write per group: the first count this simulation
                  // writes takes the node's base (a cell without its stamp)
                  uint64_t* cell = d.ov_hn + ovx * d.TGH + hs;
                  const uint64_t x = *cell;
                  const int32_t cnt = ((uint32_t)(x >> 32) == ov_stamp ? (int32_t)(uint32_t)x : d.hn0[(size_t)hs * d.NN + fn]) + 1;
                  *cell = ((uint64_t)ov_stamp << 32) | (uint32_t)cnt;
                } else {
                  ahn[(size_t)hs * ahs]++;
                }
              });
            }
          }
          pf_stage2();
          pf_stage3();
          __syncthreads();
          continue;
        }
      }

      TL(3);  // variant staging, prefetch issue, existing nodes
      // ------------------------- sort.Slice(newNodeClaims, len(Pods) asc)
      if (M > 1) {
        // the decision, identical in every wave: at most one NodeClaim changed
        // since the last sort (one pod added at modpos, or one appended)
        constexpr uint32_t FP_SMALL = 8, FP_GENERIC = 16;
        const uint32_t mk = h.modkind, q = h.modpos;
        bool inversion = false;
        if (mk == MOD_INC) inversion = q + 1 < M && s_sc[q + 1] < s_sc[q];
        else if (mk == MOD_APPEND) inversion = s_sc[M - 2] > s_sc[M - 1];
        inversion = __builtin_amdgcn_readfirstlane(inversion ? 1u : 0u) != 0;
        uint32_t fp = 0, rlo = 0, rhi = 0;
        if (!inversion) {
          // sorted input: pdqsort_func / insertionSort leave it untouched
        } else if (M <= 12) {
          fp = FP_SMALL;
        } else if (pivot_hint_wave(SplitAcc{s_sc, s_ord}, (int)M, lane) == 1 && M >= 50) {
          // partialInsertionSort fixes the single inversion: one
          // rotation; its far end by a 64-ary search over the sorted remainder
          // (INC: first k > q with count >= x; APPEND: first k < M-1 with
          // count > x)
          fp = mk;
          if (mk == MOD_INC) {
            const uint16_t x = s_sc[q];
            const uint32_t lo = wave_first(q + 1, M, lane, [&](uint32_t k) { return s_sc[k] >= x; });
            rlo = q;
            rhi = lo - 1;
          } else {
            const uint16_t x = s_sc[M - 1];
            rlo = wave_first(0, M - 1, lane, [&](uint32_t k) { return s_sc[k] > x; });
            rhi = M - 1;
          }
        } else {
          fp = FP_GENERIC;
        }
        h.modkind = MOD_NONE;
        if (tid == 0) {
          if (fp == MOD_INC || fp == MOD_APPEND) S.fast++;
          if (fp == FP_GENERIC) S.generic++;
          HN.modkind = MOD_NONE;
          const uint64_t tq = phase_clock();
          S.dbg[3] += tq - tA;
        }
        TL(4);  // sort decision
        if (fp == FP_SMALL || fp == FP_GENERIC) __syncthreads();  // every wave has decided before the order changes
        if (fp == FP_SMALL) {
          if (tid == 0) {
            SeqSort ss{{s_sc, s_ord}};
            ss.insertion_sort(0, (int)M);
          }
        } else if ((fp == MOD_INC || fp == MOD_APPEND) && wg.rotate1((int)rlo, (int)rhi, fp == MOD_INC)) {
          // done: one staged rotation
        } else if (fp == MOD_INC) {
          // X (at q, count x) moves right past the run of counts < x
          const uint32_t x = s_sc[q];
          uint32_t e = M;
          for (uint32_t base = q + 1; base < M; base += FB) {
            const uint32_t k = base + tid;
            const uint32_t m = blk.bmin((k < M && s_sc[k] >= x) ? k : INF);
            if (m != INF) {
              e = m;
              break;
            }
          }
          blk.rotate_left((int)q, (int)e - 1);
        } else if (fp == MOD_APPEND) {
          // X (at M-1, count x) moves left past the counts > x
          const uint16_t x = s_sc[M - 1];
          int e = 0;
          for (int top = (int)M - 2; top >= 0; top -= FB) {
            const int k = top - (int)tid;
            const int32_t m = blk.bmax((k >= 0 && s_sc[k] <= x) ? k : -1);
            if (m >= 0) {
              e = m + 1;
              break;
            }
          }
          blk.rotate_right(e, (int)M - 1);
        } else if (fp == FP_GENERIC) {
          blk.tog = blk_pdqsort<NT, SEQ_SORT>((lds_u16*)s_sc, (lds_u16*)s_ord, (lds_u16*)s_scr,
                                             (__attribute__((address_space(3))) Shared*)&S, tid, blk.tog, blk.half, (int)M);
        }
        if (fp) __syncthreads();  // the new order before the scan reads it
        TL(5);  // rotation / pdqsort + barrier
      }
      if (tid == 0) {
        const uint64_t tB = phase_clock();
        S.t_sort += tB - tA;
        tA = tB;
      }

      pf_stage2();
      // request codes for the LDS slack test (computed here: not live across the sort)
      uint32_t rqq[4], rqc[4];
#pragma unroll
      for (uint32_t r = 0; r < 4; r++) {
        rqq[r] = r < d.RQ ? qcode_floor(rq[r]) : 0;
        rqc[r] = r < d.RQ ? qcode_ceil(rq[r]) : 0;
      }
      // fast accept (simple pods): NodeClaim.Add changes only the requests, so
      // a claim whose threshold cursors do not move keeps its (non-empty)
      // options -- CanAdd holds without reading the claim (room test in LDS)
#ifdef GS_NO_FAST
      bool simple = false;
#else
      bool simple = !TOPO && (vr.ctb & VF_SIMPLE);
#endif
#pragma unroll
      for (uint32_t r = 4; r < RR; r++) simple = simple && rq[r] == 0;  // room covers resources 0..3
      // ---------------------- in-flight NodeClaims, first that CanAdd wins
      // A lane that finds its NodeClaim feasible keeps everything NodeClaim.Add
      // needs in registers (new option words for W <= WREG, totals, cursors);
      // the first feasible position (block min) writes them back directly.
      uint32_t f = INF;
      for (uint32_t base = 0; base < M; base += FB) {
        // kernel arguments re-read per chunk (scalar loads) instead of being
        // held across the whole pod loop: keeps SGPR spills out of this path
        KArg dpp = (KArg)__builtin_amdgcn_kernarg_segment_ptr();  // d is the only argument
        asm volatile("" : "+s"(dpp));
        const auto& dd = *dpp;
        const uint32_t cb = SIM ? S.qoff : 0u;  // this solve's claim arena
        const uint32_t pos = base + tid;
        bool feas = false, pre = false;
        uint32_t j = 0, t = 0;
        uint64_t G = 0, Gt = 0;
        uint64_t zm = 0, cm = 0;  // the NodeClaim's catalog zone / capacity-type masks
        uint64_t zset = ~0ull;  // zone domains topology allows on this NodeClaim (~0: unconstrained)
        uint64_t czf = 0;    // the NodeClaim's zone Has / flags (read only under topology)
        uint32_t czfl = 0;
        uint32_t mrow[RR];
        int64_t tot[RR];
        uint64_t nx[WREG];
#ifdef GS_FFD_DIAG
        const uint64_t c0 = __builtin_amdgcn_s_memtime();
        uint64_t c1 = 0, c2 = 0, c3 = 0;
#endif
        bool lp = false, fa = false;
        if (pos < M) {
          j = s_ord[pos];
          t = s_tmpl[j];
          // LDS-only necessary test: template tolerated and, per resource,
          // qcode_floor(request) <= qcode_ceil(slack)
          lp = (vr.tolt >> t) & 1;
          const uint64_t sq = s_slk[j];
#pragma unroll
          for (uint32_t r = 0; r < 4; r++) lp = lp && (uint64_t)rqq[r] <= ((sq >> (16 * r)) & 0xFFFFu);
          if (simple && lp) {
            // LDS-only sufficient test: qcode_ceil(request) <= qcode_floor(room)
            const uint64_t rm = s_rm[j];
            fa = true;
#pragma unroll
            for (uint32_t r = 0; r < 4; r++) fa = fa && (uint64_t)rqc[r] <= ((rm >> (16 * r)) & 0xFFFFu);
          }
        }
        // simple pods: the first fast-accept position and the first position
        // that needs the exact check, in one reduction; the exact checks run
        // only before the first fast accept (usually none)
        TL(6);
        uint32_t mfa = INF;
        bool skip_full = false;
        uint4 ph0 = make_uint4(0, 0, 0, 0), ph1 = ph0, ph3 = ph0;
        if (simple) {
          const uint64_t fam = __ballot(fa);
          if (fa && (tid & 63) == (uint32_t)(__ffsll((long long)fam) - 1)) {
            // the wave's first fast accept reads its requests now: if it wins,
            // the update needs no further round trip
            const uint4* q = (const uint4*)(dd.c_rec + cb + j);
            ph0 = q[0];
            ph1 = q[1];
            ph3 = q[3];
          }
          const uint2 m2 = wg.first2(fa, lp && !fa, base);
          mfa = m2.x;
          skip_full = m2.y == INF || (m2.x != INF && m2.y > m2.x);
        }
        TL(7);
        if (pos < M) {
          if (lp && !fa && !skip_full && pos < mfa) {
#ifdef GS_ASM_MARK
            asm volatile("; MARK_FULL_BEGIN");
#endif
            // one 64-B header read (four 16-B loads): totals, cursors, masks
            const ClaimRec* cr = dd.c_rec + cb + j;
            uint32_t cur[RR];
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
            // option words (stride OW, 16-B aligned) and the (variant, template)
            // row: they depend only on j and t, issued with the header
            const uint64_t* row = dd.rows + ((size_t)v * T + t) * OW;
            const uint64_t* opts = dd.c_opts + (size_t)(cb + j) * OW;
            if (W <= WREG) {
              // unconditional 16-B loads (stride OW >= 4 words): no per-word branches
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
            // the exact fit test is implied by the threshold rows below; the
            // LDS slack test above already rejected the clear misfits
            pre = true;
#ifdef GS_FFD_DIAG
            c1 = __builtin_amdgcn_s_memtime();
#endif
            if (pre && vr.fk_count) pre = var_fk_ok(dd, vr, dd.c_fk + (size_t)(cb + j) * F);
            if (TOPO && pre && own_n) {
              // <U> Topology.AddRequirements on the NodeClaim over its (claim
              // AND pod) zone domains; hostname groups: this NodeClaim's counts
              czf = cr->zfull;
              czfl = cr->zflags;
              const int32_t* hrow = dd.hc + (size_t)(cb + j) * dd.TGH;
              zset = topo_claim_g(dd, ts, own_n, czf & vr.zn, [&](uint32_t hs) -> int64_t { return hrow[hs]; }, OWN);
              pre = zset != 0;
              if (pre && zset != ~0ull) {
                // the domains narrow the catalog zones, or (dom_ct) capacity types
                const uint64_t dcat = topo_catmask(dd, zset);
                if (dd.dom_ct) cm &= dcat;
                else if (!dd.dom_np) zm &= dcat;
              }
            }
            if (pre) {
              G = grid_of(zm & vr.zm, cm & vr.cm, dd.Z, dd.C);
              Gt = grid_of(s_tzm[t] & vr.zm, s_tcm[t] & vr.cm, dd.Z, dd.C);
              uint32_t mm[RR];
#pragma unroll
              for (uint32_t r = 0; r < RR; r++) {
                const uint32_t o = s_thoff[r], n = s_thoff[r + 1] - o;
                mm[r] = thr_window(thr + o, n, cur[r], tot[r] + rq[r]);
              }
#pragma unroll
              for (uint32_t r = 0; r < RR; r++) {
                const uint32_t o = s_thoff[r], n = s_thoff[r + 1] - o;
                if (mm[r] == cur[r] + 4 && mm[r] < n) mm[r] = thr_search(thr + o, n, mm[r], tot[r] + rq[r]);
                mrow[r] = o + r + mm[r];
              }
#ifdef GS_FFD_DIAG
              c2 = __builtin_amdgcn_s_memtime();
#endif
              uint64_t acc = 0;
              if (W <= WREG) {
                // opts ⊆ thr_set[cur] (invariant of every Add): only a resource
                // whose cursor moves narrows the options further
#pragma unroll
                for (uint32_t r = 0; r < RR; r++) {
                  if (mm[r] != cur[r]) {
                    const uint4* tq = (const uint4*)(dd.thr_set + (size_t)mrow[r] * OW);
                    const uint4 t0 = tq[0], t1 = tq[1];
                    nx[0] &= ((uint64_t)t0.y << 32) | t0.x;
                    nx[1] &= ((uint64_t)t0.w << 32) | t0.z;
                    nx[2] &= ((uint64_t)t1.y << 32) | t1.x;
                    nx[3] &= ((uint64_t)t1.w << 32) | t1.z;
                  }
                }
                if (G != Gt) {
                  // keep the types with an available offering on the narrowed
                  // (zone, capacity-type) grid: OR of the per-pair type sets
                  uint64_t off[WREG] = {};
                  uint64_t gm = G;
                  while (gm) {
                    const uint32_t g = __ffsll((long long)gm) - 1;
                    gm &= gm - 1;
#pragma unroll
                    for (uint32_t w = 0; w < WREG; w++)
                      if (w < W) off[w] |= slot[g * W + w];
                  }
#pragma unroll
                  for (uint32_t w = 0; w < WREG; w++) nx[w] &= off[w];
                }
#pragma unroll
                for (uint32_t w = 0; w < WREG; w++) acc |= nx[w];
              } else {
                // 4 words per round trip (16-B loads; strides are multiples of
                // 4 words), stop at the first batch with a surviving type
                for (uint32_t w0 = 0; w0 < W && !acc; w0 += 4) {
                  const uint4* oq = (const uint4*)(opts + w0);
                  const uint4* rq4 = (const uint4*)(row + w0);
                  const uint4 o0 = oq[0], o1 = oq[1], r0 = rq4[0], r1 = rq4[1];
                  uint64_t x[4] = {(((uint64_t)o0.y << 32) | o0.x) & (((uint64_t)r0.y << 32) | r0.x),
                                   (((uint64_t)o0.w << 32) | o0.z) & (((uint64_t)r0.w << 32) | r0.z),
                                   (((uint64_t)o1.y << 32) | o1.x) & (((uint64_t)r1.y << 32) | r1.x),
                                   (((uint64_t)o1.w << 32) | o1.z) & (((uint64_t)r1.w << 32) | r1.z)};
#pragma unroll
                  for (uint32_t r = 0; r < RR; r++) {
                    if (mm[r] == cur[r]) continue;  // opts ⊆ thr_set[cur] already
                    const uint4* tq = (const uint4*)(dd.thr_set + (size_t)mrow[r] * OW + w0);
                    const uint4 t0 = tq[0], t1 = tq[1];
                    x[0] &= ((uint64_t)t0.y << 32) | t0.x;
                    x[1] &= ((uint64_t)t0.w << 32) | t0.z;
                    x[2] &= ((uint64_t)t1.y << 32) | t1.x;
                    x[3] &= ((uint64_t)t1.w << 32) | t1.z;
                  }
#pragma unroll
                  for (uint32_t w = 0; w < 4; w++) {
                    if (w0 + w >= W) x[w] = 0;  // padding words are not written
                    if (x[w] && G != Gt) {
                      uint64_t off = 0, gm = G;
                      while (gm) {
                        const uint32_t g = __ffsll((long long)gm) - 1;
                        gm &= gm - 1;
                        off |= slot[(size_t)g * W + w0 + w];
                      }
                      x[w] &= off;
                    }
                    acc |= x[w];
                  }
                }
              }
              feas = acc != 0;
              if (TOPO && feas && dd.tmpl[t].mv_mask) {
                // minValues over the NodeClaim's options after Add (per thread)
                feas = mv_ok(dd, dd.tmpl[t], [&](uint32_t w) -> uint64_t {
                  if (W <= WREG) return w == 0 ? nx[0] : w == 1 ? nx[1] : w == 2 ? nx[2] : nx[3];
                  uint64_t x = opts[w] & row[w];
#pragma unroll
                  for (uint32_t r = 0; r < RR; r++) x &= dd.thr_set[(size_t)mrow[r] * OW + w];
                  if (G != Gt) {
                    uint64_t off = 0;
                    for (uint64_t gm = G; gm; gm &= gm - 1) off |= slot[(size_t)(__ffsll((long long)gm) - 1) * W + w];
                    x &= off;
                  }
                  return x;
                });
              }
#ifdef GS_FFD_DIAG
              c3 = __builtin_amdgcn_s_memtime();
#endif
            }
          }
        }
#ifdef GS_FFD_DIAG
        {
          // per wave: cycles to the record test, the cursor probe, the option words
          const uint64_t b1 = __ballot(c1 != 0), b3 = __ballot(c3 != 0);
          if (b1 && (tid & 63) == (uint32_t)(__ffsll((long long)b1) - 1)) {
            atomicAdd((unsigned long long*)&S.dbg[8], (unsigned long long)(c1 - c0));
            atomicAdd((unsigned long long*)&S.dbg[11], 1ull);
          }
          if (b3 && (tid & 63) == (uint32_t)(__ffsll((long long)b3) - 1)) {
            atomicAdd((unsigned long long*)&S.dbg[9], (unsigned long long)(c2 - c1));
            atomicAdd((unsigned long long*)&S.dbg[10], (unsigned long long)(c3 - c2));
            atomicAdd((unsigned long long*)&S.dbg[12], 1ull);
          }
          if (tid == 0) atomicAdd((unsigned long long*)&S.dbg[13], (unsigned long long)(__builtin_amdgcn_s_memtime() - c0));
        }
#endif
#ifdef GS_ASM_MARK
        asm volatile("; MARK_FULL_END");
#endif
        const uint64_t pm = __ballot(pre);
        if ((tid & 63) == 0 && pm) atomicAdd((unsigned long long*)&S.cand_full, (unsigned long long)__popcll(pm));
        uint64_t tq = 0;
        if (tid == 0) tq = phase_clock();
        TL(8);  // exact checks
        if (skip_full) {
          f = mfa;  // block-uniform (from the reduction)
        } else {
          f = wg.first(feas || (fa && pos == mfa), base);
        }
        if (tid == 0) {
          const uint64_t tr_ = phase_clock();
          S.dbg[0] += tq - tA;
          S.dbg[1] += tr_ - tq;
          S.dbg[2]++;
          tA = tr_;
          S.cand += (M - base) < FB ? (M - base) : FB;
        }
        if (f != INF) {
          if (pos == f && fa) {
            // NodeClaim.Add of a simple pod on a fast-accepted claim: requests
            // only (options, cursors and requirements stay); LDS room and
            // slack shrink by the request (still a lower / upper bound)
            ClaimRec* cr = dd.c_rec + cb + j;
            const int64_t t4[4] = {(int64_t)(((uint64_t)ph0.y << 32) | ph0.x), (int64_t)(((uint64_t)ph0.w << 32) | ph0.z),
                                   (int64_t)(((uint64_t)ph1.y << 32) | ph1.x), (int64_t)(((uint64_t)ph1.w << 32) | ph1.z)};
#pragma unroll
            for (uint32_t r = 0; r < 4; r++)
              if (r < R) cr->tot_lo[r] = t4[r] + rq[r];
            cr->count = ph3.w + 1;
            const uint64_t rm = s_rm[j], sl = s_slk[j];
            uint64_t rm2 = 0, sl2 = 0;
#pragma unroll
            for (uint32_t r = 0; r < 4; r++) {
              if (r >= dd.RQ) break;
              rm2 |= (uint64_t)qcode_floor(qcode_value((uint32_t)(rm >> (16 * r)) & 0xFFFFu) - rq[r]) << (16 * r);
              sl2 |= (uint64_t)qcode_ceil(qcode_value((uint32_t)(sl >> (16 * r)) & 0xFFFFu) - rq[r]) << (16 * r);
            }
            s_rm[j] = rm2;
            s_slk[j] = sl2;
            if (s_sc[f] == 0xFFFFu) HN.status = 3;
            s_sc[f]++;
            logp[h.nlog] = LogRec{gp, v, j, 0};
            S.dbg[15]++;
          } else if (pos == f) {
            // NodeClaim.Add by the winning lane: options, requests, requirements
            ClaimRec* cr = dd.c_rec + cb + j;
            uint64_t* opts = dd.c_opts + (size_t)(cb + j) * OW;
            if (W <= WREG) {
#pragma unroll
              for (uint32_t w = 0; w < WREG; w++)
                if (w < W) opts[w] = nx[w];  // already narrowed to the grid
            } else {
              const uint64_t* row = dd.rows + ((size_t)v * T + t) * OW;
              for (uint32_t w = 0; w < W; w++) {
                uint64_t x = opts[w] & row[w];
#pragma unroll
                for (uint32_t r = 0; r < RR; r++) x &= dd.thr_set[(size_t)mrow[r] * OW + w];
                if (G != Gt) {
                  uint64_t off = 0, gm = G;
                  while (gm) {
                    const uint32_t g = __ffsll((long long)gm) - 1;
                    gm &= gm - 1;
                    off |= slot[(size_t)g * W + w];
                  }
                  x &= off;
                }
                opts[w] = x;
              }
            }
            int64_t nt[RR], ma[RR];
            uint32_t cu[RR];
#pragma unroll
            for (uint32_t r = 0; r < RR; r++) {
              nt[r] = tot[r] + rq[r];
              ma[r] = cr->maxa[r];
              cu[r] = mrow[r] - s_thoff[r] - r;
              cr->tot(r) = nt[r];
              cr->thr(r) = (uint16_t)cu[r];
            }
            s_slk[j] = pack_slack(dd, ma, nt);  // exact re-quantization: no drift
            s_rm[j] = pack_room(thr, s_thoff, cu, nt, dd.RQ);
            cr->zm = zm & vr.zm;  // zm (dom_ct: cm) carries the topology narrowing
            cr->cm = cm & vr.cm;
            cr->ctb &= vr.ctb;
            cr->count++;
            if (TOPO) {
              // zone requirement after Add (+ the topology domain), then
              // <U> Topology.Record for every group selecting the pod
              if (!own_n) {
                czf = cr->zfull;
                czfl = cr->zflags;
              }
              const uint64_t zf = czf & vr.zn & zset;
              const uint32_t zl = zset != ~0ull ? 0u : (czfl & vr.zflags);
              cr->zfull = zf;
              cr->zflags = zl;
              int32_t* hrow = dd.hc + (size_t)(cb + j) * dd.TGH;
              topo_record(dd, ts, sel_off, sel_n, zf, zl, [&](uint32_t hs) { hrow[hs] = (hrow[hs] & HC_COUNT) + 1; });
            }
            FK* cf = dd.c_fk + (size_t)(cb + j) * F;
            for (uint32_t k = 0; k < vr.fk_count; k++) {
              const FKEntry& e = dd.fk_entries[vr.fk_begin + k];
              const FK cur = cf[e.slot];
              cf[e.slot] = (cur.flags & FK_PRESENT)
                               ? fk_intersect(cur, e.st, dd.fk_ival + (size_t)e.slot * FKV, dd.fk_isint + (size_t)e.slot * FKW)
                               : e.st;
            }
            if (s_sc[f] == 0xFFFFu) HN.status = 3;
            s_sc[f]++;
            logp[h.nlog] = LogRec{gp, v, j, 0};
          }
          break;
        }
      }
      pf_stage3();
      TL(9);  // reduction + winner update
      if (tid == 0) {
        S.claim_prefix += f != INF ? f + 1 : M;
        const uint64_t tB = phase_clock();
        S.t_scan += tB - tA;
        S.dbg[14] = tB;
        tA = tB;
      }
      if (f != INF) {
        // every wave knows the pod went to the NodeClaim at sorted position f;
        // the next pod's loop-top barrier orders this pod's LDS and claim
        // updates before anything reads them
        if (tid == 0) {
          HN.modkind = MOD_INC;
          HN.modpos = f;
          HN.nlog = h.nlog + 1;
        }
        continue;
      }
      __syncthreads();

      // ------------------------------- new NodeClaim from templates, in order
      const uint32_t cbase = SIM ? qoff : 0u;
      for (uint32_t t = 0; t < T; t++) {
        const TmplRec& tr = d.tmpl[t];
        const uint64_t* row = d.rows + ((size_t)v * T + t) * OW;
        // <U> Topology on the fresh NodeClaim (template AND pod zone domains;
        // a new hostname domain has count 0, always within maxSkew >= 1):
        // the picked zone narrows the K1 row to that zone's offerings
        // (pod affinity on the fresh hostname domain, count 0: only the
        // bootstrap of a self-selecting pod while no selected pod runs)
        uint64_t tzs = ~0ull, tzcat = ~0ull;  // allowed zone domains / their catalog zones
        if (TOPO && own_n) {
          tzs = topo_claim_g(d, ts, own_n, tr.zfull & vr.zn, [](uint32_t) -> int64_t { return 0; }, OWN);
          if (tzs != 0 && tzs != ~0ull && !d.dom_np) tzcat = topo_catmask(d, tzs);
          if (tzs == 0 || tzcat == 0) continue;
        }
        // dom_ct: the picked domains are capacity types of the template's zones
        const bool dct = d.dom_ct != 0;
        const uint64_t tcm = tr.cm & vr.cm & (dct ? tzcat : ~0ull), tzsel = dct ? tr.zm & vr.zm : tzcat;
        const bool dnp = d.dom_np != 0;  // a NodePool domain narrows no offering
        auto rowx = [&](uint32_t w) -> uint64_t {
          uint64_t x = row[w];
          if (tzs != ~0ull && !dnp) {
            uint64_t off = 0;
            for (uint64_t zm_ = tzsel; zm_; zm_ &= zm_ - 1) {
              const uint32_t zc = (uint32_t)__ffsll((long long)zm_) - 1u;
              for (uint32_t c = 0; c < d.C; c++)
                if ((tcm >> c) & 1) off |= slot[(zc * d.C + c) * W + w];
            }
            x &= off;
          }
          return x;
        };
        bool any = false;
        if (d.fk_ok[(size_t)v * T + t])
          for (uint32_t w = 0; w < W; w++)
            if (rowx(w)) any = true;
        if (!any) continue;
        if (tr.has_limits) {
          // <U> filterByRemainingResources on the template's options
          uint32_t hit = INF;
          for (uint32_t i = tid; i < d.N; i += FB) {
            if (!((rowx(i >> 6) >> (i & 63)) & 1)) continue;
            bool ok = true;
            for (uint32_t r = 0; r < R; r++)
              if ((tr.limit_rmask >> r) & 1) ok = ok && d.it_cap[(size_t)r * d.N + i] <= t_rem[(size_t)t * R + r];
            if (ok) hit = 0;
          }
          if (wg.first(hit == 0, 0) == INF) continue;
        }
        if (tid < R) {
          const int64_t tot = tr.daemon[tid] + preq[tid];
          const uint32_t o = s_thoff[tid], n = s_thoff[tid + 1] - o;
          S.c0[tid] = thr_search(thr + o, n, 0, tot);
        }
        __syncthreads();
        // the fresh NodeClaim's option word w
        auto fresh = [&](uint32_t w) -> uint64_t {
          uint64_t x = rowx(w);
          // establish opts ⊆ thr_set[cursor] for the candidate scan
          for (uint32_t r = 0; r < R; r++) x &= d.thr_set[(size_t)(s_thoff[r] + r + S.c0[r]) * OW + w];
          if (tr.has_limits) {
            uint64_t y = 0, m = x;
            while (m) {
              const uint32_t b = __ffsll((long long)m) - 1;
              m &= m - 1;
              const uint32_t i = w * 64 + b;
              bool ok = true;
              for (uint32_t r = 0; r < R; r++)
                if ((tr.limit_rmask >> r) & 1) ok = ok && d.it_cap[(size_t)r * d.N + i] <= t_rem[(size_t)t * R + r];
              if (ok) y |= 1ull << b;
            }
            x = y;
          }
          return x;
        };
        if (TOPO && tr.mv_mask) {
          // minValues over the fresh NodeClaim's options (one thread)
          if (tid == 0) S.mvok = mv_ok(d, tr, fresh) ? 1u : 0u;
          __syncthreads();
          if (!S.mvok) continue;
        }
        if (M >= MCs) {
          if (tid == 0) HN.status = 1;
          __syncthreads();
          break;
        }
        const uint32_t j = M;
        ClaimRec* cr = d.c_rec + cbase + j;
        for (uint32_t w = tid; w < W; w += FB) d.c_opts[(size_t)(cbase + j) * OW + w] = fresh(w);
        if (tid < RR) {
          int64_t tot = 0;
          uint32_t c0 = 0;
          if (tid < R) {
            tot = tr.daemon[tid] + preq[tid];
            c0 = S.c0[tid];
          }
          cr->tot(tid) = tot;
          cr->thr(tid) = (uint16_t)c0;
          S.red64[tid] = 0;
        }
        // <U> Topology.Register(hostname placeholder): the claim's counts start
        // at 0 (simulations: the rows are zero at rest, see the sim's end)
        if (TOPO && !SIM) {
          for (uint32_t h = tid; h < d.TGH; h += FB) d.hc[(size_t)(cbase + j) * d.TGH + h] = 0;
          __syncthreads();
        }
        if (tid == 0) {
          cr->tmpl = t;
          cr->count = 1;
          cr->zm = tr.zm & vr.zm & (dct ? ~0ull : tzcat);
          cr->cm = tcm;
          cr->ctb = tr.ctb & vr.ctb;
          cr->zfull = tr.zfull & vr.zn & tzs;
          cr->zflags = tzs != ~0ull ? 0u : (tr.zflags & vr.zflags);
          if (TOPO && sel_n) {
            // <U> Topology.Record
            int32_t* hrow = d.hc + (size_t)(cbase + j) * d.TGH;
            topo_record(d, ts, sel_off, sel_n, cr->zfull, cr->zflags, [&](uint32_t hs) { hrow[hs] = (hrow[hs] & HC_COUNT) + 1; });
          }
          FK* cf = d.c_fk + (size_t)(cbase + j) * F;
          for (uint32_t s = 0; s < F; s++) cf[s] = d.t_fk[(size_t)t * F + s];
          for (uint32_t k = 0; k < vr.fk_count; k++) {
            const FKEntry& e = d.fk_entries[vr.fk_begin + k];
            const FK cur = cf[e.slot];
            cf[e.slot] = (cur.flags & FK_PRESENT)
                             ? fk_intersect(cur, e.st, d.fk_ival + (size_t)e.slot * FKV, d.fk_isint + (size_t)e.slot * FKW)
                             : e.st;
          }
          s_ord[M] = (uint16_t)M;
          s_sc[M] = 1;
          s_tmpl[M] = (uint8_t)t;
          HN.M = M + 1;
          HN.modkind = MOD_APPEND;
          logp[HN.nlog++] = LogRec{gp, v, j, 0};
          S.found = 1;
        }
        __syncthreads();
        // max allocatable over the new claim's options (the slack bound)
        for (uint32_t i = tid; i < d.N; i += FB) {
          if (!((d.c_opts[(size_t)(cbase + j) * OW + (i >> 6)] >> (i & 63)) & 1)) continue;
          for (uint32_t r = 0; r < R; r++) atomicMax(&S.red64[r], (unsigned long long)d.it_alloc[(size_t)r * d.N + i]);
        }
        __syncthreads();
        if (tid < RR) cr->maxa[tid] = tid < R ? (int64_t)S.red64[tid] : 0;
        if (tid == 0) {
          // LDS slack from the max allocatable over the new claim's options
          int64_t nt[RR], ma[RR];
#pragma unroll
          for (uint32_t r = 0; r < RR; r++) {
            nt[r] = r < R ? tr.daemon[r] + preq[r] : 0;
            ma[r] = r < R ? (int64_t)S.red64[r] : 0;
          }
          s_slk[j] = pack_slack(d, ma, nt);
          s_rm[j] = pack_room(thr, s_thoff, S.c0, nt, d.RQ);
        }
        __syncthreads();
        if (tr.has_limits) {
          // <U> subtractMax(remaining, nodeClaim.InstanceTypeOptions)
          if (tid < R) S.red64[tid] = 0;
          __syncthreads();
          for (uint32_t i = tid; i < d.N; i += FB) {
            if (!((d.c_opts[(size_t)(cbase + j) * OW + (i >> 6)] >> (i & 63)) & 1)) continue;
            for (uint32_t r = 0; r < R; r++)
              if ((tr.limit_rmask >> r) & 1)
                atomicMax(&S.red64[r], (unsigned long long)(d.it_cap[(size_t)r * d.N + i] + (1ll << 62)));
          }
          __syncthreads();
          if (tid < R && ((tr.limit_rmask >> tid) & 1) && S.red64[tid] != 0)
            t_rem[(size_t)t * R + tid] -= (int64_t)(S.red64[tid] - (1ull << 62));
        }
        __syncthreads();
        break;
      }
      __syncthreads();
      if (tid == 0) {
        S.dbg[14] = phase_clock();
        S.t_tmpl += S.dbg[14] - tA;
      }
      TL(10);  // new NodeClaim
      if (HN.status) break;
      if (S.found) continue;

      // ------------------------------------ failed: Relax, then Queue.Push
      if (tid == 0) {
        bool relaxed = false;
        if (v + 1 < d.var_begin[gp] + d.var_count[gp]) {
          cur_var[p] = v + 1;
          relaxed = true;
          if (TOPO && d.n_lazy) topo_relaxed(d, ts, v + 1, d.hc + (size_t)(SIM ? qoff : 0u) * d.TGH, M, 0u, 1u);
        }
        uint32_t tail = HN.qhead + HN.qlen;
        if (tail >= P) tail -= P;
        queue[tail] = p;
        HN.qlen++;
        if (relaxed) {
          HN.epoch++;
        } else {
          last_epoch[p] = HN.epoch;
          last_len[p] = HN.qlen;
        }
      }
      __syncthreads();
    }

    __syncthreads();
    if (!SIM)
      for (uint32_t i = tid; i < S.hb[par ^ 1u].M; i += FB) d.c_sorted[i] = s_ord[i];
    if (SIM && TOPO && d.TGH) {
      // the NodeClaims' hostname counts back to zero, cell by recorded cell
      // (a pod placed on NodeClaim j counted in the hostname groups of its
      // selection list), so the next simulation's NodeClaims start from zero
      // rows without writing TGH counts each
      for (uint32_t i = tid; i < S.hb[par ^ 1u].nlog; i += FB) {
        const LogRec l = logp[i];
        if (l.target & 0x80000000u) continue;
        const VarRec& lv = d.vars[l.var];
        int32_t* hrow = d.hc + (size_t)(qoff + l.target) * d.TGH;
        for (uint32_t k = 0; k < lv.sel_n; k++) {
          const uint32_t e = d.tg_list[lv.sel_off + k];
          if ((e >> 24) & TK_HOST) hrow[e & (((e >> 24) & TK_LAZY) ? 0xFFFu : 0xFFFFFFu)] = 0;
        }
      }
      // and the cells a lazy hostname group created in this simulation marked
      // HC_UNKNOWN on the NodeClaims that existed before it
      if (d.n_lazy) {
        __syncthreads();
        topo_unmark(d, ts, d.hc + (size_t)qoff * d.TGH, S.hb[par ^ 1u].M, tid, FB);
      }
    }
    if (SIM) {
      // SimulateScheduling's error pods that are not pending: still queued,
      // or placed on an uninitialized existing node
      uint32_t cnt = 0;
      for (uint32_t i = tid; i < S.hb[par ^ 1u].qlen; i += FB) {
        uint32_t slot = S.hb[par ^ 1u].qhead + i;
        if (slot >= P) slot -= P;
        cnt += gpod(queue[slot]) >= d.n_pending ? 1u : 0u;
      }
      for (uint32_t i = tid; i < S.hb[par ^ 1u].nlog; i += FB) {
        const LogRec l = logp[i];
        cnt += ((l.target & 0x80000000u) && l.pod >= d.n_pending && !d.nodes0[l.target & 0x7FFFFFFFu].init) ? 1u : 0u;
      }
      cnt = wave_sum_u32(cnt);
      if (lane == 0 && cnt) atomicAdd(&S.failed, cnt);
      __syncthreads();
    }
    if (SIM && tid == 0) {
      // the outcome in one store; the counters into this workgroup's sums
      d.sim_ctrl[sim] = SimCtrl{S.hb[par ^ 1u].status, S.hb[par ^ 1u].M, S.hb[par ^ 1u].nlog, S.failed};
      b_pops += S.hb[par ^ 1u].pops;
      b_gen += S.generic;
      b_fast += S.fast;
      b_cand += S.cand;
      b_full += S.cand_full;
      b_nev += S.node_evals;
      b_npre += S.node_prefix;
      b_cpre += S.claim_prefix;
    }
    if (!SIM && tid == 0) {
      Ctrl c;
      c.status = S.hb[par ^ 1u].status;
      c.n_claims = S.hb[par ^ 1u].M;
      c.n_log = S.hb[par ^ 1u].nlog;
      c.qhead = S.hb[par ^ 1u].qhead;
      c.qlen = S.hb[par ^ 1u].qlen;
      c.epoch = S.hb[par ^ 1u].epoch;
      c.pops = S.hb[par ^ 1u].pops;
      c.generic_sorts = S.generic;
      c.fast_sorts = S.fast;
      c.cand_evals = S.cand;
      c.cand_full = S.cand_full;
      c.node_evals = S.node_evals;
      c.node_prefix = S.node_prefix;
      c.claim_prefix = S.claim_prefix;
      c.failed = S.failed;
      c.pad = 0;
#ifdef GS_FFD_PHASES
      c.t_sort = S.t_sort;
      c.t_scan = S.t_scan;
      c.t_tmpl = S.t_tmpl;
#else
      c.t_sort = c.t_scan = c.t_tmpl = ~0ull;  // not measured: gs_result reports -1
#endif
      c.t_total = wall_clock64() - S.t0;
      S.dbg[7] = __builtin_amdgcn_s_memtime() - S.dbg[7];  // shader clock cycles over the solve
#ifdef GS_FFD_TL
      for (int q = 0; q < 16; q++) c.dbg[q] = S.tl[q];
#else
      for (int q = 0; q < 16; q++) c.dbg[q] = S.dbg[q];
#endif
      *d.ctrl = c;
    }
    __syncthreads();
  }
  if (SIM && tid == 0) {
    Ctrl c = {};
    c.pops = b_pops;
    c.generic_sorts = b_gen;
    c.fast_sorts = b_fast;
    c.cand_evals = b_cand;
    c.cand_full = b_full;
    c.node_evals = b_nev;
    c.node_prefix = b_npre;
    c.claim_prefix = b_cpre;
    d.sim_blk[blockIdx.x] = c;
  }
}

// dynamic LDS: slack + room u64, ord/sc/scr u16, tmpl u8 per claim, thresholds,
// (simulations) the touched-node bitmap, and the topology
// spread state (known domains, per-pod minimum, zone counts) of TG groups
extern "C" uint32_t gsk_ffd_lds_bytes(uint32_t max_claims, uint32_t nthr, uint32_t nb_words,
                                      uint32_t topo_bytes) {
  const uint32_t thr = nthr + 4;
  const uint32_t base = (((23u * max_claims + 7u) & ~7u) + thr * 8u + nb_words * 4u + 7u) & ~7u;
  return base + topo_bytes;
}

// every instantiation may use all LDS its static footprint leaves free
static uint32_t g_ffd_dyn_max = 0;

template <uint32_t RR, bool SIM, bool TOPO = false, uint32_t NT = SIM ? FB_SIM : FB_MAX>
static hipError_t ffd_attr(uint32_t lds_total) {
  hipFuncAttributes a;
  hipError_t e = hipFuncGetAttributes(&a, (const void*)ffd_kernel<RR, SIM, NT, TOPO>);
  if (e != hipSuccess) return e;
  const uint32_t dyn = lds_total > a.sharedSizeBytes ? lds_total - (uint32_t)a.sharedSizeBytes : 0;
  if (!g_ffd_dyn_max || dyn < g_ffd_dyn_max) g_ffd_dyn_max = dyn;
  return hipFuncSetAttribute((const void*)ffd_kernel<RR, SIM, NT, TOPO>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)dyn);
}

template <uint32_t RR>
static hipError_t ffd_attr_all(uint32_t lds_total) {
  hipError_t e = hipSuccess;
  for (hipError_t x : {ffd_attr<RR, false>(lds_total), ffd_attr<RR, false, true>(lds_total), ffd_attr<RR, true>(lds_total),
                       ffd_attr<RR, true, false, FB_SIM_NARROW>(lds_total), ffd_attr<RR, true, true, FB_SIM>(lds_total),
                       ffd_attr<RR, true, true, FB_SIM_NARROW>(lds_total)})
    if (x != hipSuccess) e = x;
  return e;
}

extern "C" hipError_t gsk_init_ffd(uint32_t lds_total) {
  hipError_t e = hipSuccess;
  for (hipError_t x : {ffd_attr_all<1>(lds_total), ffd_attr_all<2>(lds_total), ffd_attr_all<3>(lds_total),
                       ffd_attr_all<4>(lds_total), ffd_attr_all<5>(lds_total), ffd_attr_all<6>(lds_total),
                       ffd_attr_all<7>(lds_total), ffd_attr_all<8>(lds_total)})
    if (x != hipSuccess) e = x;
  return e;
}

extern "C" uint32_t gsk_ffd_dyn_lds_max(void) { return g_ffd_dyn_max; }

// resident simulation workgroups per CU for a given dynamic LDS size
template <uint32_t RR>
static hipError_t sim_occ(int* n, bool narrow, bool general, uint32_t lds) {
  if (general)
    return narrow ? hipOccupancyMaxActiveBlocksPerMultiprocessor(n, (const void*)ffd_kernel<RR, true, FB_SIM_NARROW, true>,
                                                                 FB_SIM_NARROW, lds)
                  : hipOccupancyMaxActiveBlocksPerMultiprocessor(n, (const void*)ffd_kernel<RR, true, FB_SIM, true>, FB_SIM, lds);
  return narrow ? hipOccupancyMaxActiveBlocksPerMultiprocessor(n, (const void*)ffd_kernel<RR, true, FB_SIM_NARROW, false>,
                                                               FB_SIM_NARROW, lds)
                : hipOccupancyMaxActiveBlocksPerMultiprocessor(n, (const void*)ffd_kernel<RR, true, FB_SIM, false>, FB_SIM, lds);
}

extern "C" uint32_t gsk_ffd_sim_blocks_per_cu(uint32_t R, uint32_t lds, uint32_t nt, uint32_t general) {
  int n = 0;
  hipError_t e = hipErrorInvalidValue;
  const bool narrow = nt == (uint32_t)FB_SIM_NARROW;
  switch (R) {
#define GSK_OCC(k) \
  case k: e = sim_occ<k>(&n, narrow, general != 0, lds); break;
    GSK_OCC(1) GSK_OCC(2) GSK_OCC(3) GSK_OCC(4) GSK_OCC(5) GSK_OCC(6) GSK_OCC(7) GSK_OCC(8)
#undef GSK_OCC
  }
  return e == hipSuccess && n > 0 ? (uint32_t)n : 1u;
}

// grid: 1 workgroup (provisioning Solve) or `blocks` persistent workgroups
// draining the simulation counter (consolidation)
extern "C" hipError_t gsk_ffd(const DevProblem* d, uint32_t blocks, hipStream_t s) {
  const uint32_t lds = gsk_ffd_lds_bytes(d->max_claims, d->n_thr, d->nb_words, topo_lds_bytes(d->TGZ, d->ZS, d->TGH, d->n_lazy)) +
                       (d->n_sims ? 8u * d->ovh_slots + (d->sim_lds ? 32u * d->max_claims : 0u) : 0u);
  if (lds > g_ffd_dyn_max) return hipErrorInvalidConfiguration;
  const bool sim = d->n_sims > 0;
  // shape: 0 provisioning, 1 provisioning (general variant), 2 simulations, 3 narrow simulations,
  // 4 / 5 simulations / narrow simulations, general variant (topology groups, volumes, minValues)
  if (sim && d->sim_nt != (uint32_t)FB_SIM && d->sim_nt != (uint32_t)FB_SIM_NARROW) return hipErrorInvalidValue;
  const bool general = d->TG || d->any_mv || d->any_vol;
  const uint32_t shape = sim ? (d->sim_nt == (uint32_t)FB_SIM_NARROW ? 3u : 2u) + (general ? 2u : 0u) : (general ? 1u : 0u);
  switch (d->R * 8 + shape) {
#define GSK_CASE(n)                                                                                          \
  case 8 * n: hipLaunchKernelGGL((ffd_kernel<n, false, FB_MAX, false>), dim3(1), dim3(FB_MAX), lds, s, *d); break; \
  case 8 * n + 1: hipLaunchKernelGGL((ffd_kernel<n, false, FB_MAX, true>), dim3(1), dim3(FB_MAX), lds, s, *d); break; \
  case 8 * n + 2: hipLaunchKernelGGL((ffd_kernel<n, true, FB_SIM, false>), dim3(blocks), dim3(FB_SIM), lds, s, *d); break; \
  case 8 * n + 3:                                                                                            \
    hipLaunchKernelGGL((ffd_kernel<n, true, FB_SIM_NARROW, false>), dim3(blocks), dim3(FB_SIM_NARROW), lds, s, *d); \
    break;                                                                                                    \
  case 8 * n + 4: hipLaunchKernelGGL((ffd_kernel<n, true, FB_SIM, true>), dim3(blocks), dim3(FB_SIM), lds, s, *d); break; \
  case 8 * n + 5:                                                                                            \
    hipLaunchKernelGGL((ffd_kernel<n, true, FB_SIM_NARROW, true>), dim3(blocks), dim3(FB_SIM_NARROW), lds, s, *d); \
    break;
    GSK_CASE(1) GSK_CASE(2) GSK_CASE(3) GSK_CASE(4) GSK_CASE(5) GSK_CASE(6) GSK_CASE(7) GSK_CASE(8)
#undef GSK_CASE
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ================================================ first-pass queue records
// The Solve's first pass pops pods in queue0 order with their first variant:
// the records are gathered into queue order here, on the device, from the
// arrays the upload already holds (one thread per queue position; HBM-bound,
// ~0.2 KB per pod), instead of being built on the host and copied a second
// time over PCIe.  qcodes: qcode_floor / qcode_ceil of resources 0..3 packed
// 16 bits each, the wave Solve's SWAR operands.
__global__ __launch_bounds__(256) void queue_records_kernel(DevProblem d) {
  const uint32_t k = blockIdx.x * 256 + threadIdx.x;
  if (k >= d.P) return;
  const uint32_t p = d.queue0[k];
  const uint4* src = (const uint4*)(d.vars + d.var_begin[p]);
  uint4* dst = (uint4*)(const_cast<VarRec*>(d.qvars) + k);
#pragma unroll
  for (uint32_t q = 0; q < sizeof(VarRec) / sizeof(uint4); q++) dst[q] = src[q];
  int64_t* qr = const_cast<int64_t*>(d.qreqs) + (size_t)k * d.R;
  uint64_t fl = 0, ce = 0;
  for (uint32_t r = 0; r < d.R; r++) {
    const int64_t v = d.pod_req[(size_t)p * d.R + r];
    qr[r] = v;
    if (r < 4) {
      fl |= (uint64_t)qcode_floor(v) << (16 * r);
      ce |= (uint64_t)qcode_ceil(v) << (16 * r);
    }
  }
  uint4 c;
  c.x = (uint32_t)fl;
  c.y = (uint32_t)(fl >> 32);
  c.z = (uint32_t)ce;
  c.w = (uint32_t)(ce >> 32);
  ((uint4*)const_cast<uint32_t*>(d.qcodes))[k] = c;
}

// qrun[k]: how many records from k on (at most the ring's 16) equal record k
// in every dword the wave Solve's run mode compares (all but the pod and the
// variant index): the batch of a run's pods reads it from the ring
// (ffd_wave.hpp GS_RUN_BATCH) instead of comparing 16 staged records.  One
// comparison per adjacent pair (same[x]: record x equals record x + 1) into
// LDS, block range plus a 15-entry halo, then a scan of at most 15 bits
__device__ __forceinline__ bool queue_record_same(const DevProblem& d, uint32_t a, uint32_t b) {
  const uint4* va = (const uint4*)(d.qvars + a);
  const uint4* vb = (const uint4*)(d.qvars + b);
  bool same = true;
#pragma unroll
  for (uint32_t q = 0; q < sizeof(VarRec) / 16; q++) {
    const uint4 x = va[q], y = vb[q];
    // dword 0 (pod) and the last dword (variant index) may differ
    same = same && (q == 0 || x.x == y.x) && x.y == y.y && x.z == y.z && (q == sizeof(VarRec) / 16 - 1 || x.w == y.w);
  }
  for (uint32_t r = 0; r < d.R; r++) same = same && d.qreqs[(size_t)a * d.R + r] == d.qreqs[(size_t)b * d.R + r];
  return same;  // the codes follow from the requests
}
__global__ __launch_bounds__(256) void queue_runs_kernel(DevProblem d) {
  __shared__ uint8_t s_same[256 + 16];
  const uint32_t b0 = blockIdx.x * 256;
  for (uint32_t t = threadIdx.x; t < 256 + 16; t += 256) {
    const uint32_t x = b0 + t;
    s_same[t] = x + 1 < d.P && queue_record_same(d, x, x + 1);
  }
  __syncthreads();
  const uint32_t k = b0 + threadIdx.x;
  if (k >= d.P) return;
  uint32_t n = 1;
  while (n < 16 && s_same[threadIdx.x + n - 1]) n++;
  const_cast<uint32_t*>(d.qrun)[k] = n;
}

extern "C" hipError_t gsk_queue_records(const DevProblem* d, hipStream_t s) {
  if (!d->P) return hipSuccess;
  hipLaunchKernelGGL(queue_records_kernel, dim3((d->P + 255) / 256), dim3(256), 0, s, *d);
  hipLaunchKernelGGL(queue_runs_kernel, dim3((d->P + 255) / 256), dim3(256), 0, s, *d);
  return hipGetLastError();
}
