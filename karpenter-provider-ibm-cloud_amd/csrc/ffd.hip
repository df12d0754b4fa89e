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
#include "layout.hpp"

using namespace gsd;

namespace {

constexpr int FB = 1024;
constexpr int NWAVE = FB / 64;
constexpr int SEQ_SORT = 128;  // subranges up to this length sort on thread 0
constexpr uint32_t THR_LDS_MAX = 4096;
enum : uint32_t { MOD_NONE = 0, MOD_INC = 1, MOD_APPEND = 2 };

struct Frame {
  int a, b, limit;
  int wb, wp;  // wasBalanced, wasPartitioned
};

struct Shared {
  uint32_t pod, var, stop, M, modkind, modpos, qhead, qlen, epoch, nlog, status, found;
  uint32_t fast_path, modpos_sorted;
  int piv, hint;
  uint64_t pops, generic, fast, cand, cand_full;
  uint64_t t_sort, t_scan, t_tmpl, t0;
  uint64_t dbg[8];
  uint32_t red[2][NWAVE];
  unsigned long long red64[RMAX];
  Frame stk[48];
};

__device__ __forceinline__ int bits_len(uint64_t x) { return x ? 64 - __clzll((long long)x) : 0; }

// ---------------------------------------------------------------- sequential
// Go sort.Slice (src/sort/zsortfunc.go) over u16 keys with u16 payload, one
// thread; pdq_frame() resumes a pdqsort_func loop from a given frame state.
struct SeqSort {
  uint16_t* sc;
  uint16_t* ord;
  __device__ bool less(int i, int j) const { return sc[i] < sc[j]; }
  __device__ void swap(int i, int j) const {
    uint16_t a = sc[i];
    sc[i] = sc[j];
    sc[j] = a;
    a = ord[i];
    ord[i] = ord[j];
    ord[j] = a;
  }
  __device__ void insertion_sort(int a, int b) const {
    for (int i = a + 1; i < b; i++)
      for (int j = i; j > a && less(j, j - 1); j--) swap(j, j - 1);
  }
  __device__ void sift_down(int lo, int hi, int first) const {
    int root = lo;
    for (;;) {
      int child = 2 * root + 1;
      if (child >= hi) return;
      if (child + 1 < hi && less(first + child, first + child + 1)) child++;
      if (!less(first + root, first + child)) return;
      swap(first + root, first + child);
      root = child;
    }
  }
  __device__ void heap_sort(int a, int b) const {
    int first = a, lo = 0, hi = b - a;
    for (int i = (hi - 1) / 2; i >= 0; i--) sift_down(i, hi, first);
    for (int i = hi - 1; i >= 0; i--) {
      swap(first, first + i);
      sift_down(lo, i, first);
    }
  }
  __device__ int partition(int a, int b, int pivot, bool* already) const {
    swap(a, pivot);
    int i = a + 1, j = b - 1;
    while (i <= j && less(i, a)) i++;
    while (i <= j && !less(j, a)) j--;
    if (i > j) {
      swap(j, a);
      *already = true;
      return j;
    }
    swap(i, j);
    i++;
    j--;
    for (;;) {
      while (i <= j && less(i, a)) i++;
      while (i <= j && !less(j, a)) j--;
      if (i > j) break;
      swap(i, j);
      i++;
      j--;
    }
    swap(j, a);
    *already = false;
    return j;
  }
  __device__ int partition_equal(int a, int b, int pivot) const {
    swap(a, pivot);
    int i = a + 1, j = b - 1;
    for (;;) {
      while (i <= j && !less(a, i)) i++;
      while (i <= j && less(a, j)) j--;
      if (i > j) break;
      swap(i, j);
      i++;
      j--;
    }
    return i;
  }
  __device__ bool partial_insertion_sort(int a, int b) const {
    int i = a + 1;
    for (int j = 0; j < 5; j++) {
      while (i < b && !less(i, i - 1)) i++;
      if (i == b) return true;
      if (b - a < 50) return false;
      swap(i, i - 1);
      if (i - a >= 2)
        for (int k = i - 1; k >= 1; k--) {
          if (!less(k, k - 1)) break;
          swap(k, k - 1);
        }
      if (b - i >= 2)
        for (int k = i + 1; k < b; k++) {
          if (!less(k, k - 1)) break;
          swap(k, k - 1);
        }
    }
    return false;
  }
  __device__ void break_patterns(int a, int b) const {
    int length = b - a;
    if (length >= 8) {
      uint64_t r = (uint64_t)length;
      uint64_t modulus = 1ull << bits_len((uint64_t)length);
      int idx = a + (length / 4) * 2 - 1;
      for (int i = 0; i < 3; i++) {
        r ^= r << 13;
        r ^= r >> 7;
        r ^= r << 17;
        int other = (int)(r & (modulus - 1));
        if (other >= length) other -= length;
        swap(idx - 1 + i, a + other);
      }
    }
  }
  __device__ void order2(int& a, int& b, int* swaps) const {
    if (less(b, a)) {
      (*swaps)++;
      int t = a;
      a = b;
      b = t;
    }
  }
  __device__ int median(int a, int b, int c, int* swaps) const {
    order2(a, b, swaps);
    order2(b, c, swaps);
    order2(a, b, swaps);
    return b;
  }
  // choosePivot with the (up to) 9 sampled keys loaded in one round trip;
  // same comparisons, same swaps count, same result as choose_pivot()
  __device__ int choose_pivot_fast(int a, int b, int* hint) const {
    const int l = b - a;
    int swaps = 0;
    const int i0 = a + l / 4 * 1, j0 = a + l / 4 * 2, k0 = a + l / 4 * 3;
    if (l < 8) {
      *hint = 1;
      return j0;
    }
    int idx[9] = {i0 - 1, i0, i0 + 1, j0 - 1, j0, j0 + 1, k0 - 1, k0, k0 + 1};
    uint16_t key[9];
#pragma unroll
    for (int t = 0; t < 9; t++) key[t] = (l >= 50 || t % 3 == 1) ? sc[idx[t]] : 0;
    auto med = [&](int x, int y, int z, uint16_t kx, uint16_t ky, uint16_t kz, uint16_t* km) {
      // order2(x,y); order2(y,z); order2(x,y); return y
      if (ky < kx) { swaps++; int t = x; x = y; y = t; uint16_t u = kx; kx = ky; ky = u; }
      if (kz < ky) { swaps++; int t = y; y = z; z = t; uint16_t u = ky; ky = kz; kz = u; }
      if (ky < kx) { swaps++; int t = x; x = y; y = t; uint16_t u = kx; kx = ky; ky = u; }
      *km = ky;
      return y;
    };
    int i = i0, j = j0, k = k0;
    uint16_t ki = key[1], kj = key[4], kk = key[7];
    if (l >= 50) {
      i = med(idx[0], idx[1], idx[2], key[0], key[1], key[2], &ki);
      j = med(idx[3], idx[4], idx[5], key[3], key[4], key[5], &kj);
      k = med(idx[6], idx[7], idx[8], key[6], key[7], key[8], &kk);
    }
    uint16_t km;
    j = med(i, j, k, ki, kj, kk, &km);
    *hint = swaps == 0 ? 1 : (swaps == 12 ? 2 : 0);
    return j;
  }
  // hint: 0 unknown, 1 increasing, 2 decreasing
  __device__ int choose_pivot(int a, int b, int* hint) const {
    int l = b - a, swaps = 0;
    int i = a + l / 4 * 1, j = a + l / 4 * 2, k = a + l / 4 * 3;
    if (l >= 8) {
      if (l >= 50) {
        i = median(i - 1, i, i + 1, &swaps);
        j = median(j - 1, j, j + 1, &swaps);
        k = median(k - 1, k, k + 1, &swaps);
      }
      j = median(i, j, k, &swaps);
    }
    *hint = swaps == 0 ? 1 : (swaps == 12 ? 2 : 0);
    return j;
  }
  __device__ void reverse_range(int a, int b) const {
    int i = a, j = b - 1;
    while (i < j) {
      swap(i, j);
      i++;
      j--;
    }
  }
  __device__ void pdq_frame(Frame f0) const {
    Frame st[32];
    int sp = 0;
    st[sp++] = f0;
    while (sp > 0) {
      Frame f = st[--sp];
      for (;;) {
        int length = f.b - f.a;
        if (length <= 12) {
          insertion_sort(f.a, f.b);
          break;
        }
        if (f.limit == 0) {
          heap_sort(f.a, f.b);
          break;
        }
        if (!f.wb) {
          break_patterns(f.a, f.b);
          f.limit--;
        }
        int hint;
        int pivot = choose_pivot(f.a, f.b, &hint);
        if (hint == 2) {
          reverse_range(f.a, f.b);
          pivot = (f.b - 1) - (pivot - f.a);
          hint = 1;
        }
        if (f.wb && f.wp && hint == 1) {
          if (partial_insertion_sort(f.a, f.b)) break;
        }
        if (f.a > 0 && !less(f.a - 1, pivot)) {
          f.a = partition_equal(f.a, f.b, pivot);
          continue;
        }
        bool already;
        int mid = partition(f.a, f.b, pivot, &already);
        f.wp = already;
        int leftLen = mid - f.a, rightLen = f.b - mid;
        int bal = length / 8;
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
        st[sp++] = f;
        f = child;
      }
    }
  }
};

// ------------------------------------------------------------ block-parallel
struct Blk {
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
  __device__ void pdqsort(int n) {
    SeqSort seq{sc, ord};
    if (n <= SEQ_SORT) {
      if (tid == 0) seq.pdq_frame(Frame{0, n, bits_len((uint64_t)n), 1, 1});
      sync();
      return;
    }
    int sp = 0;
    Frame f{0, n, bits_len((uint64_t)n), 1, 1};
    for (;;) {
      for (;;) {
        const int length = f.b - f.a;
        if (length <= SEQ_SORT) {
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

// first m in [m0, n) with thr[m] >= x (thresholds ascending); n if none
__device__ __forceinline__ uint32_t thr_probe(const int64_t* thr, uint32_t n, uint32_t m0, int64_t x) {
  uint32_t m = m0;
  for (int s = 0; s < 4 && m < n && thr[m] < x; s++) m++;
  if (m < n && thr[m] < x) {
    uint32_t lo = m, hi = n;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (thr[mid] < x) lo = mid + 1;
      else hi = mid;
    }
    m = lo;
  }
  return m;
}

}  // namespace

extern "C" __global__ __launch_bounds__(FB) void ffd_kernel(DevProblem d) {
  extern __shared__ uint64_t lds64[];
  __shared__ Shared S;
  const uint32_t MC = d.max_claims;
  uint16_t* s_ord = (uint16_t*)lds64;
  uint16_t* s_sc = s_ord + MC;
  uint16_t* s_scr = s_sc + MC;
  uint8_t* s_tmpl = (uint8_t*)(s_scr + MC);
  int64_t* s_thr = (int64_t*)(((uintptr_t)(s_tmpl + MC) + 7) & ~(uintptr_t)7);
  __shared__ uint64_t s_tzm[TMAX], s_tcm[TMAX];
  const uint32_t tid = threadIdx.x;
  const uint32_t W = d.W, R = d.R, F = d.F, T = d.T, P = d.P;
  const uint32_t nthr = d.thr_off[R];
  const int64_t* thr = nthr <= THR_LDS_MAX ? s_thr : d.thr_val;
  Blk blk{s_sc, s_ord, s_scr, S, tid, tid & 63, tid >> 6, 0, MC / 2};

  for (uint32_t i = tid; i < P; i += FB) {
    d.queue[i] = d.queue0[i];
    d.last_epoch[i] = 0;
    d.last_len[i] = 0;
    d.cur_var[i] = d.var_begin[i];
  }
  if (nthr <= THR_LDS_MAX)
    for (uint32_t i = tid; i < nthr; i += FB) s_thr[i] = d.thr_val[i];
  for (uint32_t i = tid; i < T * R; i += FB) d.t_rem[i] = d.tmpl[i / R].limits[i % R];
  for (uint32_t t = tid; t < T; t += FB) {
    s_tzm[t] = d.tmpl[t].zm;
    s_tcm[t] = d.tmpl[t].cm;
  }
  if (tid == 0) {
    S.M = 0;
    S.qhead = 0;
    S.qlen = P;
    S.epoch = 1;
    S.modkind = MOD_NONE;
    S.nlog = 0;
    S.pops = S.generic = S.fast = S.cand = S.cand_full = 0;
    S.t_sort = S.t_scan = S.t_tmpl = 0;
    for (int q = 0; q < 8; q++) S.dbg[q] = 0;
    S.t0 = wall_clock64();
    S.status = 0;
  }
  __syncthreads();
  const uint64_t max_pops = ((uint64_t)(d.V - d.P) + 2) * (uint64_t)P + P + 16;

  uint64_t tLoop = 0;
  for (;;) {
    // ------------------------------------------------------------ Queue.Pop
    if (tid == 0) tLoop = wall_clock64();
    if (tid == 0) {
      uint32_t stop = 0;
      if (S.pops > max_pops) {
        S.status = 2;
        stop = 1;
      } else if (S.qlen == 0) {
        stop = 1;
      } else {
        const uint32_t p = d.queue[S.qhead];
        if (d.last_epoch[p] == S.epoch && d.last_len[p] == S.qlen) {
          stop = 1;
        } else {
          S.qhead = S.qhead + 1 == P ? 0 : S.qhead + 1;
          S.qlen--;
          S.pops++;
          S.pod = p;
          S.var = d.cur_var[p];
        }
      }
      S.stop = stop;
      S.found = 0;
    }
    __syncthreads();
    if (S.stop) break;
    const uint32_t p = S.pod, v = S.var;
    const VarRec vr = d.vars[v];
    const int64_t* preq = d.pod_req + (size_t)p * R;
    const uint32_t M = S.M;
    uint64_t tA = 0;
    if (tid == 0) {
      tA = wall_clock64();
      S.dbg[4] += tA - tLoop;  // pop + variant load
    }

    // ------------------------- sort.Slice(newNodeClaims, len(Pods) asc)
    if (M > 1) {
      if (tid == 0) {
        SeqSort ss{s_sc, s_ord};
        uint32_t fast = 0, generic = 0;
        bool inversion = false;
        if (S.modkind == MOD_INC) {
          const uint32_t q = S.modpos;
          inversion = q + 1 < M && s_sc[q + 1] < s_sc[q];
        } else if (S.modkind == MOD_APPEND) {
          inversion = s_sc[M - 2] > s_sc[M - 1];
        }
        if (!inversion) {
          // sorted input: pdqsort_func / insertionSort leave it untouched
        } else if (M <= 12) {
          ss.insertion_sort(0, (int)M);
        } else {
          int hint;
          ss.choose_pivot_fast(0, (int)M, &hint);
          if (hint == 1 && M >= 50) {
            // partialInsertionSort fixes the single inversion;
            // the landing position is found by the block below
            fast = S.modkind;
            S.fast++;
          } else {
            generic = 1;
            S.generic++;
          }
        }
        S.fast_path = fast | (generic << 4);
        S.modpos_sorted = S.modpos;
        S.modkind = MOD_NONE;
      }
      __syncthreads();
      if (tid == 0) {
        const uint64_t tq = wall_clock64();
        S.dbg[3] += tq - tA;
      }
      const uint32_t fp = S.fast_path;
      if (fp == MOD_INC) {
        // X (at q, count x) moves right past the run of counts < x
        const uint32_t q = S.modpos_sorted, x = s_sc[q];
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
      } else if (fp >> 4) {
        blk.pdqsort((int)M);
      }
      __syncthreads();
    }
    if (tid == 0) {
      const uint64_t tB = wall_clock64();
      S.t_sort += tB - tA;
      tA = tB;
    }

    // ---------------------- in-flight NodeClaims, first that CanAdd wins
    int64_t rq[RMAX];
#pragma unroll
    for (uint32_t r = 0; r < RMAX; r++) rq[r] = r < R ? preq[r] : 0;
    uint32_t f = INF;
    for (uint32_t base = 0; base < M; base += FB) {
      const uint32_t pos = base + tid;
      bool feas = false, pre = false;
      if (pos < M) {
        const uint32_t j = s_ord[pos];
        const uint32_t t = s_tmpl[j];
        if ((vr.tolt >> t) & 1) {
          // one record read: totals, max-allocatable bound, cursors, masks
          const ClaimRec* cr = d.c_rec + j;
          int64_t tot[RMAX], mx[RMAX];
          uint32_t cur[RMAX];
#pragma unroll
          for (uint32_t r = 0; r < RMAX; r++) {
            tot[r] = r < R ? cr->tot[r] : 0;
            mx[r] = r < R ? cr->maxa[r] : 0;
            cur[r] = r < R ? cr->thr[r] : 0;
          }
          const uint64_t zm = cr->zm, cm = cr->cm;
          pre = true;
#pragma unroll
          for (uint32_t r = 0; r < RMAX; r++) pre = pre && (r >= R || tot[r] + rq[r] <= mx[r]);
          if (pre && vr.fk_count) pre = var_fk_ok(d, vr, d.c_fk + (size_t)j * F);
          if (pre) {
            const uint64_t G = grid_of(zm & vr.zm, cm & vr.cm, d.Z, d.C);
            const uint64_t Gt = grid_of(s_tzm[t] & vr.zm, s_tcm[t] & vr.cm, d.Z, d.C);
            uint32_t mrow[RMAX];
#pragma unroll
            for (uint32_t r = 0; r < RMAX; r++) {
              mrow[r] = 0;
              if (r < R) {
                const uint32_t o = d.thr_off[r], n = d.thr_off[r + 1] - o;
                mrow[r] = o + r + thr_probe(thr + o, n, cur[r], tot[r] + rq[r]);
              }
            }
            const uint64_t* row = d.rows + ((size_t)v * T + t) * W;
            const uint64_t* opts = d.c_opts + (size_t)j * W;
            bool any = false;
            for (uint32_t w = 0; w < W && !any; w++) {
              uint64_t x = opts[w] & row[w];
#pragma unroll
              for (uint32_t r = 0; r < RMAX; r++)
                if (r < R) x &= d.thr_set[(size_t)mrow[r] * W + w];
              if (x && G != Gt) {
                uint64_t y = 0, m = x;
                while (m) {
                  const uint32_t b = __ffsll((long long)m) - 1;
                  m &= m - 1;
                  if (d.it_pair[w * 64 + b] & G) y |= 1ull << b;
                }
                x = y;
              }
              any = x != 0;
            }
            feas = any;
          }
        }
      }
      const uint64_t pm = __ballot(pre);
      if ((tid & 63) == 0 && pm) atomicAdd((unsigned long long*)&S.cand_full, (unsigned long long)__popcll(pm));
      uint64_t tq = 0;
      if (tid == 0) tq = wall_clock64();
      f = blk.bmin(feas ? pos : INF);
      if (tid == 0) {
        const uint64_t tr_ = wall_clock64();
        S.dbg[0] += tq - tA;
        S.dbg[1] += tr_ - tq;
        S.dbg[2]++;
        tA = tr_;
        S.cand += (M - base) < FB ? (M - base) : FB;
      }
      if (f != INF) break;
    }
    if (f != INF) {
      // NodeClaim.Add, block-parallel: options words, totals/cursors, keys
      const uint32_t j = s_ord[f], t = s_tmpl[j];
      ClaimRec* cr = d.c_rec + j;
      const uint64_t G = grid_of(cr->zm & vr.zm, cr->cm & vr.cm, d.Z, d.C);
      const uint64_t Gt = grid_of(s_tzm[t] & vr.zm, s_tcm[t] & vr.cm, d.Z, d.C);
      uint32_t mrow[RMAX];
#pragma unroll
      for (uint32_t r = 0; r < RMAX; r++) {
        mrow[r] = 0;
        if (r < R) {
          const uint32_t o = d.thr_off[r], n = d.thr_off[r + 1] - o;
          mrow[r] = o + r + thr_probe(thr + o, n, cr->thr[r], cr->tot[r] + rq[r]);
        }
      }
      __syncthreads();  // every lane has read the record before it changes
      const uint64_t* row = d.rows + ((size_t)v * T + t) * W;
      uint64_t* opts = d.c_opts + (size_t)j * W;
      for (uint32_t w = tid; w < W; w += FB) {
        uint64_t x = opts[w] & row[w];
#pragma unroll
        for (uint32_t r = 0; r < RMAX; r++)
          if (r < R) x &= d.thr_set[(size_t)mrow[r] * W + w];
        if (G != Gt) {
          uint64_t off = 0, gm = G;
          while (gm) {
            const uint32_t g = __ffsll((long long)gm) - 1;
            gm &= gm - 1;
            off |= d.slot_set[(size_t)g * W + w];
          }
          x &= off;
        }
        opts[w] = x;
      }
      if (tid >= 64 && tid < 64 + R) {
        const uint32_t r = tid - 64;
        cr->tot[r] += preq[r];
        cr->thr[r] = (uint16_t)(mrow[r] - d.thr_off[r] - r);
      }
      if (tid >= 128 && tid < 128 + vr.fk_count) {
        const FKEntry& e = d.fk_entries[vr.fk_begin + (tid - 128)];
        FK* cf = d.c_fk + (size_t)j * F + e.slot;
        const FK cur = *cf;
        *cf = (cur.flags & FK_PRESENT) ? fk_intersect(cur, e.st, d.fk_ival + (size_t)e.slot * 64, d.fk_isint[e.slot])
                                       : e.st;
      }
      if (tid == 0) {
        cr->zm &= vr.zm;
        cr->cm &= vr.cm;
        cr->count++;
        if (s_sc[f] == 0xFFFFu) S.status = 3;
        s_sc[f]++;
        S.modkind = MOD_INC;
        S.modpos = f;
        d.log[S.nlog++] = LogRec{p, v, j, 0};
        S.found = 1;
      }
    }
    __syncthreads();
    if (tid == 0) {
      const uint64_t tB = wall_clock64();
      S.t_scan += tB - tA;
      tA = tB;
    }
    if (S.found) {
      if (S.status) break;
      continue;
    }

    // ------------------------------- new NodeClaim from templates, in order
    for (uint32_t t = 0; t < T; t++) {
      const TmplRec& tr = d.tmpl[t];
      const uint64_t* row = d.rows + ((size_t)v * T + t) * W;
      bool any = false;
      if (d.fk_ok[(size_t)v * T + t])
        for (uint32_t w = 0; w < W; w++)
          if (row[w]) any = true;
      if (!any) continue;
      if (tr.has_limits) {
        // <U> filterByRemainingResources on the template's options
        uint32_t hit = INF;
        for (uint32_t i = tid; i < d.N; i += FB) {
          if (!((row[i >> 6] >> (i & 63)) & 1)) continue;
          bool ok = true;
          for (uint32_t r = 0; r < R; r++)
            if ((tr.limit_rmask >> r) & 1) ok = ok && d.it_cap[(size_t)r * d.N + i] <= d.t_rem[(size_t)t * R + r];
          if (ok) hit = 0;
        }
        if (blk.bmin(hit) == INF) continue;
      }
      if (M >= MC) {
        if (tid == 0) S.status = 1;
        __syncthreads();
        break;
      }
      const uint32_t j = M;
      ClaimRec* cr = d.c_rec + j;
      for (uint32_t w = tid; w < W; w += FB) {
        uint64_t x = row[w];
        if (tr.has_limits) {
          uint64_t y = 0, m = x;
          while (m) {
            const uint32_t b = __ffsll((long long)m) - 1;
            m &= m - 1;
            const uint32_t i = w * 64 + b;
            bool ok = true;
            for (uint32_t r = 0; r < R; r++)
              if ((tr.limit_rmask >> r) & 1) ok = ok && d.it_cap[(size_t)r * d.N + i] <= d.t_rem[(size_t)t * R + r];
            if (ok) y |= 1ull << b;
          }
          x = y;
        }
        d.c_opts[(size_t)j * W + w] = x;
      }
      if (tid < RMAX) {
        int64_t tot = 0;
        uint32_t c0 = 0;
        if (tid < R) {
          tot = tr.daemon[tid] + preq[tid];
          const uint32_t o = d.thr_off[tid], n = d.thr_off[tid + 1] - o;
          c0 = thr_probe(thr + o, n, 0, tot);
        }
        cr->tot[tid] = tot;
        cr->thr[tid] = (uint16_t)c0;
        S.red64[tid] = 0;
      }
      if (tid == 0) {
        cr->tmpl = t;
        cr->count = 1;
        cr->zm = tr.zm & vr.zm;
        cr->cm = tr.cm & vr.cm;
        FK* cf = d.c_fk + (size_t)j * F;
        for (uint32_t s = 0; s < F; s++) cf[s] = d.t_fk[(size_t)t * F + s];
        for (uint32_t k = 0; k < vr.fk_count; k++) {
          const FKEntry& e = d.fk_entries[vr.fk_begin + k];
          const FK cur = cf[e.slot];
          cf[e.slot] = (cur.flags & FK_PRESENT)
                           ? fk_intersect(cur, e.st, d.fk_ival + (size_t)e.slot * 64, d.fk_isint[e.slot])
                           : e.st;
        }
        s_ord[M] = (uint16_t)M;
        s_sc[M] = 1;
        s_tmpl[M] = (uint8_t)t;
        S.M = M + 1;
        S.modkind = MOD_APPEND;
        d.log[S.nlog++] = LogRec{p, v, j, 0};
        S.found = 1;
      }
      __syncthreads();
      // max allocatable over the new claim's options (the slack bound)
      for (uint32_t i = tid; i < d.N; i += FB) {
        if (!((d.c_opts[(size_t)j * W + (i >> 6)] >> (i & 63)) & 1)) continue;
        for (uint32_t r = 0; r < R; r++) atomicMax(&S.red64[r], (unsigned long long)d.it_alloc[(size_t)r * d.N + i]);
      }
      __syncthreads();
      if (tid < RMAX) cr->maxa[tid] = tid < R ? (int64_t)S.red64[tid] : 0;
      __syncthreads();
      if (tr.has_limits) {
        // <U> subtractMax(remaining, nodeClaim.InstanceTypeOptions)
        if (tid < R) S.red64[tid] = 0;
        __syncthreads();
        for (uint32_t i = tid; i < d.N; i += FB) {
          if (!((d.c_opts[(size_t)j * W + (i >> 6)] >> (i & 63)) & 1)) continue;
          for (uint32_t r = 0; r < R; r++)
            if ((tr.limit_rmask >> r) & 1)
              atomicMax(&S.red64[r], (unsigned long long)(d.it_cap[(size_t)r * d.N + i] + (1ll << 62)));
        }
        __syncthreads();
        if (tid < R && ((tr.limit_rmask >> tid) & 1) && S.red64[tid] != 0)
          d.t_rem[(size_t)t * R + tid] -= (int64_t)(S.red64[tid] - (1ull << 62));
      }
      __syncthreads();
      break;
    }
    __syncthreads();
    if (tid == 0) S.t_tmpl += wall_clock64() - tA;
    if (S.status) break;
    if (S.found) continue;

    // ------------------------------------ failed: Relax, then Queue.Push
    if (tid == 0) {
      bool relaxed = false;
      if (v + 1 < d.var_begin[p] + d.var_count[p]) {
        d.cur_var[p] = v + 1;
        relaxed = true;
      }
      uint32_t tail = S.qhead + S.qlen;
      if (tail >= P) tail -= P;
      d.queue[tail] = p;
      S.qlen++;
      if (relaxed) {
        S.epoch++;
      } else {
        d.last_epoch[p] = S.epoch;
        d.last_len[p] = S.qlen;
      }
    }
    __syncthreads();
  }

  __syncthreads();
  for (uint32_t i = tid; i < S.M; i += FB) d.c_sorted[i] = s_ord[i];
  if (tid == 0) {
    Ctrl c;
    c.status = S.status;
    c.n_claims = S.M;
    c.n_log = S.nlog;
    c.qhead = S.qhead;
    c.qlen = S.qlen;
    c.epoch = S.epoch;
    c.pops = S.pops;
    c.generic_sorts = S.generic;
    c.fast_sorts = S.fast;
    c.cand_evals = S.cand;
    c.cand_full = S.cand_full;
    c.t_sort = S.t_sort;
    c.t_scan = S.t_scan;
    c.t_tmpl = S.t_tmpl;
    c.t_total = wall_clock64() - S.t0;
    for (int q = 0; q < 8; q++) c.dbg[q] = S.dbg[q];
    *d.ctrl = c;
  }
}

extern "C" uint32_t gsk_ffd_lds_bytes(uint32_t max_claims) {
  return ((7u * max_claims + 7u) & ~7u) + THR_LDS_MAX * 8u;
}

extern "C" hipError_t gsk_init_ffd(uint32_t lds_bytes) {
  return hipFuncSetAttribute((const void*)ffd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
}

extern "C" hipError_t gsk_ffd(const DevProblem* d, hipStream_t s) {
  hipLaunchKernelGGL(ffd_kernel, dim3(1), dim3(FB), gsk_ffd_lds_bytes(d->max_claims), s, *d);
  return hipGetLastError();
}
