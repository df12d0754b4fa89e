// ffd_common.hpp — helpers shared by the two Solve kernels (ffd.hip: block
// kernel for consolidation simulations and node-heavy Solves; ffd_wave.hip:
// the single-wave provisioning Solve): the sequential restatement of Go
// sort.Slice (pdqsort_func), threshold cursors, 16-bit quantity codes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "devutil.hpp"
#include "layout.hpp"

namespace gsd {
namespace {

struct Frame {
  int a, b, limit;
  int wb, wp;  // wasBalanced, wasPartitioned
  int uni;     // WaveSort: every key in [a, b) is known equal (0: unknown)
};

// LDS-qualified element types: a pointer of these types keeps ds_* addressing
// inside functions the compiler does not inline (WaveSort::pdqsort is one
// out-of-line body shared by every wave-kernel instantiation; through a
// generic pointer its LDS accesses become flat_* loads and stores)
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef __attribute__((address_space(3))) Frame lds_frame;

__device__ __forceinline__ int bits_len(uint64_t x) { return x ? 64 - __clzll((long long)x) : 0; }

// ---------------------------------------------------------------- sequential
// Element storage of the sorted NodeClaim order: key = len(Pods) (the
// sort.Slice comparison), payload = claim id.
//  SplitAcc:  u16 keys and u16 payload in two arrays (block kernel)
//  PackedAcc: one u32 per position, key in the low 16 bits (wave kernel: one
//             LDS access moves or reads both)
struct SplitAcc {
  uint16_t* sc;
  uint16_t* ord;
  __device__ __forceinline__ uint32_t key(int i) const { return sc[i]; }
  __device__ __forceinline__ void swap(int i, int j) const {
    uint16_t a = sc[i];
    sc[i] = sc[j];
    sc[j] = a;
    a = ord[i];
    ord[i] = ord[j];
    ord[j] = a;
  }
};
template <class U32>  // lds_u32, or uint32_t (HBM claim state)
struct PackedAccT {
  U32* so;
  __device__ __forceinline__ uint32_t key(int i) const { return so[i] & 0xFFFFu; }
  __device__ __forceinline__ void swap(int i, int j) const {
    const uint32_t a = so[i];
    so[i] = so[j];
    so[j] = a;
  }
};
using PackedAcc = PackedAccT<lds_u32>;

// Go sort.Slice (src/sort/zsortfunc.go) over 16-bit keys, one thread;
// pdq_frame() resumes a pdqsort_func loop from a given frame state.
template <class Acc>
struct SeqSortT {
  Acc acc;
  __device__ bool less(int i, int j) const { return acc.key(i) < acc.key(j); }
  __device__ void swap(int i, int j) const { acc.swap(i, j); }
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
    for (int t = 0; t < 9; t++) key[t] = (l >= 50 || t % 3 == 1) ? (uint16_t)acc.key(idx[t]) : 0;
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

// ------------------------------------------------------------ wave helpers
// compiler barrier for LDS hand-offs between lanes of the one wave: the
// hardware keeps a wave's LDS accesses in order, the compiler must too
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
// the claim scan state's hand-offs between lanes: in LDS the wave's in-order
// LDS queue orders them (wsync); in HBM (G) every store must have completed
// before another lane's load (s_waitcnt 0: a wave's stores and loads share
// the vector memory counter on gfx9, and the CU's write-through L1 serves the
// completed store)
template <bool G>
__device__ __forceinline__ void wsyncT() {
  if (G) __builtin_amdgcn_s_waitcnt(0);
  wsync();
}

// readlane as an unsigned dword (the builtin returns int: widening it
// directly would sign-extend a low dword with bit 31 set)
__device__ __forceinline__ uint32_t rlane(uint32_t x, uint32_t i) {
  return (uint32_t)__builtin_amdgcn_readlane((int)x, (int)i);
}

__device__ __forceinline__ uint32_t ffs64(uint64_t m) { return (uint32_t)__ffsll((long long)m) - 1u; }


// ------------------------------------------------- register-resident sort
// Go's pdqsort_func loop (src/sort/zsortfunc.go, restated sequentially in
// SeqSortT) over a frame of <= 64 elements held one per lane: lane x holds the
// packed element at g + x (key = low 16 bits).  Every data access is a
// readlane / writelane or a cross-lane permute, so the control stays scalar
// and no step waits on an LDS round trip.  The parallel steps are exact:
//  - insertionSort is stable, so a rank (keys below + equal keys before) is
//    its permutation;
//  - partition / partitionEqual swap the k-th misplaced element of the left
//    side (ascending) with the k-th of the right side (descending), as the
//    wave sort's lists do (WaveSort::partition);
//  - partialInsertionSort's two shifts are one rotation each.
// heapSort (limit exhausted, rare) runs SeqSortT on lane 0 over the array.
// A shift left never passes the frame start: every key before it is <= the
// frame's keys (pdqsort's partitions), and Less is strict.
__device__ __forceinline__ uint32_t wlane(uint32_t v, int i, uint32_t x) {
  return (int)(threadIdx.x & 63u) == i ? x : v;  // v_cmp + v_cndmask
}
// position of the r-th (0-based) set bit of m from the bottom; r < popc(m)
__device__ __forceinline__ uint32_t nth_bit(uint64_t m, uint32_t r) {
  uint32_t pos = 0;
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const uint32_t c = (uint32_t)__popcll(m & ((1ull << w) - 1ull));
    const bool up = r >= c;
    r = up ? r - c : r;
    m = up ? m >> w : m;
    pos += up ? (uint32_t)w : 0u;
  }
  return pos;
}
// the array a RegSort frame lives in: packed u32 words (the wave Solve's
// order, LDS or HBM)
template <class U32, bool G>
struct PackedArr {
  U32* so;
  __device__ __forceinline__ uint32_t load(int i) const { return (uint32_t)so[i]; }
  __device__ __forceinline__ void store(int i, uint32_t v) const { so[i] = v; }
  __device__ __forceinline__ void heap_sort(int a, int b) const { SeqSortT<PackedAccT<U32>>{{so}}.heap_sort(a, b); }
  __device__ __forceinline__ void sync() const { wsyncT<G>(); }
};
template <class Arr>
struct RegSort {
  uint32_t v;      // lane x: element g + x
  uint32_t lane;
  int g;           // the frame's first array position
  uint32_t prevk;  // key at g - 1 (g > 0): never moved while this frame runs

  __device__ __forceinline__ uint32_t key(int i) const { return rlane(v, (uint32_t)i) & 0xFFFFu; }
  __device__ __forceinline__ void swap(int i, int j) {
    const uint32_t x = rlane(v, (uint32_t)i), y = rlane(v, (uint32_t)j);
    v = wlane(v, i, y);
    v = wlane(v, j, x);
  }
  // stable: rank = keys below + equal keys at lower positions
  __device__ void insertion_sort(int a, int b) {
    const uint32_t k = v & 0xFFFFu;
    int r = a;
    for (int j = a; j < b; j++) {
      const uint32_t kj = key(j);
      r += (kj < k || (kj == k && j < (int)lane)) ? 1 : 0;
    }
    const bool in = (int)lane >= a && (int)lane < b;
    v = (uint32_t)__builtin_amdgcn_ds_permute((in ? r : (int)lane) * 4, (int)v);
  }
  // the misplaced pairs of a partition with left side (a, mid]: lanes of lm
  // (ascending) trade with lanes of rm (descending), k-th with k-th
  __device__ void swap_misplaced(uint64_t lm, uint64_t rm) {
    const uint64_t me = 1ull << lane;
    const uint64_t below = me - 1ull;
    uint32_t partner = lane;
    if (lm & me) {
      const uint32_t r = (uint32_t)__popcll(lm & below);
      partner = nth_bit(rm, (uint32_t)__popcll(rm) - 1u - r);
    } else if (rm & me) {
      const uint32_t r = (uint32_t)__popcll(rm & ~below & ~me);
      partner = nth_bit(lm, r);
    }
    v = (uint32_t)__shfl((int)v, (int)partner);
  }
  __device__ int partition(int a, int b, int pivot, bool* already) {
    swap(a, pivot);
    const uint32_t p = key(a), k = v & 0xFFFFu;
    const bool inr = (int)lane > a && (int)lane < b;
    const bool lt = k < p;
    const int mid = a + (int)__popcll(__ballot(inr && lt));
    const bool inl = (int)lane > a && (int)lane <= mid;
    const uint64_t lm = __ballot(inl && !lt), rm = __ballot(inr && !inl && lt);
    if (lm) swap_misplaced(lm, rm);
    swap(mid, a);
    *already = lm == 0;
    return mid;
  }
  __device__ int partition_equal(int a, int b, int pivot) {
    swap(a, pivot);
    const uint32_t p = key(a), k = v & 0xFFFFu;
    const bool inr = (int)lane > a && (int)lane < b;
    const bool le = k <= p;
    const int mid = a + (int)__popcll(__ballot(inr && le));
    const bool inl = (int)lane > a && (int)lane <= mid;
    const uint64_t lm = __ballot(inl && !le), rm = __ballot(inr && !inl && le);
    if (lm) swap_misplaced(lm, rm);
    return mid + 1;
  }
  __device__ void reverse_range(int a, int b) {
    const bool in = (int)lane >= a && (int)lane < b;
    v = (uint32_t)__shfl((int)v, in ? a + b - 1 - (int)lane : (int)lane);
  }
  // the element at hi moves to lo, [lo, hi) one position up
  __device__ void rotate_up(int lo, int hi) {
    const uint32_t x = rlane(v, (uint32_t)hi);
    const bool in = (int)lane > lo && (int)lane <= hi;
    const uint32_t y = (uint32_t)__shfl((int)v, in ? (int)lane - 1 : (int)lane);
    v = (int)lane == lo ? x : y;
  }
  // the element at lo moves to hi, (lo, hi] one position down
  __device__ void rotate_down(int lo, int hi) {
    const uint32_t x = rlane(v, (uint32_t)lo);
    const bool in = (int)lane >= lo && (int)lane < hi;
    const uint32_t y = (uint32_t)__shfl((int)v, in ? (int)lane + 1 : (int)lane);
    v = (int)lane == hi ? x : y;
  }
  __device__ bool partial_insertion_sort(int a, int b) {
    int i = a + 1;
    for (int j = 0; j < 5; j++) {
      const uint32_t k = v & 0xFFFFu;
      const uint32_t pk = (uint32_t)__shfl((int)v, (int)lane - 1) & 0xFFFFu;
      const uint64_t inv = __ballot((int)lane >= i && (int)lane < b && k < pk);
      if (!inv) return true;
      i = (int)ffs64(inv);
      if (b - a < 50) return false;
      swap(i, i - 1);
      if (i - a >= 2) {
        // the smaller element (at i - 1) passes the strictly greater ones
        const uint32_t x = key(i - 1);
        const uint64_t hm = __ballot((int)lane <= i - 2 && (v & 0xFFFFu) <= x);
        const int q = hm ? 63 - (int)__clzll((long long)hm) : -1;
        rotate_up(q + 1, i - 1);
      }
      if (b - i >= 2) {
        // the greater element (at i) passes the strictly smaller ones
        const uint32_t y = key(i);
        const uint64_t em = __ballot((int)lane > i && (int)lane < b && (v & 0xFFFFu) >= y);
        const int e = em ? (int)ffs64(em) : b;
        rotate_down(i, e - 1);
      }
    }
    return false;
  }
  __device__ void break_patterns(int a, int b) {
    const int length = b - a;
    if (length >= 8) {
      uint64_t r = (uint64_t)length;
      const uint64_t modulus = 1ull << bits_len((uint64_t)length);
      const int idx = a + (length / 4) * 2 - 1;
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
  __device__ int choose_pivot(int a, int b, int* hint) const {
    const int l = b - a;
    int swaps = 0;
    int i = a + l / 4 * 1, j = a + l / 4 * 2, k = a + l / 4 * 3;
    auto med = [&](int x, int y, int z) {
      if (key(y) < key(x)) { swaps++; const int t = x; x = y; y = t; }
      if (key(z) < key(y)) { swaps++; const int t = y; y = z; z = t; }
      if (key(y) < key(x)) { swaps++; const int t = x; x = y; y = t; }
      return y;
    };
    if (l >= 8) {
      if (l >= 50) {
        i = med(i - 1, i, i + 1);
        j = med(j - 1, j, j + 1);
        k = med(k - 1, k, k + 1);
      }
      j = med(i, j, k);
    }
    *hint = swaps == 0 ? 1 : (swaps == 12 ? 2 : 0);
    return j;
  }
  __device__ void heap_sort(const Arr& arr, int a, int b) {
    if ((int)lane < b && (int)lane >= a) arr.store(g + (int)lane, v);
    arr.sync();
    if (lane == 0) arr.heap_sort(g + a, g + b);
    arr.sync();
    if ((int)lane < b && (int)lane >= a) v = arr.load(g + (int)lane);
    arr.sync();
  }
  // pdqsort_func's loop from frame f (array positions), recursion on a stack
  // of packed frames in one VGPR (depth <= 6 for 64 elements)
  __device__ void run(const Arr& arr, Frame f) {
    int a = f.a - g, b = f.b - g, limit = f.limit, wb = f.wb, wp = f.wp;
    uint32_t stk = 0;
    int sp = 0;
    for (;;) {
      for (;;) {
        // wave-uniform loop state (scalar registers and branches)
        a = __builtin_amdgcn_readfirstlane(a);
        b = __builtin_amdgcn_readfirstlane(b);
        limit = __builtin_amdgcn_readfirstlane(limit);
        wb = __builtin_amdgcn_readfirstlane(wb);
        wp = __builtin_amdgcn_readfirstlane(wp);
        const int length = b - a;
        if (length <= 12) {
          insertion_sort(a, b);
          break;
        }
        if (limit == 0) {
          heap_sort(arr, a, b);
          break;
        }
        if (!wb) {
          break_patterns(a, b);
          limit--;
        }
        int hint;
        int pivot = choose_pivot(a, b, &hint);
        if (hint == 2) {
          reverse_range(a, b);
          pivot = (b - 1) - (pivot - a);
          hint = 1;
        }
        if (wb && wp && hint == 1 && partial_insertion_sort(a, b)) break;
        if (g + a > 0 && !((a > 0 ? key(a - 1) : prevk) < key(pivot))) {
          a = partition_equal(a, b, pivot);
          continue;
        }
        bool already;
        const int mid = partition(a, b, pivot, &already);
        wp = already ? 1 : 0;
        const int left_len = mid - a, right_len = b - mid, bal = length / 8;
        int ca, cb;
        if (left_len < right_len) {
          wb = left_len >= bal;
          ca = a;
          cb = mid;
          a = mid + 1;
        } else {
          wb = right_len >= bal;
          ca = mid + 1;
          cb = b;
          b = mid;
        }
        // Go recurses into the smaller side first (fresh wasBalanced /
        // wasPartitioned), then continues this frame
        stk = wlane(stk, sp, (uint32_t)a | (uint32_t)b << 8 | (uint32_t)limit << 16 | (uint32_t)wb << 24 |
                                 (uint32_t)wp << 25);
        sp++;
        a = ca;
        b = cb;
        wb = 1;
        wp = 1;
      }
      sp = __builtin_amdgcn_readfirstlane(sp);
      if (sp == 0) break;
      sp--;
      const uint32_t e = rlane(stk, (uint32_t)sp);
      a = (int)(e & 0xFFu);
      b = (int)((e >> 8) & 0xFFu);
      limit = (int)((e >> 16) & 0xFFu);
      wb = (int)((e >> 24) & 1u);
      wp = (int)((e >> 25) & 1u);
    }
  }
};
// the frame [f.a, f.b) (f.b - f.a <= 64) through RegSort, on one wave: out
// of line, scalar arguments (no `this` in scratch)
template <class Arr>
__device__ __noinline__ void reg_pdq_frame(Arr arr, int fa, int fb, int limit, int wb, int wp) {
  // arguments arrive in VGPRs: made wave-uniform, so the control flow below
  // compiles to scalar branches instead of exec-masked divergent loops
  fa = __builtin_amdgcn_readfirstlane(fa);
  fb = __builtin_amdgcn_readfirstlane(fb);
  limit = __builtin_amdgcn_readfirstlane(limit);
  wb = __builtin_amdgcn_readfirstlane(wb);
  wp = __builtin_amdgcn_readfirstlane(wp);
  const uint32_t lane = threadIdx.x & 63u;
  const int n = fb - fa;
  const uint32_t prevk = fa > 0 ? (uint32_t)__builtin_amdgcn_readfirstlane((int)arr.load(fa - 1)) & 0xFFFFu : 0u;
  RegSort<Arr> r{(int)lane < n ? arr.load(fa + (int)lane) : 0u, lane, fa, prevk};
  r.run(arr, Frame{fa, fb, limit, wb, wp, 0});
  if ((int)lane < n) arr.store(fa + (int)lane, r.v);
  arr.sync();
}

// first m in [m0, n) with thr[m] >= x (thresholds ascending); n if none
// Cursor advance over one resource's ascending thresholds: the first m >= m0
// with thr[m] >= x.  A 4-wide window read in one LDS round trip covers the
// common case; thr has 4 readable entries past every range.
using SeqSort = SeqSortT<SplitAcc>;
using SeqSortP = SeqSortT<PackedAcc>;
using SeqSortPG = SeqSortT<PackedAccT<uint32_t>>;

__device__ __forceinline__ uint32_t thr_window(const int64_t* thr, uint32_t n, uint32_t m0, int64_t x) {
  uint32_t m = m0;
#pragma unroll
  for (uint32_t k = 0; k < 4; k++) {
    const int64_t vk = thr[m0 + k];  // unconditional: the padded LDS copy covers m0 + 3
    m += (m0 + k < n && vk < x) ? 1u : 0u;
  }
  return m;
}

__device__ __forceinline__ uint32_t thr_search(const int64_t* thr, uint32_t n, uint32_t lo, int64_t x) {
  uint32_t hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (thr[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// choosePivot's hint for sort.Slice over sc[0, M), M > 12: the (up to) nine
// sampled keys read by nine lanes in one LDS round trip, the median-of-three
// comparisons on scalars (same swap count as SeqSort::choose_pivot)
template <class Acc>
__device__ __forceinline__ int pivot_hint_wave(const Acc& acc, int l, uint32_t lane) {
  const int i0 = l / 4 * 1, j0 = l / 4 * 2, k0 = l / 4 * 3;
  const int idx[9] = {i0 - 1, i0, i0 + 1, j0 - 1, j0, j0 + 1, k0 - 1, k0, k0 + 1};
  int mine = 0;
#pragma unroll
  for (int t = 0; t < 9; t++)
    if ((int)lane == t) mine = idx[t];
  const uint32_t kl = lane < 9 && (l >= 50 || lane % 3 == 1) ? acc.key(mine) : 0u;
  uint32_t key[9];
#pragma unroll
  for (int t = 0; t < 9; t++) key[t] = __builtin_amdgcn_readlane(kl, t);
  int swaps = 0;
  auto med = [&](uint32_t kx, uint32_t ky, uint32_t kz) {
    // order2(x,y); order2(y,z); order2(x,y); the middle key
    if (ky < kx) { swaps++; const uint32_t u = kx; kx = ky; ky = u; }
    if (kz < ky) { swaps++; const uint32_t u = ky; ky = kz; kz = u; }
    if (ky < kx) { swaps++; const uint32_t u = kx; kx = ky; ky = u; }
    return ky;
  };
  uint32_t ki = key[1], kj = key[4], kk = key[7];
  if (l >= 50) {
    ki = med(key[0], key[1], key[2]);
    kj = med(key[3], key[4], key[5]);
    kk = med(key[6], key[7], key[8]);
  }
  med(ki, kj, kk);
  return swaps == 0 ? 1 : (swaps == 12 ? 2 : 0);
}

// first k in [lo, hi) with pred(k) for a monotone pred (false...true), hi if
// none: a 64-ary search, one LDS round trip per level (two up to 4096)
template <class Pred>
__device__ __forceinline__ uint32_t wave_first(uint32_t lo, uint32_t hi, uint32_t lane, Pred pred) {
  while (hi - lo > 64) {
    const uint32_t step = (hi - lo + 63) / 64;
    const uint32_t k = lo + lane * step + step - 1;  // last index of this lane's segment
    const uint64_t b = __ballot(k >= hi || pred(k));
    if (!b) return hi;
    const uint32_t i = (uint32_t)__ffsll((long long)b) - 1;
    lo = lo + i * step;
    hi = lo + step < hi ? lo + step : hi;
  }
  const uint32_t k = lo + lane;
  const uint64_t b = __ballot(k < hi && pred(k));
  return b ? lo + (uint32_t)__ffsll((long long)b) - 1 : hi;
}

// phase timers (t_sort / t_scan / t_tmpl, Ctrl.dbg): s_memrealtime costs
// hundreds of cycles on the pod loop's critical path, so only GS_FFD_PHASES
// builds read the clock
__device__ __forceinline__ uint64_t phase_clock() {
#ifdef GS_FFD_PHASES
  return wall_clock64();
#else
  return 0;
#endif
}

// the kernel argument block, addressed in the constant (kernarg) space
typedef const __attribute__((address_space(4))) DevProblem* KArg;

// wave-uniform 64-bit value into SGPRs (readfirstlane is 32-bit)
__device__ __forceinline__ int64_t uniform_i64(int64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)x >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// Monotone 16-bit code of a non-negative quantity: exact below 1024, then a
// 9-bit mantissa per binade (relative step <= 2^-9).  codes are consecutive
// in value order, so floor/ceil differ by at most one.
__device__ __forceinline__ uint32_t qcode_floor(int64_t v) {
  if (v <= 0) return 0;
  const uint64_t x = (uint64_t)v;
  const uint32_t b = 64u - (uint32_t)__clzll((long long)x);
  if (b <= 10) return (uint32_t)x;
  const uint32_t s = b - 10;
  return 1024u + (s - 1) * 512u + (uint32_t)((x >> s) - 512u);
}
__device__ __forceinline__ uint32_t qcode_ceil(int64_t v) {
  if (v <= 0) return 0;
  const uint64_t x = (uint64_t)v;
  const uint32_t b = 64u - (uint32_t)__clzll((long long)x);
  if (b <= 10) return (uint32_t)x;
  const uint32_t s = b - 10;
  const uint32_t c = 1024u + (s - 1) * 512u + (uint32_t)((x >> s) - 512u);
  return c + ((x & ((1ull << s) - 1)) ? 1u : 0u);
}

// the value a code stands for: qcode_floor(v) <= v's code <= qcode_ceil(v)
// and qcode_value(qcode_floor(v)) <= v <= qcode_value(qcode_ceil(v))
__device__ __forceinline__ int64_t qcode_value(uint32_t c) {
  if (c < 1024u) return (int64_t)c;
  const uint32_t s = (c - 1024u) / 512u + 1u, m = (c - 1024u) % 512u + 512u;
  return (int64_t)((uint64_t)m << s);
}

// LDS room of a NodeClaim: qcode_floor(thr[cursor] - tot) per resource (<= 4),
// a lower bound of what a pod may add before any threshold cursor moves
__device__ __forceinline__ uint64_t pack_room(const int64_t* thr, const uint32_t* thoff, const uint32_t* cur,
                                              const int64_t* tot, uint32_t RQ) {
  uint64_t s = 0;
#pragma unroll
  for (uint32_t r = 0; r < 4; r++) {
    if (r >= RQ) break;
    const uint32_t o = thoff[r], n = thoff[r + 1] - o;
    const int64_t room = cur[r] < n ? thr[o + cur[r]] - tot[r] : 0;
    s |= (uint64_t)qcode_floor(room) << (16 * r);
  }
  return s;
}

// LDS slack of a NodeClaim: qcode_ceil(maxa - tot) per resource (<= 4)
template <class DP>
__device__ __forceinline__ uint64_t pack_slack(const DP& d, const int64_t* maxa, const int64_t* tot) {
  uint64_t s = 0;
#pragma unroll
  for (uint32_t r = 0; r < 4; r++) {
    if (r >= d.RQ) break;
    s |= (uint64_t)qcode_ceil(maxa[r] - tot[r]) << (16 * r);
  }
  return s;
}

// <U> InstanceTypes.SatisfiesMinValues (Strict policy) on the template's IT
// keys: the distinct values of key k over an option set reach tr.mv[k].
// word(w) yields the set's w-th word; the caller keeps word() uniform when
// it evaluates per wave.  Keys with a distinct value per type count types;
// the others OR dense value ids (< 256, checked by the encoder) into a
// 256-bit set.  Every loop stops once the minimum is reached.
template <class DP, class WordFn>
__device__ inline bool mv_ok(const DP& d, const TmplRec& tr, WordFn word) {
  for (uint32_t mm = tr.mv_mask; mm; mm &= mm - 1) {
    const uint32_t k = (uint32_t)__builtin_ctz(mm);
    const uint32_t need = tr.mv[k];
    uint32_t n = 0;
    if ((d.it_key_unique >> k) & 1) {
      for (uint32_t w = 0; w < d.W && n < need; w++) n += (uint32_t)__popcll(word(w));
    } else {
      const uint16_t* dv = d.it_dvid + (size_t)k * d.N;
      uint64_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
      for (uint32_t w = 0; w < d.W && n < need; w++)
        for (uint64_t m = word(w); m && n < need; m &= m - 1) {
          const uint32_t x = dv[w * 64 + (uint32_t)__builtin_ctzll(m)];
          const uint32_t q = x >> 6;
          const uint64_t bit = 1ull << (x & 63);
          const uint64_t cur = q == 0 ? s0 : q == 1 ? s1 : q == 2 ? s2 : s3;
          if (!(cur & bit)) {
            n++;
            s0 |= q == 0 ? bit : 0;
            s1 |= q == 1 ? bit : 0;
            s2 |= q == 2 ? bit : 0;
            s3 |= q == 3 ? bit : 0;
          }
        }
    }
    if (n < need) return false;
  }
  return true;
}

// ---------------------------------------------------------------- topology
// <U> Topology state of one Solve in LDS (layout.hpp topo_lds_bytes): known
// domains per zone group, the current pod's minimum count per owned group
// (domainMinCount, by own-list index), zone counts per zone group, and per
// hostname group the count over all domains (pod affinity's bootstrap rule).
// Hostname counts per existing node / NodeClaim stay in global memory (hn,
// hc); the callers pass them in as functors.
struct TopoS {
  uint64_t* known;  // [TGZ]
  int64_t* tmin;    // [OWNMAX]
  int32_t* zcnt;    // [TGZ][ZS]
  int32_t* htot;    // [TGH]
  uint64_t* lazy;   // [(n_lazy + 63) / 64] the lazy groups (TK_LAZY) some pod has relaxed into
  int32_t* lmind;   // [n_lazy] their minDomains (the creating pod's)
};
__device__ __forceinline__ TopoS topo_lds(char* base, uint32_t tgz, uint32_t zs, uint32_t tgh, uint32_t nl) {
  TopoS t;
  t.known = (uint64_t*)base;
  t.tmin = (int64_t*)(base + tgz * 8u);
  t.zcnt = (int32_t*)(base + tgz * 8u + (uint32_t)OWNMAX * 8u);
  t.htot = (int32_t*)(base + tgz * 8u + (uint32_t)OWNMAX * 8u + tgz * zs * 4u);
  t.lazy = (uint64_t*)(base + topo_lazy_off(tgz, zs, tgh));
  t.lmind = (int32_t*)(base + topo_lazy_off(tgz, zs, tgh) + ((nl + 63u) / 64u) * 8u);
  return t;
}

// the counts before the Solve; i/stride: this thread's share
template <class DP>
__device__ __forceinline__ void topo_init(const DP& d, const TopoS& ts, uint64_t known0, uint32_t i, uint32_t stride) {
  for (uint32_t k = i; k < d.TGZ * d.ZS; k += stride) ts.zcnt[k] = d.zcnt0[k];
  for (uint32_t k = i; k < d.TGZ; k += stride) ts.known[k] = known0;
  for (uint32_t k = i; k < d.TGH; k += stride) ts.htot[k] = d.htot0[k];
  for (uint32_t k = i; k < (d.n_lazy + 63u) / 64u; k += stride) ts.lazy[k] = 0;
}

// <U> Topology.Update after Relax: the lazy groups the pod's new variant
// owns that no pod created before exist from now on, with that pod's
// minDomains: Record counts into them, and the in-flight NodeClaims [0, M)
// are no domains of the hostname ones among them (Topology.Register ran
// before the group existed).  i / stride: this thread's share of the marks;
// thread i == 0 sets the created bits (the caller orders the threads: a
// wave's own program order, or a barrier)
template <class DP>
__device__ __forceinline__ void topo_relaxed(const DP& d, const TopoS& ts, uint32_t new_var, int32_t* hc_rows, uint32_t M,
                                             uint32_t i, uint32_t stride) {
  const uint32_t b = d.var_lz_off[2u * new_var], e = d.var_lz_off[2u * new_var + 1u];
  for (uint32_t k = b; k < e; k++) {
    const uint32_t li = d.lz_idx[k];
    if ((ts.lazy[li >> 6] >> (li & 63u)) & 1ull) continue;
    const uint32_t s = d.lazy_slot[li];
    if (s & LZ_HOST)
      for (uint32_t j = i; j < M; j += stride) hc_rows[(size_t)j * d.TGH + (s & 0xFFFFu)] = HC_UNKNOWN;
    if (i == 0) {
      ts.lmind[li] = d.lz_mind[k];
      ts.lazy[li >> 6] |= 1ull << (li & 63u);
    }
  }
}
// a simulation's end: the cells topo_relaxed marked go back to zero (the
// NodeClaims' hostname rows are zero at rest)
template <class DP>
__device__ __forceinline__ void topo_unmark(const DP& d, const TopoS& ts, int32_t* hc_rows, uint32_t M, uint32_t i,
                                            uint32_t stride) {
  for (uint32_t w = 0; w < (d.n_lazy + 63u) / 64u; w++)
    for (uint64_t x = ts.lazy[w]; x; x &= x - 1) {
      const uint32_t s = d.lazy_slot[w * 64u + (uint32_t)__ffsll((long long)x) - 1u];
      if (s & LZ_HOST)
        for (uint32_t j = i; j < M; j += stride) hc_rows[(size_t)j * d.TGH + (s & 0xFFFFu)] = 0;
    }
}

// domainMinCount of every owned zone spread group over the pod's strict zone
// domains vzs; lane k < own_n (<= OWNMAX) handles own-list entry k
template <class DP>
__device__ __forceinline__ void topo_tmin(const DP& d, const TopoS& ts, uint32_t own_off, uint32_t own_n, uint64_t vzs,
                                          uint32_t lane) {
  if (lane >= own_n) return;
  const TGroupRec& tr = d.tgroups[d.tg_list[own_off + lane] & TL_GID];
  if (tr.kind & (TK_HOST | TK_ANTI)) return;
  const uint64_t cand = ts.known[tr.slot] & vzs;
  int64_t mn = INT32_MAX;
  int32_t n = 0;
  for (uint64_t m = cand; m; m &= m - 1) {
    n++;
    const int64_t c = ts.zcnt[tr.slot * d.ZS + (uint32_t)__ffsll((long long)m) - 1u];
    mn = c < mn ? c : mn;
  }
  const int32_t mind = tr.mind < 0 ? ts.lmind[-tr.mind - 1] : tr.mind;
  if (mind && n < mind) mn = 0;
  ts.tmin[lane] = mn;
}

// one owned group as the topology checks use it: its own-list entry (group
// id | TL_SELF) and the group's skew, slot and kind
struct OwnG {
  uint32_t e;
  int32_t skew;
  uint32_t slot, kind;
};
// the own list read from HBM at each use (own(k) of an own list at own_off)
template <class DP>
struct OwnMem {
  const DP& d;
  uint32_t own_off;
  __device__ __forceinline__ OwnG operator()(uint32_t k) const {
    const uint32_t e = d.tg_list[own_off + k];
    const TGroupRec& tr = d.tgroups[e & TL_GID];
    return OwnG{e, tr.skew, tr.slot, tr.kind};
  }
};

// <U> Topology.AddRequirements for an existing node: its zone label z is its
// only zone domain (a node without one fails the strict Compatible), its
// hostname count in group slot is hcount(slot)
template <class DP, class HCount, class Own>
__device__ __forceinline__ bool topo_node_ok_g(const DP& d, const TopoS& ts, uint32_t own_n, uint32_t z, HCount hcount,
                                               Own own) {
  for (uint32_t k = 0; k < own_n; k++) {
    const OwnG tr = own(k);
    const uint32_t e = tr.e;
    const int64_t self = (e & TL_SELF) ? 1 : 0;
    if (tr.kind & TK_HOST) {
      const int64_t c = hcount(tr.slot);
      if (tr.kind & TK_AFF) {
        if (!(c > 0 || (ts.htot[tr.slot] == 0 && self))) return false;
      } else if (c + self > tr.skew) {
        return false;
      }
    } else {
      if (z >= d.ZS || !((ts.known[tr.slot] >> z) & 1)) return false;
      const int64_t c = ts.zcnt[tr.slot * d.ZS + z];
      if (tr.kind & TK_ANTI) {
        if (c != 0) return false;
      } else if (c + self - ts.tmin[k] > tr.skew) {
        return false;
      }
    }
  }
  return true;
}
template <class DP, class HCount>
__device__ __forceinline__ bool topo_node_ok(const DP& d, const TopoS& ts, uint32_t own_off, uint32_t own_n, uint32_t z,
                                             HCount hcount) {
  return topo_node_ok_g(d, ts, own_n, z, hcount, OwnMem<DP>{d, own_off});
}

// <U> Topology.AddRequirements for a NodeClaim whose zone domains (claim AND
// pod requirements) are D: every owned zone group's domains, intersected --
// a spread group's minimum-count known domain within maxSkew (nextDomain-
// TopologySpread, ties by name), an anti-affinity group's known domains with
// count 0 (nextDomainAntiAffinity).  Hostname groups test the claim's count
// hcount(slot) (0 on a fresh NodeClaim).  Returns the allowed zone set, ~0 when
// no zone group applies, 0 when some group leaves no domain.
template <class DP, class HCount, class Own>
__device__ __forceinline__ uint64_t topo_claim_g(const DP& d, const TopoS& ts, uint32_t own_n, uint64_t D, HCount hcount,
                                                 Own own) {
  uint64_t allow = ~0ull;
  for (uint32_t k = 0; k < own_n; k++) {
    const OwnG tr = own(k);
    const uint32_t e = tr.e;
    const int64_t self = (e & TL_SELF) ? 1 : 0;
    if (tr.kind & TK_HOST) {
      const int64_t c = hcount(tr.slot);
      const bool ok = (tr.kind & TK_AFF) ? (c > 0 || (ts.htot[tr.slot] == 0 && self)) : c + self <= tr.skew;
      if (!ok) return 0;
      continue;
    }
    const uint64_t cand = D & ts.known[tr.slot];
    uint64_t m = 0;
    if (tr.kind & TK_ANTI) {
      for (uint64_t x = cand; x; x &= x - 1) {
        const uint32_t z = (uint32_t)__ffsll((long long)x) - 1u;
        if (ts.zcnt[tr.slot * d.ZS + z] == 0) m |= 1ull << z;
      }
    } else if (cand) {
      const int64_t mn = ts.tmin[k], skew = tr.skew;
      uint32_t best = NONE;
      int64_t bc = INT32_MAX;
      for (uint32_t q = 0; q < d.NZV; q++) {
        const uint32_t z = d.zone_order[q];
        if (!((cand >> z) & 1)) continue;
        const int64_t c = (int64_t)ts.zcnt[tr.slot * d.ZS + z] + self;
        if (c - mn <= skew && c < bc) {
          best = z;
          bc = c;
        }
      }
      m = best == NONE ? 0 : 1ull << best;
    }
    allow &= m;
    if (!allow) return 0;
  }
  return allow;
}
template <class DP, class HCount>
__device__ __forceinline__ uint64_t topo_claim(const DP& d, const TopoS& ts, uint32_t own_off, uint32_t own_n, uint64_t D,
                                               HCount hcount) {
  return topo_claim_g(d, ts, own_n, D, hcount, OwnMem<DP>{d, own_off});
}

// catalog zone mask of a zone-vocabulary set (zones outside the catalog have no offerings)
template <class DP>
__device__ __forceinline__ uint64_t topo_catmask(const DP& d, uint64_t zset) {
  uint64_t c = 0;
  for (uint64_t x = zset; x; x &= x - 1) {
    const uint32_t zc = d.zone_cat[(uint32_t)__ffsll((long long)x) - 1u];
    if (zc < 64) c |= 1ull << zc;
  }
  return c;
}

// <U> Topology.Record: every group selecting the pod counts the domain it
// landed in -- a hostname group the target's own count (hinc(slot)), a zone
// spread group a single non-complement zone, an anti-affinity group (or its
// inverse) every zone of a non-complement requirement (zf, zl: the target's
// zone Has and flags; an existing node: its label)
template <class DP, class HInc, class Sel>
__device__ __forceinline__ void topo_record_g(const DP& d, const TopoS& ts, uint32_t sel_n, uint64_t zf, uint32_t zl,
                                              HInc hinc, Sel sel) {
  const uint64_t zmask = d.ZS >= 64 ? ~0ull : (1ull << d.ZS) - 1ull;
  zf &= zmask;
  for (uint32_t k = 0; k < sel_n; k++) {
    const uint32_t e = sel(k);
    uint32_t slot = e & 0xFFFFFFu;
    const uint32_t kind = e >> 24;
    if (kind & TK_LAZY) {
      const uint32_t li = (e >> 12) & 0xFFFu;
      if (!((ts.lazy[li >> 6] >> (li & 63u)) & 1ull)) continue;  // not created yet
      slot = e & 0xFFFu;
    }
    if (kind & TK_HOST) {
      hinc(slot);
      ts.htot[slot]++;
    } else if (!(zl & ZF_COMP)) {
      if (kind & TK_ANTI) {
        for (uint64_t x = zf; x; x &= x - 1) ts.zcnt[slot * d.ZS + (uint32_t)__ffsll((long long)x) - 1u]++;
        ts.known[slot] |= zf;
      } else if (__popcll(zf) == 1) {
        ts.zcnt[slot * d.ZS + (uint32_t)__ffsll((long long)zf) - 1u]++;
        ts.known[slot] |= zf;
      }
    }
  }
}
template <class DP, class HInc>
__device__ __forceinline__ void topo_record(const DP& d, const TopoS& ts, uint32_t sel_off, uint32_t sel_n, uint64_t zf,
                                            uint32_t zl, HInc hinc) {
  topo_record_g(d, ts, sel_n, zf, zl, hinc, [&](uint32_t k) -> uint32_t { return d.tg_list[sel_off + k]; });
}

}  // namespace
}  // namespace gsd
