// kernels.hip — gfx950 (CDNA4, wave64) kernels of the provisioning solve.
//
//  K1/K2 feas_kernel   pod-variant x template x instance-type feasibility rows
//                      (one wave per (variant, template); lane = instance type;
//                      __ballot packs 64 ITs per word) + wave argmin of the
//                      cheapest compatible offering, key (price_rank<<32|name_rank)
//  K4    ffd_kernel    the sequential Scheduler.Solve queue loop as ONE
//                      persistent workgroup: in-flight NodeClaims are scored in
//                      parallel (256 candidates per step) in the exact order an
//                      emulated Go sort.Slice leaves them
//  K3    trunc_kernel  per NodeClaim: OrderByPrice + Truncate(60)
//
// All integer/bitset work: no MFMA.  Semantics cited as <U> restate
// sigs.k8s.io/karpenter@v1.13.0 ("parity").
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "layout.hpp"

using namespace gsd;

namespace {

constexpr int BLOCK = 256;
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
__device__ __forceinline__ bool fk_exempt(const FK& q) {
  // Operator() in {NotIn, DoesNotExist}
  return (q.flags & FK_COMP) ? (q.excl != 0) : (q.has == 0);
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
    len0 = (c.has & p.has) == 0;
  }
  return !len0 || (fk_exempt(c) && fk_exempt(p));
}

// <U> Requirement.Intersection for one free key
__device__ FK fk_intersect(const FK& a, const FK& b, const int64_t* ival, uint64_t isint) {
  FK r;
  r.pad = 0;
  bool comp = (a.flags & FK_COMP) && (b.flags & FK_COMP);
  bool hg = (a.flags | b.flags) & FK_GT, hl = (a.flags | b.flags) & FK_LT;
  int64_t gt = (a.flags & FK_GT) ? a.gt : b.gt;
  if ((a.flags & FK_GT) && (b.flags & FK_GT)) gt = a.gt > b.gt ? a.gt : b.gt;
  int64_t lt = (a.flags & FK_LT) ? a.lt : b.lt;
  if ((a.flags & FK_LT) && (b.flags & FK_LT)) lt = a.lt < b.lt ? a.lt : b.lt;
  if (hg && hl && gt >= lt) {
    r.has = 0;
    r.excl = 0;
    r.gt = r.lt = 0;
    r.flags = FK_PRESENT;
    return r;
  }
  r.has = a.has & b.has;
  if (comp) {
    uint64_t w = ~0ull;
    if (hg || hl) {
      w = 0;
      for (int i = 0; i < 64; i++) {
        if (!((isint >> i) & 1)) continue;
        int64_t x = ival[i];
        if (hg && gt >= x) continue;
        if (hl && lt <= x) continue;
        w |= 1ull << i;
      }
    }
    r.excl = (a.excl | b.excl) & w;
    r.gt = hg ? gt : 0;
    r.lt = hl ? lt : 0;
    r.flags = FK_PRESENT | FK_COMP | (hg ? FK_GT : 0) | (hl ? FK_LT : 0);
  } else {
    r.excl = 0;
    r.gt = r.lt = 0;
    r.flags = FK_PRESENT;
  }
  return r;
}

__device__ __forceinline__ bool var_fk_ok(const DevProblem& d, const VarRec& vr, const FK* claim_fk) {
  for (uint32_t k = 0; k < vr.fk_count; k++) {
    const FKEntry& e = d.fk_entries[vr.fk_begin + k];
    if (!fk_compatible(claim_fk[e.slot], e.st, (d.wk_slots >> e.slot) & 1)) return false;
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
  const uint32_t pair = blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6);
  if (pair >= d.V * d.T) return;  // wave-uniform
  const uint32_t v = pair / d.T, t = pair % d.T;
  const VarRec vr = d.vars[v];
  const TmplRec& tr = d.tmpl[t];
  uint64_t* rowout = d.rows + (size_t)pair * d.W;

  // wave-uniform parts of NodeClaim.CanAdd on a fresh NodeClaim
  bool ok_all = (tr.taints & ~vr.tol) == 0;  // <U> Taints.ToleratesPod
  const bool fk_ok = var_fk_ok(d, vr, d.t_fk + (size_t)t * d.F);
  if (static_mode) ok_all = ok_all && fk_ok;
  int64_t dem[RMAX];
  const int64_t* preq = d.pod_req + (size_t)vr.pod * d.R;
  for (uint32_t r = 0; r < d.R; r++) dem[r] = tr.daemon[r] + preq[r];  // Merge(daemon, pod)
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
      for (uint32_t r = 0; r < d.R; r++) ok = ok && d.it_alloc[(size_t)r * d.N + i] >= dem[r];
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

// ========================================================================= K4
namespace {

// Go sort.Slice (pdqsort_func) over LDS keys sc[] with payload ord[], run by
// one thread.  Restated for the device from src/sort/zsortfunc.go.
struct DevSort {
  uint32_t* sc;
  uint32_t* ord;
  __device__ bool less(int i, int j) const { return sc[i] < sc[j]; }
  __device__ void swap(int i, int j) const {
    uint32_t a = sc[i];
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
  __device__ static int bits_len(uint64_t x) { return x ? 64 - __clzll((long long)x) : 0; }
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
  // returns pivot; hint: 0 unknown, 1 increasing, 2 decreasing
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
  // iterative pdqsort (explicit stack for the recursion on the smaller side)
  __device__ void pdqsort(int a0, int b0) const {
    struct Frame {
      int a, b, limit;
      bool wasBalanced, wasPartitioned;
    };
    Frame st[64];
    int sp = 0;
    st[sp++] = Frame{a0, b0, bits_len((uint64_t)(b0 - a0)), true, true};
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
        if (!f.wasBalanced) {
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
        if (f.wasBalanced && f.wasPartitioned && hint == 1) {
          if (partial_insertion_sort(f.a, f.b)) break;
        }
        if (f.a > 0 && !less(f.a - 1, pivot)) {
          f.a = partition_equal(f.a, f.b, pivot);
          continue;
        }
        bool already;
        int mid = partition(f.a, f.b, pivot, &already);
        f.wasPartitioned = already;
        int leftLen = mid - f.a, rightLen = f.b - mid;
        int bal = length / 8;
        Frame child;
        if (leftLen < rightLen) {
          f.wasBalanced = leftLen >= bal;
          child = Frame{f.a, mid, f.limit, true, true};
          f.a = mid + 1;
        } else {
          f.wasBalanced = rightLen >= bal;
          child = Frame{mid + 1, f.b, f.limit, true, true};
          f.b = mid;
        }
        // recurse: child first, then resume this frame's loop
        st[sp++] = f;
        f = child;
      }
    }
  }
};

enum : uint32_t { MOD_NONE = 0, MOD_INC = 1, MOD_APPEND = 2 };

struct FfdShared {
  uint32_t pod, var, stop, first, M, modkind, modpos, qhead, qlen, epoch, nlog, status;
  uint32_t found, fast_path, e0, e1;
  uint64_t pops, generic, fast, cand;
};

}  // namespace

// one persistent workgroup runs the whole <U> Scheduler.Solve queue loop
extern "C" __global__ __launch_bounds__(BLOCK) void ffd_kernel(DevProblem d) {
  extern __shared__ uint32_t lds[];
  uint32_t* s_ord = lds;
  uint32_t* s_sc = lds + d.max_claims;
  __shared__ FfdShared S;
  const uint32_t tid = threadIdx.x;
  const uint32_t W = d.W, R = d.R, F = d.F, T = d.T, P = d.P;

  for (uint32_t i = tid; i < P; i += BLOCK) {
    d.queue[i] = d.queue0[i];
    d.last_epoch[i] = 0;
    d.last_len[i] = 0;
    d.cur_var[i] = d.var_begin[i];
  }
  for (uint32_t i = tid; i < T * R; i += BLOCK) d.t_rem[i] = d.tmpl[i / R].limits[i % R];
  if (tid == 0) {
    S.M = 0;
    S.qhead = 0;
    S.qlen = P;
    S.epoch = 1;
    S.modkind = MOD_NONE;
    S.nlog = 0;
    S.pops = 0;
    S.generic = 0;
    S.fast = 0;
    S.cand = 0;
    S.status = 0;
  }
  __syncthreads();
  // safety net only: the <U> loop performs at most (relaxations+2)*P pops
  const uint64_t max_pops = ((uint64_t)(d.V - d.P) + 2) * (uint64_t)P + P + 16;

  for (;;) {
    // ------------------------------------------------------------ Queue.Pop
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

    // ------------------------- sort.Slice(newNodeClaims, len(Pods) asc)
    if (M > 1) {
      if (tid == 0) {
        DevSort ds{s_sc, s_ord};
        uint32_t fast = 0, e0 = 0, e1 = 0;
        bool inversion = false;
        if (S.modkind == MOD_INC) {
          const uint32_t q = S.modpos;
          inversion = q + 1 < M && s_sc[q + 1] < s_sc[q];
        } else if (S.modkind == MOD_APPEND) {
          inversion = s_sc[M - 2] > s_sc[M - 1];
        }
        if (!inversion) {
          // sorted input: pdqsort/insertion sort leave it untouched
        } else if (M <= 12) {
          ds.insertion_sort(0, (int)M);
        } else {
          int hint;
          ds.choose_pivot(0, (int)M, &hint);
          if (hint == 1 && M >= 50) {
            // partialInsertionSort fixes the single inversion: see DESIGN.md
            fast = S.modkind;
            if (S.modkind == MOD_INC) {
              const uint32_t q = S.modpos, x = s_sc[q];
              uint32_t lo = q + 1, hi = M;  // first index > q with sc >= x
              while (lo < hi) {
                uint32_t mid = (lo + hi) >> 1;
                if (s_sc[mid] < x) lo = mid + 1;
                else hi = mid;
              }
              e0 = q;
              e1 = lo;  // rotate-left [q, lo): X lands at lo-1
            } else {
              const uint32_t x = s_sc[M - 1];
              uint32_t lo = 0, hi = M - 1;  // first index with sc > x
              while (lo < hi) {
                uint32_t mid = (lo + hi) >> 1;
                if (s_sc[mid] <= x) lo = mid + 1;
                else hi = mid;
              }
              e0 = lo;
              e1 = M;  // rotate-right [lo, M): X lands at lo
            }
            S.fast++;
          } else {
            ds.pdqsort(0, (int)M);
            S.generic++;
          }
        }
        S.fast_path = fast;
        S.e0 = e0;
        S.e1 = e1;
        S.modkind = MOD_NONE;
      }
      __syncthreads();
      if (S.fast_path) {
        const uint32_t e0 = S.e0, e1 = S.e1;
        const uint32_t xo = s_ord[S.fast_path == MOD_INC ? e0 : e1 - 1];
        const uint32_t xs = s_sc[S.fast_path == MOD_INC ? e0 : e1 - 1];
        __syncthreads();
        if (S.fast_path == MOD_INC) {
          for (uint32_t base = e0; base + 1 < e1; base += BLOCK) {
            const uint32_t i = base + tid;
            uint32_t o = 0, s = 0;
            const bool act = i + 1 < e1;
            if (act) {
              o = s_ord[i + 1];
              s = s_sc[i + 1];
            }
            __syncthreads();
            if (act) {
              s_ord[i] = o;
              s_sc[i] = s;
            }
            __syncthreads();
          }
          if (tid == 0) {
            s_ord[e1 - 1] = xo;
            s_sc[e1 - 1] = xs;
          }
        } else {
          // shift [e0, e1-1) right by one, from the top down
          const uint32_t n = e1 - 1 - e0;
          for (uint32_t done = 0; done < n; done += BLOCK) {
            const int64_t i = (int64_t)e1 - 2 - done - tid;
            uint32_t o = 0, s = 0;
            const bool act = i >= (int64_t)e0;
            if (act) {
              o = s_ord[i];
              s = s_sc[i];
            }
            __syncthreads();
            if (act) {
              s_ord[i + 1] = o;
              s_sc[i + 1] = s;
            }
            __syncthreads();
          }
          if (tid == 0) {
            s_ord[e0] = xo;
            s_sc[e0] = xs;
          }
        }
      }
      __syncthreads();
    }

    // ---------------------- in-flight NodeClaims, first that CanAdd wins
    for (uint32_t base = 0; base < M; base += BLOCK) {
      const uint32_t pos = base + tid;
      bool feas = false;
      uint32_t j = 0;
      uint64_t G = 0;
      const uint64_t* row = nullptr;
      const uint64_t* thr[RMAX];
      if (pos < M) {
        j = s_ord[pos];
        const ClaimHdr h = d.c_hdr[j];
        const TmplRec& tr = d.tmpl[h.tmpl];
        feas = (tr.taints & ~vr.tol) == 0 && var_fk_ok(d, vr, d.c_fk + (size_t)j * F);
        if (feas) {
          G = grid_of(h.zm & vr.zm, h.cm & vr.cm, d.Z, d.C);
          const uint64_t Gt = grid_of(tr.zm & vr.zm, tr.cm & vr.cm, d.Z, d.C);
          row = d.rows + ((size_t)v * T + h.tmpl) * W;
          for (uint32_t r = 0; r < R; r++) {
            const int64_t dem = d.c_tot[(size_t)j * R + r] + preq[r];
            const uint32_t o = d.thr_off[r], n = d.thr_off[r + 1] - o;
            const uint32_t m = lower_bound_i64(d.thr_val + o, n, dem);
            thr[r] = d.thr_set + (size_t)(o + r + m) * W;
          }
          bool any = false;
          const uint64_t* opts = d.c_opts + (size_t)j * W;
          for (uint32_t w = 0; w < W && !any; w++) {
            uint64_t x = opts[w] & row[w];
            for (uint32_t r = 0; r < R; r++) x &= thr[r][w];
            if (G != Gt) {
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
      if (tid == 0) {
        S.first = INF;
        S.cand += (M - base) < BLOCK ? (M - base) : BLOCK;
      }
      __syncthreads();
      if (feas) atomicMin(&S.first, pos);
      __syncthreads();
      const uint32_t f = S.first;
      if (f != INF) {
        if (pos == f) {
          // NodeClaim.Add: options, requests, requirements, pods
          const uint64_t* opts = d.c_opts + (size_t)j * W;
          uint64_t* nopts = d.c_opts + (size_t)j * W;
          for (uint32_t w = 0; w < W; w++) {
            uint64_t x = opts[w] & row[w];
            for (uint32_t r = 0; r < R; r++) x &= thr[r][w];
            uint64_t off = 0;
            uint64_t gm = G;
            while (gm) {
              const uint32_t g = __ffsll((long long)gm) - 1;
              gm &= gm - 1;
              off |= d.slot_set[(size_t)g * W + w];
            }
            nopts[w] = x & off;
          }
          for (uint32_t r = 0; r < R; r++) d.c_tot[(size_t)j * R + r] += preq[r];
          ClaimHdr h = d.c_hdr[j];
          h.zm &= vr.zm;
          h.cm &= vr.cm;
          h.count++;
          d.c_hdr[j] = h;
          FK* cf = d.c_fk + (size_t)j * F;
          for (uint32_t k = 0; k < vr.fk_count; k++) {
            const FKEntry& e = d.fk_entries[vr.fk_begin + k];
            const FK cur = cf[e.slot];
            cf[e.slot] = (cur.flags & FK_PRESENT)
                             ? fk_intersect(cur, e.st, d.fk_ival + (size_t)e.slot * 64, d.fk_isint[e.slot])
                             : e.st;
          }
          s_sc[pos]++;
          S.modkind = MOD_INC;
          S.modpos = pos;
          const uint32_t li = S.nlog++;
          d.log[li] = LogRec{p, v, j, 0};
          S.found = 1;
        }
        break;
      }
    }
    __syncthreads();
    if (S.found) continue;

    // ------------------------------- new NodeClaim from templates, in order
    for (uint32_t t = 0; t < T; t++) {
      const TmplRec& tr = d.tmpl[t];
      const uint64_t* row = d.rows + ((size_t)v * T + t) * W;
      // row & limits mask (filterByRemainingResources), one IT per thread
      bool any = false;
      if (d.fk_ok[(size_t)v * T + t])
        for (uint32_t w = 0; w < W; w++)
          if (row[w]) any = true;
      if (!any) continue;
      if (tr.has_limits) {
        if (tid == 0) S.first = 0;
        __syncthreads();
        for (uint32_t i = tid; i < W * 64; i += BLOCK) {
          if (i >= d.N || !((row[i >> 6] >> (i & 63)) & 1)) continue;
          bool ok = true;
          for (uint32_t r = 0; r < R; r++)
            if ((tr.limit_rmask >> r) & 1) ok = ok && d.it_cap[(size_t)r * d.N + i] <= d.t_rem[(size_t)t * R + r];
          if (ok) atomicOr(&S.first, 1u);
        }
        __syncthreads();
        any = S.first != 0;
        __syncthreads();
        if (!any) continue;
      }
      // create: NewNodeClaim + CanAdd succeeded (the row already carries it)
      if (M >= d.max_claims) {
        if (tid == 0) S.status = 1;
        __syncthreads();
        break;
      }
      const uint32_t j = M;
      for (uint32_t w = tid; w < W; w += BLOCK) {
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
      if (tid == 0) {
        for (uint32_t r = 0; r < R; r++) d.c_tot[(size_t)j * R + r] = tr.daemon[r] + preq[r];
        ClaimHdr h;
        h.tmpl = t;
        h.count = 1;
        h.zm = tr.zm & vr.zm;
        h.cm = tr.cm & vr.cm;
        d.c_hdr[j] = h;
        FK* cf = d.c_fk + (size_t)j * F;
        for (uint32_t s = 0; s < F; s++) cf[s] = d.t_fk[(size_t)t * F + s];
        for (uint32_t k = 0; k < vr.fk_count; k++) {
          const FKEntry& e = d.fk_entries[vr.fk_begin + k];
          const FK cur = cf[e.slot];
          cf[e.slot] = (cur.flags & FK_PRESENT)
                           ? fk_intersect(cur, e.st, d.fk_ival + (size_t)e.slot * 64, d.fk_isint[e.slot])
                           : e.st;
        }
        s_ord[M] = M;
        s_sc[M] = 1;
        S.M = M + 1;
        S.modkind = MOD_APPEND;
        const uint32_t li = S.nlog++;
        d.log[li] = LogRec{p, v, j, 0};
        S.found = 1;
      }
      __syncthreads();
      if (tr.has_limits) {
        // <U> subtractMax(remaining, nodeClaim.InstanceTypeOptions)
        for (uint32_t r = 0; r < R; r++) {
          if (!((tr.limit_rmask >> r) & 1)) continue;
          int64_t mx = INT64_MIN;
          for (uint32_t i = 0; i < d.N; i++)
            if ((d.c_opts[(size_t)j * W + (i >> 6)] >> (i & 63)) & 1) {
              const int64_t c = d.it_cap[(size_t)r * d.N + i];
              mx = c > mx ? c : mx;
            }
          if (tid == 0 && mx != INT64_MIN) d.t_rem[(size_t)t * R + r] -= mx;
        }
      }
      __syncthreads();
      break;
    }
    __syncthreads();
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
  for (uint32_t i = tid; i < S.M; i += BLOCK) d.c_sorted[i] = s_ord[i];
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
    *d.ctrl = c;
  }
}

// ========================================================================= K3
// <U> InstanceTypes.OrderByPrice(reqs) + Truncate(60): key per option IT =
// (rank of its cheapest available compatible offering price, name rank)
extern "C" __global__ __launch_bounds__(BLOCK) void trunc_kernel(DevProblem d) {
  extern __shared__ uint64_t keys[];
  __shared__ uint32_t cnt;
  const uint32_t j = blockIdx.x;
  if (j >= d.ctrl->n_claims) return;
  const uint32_t tid = threadIdx.x;
  const ClaimHdr h = d.c_hdr[j];
  const uint64_t G = grid_of(h.zm, h.cm, d.Z, d.C);
  if (tid == 0) cnt = 0;
  __syncthreads();
  for (uint32_t i = tid; i < d.N; i += BLOCK) {
    if (!((d.c_opts[(size_t)j * d.W + (i >> 6)] >> (i & 63)) & 1)) continue;
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
  for (uint32_t i = tid; i < take; i += BLOCK) d.c_its[(size_t)j * 60 + i] = d.rank_to_it[(uint32_t)keys[i]];
  if (tid == 0) d.c_nits[j] = take;
}

// ------------------------------------------------------------ host launchers
extern "C" hipError_t gsk_init(uint32_t ffd_lds_bytes, uint32_t trunc_lds_bytes) {
  hipError_t e = hipFuncSetAttribute((const void*)ffd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)ffd_lds_bytes);
  if (e != hipSuccess) return e;
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

extern "C" hipError_t gsk_ffd(const DevProblem* d, hipStream_t s) {
  hipLaunchKernelGGL(ffd_kernel, dim3(1), dim3(BLOCK), d->max_claims * 8, s, *d);
  return hipGetLastError();
}

extern "C" hipError_t gsk_trunc(const DevProblem* d, uint32_t lds_bytes, hipStream_t s) {
  hipLaunchKernelGGL(trunc_kernel, dim3(d->max_claims), dim3(BLOCK), lds_bytes, s, *d);
  return hipGetLastError();
}
