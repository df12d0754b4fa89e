// rank.hip — autoplacement ranking on gfx950:
// IBMInstanceTypeProvider.FilterInstanceTypes + rankInstanceTypes
// (pkg/providers/common/instancetype/instancetype.go:259-379), and
// RankInstanceTypes (:381-420) with the filters off.  C-ABI in
// include/gpusched.h (gs_rank_instance_types).
//
// One workgroup (the catalog is a few hundred to a few thousand types):
//   1. per type, the four filters and calculateInstanceTypeScore (:90-110) in
//      float64; kept types are compacted IN LIST ORDER into LDS with a ballot
//      prefix per 256-type chunk (sort.Slice's input order decides tie order);
//   2. one lane runs Go's sort.Slice (pdqsort_func, src/sort/zsortfunc.go)
//      over (score, index) pairs in LDS, Less = score[i] < score[j];
//   3. the block writes the ranked indices and scores back.
// The work is latency-bound (a single launch over <= 4096 types: 12 B per
// type in, 12 B out); there is nothing here for MFMA or the HBM roofline.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "../../include/gpusched.h"

namespace {

constexpr uint32_t RK_NT = 256;
constexpr uint32_t RK_NWAVE = RK_NT / 64;

struct RankArgs {
  const int64_t* cpu_milli;
  const int64_t* memory_bytes;
  const double* price;
  const uint32_t* arch;
  uint32_t* out_order;
  double* out_score;
  uint32_t* out_n;
  int64_t min_cpu, min_memory_gb;
  double max_price;
  uint32_t n, want_arch;
};

__device__ __forceinline__ int bits_len_u64(uint64_t x) { return x ? 64 - __clzll((long long)x) : 0; }

// Go sort.Slice over LDS (score, index) pairs, one thread.  Same control flow
// as zsortfunc.go: insertionSort_func, heapSort_func, pdqsort_func,
// partition_func, partitionEqual_func, partialInsertionSort_func,
// breakPatterns_func, choosePivot_func, reverseRange_func.  pdqsort_func's
// recursion on the shorter side becomes an explicit frame stack (the two
// sides are disjoint, so the processing order does not change the result).
struct PairSort {
  double* sc;
  uint32_t* ix;
  struct Frame {
    int a, b, limit;
    bool wb, wp;
  };
  __device__ bool less(int i, int j) const { return sc[i] < sc[j]; }
  __device__ void swap(int i, int j) const {
    const double s = sc[i];
    sc[i] = sc[j];
    sc[j] = s;
    const uint32_t t = ix[i];
    ix[i] = ix[j];
    ix[j] = t;
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
    const int first = a, hi = b - a;
    for (int i = (hi - 1) / 2; i >= 0; i--) sift_down(i, hi, first);
    for (int i = hi - 1; i >= 0; i--) {
      swap(first, first + i);
      sift_down(0, i, first);
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
    const int maxSteps = 5, shortestShifting = 50;
    int i = a + 1;
    for (int step = 0; step < maxSteps; step++) {
      while (i < b && !less(i, i - 1)) i++;
      if (i == b) return true;
      if (b - a < shortestShifting) return false;
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
    const int length = b - a;
    if (length < 8) return;
    uint64_t r = (uint64_t)length;  // xorshift seeded with the length
    const uint64_t modulus = 1ull << bits_len_u64((uint64_t)length);
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
  __device__ void order2(int& a, int& b, int* swaps) const {
    if (less(b, a)) {
      (*swaps)++;
      const int t = a;
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
  // hint: 0 unknown, 1 increasing, 2 decreasing
  __device__ int choose_pivot(int a, int b, int* hint) const {
    const int l = b - a;
    int swaps = 0;
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
    for (int i = a, j = b - 1; i < j; i++, j--) swap(i, j);
  }
  __device__ void slice(int n) const {
    Frame st[40];
    int sp = 0;
    st[sp++] = Frame{0, n, bits_len_u64((uint64_t)n), true, true};
    while (sp > 0) {
      Frame f = st[--sp];
      for (;;) {
        const int length = f.b - f.a;
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
        const int mid = partition(f.a, f.b, pivot, &already);
        f.wp = already;
        const int leftLen = mid - f.a, rightLen = f.b - mid;
        const int bal = length / 8;
        Frame child;
        if (leftLen < rightLen) {
          f.wb = leftLen >= bal;
          child = Frame{f.a, mid, f.limit, true, true};
          f.a = mid + 1;
        } else {
          f.wb = rightLen >= bal;
          child = Frame{mid + 1, f.b, f.limit, true, true};
          f.b = mid;
        }
        st[sp++] = f;  // the longer side resumes after the shorter one
        f = child;
      }
    }
  }
};

__global__ __launch_bounds__(RK_NT) void rank_kernel(RankArgs a) {
  extern __shared__ double rk_lds[];
  double* sc = rk_lds;                          // [n] scores, compacted
  uint32_t* ix = (uint32_t*)(rk_lds + a.n);     // [n] List indices, compacted
  __shared__ uint32_t wcnt[RK_NWAVE];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  uint32_t kept = 0;
  for (uint32_t c = 0; c < a.n; c += RK_NT) {
    const uint32_t i = c + tid;
    bool keep = false;
    double s = 0.0;
    if (i < a.n) {
      const int64_t cm = a.cpu_milli[i], mb = a.memory_bytes[i];
      const double p = a.price[i];
      // Capacity.Cpu().Value() and Memory().ScaledValue(Giga) round up
      const int64_t cpu = (cm + 999) / 1000;
      const int64_t mem_gb = (mb + 999999999) / 1000000000;
      keep = (a.want_arch == GS_ARCH_ANY || a.arch[i] == a.want_arch) && (a.min_cpu <= 0 || cpu >= a.min_cpu) &&
             (a.min_memory_gb <= 0 || !((double)mb / 1073741824.0 < (double)a.min_memory_gb)) &&
             (!(a.max_price > 0) || !(p > a.max_price));
      if (p <= 0) {
        s = (double)cpu + (double)mem_gb;
      } else {
        const double ce = p / (double)cpu;
        const double me = p / (double)mem_gb;
        s = (ce + me) / 2;
      }
    }
    const uint64_t b = __ballot(keep);
    if (lane == 0) wcnt[wave] = (uint32_t)__popcll(b);
    __syncthreads();
    uint32_t off = kept, total = 0;
    for (uint32_t w = 0; w < RK_NWAVE; w++) {
      if (w < wave) off += wcnt[w];
      total += wcnt[w];
    }
    if (keep) {
      const uint32_t at = off + (uint32_t)__popcll(b & ((1ull << lane) - 1ull));
      sc[at] = s;
      ix[at] = i;
    }
    kept += total;
    __syncthreads();  // wcnt reuse, and the compacted arrays before the sort
  }
  if (tid == 0) {
    PairSort ps{sc, ix};
    ps.slice((int)kept);
    *a.out_n = kept;
  }
  __syncthreads();
  for (uint32_t k = tid; k < kept; k += RK_NT) {
    a.out_order[k] = ix[k];
    a.out_score[k] = sc[k];
  }
}

}  // namespace

extern "C" gs_status gs_rank_instance_types(uint32_t n, const int64_t* cpu_milli, const int64_t* memory_bytes,
                                            const double* price, const uint32_t* arch, uint32_t want_arch,
                                            int64_t min_cpu, int64_t min_memory_gb, double max_price,
                                            uint32_t* out_order, uint32_t* out_n, double* out_score) {
  if (!out_n || (n && (!cpu_milli || !memory_bytes || !price || !arch || !out_order || !out_score)))
    return GS_E_INVALID;
  if (n > GS_RANK_MAX) return GS_E_CAPACITY;
  for (uint32_t i = 0; i < n; i++)
    if (cpu_milli[i] < 0 || memory_bytes[i] < 0) return GS_E_INVALID;
  *out_n = 0;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return GS_E_NO_DEVICE;
  if (n == 0) return GS_OK;
  // one grow-once device buffer (serialized by a mutex): inputs packed as
  // cpu | mem | price (8 B each) | arch (4 B), outputs score (8 B) | order
  // (4 B) | count; one H2D copy in, one D2H copy out
  static std::mutex mu;
  static char* dbuf = nullptr;
  static size_t dcap = 0;
  static std::vector<char> hin, hout;
  std::lock_guard<std::mutex> lock(mu);
  const size_t nn = n;
  const size_t in_bytes = nn * 28, out_bytes = nn * 12 + 8;
  const size_t bytes = ((in_bytes + 255) & ~(size_t)255) + out_bytes;
  if (bytes > dcap) {
    if (dbuf) (void)hipFree(dbuf);
    dbuf = nullptr;
    dcap = 0;
    if (hipMalloc(&dbuf, bytes) != hipSuccess) return GS_E_HIP;
    dcap = bytes;
  }
  char* d = dbuf;
  char* dout = d + ((in_bytes + 255) & ~(size_t)255);
  hin.resize(in_bytes);
  hout.resize(out_bytes);
  memcpy(hin.data(), cpu_milli, nn * 8);
  memcpy(hin.data() + nn * 8, memory_bytes, nn * 8);
  memcpy(hin.data() + nn * 16, price, nn * 8);
  memcpy(hin.data() + nn * 24, arch, nn * 4);
  RankArgs a{};
  a.cpu_milli = (const int64_t*)d;
  a.memory_bytes = (const int64_t*)(d + nn * 8);
  a.price = (const double*)(d + nn * 16);
  a.arch = (const uint32_t*)(d + nn * 24);
  a.out_score = (double*)dout;
  a.out_order = (uint32_t*)(dout + nn * 8);
  a.out_n = (uint32_t*)(dout + nn * 12);
  a.min_cpu = min_cpu;
  a.min_memory_gb = min_memory_gb;
  a.max_price = max_price;
  a.n = n;
  a.want_arch = want_arch;
  const size_t lds = nn * (sizeof(double) + sizeof(uint32_t));
  if (hipMemcpy(d, hin.data(), in_bytes, hipMemcpyHostToDevice) != hipSuccess) return GS_E_HIP;
  hipLaunchKernelGGL(rank_kernel, dim3(1), dim3(RK_NT), lds, 0, a);
  if (hipGetLastError() != hipSuccess ||
      hipMemcpy(hout.data(), dout, out_bytes, hipMemcpyDeviceToHost) != hipSuccess)  // null stream: after the kernel
    return GS_E_HIP;
  uint32_t kept;
  memcpy(&kept, hout.data() + nn * 12, 4);
  if (kept > n) return GS_E_HIP;
  memcpy(out_score, hout.data(), (size_t)kept * 8);
  memcpy(out_order, hout.data() + nn * 8, (size_t)kept * 4);
  *out_n = kept;
  return GS_OK;
}
