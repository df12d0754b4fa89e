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
//      rank_key_kernel (grid-wide) gives each kept score a u16 key = how many
//      kept scores are strictly below it (ties share a key, so every Less
//      outcome is the float64 one);
//   2. rank_sort_kernel (ffd_wave.hip) runs the single-wave restatement of
//      Go's sort.Slice (pdqsort_func) that orders in-flight NodeClaims, on
//      (key, position) pairs packed in LDS;
//   3. rank_gather_kernel writes the ranked List indices and scores.
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
  // device scratch: compacted scores / List indices, sort keys and positions
  double* cscore;
  uint32_t* cidx;
  uint16_t* keys;
  uint16_t* pos;
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
  for (uint32_t k = tid; k < kept; k += RK_NT) {
    a.cscore[k] = sc[k];
    a.cidx[k] = ix[k];
  }
  if (tid == 0) *a.out_n = kept;
}

// sort keys: key[k] = how many kept scores are strictly below score k (ties
// share a key; key order == float64 order), payload the compacted position.
// Workgroup b owns k in [64b, 64b + 64) (lane = k); it stages every kept
// score in LDS with one coalesced pass, its 4 waves split the j range (a
// broadcast LDS read per j) and add their partial counts in LDS.
__global__ __launch_bounds__(RK_NT) void rank_key_kernel(RankArgs a) {
  extern __shared__ double rk_all[];  // [kept] scores
  __shared__ uint32_t part[RK_NWAVE][64];
  const uint32_t kept = *a.out_n;
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t k = blockIdx.x * 64u + lane;
  for (uint32_t j = threadIdx.x; j < kept; j += RK_NT) rk_all[j] = a.cscore[j];
  __syncthreads();
  const double x = k < kept ? rk_all[k] : 0.0;
  const uint32_t per = (kept + RK_NWAVE - 1) / RK_NWAVE;
  const uint32_t j0 = wave * per, j1 = j0 + per < kept ? j0 + per : kept;
  uint32_t below = 0;
#pragma unroll 8
  for (uint32_t j = j0; j < j1; j++) below += rk_all[j] < x;
  part[wave][lane] = below;
  __syncthreads();
  if (wave == 0 && k < kept) {
    uint32_t t = 0;
    for (uint32_t w = 0; w < RK_NWAVE; w++) t += part[w][lane];
    a.keys[k] = (uint16_t)t;
    a.pos[k] = (uint16_t)k;
  }
}

// after rank_sort_kernel: ranked List indices and scores
__global__ __launch_bounds__(RK_NT) void rank_gather_kernel(RankArgs a) {
  const uint32_t kept = *a.out_n;
  for (uint32_t k = blockIdx.x * RK_NT + threadIdx.x; k < kept; k += gridDim.x * RK_NT) {
    const uint32_t p = a.pos[k];
    a.out_order[k] = a.cidx[p];
    a.out_score[k] = a.cscore[p];
  }
}

}  // namespace

extern "C" hipError_t gsk_rank_sort(uint16_t* keys, uint16_t* pos, const uint32_t* np, uint32_t cap, int x,
                                    hipStream_t s);

extern "C" gs_status gs_rank_instance_types(uint32_t n, const int64_t* cpu_milli, const int64_t* memory_bytes,
                                            const double* price, const uint32_t* arch, uint32_t want_arch,
                                            int64_t min_cpu, int64_t min_memory_gb, double max_price,
                                            uint32_t* out_order, uint32_t* out_n, double* out_score) {
  if (!out_n || (n && (!cpu_milli || !memory_bytes || !price || !arch || !out_order || !out_score)))
    return GS_E_INVALID;
  if (n > GS_RANK_MAX) return GS_E_CAPACITY;
  for (uint32_t i = 0; i < n; i++)
    if (cpu_milli[i] < 0 || memory_bytes[i] < 0 || price[i] != price[i]) return GS_E_INVALID;  // NaN price
  *out_n = 0;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return GS_E_NO_DEVICE;
  if (n == 0) return GS_OK;
  // one grow-once buffer per device (the call runs on the calling thread's
  // current device; cgo may move a goroutine between OS threads, so a buffer
  // is never reused on another device), serialized by a mutex: inputs packed
  // as cpu | mem | price (8 B each) | arch (4 B), outputs score (8 B) | order
  // (4 B) | count; one H2D copy in, one D2H copy out
  constexpr int kMaxDev = 64;
  static std::mutex mu;
  static char* dbufs[kMaxDev] = {};
  static size_t dcaps[kMaxDev] = {};
  static std::vector<char> hin, hout;
  std::lock_guard<std::mutex> lock(mu);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return GS_E_NO_DEVICE;
  char*& dbuf = dbufs[dev];
  size_t& dcap = dcaps[dev];
  const size_t nn = n;
  const size_t in_bytes = nn * 28, out_bytes = nn * 12 + 8;
  const size_t out_off = (in_bytes + 255) & ~(size_t)255;
  const size_t scr_off = (out_off + out_bytes + 255) & ~(size_t)255;
  const size_t bytes = scr_off + nn * 16;  // cscore | cidx | keys | pos
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
  a.cscore = (double*)(d + scr_off);
  a.cidx = (uint32_t*)(d + scr_off + nn * 8);
  a.keys = (uint16_t*)(d + scr_off + nn * 12);
  a.pos = (uint16_t*)(d + scr_off + nn * 14);
  const size_t lds = nn * (sizeof(double) + sizeof(uint32_t));
  if (hipMemcpy(d, hin.data(), in_bytes, hipMemcpyHostToDevice) != hipSuccess) return GS_E_HIP;
  hipLaunchKernelGGL(rank_kernel, dim3(1), dim3(RK_NT), lds, 0, a);
  hipLaunchKernelGGL(rank_key_kernel, dim3((n + 63) / 64), dim3(RK_NT), nn * sizeof(double), 0, a);
  if (hipGetLastError() != hipSuccess || gsk_rank_sort(a.keys, a.pos, a.out_n, n, -1, 0) != hipSuccess) return GS_E_HIP;
  hipLaunchKernelGGL(rank_gather_kernel, dim3((n + RK_NT - 1) / RK_NT), dim3(RK_NT), 0, 0, a);
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

// Test hook (not in gpusched.h; tests/test_wave_sort.py binds it): the
// single-wave sort.Slice restatement (WaveSort, the Solve's NodeClaim sort)
// over n u16 keys on the current device; perm[k] = the input index that lands
// at position k.  Parity with Go's pdqsort is checked against the oracle's
// restatement on adversarial key arrays (one raised key, two or three values).
extern "C" gs_status gs_debug_go_sort_known(const uint16_t* keys, uint32_t n, int32_t x, uint32_t* perm);
extern "C" gs_status gs_debug_go_sort(const uint16_t* keys, uint32_t n, uint32_t* perm) {
  return gs_debug_go_sort_known(keys, n, -1, perm);
}
// ... with x: the caller states that every position but x is in order (the
// Solve's one-change sorts), so the first partition takes partition_known
extern "C" gs_status gs_debug_go_sort_known(const uint16_t* keys, uint32_t n, int32_t x, uint32_t* perm) {
  if (n && (!keys || !perm)) return GS_E_INVALID;
  if (n > GS_RANK_MAX) return GS_E_CAPACITY;
  if (n == 0) return GS_OK;
  std::vector<uint16_t> h((size_t)n * 2);
  for (uint32_t k = 0; k < n; k++) {
    h[k] = keys[k];
    h[n + k] = (uint16_t)k;
  }
  void* d = nullptr;
  const size_t bytes = (size_t)n * 4 + 16;
  if (hipMalloc(&d, bytes) != hipSuccess) return GS_E_HIP;
  uint16_t* dk = (uint16_t*)d;
  uint16_t* dp = dk + n;
  uint32_t* dn = (uint32_t*)((char*)d + (((size_t)n * 4 + 3) & ~(size_t)3));
  gs_status st = GS_OK;
  if (hipMemcpy(dk, h.data(), (size_t)n * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(dn, &n, 4, hipMemcpyHostToDevice) != hipSuccess || gsk_rank_sort(dk, dp, dn, n, x, 0) != hipSuccess ||
      hipMemcpy(h.data(), dk, (size_t)n * 4, hipMemcpyDeviceToHost) != hipSuccess)
    st = GS_E_HIP;
  (void)hipFree(d);
  if (st == GS_OK)
    for (uint32_t k = 0; k < n; k++) perm[k] = h[n + k];
  return st;
}
