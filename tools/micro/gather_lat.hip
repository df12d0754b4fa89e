// Microbenchmark: latency of a divergent 192-B record gather by a single
// 1024-thread workgroup (the FFD candidate-scan access pattern).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>

struct alignas(64) Rec {
  int64_t tot[8], maxa[8];
  uint64_t zm, cm;
  uint16_t thr[8];
  uint32_t tmpl, count;
  uint32_t pad[6];
};

__global__ __launch_bounds__(1024) void gather(const Rec* rec, const uint16_t* idx, uint32_t K, uint32_t iters,
                                               uint32_t active_mod, uint32_t mode, uint64_t* out, int64_t* sink) {
  __shared__ uint64_t acc_cyc;
  __shared__ int32_t red;
  if (threadIdx.x == 0) { acc_cyc = 0; red = 0; }
  __syncthreads();
  int64_t s = 0;
  const uint32_t tid = threadIdx.x;
  for (uint32_t it = 0; it < iters; it++) {
    __syncthreads();
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    const uint32_t j = idx[(it * 1024u + tid) % K];
    bool act = (j % active_mod) == 0;
    int64_t v = 0;
    if (act) {
      const Rec* r = rec + j;
      if (mode == 0) {
        for (int k = 0; k < 4; k++) v += r->tot[k] + r->maxa[k];
        v += (int64_t)r->zm + r->cm + r->thr[0];
      } else if (mode == 1) {
        v = r->tot[0];
      } else if (mode == 2) {
        const uint4* q = (const uint4*)r;
        uint4 a = q[0], b = q[1], c = q[2], e = q[3];
        v = (int64_t)a.x + b.y + c.z + e.w;
      }
    }
    if (mode == 3) {
      // compact active lanes into the first waves, then gather 64 B each
      __shared__ uint32_t list[1024];
      __shared__ uint32_t wcnt[16];
      const uint64_t bm = __ballot(act);
      const uint32_t lane = tid & 63, w = tid >> 6;
      if (lane == 0) wcnt[w] = __popcll(bm);
      __syncthreads();
      uint32_t off = 0, tot = 0;
      for (uint32_t k = 0; k < 16; k++) { off += k < w ? wcnt[k] : 0; tot += wcnt[k]; }
      if (act) list[off + __popcll(bm & ((1ull << lane) - 1))] = j;
      __syncthreads();
      if (tid < tot) {
        const uint4* q = (const uint4*)(rec + list[tid]);
        uint4 a = q[0], b = q[1], c = q[2], e = q[3];
        v = (int64_t)a.x + b.y + c.z + e.w;
      }
    }
    const bool pre = v > 0x7000000000000000ll;
    if (__ballot(pre) && (tid & 63) == 0) atomicAdd(&red, 1);
    s += v;
    __syncthreads();
    if (tid == 0) acc_cyc += __builtin_amdgcn_s_memtime() - c0;
  }
  sink[tid] = s;
  if (tid == 0) out[0] = acc_cyc;
}

int main() {
  const uint32_t K = 1700, iters = 20000;
  std::vector<Rec> h(8192);
  for (auto& r : h) for (int k = 0; k < 8; k++) { r.tot[k] = k; r.maxa[k] = 2 * k; }
  std::vector<uint16_t> idx(K * 64);
  std::mt19937 g(1);
  for (auto& x : idx) x = g() % K;
  Rec* d_rec; uint16_t* d_idx; uint64_t* d_out; int64_t* d_sink;
  hipMalloc(&d_rec, h.size() * sizeof(Rec));
  hipMalloc(&d_idx, idx.size() * 2);
  hipMalloc(&d_out, 8);
  hipMalloc(&d_sink, 1024 * 8);
  hipMemcpy(d_rec, h.data(), h.size() * sizeof(Rec), hipMemcpyHostToDevice);
  hipMemcpy(d_idx, idx.data(), idx.size() * 2, hipMemcpyHostToDevice);
  for (uint32_t mode = 0; mode < 4; mode++)
    for (uint32_t am : {1u, 14u, 1000000u}) {
      hipLaunchKernelGGL(gather, dim3(1), dim3(1024), 0, 0, d_rec, d_idx, (uint32_t)idx.size(), iters, am, mode, d_out, d_sink);
      uint64_t cyc = 0;
      hipMemcpy(&cyc, d_out, 8, hipMemcpyDeviceToHost);
      printf("mode=%u active=1/%u: %.0f cycles per iteration\n", mode, am, (double)cyc / iters);
    }
  return 0;
}
