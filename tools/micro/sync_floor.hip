// Micro-benchmark (diagnostic): per-iteration cost of the building blocks of
// the FFD pod loop in ONE workgroup -- barrier, block min, dependent LDS
// chain, global load round trip -- for NT = 256 / 512 / 1024 threads.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int NT, int MODE>
__global__ __launch_bounds__(NT, 1) void floor_kernel(uint32_t iters, uint32_t* out, const uint32_t* g, uint64_t* cyc) {
  __shared__ uint32_t red[2][16];
  __shared__ uint32_t chain[1024];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (uint32_t i = tid; i < 1024; i += NT) chain[i] = (i * 7 + 3) & 1023;
  __syncthreads();
  uint32_t acc = 0, tog = 0, x = tid;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t it = 0; it < iters; it++) {
    if (MODE == 0) {  // bare barrier
      __syncthreads();
    } else if (MODE == 1) {  // block min (shuffles + LDS + barrier)
      uint32_t v = (tid * 2654435761u + it) >> 7;
      for (int m = 32; m >= 1; m >>= 1) {
        const uint32_t y = (uint32_t)__shfl_xor((int)v, m);
        v = y < v ? y : v;
      }
      if (lane == 0) red[tog][wave] = v;
      __syncthreads();
      uint32_t r = red[tog][0];
      for (int w = 1; w < NT / 64; w++) r = red[tog][w] < r ? red[tog][w] : r;
      tog ^= 1;
      acc += r;
    } else if (MODE == 2) {  // 8 dependent LDS reads (one wave's chain), then a barrier
      if (wave == 0)
        for (int k = 0; k < 8; k++) x = chain[x & 1023];
      __syncthreads();
    } else if (MODE == 3) {  // one dependent global load round trip by wave 0, then a barrier
      if (wave == 0) x = g[(x & 1023) + lane];
      __syncthreads();
    } else if (MODE == 4) {  // wave 0: a global store, then a dependent global load
      if (wave == 0) {
        out[16 + (it & 255) * 64 + lane] = x;
        x = g[(x & 1023) + lane];
      }
      __syncthreads();
    } else if (MODE == 5) {  // wave 0: a global store, then 8 dependent LDS reads
      if (wave == 0) {
        out[16 + (it & 255) * 64 + lane] = x;
        for (int k = 0; k < 8; k++) x = chain[x & 1023];
      }
      __syncthreads();
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) {
    out[0] = acc + x;
    cyc[0] = t1 - t0;
  }
}

template <int NT, int MODE>
static void run(const char* name, uint32_t* out, const uint32_t* g, uint64_t* cyc) {
  const uint32_t iters = 100000;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  floor_kernel<NT, MODE><<<1, NT>>>(1000, out, g, cyc);
  hipEventRecord(a);
  floor_kernel<NT, MODE><<<1, NT>>>(iters, out, g, cyc);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  uint64_t c = 0;
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("NT=%4d %-22s %8.1f ns/iter %8.1f cycles/iter\n", NT, name, ms * 1e6 / iters, (double)c / iters);
}

int main() {
  uint32_t *out, *g;
  uint64_t* cyc;
  hipMalloc(&out, (16 + 256 * 64) * 4);
  hipMalloc(&g, 4096 * 4);
  hipMemset(g, 0, 4096 * 4);
  hipMalloc(&cyc, 8);
#define ALL(NT)                                               \
  run<NT, 0>("barrier", out, g, cyc);                         \
  run<NT, 1>("block-min", out, g, cyc);                       \
  run<NT, 2>("8 dep LDS + barrier", out, g, cyc);             \
  run<NT, 3>("global RT + barrier", out, g, cyc);                \
  run<NT, 4>("store + global RT + bar", out, g, cyc);            \
  run<NT, 5>("store + 8 dep LDS + bar", out, g, cyc);
  ALL(256) ALL(512) ALL(1024)
  return 0;
}
