// Micro-benchmark (diagnostic): dependent-chain latency, in shader cycles, of
// the single-wave FFD building blocks on gfx950 -- LDS read, ds_bpermute,
// readlane round trip, ballot, DPP wave shift, s_memtime, dynamic VGPR index.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef uint32_t v32u __attribute__((ext_vector_type(32)));

template <int MODE>
__global__ __launch_bounds__(64, 1) void lat(uint32_t iters, uint32_t* out, uint64_t* cyc) {
  __shared__ uint32_t chain[4096];
  const uint32_t lane = threadIdx.x;
  for (uint32_t i = lane; i < 4096; i += 64) chain[i] = (i * 7 + 3) & 4095;
  __syncthreads();
  uint32_t x = lane, acc = 0;
  v32u V;
  for (int k = 0; k < 32; k++) V[k] = lane * 3 + k;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t it = 0; it < iters; it++) {
    if (MODE == 0) {  // dependent LDS read
      x = chain[x & 4095];
    } else if (MODE == 1) {  // dependent ds_bpermute
      x = (uint32_t)__shfl((int)x, (int)((x + 1) & 63)) + 1;
    } else if (MODE == 2) {  // VALU -> readlane -> SALU -> VALU
      x = __builtin_amdgcn_readlane((int)(x + lane), (int)(it & 63)) + lane;
    } else if (MODE == 3) {  // ballot -> ffs -> VALU
      const uint64_t b = __ballot((x & 3) == 0);
      x = x + (uint32_t)__ffsll((long long)b) + lane;
    } else if (MODE == 4) {  // DPP wave_shl1
      x = (uint32_t)__builtin_amdgcn_update_dpp((int)0, (int)x, 0x130, 0xF, 0xF, false) + 1;
    } else if (MODE == 5) {  // s_memtime
      acc += (uint32_t)__builtin_amdgcn_s_memtime();
      x += acc;
    } else if (MODE == 6) {  // dynamic VGPR index (extract)
      x = V[(x + it) & 31] + 1;
    } else if (MODE == 7) {  // dynamic VGPR index (insert + extract)
      V[(x + it) & 31] = x;
      x = V[(it * 5) & 31] + 1;
    } else if (MODE == 8) {  // LDS read-after-write by another lane (store, then dependent load)
      chain[(x + lane) & 4095] = x;
      x = chain[(x + 1) & 4095] + 1;
    } else if (MODE == 9) {  // 64-bit SWAR compare + ballot, dependent
      const uint64_t a = ((uint64_t)x << 20) | x, b = 0x0001000100010001ull * (x & 7);
      const bool ge = ((((a | 0x8000800080008000ull) - b) & 0x8000800080008000ull) == 0x8000800080008000ull);
      x += (uint32_t)__popcll(__ballot(ge)) + 1;
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[lane] = x + acc;
  for (int k = 0; k < 32; k++) out[64 + lane] += V[k];
  if (lane == 0) *cyc = t1 - t0;
}

template <int MODE>
static void run(const char* name, uint32_t* o, uint64_t* c) {
  const uint32_t iters = 100000;
  hipLaunchKernelGGL(lat<MODE>, dim3(1), dim3(64), 0, 0, iters, o, c);
  uint64_t cyc = 0;
  (void)hipMemcpy(&cyc, c, 8, hipMemcpyDeviceToHost);
  printf("%-28s %8.1f cycles per step\n", name, (double)cyc / iters);
}

int main() {
  uint32_t* o; uint64_t* c;
  (void)hipMalloc(&o, 4096); (void)hipMalloc(&c, 8);
  (void)hipMemset(o, 0, 4096);
  run<0>("lds_read_dep", o, c);
  run<1>("ds_bpermute_dep", o, c);
  run<2>("readlane_roundtrip", o, c);
  run<3>("ballot_ffs", o, c);
  run<4>("dpp_wave_shl1", o, c);
  run<5>("s_memtime", o, c);
  run<6>("vgpr_dyn_extract", o, c);
  run<7>("vgpr_dyn_insert_extract", o, c);
  run<8>("lds_store_then_load", o, c);
  run<9>("swar64_ballot", o, c);
  return 0;
}
