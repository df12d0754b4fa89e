// DPP wave_shl:1 / wave_shr:1 lane direction on gfx950 (which lane each lane reads)
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(int* o) {
  const int x = threadIdx.x;
  o[threadIdx.x] = __builtin_amdgcn_update_dpp(-1, x, 0x130, 0xF, 0xF, false);
  o[64 + threadIdx.x] = __builtin_amdgcn_update_dpp(-1, x, 0x138, 0xF, 0xF, false);
  o[128 + threadIdx.x] = __builtin_amdgcn_update_dpp(-1, x, 0x134, 0xF, 0xF, false);  // wave_rol1
  o[192 + threadIdx.x] = __builtin_amdgcn_update_dpp(-1, x, 0x13C, 0xF, 0xF, false);  // wave_ror1
}
int main() {
  int* d; hipMalloc(&d, 256 * 4); k<<<1, 64>>>(d); int h[256]; hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  const char* nm[4] = {"shl1", "shr1", "rol1", "ror1"};
  for (int t = 0; t < 4; t++) { printf("%s:", nm[t]); for (int i = 0; i < 64; i++) printf(" %d", h[t * 64 + i]); printf("\n"); }
  return 0;
}
