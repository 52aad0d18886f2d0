// Dev probe: lane mapping of v_permlane16_swap_b32 and the DPP row_mirror /
// row_half_mirror / quad_perm moves used by the k-means filter epilogue.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/perm_probe tools/perm_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
  const unsigned l = threadIdx.x;
  auto r = __builtin_amdgcn_permlane16_swap(l, 100u + l, false, false);
  out[l] = r[0];
  out[64 + l] = r[1];
  out[128 + l] = __builtin_amdgcn_update_dpp(0, (int)l, 0x140, 0xF, 0xF, false);
  out[192 + l] = __builtin_amdgcn_update_dpp(0, (int)l, 0x141, 0xF, 0xF, false);
  out[256 + l] = __builtin_amdgcn_update_dpp(0, (int)l, 0x4E, 0xF, 0xF, false);
  out[320 + l] = __builtin_amdgcn_update_dpp(0, (int)l, 0xB1, 0xF, 0xF, false);
}
int main() {
  unsigned* d;
  unsigned h[384];
  (void)hipMalloc(&d, sizeof(h));
  k<<<1, 64>>>(d);
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* names[] = {"swap.vdst", "swap.vsrc", "row_mirror", "row_half_mirror", "quad 0x4E", "quad 0xB1"};
  for (int t = 0; t < 6; ++t) {
    printf("%-16s", names[t]);
    for (int l = 0; l < 64; ++l) printf(" %u", h[64 * t + l]);
    printf("\n");
  }
  return 0;
}
