// Dev probe: kb_top2_lanes (k-means filter epilogue step B) against a
// brute-force top-2 over the 32 lanes of each half.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -o tools/bin/top2_probe tools/top2_probe.hip
#include "../spartan_amd/csrc/spx.hip"
#include <algorithm>
#include <vector>

__global__ void k_probe(const float* lo_in, const float* sec_in, float* lo_out, float* sec_out, int* li_out) {
  const int lane = threadIdx.x;
  float lo[16], sec[16];
  int li[16];
  for (int q = 0; q < 16; ++q) {
    lo[q] = lo_in[lane * 16 + q];
    sec[q] = sec_in[lane * 16 + q];
    li[q] = lane & 31;
  }
  kb_top2_lanes(lo, sec, li, lane);
  lo_out[lane] = lo[0];
  sec_out[lane] = sec[0];
  li_out[lane] = li[0];
}

int main() {
  std::vector<float> lo(64 * 16), sec(64 * 16);
  unsigned s = 12345;
  for (int i = 0; i < 64 * 16; ++i) {
    s = s * 1664525u + 1013904223u;
    lo[i] = (float)(s >> 8) / 16777216.0f;
    s = s * 1664525u + 1013904223u;
    sec[i] = lo[i] + (float)(s >> 8) / 16777216.0f;
  }
  float *dl, *ds, *ol, *os;
  int* oi;
  (void)hipMalloc(&dl, 4096 * 4); (void)hipMalloc(&ds, 4096 * 4);
  (void)hipMalloc(&ol, 256); (void)hipMalloc(&os, 256); (void)hipMalloc(&oi, 256);
  (void)hipMemcpy(dl, lo.data(), 4096, hipMemcpyHostToDevice);
  (void)hipMemcpy(ds, sec.data(), 4096, hipMemcpyHostToDevice);
  k_probe<<<1, 64>>>(dl, ds, ol, os, oi);
  float hl[64], hs[64];
  int hi[64];
  (void)hipMemcpy(hl, ol, 256, hipMemcpyDeviceToHost);
  (void)hipMemcpy(hs, os, 256, hipMemcpyDeviceToHost);
  (void)hipMemcpy(hi, oi, 256, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int lane = 0; lane < 64; ++lane) {
    const int h = lane >> 5, q = (lane & 31) >> 1;
    std::vector<std::pair<float, int>> all;
    for (int r = 0; r < 32; ++r) {
      all.push_back({lo[(32 * h + r) * 16 + q], r});
      all.push_back({sec[(32 * h + r) * 16 + q], 100 + r});
    }
    std::sort(all.begin(), all.end());
    const bool ok = hl[lane] == all[0].first && hs[lane] == all[1].first && hi[lane] == all[0].second;
    if (!ok) {
      ++bad;
      if (bad < 6) printf("lane %d: got (%g %g %d) want (%g %g %d)\n", lane, hl[lane], hs[lane], hi[lane],
                          all[0].first, all[1].first, all[0].second);
    }
  }
  printf("top2 probe: %d / 64 lanes wrong\n", bad);
  return bad != 0;
}
