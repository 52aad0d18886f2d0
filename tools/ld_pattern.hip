// Dev microbenchmark (GPU box): HBM read rate of the k-means screen's A-load
// pattern (lane (h, r) of a wave reads row r of a 32-row tile, 16-byte pieces,
// 32 rows x 32 B per instruction) against a coalesced pattern over the same
// bytes (1 KiB contiguous per instruction), persistent grid of one 512-thread
// block per CU like the screen.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/ld_pattern tools/ld_pattern.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef float f4 __attribute__((ext_vector_type(4)));
typedef long long i64;

template <int MODE, int W>
__global__ __launch_bounds__(W * 64) void k_ld(i64 N, const float* __restrict__ P, float* __restrict__ out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const i64 ntiles = N / 32;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (i64 tile = (i64)blockIdx.x * W + w; tile < ntiles; tile += (i64)gridDim.x * W) {
    f4 ra[16];
    if (MODE == 0) {
      const float* p = P + (tile * 32 + r) * 128 + 4 * h;
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        ra[2 * ks] = *(const f4*)(p + ks * 16);
        ra[2 * ks + 1] = *(const f4*)(p + ks * 16 + 8);
      }
    } else if (MODE == 1) {
      const float* p = P + tile * 32 * 128 + 4 * lane;
#pragma unroll
      for (int j = 0; j < 16; ++j) ra[j] = *(const f4*)(p + j * 256);
    } else {  // MODE 2: coalesced, non-temporal
      const float* p = P + tile * 32 * 128 + 4 * lane;
#pragma unroll
      for (int j = 0; j < 16; ++j) ra[j] = __builtin_nontemporal_load((const f4*)(p + j * 256));
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) acc += ra[j];
  }
  out[(blockIdx.x * W + w) * 64 + lane] = acc[0] + acc[1] + acc[2] + acc[3];
}

template <int MODE, int W>
static float run(i64 N, const float* P, float* out, int grid) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k_ld<MODE, W><<<grid, W * 64>>>(N, P, out);
  hipEventRecord(e0);
  const int reps = 10;
  for (int i = 0; i < reps; ++i) k_ld<MODE, W><<<grid, W * 64>>>(N, P, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

int main(int argc, char** argv) {
  const i64 N = argc > 1 ? atoll(argv[1]) : 100000000LL;
  float* P;
  float* out;
  if (hipMalloc(&P, (size_t)N * 128 * 4) != hipSuccess || hipMalloc(&out, 1 << 24) != hipSuccess) return 1;
  hipMemset(P, 0, (size_t)N * 128 * 4);
  const double gb = (double)N * 128 * 4 / 1e9;
  float t;
  t = run<0, 8>(N, P, out, 256);  printf("screen pattern   8 waves/CU: %7.3f ms  %7.1f GB/s\n", t, gb / t * 1e3);
  t = run<1, 8>(N, P, out, 256);  printf("coalesced        8 waves/CU: %7.3f ms  %7.1f GB/s\n", t, gb / t * 1e3);
  t = run<0, 16>(N, P, out, 256); printf("screen pattern  16 waves/CU: %7.3f ms  %7.1f GB/s\n", t, gb / t * 1e3);
  t = run<1, 16>(N, P, out, 256); printf("coalesced       16 waves/CU: %7.3f ms  %7.1f GB/s\n", t, gb / t * 1e3);
  t = run<0, 8>(N, P, out, 512);  printf("screen pattern  2x8 waves/CU: %7.3f ms  %7.1f GB/s\n", t, gb / t * 1e3);
  t = run<2, 8>(N, P, out, 256);  printf("coalesced nt     8 waves/CU: %7.3f ms  %7.1f GB/s\n", t, gb / t * 1e3);
  t = run<2, 16>(N, P, out, 256); printf("coalesced nt    16 waves/CU: %7.3f ms  %7.1f GB/s\n", t, gb / t * 1e3);
  t = run<2, 16>(N, P, out, 512); printf("coalesced nt  2x16 waves/CU: %7.3f ms  %7.1f GB/s\n", t, gb / t * 1e3);
  t = run<1, 16>(N, P, out, 512); printf("coalesced     2x16 waves/CU: %7.3f ms  %7.1f GB/s\n", t, gb / t * 1e3);
  return 0;
}
