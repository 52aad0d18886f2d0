// Dev tool: time the bf16x3 k-means filter kernel (k_kmeans_filter_b3 in
// spartan_amd/csrc/spx.hip, included) alone; build twice, with and without
// -DKB_DEV_NO_EPILOGUE, to split main loop and epilogue.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 [-DKB_DEV_NO_EPILOGUE] -o tools/bin/kb_split tools/kb_split.hip
//   ./tools/bin/kb_split <N> <D> <K>
#include "../spartan_amd/csrc/spx.hip"

#include <cstdlib>

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

__global__ void k_uniform(float* x, i64 n, uint64_t seed) {
  for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x) {
    uint64_t z = seed + 0x9e3779b97f4a7c15ULL * (uint64_t)(i + 1);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    z ^= z >> 31;
    x[i] = (float)((z >> 40) * (1.0 / 16777216.0));
  }
}

__global__ void k_to_f64(const float* x, double* y, i64 n) {
  for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x) y[i] = x[i];
}

int main(int argc, char** argv) {
  const i64 N = argc > 1 ? atoll(argv[1]) : 20000000, D = argc > 2 ? atoll(argv[2]) : 128;
  const i64 K = argc > 3 ? atoll(argv[3]) : 256;
  float* P;
  double* C;
  CK(hipMalloc(&P, N * D * 4));
  CK(hipMalloc(&C, K * D * 8));
  k_uniform<<<4096, 256>>>(P, N * D, 21);
  k_to_f64<<<64, 256>>>(P, C, K * D);
  const i64 Kp = kf_kp(K);
  const i64 ws_bytes = spx_kmeans_assign_workspace(SPX_F32, N, D, K);
  unsigned char* ws;
  CK(hipMalloc(&ws, ws_bytes));
  unsigned char* q = ws;
  __bf16* CBh = (__bf16*)q;
  __bf16* CBl = CBh + 256 * D;
  q += (D * Kp * 4 + 15) / 16 * 16;
  float* cnf = (float*)q;
  q += Kp * 8;
  double* cmax = (double*)q;
  q += 16;
  unsigned int* counters = (unsigned int*)q;
  q += 16;
  i64* full_list = (i64*)q;
  q += N * 8;
  KfCand* cand = (KfCand*)q;
  k_kmeans_prep_b3<<<1, 256>>>(D, K, 256, C, CBh, CBl, cnf, cmax);
  i64* lab;
  CK(hipMalloc(&lab, N * 8));
  int dev = 0, ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CK(hipMemset(counters, 0, 8));
    CK(hipEventRecord(e0));
    kb_launch<8>(0, N, D, P, D, CBh, CBl, cnf, cmax, lab, counters, full_list, cand, ncu);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipGetLastError());
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
  }
  unsigned int c[2];
  CK(hipMemcpy(c, counters, 8, hipMemcpyDeviceToHost));
  const double flops = 3.0 * 2.0 * N * 256 * D;
#ifdef KB_DEV_NO_EPILOGUE
  const char* mode = "main loop only";
#else
  const char* mode = "full kernel";
#endif
  printf("%-16s N=%lld: %8.3f ms  bf16 %7.1f TF/s (%.1f%% of 2500)  undecided %u + %u\n", mode, (long long)N, best,
         flops / best / 1e9, flops / best / 1e9 / 25.0, c[0], c[1]);
  return 0;
}
