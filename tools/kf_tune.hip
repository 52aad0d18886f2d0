// Dev tool: time configurations of the k-means certified filter kernel
// (k_kmeans_filter in spartan_amd/csrc/spx.hip, included here so the tuner
// times the product code) on U[0,1) points, interleaved rounds; every
// configuration must certify the same points with the same labels and leave
// the same undecided counts as the first.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -o tools/bin/kf_tune tools/kf_tune.hip
//   ./tools/bin/kf_tune <N> <D> <K> <rounds>
#include "../spartan_amd/csrc/spx.hip"

#include <cstdlib>
#include <vector>

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

typedef void (*LaunchFn)(i64, hipStream_t, i64, i64, i64, i64, const void*, i64, const float*, const double*,
                         const double*, i64*, unsigned int*, i64*, KfCand*);
struct Var {
  const char* name;
  int bm;
  LaunchFn fn;
};
#define VAR(BM, PA, PB, MW) \
  { "BM" #BM " PA" #PA " PB" #PB " W" #MW, BM, &KfConf<BM, PA, PB, MW>::launch<float, true> }

int main(int argc, char** argv) {
  const i64 N = argc > 1 ? atoll(argv[1]) : 4000000, D = argc > 2 ? atoll(argv[2]) : 128;
  const i64 K = argc > 3 ? atoll(argv[3]) : 256;
  const int rounds = argc > 4 ? atoi(argv[4]) : 5;
  Var vars[] = {VAR(64, 2, 0, 3),   VAR(64, 32, 32, 3), VAR(64, 32, 32, 2),  VAR(64, 2, 0, 2),
                VAR(128, 2, 0, 2),  VAR(128, 32, 32, 2), VAR(128, 32, 32, 4), VAR(256, 32, 32, 4),
                VAR(256, 2, 0, 4)};
  const int nv = sizeof(vars) / sizeof(vars[0]);
  float* P;
  double* C;
  CK(hipMalloc(&P, N * D * 4));
  CK(hipMalloc(&C, K * D * 8));
  k_uniform<<<4096, 256>>>(P, N * D, 21);
  k_to_f64<<<64, 256>>>(P, C, K * D);  // centres = first K points
  const i64 Kp = kf_kp(K);
  const i64 ws_bytes = spx_kmeans_assign_workspace(SPX_F32, N, D, K);
  unsigned char* ws;
  CK(hipMalloc(&ws, ws_bytes));
  float* CT = (float*)ws;
  unsigned char* q = ws + (D * Kp * 4 + 15) / 16 * 16;
  double* cn = (double*)q;
  q += Kp * 8;
  double* cmax = (double*)q;
  q += 16;
  unsigned int* counters = (unsigned int*)q;
  q += 16;
  i64* full_list = (i64*)q;
  q += N * 8;
  KfCand* cand = (KfCand*)q;
  k_kmeans_prep<<<1, 256>>>(D, K, Kp, C, CT, cn, cmax, 0.0);  // fp64 distances: no fp32 tie margin
  i64* lab;
  CK(hipMalloc(&lab, N * 8));
  std::vector<i64> ref(N), got(N);
  unsigned int cref[2] = {0, 0};
  std::vector<double> best(nv, 1e30);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < rounds; ++r) {
    for (int v = 0; v < nv; ++v) {
      CK(hipMemset(lab, 0xff, N * 8));
      CK(hipMemset(counters, 0, 8));
      const i64 g = (N + vars[v].bm - 1) / vars[v].bm;
      CK(hipEventRecord(e0));
      vars[v].fn(g, 0, N, D, K, Kp, P, D, CT, cn, cmax, lab, counters, full_list, cand);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipGetLastError());
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best[v]) best[v] = ms;
      unsigned int c[2];
      CK(hipMemcpy(c, counters, 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(got.data(), lab, N * 8, hipMemcpyDeviceToHost));
      if (r == 0 && v == 0) {
        ref = got;
        cref[0] = c[0];
        cref[1] = c[1];
        printf("undecided: full %u, candidate %u of %lld (%.3f%%)\n", c[0], c[1], (long long)N,
               100.0 * (c[0] + c[1]) / N);
      } else if (got != ref || c[0] != cref[0] || c[1] != cref[1]) {
        printf("MISMATCH %s\n", vars[v].name);
        return 1;
      }
    }
  }
  const double flops = 2.0 * N * Kp * D;
  for (int v = 0; v < nv; ++v)
    printf("%-22s %8.3f ms  %7.1f TF/s (%.1f%% of 157.3)\n", vars[v].name, best[v], flops / best[v] / 1e9,
           flops / best[v] / 1e9 / 1573.0);
  return 0;
}
