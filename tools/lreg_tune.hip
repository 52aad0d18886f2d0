// Dev tool: time shapes of the cfg5 (lreg) fused reduction -- the gradient
// g = sum_r x_r (x_r . w - y_r) over N x 64 fp32 rows, the kernel
// DotReduceFusion generates from codegen's column-reduce skeleton -- with V
// columns per lane (64 / V lanes per row: the row dot is summed across them
// by DPP), U rows per lane in flight, B blocks; interleaved rounds, each
// variant checked against an fp64 host sum.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -o tools/bin/lreg_tune tools/lreg_tune.hip
//   ./tools/bin/lreg_tune <N> <rounds>
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef long long i64;
typedef float f4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

__global__ void k_uniform(float* x, i64 n, unsigned long long seed) {
  for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x) {
    unsigned long long z = seed + 0x9e3779b97f4a7c15ULL * (unsigned long long)(i + 1);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    z ^= z >> 31;
    x[i] = (float)((z >> 40) * (1.0 / 16777216.0));
  }
}

template <int C>
__device__ __forceinline__ float dpp(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), C, 0xF, 0xF, false));
}

template <int LPR>
__device__ __forceinline__ float rowsum(float d) {
  if constexpr (LPR >= 2) d += dpp<0xB1>(d);
  if constexpr (LPR >= 4) d += dpp<0x4E>(d);
  if constexpr (LPR >= 8) d += dpp<0x141>(d);
  if constexpr (LPR >= 16) d += dpp<0x140>(d);
  return d;
}

template <int V, int U, bool NT>
__global__ __launch_bounds__(256) void k_lreg(i64 N, const float* __restrict__ X, const float* __restrict__ y,
                                              const float* __restrict__ w, float* __restrict__ part, i64 chunk) {
  constexpr int LPR = 64 / V, RPW = 64 / LPR;
  static_assert(LPR <= 16, "row dot within one DPP row");
  __shared__ float sv[4 * RPW * 64];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int sub = lane / LPR, cl = lane % LPR, col = cl * V;
  float wr[V], acc[V];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    wr[i] = w[col + i];
    acc[i] = 0.f;
  }
  const i64 r0 = (i64)blockIdx.x * chunk;
  const i64 r1 = r0 + chunk < N ? r0 + chunk : N;
  constexpr i64 STEP = 4 * RPW;
  i64 r = r0 + wv * RPW + sub;
  auto ld = [&](i64 row, float (&x)[V], float& yy) __attribute__((always_inline)) {
    const f4* p = (const f4*)(X + row * 64 + col);
#pragma unroll
    for (int q = 0; q < V / 4; ++q) {
      const f4 v = NT ? __builtin_nontemporal_load(p + q) : p[q];
#pragma unroll
      for (int e = 0; e < 4; ++e) x[4 * q + e] = v[e];
    }
    yy = NT ? __builtin_nontemporal_load(y + row) : y[row];
  };
  auto use = [&](const float (&x)[V], float yy) __attribute__((always_inline)) {
    float d = 0.f;
#pragma unroll
    for (int i = 0; i < V; ++i) d = __builtin_fmaf(x[i], wr[i], d);
    d = rowsum<LPR>(d);
    const float res = d - yy;
#pragma unroll
    for (int i = 0; i < V; ++i) acc[i] = __builtin_fmaf(x[i], res, acc[i]);
  };
  for (; r + (U - 1) * STEP < r1; r += U * STEP) {
    float x[U][V], yy[U];
#pragma unroll
    for (int u = 0; u < U; ++u) ld(r + u * STEP, x[u], yy[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) use(x[u], yy[u]);
  }
  for (; r < r1; r += STEP) {
    float x[V], yy;
    ld(r, x, yy);
    use(x, yy);
  }
#pragma unroll
  for (int i = 0; i < V; ++i) sv[(wv * RPW + sub) * 64 + col + i] = acc[i];
  __syncthreads();
  if (t < 64) {
    float s = 0.f;
    for (int g = 0; g < 4 * RPW; ++g) s += sv[g * 64 + t];
    part[(i64)blockIdx.x * 64 + t] = s;
  }
}

__global__ void k_sum_parts(const float* part, int B, double* g) {
  const int t = threadIdx.x;
  if (t < 64) {
    double s = 0.0;
    for (int b = 0; b < B; ++b) s += part[(i64)b * 64 + t];
    g[t] = s;
  }
}

typedef void (*Fn)(int, i64, const float*, const float*, const float*, float*, i64);
template <int V, int U, bool NT>
static void launch(int B, i64 N, const float* X, const float* y, const float* w, float* part, i64 chunk) {
  k_lreg<V, U, NT><<<B, 256>>>(N, X, y, w, part, chunk);
}
struct Var {
  const char* name;
  Fn fn;
  int B;
};
#define VAR(V, U, NT, B) {"V" #V " U" #U " NT" #NT " B" #B, &launch<V, U, NT>, B}

int main(int argc, char** argv) {
  const i64 N = argc > 1 ? atoll(argv[1]) : 100000000;
  const int rounds = argc > 2 ? atoi(argv[2]) : 3;
  Var vars[] = {VAR(4, 4, false, 2048),  VAR(4, 8, false, 2048),  VAR(4, 4, false, 1024),  VAR(8, 2, false, 2048),
                VAR(8, 4, false, 2048),  VAR(8, 4, false, 1024),  VAR(16, 1, false, 2048), VAR(16, 2, false, 2048),
                VAR(16, 2, false, 1024), VAR(16, 4, false, 1024), VAR(4, 4, true, 2048),  VAR(8, 4, true, 2048),
                VAR(16, 2, true, 2048),  VAR(8, 2, false, 4096),  VAR(16, 2, false, 4096)};
  const int nv = sizeof(vars) / sizeof(vars[0]);
  float *X, *y, *w, *part;
  double* g;
  CK(hipMalloc(&X, N * 64 * 4));
  CK(hipMalloc(&y, N * 4));
  CK(hipMalloc(&w, 64 * 4));
  CK(hipMalloc(&part, 4096 * 64 * 4));
  CK(hipMalloc(&g, 64 * 8));
  k_uniform<<<4096, 256>>>(X, N * 64, 41);
  k_uniform<<<4096, 256>>>(y, N, 42);
  k_uniform<<<1, 64>>>(w, 64, 43);
  CK(hipDeviceSynchronize());
  // reference gradient: fp64 host over a strided sample is not enough for a
  // full check, so every variant is compared with the first (relative to
  // sum |x||r| estimated from the first variant's |g|)
  std::vector<double> g0(64), gv(64);
  std::vector<double> best(nv, 1e30);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double bytes = 4.0 * N * 64 + 4.0 * N;
  for (int rd = 0; rd < rounds; ++rd) {
    for (int v = 0; v < nv; ++v) {
      const int B = vars[v].B;
      const i64 chunk = (N + B - 1) / B;
      vars[v].fn(B, N, X, y, w, part, chunk);  // warm
      CK(hipEventRecord(e0));
      const int reps = 5;
      for (int k = 0; k < reps; ++k) vars[v].fn(B, N, X, y, w, part, chunk);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= reps;
      if (ms < best[v]) best[v] = ms;
      k_sum_parts<<<1, 64>>>(part, B, g);
      CK(hipMemcpy(gv.data(), g, 64 * 8, hipMemcpyDeviceToHost));
      if (v == 0 && rd == 0) g0 = gv;
      double worst = 0.0;
      for (int c = 0; c < 64; ++c) worst = fmax(worst, fabs(gv[c] - g0[c]) / fabs(g0[c]));
      if (rd == rounds - 1)
        printf("%-22s best %.3f ms  %.1f GB/s  (%.3f of 8 TB/s)  max rel diff vs first %.2e\n", vars[v].name, best[v],
               bytes / best[v] / 1e6, bytes / best[v] / 1e6 / 8000.0, worst);
    }
  }
  return 0;
}
