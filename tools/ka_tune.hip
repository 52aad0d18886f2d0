// Dev tool: time variants of the k-means centroid accumulation
// (k_kmeans_accum in spartan_amd/csrc/spx.hip, included so the product
// kernel is what is timed) against pure streaming floors of the same
// (group, column-tile) partition.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -o tools/bin/ka_tune tools/ka_tune.hip
//   ./tools/bin/ka_tune <N> <D> <K>
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

__global__ void k_init(float* x, i64 n, i64* lab, i64 N, i64 K) {
  for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x) {
    uint64_t z = 0x9e3779b97f4a7c15ULL * (uint64_t)(i + 1);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    z ^= z >> 31;
    x[i] = (float)((z >> 40) * (1.0 / 16777216.0));
    if (i < N) lab[i] = (i64)((z >> 8) % (uint64_t)K);
  }
}

// streaming floor, partition as k_kmeans_accum: block (x, y) reads column
// tile y of groups x, x+G, ...; MODE 0: one float per lane per row (wave w
// rows w, w+16, ...), MODE 1: float4 per lane (16 lanes per row).
template <int MODE>
__global__ __launch_bounds__(1024) void k_stream(i64 N, i64 D, const float* __restrict__ P, i64 ldp, int ndb,
                                                 float* out) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int db = blockIdx.y % ndb;
  const i64 d0 = (i64)db * 64;
  const i64 ngr = (N + 255) / 256;
  float s = 0.f;
  for (i64 g = blockIdx.x; g < ngr; g += gridDim.x) {
    const i64 p0 = g * 256;
    if (MODE == 0) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const i64 p = p0 + w + 16 * k;
        if (p < N) s += P[p * ldp + d0 + lane];
      }
    } else {
      typedef float V __attribute__((ext_vector_type(4)));
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const i64 p = p0 + w * 16 + k * 4 + lane / 16;
        if (p < N) {
          V v = *(const V*)(P + p * ldp + d0 + (lane % 16) * 4);
          s += v[0] + v[1] + v[2] + v[3];
        }
      }
    }
  }
  if (s == 12345.f) out[0] = s;
}


// Variants of the LDS-accumulator design (float4 staging, one xs buffer):
// MODE 0 staging + barriers only, 1 one LDS read-add-write per point,
// 2 pipelined with run merge, 3 LDS fp64 atomics over (point, column)
// elements (non-deterministic: ceiling only).
template <int MODE>
__global__ __launch_bounds__(1024) void k_var(i64 N, i64 D, i64 K, const float* __restrict__ P, i64 ldp,
                                             const i64* __restrict__ labels, double* __restrict__ psum, int ndb) {
  constexpr int CH = 64, ST = 4;
  typedef float V __attribute__((ext_vector_type(4)));
  __shared__ double acc[256 * 64];
  __shared__ float xs[CH * 64];
  __shared__ int lab_s[CH];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int db = blockIdx.y % ndb;
  const i64 d0 = (i64)db * 64;
  const i64 nch = (N + CH - 1) / CH;
  const int lp = t / 16, lc = (t % 16) * 4;
  for (int i = t; i < 256 * 64; i += 1024) acc[i] = 0.0;
  V pf[ST];
  i64 plab[ST];
  auto load = [&](int s, i64 ch) {
    const i64 p0 = (ch < nch ? ch : nch - 1) * CH;
    const i64 pr = p0 + lp < N ? p0 + lp : N - 1;
    pf[s] = *(const V*)(P + pr * ldp + d0 + lc);
    if (t < CH) plab[s] = labels[p0 + t < N ? p0 + t : N - 1];
  };
  const i64 G = gridDim.x;
#pragma unroll
  for (int s = 0; s < ST; ++s) load(s, blockIdx.x + s * G);
  for (i64 base = blockIdx.x; base < nch; base += ST * G) {
#pragma unroll
    for (int s = 0; s < ST; ++s) {
      const i64 ch = base + s * G;
      if (ch >= nch) break;
      __syncthreads();
      *(V*)&xs[lp * 64 + lc] = pf[s];
      if (t < CH) lab_s[t] = (int)plab[s];
      __syncthreads();
      load(s, ch + ST * G);
      if (MODE == 0) {
        if (lab_s[lane] == 12345) acc[lane] += xs[lane];
      } else if (MODE == 3) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int e = t + 1024 * k, p = e / 64, c = e % 64;
          atomicAdd(&acc[lab_s[p] * 64 + c], (double)xs[e]);
        }
      } else {
        const int r = lab_s[lane];
        unsigned long long m = __ballot((r % 16) == w);
        if (MODE == 1) {
          while (m) {
            const int p = __ffsll((long long)m) - 1;
            m &= m - 1;
            const int rr = __builtin_amdgcn_readlane(r, p);
            acc[rr * 64 + lane] += (double)xs[p * 64 + lane];
          }
        } else if (m) {
          int p = __ffsll((long long)m) - 1;
          m &= m - 1;
          int rc = __builtin_amdgcn_readlane(r, p);
          double xc = (double)xs[p * 64 + lane];
          double ac = acc[rc * 64 + lane];
          while (m) {
            p = __ffsll((long long)m) - 1;
            m &= m - 1;
            const int rn = __builtin_amdgcn_readlane(r, p);
            const double xn = (double)xs[p * 64 + lane];
            if (rn == rc) {
              xc += xn;
              continue;
            }
            const double an = acc[rn * 64 + lane];
            acc[rc * 64 + lane] = ac + xc;
            rc = rn;
            xc = xn;
            ac = an;
          }
          acc[rc * 64 + lane] = ac + xc;
        }
      }
    }
  }
  __syncthreads();
  for (int i = t; i < 256 * 64; i += 1024) psum[(blockIdx.x * 256 + i / 64) * D + d0 + i % 64] = acc[i];
}

int main(int argc, char** argv) {
  const i64 N = argc > 1 ? atoll(argv[1]) : 100000000, D = argc > 2 ? atoll(argv[2]) : 128,
            K = argc > 3 ? atoll(argv[3]) : 256;
  float* P;
  i64* lab;
  CK(hipMalloc(&P, N * D * 4));
  CK(hipMalloc(&lab, N * 8));
  k_init<<<4096, 256>>>(P, N * D, lab, N, K);
  const int64_t ws = spx_kmeans_accumulate_workspace(SPX_F32, N, D, K);
  void* w;
  CK(hipMalloc(&w, ws));
  double* sums;
  uint64_t* cnts;
  CK(hipMalloc(&sums, K * D * 8));
  CK(hipMalloc(&cnts, K * 8));
  float* out;
  CK(hipMalloc(&out, 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  i64 G, ndb, ncb;
  ka_grid(SPX_F32, N, D, K, &G, &ndb, &ncb);
  const double gb = (double)N * D * 4 / 1e9;
  for (int round = 0; round < 2; ++round) {
    for (int v = 0; v < 7; ++v) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, 0));
      const char* name = "";
      if (v == 0) {
        name = "product k_kmeans_accum (+reduce)";
        if (spx_kmeans_accumulate(SPX_F32, N, D, K, P, D, lab, sums, cnts, 1, w, ws, 0)) printf("err %s\n", spx_last_error());
      } else if (v == 1) {
        name = "stream floor, 1 float/lane";
        k_stream<0><<<dim3((unsigned)G, (unsigned)(ndb * ncb)), 1024>>>(N, D, P, D, (int)ndb, out);
      } else if (v == 2) {
        name = "stream floor, float4/lane";
        k_stream<1><<<dim3((unsigned)G, (unsigned)(ndb * ncb)), 1024>>>(N, D, P, D, (int)ndb, out);
      } else {
        static const char* names[] = {"var: staging only", "var: 1 LDS RMW per point", "var: pipelined run merge",
                                      "var: LDS f64 atomics (nondeterministic)"};
        name = names[v - 3];
        double* ps = (double*)w;
        dim3 gr((unsigned)G, (unsigned)ndb);
        if (v == 3) k_var<0><<<gr, 1024>>>(N, D, K, P, D, lab, ps, (int)ndb);
        if (v == 4) k_var<1><<<gr, 1024>>>(N, D, K, P, D, lab, ps, (int)ndb);
        if (v == 5) k_var<2><<<gr, 1024>>>(N, D, K, P, D, lab, ps, (int)ndb);
        if (v == 6) k_var<3><<<gr, 1024>>>(N, D, K, P, D, lab, ps, (int)ndb);
      }
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("%-40s %8.3f ms  %7.1f GB/s\n", name, ms, gb / ms * 1e3);
    }
  }
  return 0;
}
