// Dev tool: time GEMM configurations of spartan_amd/csrc/gemm_kernels.h (the
// product kernels) in one process, interleaved rounds (cdna_hip_programming.md
// 5.4 rule 24), each checked against the first configuration of its dtype.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -o tools/devbin/gemm_tune tools/gemm_tune.hip
//   ./tools/devbin/gemm_tune <size> <rounds> <f32|f64|both>
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../spartan_amd/csrc/gemm_kernels.h"

using spx_mfma::Config;
using spx_mfma::i64;

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

template <typename T>
struct Variant {
  std::string name;
  hipError_t (*launch)(i64, i64, i64, const T*, i64, const T*, i64, T*, i64, T, T, bool, hipStream_t);
};

#define V(T, BM, BN, BK, WM, WN, GM) \
  Variant<T>{#BM "x" #BN "x" #BK " w" #WM "x" #WN " g" #GM, Config<T, BM, BN, BK, WM, WN, GM>::launch}
#define VG(T, BM, BN, BK, WM, WN, GM, GFL) \
  Variant<T>{#BM "x" #BN "x" #BK " w" #WM "x" #WN " g" #GM " gfl" #GFL, Config<T, BM, BN, BK, WM, WN, GM, 0, GFL>::launch}
#define VS(T, BM, BN, BK, WM, WN, GM, SEG) \
  Variant<T>{#BM "x" #BN "x" #BK " w" #WM "x" #WN " g" #GM " seg" #SEG, Config<T, BM, BN, BK, WM, WN, GM, SEG>::launch}

template <typename T>
__global__ void init(T* p, i64 n, unsigned seed) {
  for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x) {
    unsigned long long z = (i + 1) * 0x9E3779B97F4A7C15ULL + seed;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    p[i] = (T)((double)((z ^ (z >> 31)) >> 11) * 1.1102230246251565e-16);
  }
}

// max over all elements of |C - R| / max(|R|, 1e-30), as ordered int bits (non-negative floats)
template <typename T>
__global__ void maxrel(const T* C, const T* R, i64 n, unsigned int* out) {
  float m = 0.f;
  for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x) {
    const double r = (double)R[i], d = fabs((double)C[i] - r) / fmax(fabs(r), 1e-30);
    m = fmaxf(m, d == d ? (float)d : 3e38f);
  }
  atomicMax(out, __float_as_uint(m));
}

hipError_t p3_8(i64 M, i64 N, i64 K, const float* A, i64 lda, const float* B, i64 ldb, float* C, i64 ldc, float alpha,
                float beta, bool, hipStream_t s) {
  return spx_mfma::p3_launch<8>(M, N, K, A, lda, B, ldb, C, ldc, alpha, beta, s);
}
hipError_t p3_4(i64 M, i64 N, i64 K, const float* A, i64 lda, const float* B, i64 ldb, float* C, i64 ldc, float alpha,
                float beta, bool, hipStream_t s) {
  return spx_mfma::p3_launch<4>(M, N, K, A, lda, B, ldb, C, ldc, alpha, beta, s);
}
hipError_t p3_16(i64 M, i64 N, i64 K, const float* A, i64 lda, const float* B, i64 ldb, float* C, i64 ldc, float alpha,
                 float beta, bool, hipStream_t s) {
  return spx_mfma::p3_launch<16>(M, N, K, A, lda, B, ldb, C, ldc, alpha, beta, s);
}
hipError_t p3_fl(i64 M, i64 N, i64 K, const float* A, i64 lda, const float* B, i64 ldb, float* C, i64 ldc,
                 float alpha, float beta, bool, hipStream_t s) {
  return spx_mfma::p3_launch<8, 0, 512>(M, N, K, A, lda, B, ldb, C, ldc, alpha, beta, s);
}
hipError_t p3_flbt(i64 M, i64 N, i64 K, const float* A, i64 lda, const float* B, i64 ldb, float* C, i64 ldc,
                   float alpha, float beta, bool, hipStream_t s) {
  return spx_mfma::p3_launch<8, 0, 512, 1>(M, N, K, A, lda, B, ldb, C, ldc, alpha, beta, s);
}
hipError_t p3_bt(i64 M, i64 N, i64 K, const float* A, i64 lda, const float* B, i64 ldb, float* C, i64 ldc,
                 float alpha, float beta, bool, hipStream_t s) {
  return spx_mfma::p3_launch<8, 0, 0, 1>(M, N, K, A, lda, B, ldb, C, ldc, alpha, beta, s);
}
template <int WN, int FL>
hipError_t p3g(i64 M, i64 N, i64 K, const float* A, i64 lda, const float* B, i64 ldb, float* C, i64 ldc, float alpha,
               float beta, bool, hipStream_t s) {
  return spx_mfma::p3_launch<8, 0, FL, 1, WN, 1, 1>(M, N, K, A, lda, B, ldb, C, ldc, alpha, beta, s);
}
template <int ABL>
hipError_t p3wa(i64 M, i64 N, i64 K, const float* A, i64 lda, const float* B, i64 ldb, float* C, i64 ldc, float alpha,
                float beta, bool, hipStream_t s) {
  return spx_mfma::p3_launch<8, ABL, 0, 1, 4>(M, N, K, A, lda, B, ldb, C, ldc, alpha, beta, s);
}
template <int WN, int BT, int FL, int SCH = 1, int GM = 8>
hipError_t p3w(i64 M, i64 N, i64 K, const float* A, i64 lda, const float* B, i64 ldb, float* C, i64 ldc, float alpha,
               float beta, bool, hipStream_t s) {
  return spx_mfma::p3_launch<GM, 0, FL, BT, WN, SCH>(M, N, K, A, lda, B, ldb, C, ldc, alpha, beta, s);
}
// the K-chunked form spx_gemm runs: chains of at most 8192 k, beta = 1 after the first chunk
hipError_t p3_8c(i64 M, i64 N, i64 K, const float* A, i64 lda, const float* B, i64 ldb, float* C, i64 ldc,
                 float alpha, float beta, bool, hipStream_t s) {
  for (i64 k0 = 0; k0 < K; k0 += 8192) {
    const i64 kc = K - k0 < 8192 ? K - k0 : 8192;
    hipError_t e = spx_mfma::p3_launch<8>(M, N, kc, A + k0, lda, B + k0 * ldb, ldb, C, ldc, alpha, k0 ? 1.f : beta, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

template <int WN, int GM = 8, int ABL = 0>
hipError_t p3dw(i64 M, i64 N, i64 K, const double* A, i64 lda, const double* B, i64 ldb, double* C, i64 ldc,
                double alpha, double beta, bool, hipStream_t s) {
  return spx_mfma::p3d_launch<GM, 16, ABL, WN>(M, N, K, A, lda, B, ldb, C, ldc, alpha, beta, s);
}
template <int ABL>
hipError_t p3da(i64 M, i64 N, i64 K, const double* A, i64 lda, const double* B, i64 ldb, double* C, i64 ldc,
                double alpha, double beta, bool, hipStream_t s) {
  return spx_mfma::p3d_launch<8, 16, ABL>(M, N, K, A, lda, B, ldb, C, ldc, alpha, beta, s);
}
hipError_t p3d_16(i64 M, i64 N, i64 K, const double* A, i64 lda, const double* B, i64 ldb, double* C, i64 ldc,
                  double alpha, double beta, bool, hipStream_t s) {
  return spx_mfma::p3d_launch<8, 16>(M, N, K, A, lda, B, ldb, C, ldc, alpha, beta, s);
}

template <int ABL>
hipError_t p3a(i64 M, i64 N, i64 K, const float* A, i64 lda, const float* B, i64 ldb, float* C, i64 ldc, float alpha,
               float beta, bool, hipStream_t s) {
  return spx_mfma::p3_launch<8, ABL>(M, N, K, A, lda, B, ldb, C, ldc, alpha, beta, s);
}

template <typename T>
void run(i64 S, int rounds, std::vector<Variant<T>> vs, double peak) {
  T *A, *B, *C, *R;
  size_t n = (size_t)S * S;
  CK(hipMalloc(&A, n * sizeof(T)));
  CK(hipMalloc(&B, n * sizeof(T)));
  CK(hipMalloc(&C, n * sizeof(T)));
  CK(hipMalloc(&R, n * sizeof(T)));
  init<<<4096, 256>>>(A, (i64)n, 1);
  init<<<4096, 256>>>(B, (i64)n, 2);
  CK(vs[0].launch(S, S, S, A, S, B, S, R, S, (T)1, (T)0, true, 0));
  CK(hipDeviceSynchronize());
  std::vector<T> ref(64), got(64);
  CK(hipMemcpy(ref.data(), R + 12345, 64 * sizeof(T), hipMemcpyDeviceToHost));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<float>> ms(vs.size());
  for (int r = 0; r < rounds; ++r)
    for (size_t v = 0; v < vs.size(); ++v) {
      CK(vs[v].launch(S, S, S, A, S, B, S, C, S, (T)1, (T)0, true, 0));
      CK(hipEventRecord(e0));
      CK(vs[v].launch(S, S, S, A, S, B, S, C, S, (T)1, (T)0, true, 0));
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms[v].push_back(t);
      CK(hipMemcpy(got.data(), C + 12345, 64 * sizeof(T), hipMemcpyDeviceToHost));
      double err = 0;
      for (int i = 0; i < 64; ++i) err = fmax(err, fabs((double)got[i] - (double)ref[i]) / fabs((double)ref[i]));
      if (err > (sizeof(T) == 8 ? 1e-12 : 1e-5)) printf("  MISMATCH %s rel %g\n", vs[v].name.c_str(), err);
    }
  {  // every element of every variant against the first
    unsigned int* dm;
    CK(hipMalloc(&dm, 4));
    for (size_t v = 1; v < vs.size(); ++v) {
      CK(hipMemset(dm, 0, 4));
      CK(vs[v].launch(S, S, S, A, S, B, S, C, S, (T)1, (T)0, true, 0));
      maxrel<T><<<1024, 256>>>(C, R, (i64)n, dm);
      unsigned int hm;
      CK(hipMemcpy(&hm, dm, 4, hipMemcpyDeviceToHost));
      float fm;
      memcpy(&fm, &hm, 4);
      printf("  %-24s max rel diff vs %s over all %zu elements: %.3g\n", vs[v].name.c_str(), vs[0].name.c_str(), n, fm);
    }
    CK(hipFree(dm));
  }
  double fl = 2.0 * S * S * S;
  for (size_t v = 0; v < vs.size(); ++v) {
    float best = 1e30f;
    for (float t : ms[v]) best = fminf(best, t);
    printf("%s %-24s S=%lld best %9.3f ms %7.1f TF (%.1f%% of %.1f)\n", sizeof(T) == 8 ? "f64" : "f32",
           vs[v].name.c_str(), (long long)S, best, fl / best / 1e9, fl / best / 1e9 / peak * 100, peak);
  }
  CK(hipFree(A));
  CK(hipFree(B));
  CK(hipFree(C));
  CK(hipFree(R));
}

int main(int argc, char** argv) {
  i64 S = argc > 1 ? atoll(argv[1]) : 8192;
  int rounds = argc > 2 ? atoi(argv[2]) : 2;
  std::string which = argc > 3 ? argv[3] : "both";
  if (which == "big") {  // round 6: one wave per SIMD with 128 x 128 (or 128 x 64) wave tiles, against the product
    run<float>(S, rounds,
               {VG(float, 256, 128, 16, 4, 2, 8, 512), VG(float, 256, 256, 16, 2, 2, 8, 512),
                VG(float, 256, 256, 32, 2, 2, 8, 256), VG(float, 256, 128, 16, 2, 1, 8, 512),
                VG(float, 128, 256, 16, 1, 2, 8, 512), VG(float, 256, 256, 16, 2, 4, 8, 512),
                VG(float, 256, 128, 32, 2, 2, 8, 256)},
               157.3);
    run<double>(S, rounds,
                {V(double, 128, 128, 16, 4, 4, 0), V(double, 128, 128, 16, 2, 2, 0), V(double, 128, 128, 16, 2, 2, 8),
                 V(double, 256, 128, 16, 2, 2, 8), V(double, 128, 128, 32, 2, 2, 8), V(double, 256, 256, 16, 2, 2, 8),
                 V(double, 128, 256, 16, 2, 2, 8)},
                78.6);
    return 0;
  }
  if (which == "p3") {  // the three-stage one-wave-per-SIMD kernel against the product
    run<float>(S, rounds,
               {VG(float, 256, 128, 16, 4, 2, 8, 512), Variant<float>{"p3 g8", p3_8}, Variant<float>{"p3 g4", p3_4},
                Variant<float>{"p3 g16", p3_16}, Variant<float>{"p3 g8 kchunk8192", p3_8c},
                Variant<float>{"p3 g8 fl512", p3_fl}},
               157.3);
    return 0;
  }
  if (which == "p3bt") {  // B as one ds_read_b128 per step (interleaved columns)
    run<float>(S, rounds,
               {VG(float, 256, 128, 16, 4, 2, 8, 512), Variant<float>{"p3 fl512", p3_fl},
                Variant<float>{"p3 fl512 bt", p3_flbt}, Variant<float>{"p3", p3_8}, Variant<float>{"p3 bt", p3_bt}},
               157.3);
    return 0;
  }
  if (which == "p3gl") {  // staging by global_load_lds
    run<float>(S, rounds,
               {Variant<float>{"p3 w8 bt fl512", p3w<4, 1, 512>}, Variant<float>{"p3 w8 bt fl512 glds", p3g<4, 512>},
                Variant<float>{"p3 w4 bt fl512 glds", p3g<2, 512>}, Variant<float>{"p3 w8 bt glds", p3g<4, 0>}},
               157.3);
    return 0;
  }
  if (which == "p3wabl") {  // ablations of the 8-wave form (wrong results by design past 0)
    run<float>(S, rounds,
               {Variant<float>{"p3w8", p3wa<0>}, Variant<float>{"p3w8 abl1 no-ldst", p3wa<1>},
                Variant<float>{"p3w8 abl2 +no-bar", p3wa<2>}, Variant<float>{"p3w8 abl3 +no-aread", p3wa<3>},
                Variant<float>{"p3w8 abl4 +no-bread", p3wa<4>}},
               157.3);
    return 0;
  }
  if (which == "p3w2") {  // the 8-wave form: scheduling and grouping
    run<float>(S, rounds,
               {Variant<float>{"p3 w8 bt fl512", p3w<4, 1, 512>}, Variant<float>{"p3 w8 bt fl512 nosch", p3w<4, 1, 512, 0>},
                Variant<float>{"p3 w8 bt fl512 g4", p3w<4, 1, 512, 1, 4>},
                Variant<float>{"p3 w8 bt fl512 g16", p3w<4, 1, 512, 1, 16>},
                Variant<float>{"p3 w8 bt fl1024", p3w<4, 1, 1024>}},
               157.3);
    return 0;
  }
  if (which == "p3w") {  // 4 waves (one per SIMD) vs 8 waves (two per SIMD) of the three-stage kernel
    run<float>(S, rounds,
               {VG(float, 256, 128, 16, 4, 2, 8, 512), Variant<float>{"p3 w4 bt fl512", p3w<2, 1, 512>},
                Variant<float>{"p3 w8 bt fl512", p3w<4, 1, 512>}, Variant<float>{"p3 w8 fl512", p3w<4, 0, 512>},
                Variant<float>{"p3 w8 bt", p3w<4, 1, 0>}},
               157.3);
    return 0;
  }
  if (which == "p3abl") {  // ablations of the p3 kernel (results wrong by design for 1-3)
    run<float>(S, rounds,
               {Variant<float>{"p3", p3a<0>}, Variant<float>{"p3 abl1 no-ldst", p3a<1>},
                Variant<float>{"p3 abl2 +no-bar", p3a<2>}, Variant<float>{"p3 abl3 +no-aread", p3a<3>},
                Variant<float>{"p3 abl4 +no-bread", p3a<4>}},
               157.3);
    return 0;
  }
  if (which == "p3dw") {
    run<double>(S, rounds,
                {V(double, 128, 128, 16, 4, 4, 0), Variant<double>{"p3d w4", p3dw<2>}, Variant<double>{"p3d w8", p3dw<4>},
                 Variant<double>{"p3d w8 g0", p3dw<4, 0>}},
                78.6);
    return 0;
  }
  if (which == "p3dwabl") {
    run<double>(S, rounds,
                {V(double, 128, 128, 16, 4, 4, 0), Variant<double>{"p3d w8", p3dw<4>},
                 Variant<double>{"p3d w8 abl1", p3dw<4, 8, 1>}, Variant<double>{"p3d w8 abl3", p3dw<4, 8, 3>},
                 Variant<double>{"p3d w8 abl4", p3dw<4, 8, 4>}},
                78.6);
    return 0;
  }
  if (which == "p3dabl") {
    run<double>(S, rounds,
                {Variant<double>{"p3d", p3da<0>}, Variant<double>{"p3d abl1 no-ldst", p3da<1>},
                 Variant<double>{"p3d abl3 +no-aread", p3da<3>}, Variant<double>{"p3d abl4 +no-bread", p3da<4>}},
                78.6);
    return 0;
  }
  if (which == "p3d") {  // fp64 three-stage one-wave-per-SIMD kernels against the product
    run<double>(S, rounds,
                {V(double, 128, 128, 16, 4, 4, 0), Variant<double>{"p3d bk16 g8", p3d_16}},
                78.6);
    return 0;
  }
  if (which == "big2") {  // 128 x 128 wave tiles without the in-kernel flush (a K-chunked launch instead)
    run<float>(S, rounds,
               {VG(float, 256, 128, 16, 4, 2, 8, 512), V(float, 256, 256, 16, 2, 2, 8), V(float, 256, 256, 32, 2, 2, 8),
                V(float, 256, 256, 16, 2, 2, 4), V(float, 256, 256, 16, 2, 2, 16), V(float, 256, 256, 16, 2, 2, 0)},
               157.3);
    return 0;
  }
  if (which == "gfl") {  // one accumulator set, flushed into C every GFL K-tiles, against SEG and one chain
    run<float>(S, rounds,
               {V(float, 256, 128, 16, 4, 2, 8), VS(float, 256, 128, 16, 4, 2, 8, 16), VG(float, 256, 128, 16, 4, 2, 8, 128),
                VG(float, 256, 128, 16, 4, 2, 8, 256), VG(float, 256, 128, 16, 4, 2, 8, 512),
                VS(float, 256, 128, 32, 8, 2, 8, 8)},
               157.3);
    return 0;
  }
  if (which == "gfl2") {  // tile / grouping sweep of the GFL 512 form
    run<float>(S, rounds,
               {VG(float, 256, 128, 16, 4, 2, 8, 512), VG(float, 256, 128, 16, 4, 2, 4, 512),
                VG(float, 256, 128, 16, 4, 2, 16, 512), VG(float, 128, 256, 16, 2, 4, 8, 512),
                VG(float, 256, 256, 16, 4, 4, 8, 512), VG(float, 256, 128, 32, 4, 2, 8, 256),
                VG(float, 128, 128, 16, 2, 2, 8, 512), VG(float, 256, 128, 16, 4, 2, 8, 1024)},
               157.3);
    return 0;
  }
  if (which == "seg2") {  // two-level accumulation at <= 128 registers (32 x 64 / 64 x 32 wave tiles)
    run<float>(S, rounds,
               {V(float, 256, 128, 16, 4, 2, 8), VS(float, 256, 128, 16, 4, 2, 8, 16), VS(float, 128, 128, 16, 4, 2, 8, 16),
                VS(float, 128, 128, 16, 2, 4, 8, 16), VS(float, 256, 128, 16, 8, 2, 8, 16), VS(float, 256, 128, 32, 8, 2, 8, 8),
                VS(float, 128, 256, 16, 4, 4, 8, 16), VS(float, 256, 128, 16, 4, 4, 8, 16), VS(float, 128, 128, 32, 4, 2, 8, 8)},
               157.3);
    return 0;
  }
  if (which == "seg") {  // two-level accumulation (SEG K-tiles per fresh accumulator) against one chain
    run<float>(S, rounds,
               {V(float, 256, 128, 16, 4, 2, 8), VS(float, 256, 128, 16, 4, 2, 8, 16), VS(float, 256, 128, 16, 4, 2, 8, 32),
                VS(float, 256, 128, 16, 4, 2, 8, 64), VS(float, 256, 128, 32, 4, 2, 8, 16), VS(float, 128, 128, 16, 2, 2, 8, 16),
                VS(float, 256, 256, 16, 4, 4, 8, 16), VS(float, 128, 256, 16, 2, 4, 8, 16), VS(float, 256, 128, 16, 2, 4, 8, 16)},
               157.3);
    return 0;
  }
  if (which != "f64") {
    run<float>(S, rounds,
               {V(float, 128, 128, 16, 2, 2, 0), V(float, 128, 128, 16, 2, 2, 8), V(float, 128, 128, 32, 2, 2, 8),
                V(float, 256, 128, 16, 4, 2, 8), V(float, 128, 256, 16, 2, 4, 8), V(float, 256, 256, 16, 4, 4, 8),
                V(float, 128, 128, 32, 4, 4, 8), V(float, 256, 128, 32, 4, 2, 8), V(float, 256, 256, 32, 4, 4, 8),
                V(float, 256, 256, 16, 2, 4, 8), V(float, 256, 256, 32, 2, 4, 8), V(float, 256, 128, 16, 4, 2, 4),
                V(float, 256, 128, 16, 4, 2, 16), V(float, 256, 128, 16, 2, 2, 8),
                V(float, 256, 64, 16, 4, 1, 8), V(float, 256, 128, 16, 2, 4, 8), V(float, 256, 256, 16, 2, 8, 8),
                V(float, 128, 128, 16, 1, 4, 8)},
               157.3);
  }
  if (which != "f32") {
    run<double>(S, rounds,
                {V(double, 128, 128, 8, 2, 2, 0), V(double, 128, 128, 16, 4, 4, 8), V(double, 128, 128, 16, 4, 4, 0),
                 V(double, 128, 128, 16, 2, 2, 8), V(double, 256, 128, 16, 4, 4, 8), V(double, 128, 256, 16, 4, 4, 8),
                 V(double, 256, 256, 16, 4, 4, 8), V(double, 128, 128, 32, 4, 4, 8)},
                78.6);
  }
  return 0;
}
