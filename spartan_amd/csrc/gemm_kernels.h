// MFMA GEMM kernels for gfx950, shared by libspx.so (spx.hip) and the
// tuning harness (tools/gemm_tune.hip) so the tuner times the product code.
//
// C[M,N] = alpha * A[M,K] @ B[K,N] + beta * C, row-major, leading dims
// lda/ldb/ldc.  Block tile BM x BN, K-tile BK, WM x WN waves; each wave owns a
// (BM/WM) x (BN/WN) sub-tile of MFMA accumulators:
//   float : v_mfma_f32_32x32x2_f32  (A[i=l&31][k=l>>5], B[k=l>>5][j=l&31];
//           C/D row = (r&3) + 8*(r>>2) + 4*(l>>5), col = l&31)
//   double: v_mfma_f64_16x16x4_f64  (A[i=l&15][k=l>>4], B[k=l>>4][j=l&15];
//           C/D row = (l>>4) + 4*r, col = l&15)
// A is staged transposed in LDS (As[k][m]) so each operand read is a run of
// consecutive dwords per lane group; B row-major (Bs[k][n]).  Global loads are
// 16 B per lane into registers, issued for K-tile t+1 before the MFMAs of
// tile t (two LDS buffers, one barrier per K-tile).  The block -> tile map is
// XCD-aware (blocks b and b+8 share an XCD: give each XCD a contiguous range)
// and optionally grouped (GM row panels swept column-major) so that the tiles
// resident at once share A and B panels in L2.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace spx_mfma {

typedef int64_t i64;
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

template <typename T>
struct Mfma;

template <>
struct Mfma<float> {
  static constexpr int TILE = 32, KS = 2, NREG = 16;
  typedef f32x16 acc_t;
  typedef float vec_t __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ acc_t zero() { return (acc_t){}; }
  static __device__ __forceinline__ acc_t mma(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ int opi(int l) { return l & 31; }
  static __device__ __forceinline__ int opk(int l) { return l >> 5; }
  static __device__ __forceinline__ int crow(int l, int r) { return (r & 3) + 8 * (r >> 2) + 4 * (l >> 5); }
  static __device__ __forceinline__ int ccol(int l) { return l & 31; }
};

template <>
struct Mfma<double> {
  static constexpr int TILE = 16, KS = 4, NREG = 4;
  typedef f64x4 acc_t;
  typedef double vec_t __attribute__((ext_vector_type(2)));
  static __device__ __forceinline__ acc_t zero() { return (acc_t){0, 0, 0, 0}; }
  static __device__ __forceinline__ acc_t mma(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ int opi(int l) { return l & 15; }
  static __device__ __forceinline__ int opk(int l) { return l >> 4; }
  static __device__ __forceinline__ int crow(int l, int r) { return (l >> 4) + 4 * r; }
  static __device__ __forceinline__ int ccol(int l) { return l & 15; }
};

// tile index for block id: XCD-contiguous ranges, then optional grouping
__device__ __forceinline__ void tile_of(int bid, int ntiles, int tiles_n, int GM, int& tm, int& tn) {
  int q = ntiles / 8, rr = ntiles % 8, xcd = bid % 8;
  bid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
  if (GM > 0) {
    int tiles_m = ntiles / tiles_n;
    int per_group = GM * tiles_n;
    int g = bid / per_group, first_m = g * GM;
    int gm = (tiles_m - first_m) < GM ? (tiles_m - first_m) : GM;
    int l = bid - g * per_group;
    tm = first_m + l % gm;
    tn = l / gm;
  } else {
    tm = bid / tiles_n;
    tn = bid - tm * tiles_n;
  }
}

// SEG > 0: two-level accumulation -- the MFMA accumulators restart from zero
// every SEG K-tiles and are added into running sums, so an fp32 element is a
// chain of SEG * BK / 2 MFMA steps plus K / (SEG * BK) additions instead of
// one chain of K / 2 steps (K = 32768: 128 + 128 roundings instead of 16384;
// the relative error's spread drops from ~4e-6 to ~6e-7, well inside the fp32
// tolerance of 1e-5 at every element, where one long chain exceeded it in a
// few elements per row).
//
// GFL > 0: the same bound without the register cost -- every GFL K-tiles the
// wave adds its accumulators into C in global memory (the first flush
// applies beta) and restarts them from zero, so an element is a chain of
// GFL * BK / 2 MFMA steps plus K / (GFL * BK) fp32 additions in memory; the
// kernel keeps one accumulator set (and the occupancy of the one-chain
// form), at the cost of K / (GFL BK) read-modify-writes of C.
template <typename T, int BM, int BN, int BK, int WM, int WN, int GM, bool ALIGNED, int SEG = 0, int GFL = 0>
__global__ __launch_bounds__(64 * WM* WN) void gemm(i64 M, i64 N, i64 K, const T* __restrict__ A, i64 lda,
                                                     const T* __restrict__ B, i64 ldb, T* __restrict__ C,
                                                     i64 ldc, T alpha, T beta, int tiles_n, int ntiles) {
  typedef Mfma<T> F;
  typedef typename F::vec_t V;
  constexpr int NT = 64 * WM * WN;
  constexpr int VE = 16 / sizeof(T);  // elements per 16-byte load
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / F::TILE, TN = WTN / F::TILE;
  // 16-byte loads per thread and K-tile (a block of more threads than a
  // tile has 16-byte pieces leaves the upper threads idle for that operand)
  constexpr int NA = BM * BK / VE, NB = BK * BN / VE;
  constexpr int LA = (NA + NT - 1) / NT, LB = (NB + NT - 1) / NT;
  constexpr int PADA = 16 / sizeof(T) / 2 > 0 ? 16 / sizeof(T) / 2 : 1;
  static_assert((NA % NT == 0 || NA < NT) && (NB % NT == 0 || NB < NT), "bad tiling");
  static_assert(TM >= 1 && TN >= 1 && BK % F::KS == 0, "bad wave tiling");
  // AK (fp32): A kept k-contiguous in LDS ([m][k], rows padded to BK + 4)
  // and the tile's K split between the two lane halves: MFMA step kk takes
  // k = kk from lanes 0-31 and k = BK/2 + kk from lanes 32-63 (B read the
  // same way), so a lane's BK/2 A values are two ds_read_b128 per K-tile
  // and the staging store is one ds_write_b128 -- instead of BK/2 ds_read_b32
  // and a 4-way transposing scalar store.
  constexpr bool AK = sizeof(T) == 4 && F::KS == 2 && BK % 8 == 0;
  __shared__ __attribute__((aligned(16))) T As[AK ? 1 : 2][AK ? 1 : BK][AK ? 1 : BM + PADA];
  __shared__ __attribute__((aligned(16))) T Ak[AK ? 2 : 1][AK ? BM : 1][AK ? BK + 4 : 1];
  __shared__ __attribute__((aligned(16))) T Bs[2][BK][BN];
  int tm, tn;
  tile_of(blockIdx.x, ntiles, tiles_n, GM, tm, tn);
  const i64 row0 = (i64)tm * BM, col0 = (i64)tn * BN;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w / WN, wn = w % WN;
  typename F::acc_t acc[TM][TN], run[SEG > 0 ? TM : 1][SEG > 0 ? TN : 1];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = F::zero();
  if constexpr (SEG > 0) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) run[i][j] = F::zero();
  }
  V ra[LA], rb[LB];
  auto load = [&](i64 k0) {
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = t + i * NT;
      if (NA < NT && idx >= NA) break;
      const int r = idx / (BK / VE), kq = idx % (BK / VE);
      const i64 gr = row0 + r, gk = k0 + kq * VE;
      if (ALIGNED) {
        ra[i] = *(const V*)(A + gr * lda + gk);
      } else {
#pragma unroll
        for (int j = 0; j < VE; ++j) ra[i][j] = (gr < M && gk + j < K) ? A[gr * lda + gk + j] : (T)0;
      }
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int idx = t + i * NT;
      if (NB < NT && idx >= NB) break;
      const int kr = idx / (BN / VE), cq = idx % (BN / VE);
      const i64 bk = k0 + kr, bc = col0 + cq * VE;
      if (ALIGNED) {
        rb[i] = *(const V*)(B + bk * ldb + bc);
      } else {
#pragma unroll
        for (int j = 0; j < VE; ++j) rb[i][j] = (bk < K && bc + j < N) ? B[bk * ldb + bc + j] : (T)0;
      }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = t + i * NT;
      if (NA < NT && idx >= NA) break;
      const int r = idx / (BK / VE), kq = idx % (BK / VE);
      if constexpr (AK) {
        *(V*)(&Ak[buf][r][kq * VE]) = ra[i];
      } else {
#pragma unroll
        for (int j = 0; j < VE; ++j) As[buf][kq * VE + j][r] = ra[i][j];
      }
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int idx = t + i * NT;
      if (NB < NT && idx >= NB) break;
      const int kr = idx / (BN / VE), cq = idx % (BN / VE);
      *(V*)(&Bs[buf][kr][cq * VE]) = rb[i];
    }
  };
  // acc (times alpha) into C.  With GFL > 0 the kernel runs with beta 0 or 1
  // (spx_gemm scales C first for other betas): the first write of an element
  // is a plain store when beta is 0, every other one a no-return fp32 atomic
  // add -- C is never read back into registers (64 loads in flight would
  // double the kernel's registers), and one wave owns each element, so its
  // adds land in program order: deterministic.  Without GFL: the one
  // epilogue, alpha * acc + beta * C.
  const bool use_beta = beta != (T)0;
  auto flush_c = [&](bool again) {
    int fl = lane;
    asm volatile("" : "+v"(fl));  // C's addresses are loop-invariant: do not hoist them out of the K loop
    // this lane's element (i, j, r) sits at cb + (i TILE + crow(0, r)) ldc + j TILE
    T* const cb = C + (row0 + wm * WTM + F::crow(fl, 0)) * ldc + col0 + wn * WTN + F::ccol(fl);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < F::NREG; ++r) {
          const i64 gr = row0 + wm * WTM + i * F::TILE + F::crow(fl, r);
          const i64 gc = col0 + wn * WTN + j * F::TILE + F::ccol(fl);
          if (ALIGNED || (gr < M && gc < N)) {
            T v = alpha * acc[i][j][r];
            if constexpr (GFL > 0) {
              T* const pc = cb + (i64)(i * F::TILE + F::crow(0, r) - F::crow(0, 0)) * ldc + j * F::TILE;
              if (again || use_beta)
                unsafeAtomicAdd(pc, v);
              else
                *pc = v;
            } else {
              if (use_beta) v += beta * C[gr * ldc + gc];
              C[gr * ldc + gc] = v;
            }
          }
        }
  };
  bool flushed = false;
  const int nk = (int)((K + BK - 1) / BK);
  load(0);
  store(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load((i64)(kt + 1) * BK);
    if constexpr (AK) {
      constexpr int KH = BK / 2;
      const int kb = KH * F::opk(lane);
      T av[TM][KH];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const T* ap = &Ak[cur][wm * WTM + i * F::TILE + F::opi(lane)][kb];
#pragma unroll
        for (int q = 0; q < KH; q += VE) {
          const V v = *(const V*)(ap + q);
#pragma unroll
          for (int e = 0; e < VE; ++e) av[i][q + e] = v[e];
        }
      }
#pragma unroll
      for (int kk = 0; kk < KH; ++kk) {
        T b[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) b[j] = Bs[cur][kb + kk][wn * WTN + j * F::TILE + F::opi(lane)];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = F::mma(av[i][kk], b[j], acc[i][j]);
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < BK / F::KS; ++kk) {
        const int k = kk * F::KS + F::opk(lane);
        T a[TM], b[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) a[i] = As[cur][k][wm * WTM + i * F::TILE + F::opi(lane)];
#pragma unroll
        for (int j = 0; j < TN; ++j) b[j] = Bs[cur][k][wn * WTN + j * F::TILE + F::opi(lane)];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = F::mma(a[i], b[j], acc[i][j]);
      }
    }
    if constexpr (GFL > 0) {
      if ((kt + 1) % GFL == 0 && kt + 1 < nk) {  // block-uniform: flush into C
        flush_c(flushed);
        flushed = true;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = F::zero();
      }
    }
    if constexpr (SEG > 0) {
      if ((kt + 1) % SEG == 0) {  // block-uniform
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            run[i][j] += acc[i][j];
            acc[i][j] = F::zero();
          }
      }
    }
    if (kt + 1 < nk) store(cur ^ 1);
    __syncthreads();
  }
  if constexpr (SEG > 0) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] += run[i][j];
  }
  flush_c(flushed);
}

template <typename T, int BM, int BN, int BK, int WM, int WN, int GM, int SEG = 0, int GFL = 0>
struct Config {
  static constexpr int bm = BM, bn = BN, bk = BK, threads = 64 * WM * WN;
  static hipError_t launch(i64 M, i64 N, i64 K, const T* A, i64 lda, const T* B, i64 ldb, T* C, i64 ldc,
                           T alpha, T beta, bool aligned, hipStream_t s) {
    i64 tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
    int nt = (int)(tm * tn);
    if (aligned)
      gemm<T, BM, BN, BK, WM, WN, GM, true, SEG, GFL><<<nt, threads, 0, s>>>(M, N, K, A, lda, B, ldb, C, ldc, alpha,
                                                                        beta, (int)tn, nt);
    else
      gemm<T, BM, BN, BK, WM, WN, GM, false, SEG, GFL><<<nt, threads, 0, s>>>(M, N, K, A, lda, B, ldb, C, ldc, alpha,
                                                                         beta, (int)tn, nt);
    return hipGetLastError();
  }
  static bool is_aligned(i64 M, i64 N, i64 K, const void* A, i64 lda, const void* B, i64 ldb) {
    constexpr int VE = 16 / sizeof(T);
    return M % BM == 0 && N % BN == 0 && K % BK == 0 && lda % VE == 0 && ldb % VE == 0 &&
           (uintptr_t)A % 16 == 0 && (uintptr_t)B % 16 == 0;
  }
};

}  // namespace spx_mfma
