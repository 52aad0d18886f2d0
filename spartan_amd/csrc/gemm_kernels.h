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

// fp32, a 256 x 256 block tile over 2 x WN waves -- WN = 2: one wave per
// SIMD, each 128 x 128 = 4 x 4 v_mfma_f32_32x32x2_f32 tiles (256 accumulator
// registers); WN = 4: two waves per SIMD, each 128 x 64 -- K-tiles of 16.
// Three LDS stages: tile t + 2 is staged during tile t's MFMAs (its global
// loads were issued during tile t - 1), and tile t + 1's A fragments and
// first B fragments are read into registers before the one barrier that ends
// tile t, so after the barrier the wave's next MFMA has its operands.
// Hazards (buffer b = t mod 3):
//   * tile t + 2 goes into buffer (t + 2) % 3 = (t - 1) % 3, last read in
//     tile t - 1 (B reads) and tile t - 2 (its A fragment prefetch): both
//     before the barrier that ended tile t - 1;
//   * tile t + 1 (buffer (t + 1) % 3) was written in tile t - 1 by every
//     wave: visible after the barrier that ended tile t - 1.
// Requires M % 256 == N % 256 == K % 16 == 0, lda % 4 == ldb % 4 == 0 and
// 16-byte aligned A, B (p3_ok).  FL > 0: the accumulators go into C every FL
// K-tiles (in-kernel chunks, see flush); else one chain spans K.
constexpr int P3_AST = 20;                            // A row stride (floats): k-contiguous, +4 pad
constexpr int P3_SA = 256 * P3_AST, P3_SB = 16 * 256;  // floats per stage
constexpr int P3_LDS = 3 * (P3_SA + P3_SB) * 4;       // bytes
template <int GM, int ABL = 0, int FL = 0, int BT = 0, int WN = 2, int SCH = 1, int GL = 0>
__global__ __launch_bounds__(128 * WN, 1) void gemm_f32_p3(i64 M, i64 N, i64 K, const float* __restrict__ A, i64 lda,
                                                         const float* __restrict__ B, i64 ldb, float* __restrict__ C,
                                                         i64 ldc, float alpha, float beta, int tiles_n, int ntiles) {
  typedef float V __attribute__((ext_vector_type(4)));
  constexpr int NT = 128 * WN, WTN = 256 / WN, TN = WTN / 32;
  constexpr int NPA = 1024 / NT, NPB = 1024 / NT, NP = NPA + NPB;  // 16-byte staging pieces per thread
  static_assert(WN == 2 || WN == 4, "2 x 2 or 2 x 4 waves");
  typedef float VB __attribute__((ext_vector_type(TN)));
  // GL = 1: tiles staged by global_load_lds (no staging registers, no LDS
  // write instructions); A rows then unpadded (16 floats) with the 16-byte
  // chunks XOR-swizzled by row ((row >> 2) & 3, on the global SOURCE address:
  // the DMA's LDS destination is lane-linear) so the fragment reads stay
  // conflict-free; NG pieces (1 KiB DMA instructions) per wave and tile
  constexpr int AST = GL ? 16 : P3_AST, SA = 256 * AST, SST = SA + P3_SB;
  constexpr int NG = 32 / (2 * WN), NGA = NG / 2;
  typedef __attribute__((address_space(3))) void* lds_ptr;
  extern __shared__ __attribute__((aligned(16))) float p3_lds[];
  int tm, tn;
  tile_of(blockIdx.x, ntiles, tiles_n, GM, tm, tn);
  const i64 row0 = (i64)tm * 256, col0 = (i64)tn * 256;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w / WN, wn = w % WN;
  const int li = lane & 31, kb = 8 * (lane >> 5);
  f32x16 acc[4][TN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x16){};
  // staging: A piece i = rows (t >> 2) + NT / 4 i, k quad t & 3; B piece i =
  // rows (t >> 6) + NT / 64 i, column quad t & 63
  V ra[NPA], rb[NPB];
  const float* ag = A + (row0 + (t >> 2)) * lda + 4 * (t & 3);
  const float* bg = B + (i64)(t >> 6) * ldb + col0 + 4 * (t & 63);
  auto abuf = [&](int s) __attribute__((always_inline)) { return p3_lds + s * SST; };
  auto gl_piece = [&](i64 k0, int sb, int q) __attribute__((always_inline)) {
    if (q < NGA) {
      const int rb = NGA * w + q, m = 16 * rb + (lane >> 2);
      const int c = (lane & 3) ^ ((lane >> 4) & 3);  // the source chunk of this lane's LDS slot
      __builtin_amdgcn_global_load_lds(A + (row0 + m) * lda + k0 + 4 * c, (lds_ptr)(abuf(sb) + 16 * 16 * rb), 16, 0,
                                       0);
    } else {
      const int r = (NG - NGA) * w + (q - NGA);
      __builtin_amdgcn_global_load_lds(B + (k0 + r) * ldb + col0 + 4 * lane, (lds_ptr)(abuf(sb) + SA + 256 * r), 16,
                                       0, 0);
    }
  };
  auto gl_tile = [&](i64 k0, int sb) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < NG; ++q) gl_piece(k0, sb, q);
  };
  auto load_piece = [&](i64 k0, int q) __attribute__((always_inline)) {
    if (q < NPA)
      ra[q] = *(const V*)(ag + (i64)(NT / 4) * q * lda + k0);
    else
      rb[q - NPA] = *(const V*)(bg + (k0 + (NT / 64) * (q - NPA)) * ldb);
  };
  auto store_piece = [&](int sb, int q) __attribute__((always_inline)) {
    if (q < NPA)
      *(V*)(abuf(sb) + ((t >> 2) + (NT / 4) * q) * AST + 4 * (t & 3)) = ra[q];
    else
      *(V*)(abuf(sb) + SA + ((t >> 6) + (NT / 64) * (q - NPA)) * 256 + 4 * (t & 63)) = rb[q - NPA];
  };
  auto load = [&](i64 k0) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < NP; ++q) load_piece(k0, q);
  };
  auto store = [&](int sb) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < NP; ++q) store_piece(sb, q);
  };
  // a lane's A values of a whole K-tile (k = kb .. kb + 7 of rows wm 128 + 32 i + li): 8 pieces
  auto read_a_piece = [&](int sb, float (&av)[4][8], int q) __attribute__((always_inline)) {
    const int i = q >> 1, hf = q & 1;
    const int ch = GL ? (((kb >> 2) + hf) ^ ((li >> 2) & 3)) : (kb >> 2) + hf;  // (swizzled) 16-byte chunk
    const V v = *(const V*)(abuf(sb) + (wm * 128 + li + 32 * i) * AST + 4 * ch);
#pragma unroll
    for (int e = 0; e < 4; ++e) av[i][4 * hf + e] = v[e];
  };
  auto read_a = [&](int sb, float (&av)[4][8]) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 8; ++q) read_a_piece(sb, av, q);
  };
  // BT = 0: MFMA tile j's lane li is output column wn WTN + 32 j + li (TN
  // b32 reads per step); BT = 1: column wn WTN + TN li + j, so a lane's TN
  // B values of a step are one ds_read_b128 (b64 for TN = 2)
  auto read_b = [&](int sb, int kk, float (&b)[TN]) __attribute__((always_inline)) {
    if constexpr (BT) {
      const VB v = *(const VB*)(abuf(sb) + SA + (kb + kk) * 256 + wn * WTN + TN * li);
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = v[j];
    } else {
      const float* p = abuf(sb) + SA + (kb + kk) * 256 + wn * WTN + li;
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = p[32 * j];
    }
  };
  auto ccol = [&](int j, int l) __attribute__((always_inline)) { return BT ? TN * l + j : 32 * j + l; };
  // K runs in chunks of FL K-tiles (FL > 0; one chunk otherwise), each with
  // its own pipeline fill; between chunks the accumulators go into C (see
  // flush below) -- there no pipeline state is live, so the flush needs no
  // registers the K loop holds (in the loop it spilled)
  const int nkt = (int)(K / 16);
  int kb0 = 0, nk = nkt;
  float avA[4][8], avB[4][8], bn[2][TN];
  // one K-tile: MFMAs from av (this tile's A fragments), B read two steps
  // ahead (a ring of three; steps 6 / 7 read the next tile's steps 0 / 1);
  // woven between each step's four MFMA groups: a piece of tile kt + 2's LDS
  // stage, the global load of the same piece of tile kt + 3 into the staging
  // register it just freed, and one ds_read_b128 of tile kt + 1's A
  // fragments -- one memory instruction between MFMA groups instead of
  // bursts (a burst held the wave's in-order issue, and with one wave per
  // SIMD the matrix pipe: tools/gemm_tune p3abl).  Sched barriers pin the
  // weave.  The memory instructions are unconditional (a branch around one
  // made hipcc wait vmcnt(0) at every store): past the last tile a stage
  // writes a buffer nobody reads again and the loads re-read the last tile.
  // (ABL: dev ablations, results wrong by design -- 1: no global loads or
  // LDS stores in the loop, 2: also no barrier, 3: also no next-tile A reads,
  // 4: also no per-step B reads; tools/gemm_tune.hip p3abl)
  constexpr int PSTEP = 8 / NP;  // k-steps per staging piece
  auto tile = [&](int kt, int s, float (&av)[4][8], float (&avn)[4][8]) __attribute__((always_inline)) {
    const int s1 = s == 2 ? 0 : s + 1, s2 = s1 == 2 ? 0 : s1 + 1;
    constexpr bool st = ABL < 1 && !GL, ld = ABL < 1 && !GL, ra_ = ABL < 3, gl = ABL < 1 && GL;
    const i64 k3 = (i64)(kb0 + (kt + 3 < nk ? kt + 3 : nk - 1)) * 16;
    const i64 k2 = (i64)(kb0 + (kt + 2 < nk ? kt + 2 : nk - 1)) * 16;
    float b[3][TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      b[0][j] = bn[0][j];
      b[1][j] = bn[1][j];
    }
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      if (ABL < 4 && kk + 2 < 8) read_b(s, kk + 2, b[(kk + 2) % 3]);
      if (ABL >= 4 && kk + 2 < 8)
#pragma unroll
        for (int j = 0; j < TN; ++j) b[(kk + 2) % 3][j] = bn[0][j];
      if (kk >= 6) read_b(s1, kk - 6, bn[kk - 6]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (SCH) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i][kk], b[kk % 3][j], acc[i][j], 0, 0, 0);
        if constexpr (SCH) __builtin_amdgcn_sched_barrier(0);
        if (kk % PSTEP == 0) {
          if (i == 0 && st) store_piece(s2, kk / PSTEP);
          if (i == 1 && ld) load_piece(k3, kk / PSTEP);
        }
        // GL: tile kt + 2's DMA pieces early in the tile (the barrier that
        // ends it waits for them)
        if (gl && i == 1 && kk < NG) gl_piece(k2, s2, kk);
        if (i == 2 && ra_) read_a_piece(s1, avn, kk);
      }
    }
    if (ABL < 2) __syncthreads();
  };
  // FL > 0: every FL K-tiles the accumulators go into C and restart from
  // zero (chains of 8 FL MFMA steps; the generic kernel's GFL): the first
  // flush stores (beta 0) or adds, later ones add by no-return fp32 atomics
  // (one wave owns each element, so its adds land in program order:
  // deterministic).  The caller passes beta 0 or 1 when FL > 0.
  const bool use_beta = beta != 0.f;
  bool flushed = false;
  auto flush = [&](bool again) __attribute__((always_inline)) {
    int fl = lane;
    i64 ldf = ldc;
    // the addresses are invariant across chunks: opaque operands keep the
    // compiler from hoisting all of them (two registers each) out of the loop
    asm volatile("" : "+v"(fl));
    asm volatile("" : "+s"(ldf));
    float* const cb = C + (row0 + wm * 128 + Mfma<float>::crow(fl, 0)) * ldf + col0 + wn * WTN + ccol(0, fl & 31);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float* const pc = cb + (i64)(i * 32 + Mfma<float>::crow(0, r)) * ldf + ccol(j, 0);
          const float v = alpha * acc[i][j][r];
          if (again || use_beta)
            unsafeAtomicAdd(pc, v);
          else
            *pc = v;
        }
        acc[i][j] = (f32x16){};
        __builtin_amdgcn_sched_barrier(0);  // one accumulator tile's 16 values in VGPRs at a time
      }
  };
  constexpr int CH = FL > 0 ? FL : (1 << 30);
  for (kb0 = 0; kb0 < nkt; kb0 += CH) {
    nk = nkt - kb0 < CH ? nkt - kb0 : CH;
    if constexpr (GL) {
      gl_tile((i64)kb0 * 16, 0);
      gl_tile((i64)(kb0 + (nk > 1 ? 1 : 0)) * 16, 1);
      __syncthreads();
    } else {
      load((i64)kb0 * 16);
      store(0);
      if (nk > 1) {
        load((i64)(kb0 + 1) * 16);
        store(1);
      }
      __syncthreads();
    }
    read_a(0, avA);
    read_b(0, 0, bn[0]);
    read_b(0, 1, bn[1]);
    if constexpr (!GL) load((i64)(kb0 + (nk > 2 ? 2 : nk - 1)) * 16);
    int s = 0;
    int kt = 0;
    for (; kt + 1 < nk; kt += 2) {
      tile(kt, s, avA, avB);
      s = s == 2 ? 0 : s + 1;
      tile(kt + 1, s, avB, avA);
      s = s == 2 ? 0 : s + 1;
    }
    if (kt < nk) tile(kt, s, avA, avB);
    if constexpr (FL > 0) {
      if (kb0 + CH < nkt) {  // block-uniform
        flush(flushed);
        flushed = true;
      }
    }
  }
  if (FL > 0 && flushed) {
    flush(true);
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const i64 gr = row0 + wm * 128 + i * 32 + Mfma<float>::crow(lane, r);
        const i64 gc = col0 + wn * WTN + ccol(j, li);
        float v = alpha * acc[i][j][r];
        if (use_beta) v += beta * C[gr * ldc + gc];
        C[gr * ldc + gc] = v;
      }
}

// fp64, the same three-stage one-wave-per-SIMD structure: a 128 x 128 block
// tile, 4 waves (2 x 2), each 64 x 64 = 4 x 4 v_mfma_f64_16x16x4_f64 tiles,
// K-tiles of BK.  The K-tile is split between the four lane groups g = l >> 4
// (step kk takes k = g BK / 4 + kk from group g, for A and B alike), so a
// lane's A values for the whole K-tile are BK / 4 consecutive doubles of its
// row (ds_read_b128) and a B value is one ds_read_b64.  Strides: A rows
// BK + 2 (BK = 16) or BK + 2 doubles (the b128 reads of 16 rows spread
// over the banks), B rows 128 + 4 doubles (the four lane groups' rows two
// by two on different bank halves).
template <int BK>
struct P3d {
  static constexpr int AST = BK + 2, BST = 132, SA = 128 * AST, SB = BK * BST, LDS = 3 * (SA + SB) * 8, KQ = BK / 4;
};
template <int GM, int BK, int ABL = 0, int WN = 2>
__global__ __launch_bounds__(128 * WN, 1) void gemm_f64_p3(i64 M, i64 N, i64 K, const double* __restrict__ A,
                                                         i64 lda, const double* __restrict__ B, i64 ldb,
                                                         double* __restrict__ C, i64 ldc, double alpha, double beta,
                                                         int tiles_n, int ntiles) {
  typedef P3d<BK> P;
  typedef double V __attribute__((ext_vector_type(2)));
  // WN = 2: 4 waves of 64 x 64 (one per SIMD); WN = 4: 8 waves of 64 x 32
  // (two per SIMD: 128 accumulator dwords fewer per wave, so hipcc keeps them
  // in VGPRs instead of copying 256 of them between AGPRs and VGPRs every
  // two K-tiles, as it did for the one-wave form)
  constexpr int NT = 128 * WN, WTN = 128 / WN, TN = WTN / 16, KQ = P::KQ;
  constexpr int APR = BK / 2, NPA = 128 * APR / NT, NPB = BK * 64 / NT, NP = NPA + NPB;
  static_assert(BK == 16 && (WN == 2 || WN == 4), "BK 16; 2 x 2 or 2 x 4 waves");
  extern __shared__ __attribute__((aligned(16))) double p3d_lds[];
  int tm, tn;
  tile_of(blockIdx.x, ntiles, tiles_n, GM, tm, tn);
  const i64 row0 = (i64)tm * 128, col0 = (i64)tn * 128;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w / WN, wn = w % WN;
  const int li = lane & 15, g = lane >> 4, kb = KQ * g;
  f64x4 acc[4][TN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f64x4){0, 0, 0, 0};
  V ra[NPA], rb[NPB];
  auto abuf = [&](int s) __attribute__((always_inline)) { return p3d_lds + s * (P::SA + P::SB); };
  // 16-byte staging pieces: A 128 rows x APR, B BK rows x 64
  auto load_piece = [&](i64 k0, int q) __attribute__((always_inline)) {
    if (q < NPA) {
      const int idx = t + NT * q;
      ra[q] = *(const V*)(A + (row0 + idx / APR) * lda + k0 + 2 * (idx % APR));
    } else {
      const int idx = t + NT * (q - NPA);
      rb[q - NPA] = *(const V*)(B + (k0 + (idx >> 6)) * ldb + col0 + 2 * (idx & 63));
    }
  };
  auto store_piece = [&](int sb, int q) __attribute__((always_inline)) {
    if (q < NPA) {
      const int idx = t + NT * q;
      *(V*)(abuf(sb) + (idx / APR) * P::AST + 2 * (idx % APR)) = ra[q];
    } else {
      const int idx = t + NT * (q - NPA);
      *(V*)(abuf(sb) + P::SA + (idx >> 6) * P::BST + 2 * (idx & 63)) = rb[q - NPA];
    }
  };
  auto read_a_piece = [&](int sb, double (&av)[4][KQ], int q) __attribute__((always_inline)) {
    const int i = q >> 1, hf = q & 1;
    const V v = *(const V*)(abuf(sb) + (wm * 64 + li) * P::AST + kb + 16 * i * P::AST + 2 * hf);
    av[i][2 * hf] = v[0];
    av[i][2 * hf + 1] = v[1];
  };
  auto read_b = [&](int sb, int kk, double (&b)[TN]) __attribute__((always_inline)) {
    const double* p = abuf(sb) + P::SA + (kb + kk) * P::BST + wn * WTN + li;
#pragma unroll
    for (int j = 0; j < TN; ++j) b[j] = p[16 * j];
  };
  const int nk = (int)(K / BK);
  double avA[4][KQ], avB[4][KQ], bn[TN];
#pragma unroll
  for (int q = 0; q < NP; ++q) load_piece(0, q);
#pragma unroll
  for (int q = 0; q < NP; ++q) store_piece(0, q);
  if (nk > 1) {
#pragma unroll
    for (int q = 0; q < NP; ++q) load_piece(BK, q);
#pragma unroll
    for (int q = 0; q < NP; ++q) store_piece(1, q);
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 8; ++q) read_a_piece(0, avA, q);
  read_b(0, 0, bn);
#pragma unroll
  for (int q = 0; q < NP; ++q) load_piece((i64)(nk > 2 ? 2 : nk - 1) * BK, q);
  // the fp32 kernel's weave (see there): per k-step, between its four MFMA
  // groups, NP / 4 pieces of tile kt + 2's stage, the loads of the same
  // pieces of tile kt + 3 and two of tile kt + 1's A fragment reads
  constexpr int PPS = NP / KQ;  // staging pieces per k-step: 2 or 1
  auto tile = [&](int kt, int s, double (&av)[4][KQ], double (&avn)[4][KQ]) __attribute__((always_inline)) {
    const int s1 = s == 2 ? 0 : s + 1, s2 = s1 == 2 ? 0 : s1 + 1;
    const i64 k3 = (i64)(kt + 3 < nk ? kt + 3 : nk - 1) * BK;
    double b[2][TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) b[0][j] = bn[j];
#pragma unroll
    for (int kk = 0; kk < KQ; ++kk) {
      if (ABL < 4 && kk + 1 < KQ) read_b(s, kk + 1, b[(kk + 1) & 1]);
      if (ABL >= 4 && kk + 1 < KQ)
#pragma unroll
        for (int j = 0; j < TN; ++j) b[(kk + 1) & 1][j] = bn[j];
      if (kk == KQ - 1) read_b(s1, 0, bn);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[i][kk], b[kk & 1][j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        // (ABL: dev ablations as in the fp32 kernel: 1 no staging, 3 also no
        // next-tile A reads, 4 also no per-step B reads)
        const int qs = PPS * kk + (i >> 1);
        if (ABL < 1 && (i & 1) == 0 && (i >> 1) < PPS) store_piece(s2, qs);
        if ((i & 1) == 1) {
          if (ABL < 1 && (i >> 1) < PPS) load_piece(k3, qs);
          if (ABL < 3) read_a_piece(s1, avn, 2 * kk + (i >> 1));
        }
      }
    }
    __syncthreads();
  };
  int s = 0;
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    tile(kt, s, avA, avB);
    s = s == 2 ? 0 : s + 1;
    tile(kt + 1, s, avB, avA);
    s = s == 2 ? 0 : s + 1;
  }
  if (kt < nk) tile(kt, s, avA, avB);
  const bool use_beta = beta != 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const i64 gr = row0 + wm * 64 + i * 16 + Mfma<double>::crow(lane, r);
        const i64 gc = col0 + wn * WTN + j * 16 + li;
        double v = alpha * acc[i][j][r];
        if (use_beta) v += beta * C[gr * ldc + gc];
        C[gr * ldc + gc] = v;
      }
}

template <int BK>
__host__ inline bool p3d_ok(i64 M, i64 N, i64 K, const void* A, i64 lda, const void* B, i64 ldb) {
  return M % 128 == 0 && N % 128 == 0 && K % BK == 0 && K > 0 && lda % 2 == 0 && ldb % 2 == 0 &&
         (uintptr_t)A % 16 == 0 && (uintptr_t)B % 16 == 0;
}

template <int GM, int BK, int ABL = 0, int WN = 2>
__host__ inline hipError_t p3d_launch(i64 M, i64 N, i64 K, const double* A, i64 lda, const double* B, i64 ldb,
                                      double* C, i64 ldc, double alpha, double beta, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)gemm_f64_p3<GM, BK, ABL, WN>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       P3d<BK>::LDS);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const i64 tn = N / 128, nt = (M / 128) * tn;
  gemm_f64_p3<GM, BK, ABL, WN><<<(unsigned)nt, 128 * WN, P3d<BK>::LDS, s>>>(M, N, K, A, lda, B, ldb, C, ldc, alpha, beta, (int)tn,
                                                             (int)nt);
  return hipGetLastError();
}

__host__ inline bool p3_ok(i64 M, i64 N, i64 K, const void* A, i64 lda, const void* B, i64 ldb) {
  return M % 256 == 0 && N % 256 == 0 && K % 16 == 0 && K > 0 && lda % 4 == 0 && ldb % 4 == 0 &&
         (uintptr_t)A % 16 == 0 && (uintptr_t)B % 16 == 0;
}

template <int GM, int ABL = 0, int FL = 0, int BT = 0, int WN = 2, int SCH = 1, int GL = 0>
__host__ inline hipError_t p3_launch(i64 M, i64 N, i64 K, const float* A, i64 lda, const float* B, i64 ldb,
                                     float* C, i64 ldc, float alpha, float beta, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)gemm_f32_p3<GM, ABL, FL, BT, WN, SCH, GL>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, P3_LDS);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const i64 tn = N / 256, nt = (M / 256) * tn;
  gemm_f32_p3<GM, ABL, FL, BT, WN, SCH, GL><<<(unsigned)nt, 128 * WN, P3_LDS, s>>>(M, N, K, A, lda, B, ldb, C, ldc, alpha, beta, (int)tn, (int)nt);
  return hipGetLastError();
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
