// libspx.so -- MI355X (gfx950) tile-execution kernels behind include/spx.h.
//
// This file holds the ahead-of-time kernels (fills, reduction finalize, tile
// merge, region copy, MFMA GEMM, arg-reduction combine) and the module/launch
// plumbing for the fused map / map+reduce kernels that spartan_amd/codegen.py
// generates per expression.  Reference call sites replaced are cited per
// entry point in include/spx.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>
#include <utility>

#include "../../include/spx.h"

typedef int64_t i64;
typedef uint64_t u64;

// ------------------------------------------------------------------ errors
static thread_local std::string g_err;

static int set_err(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                         \
  do {                                                                        \
    hipError_t e_ = (expr);                                                   \
    if (e_ != hipSuccess)                                                     \
      return set_err(SPX_EHIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

#define LAUNCH_CHECK(name)                                                    \
  do {                                                                        \
    hipError_t e_ = hipGetLastError();                                        \
    if (e_ != hipSuccess)                                                     \
      return set_err(SPX_EHIP, "%s launch failed: %s", name,                  \
                     hipGetErrorString(e_));                                  \
  } while (0)

extern "C" int spx_abi_version(void) { return SPX_ABI_VERSION; }
extern "C" const char* spx_last_error(void) { return g_err.c_str(); }
// error text from the host-only translation units (comm.cpp)
extern "C" int spx_comm_set_error(const char* msg) {
  g_err = msg ? msg : "";
  return 0;
}

static inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

static bool valid_dtype(int d) { return d >= SPX_BOOL && d <= SPX_F64; }

// ----------------------------------------------------- dtype-generic access
// Used by the non-hot-path kernels (merge / copy / finalize) where a uniform
// per-element switch is cheaper than instantiating every dtype pair.
__device__ __forceinline__ double ld_f(const void* p, int dt, i64 i) {
  switch (dt) {
    case SPX_BOOL: return (double)((const uint8_t*)p)[i];
    case SPX_I32: return (double)((const int32_t*)p)[i];
    case SPX_I64: return (double)((const int64_t*)p)[i];
    case SPX_F32: return (double)((const float*)p)[i];
    default: return ((const double*)p)[i];
  }
}
__device__ __forceinline__ i64 ld_i(const void* p, int dt, i64 i) {
  switch (dt) {
    case SPX_BOOL: return (i64)((const uint8_t*)p)[i];
    case SPX_I32: return (i64)((const int32_t*)p)[i];
    case SPX_I64: return ((const int64_t*)p)[i];
    case SPX_F32: return (i64)((const float*)p)[i];
    default: return (i64)((const double*)p)[i];
  }
}
__device__ __forceinline__ bool is_float_dt(int dt) { return dt == SPX_F32 || dt == SPX_F64; }

__device__ __forceinline__ void st_f(void* p, int dt, i64 i, double v) {
  switch (dt) {
    case SPX_BOOL: ((uint8_t*)p)[i] = (v != 0.0); break;
    case SPX_I32: ((int32_t*)p)[i] = (int32_t)(i64)v; break;
    case SPX_I64: ((int64_t*)p)[i] = (i64)v; break;
    case SPX_F32: ((float*)p)[i] = (float)v; break;
    default: ((double*)p)[i] = v; break;
  }
}
__device__ __forceinline__ void st_i(void* p, int dt, i64 i, i64 v) {
  switch (dt) {
    case SPX_BOOL: ((uint8_t*)p)[i] = (v != 0); break;
    case SPX_I32: ((int32_t*)p)[i] = (int32_t)v; break;  // wraps like astype
    case SPX_I64: ((int64_t*)p)[i] = v; break;
    case SPX_F32: ((float*)p)[i] = (float)v; break;
    default: ((double*)p)[i] = (double)v; break;
  }
}

struct Geom {  // up to 8-d row-major geometry passed by value
  int ndim;
  i64 a[8];
  i64 b[8];
  i64 c[8];
  i64 d[8];
};

static int grid_for(i64 n, int per_thread = 1) {
  i64 g = (n + 256LL * per_thread - 1) / (256LL * per_thread);
  if (g < 1) g = 1;
  if (g > 65536) g = 65536;
  return (int)g;
}

// Streamed once-read loads carry the non-temporal hint (global_load ... nt;
// measured +5-9 % on the generated streaming kernels).
template <typename T>
__device__ __forceinline__ T ld_stream(const T* p) {
  return __builtin_nontemporal_load(p);
}

// =================================================================== fills
__device__ __forceinline__ u64 mix64(u64 z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
// counter-based splitmix64 stream: value at global flat index g
__device__ __forceinline__ u64 rng_at(u64 seed, u64 g) {
  return mix64(seed * 0xD1B54A32D192ED03ULL + (g + 1ULL) * 0x9E3779B97F4A7C15ULL);
}

// standard normal at global flat index g: Box-Muller over the two counter
// streams 2g (u1 in (0,1]) and 2g+1 (u2 in [0,1)), computed in fp64
__device__ __forceinline__ double normal_at(u64 seed, i64 g) {
  double u1 = (double)((rng_at(seed, 2ULL * (u64)g) >> 11) + 1ULL) * 1.1102230246251565e-16;
  double u2 = (double)(rng_at(seed, 2ULL * (u64)g + 1ULL) >> 11) * 1.1102230246251565e-16;
  double r = sqrt(-2.0 * log(u1));
  return r * cos(6.283185307179586 * u2);
}

template <typename T>
__device__ __forceinline__ T fill_value(int kind, int dt, double a, double b, u64 seed, i64 g);

template <>
__device__ __forceinline__ float fill_value<float>(int kind, int, double a, double b, u64 seed, i64 g) {
  if (kind == SPX_FILL_CONST) return (float)a;
  if (kind == SPX_FILL_ARANGE) return (float)(a + b * (double)g);
  if (kind == SPX_FILL_NORMAL) return (float)(a + b * normal_at(seed, g));
  float u = (float)(rng_at(seed, (u64)g) >> 40) * 5.9604644775390625e-08f;  // 2^-24
  float lo = (float)a, span = (float)(b - a);
  float t = span * u;  // separate rounding steps (fp-contract off) -- oracle does the same
  return lo + t;
}
template <>
__device__ __forceinline__ double fill_value<double>(int kind, int, double a, double b, u64 seed, i64 g) {
  if (kind == SPX_FILL_CONST) return a;
  if (kind == SPX_FILL_ARANGE) return a + b * (double)g;
  if (kind == SPX_FILL_NORMAL) return a + b * normal_at(seed, g);
  double u = (double)(rng_at(seed, (u64)g) >> 11) * 1.1102230246251565e-16;  // 2^-53
  double t = (b - a) * u;
  return a + t;
}
__device__ __forceinline__ i64 sat_i64(double a) {  // saturating double -> int64
  if (a >= 9.2233720368547758e18) return 0x7fffffffffffffffLL;
  if (a <= -9.2233720368547758e18) return (i64)(-0x7fffffffffffffffLL - 1);
  return (i64)a;
}
template <typename T>
__device__ __forceinline__ T fill_value_int(int kind, double a, double b, u64 seed, i64 g) {
  if (kind == SPX_FILL_CONST) return (T)sat_i64(a);
  if (kind == SPX_FILL_ARANGE) return (T)((i64)a + (i64)b * g);
  if (kind == SPX_FILL_NORMAL) return (T)(i64)floor(a + b * normal_at(seed, g));
  double u = (double)(rng_at(seed, (u64)g) >> 11) * 1.1102230246251565e-16;
  return (T)(i64)floor(a + (b - a) * u);
}

template <typename T>
__global__ __launch_bounds__(256) void k_fill(T* out, i64 n, Geom geo, int contiguous, i64 base,
                                              int kind, int dt, double a, double b, u64 seed) {
  i64 stride = (i64)gridDim.x * 256;
  for (i64 e = (i64)blockIdx.x * 256 + threadIdx.x; e < n; e += stride) {
    i64 g;
    if (contiguous) {
      g = base + e;
    } else {  // unravel over tile shape (a), shift by ul (b), ravel over array shape (c)
      i64 rem = e, mul = 1;
      g = 0;
      for (int d = geo.ndim - 1; d >= 0; --d) {
        i64 li = rem % geo.a[d];
        rem /= geo.a[d];
        g += (li + geo.b[d]) * mul;
        mul *= geo.c[d];
      }
    }
    T v;
    if constexpr (sizeof(T) == 4 && (T)0.5f != (T)0) v = fill_value<float>(kind, dt, a, b, seed, g);
    else if constexpr (sizeof(T) == 8 && (T)0.5 != (T)0) v = fill_value<double>(kind, dt, a, b, seed, g);
    else v = fill_value_int<T>(kind, a, b, seed, g);
    out[e] = v;
  }
}

extern "C" int spx_fill(int dtype, int kind, void* out, int ndim, const int64_t* tile_shape,
                        const int64_t* ul, const int64_t* array_shape, double a, double b,
                        uint64_t seed, void* stream) {
  if (!valid_dtype(dtype)) return set_err(SPX_EINVAL, "spx_fill: bad dtype %d", dtype);
  if (ndim < 0 || ndim > 8) return set_err(SPX_EINVAL, "spx_fill: ndim %d > 8", ndim);
  if (kind < SPX_FILL_CONST || kind > SPX_FILL_NORMAL)
    return set_err(SPX_EINVAL, "spx_fill: bad kind %d", kind);
  Geom geo{};
  geo.ndim = ndim;
  i64 n = 1;
  for (int d = 0; d < ndim; ++d) {
    geo.a[d] = tile_shape[d] > 0 ? tile_shape[d] : 1;
    geo.b[d] = ul[d];
    geo.c[d] = array_shape[d] > 0 ? array_shape[d] : 1;
    n *= tile_shape[d];
  }
  if (n == 0) return SPX_OK;
  if (!out) return set_err(SPX_EINVAL, "spx_fill: null output");
  // contiguous in the global flat index iff all dims after the first equal the array's
  int contiguous = 1;
  for (int d = 1; d < ndim; ++d)
    if (geo.a[d] != geo.c[d] || geo.b[d] != 0) contiguous = 0;
  i64 base = 0, mul = 1;
  for (int d = ndim - 1; d >= 0; --d) {
    base += geo.b[d] * mul;
    mul *= geo.c[d];
  }
  int g = grid_for(n, 4);
  switch (dtype) {
    case SPX_F32: k_fill<float><<<g, 256, 0, S(stream)>>>((float*)out, n, geo, contiguous, base, kind, dtype, a, b, seed); break;
    case SPX_F64: k_fill<double><<<g, 256, 0, S(stream)>>>((double*)out, n, geo, contiguous, base, kind, dtype, a, b, seed); break;
    case SPX_I32: k_fill<int32_t><<<g, 256, 0, S(stream)>>>((int32_t*)out, n, geo, contiguous, base, kind, dtype, a, b, seed); break;
    case SPX_I64: k_fill<int64_t><<<g, 256, 0, S(stream)>>>((int64_t*)out, n, geo, contiguous, base, kind, dtype, a, b, seed); break;
    default: k_fill<uint8_t><<<g, 256, 0, S(stream)>>>((uint8_t*)out, n, geo, contiguous, base, kind, dtype, a, b, seed); break;
  }
  LAUNCH_CHECK("spx_fill");
  return SPX_OK;
}

// ======================================================== reduce finalize
__device__ __forceinline__ bool dnan(double x) { return x != x; }

__device__ __forceinline__ double comb_f(int op, double acc, double v) {
  if (op == SPX_OP_SUM) return acc + v;
  if (dnan(acc) || dnan(v)) return dnan(acc) ? acc : v;  // NaN propagates (np.minimum)
  if (op == SPX_OP_MIN) return v < acc ? v : acc;
  return v > acc ? v : acc;
}
__device__ __forceinline__ i64 comb_i(int op, i64 acc, i64 v) {
  if (op == SPX_OP_SUM) return (i64)((u64)acc + (u64)v);
  if (op == SPX_OP_MIN) return v < acc ? v : acc;
  return v > acc ? v : acc;
}
// index value marking an empty (value, index) slot: never wins, always loses
#define ARG_EMPTY 0x7fffffffffffffffLL
// (value, index) "is candidate better than best" for ARGMIN/ARGMAX with
// numpy's NaN rule (first NaN wins) and first-index tie break.
__device__ __forceinline__ bool arg_better(int op, double v, i64 vi, double b, i64 bi) {
  bool vn = dnan(v), bn = dnan(b);
  if (vn || bn) {
    if (vn && !bn) return true;
    if (!vn && bn) return false;
    return vi < bi;
  }
  if (v == b) return vi < bi;
  return op == SPX_OP_ARGMIN ? (v < b) : (v > b);
}
// integer values compare as int64 (a double compare would merge distinct
// values above 2^53 and hand the tie to the lower index)
__device__ __forceinline__ bool arg_better_i(int op, i64 v, i64 vi, i64 b, i64 bi) {
  if (v == b) return vi < bi;
  return op == SPX_OP_ARGMIN ? (v < b) : (v > b);
}
// fold partial p = (v, vi) into the running best (b, bi); ARG_EMPTY slots
// never win
template <typename V>
__device__ __forceinline__ void arg_fold(int op, V v, i64 vi, V& b, i64& bi) {
  bool better;
  if constexpr (std::is_same<V, double>::value) better = arg_better(op, v, vi, b, bi);
  else better = arg_better_i(op, v, vi, b, bi);
  if (vi != ARG_EMPTY && (bi == ARG_EMPTY || better)) { b = v; bi = vi; }
}

__global__ __launch_bounds__(256) void k_finalize(int op, int acc_dt, int out_dt, const void* pv,
                                                  const i64* pi, i64 P, i64 n, void* out,
                                                  void* out_val) {
  i64 stride = (i64)gridDim.x * 256;
  for (i64 i = (i64)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    if ((op == SPX_OP_ARGMIN || op == SPX_OP_ARGMAX) && is_float_dt(acc_dt)) {
      double b = ld_f(pv, acc_dt, i);
      i64 bi = pi[i];
      for (i64 p = 1; p < P; ++p) arg_fold(op, ld_f(pv, acc_dt, p * n + i), pi[p * n + i], b, bi);
      ((i64*)out)[i] = bi;
      if (out_val) st_f(out_val, acc_dt, i, b);
    } else if (op == SPX_OP_ARGMIN || op == SPX_OP_ARGMAX) {
      i64 b = ld_i(pv, acc_dt, i);
      i64 bi = pi[i];
      for (i64 p = 1; p < P; ++p) arg_fold(op, ld_i(pv, acc_dt, p * n + i), pi[p * n + i], b, bi);
      ((i64*)out)[i] = bi;
      if (out_val) st_i(out_val, acc_dt, i, b);
    } else if (is_float_dt(acc_dt)) {
      double acc = ld_f(pv, acc_dt, i);
      if (acc_dt == SPX_F32) {  // keep fp32 rounding of each step for fp32 accumulators
        float facc = (float)acc;
        for (i64 p = 1; p < P; ++p) {
          float v = ((const float*)pv)[p * n + i];
          facc = (op == SPX_OP_SUM) ? facc + v : (float)comb_f(op, (double)facc, (double)v);
        }
        acc = facc;
      } else {
        for (i64 p = 1; p < P; ++p) acc = comb_f(op, acc, ld_f(pv, acc_dt, p * n + i));
      }
      if (is_float_dt(out_dt)) st_f(out, out_dt, i, acc);
      else st_i(out, out_dt, i, (i64)acc);
    } else {
      i64 acc = ld_i(pv, acc_dt, i);
      for (i64 p = 1; p < P; ++p) acc = comb_i(op, acc, ld_i(pv, acc_dt, p * n + i));
      st_i(out, out_dt, i, acc);
    }
  }
}

// Many partials per output (a tall column reduce splits R over P ~ 2048
// blocks, e.g. cfg5's (1e8, 64) gradient): one block per output, threads
// stride over P in order, then a fixed-shape LDS tree -- deterministic run to
// run.  Float partials are combined in fp64.
__global__ __launch_bounds__(256) void k_finalize_wide(int op, int acc_dt, int out_dt, const void* pv,
                                                       const i64* pi, i64 P, i64 n, void* out,
                                                       void* out_val) {
  __shared__ double sv[256];
  __shared__ i64 si[256];
  __shared__ i64 sw[256];  // integer arg values (compared as int64)
  const int t = threadIdx.x;
  const bool arg = op == SPX_OP_ARGMIN || op == SPX_OP_ARGMAX;
  const bool fl = is_float_dt(acc_dt);
  for (i64 i = blockIdx.x; i < n; i += gridDim.x) {
    double b = 0.0;
    i64 bw = 0;
    i64 bi = ARG_EMPTY;
    bool have = false;
    for (i64 p = t; p < P; p += 256) {
      if (arg && fl) {
        arg_fold(op, ld_f(pv, acc_dt, p * n + i), pi[p * n + i], b, bi);
      } else if (arg) {
        arg_fold(op, ld_i(pv, acc_dt, p * n + i), pi[p * n + i], bw, bi);
      } else if (fl) {
        double v = ld_f(pv, acc_dt, p * n + i);
        b = have ? comb_f(op, b, v) : v;
      } else {
        i64 v = ld_i(pv, acc_dt, p * n + i);
        bi = have ? comb_i(op, bi, v) : v;
      }
      have = true;
    }
    sv[t] = b;
    si[t] = bi;
    sw[t] = bw;
    __syncthreads();
    // lanes with no partial (P < 256) hold have=false: they are skipped by
    // letting the tree only combine slots < min(P, 256)
    const int m = P < 256 ? (int)P : 256;
    for (int h = 128; h > 0; h >>= 1) {
      if (t < h && t + h < m) {
        if (arg && fl) {
          double vb = sv[t];
          i64 ib = si[t];
          arg_fold(op, sv[t + h], si[t + h], vb, ib);
          sv[t] = vb;
          si[t] = ib;
        } else if (arg) {
          i64 vb = sw[t];
          i64 ib = si[t];
          arg_fold(op, sw[t + h], si[t + h], vb, ib);
          sw[t] = vb;
          si[t] = ib;
        } else if (fl) {
          sv[t] = comb_f(op, sv[t], sv[t + h]);
        } else {
          si[t] = comb_i(op, si[t], si[t + h]);
        }
      }
      __syncthreads();
    }
    if (t == 0) {
      if (arg) {
        ((i64*)out)[i] = si[0];
        if (out_val) {
          if (fl) st_f(out_val, acc_dt, i, sv[0]);
          else st_i(out_val, acc_dt, i, sw[0]);
        }
      } else if (fl) {
        if (is_float_dt(out_dt)) st_f(out, out_dt, i, sv[0]);
        else st_i(out, out_dt, i, (i64)sv[0]);
      } else {
        st_i(out, out_dt, i, si[0]);
      }
    }
    __syncthreads();
  }
}

extern "C" int spx_reduce_finalize(int op, int acc_dtype, int out_dtype, const void* part_val,
                                   const int64_t* part_idx, int64_t P, int64_t n, void* out,
                                   void* out_val, void* stream) {
  if (!valid_dtype(acc_dtype) || !valid_dtype(out_dtype))
    return set_err(SPX_EINVAL, "spx_reduce_finalize: bad dtype");
  if (op < SPX_OP_SUM || op > SPX_OP_ARGMAX) return set_err(SPX_EINVAL, "spx_reduce_finalize: bad op %d", op);
  if (P < 1 || n < 0) return set_err(SPX_EINVAL, "spx_reduce_finalize: bad P/n");
  if (n == 0) return SPX_OK;
  if ((op == SPX_OP_ARGMIN || op == SPX_OP_ARGMAX) && !part_idx)
    return set_err(SPX_EINVAL, "spx_reduce_finalize: arg op needs part_idx");
  if (P >= 32 && n <= 16384)
    k_finalize_wide<<<(unsigned)(n < 4096 ? n : 4096), 256, 0, S(stream)>>>(op, acc_dtype, out_dtype, part_val,
                                                                            part_idx, P, n, out, out_val);
  else
    k_finalize<<<grid_for(n), 256, 0, S(stream)>>>(op, acc_dtype, out_dtype, part_val, part_idx, P, n,
                                                   out, out_val);
  LAUNCH_CHECK("spx_reduce_finalize");
  return SPX_OK;
}

// =================================================================== merge
__global__ __launch_bounds__(256) void k_merge(int op, int dt, void* dst, uint8_t* mask, Geom g,
                                               i64 n, const void* src, int sdt, int fast,
                                               int fast_reduce) {
  // g.a = dst_shape, g.b = region_ul, g.c = region_shape
  i64 stride = (i64)gridDim.x * 256;
  for (i64 e = (i64)blockIdx.x * 256 + threadIdx.x; e < n; e += stride) {
    i64 di;
    if (fast) {
      di = e;
    } else {
      i64 rem = e, mul = 1;
      di = 0;
      for (int d = g.ndim - 1; d >= 0; --d) {
        i64 li = rem % g.c[d];
        rem /= g.c[d];
        di += (li + g.b[d]) * mul;
        mul *= g.a[d];
      }
    }
    bool reduce;
    if (op == SPX_OP_REPLACE) reduce = false;
    else if (fast) reduce = fast_reduce;
    else reduce = mask ? (mask[di] != 0) : true;
    if (is_float_dt(dt)) {
      double v = ld_f(src, sdt, e);
      if (reduce) v = comb_f(op, ld_f(dst, dt, di), v);
      st_f(dst, dt, di, v);
    } else {
      i64 v = is_float_dt(sdt) ? (i64)ld_f(src, sdt, e) : ld_i(src, sdt, e);
      if (reduce) v = comb_i(op, ld_i(dst, dt, di), v);
      st_i(dst, dt, di, v);
    }
    if (mask) mask[di] = 1;
  }
}

extern "C" int spx_merge(int op, int dtype, void* dst, uint8_t* mask, int ndim,
                         const int64_t* dst_shape, const int64_t* region_ul,
                         const int64_t* region_shape, const void* src, int src_dtype,
                         int full_tile_fastpath, void* stream) {
  if (!valid_dtype(dtype) || !valid_dtype(src_dtype)) return set_err(SPX_EINVAL, "spx_merge: bad dtype");
  if (!(op == SPX_OP_SUM || op == SPX_OP_MIN || op == SPX_OP_MAX || op == SPX_OP_REPLACE))
    return set_err(SPX_EINVAL, "spx_merge: bad op %d", op);
  if (ndim < 0 || ndim > 8) return set_err(SPX_EINVAL, "spx_merge: ndim > 8");
  Geom g{};
  g.ndim = ndim;
  i64 n = 1;
  bool full = true;
  for (int d = 0; d < ndim; ++d) {
    g.a[d] = dst_shape[d];
    g.b[d] = region_ul[d];
    g.c[d] = region_shape[d];
    if (region_ul[d] < 0 || region_ul[d] + region_shape[d] > dst_shape[d])
      return set_err(SPX_EINVAL, "spx_merge: region out of bounds on dim %d", d);
    if (region_ul[d] != 0 || region_shape[d] != dst_shape[d]) full = false;
    n *= region_shape[d];
  }
  if (n == 0) return SPX_OK;
  if (!dst || !src) return set_err(SPX_EINVAL, "spx_merge: null pointer");
  int fast = (full && full_tile_fastpath) ? 1 : 0;
  int fast_reduce = 0;
  if (fast && op != SPX_OP_REPLACE) {
    if (mask) {
      uint8_t m0 = 0;
      HIP_TRY(hipMemcpyAsync(&m0, mask, 1, hipMemcpyDeviceToHost, S(stream)));
      HIP_TRY(hipStreamSynchronize(S(stream)));
      fast_reduce = m0 != 0;
    } else {
      fast_reduce = 1;
    }
  }
  k_merge<<<grid_for(n), 256, 0, S(stream)>>>(op, dtype, dst, mask, g, n, src, src_dtype, fast, fast_reduce);
  LAUNCH_CHECK("spx_merge");
  return SPX_OK;
}

// ============================================================= copy region
struct Geom2 {
  int ndim;
  i64 dshape[8], dul[8], sshape[8], sul[8], cshape[8];
};

__global__ __launch_bounds__(256) void k_copy2(int ddt, void* dst, int sdt, const void* src,
                                               Geom2 g, i64 n) {
  i64 stride = (i64)gridDim.x * 256;
  for (i64 e = (i64)blockIdx.x * 256 + threadIdx.x; e < n; e += stride) {
    i64 rem = e, dm = 1, sm = 1, di = 0, si = 0;
    for (int d = g.ndim - 1; d >= 0; --d) {
      i64 li = rem % g.cshape[d];
      rem /= g.cshape[d];
      di += (li + g.dul[d]) * dm;
      si += (li + g.sul[d]) * sm;
      dm *= g.dshape[d];
      sm *= g.sshape[d];
    }
    if (ddt == sdt) {
      switch (ddt) {
        case SPX_BOOL: ((uint8_t*)dst)[di] = ((const uint8_t*)src)[si]; break;
        case SPX_I32: ((int32_t*)dst)[di] = ((const int32_t*)src)[si]; break;
        case SPX_F32: ((float*)dst)[di] = ((const float*)src)[si]; break;
        case SPX_I64: ((int64_t*)dst)[di] = ((const int64_t*)src)[si]; break;
        default: ((double*)dst)[di] = ((const double*)src)[si]; break;
      }
    } else if (is_float_dt(sdt)) {
      if (is_float_dt(ddt)) st_f(dst, ddt, di, ld_f(src, sdt, si));
      else st_i(dst, ddt, di, (i64)ld_f(src, sdt, si));
    } else {
      st_i(dst, ddt, di, ld_i(src, sdt, si));
    }
  }
}

extern "C" int spx_copy_region(int dst_dtype, void* dst, const int64_t* dst_shape,
                               const int64_t* dst_ul, int src_dtype, const void* src,
                               const int64_t* src_shape, const int64_t* src_ul, int ndim,
                               const int64_t* copy_shape, void* stream) {
  if (!valid_dtype(dst_dtype) || !valid_dtype(src_dtype)) return set_err(SPX_EINVAL, "spx_copy_region: bad dtype");
  if (ndim < 0 || ndim > 8) return set_err(SPX_EINVAL, "spx_copy_region: ndim > 8");
  Geom2 g{};
  g.ndim = ndim;
  i64 n = 1;
  for (int d = 0; d < ndim; ++d) {
    g.dshape[d] = dst_shape[d];
    g.dul[d] = dst_ul[d];
    g.sshape[d] = src_shape[d];
    g.sul[d] = src_ul[d];
    g.cshape[d] = copy_shape[d];
    if (dst_ul[d] < 0 || dst_ul[d] + copy_shape[d] > dst_shape[d] || src_ul[d] < 0 ||
        src_ul[d] + copy_shape[d] > src_shape[d])
      return set_err(SPX_EINVAL, "spx_copy_region: region out of bounds on dim %d", d);
    n *= copy_shape[d];
  }
  if (n == 0) return SPX_OK;
  if (!dst || !src) return set_err(SPX_EINVAL, "spx_copy_region: null pointer");
  k_copy2<<<grid_for(n), 256, 0, S(stream)>>>(dst_dtype, dst, src_dtype, src, g, n);
  LAUNCH_CHECK("spx_copy_region");
  return SPX_OK;
}

// ================================================== arg-reduction combine
__global__ __launch_bounds__(256) void k_argcombine(int op, int dt, const void* vals, const i64* idx,
                                                    i64 R, i64 n, void* out_val, i64* out_idx) {
  i64 stride = (i64)gridDim.x * 256;
  for (i64 i = (i64)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    if (is_float_dt(dt)) {
      double b = ld_f(vals, dt, i);
      i64 bi = idx[i];
      for (i64 r = 1; r < R; ++r) arg_fold(op, ld_f(vals, dt, r * n + i), idx[r * n + i], b, bi);
      out_idx[i] = bi;
      if (out_val) st_f(out_val, dt, i, b);
    } else {
      i64 b = ld_i(vals, dt, i);
      i64 bi = idx[i];
      for (i64 r = 1; r < R; ++r) arg_fold(op, ld_i(vals, dt, r * n + i), idx[r * n + i], b, bi);
      out_idx[i] = bi;
      if (out_val) st_i(out_val, dt, i, b);
    }
  }
}

extern "C" int spx_argreduce_combine(int op, int dtype, const void* vals, const int64_t* idx,
                                     int64_t R, int64_t n, void* out_val, int64_t* out_idx,
                                     void* stream) {
  if (op != SPX_OP_ARGMIN && op != SPX_OP_ARGMAX) return set_err(SPX_EINVAL, "spx_argreduce_combine: bad op");
  if (!valid_dtype(dtype)) return set_err(SPX_EINVAL, "spx_argreduce_combine: bad dtype");
  if (R < 1 || n < 0) return set_err(SPX_EINVAL, "spx_argreduce_combine: bad R/n");
  if (n == 0) return SPX_OK;
  if (!vals || !idx || !out_idx) return set_err(SPX_EINVAL, "spx_argreduce_combine: null pointer");
  k_argcombine<<<grid_for(n), 256, 0, S(stream)>>>(op, dtype, vals, idx, R, n, out_val, out_idx);
  LAUNCH_CHECK("spx_argreduce_combine");
  return SPX_OK;
}

// ==================================================================== GEMM
// fp32 / fp64 MFMA kernels live in gemm_kernels.h (shared with the tuning
// harness tools/gemm_tune.hip).  Configurations chosen by measurement on
// MI355X (profiles/r01_gemm_tune.txt):
//   fp32 large: 256x256x16, 16 waves (4x4), grouped order GM=8  -> 136 TF (86.6 %)
//   fp32 small: 128x128x16, 4 waves (2x2), GM=8                 -> 131 TF at 8192
//   fp64      : 128x128x16, 16 waves (4x4)                      -> 69.3 TF (88.2 %)
// (the 4-wave fp64 layout needs 304 registers -> 1 wave per SIMD -> 40 TF).
#include "gemm_kernels.h"

// fp32: 256x128x16, 8 waves (with the k-contiguous A staging: 141.4 TF = 89.9 %
// of 157.3 at 32768^3 against 135.6 TF for the 256x256x16 16-wave tile,
// profiles/r02_gemm_tune_ak.txt)
// fp32: one accumulator set, flushed into C every 512 K-tiles (gemm_kernels.h
// GFL): chains of 4096 MFMA steps instead of K / 2 (four flushes at cfg4's
// K = 32768), at the one-chain form's registers and occupancy (round 3's
// register two-level form, SEG, cost 6 %).  Round 5, the cfg4 product against
// fp64 at EVERY one of its 2^30 elements (tools/gemm_margin.py,
// profiles/r05_gemm_gfl_margin.txt, one box): GFL 1024 141.0 TF, max rel err
// 7.32e-6 (73 % of the 1e-5 budget); 512 140.4 TF, 3.71e-6; 256 140.2 TF,
// 1.80e-6 -- 512 keeps 40 % of the budget in reserve for 0.4 TF
// (test_dot_cfg4_full_size asserts <= 0.6e-5 over all elements).
constexpr int SPX_GEMM_GFL = 512;
typedef spx_mfma::Config<float, 256, 128, 16, 4, 2, 8, 0, SPX_GEMM_GFL> GemmF32Big;
typedef spx_mfma::Config<float, 128, 128, 16, 2, 2, 8, 0, SPX_GEMM_GFL> GemmF32Small;

// C *= beta (the GFL kernels take beta 0 or 1)
__global__ __launch_bounds__(256) void k_scale_rows(i64 M, i64 N, float* C, i64 ldc, float beta) {
  for (i64 i = (i64)blockIdx.x * 256 + threadIdx.x; i < M * N; i += (i64)gridDim.x * 256) {
    const i64 r = i / N, c = i % N;
    C[r * ldc + c] *= beta;
  }
}
typedef spx_mfma::Config<double, 128, 128, 16, 4, 4, 0> GemmF64;

// Round 6: the three-stage one-wave-per-SIMD kernels (gemm_kernels.h
// gemm_f32_p3 / gemm_f64_p3) for large aligned products.  fp32: chains of
// SPX_GEMM_GFL K-tiles flushed into C inside the kernel, as the two-stage
// kernel's GFL (the same chains: the cfg4 product is bit-identical to it);
// fp64 (experimental, SPX_GEMM_P3=2): K in launches of SPX_GEMM_KCHUNK.
// SPX_GEMM_P3=0 in the environment selects the two-stage kernels (A/B; read
// once).
constexpr i64 SPX_GEMM_KCHUNK = 8192;
static int gemm_p3_on() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("SPX_GEMM_P3");
    v = e ? atoi(e) : 1;
  }
  return v;
}
template <typename T, typename F>
static hipError_t gemm_kchunks(i64 K, const T* a, const T* b, i64 ldb, T beta, F launch) {
  for (i64 k0 = 0; k0 < K; k0 += SPX_GEMM_KCHUNK) {
    const i64 kc = K - k0 < SPX_GEMM_KCHUNK ? K - k0 : SPX_GEMM_KCHUNK;
    const hipError_t e = launch(kc, a + k0, b + k0 * ldb, k0 ? (T)1 : beta);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// integer GEMM (exact, wrap-around like NumPy's int matmul): 16x16 output
// tile per 256-thread block, K staged through LDS.  Used for integer dot
// products (the reference's tests multiply arange ints); not a hot path.
template <typename T>
__global__ __launch_bounds__(256) void k_gemm_int(i64 M, i64 N, i64 K, const T* __restrict__ A, i64 lda,
                                                  const T* __restrict__ B, i64 ldb, T* __restrict__ C,
                                                  i64 ldc, T alpha, T beta) {
  __shared__ T As[16][17];
  __shared__ T Bs[16][17];
  int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  i64 row = (i64)blockIdx.y * 16 + ty, col = (i64)blockIdx.x * 16 + tx;
  typedef typename std::conditional<sizeof(T) == 8, u64, uint32_t>::type U;
  U acc = 0;
  for (i64 k0 = 0; k0 < K; k0 += 16) {
    As[ty][tx] = (row < M && k0 + tx < K) ? A[row * lda + k0 + tx] : (T)0;
    Bs[ty][tx] = (k0 + ty < K && col < N) ? B[(k0 + ty) * ldb + col] : (T)0;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) acc += (U)As[ty][k] * (U)Bs[k][tx];
    __syncthreads();
  }
  if (row < M && col < N) {
    U v = (U)alpha * acc;
    if (beta != 0) v += (U)beta * (U)C[row * ldc + col];
    C[row * ldc + col] = (T)v;
  }
}

extern "C" int spx_gemm(int dtype, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
                        const void* B, int64_t ldb, void* C, int64_t ldc, double alpha,
                        double beta, void* stream) {
  if (dtype != SPX_F32 && dtype != SPX_F64 && dtype != SPX_I32 && dtype != SPX_I64)
    return set_err(SPX_ENOTSUP, "spx_gemm: dtype %d not supported (F32/F64/I32/I64)", dtype);
  if (M < 0 || N < 0 || K < 0) return set_err(SPX_EINVAL, "spx_gemm: negative dimension");
  if (lda < K || ldb < N || ldc < N) return set_err(SPX_EINVAL, "spx_gemm: leading dimension too small");
  if (M == 0 || N == 0) return SPX_OK;
  if (!A || !B || !C) return set_err(SPX_EINVAL, "spx_gemm: null pointer");
  if (K == 0) {  // C = beta * C
    return set_err(SPX_ENOTSUP, "spx_gemm: K == 0 not supported");
  }
  if (dtype == SPX_I32 || dtype == SPX_I64) {
    dim3 grid((unsigned)((N + 15) / 16), (unsigned)((M + 15) / 16));
    if (dtype == SPX_I64)
      k_gemm_int<int64_t><<<grid, 256, 0, S(stream)>>>(M, N, K, (const int64_t*)A, lda, (const int64_t*)B, ldb,
                                                       (int64_t*)C, ldc, (int64_t)alpha, (int64_t)beta);
    else
      k_gemm_int<int32_t><<<grid, 256, 0, S(stream)>>>(M, N, K, (const int32_t*)A, lda, (const int32_t*)B, ldb,
                                                       (int32_t*)C, ldc, (int32_t)alpha, (int32_t)beta);
    LAUNCH_CHECK("spx_gemm(int)");
    return SPX_OK;
  }
  hipError_t e;
  if (dtype == SPX_F32) {
    const float *a = (const float*)A, *b = (const float*)B;
    if (beta != 0.0 && beta != 1.0) {
      k_scale_rows<<<(unsigned)std::min<i64>((M * N + 255) / 256, 4096), 256, 0, S(stream)>>>(M, N, (float*)C, ldc,
                                                                                           (float)beta);
      LAUNCH_CHECK("spx_gemm(scale C)");
      beta = 1.0;
    }
    i64 big_tiles = ((M + 255) / 256) * ((N + 255) / 256);
    if (big_tiles >= 512 && big_tiles <= 0x7fffffffLL && gemm_p3_on() && spx_mfma::p3_ok(M, N, K, A, lda, B, ldb)) {
      // one launch, K in chunks of SPX_GEMM_GFL K-tiles inside the kernel
      // (beta is 0 or 1 here, as the flush needs)
      e = spx_mfma::p3_launch<8, 0, SPX_GEMM_GFL, 1, 4>(M, N, K, a, lda, b, ldb, (float*)C, ldc, (float)alpha,
                                                         (float)beta, S(stream));
    } else if (big_tiles >= 512) {
      if (big_tiles > 0x7fffffffLL) return set_err(SPX_EINVAL, "spx_gemm: too many tiles");
      e = GemmF32Big::launch(M, N, K, a, lda, b, ldb, (float*)C, ldc, (float)alpha, (float)beta,
                             GemmF32Big::is_aligned(M, N, K, A, lda, B, ldb), S(stream));
    } else {
      e = GemmF32Small::launch(M, N, K, a, lda, b, ldb, (float*)C, ldc, (float)alpha, (float)beta,
                               GemmF32Small::is_aligned(M, N, K, A, lda, B, ldb), S(stream));
    }
    if (e != hipSuccess) return set_err(SPX_EHIP, "spx_gemm(f32) launch failed: %s", hipGetErrorString(e));
  } else {
    i64 tiles = ((M + 127) / 128) * ((N + 127) / 128);
    if (tiles > 0x7fffffffLL) return set_err(SPX_EINVAL, "spx_gemm: too many tiles");
    if (tiles >= 1024 && gemm_p3_on() > 1 && spx_mfma::p3d_ok<16>(M, N, K, A, lda, B, ldb)) {
      const double *a = (const double*)A, *b = (const double*)B;
      e = gemm_kchunks<double>(K, a, b, ldb, beta, [&](i64 kc, const double* ak, const double* bk, double bt) {
        return spx_mfma::p3d_launch<8, 16, 0, 4>(M, N, kc, ak, lda, bk, ldb, (double*)C, ldc, alpha, bt, S(stream));
      });
    } else
    e = GemmF64::launch(M, N, K, (const double*)A, lda, (const double*)B, ldb, (double*)C, ldc, alpha, beta,
                        GemmF64::is_aligned(M, N, K, A, lda, B, ldb), S(stream));
    if (e != hipSuccess) return set_err(SPX_EHIP, "spx_gemm(f64) launch failed: %s", hipGetErrorString(e));
  }
  return SPX_OK;
}

// ================================================================ k-means
// The provisional adds' bookkeeping of spx_kmeans_step (k_kmeans_pp added
// every finite undecided row under its screen-best centre p and left the
// label code -2 - p, or -1 for a row it did not add): when a list pass
// writes such a row's final label it sets the row's bit in `add` if the row
// must be added under that label (not added, or added under another centre)
// and in `sub`, with pside[row] = p, if it must come out of p.  The struct
// sits in the workspace at counters + 4, null outside the step.
struct KmMove {
  unsigned long long* add;
  unsigned long long* sub;
  i64* pside;
};
__device__ __forceinline__ void km_label(i64* labels, const unsigned int* counters, i64 row, i64 lab) {
  const KmMove* mv = (const KmMove*)(counters + 4);
  unsigned long long* const add = mv->add;
  if (add) {
    const i64 code = labels[row];
    const i64 p = code <= -2 ? -2 - code : -1;
    const bool sb = p >= 0 && p != lab;
    const unsigned long long bit = 1ull << (row & 31);
    if (code == -1 || sb) atomicOr(add + (row >> 5), bit);
    if (sb) {
      atomicOr(mv->sub + (row >> 5), bit);
      mv->pside[row] = p;
    }
  }
  labels[row] = lab;
}
// km_label with the move bookkeeping read ahead: mv = the workspace's KmMove
// (read once per kernel) and code = labels[row] as it was before this write
// (read before the caller's next loads, so no wait on them)
// (global-address-space pointers: the KmMove fields are generic pointers read
// from memory, and flat stores / atomics would make the compiler's waits
// count the LDS queue too, so every wait after them became a full drain)
typedef __attribute__((address_space(1))) unsigned long long kg_u64;
typedef __attribute__((address_space(1))) i64 kg_i64;
__device__ __forceinline__ void km_label_pre(i64* labels, const KmMove& mv, i64 row, i64 lab, i64 code) {
  if (mv.add) {
    const i64 p = code <= -2 ? -2 - code : -1;
    const bool sb = p >= 0 && p != lab;
    const unsigned long long bit = 1ull << (row & 31);
    if (code == -1 || sb) __hip_atomic_fetch_or((kg_u64*)mv.add + (row >> 5), bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (sb) {
      __hip_atomic_fetch_or((kg_u64*)mv.sub + (row >> 5), bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ((kg_i64*)mv.pside)[row] = p;
    }
  }
  labels[row] = lab;
}
__global__ void k_km_setmove(KmMove* dst, unsigned long long* add, unsigned long long* sub, i64* pside) {
  if (threadIdx.x == 0) *dst = KmMove{add, sub, pside};
}

// Assignment: labels[p] = argmin_c ||P[p] - C[c]||_2 in exactly the order of
// scipy.spatial.distance.cdist (k_means_.py:58 via kmeans_dist_mapper): fp64,
// s = sum_d (x_d - c_d)^2 accumulated sequentially over d with separately
// rounded multiply and add (this file is compiled with -ffp-contract=off),
// dist = sqrt(s); first index wins ties of the sqrt'd distances
// (argmin(distances, axis=1), builtins.py:631-647).  Zero-padding the d loop
// past D appends exact +0.0 terms, so chunking does not change a bit.
// One point per lane; KM_CC centre accumulators live in registers while the
// dims stream through KM_DC-wide register chunks; the centre tile is staged
// in LDS and read as a broadcast.
#define KM_CC 64
#define KM_DC 16
template <typename TP>
__global__ __launch_bounds__(256) void k_kmeans_assign(i64 N, i64 D, i64 K, const TP* __restrict__ P, i64 ldp,
                                                       const double* __restrict__ C, i64* __restrict__ labels,
                                                       double* __restrict__ mind, const i64* __restrict__ rows,
                                                       const unsigned int* __restrict__ nrows, int r32) {
  // rows != NULL: only the *nrows points rows[0..*nrows) (the filter's
  // undecided points); the grid is sized for the worst case.  r32: the
  // distances are rounded to fp32 before the argmin (an outer product whose
  // target is fp32 stores them so: the reference's target.update casts).
  __shared__ double Cs[KM_CC][KM_DC];
  const i64 n = rows ? (i64)*nrows : N;
  for (i64 base = (i64)blockIdx.x * 256; base < n; base += (i64)gridDim.x * 256) {  // block-uniform
  const i64 q = base + threadIdx.x;
  const bool valid = q < n;
  const i64 p = valid ? (rows ? rows[q] : q) : 0;
  double best = 0.0;
  i64 bi = -1;
  for (i64 c0 = 0; c0 < K; c0 += KM_CC) {
    double s[KM_CC];
#pragma unroll
    for (int cc = 0; cc < KM_CC; ++cc) s[cc] = 0.0;
    for (i64 d0 = 0; d0 < D; d0 += KM_DC) {
      __syncthreads();
      for (int e = threadIdx.x; e < KM_CC * KM_DC; e += 256) {
        int cc = e / KM_DC, dd = e % KM_DC;
        Cs[cc][dd] = (c0 + cc < K && d0 + dd < D) ? C[(c0 + cc) * D + d0 + dd] : 0.0;
      }
      __syncthreads();
      double x[KM_DC];
#pragma unroll
      for (int dd = 0; dd < KM_DC; ++dd) x[dd] = (valid && d0 + dd < D) ? (double)P[p * ldp + d0 + dd] : 0.0;
#pragma unroll
      for (int cc = 0; cc < KM_CC; ++cc) {
        double acc = s[cc];
#pragma unroll
        for (int dd = 0; dd < KM_DC; ++dd) {
          double df = x[dd] - Cs[cc][dd];
          double sq = df * df;
          acc = acc + sq;
        }
        s[cc] = acc;
      }
    }
#pragma unroll
    for (int cc = 0; cc < KM_CC; ++cc) {
      if (c0 + cc < K) {
        double dist = sqrt(s[cc]);
        if (r32) dist = (double)(float)dist;
        if (bi < 0 || dist < best || (dist != dist && best == best)) {
          best = dist;
          bi = c0 + cc;
        }
      }
    }
  }
  if (valid) {
    if (rows) km_label(labels, nrows, p, bi);  // list mode: nrows is the workspace's counters
    else labels[p] = bi;
    if (mind) mind[p] = best;
  }
  }
}

// Certified fast assignment.  Exact-order fp64 distances cost 3 fp64 VALU
// ops per (point, centre, dim); instead an fp32 MFMA GEMM gives
//   a'(p, c) = fl(|c|^2 - 2 p.c)   (= d^2(p, c) - |p|^2 up to rounding)
// for every centre, and a point is labelled here only when its best and
// second-best a' are separated by more than twice a rigorous bound e on
// |a' - a|:
//   2 (D + 3) u |p| |c|     fp32 fma-chain dot over D terms of fp32-rounded
//                           operands (v_mfma_f32_32x32x2_f32 is exactly such
//                           a chain), u = 2^-24;
//   2 u (|c|^2 + |p| |c|)   fp32 |c|^2 and the final fma;
//   4 D 1.2e-38 (1 + |c|)   fp32 underflow;
//   1e-8 (|p|^2 + |c|^2)    slack that dwarfs the fp64 rounding of scipy's
//                           sum and of the sqrt, so the certified winner is
//                           the strict, hence first-index, exact argmin;
// with |p|, |c| upper bounds (max over centres for |c|).  Undecided points
// (near-ties, non-finite values) are labelled in exactly scipy's order: for
// K <= 256 only the candidate centres (a' <= best + 2e, a 256-bit mask per
// point) are recomputed (k_kmeans_cand), otherwise every centre
// (k_kmeans_assign in list mode).  The labels are bit-identical to the
// all-exact kernel's.
// Layout: block = BM points x all centres in 256-centre tiles, waves of
// v_mfma_f32_32x32x2_f32 (BM/64 x 4 waves, 64 x 64 each), BK = 16,
// register-staged double buffering as in gemm_kernels.h; several blocks per
// CU so one block's epilogue overlaps another's MFMAs (KfProd, tuned with
// tools/kf_tune.hip).  The epilogue transposes each 64-row
// half of the S tile through LDS (row stride 264 floats: conflict-free both
// ways) and 8 lanes per row scan 32 centres each for the top two (fp32),
// merged by xor-shuffles.  |p| comes from the A tiles already in LDS.
constexpr int KF_BN = 256, KF_BK = 16;
constexpr int KF_EP = 264;  // epilogue row stride (floats)

struct KfCand {
  i64 row;
  unsigned int mask[8];  // bit k of word w <-> centre w + 8 k
};

__device__ __forceinline__ void kf_merge(float& b1, int& i1, float& b2, float o1, int oi, float o2) {
  if (o1 < b1 || (o1 == b1 && oi < i1)) {
    b2 = b1 < o2 ? b1 : o2;
    b1 = o1;
    i1 = oi;
  } else {
    b2 = b2 < o1 ? b2 : o1;
  }
}

// BM points per block (BM / 64 x 4 waves), LDS row padding PA (A) / PB (B),
// MINW = min waves per SIMD for the register budget.
template <typename TP, bool ALIGNED, int BM, int PA, int PB, int MINW>
__global__ __launch_bounds__(BM * 4, MINW) void k_kmeans_filter(i64 N, i64 D, i64 K, i64 Kp,
                                                                const TP* __restrict__ P, i64 ldp,
                                                                const float* __restrict__ CT,
                                                                const double* __restrict__ cn, const double* cmax_p,
                                                                i64* __restrict__ labels,
                                                                unsigned int* __restrict__ counters,
                                                                i64* __restrict__ full_list,
                                                                KfCand* __restrict__ cand_list) {
  typedef spx_mfma::Mfma<float> F;
  typedef float V __attribute__((ext_vector_type(4)));
  constexpr int BN = KF_BN, BK = KF_BK, NT = BM * 4, WN = 4;
  constexpr int WTM = 64, WTN = 64, TM = 2, TN = 2, HR = BM / 2;  // HR: rows per epilogue half
  constexpr int LB = BK * BN / 4 / NT;  // B loads per lane (A: 1)
  constexpr int MAIN_BYTES = (2 * BK * (BM + PA) + 2 * BK * (BN + PB)) * 4;
  constexpr int EPI_BYTES = HR * KF_EP * 4;
  static_assert(BM * BK / 4 == NT && LB * NT * 4 == BK * BN && HR * 8 == NT && PB % 4 == 0, "tiling");
  __shared__ __attribute__((aligned(16))) unsigned char lds[MAIN_BYTES > EPI_BYTES ? MAIN_BYTES : EPI_BYTES];
  __shared__ float pnp[4][BM];
  __shared__ float cns[BN];
  float(*As)[BK][BM + PA] = (float(*)[BK][BM + PA])lds;
  float(*Bs)[BK][BN + PB] = (float(*)[BK][BN + PB])(lds + 2 * BK * (BM + PA) * 4);
  float* E = (float*)lds;
  const i64 row0 = (i64)blockIdx.x * BM;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wm = w / WN, wn = w % WN;
  const int rl = t >> 3, sub = t & 7;                   // epilogue: row (of HR) and column phase
  const int nm = t & (BM - 1), nq = t / BM;             // row norm: row and k quarter
  const bool single = Kp == BN;
  float pn = 0.f;
  float s1[TM], s2[TM];
  int si[TM];
  bool bad[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    s1[i] = INFINITY;
    s2[i] = INFINITY;
    si[i] = -1;
    bad[i] = false;
  }
  const double cmax = cmax_p[0];
  // fp32 target: two exact distances whose squares differ by more than
  // 2^-21 (|p| + |c|)^2 are more than 2 fp32 ulps apart, so they cannot
  // round to one value; the margin is folded into e (gap > 2e + margin)
  const double mcoef = cmax_p[1];
  const double u32 = 5.9604644775390625e-08;
  V ra, rb[LB];
  for (i64 c0 = 0; c0 < Kp; c0 += BN) {
    const bool last = c0 + BN >= Kp;
    F::acc_t acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = F::zero();
    auto load = [&](i64 k0) {
      {
        const int r = t / (BK / 4), kq = t % (BK / 4);
        const i64 gr = row0 + r, gk = k0 + kq * 4;
        if (ALIGNED && gr < N) {
          ra = *(const V*)(P + gr * ldp + gk);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) ra[j] = (gr < N && gk + j < D) ? (float)P[gr * ldp + gk + j] : 0.f;
        }
      }
#pragma unroll
      for (int l = 0; l < LB; ++l) {
        const int idx = t + l * NT, kr = idx / (BN / 4), cq = idx % (BN / 4);
        const i64 bk = k0 + kr;
        rb[l] = bk < D ? *(const V*)(CT + bk * Kp + c0 + cq * 4) : (V){0.f, 0.f, 0.f, 0.f};
      }
    };
    auto store = [&](int buf) {
      const int r = t / (BK / 4), kq = t % (BK / 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) As[buf][kq * 4 + j][r] = ra[j];
#pragma unroll
      for (int l = 0; l < LB; ++l) {
        const int idx = t + l * NT, kr = idx / (BN / 4), cq = idx % (BN / 4);
        *(V*)(&Bs[buf][kr][cq * 4]) = rb[l];
      }
    };
    const int nk = (int)((D + BK - 1) / BK);
    __syncthreads();  // previous epilogue done with the shared buffers
    if (t < BN) cns[t] = (float)cn[c0 + t];
    load(0);
    store(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) load((i64)(kt + 1) * BK);
      if (c0 == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float v = As[cur][nq * 4 + k][nm];
          pn += v * v;
        }
      }
#pragma unroll
      for (int kk = 0; kk < BK / F::KS; ++kk) {
        const int k = kk * F::KS + F::opk(lane);
        float a[TM], b[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) a[i] = As[cur][k][wm * WTM + i * F::TILE + F::opi(lane)];
#pragma unroll
        for (int j = 0; j < TN; ++j) b[j] = Bs[cur][k][wn * WTN + j * F::TILE + F::opi(lane)];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = F::mma(a[i], b[j], acc[i][j]);
      }
      if (kt + 1 < nk) store(cur ^ 1);
      __syncthreads();
    }
    if (c0 == 0) pnp[nq][nm] = pn;
    // epilogue: half i holds rows wm*64 + i*32 + [0, 32) of both wm
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      if (i) __syncthreads();
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < F::NREG; ++r)
          E[(wm * 32 + F::crow(lane, r)) * KF_EP + wn * WTN + j * F::TILE + F::ccol(lane)] = acc[i][j][r];
      __syncthreads();
      float b1 = INFINITY, b2 = INFINITY;
      int i1 = -1;
      bool nf = false;
#pragma unroll 8
      for (int k = 0; k < BN / 8; ++k) {
        const int col = sub + 8 * k;
        const float a = __builtin_fmaf(-2.f, E[rl * KF_EP + col], cns[col]);
        nf |= a != a;
        if (a < b1) {
          b2 = b1;
          b1 = a;
          i1 = (int)c0 + col;
        } else if (a < b2) {
          b2 = a;
        }
      }
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) {
        const float o1 = __shfl_xor(b1, o, 64), o2 = __shfl_xor(b2, o, 64);
        const int oi = __shfl_xor(i1, o, 64);
        nf |= __shfl_xor((int)nf, o, 64) != 0;
        kf_merge(b1, i1, b2, o1, oi, o2);
      }
      kf_merge(s1[i], si[i], s2[i], b1, i1, b2);
      bad[i] |= nf;
      if (!last) continue;
      // decision for this half's rows (the 8 lanes of a row agree)
      const int lr = (rl / 32) * WTM + i * 32 + (rl % 32);  // row within the block
      const i64 row = row0 + lr;
      if (row >= N) continue;
      static_assert(BM / 64 * 32 == HR, "halves");
      const float p2f = pnp[0][lr] + pnp[1][lr] + pnp[2][lr] + pnp[3][lr];
      const double p2 = (double)p2f * 1.001 + (double)D * 2e-45;
      const double pnorm = sqrt(p2) * 1.0001;
      const double e = 2.0 * (double)(D + 3) * 1.01 * u32 * pnorm * cmax +
                       2.02 * u32 * (cmax * cmax + pnorm * cmax) + 4.0 * (double)D * 1.2e-38 * (1.0 + cmax) +
                       1e-8 * (p2 + cmax * cmax) + 0.5 * mcoef * (pnorm + cmax) * (pnorm + cmax) + 1e-300;
      const bool fin = !bad[i] && isfinite(s1[i]) && isfinite(e);
      if (fin && (double)s2[i] - (double)s1[i] > 2.0 * e) {
        if (sub == 0) labels[row] = si[i];
      } else if (fin && single) {
        const double thr = (double)s1[i] + 2.0 * e;
        unsigned int m = 0;
#pragma unroll 8
        for (int k = 0; k < BN / 8; ++k) {
          const int col = sub + 8 * k;
          const float a = __builtin_fmaf(-2.f, E[rl * KF_EP + col], cns[col]);
          if ((double)a <= thr) m |= 1u << k;
        }
        unsigned int slot = 0;
        if (sub == 0) slot = atomicAdd(&counters[1], 1u);
        slot = __shfl(slot, lane & ~7, 64);
        cand_list[slot].mask[sub] = m;
        if (sub == 0) cand_list[slot].row = row;
      } else if (sub == 0) {
        full_list[atomicAdd(&counters[0], 1u)] = row;
      }
    }
  }
}

template <int BM_, int PA, int PB, int MINW>
struct KfConf {
  static constexpr int BM = BM_;
  template <typename TP, bool AL>
  static void launch(i64 grid, hipStream_t s, i64 N, i64 D, i64 K, i64 Kp, const void* P, i64 ldp, const float* CT,
                     const double* cn, const double* cmax, i64* labels, unsigned int* counters, i64* full_list,
                     KfCand* cand_list) {
    k_kmeans_filter<TP, AL, BM, PA, PB, MINW><<<(unsigned)grid, BM * 4, 0, s>>>(
        N, D, K, Kp, (const TP*)P, ldp, CT, cn, cmax, labels, counters, full_list, cand_list);
  }
};
typedef KfConf<64, 2, 0, 3> KfProd;

// ---------------------------------------------------------------------------
// bf16x3 certified filter (fp32 points, K <= 256, D % 64 == 0, D <= 128).
// The fp32 filter above runs v_mfma_f32_32x32x2_f32 at the fp32 rate (1/16
// of bf16).  Here every fp32 operand is split exactly-enough into two bf16
// terms, x = xh + xl + rx with xh = bf16(x), xl = bf16(x - xh), |rx| <=
// 2^-18 |x|, and p.c is taken as ph.ch + ph.cl + pl.ch: three
// v_mfma_f32_32x32x16_bf16 per 32x32x16 block, 16/3 x the fp32 MFMA rate.
// Rigorous bound on |S - p.c| (S the computed dot product):
//   2^-24 |p||c|             centre fp64 -> fp32 rounding;
//   3.1 * 2^-18 |p||c|       the neglected pl.cl, rp.c and ph.rc terms
//                            (Cauchy-Schwarz over the elementwise bounds);
//   2 (48 G + D/(16 G) + 3) 2^-24 |p||c|  fp32 accumulation: the 48 G
//                            exact products per output of G = KB_GRP k-steps
//                            are summed into a fresh accumulator (an fma chain
//                            of 48 G) that is then added to the running sum
//                            (D/(16 G) adds; VALU adds out of the MFMA result,
//                            so G trades bound for issue slots); a factor 2
//                            covers directed rounding inside the MFMA;
//   1e-28 D (1 + |c|)^2      bf16 / fp32 underflow of the small terms;
// and the decision is the fp32 filter's: a'(p, c) = fl(|c|^2 - 2 S), a point
// is labelled here iff best and second-best a' differ by more than 2e.  The
// rest (near-ties; non-finite values) get exactly scipy's order as before:
// the candidate centres (a' <= best + 2e, natural mask layout: bit b of word
// w <-> centre 32 w + b) through k_kmeans_cand, non-finite points through
// the all-centre exact kernel.  Labels are bit-identical to the exact kernel.
// Layout: persistent blocks of KB_WAVES waves, one per CU (the split
// centres, 2 x 32 NCT x (D + 8) bf16, stay resident in LDS; rows padded by
// 16 B so the 32 lanes' ds_read_b128 of a B fragment are conflict-free);
// wave = 32 points x all 32 NCT centres (NCT accumulator tiles of 16
// registers); A fragments are loaded straight from global memory (lane
// (r, h) holds point r's dims 8h..8h+7 of the 16-dim k-step: row-major
// points ARE the A operand layout) through a 4-deep register ring; the
// epilogue reduces each point's top two across the 32 lanes of its half with
// xor-shuffles.
constexpr int KB_WAVES = 4;
constexpr int KB_DMAX = 128;
constexpr int KB_GRP = 4;  // k-steps per MFMA group (divides 4)
typedef __bf16 kb_bf8 __attribute__((ext_vector_type(8)));
typedef float kb_acc __attribute__((ext_vector_type(16)));
typedef float kb_f4 __attribute__((ext_vector_type(4)));

// Centred centres for the bf16x3 filters.  mu = fp32 mean of the centres;
// c' = C[c] - mu.  For every point x
//   |x - C[c]|^2 = |x - mu|^2 + (|c'|^2 + 2 mu.c' - 2 x.c'),
// and the first term does not depend on c, so the filters rank the centres
// by a'(x, c) = cc[c] - 2 x.c' with cc[c] = |c'|^2 + 2 mu.c'.  The bf16x3
// error of x.c' scales with |x| |c'| instead of |x| |c|: for points far from
// the origin (U[0,1)^128: |c| ~ 6.5, |c'| ~ 1.5-3.7) the certified bound e
// shrinks 2-4x and so does the share of undecided rows the exact path has to
// recompute (cfg3: 1.0 / 3.1 % -> 0.5 / 0.8 %).
// CBh / CBl[c][d]: bf16 split of (float)c'[d] (zero past K); cnf[c] =
// (float)cc[c] (huge past K); cmax[0] = max_c |c'|, cmax[2] = |mu| (one block).
// One block of 1024 threads: mu from 8 column partial sums per dimension
// (combined in a fixed order), then one wave per centre (lane = dimension,
// coalesced), wave-reduced |c'|^2 and mu.c' in a fixed shuffle order.
// For the fp16 screen (k_kmeans_filter_as MODE 1, which centres the points as
// well): cnf2[c] = (float)|c'|^2, muf = mu, cmax[3] = max_c |c' - fp16(hi + lo)|
// (the screen's own rounding of each centre, measured exactly).
__global__ __launch_bounds__(1024) void k_kmeans_prep_b3(i64 D, i64 K, i64 Kp, const double* __restrict__ C,
                                                         __bf16* __restrict__ CBh, __bf16* __restrict__ CBl,
                                                         float* __restrict__ cnf, double* __restrict__ cmax,
                                                         double mcoef, float* __restrict__ cnf2,
                                                         float* __restrict__ muf) {
  __shared__ double part[8][KB_DMAX];
  __shared__ float mus[KB_DMAX];
  __shared__ double red[16], redc[16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  for (int i = t; i < 8 * (int)D; i += 1024) {
    const int d = i % (int)D, g = i / (int)D;
    double m = 0.0;
    for (i64 c = g; c < K; c += 8) m += C[c * D + d];
    part[g][d] = m;
  }
  __syncthreads();
  if (t < D) {
    double m = 0.0;
    for (int g = 0; g < 8; ++g) m += part[g][t];
    mus[t] = (float)(m / (double)K);
    muf[t] = mus[t];
  }
  __syncthreads();
  double mx = 0.0, mdc = 0.0;
  for (i64 c = w; c < Kp; c += 16) {
    double s = 0.0, sm = 0.0, dc = 0.0;
    for (int d = lane; d < D; d += 64) {
      const double v = c < K ? C[c * D + d] - (double)mus[d] : 0.0;
      const float v32 = (float)v;
      const __bf16 hi = (__bf16)v32;
      const __bf16 lo = (__bf16)(v32 - (float)hi);
      CBh[c * D + d] = hi;
      CBl[c * D + d] = lo;
      // the screen's fp16 centre (staged as fp16(hi + lo)) against the fp32 c'
      const double e16 = (double)v32 - (double)(float)(_Float16)((float)hi + (float)lo);
      s += v * v;
      sm += (double)mus[d] * v;
      dc += e16 * e16;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      s += __shfl_xor(s, o, 64);
      sm += __shfl_xor(sm, o, 64);
      dc += __shfl_xor(dc, o, 64);
    }
    // padding centres: a huge FINITE cc (the filter tags a' mantissa bits,
    // which would turn +inf into NaN); they never win, and a lone real centre
    // is certified against them
    if (lane == 0) cnf[c] = c < K ? (float)(s + 2.0 * sm) : 3.0e38f;
    if (lane == 0) cnf2[c] = c < K ? (float)s : 3.0e38f;
    if (c < K) mx = (s > mx || s != s) ? s : mx;
    if (c < K) mdc = (dc > mdc || dc != dc) ? dc : mdc;
  }
  if (lane == 0) red[w] = mx;
  if (lane == 0) redc[w] = mdc;
  __syncthreads();
  if (t == 0) {
    double mc = redc[0];
    for (int k = 1; k < 16; ++k) mc = (redc[k] > mc || redc[k] != redc[k]) ? redc[k] : mc;
    cmax[3] = sqrt(mc) * 1.001;
    double m = red[0];
    for (int k = 1; k < 16; ++k) m = (red[k] > m || red[k] != red[k]) ? red[k] : m;
    double mn = 0.0;
    for (i64 d = 0; d < D; ++d) mn += (double)mus[d] * (double)mus[d];
    cmax[0] = sqrt(m) * 1.001;
    cmax[1] = mcoef;  // fp32 tie margin coefficient (0: fp64 distances), read by the filters
    cmax[2] = sqrt(mn) * 1.001;
  }
}

// The certified gap bound e of one point for the bf16x3 filters (a point is
// labelled iff b2 - b1 > 2e).  eS |p|: the bf16x3 product error of x.c'
// (split residuals, fp32 accumulation chains); 2.02 u (cmax^2 + 2|mu| cmax +
// |p| cmax): rounding of c' to fp32 (in x.c' and in |c'|^2) and of cc to
// fp32; the 1e-28 / 1e-8 terms: bf16 underflow and slack; 8 eps amax: the fp32
// fma a' = cc - 2S and the 3-bit tile tag; mcoef: the fp32-target tie margin
// over |x - c| <= |p| + |mu| + cmax.
__device__ __forceinline__ double kc_bound(double eS, double pn, double cmax, double mun, double pp2, double amax,
                                           double mcoef, i64 D) {
  const double u32 = 5.9604644775390625e-08;
  const double dm = pn + mun + cmax;
  return 2.0 * eS * pn + 2.02 * u32 * (cmax * cmax + 2.0 * mun * cmax + pn * cmax) +
         1e-28 * (double)D * (1.0 + cmax) * (1.0 + cmax) + 1e-8 * (pp2 + cmax * cmax + mun * mun) +
         8.0 * 1.1920928955078125e-07 * amax + 0.5 * mcoef * dm * dm + 1e-300;
}

// kc_bound as e(|p|) = k0 + k1 |p| + k2 |p|^2 (|p|^2 >= pp2), coefficients
// rounded up to fp32, for a per-row evaluation in fp32.
__device__ __forceinline__ void kc_coef(double eS, double cmax, double mun, double mcoef, i64 D, float (&k)[3],
                                        double xk1 = 0.0, double xk0 = 0.0) {
  const double u32 = 5.9604644775390625e-08, eps = 1.1920928955078125e-07;
  const double cm2 = cmax * cmax + 2.0 * mun * cmax, m = mun + cmax;
  const double k0 = 2.02 * u32 * cm2 + 1e-28 * (double)D * (1.0 + cmax) * (1.0 + cmax) +
                    1e-8 * (cmax * cmax + mun * mun) + 8.0 * eps * cm2 + 0.5 * mcoef * m * m + 1e-30 + xk0;
  const double k1 = 2.0 * eS + 2.02 * u32 * cmax + 16.0 * eps * cmax + mcoef * m + xk1;
  const double k2 = 1e-8 + 0.5 * mcoef;
  const double up = 1.0 + 2.384185791015625e-07;  // 2^-22: covers the rounding to fp32
  k[0] = (float)(k0 * up);
  k[1] = (float)(k1 * up);
  k[2] = (float)(k2 * up);
}

static size_t kb_lds_bytes(i64 D, int nct) { return (size_t)2 * 32 * nct * (D + 8) * 2 + (size_t)32 * nct * 4 + 4 * D; }

// Step (B) of the bf16x3 filter epilogue, as a function (tools/perm_probe.hip
// checks it against a brute-force top-2).
__device__ __forceinline__ void kb_top2_lanes(float (&lo)[16], float (&sec)[16], int (&li)[16], int lane) {
    // (B) across the 32 lanes of each half, halving the registers per lane at
  // every step: a lane keeps the half its lane bit picks and receives the
  // partner's copy of it.  Partners differ in the step's lane bit and agree
  // on the bits already processed, which is all a min-reduction over the
  // 32 centres needs: bit 4 by ds_swizzle (lane ^ 16), bits 3 / 2 / 1 / 0 by
  // DPP row_mirror (lane ^ 15), row_half_mirror (^ 7), quad_perm ^ 2 and ^ 1
  // -- VALU moves instead of ds_bpermute round trips (tools/perm_probe.hip,
  // tools/top2_probe.hip).
  // Lane (h, r) ends with register q = r >> 1, i.e. row rt(q, h), over all
  // centres.  A (value, index) pair combines to the smaller value, the
  // lower index on equal values.
  auto comb = [](float a, int ai, float as, float b, int bi, float bs, float& l, int& li2, float& s2) {
    s2 = __builtin_amdgcn_fmed3f(a, b, fminf(as, bs));
    li2 = (b < a || (b == a && bi < ai)) ? bi : ai;
    l = fminf(a, b);
  };
  // bit 4: ds_swizzle (bit mode, xor 16 within each 32-lane half; no address
  // operand, no memory access).  v_permlane16_swap would do it in one VALU
  // op, but the compiler folded its two results into one (tools/top2_probe).
  auto xor16 = [](int v) { return __builtin_amdgcn_ds_swizzle(v, 0x401F); };
  {
    const bool up = (lane & 16) != 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float kl = up ? lo[k + 8] : lo[k], ks2 = up ? sec[k + 8] : sec[k];
      const int ki = up ? li[k + 8] : li[k];
      const float sl = up ? lo[k] : lo[k + 8], ss = up ? sec[k] : sec[k + 8];
      const int si = up ? li[k] : li[k + 8];
      comb(kl, ki, ks2, __builtin_bit_cast(float, xor16(__builtin_bit_cast(int, sl))), xor16(si),
           __builtin_bit_cast(float, xor16(__builtin_bit_cast(int, ss))), lo[k], li[k], sec[k]);
    }
  }
  auto dpp_step = [&](auto ctrl, int n, int o) {
    constexpr int C = decltype(ctrl)::value;
    const bool up = (lane & o) != 0;
#pragma unroll
    for (int k = 0; k < n; ++k) {
      const float kl = up ? lo[k + n] : lo[k], ks2 = up ? sec[k + n] : sec[k];
      const int ki = up ? li[k + n] : li[k];
      const float sl = up ? lo[k] : lo[k + n], ss = up ? sec[k] : sec[k + n];
      const int si = up ? li[k] : li[k + n];
      const float ol = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, sl), C, 0xF, 0xF, false));
      const float os = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, ss), C, 0xF, 0xF, false));
      const int oi = __builtin_amdgcn_update_dpp(0, si, C, 0xF, 0xF, false);
      comb(kl, ki, ks2, ol, oi, os, lo[k], li[k], sec[k]);
    }
  };
  dpp_step(std::integral_constant<int, 0x140>{}, 4, 8);  // row_mirror: lane ^ 15
  dpp_step(std::integral_constant<int, 0x141>{}, 2, 4);  // row_half_mirror: lane ^ 7
  dpp_step(std::integral_constant<int, 0x4E>{}, 1, 2);   // quad_perm [2,3,0,1]: lane ^ 2
  {
    const float ol = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, lo[0]), 0xB1, 0xF, 0xF, false));
    const float os = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, sec[0]), 0xB1, 0xF, 0xF, false));
    const int oi = __builtin_amdgcn_update_dpp(0, li[0], 0xB1, 0xF, 0xF, false);
    comb(lo[0], li[0], sec[0], ol, oi, os, lo[0], li[0], sec[0]);
  }
}

template <int NCT>
__global__ __launch_bounds__(KB_WAVES * 64) void k_kmeans_filter_b3(i64 N, i64 D, const float* __restrict__ P, i64 ldp,
                                                                    const __bf16* __restrict__ CBh,
                                                                    const __bf16* __restrict__ CBl,
                                                                    const float* __restrict__ cnf, const double* cmax_p,
                                                                    i64* __restrict__ labels,
                                                                    unsigned int* __restrict__ counters,
                                                                    i64* __restrict__ full_list,
                                                                    KfCand* __restrict__ cand_list,
                                                                    const i64* __restrict__ rows_in,
                                                                    const unsigned int* __restrict__ nrows_in,
                                                                    const float* __restrict__ muf) {
  // rows_in != NULL (list mode): only the *nrows_in points rows_in[0..n) --
  // the rows the A-stationary filter left undecided; slot s of the list plays
  // the role of row s below.  The points are centred like the centres (x' =
  // fl(x - mu), mu = muf in LDS): a' = |c'|^2 - 2 x'.c' (cnf = cnf2 of the
  // prep), so the bound and the candidate masks scale with |x'|, not |x|.
  extern __shared__ __attribute__((aligned(16))) unsigned char kb_lds[];
  constexpr int NC = 32 * NCT;
  const int Dp = (int)D + 8;
  __bf16* Bh = (__bf16*)kb_lds;
  __bf16* Bl = Bh + NC * Dp;
  float* cns = (float*)(Bl + NC * Dp);
  float* mul = cns + NC;  // mu in the row's dim order
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, r = lane & 31, h = lane >> 5;
  {
    // k-order inside every 16-dim step is permuted (dim quads 1 and 2
    // swapped) so that an A lane's two 16-byte loads are adjacent in its row
    // (lane h takes dims 4h..4h+3 and 8+4h..8+4h+3): the B rows are stored in
    // the same order, so the dot products are unchanged up to summation order
    typedef unsigned int kb_u2 __attribute__((ext_vector_type(2)));
    const int D4 = (int)D / 4;
    for (int i = t; i < NC * D4; i += KB_WAVES * 64) {
      const int c = i / D4, q = i % D4, qi = q & 3;
      const int pq = (q & ~3) | (qi == 1 ? 2 : qi == 2 ? 1 : qi);
      *(kb_u2*)&Bh[c * Dp + 4 * pq] = *(const kb_u2*)&CBh[(i64)c * D + 4 * q];
      *(kb_u2*)&Bl[c * Dp + 4 * pq] = *(const kb_u2*)&CBl[(i64)c * D + 4 * q];
    }
    for (int i = t; i < NC; i += KB_WAVES * 64) cns[i] = cnf[i];
    for (int i = t; i < (int)D; i += KB_WAVES * 64) mul[i] = muf[i];
  }
  __syncthreads();
  float cnr[NCT];  // |c|^2 of this lane's centre in every tile
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) cnr[ct] = cns[ct * 32 + r];
  const double cmax = cmax_p[0];
  // fp32 target: two exact distances whose squares differ by more than
  // 2^-21 (|p| + |c|)^2 are more than 2 fp32 ulps apart, so they cannot
  // round to one value; the margin is folded into e (gap > 2e + margin)
  const double mcoef = cmax_p[1], mun = cmax_p[2];
  const double u32 = 5.9604644775390625e-08;
  const int KS = (int)D / 16;
  // chain length of one accumulator: the 48 KB_GRP products of a group go
  // into a fresh accumulator, small cross terms first (32 KB_GRP additions of
  // partial sums <= 2 * 2^-8 * 1.004 |x'| cmax, then 16 KB_GRP of <= 1.016
  // |x'| cmax: within 16.5 KB_GRP of |x'| cmax), then KS / KB_GRP adds
  const double chain = 16.5 * KB_GRP + (double)(KS / KB_GRP);
  // (one u cmax per |x'| for x' = fl(x - mu))
  const double eS = (2.0 * u32 + 3.1 * 3.814697265625e-06 + 2.0 * (chain + 3.0) * u32) * 1.01 * cmax;
  const i64 nslots = rows_in ? (i64)*nrows_in : N;
  if (nslots == 0) return;
  const i64 ntiles = (nslots + 31) / 32;
  const i64 stride = (i64)gridDim.x * KB_WAVES;
  i64 tile = (i64)blockIdx.x * KB_WAVES + w;
  auto row_of = [&](i64 slot) -> i64 {
    slot = slot < nslots ? slot : nslots - 1;
    return rows_in ? rows_in[slot] : slot;
  };
  // A ring: 4 k-steps in flight, addresses clamped into the array
  kb_f4 ra[4][2];
  auto load = [&](int s, i64 tl, int ks) {
    const i64 row = row_of(tl * 32 + r);
    const float* p = P + row * ldp + ks * 16 + 4 * h;
    ra[s][0] = *(const kb_f4*)p;  // dims 4h..4h+3 (nt measured no faster here)
    ra[s][1] = *(const kb_f4*)(p + 8);  // dims 8+4h..8+4h+3
  };
#pragma unroll
  for (int s = 0; s < 4; ++s) load(s, tile, s);
  for (; tile < ntiles; tile += stride) {
    kb_acc acc[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) acc[ct] = (kb_acc){};
    float p2 = 0.f;
    for (int ks0 = 0; ks0 < KS; ks0 += 4) {
#pragma unroll
      for (int g0 = 0; g0 < 4; g0 += KB_GRP) {
        kb_bf8 ah[KB_GRP], al[KB_GRP];
#pragma unroll
        for (int g = 0; g < KB_GRP; ++g) {
          const int s = g0 + g, ks = ks0 + s;
          float x[8];
          const kb_f4 m0 = *(const kb_f4*)(mul + ks * 16 + 4 * h), m1 = *(const kb_f4*)(mul + ks * 16 + 8 + 4 * h);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            x[j] = ra[s][0][j] - m0[j];
            x[j + 4] = ra[s][1][j] - m1[j];
          }
          {
            int nks = ks + 4;
            i64 ntl = tile;
            if (nks >= KS) {
              nks -= KS;
              ntl += stride;
            }
            load(s, ntl, nks);
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            p2 += x[j] * x[j];
            ah[g][j] = (__bf16)x[j];
            al[g][j] = (__bf16)(x[j] - (float)ah[g][j]);
          }
        }
        // B fragments of tile ct + 1 are read while tile ct's MFMAs run (one
        // wave per SIMD: an LDS read right before its MFMA exposes its latency)
        kb_bf8 bh[2][KB_GRP], bl[2][KB_GRP];
        auto bload = [&](int buf, int ct) {
#pragma unroll
          for (int g = 0; g < KB_GRP; ++g) {
            const int ko = (ks0 + g0 + g) * 16 + 8 * h;
            bh[buf][g] = *(const kb_bf8*)&Bh[(ct * 32 + r) * Dp + ko];
            bl[buf][g] = *(const kb_bf8*)&Bl[(ct * 32 + r) * Dp + ko];
          }
        };
        bload(0, 0);
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) {
          if (ct + 1 < NCT) bload((ct + 1) & 1, ct + 1);
          // the 48 KB_GRP products per output of KB_GRP k-steps go into a
          // fresh accumulator that is then added to the running sum: the
          // rounding bound is that chain + D / (16 KB_GRP) adds instead of
          // one 3D-long chain
          // (the small cross terms of the group first, then its xh.ch terms:
          // only those 16 KB_GRP additions see partial sums of size |x'| cmax)
          kb_acc tk = (kb_acc){};
#pragma unroll
          for (int g = 0; g < KB_GRP; ++g) {
            tk = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[g], bl[ct & 1][g], tk, 0, 0, 0);
            tk = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[g], bh[ct & 1][g], tk, 0, 0, 0);
          }
#pragma unroll
          for (int g = 0; g < KB_GRP; ++g) tk = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[g], bh[ct & 1][g], tk, 0, 0, 0);
          acc[ct] += tk;
        }
      }
    }
    p2 += __shfl_xor(p2, 32, 64);  // row r's |p|^2 in lanes r and r + 32
    // ---- epilogue.  Register reg of tile ct holds S(row rt(reg, h), centre
    // 32 ct + r), rt = (reg&3) + 8(reg>>2) + 4h.
    // (A) per register: a' = fl(|c|^2 - 2S) with the tile index ct written
    // into the 3 low mantissa bits (a <= 7-ulp perturbation, priced into the
    // bound below; the exact winner only matters once the gap certifies it),
    // then the two smallest over the NCT tiles by a min / med3 network.
    float lo[16], sec[16];
    int li[16];
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      float v[NCT];
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        const float a = __builtin_fmaf(-2.f, acc[ct][reg], cnr[ct]);
        v[ct] = __builtin_bit_cast(float, (__builtin_bit_cast(unsigned int, a) & ~7u) | (unsigned int)ct);
      }
      float l = v[0], s2 = INFINITY;
      if constexpr (NCT >= 2) {
        float pl[NCT / 2], ps[NCT / 2];
#pragma unroll
        for (int k = 0; k < NCT / 2; ++k) {
          pl[k] = fminf(v[2 * k], v[2 * k + 1]);
          ps[k] = fmaxf(v[2 * k], v[2 * k + 1]);
        }
#pragma unroll
        for (int n = NCT / 2; n > 1; n >>= 1) {
#pragma unroll
          for (int k = 0; k < n / 2; ++k) {
            const float a0 = pl[2 * k], a1 = pl[2 * k + 1];
            ps[k] = __builtin_amdgcn_fmed3f(a0, a1, fminf(ps[2 * k], ps[2 * k + 1]));
            pl[k] = fminf(a0, a1);
          }
        }
        l = pl[0];
        s2 = ps[0];
      }
      lo[reg] = l;
      sec[reg] = s2;
      li[reg] = r;
    }
    kb_top2_lanes(lo, sec, li, lane);
    // (C) one decision per row, by the even lane of its pair
    const int q = r >> 1;
    const int rt = (q & 3) + 8 * (q >> 2) + 4 * h;
    const i64 gslot = tile * 32 + rt;
    const i64 grow = row_of(gslot);
    const float b1 = lo[0], b2 = sec[0];
    const int i1 = 32 * (int)(__builtin_bit_cast(unsigned int, b1) & 7u) + li[0];
    const float p2f = __shfl(p2, rt, 64);
    const double pp2 = (double)p2f * 1.001 + (double)D * 2e-45;
    const double pn = sqrt(pp2) * 1.0001;
    // |a'| <= amax = cmax^2 + 2 |mu| cmax + 2 |p| cmax: the 7-ulp index tag
    // adds 2 * 8 * 2^-23 of that to the gap test
    const double amax = cmax * cmax + 2.0 * mun * cmax + 2.0 * pn * cmax;
    const double e = kc_bound(eS, pn, cmax, mun, pp2, amax, mcoef, D);
    const bool live = gslot < nslots && (r & 1) == 0;
    // finite point, no overflow possible in S or a' (every a' then finite)
    const bool fin = isfinite(p2f) && isfinite(e) && pn * cmax < 1e36 && cmax * cmax < 1e36 &&
                     mun * cmax < 1e36 && isfinite(b1) && isfinite(b2);
    const bool dec = fin && (double)b2 - (double)b1 > 2.0 * e;
    if (live && dec) km_label(labels, counters, grow, i1);
    if (live && !fin) full_list[atomicAdd(&counters[0], 1u)] = grow;
    // undecided rows: one slot each (one atomic per wave), then per register
    // q holding such a row, the masks of the centres with a' <= b1 + 2e by
    // ballots (e prices the index tags in: every centre that can be the
    // exact argmin is kept)
    const bool needc = live && fin && !dec;
    const unsigned long long und = __ballot(needc);
    if (und) {  // wave-uniform
      unsigned int base = 0;
      if (lane == 0) base = atomicAdd(&counters[1], (unsigned int)__popcll(und));
      base = __builtin_amdgcn_readfirstlane(base);
      const unsigned int myslot = base + (unsigned int)__popcll(und & ((1ull << lane) - 1ull));
      if (needc) cand_list[myslot].row = grow;
      const double thr = (double)b1 + 2.0 * e;
#pragma unroll
      for (int qq = 0; qq < 16; ++qq) {
        const bool n0 = (und >> (2 * qq)) & 1ull, n1 = (und >> (32 + 2 * qq)) & 1ull;
        if (n0 || n1) {  // wave-uniform
          const double tq = __shfl(thr, 2 * qq + 32 * h, 64);
          const unsigned int s0 = __builtin_amdgcn_readlane(myslot, 2 * qq);
          const unsigned int s1 = __builtin_amdgcn_readlane(myslot, 32 + 2 * qq);
          // the 8 mask words of both rows are moved into lanes 0-7 / 32-39
          // and written by ONE store (was 16 single-lane stores per register)
          unsigned int mw = 0;
#pragma unroll
          for (int ct = 0; ct < 8; ++ct) {
            unsigned long long m = 0;
            if (ct < NCT) {
              const float a = __builtin_fmaf(-2.f, acc[ct < NCT ? ct : 0][qq], cnr[ct < NCT ? ct : 0]);
              m = __ballot((double)a <= tq);
            }
            mw = lane == ct ? (unsigned int)m : lane == 32 + ct ? (unsigned int)(m >> 32) : mw;
          }
          if ((r < 8) && (h ? n1 : n0)) cand_list[h ? s1 : s0].mask[r] = mw;
        }
      }
    }
  }
}

template <int NCT>
static void kb_launch(hipStream_t s, i64 N, i64 D, const float* P, i64 ldp, const __bf16* CBh, const __bf16* CBl,
                      const float* cnf, const double* cmax, i64* labels, unsigned int* counters, i64* full_list,
                      KfCand* cand_list, int grid, const i64* rows_in, const unsigned int* nrows_in,
                      const float* muf) {
  const size_t lds = kb_lds_bytes(D, NCT);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_kmeans_filter_b3<NCT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)kb_lds_bytes(KB_DMAX, 8));
    attr = true;
  }
  k_kmeans_filter_b3<NCT><<<grid, KB_WAVES * 64, lds, s>>>(N, D, P, ldp, CBh, CBl, cnf, cmax, labels, counters,
                                                           full_list, cand_list, rows_in, nrows_in, muf);
}

// ---------------------------------------------------------------------------
// A-stationary bf16x3 filter: the fast first pass of the certified
// assignment (same bf16 split, same rigorous bound e and same decision rule
// a point is labelled iff b2 - b1 > 2e as k_kmeans_filter_b3 above).
// k_kmeans_filter_b3 keeps all NCT accumulator tiles (128 registers) live so
// that it can emit candidate masks, which forces one wave per SIMD (no
// partner to cover the A loads or the epilogue, which follows all 192
// MFMAs).  Here a wave instead holds its 32-point tile as the bf16 split for
// the whole centre sweep (8 KS registers) and sweeps the centre tiles one at
// a time: 3 KS MFMAs into two accumulator chains of KS / 2 k-steps each
// (added once: the fresh-accumulator bound with G = KS / 2), then the tile's
// a' = fl(|c|^2 - 2S), tagged with ct in its 3 low mantissa bits, are folded
// into a per-lane running top-2 (fma, and-or, med3, min per value), so the
// epilogue work sits between MFMAs instead of after all of them.  The next
// point tile's loads are issued right after the split, into the registers
// the split just freed, and land during the sweep.  ~230 registers: two
// waves per SIMD, 8 waves per block, one block per CU (the split centres,
// 137 KiB for K = 256, D = 128, stay resident in LDS).  Undecided rows
// (near-ties, ~1-3 %) go to a row list; the list-mode run of
// k_kmeans_filter_b3 gives them candidate masks (k_kmeans_cand then
// recomputes the candidates in scipy's exact order); non-finite rows go to
// the all-centre exact kernel as before.
// Waves per block (one block per CU): 8 = two per SIMD (<= 256 registers),
// for both the bf16x3 filter and the fp16 screen (MODE 1).  Measured and not
// kept: one or three waves per SIMD, a next-tile prefetch, the
// |x'|^2 fmas pinned after the split, an unpipelined sweep.
constexpr int KS_WAVES = 8;
__host__ __device__ constexpr int ks_waves(int) { return KS_WAVES; }

// LDS row of centre c: [hi: D bf16][lo: D bf16][-cc/2 as 3 bf16 + 5 zeros]
// [8 zero bf16][16-byte pad]; the row stride is 4 D + 48 bytes = 12 (mod 64)
// banks, so the 16-lane groups of a ds_read_b128 (rows 0-3, 12-15, 20-27 ...)
// hit 16 distinct 4-bank quads, and every read of a tile's k-loop is one base
// register + an immediate.
// MODE 1 (the fp16 screen below): [hi: D fp16][-cc/2 as 3 bf16 + 5 zeros][8
// zero bf16][16-byte pad], 2 D + 48 bytes: also an odd multiple of 4 banks
// for D = 64 and 128, so conflict-free the same way.
__host__ __device__ constexpr int ks_row_bytes(int D, int mode = 0) { return (mode == 0 ? 4 : 2) * D + 48; }
// (then the D fp32 centre mean, which both modes subtract from the points)
static size_t ks_lds_bytes(i64 D, int nct, int mode = 0) {
  return (size_t)32 * nct * ks_row_bytes((int)D, mode) + 4 * D;
}
typedef _Float16 kh_f8 __attribute__((ext_vector_type(8)));

// Plain v_med3_f32 / v_max_f32: fmaxf / fmed3 on values built by bit
// operations make the compiler canonicalize every operand first (a v_max_f32
// x, x each), which doubled the per-value epilogue here.  The operands are
// finite or -inf (non-finite points are routed by the |p|^2 / cmax checks
// before any of these values is used) and never a fresh MFMA result (inline
// asm gets no MFMA -> VALU wait states from the hazard recognizer).
__device__ __forceinline__ float ks_med3(float a, float b, float c) {
  float r;
  asm("v_med3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float ks_max(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float ks_max3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
// (bits(a) & ~7) | ct, ct < 8 (a centre tile; uniform).  Plain C, not inline
// asm: its operand comes straight from an MFMA accumulator, and only
// compiler-generated instructions get the MFMA -> VALU read wait states from
// the hazard recognizer (an asm v_and_or_b32 there read stale accumulators:
// ~5 % wrong labels, caught by the exact-kernel comparison).  The empty asm
// hides ct's range from the compiler: with ct known < 8 it proved the or
// disjoint and emitted v_and + v_add (two VALU per value) instead of one
// v_and_or_b32.
__device__ __forceinline__ float ks_tag(float a, unsigned int ct) {
  asm("" : "+s"(ct));
  return __builtin_bit_cast(float, (__builtin_bit_cast(unsigned int, a) & ~7u) | ct);
}

// Top-2 (largest) VALUES across the 32 lanes of each half (register halving
// as in kb_top2_lanes, without carrying an index: the best lane is found
// afterwards by one ballot per row).  Lane (h, r) ends with register 0 =
// row rt(r >> 1, h) over all 32 centres of every tile.
__device__ __forceinline__ void ks_top2_vals(float (&lo)[16], float (&sec)[16], int lane) {
  auto comb = [](float a, float as, float b, float bs, float& l, float& s2) {
    s2 = ks_med3(a, b, ks_max(as, bs));
    l = ks_max(a, b);
  };
  auto xor16 = [](float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, v), 0x401F));
  };
  {
    const bool up = (lane & 16) != 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float kl = up ? lo[k + 8] : lo[k], ks2 = up ? sec[k + 8] : sec[k];
      const float sl = up ? lo[k] : lo[k + 8], ss = up ? sec[k] : sec[k + 8];
      comb(kl, ks2, xor16(sl), xor16(ss), lo[k], sec[k]);
    }
  }
  auto dpp_step = [&](auto ctrl, int n, int o) {
    constexpr int C = decltype(ctrl)::value;
    const bool up = (lane & o) != 0;
#pragma unroll
    for (int k = 0; k < n; ++k) {
      const float kl = up ? lo[k + n] : lo[k], ks2 = up ? sec[k + n] : sec[k];
      const float sl = up ? lo[k] : lo[k + n], ss = up ? sec[k] : sec[k + n];
      const float ol = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, sl), C, 0xF, 0xF, false));
      const float os = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, ss), C, 0xF, 0xF, false));
      comb(kl, ks2, ol, os, lo[k], sec[k]);
    }
  };
  dpp_step(std::integral_constant<int, 0x140>{}, 4, 8);  // row_mirror: lane ^ 15
  dpp_step(std::integral_constant<int, 0x141>{}, 2, 4);  // row_half_mirror: lane ^ 7
  dpp_step(std::integral_constant<int, 0x4E>{}, 1, 2);   // quad_perm [2,3,0,1]: lane ^ 2
  {
    const float ol = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, lo[0]), 0xB1, 0xF, 0xF, false));
    const float os = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, sec[0]), 0xB1, 0xF, 0xF, false));
    comb(lo[0], sec[0], ol, os, lo[0], sec[0]);
  }
}

// f(integral_constant<int, Q>) for every Q of the sequence (compile-time Q)
template <typename F, int... Q>
__device__ __forceinline__ void ks_unroll(F&& f, std::integer_sequence<int, Q...>) {
  (f(std::integral_constant<int, Q>{}), ...);
}

// MODE 0: the bf16x3 filter described above.  MODE 1: the fp16 screen -- the
// same sweep with ONE v_mfma_f32_32x32x16_f16 per k-step, a third of the
// MFMAs and no lo split.  The screen centres the points too: it ranks by
// a'' = |c'|^2 - 2 x'.c' with x' = fl(x - mu) (= |x - c|^2 - |x - mu|^2 up
// to the roundings priced below), so its error scales with |x - mu| instead
// of |x|; x' and c' are rounded to fp16 (11 significant bits): x' within
// 2^-11 |x'| (+ 2^-25 per component below the fp16 normal range), c' within
// the measured dcmax = max_c |c' - fp16(c')| (k_kmeans_prep_b3).  Its bound
// is still several times bf16x3's, so a few % of cfg3's rows stay
// undecided; they go to a row list that the MODE 0 kernel re-runs in list
// mode (rows_in / nrows_in: slot s of the list plays the role of row s).
// In MODE 1 rows the screen cannot evaluate (non-finite values, fp16
// overflow, cmax beyond the fp16 range) are undecided too: the MODE 0 pass
// routes them.  cnf is |c'|^2 (cnf2 of the prep) in MODE 1.
template <int NCT, int KS, int MODE>
__global__ __launch_bounds__(ks_waves(MODE) * 64) void k_kmeans_filter_as(i64 N, const float* __restrict__ P, i64 ldp,
                                                                    const __bf16* __restrict__ CBh,
                                                                    const __bf16* __restrict__ CBl,
                                                                    const float* __restrict__ cnf,
                                                                    const double* cmax_p, i64* __restrict__ labels,
                                                                    unsigned int* __restrict__ counters,
                                                                    i64* __restrict__ full_list,
                                                                    unsigned long long* __restrict__ und_mask,
                                                                    const i64* __restrict__ rows_in,
                                                                    const unsigned int* __restrict__ nrows_in,
                                                                    const float* __restrict__ muf) {
  extern __shared__ __attribute__((aligned(16))) unsigned char kb_lds[];
  // the screen always runs over every row: no list lookups in its code (a
  // run-time-null list still cost a guarded load and a vmcnt(0) per tile)
  if constexpr (MODE == 1) rows_in = nullptr;
  constexpr int NC = 32 * NCT, D = 16 * KS, RB = ks_row_bytes(D, MODE);
  constexpr int CCOFF = MODE == 0 ? 4 * D : 2 * D;  // byte offset of the -cc/2 pieces in a row
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, r = lane & 31, h = lane >> 5;
  {
    // centre rows in the permuted k order of k_kmeans_filter_b3 (dim quads
    // 1 and 2 of every 16-dim step swapped: an A lane's two 16-byte loads
    // are adjacent in its row)
    typedef unsigned int kb_u2 __attribute__((ext_vector_type(2)));
    typedef __bf16 kb_b4 __attribute__((ext_vector_type(4)));
    typedef _Float16 kh_f4 __attribute__((ext_vector_type(4)));
    constexpr int D4 = D / 4;
    for (int i = t; i < NC * D4; i += ks_waves(MODE) * 64) {
      const int c = i / D4, q = i % D4, qi = q & 3;
      const int pq = (q & ~3) | (qi == 1 ? 2 : qi == 2 ? 1 : qi);
      unsigned char* row = kb_lds + c * RB;
      if constexpr (MODE == 0) {
        *(kb_u2*)(row + 8 * pq) = *(const kb_u2*)&CBh[(i64)c * D + 4 * q];
        *(kb_u2*)(row + 2 * D + 8 * pq) = *(const kb_u2*)&CBl[(i64)c * D + 4 * q];
      } else {
        // fp16(hi + lo): hi + lo is c' to 2^-16 (priced in the bound)
        const kb_b4 bh = *(const kb_b4*)&CBh[(i64)c * D + 4 * q];
        const kb_b4 bl = *(const kb_b4*)&CBl[(i64)c * D + 4 * q];
        kh_f4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = (_Float16)((float)bh[j] + (float)bl[j]);
        *(kh_f4*)(row + 8 * pq) = v;
      }
    }
    // -cc/2 split exactly into three bf16 (8 + 8 + 8 significant bits of
    // the fp32 value), for the k-step that adds it on the MFMA (lanes of the
    // upper half read the zeros next to it)
    for (int i = t; i < NC; i += ks_waves(MODE) * 64) {
      const float v = -0.5f * cnf[i];
      const __bf16 b1 = (__bf16)v;
      const float v1 = v - (float)b1;
      const __bf16 b2 = (__bf16)v1;
      const __bf16 b3 = (__bf16)(v1 - (float)b2);
      const __bf16 z = (__bf16)0.f;
      unsigned char* row = kb_lds + i * RB;
      *(kb_bf8*)(row + CCOFF) = (kb_bf8){b1, b2, b3, z, z, z, z, z};
      *(kb_bf8*)(row + CCOFF + 16) = (kb_bf8){z, z, z, z, z, z, z, z};
    }
    {
      float* mul = (float*)(kb_lds + NC * RB);
      for (int i = t; i < D; i += ks_waves(MODE) * 64) mul[i] = muf[i];
    }
  }
  __syncthreads();
  const double cmax = cmax_p[0];
  // fp32 target: two exact distances whose squares differ by more than
  // 2^-21 (|p| + |c|)^2 are more than 2 fp32 ulps apart, so they cannot
  // round to one value; the margin is folded into e (gap > 2e + margin)
  const double mcoef = cmax_p[1], mun = cmax_p[2];
  const double u32 = 5.9604644775390625e-08;
  // one accumulator chain: 48 (bf16x3) or 16 (fp16) products per k-step
  // over KS k-steps
  // (MODE 0: the two-phase chain below -- 32 KS additions of partial sums
  // <= 2 * 2^-8 * 1.004 |x'| cmax, then 16 KS of <= 1.016 |x'| cmax, within
  // 16.5 KS additions of |x'| cmax, and the 1.01 factor of eS covers the rest)
  const double chain = (MODE == 0 ? 16.5 : 16.0) * (double)KS;
  // error of x'.c' per |x'| (both modes centre the points, x' = fl(x - mu),
  // u cmax): bf16x3 (u + u + 3.1 * 2^-18 + chain) cmax.  fp16
  // screen: u cmax (x') + 2^-11 cmax (x' to fp16) +
  // 1.001 dcmax (c' to fp16, measured) + the chain over |xh| |ch| <=
  // 1.001 |x'| (cmax + dcmax)
  const double dcmax = MODE == 1 ? cmax_p[3] : 0.0;
  const double eS = MODE == 0 ? (2.0 * u32 + 3.1 * 3.814697265625e-06 + 2.0 * (chain + 3.0) * u32) * 1.01 * cmax
                              : (u32 * cmax + 4.8828125e-04 * cmax + 1.001 * dcmax +
                                 2.0 * (chain + 3.0) * u32 * 1.001 * (cmax + dcmax)) * 1.01;
  float kq[3];
  // the chain ends with one MFMA that adds -cc/2 (three nonzero products):
  // its roundings, at most 16 of <= 2u |S - cc/2 + ...| each, priced in a'
  // units as 64u |p| cmax + 32u (cmax^2 + 2|mu| cmax); the fma a' = cc - 2S
  // is gone, and the tile tag on the accumulator (7 ulp of |S - cc/2|, i.e.
  // 14 eps (|p| cmax + cm2 / 2) in a' units) stays inside kc_coef's 8 eps amax.
  // fp16 underflow of x' (MODE 1): each rounded component is off by at most
  // 2^-25 absolute besides the relative 2^-11, i.e. 2^-25 sqrt(D) (cmax +
  // dcmax) + D 2^-50 on S (dcmax already holds the centres' underflow),
  // doubled in a'' units with slack.  The a'' form (|c'|^2 instead of cc)
  // and |x - c| <= |x'| + cmax keep every other term of kc_coef an upper
  // bound with |p| = |x'|.
  double xk1 = 64.0 * u32 * cmax, xk0 = 32.0 * u32 * (cmax * cmax + 2.0 * mun * cmax);
  if constexpr (MODE == 1)
    xk0 += sqrt((double)D) * 1.1920928955078125e-07 * (cmax + dcmax) + (double)D * 3.552713678800501e-15;
  kc_coef(eS, cmax, mun, mcoef, D, kq, xk1, xk0);
  // no overflow in S or a' (every a' finite): |p| cmax, cmax^2, |mu| cmax < 1e36;
  // MODE 1: every fp16 centre component finite (|c'_d| <= cmax < 3e4)
  const bool cok = cmax * cmax < 1e36 && mun * cmax < 1e36 && (MODE == 0 || (cmax < 3.0e4 && dcmax == dcmax));
  const float pn_lim = (float)(cmax > 0.0 ? 1e36 / cmax : 1e36);
  // list mode: slot s < nrows stands for row rows_in[s]
  const i64 nlim = rows_in ? (i64)*nrows_in : N;
  const i64 ntiles = (nlim + 31) / 32;
  const i64 stride = (i64)gridDim.x * ks_waves(MODE);
  i64 tile = (i64)blockIdx.x * ks_waves(MODE) + w;
  kb_f4 ra[KS][2];
  // the point row lane (r, h) loads for tile tl (list mode: a gather through rows_in)
  constexpr bool LPF = MODE == 0;  // (MODE 0 runs in list mode only: rows_in is never null)
  auto lrow = [&](i64 tl) __attribute__((always_inline)) {
    i64 row = tl * 32 + r;
    row = row < nlim ? row : nlim - 1;
    if constexpr (LPF) return rows_in[row];
    else return rows_in ? rows_in[row] : row;
  };
  auto load_row = [&](i64 row) __attribute__((always_inline)) {
    const float* p = P + row * ldp + 4 * h;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      ra[ks][0] = *(const kb_f4*)(p + ks * 16);      // dims 4h..4h+3 of the k-step
      ra[ks][1] = *(const kb_f4*)(p + ks * 16 + 8);  // dims 8+4h..8+4h+3
    }
  };
  // list mode (LPF): the gather's two dependent loads (the row index, then
  // the row) were issued at the top of each tile, and with two waves per
  // SIMD the partner's sweep did not cover both latencies (the list pass ran
  // at ~47 % of its MFMA time).  Now the next tile's row indices are loaded
  // a whole tile ahead, its rows right after this tile's sweep (the split's
  // registers are free again: |x'|^2 is pinned at the split) so that they
  // land during the decision, and the decision's own row index (rows_in of
  // its slot) at the top of the tile.  The screen (MODE 1) streams every row
  // in order and keeps the measured top-of-tile load.
  // Every load of the loop is unconditional (clamped to a valid row), so
  // the compiler's count of outstanding loads is the same on every path and
  // its waits stay partial: per tile, in issue order, the decision's row
  // index (top), then after the sweep the row indices of the tile after
  // next, the decided rows' old label codes and the next tile's rows.
  const int qd = r >> 1, rtd = (qd & 3) + 8 * (qd >> 2) + 4 * h;  // the decision lanes' row in the tile
  i64 nrow = 0;
  KmMove mv{nullptr, nullptr, nullptr};
  if constexpr (LPF) {
    mv = *(const KmMove*)(counters + 4);
    if (tile < ntiles) {
      load_row(lrow(tile));
      nrow = lrow(tile + stride);
    }
  }
  for (; tile < ntiles; tile += stride) {
    if constexpr (!LPF) load_row(lrow(tile));  // the partner wave's sweep covers the latency
    i64 grow_pf = 0;
    if constexpr (LPF) {
      const i64 sl = tile * 32 + rtd;
      const i64 slc = sl < nlim ? sl : nlim - 1;
      grow_pf = rows_in[slc];
    }
    using AT = std::conditional_t<MODE == 0, kb_bf8, kh_f8>;
    AT ah[KS];
    kb_bf8 al[MODE == 0 ? KS : 1];
    // |p|^2 only feeds the bound (x 1.001 slack): four independent partial
    // chains instead of one 64-deep dependent fma chain
    float p2q[4] = {0.f, 0.f, 0.f, 0.f};
    {  // x' = x - mu, mu read from LDS in the lane's dim order
      const float* mul = (const float*)(kb_lds + NC * RB) + 4 * h;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        ra[ks][0] -= *(const kb_f4*)(mul + ks * 16);
        ra[ks][1] -= *(const kb_f4*)(mul + ks * 16 + 8);
      }
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x = j < 4 ? ra[ks][0][j] : ra[ks][1][j - 4];
        p2q[j & 3] = __builtin_fmaf(x, x, p2q[j & 3]);
        if constexpr (MODE == 0) {
          ah[ks][j] = (__bf16)x;
          al[ks][j] = (__bf16)(x - (float)ah[ks][j]);
        } else {
          ah[ks][j] = (_Float16)x;
        }
      }
    }
    float p2 = (p2q[0] + p2q[1]) + (p2q[2] + p2q[3]);
    // (the compiler sinks the 64 |p|^2 fmas to the decision, keeping the raw
    // tile live through the sweep; pinning them here frees 47 registers but
    // measured 2 % slower for the screen, gpurun_out ksv4; the list pass pins
    // them: its next tile's rows land in those registers)
    if constexpr (LPF) {
      asm volatile("" : "+v"(p2));
      __builtin_amdgcn_sched_barrier(0);
    }
    // running top-2 of acc = S - cc/2 = -a'/2 (the best centre has the
    // LARGEST acc); lo / sec keep their names from the a' form
    float lo[16], sec[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      lo[q] = -INFINITY;
      sec[q] = -INFINITY;
    }
    const unsigned char* rowp = kb_lds + r * RB + 16 * h;
    // A operand of the -cc/2 k-step: all ones against the three bf16 pieces
    // and zeros (the step's sum is the pieces' sum whatever the k order of the
    // fragment; every product is exact)
    const __bf16 one = (__bf16)1.f;
    const kb_bf8 a_one = (kb_bf8){one, one, one, one, one, one, one, one};
    // one centre tile: 3 KS MFMAs of x.c' in one chain, then the -cc/2 step
    // LAST (so only its own roundings see |cc|: the bound in kc_coef)
    // k-step ks of x.c' for the centre tile at rp: three bf16 MFMAs (MODE 0)
    // or one fp16 MFMA (MODE 1)
    auto kstep = [&](int ks, const unsigned char* rp, kb_acc& c0) {
      if constexpr (MODE == 0) {
        const kb_bf8 bh = *(const kb_bf8*)(rp + 32 * ks);
        const kb_bf8 bl = *(const kb_bf8*)(rp + 2 * D + 32 * ks);
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[ks], bh, c0, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[ks], bl, c0, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[ks], bh, c0, 0, 0, 0);
      } else {
        const kh_f8 bh = *(const kh_f8*)(rp + 32 * ks);
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[ks], bh, c0, 0, 0, 0);
      }
    };
    // MODE 0 runs a tile's chain in two phases: the small cross terms xh.cl
    // and xl.ch of every k-step first (their partial sums stay below
    // 2 * 2^-8 |x'| cmax), then the xh.ch terms -- so only the 16 KS
    // additions of the second phase see partial sums of size |x'| cmax and
    // the chain bound is ~16.5 KS additions instead of 48 KS (B hi is read
    // twice per k-step).  Step i of NST: MODE 0 i < KS small terms of k-step
    // i, else the big term of k-step i - KS; MODE 1 = kstep(i).
    constexpr int NST = MODE == 0 ? 2 * KS : KS;
    auto step = [&](int i, const unsigned char* rp, kb_acc& c0) {
      if constexpr (MODE == 0) {
        if (i < KS) {
          const kb_bf8 bh = *(const kb_bf8*)(rp + 32 * i);
          const kb_bf8 bl = *(const kb_bf8*)(rp + 2 * D + 32 * i);
          c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl, c0, 0, 0, 0);
          c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh, c0, 0, 0, 0);
        } else {
          const kb_bf8 bh = *(const kb_bf8*)(rp + 32 * (i - KS));
          c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i - KS], bh, c0, 0, 0, 0);
        }
      } else {
        kstep(i, rp, c0);
      }
    };
    auto chain = [&](int ct, kb_acc& c0) {
      c0 = (kb_acc){};
      const unsigned char* rp = rowp + ct * 32 * RB;
#pragma unroll
      for (int i = 0; i < NST; ++i) step(i, rp, c0);
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_one, *(const kb_bf8*)(rp + CCOFF), c0, 0, 0, 0);
    };
    // fold tile ct's acc, tagged with ct, into the running top-2 (3 VALU per
    // value: the a' = cc - 2S fma of the earlier form is the MFMA step above)
    auto fold1 = [&](int q, int ct, float acc) {
      const float v = ks_tag(acc, (unsigned int)ct);
      sec[q] = ks_med3(v, lo[q], sec[q]);
      lo[q] = ks_max(lo[q], v);
    };
    auto fold = [&](int ct, const kb_acc& c0) {
#pragma unroll
      for (int q = 0; q < 16; ++q) fold1(q, ct, c0[q]);
    };
    // software pipeline: tile ct's fold (VALU) is independent of tile ct+1's
    // MFMAs, so each wave fills its own MFMA gaps with it: the fold of the
    // previous tile is written into the k-loop of the next tile's chain (16 / KS
    // values per k-step) and the sched barriers keep each region to one chain
    // + one fold (the scheduler otherwise hoists both tiles' B reads: spills).
    auto chain_fold = [&](int ct, kb_acc& c0, int pct, const kb_acc& p0) {
      c0 = (kb_acc){};
      const unsigned char* rp = rowp + ct * 32 * RB;
#pragma unroll
      for (int i = 0; i < NST; ++i) {
        step(i, rp, c0);
#pragma unroll
        for (int qq = 0; qq < 16 / NST; ++qq) fold1(i * (16 / NST) + qq, pct, p0[i * (16 / NST) + qq]);
      }
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_one, *(const kb_bf8*)(rp + CCOFF), c0, 0, 0, 0);
    };
    // pairwise fold (screen only): two tiles' values a, b of one
    // row fold as sec = max(sec, med3(lo, a, b)), lo = max3(lo, a, b) -- the
    // top two of {lo, sec, a, b} with lo >= sec -- 5 VALU per 2 values
    // instead of 6; needs both tiles' accumulators live (a third and fourth
    // set: the screen has the registers, MODE 0 does not)
    constexpr bool PAIRF = MODE == 1 && NCT >= 2;
    auto fold2 = [&](int q, int ct, float a, float b) {
      const float ta = ks_tag(a, (unsigned int)ct), tb = ks_tag(b, (unsigned int)(ct + 1));
      sec[q] = ks_max(sec[q], ks_med3(lo[q], ta, tb));
      lo[q] = ks_max3(lo[q], ta, tb);
    };
    // chains of tiles ct, ct + 1 into c0, c1, with the pair fold of tiles
    // pct, pct + 1 (p0, p1) written into their k-loops (16 / KS / 2 rows per k-step)
    auto chain2_fold = [&](int ct, kb_acc& c0, kb_acc& c1, int pct, const kb_acc& p0, const kb_acc& p1) {
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        kb_acc& c = half ? c1 : c0;
        c = (kb_acc){};
        const unsigned char* rp = rowp + (ct + half) * 32 * RB;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          kstep(ks, rp, c);
#pragma unroll
          for (int qq = 0; qq < 8 / KS + (KS > 8 ? 1 : 0); ++qq) {
            const int q = half * 8 + ks * (8 / KS) + qq;
            if (q < 16) fold2(q, pct, p0[q], p1[q]);
          }
        }
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_one, *(const kb_bf8*)(rp + CCOFF), c, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    if constexpr (PAIRF) {
      kb_acc a0, a1, b0, b1;
      chain(0, a0);
      chain(1, a1);
#pragma unroll 1
      for (int cp = 2; cp < NCT; cp += 4) {
        chain2_fold(cp, b0, b1, cp - 2, a0, a1);
        if (cp + 2 < NCT) chain2_fold(cp + 2, a0, a1, cp, b0, b1);
      }
      if constexpr (((NCT - 2) / 2) & 1) {
#pragma unroll
        for (int q = 0; q < 16; ++q) fold2(q, NCT - 2, b0[q], b1[q]);
      } else {
#pragma unroll
        for (int q = 0; q < 16; ++q) fold2(q, NCT - 2, a0[q], a1[q]);
      }
    } else {
      kb_acc a0, b0;
      // the sweep at wave priority 1: with two waves per SIMD the one in its
      // MFMA sweep issues first and the partner's split / decision VALU fills
      // the gaps (list pass 1.22 -> 1.16 ms at cfg3, tools/kp_ablate.sh as_prio)
      __builtin_amdgcn_s_setprio(1);
      chain(0, a0);
      if constexpr (NCT == 1) {
        fold(0, a0);
      } else {
#pragma unroll 1
        for (int cp = 0; cp < NCT - 2; cp += 2) {
          chain_fold(cp + 1, b0, cp, a0);
          __builtin_amdgcn_sched_barrier(0);
          chain_fold(cp + 2, a0, cp + 1, b0);
          __builtin_amdgcn_sched_barrier(0);
        }
        chain_fold(NCT - 1, b0, NCT - 2, a0);
        __builtin_amdgcn_sched_barrier(0);
        fold(NCT - 1, b0);
      }
      __builtin_amdgcn_s_setprio(0);
    }
    float lo0[16];  // this lane's best per register (its centre r over all tiles)
#pragma unroll
    for (int q = 0; q < 16; ++q) lo0[q] = lo[q];
    ks_top2_vals(lo, sec, lane);
    i64 code_pf = 0;
    if constexpr (LPF) {
      // the decided rows' old label codes (km_label_pre), then the next
      // tile's rows (the split is dead since the sweep, the top-2 lists
      // since the line above) and the row indices of the tile after it
      const i64 nrow2 = lrow(tile + 2 * stride);
      code_pf = labels[grow_pf];
      load_row(nrow);
      nrow = nrow2;
    }
    // the centre of each row's best: lane (h, 2q) holds row rt(q, h)'s
    // b1; the lowest lane of that half whose own best equals it is the
    // centre r (ties in the tagged value share the tile, so the lowest r is
    // the lowest centre index, the first occurrence)
    // (branch-free: the ballot's first set bit goes straight into lane 2q /
    // 32 + 2q by writelane; a row always matches in its own half, so the
    // empty-mask case never decides a label)
    int rmin = 0;
    auto rmin_q = [&](auto qc) {
      constexpr int q = decltype(qc)::value;
      const float b0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, lo[0]), 2 * q));
      const float b1h = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, lo[0]), 32 + 2 * q));
      const unsigned long long m = __ballot(lo0[q] == (h ? b1h : b0));
      const int r0 = __builtin_ctz((unsigned int)m | 0x80000000u);
      const int r1 = __builtin_ctz((unsigned int)(m >> 32) | 0x80000000u);
      // lane selects are inline constants (no SGPR lane-select hazard)
      int v = rmin;
      asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(r0), "n"(2 * q));
      asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(r1), "n"(32 + 2 * q));
      rmin = v;
    };
    ks_unroll(rmin_q, std::make_integer_sequence<int, 16>{});
    p2 += __shfl_xor(p2, 32, 64);  // row r's |p|^2 in lanes r and r + 32
    // one decision per row, by the even lane of its pair (as in k_kmeans_filter_b3)
    const int rt = rtd;
    const i64 slot = tile * 32 + rt;
    const bool live = slot < nlim && (r & 1) == 0;
    const i64 grow = LPF ? grow_pf : rows_in ? (live ? rows_in[slot] : 0) : slot;
    const float b1 = lo[0], b2 = sec[0];
    const int i1 = 32 * (int)(__builtin_bit_cast(unsigned int, b1) & 7u) + rmin;
    const float p2f = __shfl(p2, rt, 64);
    // the bound in fp32 (kc_coef): |p| from the fp32 sum of squares with
    // slack for its rounding and for underflowed squares, e(|p|) by two fmas,
    // each rounding priced by the 1.0001 factors
    // (v_sqrt_f32 directly: its ~1 ulp is inside the 1.0001 slack, and the
    // argument is >= 1e-37, a normal number)
    const float pn = __builtin_amdgcn_sqrtf(__builtin_fmaf(p2f, 1.001f, 1e-37f)) * 1.0001f;
    const float e = __builtin_fmaf(__builtin_fmaf(kq[2], pn, kq[1]), pn, kq[0]) * 1.0001f;
    const bool fin = cok && isfinite(p2f) && isfinite(e) && pn < pn_lim && isfinite(b1) && isfinite(b2);
    // acc = -a'/2: a' gap > 2e  <=>  acc gap b1 - b2 > e
    const bool dec = fin && b1 - b2 > 1.0001f * e;
    // (the old codes are waited for here, on every path: a wait inside the
    // label branch left a later reuse of their registers to a full drain)
    if constexpr (LPF) asm volatile("" ::"v"(code_pf));
    if (live && dec) {
      if constexpr (LPF) km_label_pre(labels, mv, grow, i1, code_pf);
      else km_label(labels, counters, grow, i1);
    }
    if (MODE == 0 && live && !fin) full_list[atomicAdd(&counters[0], 1u)] = grow;
    const bool needc = live && !dec && (MODE == 1 || fin);
    // the tile's undecided rows as one lane mask, compacted into a row list
    // by k_ks_compact (one global atomic per tile on a single counter
    // serialised at its L2 channel: 31 ms for the screen's 3.1 M tiles)
    const unsigned long long und = __ballot(needc);
    if (lane == 0) und_mask[tile] = und;
  }
}

// Row list of the undecided rows from the per-tile lane masks of
// k_kmeans_filter_as (bit l: lane (h, r) = (l >> 5, l & 31) decided row rt(r >> 1, h)
// of the tile); rows_in: the tile slots stand for rows_in[slot].  A block
// covers KC_TPB = 256 x KC_TPT tiles (coalesced mask loads, tile j * 256 + t of
// the chunk to thread t) and takes its range with ONE atomic: one atomic per
// 256 tiles serialised on the counter's L2 channel (147 us at cfg3's 3.1 M
// tiles, 25 MB of masks).
// KC_TPT tiles per thread: 16 for the sparse full-row pass (~5 % of rows at
// cfg3), 1 for the dense list pass (~20 % of its slots): a thread's rows are
// written one after another, so a dense mask wants few tiles per thread.
// LAYOUT 2 (k_kmeans_pp): bit l < 32 <-> row 32 tile + l.  base_in (the
// deterministic form, k_ks_count + k_exscan_u32): the block's first list slot
// instead of an atomic on cnt -- the list is then in row order.
template <int KC_TPT, int LAYOUT = 0>
__global__ __launch_bounds__(256) void k_ks_compact(i64 N, const unsigned long long* __restrict__ mask,
                                                    const i64* __restrict__ rows_in,
                                                    const unsigned int* __restrict__ nrows_in, i64* __restrict__ out,
                                                    unsigned int* __restrict__ cnt,
                                                    const unsigned int* __restrict__ base_in = nullptr,
                                                    const i64* __restrict__ vals_in = nullptr,
                                                    i64* __restrict__ vals_out = nullptr) {
  // vals_in / vals_out (optional): vals_out[pos] = vals_in[slot] beside the list
  __shared__ unsigned int wsum[4];
  __shared__ unsigned int base;
  const i64 nlim = rows_in ? (i64)*nrows_in : N;
  const i64 ntiles = (nlim + 31) / 32;
  const i64 t0 = (i64)blockIdx.x * 256 * KC_TPT;
  if (t0 >= ntiles) return;  // block-uniform
  unsigned long long m[KC_TPT];
  unsigned int n = 0;
#pragma unroll
  for (int j = 0; j < KC_TPT; ++j) {
    const i64 tl = t0 + j * 256 + threadIdx.x;
    m[j] = tl < ntiles ? mask[tl] : 0ull;
    n += (unsigned int)__popcll(m[j]);
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned int inc = n;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned int v = __shfl_up(inc, o, 64);
    if (lane >= o) inc += v;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  if (threadIdx.x == 0) base = base_in ? base_in[blockIdx.x] : atomicAdd(cnt, wsum[0] + wsum[1] + wsum[2] + wsum[3]);
  __syncthreads();
  unsigned int pos = base + inc - n;
  for (int k = 0; k < w; ++k) pos += wsum[k];
#pragma unroll
  for (int j = 0; j < KC_TPT; ++j) {
    const i64 tl = t0 + j * 256 + threadIdx.x;
    unsigned long long mm = m[j];
    while (mm) {
      const int l = __builtin_ctzll(mm);
      mm &= mm - 1;
      i64 slot;
      if (LAYOUT == 0) {  // 32x32 output layout (k_kmeans_filter_as)
        const int q = (l & 31) >> 1, h = l >> 5;
        slot = tl * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
      } else {  // point order (k_kmeans_pp)
        slot = tl * 32 + l;
      }
      if (vals_out) vals_out[pos] = vals_in[slot];
      out[pos++] = rows_in ? rows_in[slot] : slot;
    }
  }
}

template <int NCT, int KS, int MODE>
static void ks_launch(hipStream_t s, i64 N, const float* P, i64 ldp, const __bf16* CBh, const __bf16* CBl,
                      const float* cnf, const double* cmax, i64* labels, unsigned int* counters, i64* full_list,
                      unsigned long long* und_mask, const i64* rows_in, const unsigned int* nrows_in,
                      const float* muf, int grid) {
  const size_t lds = ks_lds_bytes(16 * KS, NCT, MODE);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_kmeans_filter_as<NCT, KS, MODE>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)ks_lds_bytes(KB_DMAX, 8));
    attr = true;
  }
  k_kmeans_filter_as<NCT, KS, MODE><<<grid, ks_waves(MODE) * 64, lds, s>>>(N, P, ldp, CBh, CBl, cnf, cmax, labels, counters,
                                                                     full_list, und_mask, rows_in, nrows_in, muf);
}

template <int NCT, int MODE>
static void ks_launch_d(hipStream_t s, i64 N, i64 D, const float* P, i64 ldp, const __bf16* CBh, const __bf16* CBl,
                        const float* cnf, const double* cmax, i64* labels, unsigned int* counters, i64* full_list,
                        unsigned long long* und_mask, const i64* rows_in, const unsigned int* nrows_in,
                        const float* muf, int grid) {
  if (D == 64)
    ks_launch<NCT, 4, MODE>(s, N, P, ldp, CBh, CBl, cnf, cmax, labels, counters, full_list, und_mask, rows_in,
                            nrows_in, muf, grid);
  else
    ks_launch<NCT, 8, MODE>(s, N, P, ldp, CBh, CBl, cnf, cmax, labels, counters, full_list, und_mask, rows_in,
                            nrows_in, muf, grid);
}

template <int MODE>
static void ks_launch_n(int nct, hipStream_t s, i64 N, i64 D, const float* P, i64 ldp, const __bf16* CBh,
                        const __bf16* CBl, const float* cnf, const double* cmax, i64* labels, unsigned int* counters,
                        i64* full_list, unsigned long long* und_mask, const i64* rows_in,
                        const unsigned int* nrows_in, const float* muf, int grid) {
  switch (nct) {
    case 1: ks_launch_d<1, MODE>(s, N, D, P, ldp, CBh, CBl, cnf, cmax, labels, counters, full_list, und_mask, rows_in, nrows_in, muf, grid); break;
    case 2: ks_launch_d<2, MODE>(s, N, D, P, ldp, CBh, CBl, cnf, cmax, labels, counters, full_list, und_mask, rows_in, nrows_in, muf, grid); break;
    case 4: ks_launch_d<4, MODE>(s, N, D, P, ldp, CBh, CBl, cnf, cmax, labels, counters, full_list, und_mask, rows_in, nrows_in, muf, grid); break;
    default: ks_launch_d<8, MODE>(s, N, D, P, ldp, CBh, CBl, cnf, cmax, labels, counters, full_list, und_mask, rows_in, nrows_in, muf, grid); break;
  }
}

// ---------------------------------------------------------------------------
// Fused k-means step (k_kmeans_pp): the fp16 screen AND the centroid
// accumulation in ONE pass over the points (spx_kmeans_step;
// kmeans_dist_mapper + argmin + kmeans_count_mapper + kmeans_center_mapper,
// k_means_.py:52-89, 126-136).
//
// Ping-pong over 32-row units.  One block per CU, 8 waves in two groups:
// waves 0-3 (group 0) and 4-7 (group 1), wave s of each group on SIMD s
// (a workgroup's waves w and w + 4 share a SIMD).  Unit u belongs to group
// u & 1.  Slot t (one barrier each): group t & 1 plays the MATRIX role, the
// other group the VECTOR role, so on every SIMD one wave keeps the matrix
// pipe busy while its partner does vector / LDS work (MI355X_MICROARCH.md
// "Two waves per SIMD"):
//   matrix role (group t & 1): the screen of unit t -- wave s holds centre
//     tiles 2s, 2s + 1 (64 centres) as the fp16 MFMA A operand; two chains
//     of 8 v_mfma_f32_32x32x16_f16 over unit t's fp16 x' (LDS), started from
//     -cc/2 (an LDS table in accumulator order), give S - cc/2 = -a''/2 for
//     64 centres x 32 rows.  Woven between those MFMAs: the read-add-writes of
//     unit t - 4's decided rows (this group's unit whose decision the other
//     group made in slot t - 2) into the LDS sums; then that unit's labels
//     and undecided bits, and the loads of unit t + 4;
//   vector role (the other group): the decision of unit t - 2 (the matrix
//     group's unit, folded in slot t - 1; wave 0) with the add rounds of its rows,
//     written to LDS for its adds in slot t + 2; the fold of unit t - 1's
//     accumulators (this group's matrix role of slot t - 1) to per-row top-2
//     candidates; the staging of unit t + 1 (x' = fl(x - mu), fp16(x') to
//     LDS, |x'|^2 column partials).  The decision's LDS round trips are
//     hidden behind the fold's vector work, and none of them sits in front
//     of an MFMA.
// Every cross-wave hand-off crosses at least one barrier: x' is staged one
// slot before its MFMAs (xh by unit parity), candidates are folded one slot
// before their decision (exv by unit parity), |x'|^2 partials three slots
// before (p2p by unit mod 4), decisions two slots before the adds (dres by
// unit mod 4); the sums are written by the matrix group only.
// The certified decision is k_kmeans_filter_as MODE 1's (same MFMA chains,
// bound, kq and finiteness checks; 4-bit register tags per centre tile).
// Accumulation: the block's per-centre sums live in LDS as fp32 [256][D].
// Lane (jr, hr) of wave s holds columns D/4 s + D/8 hr .. + D/8 of row jr
// (row-rotated quads, see below), so a wave adds its rows from the registers
// the loads landed in and waves never share an address.  Two rows of one
// centre in one unit would race in a plain read-add-write, so the adds go in
// rounds: a row's round is its rank among the unit's rows of its centre,
// from one LDS atomic increment per decided row on a counter table (wave
// 0, the decision's; the lanes of one instruction that hit one counter are
// ordered the same way every time), and the round loop runs to the unit's
// largest rank (< 32 by construction: no data-dependent bound to guard).
// The order of every add is fixed: the sums are deterministic.  Every KP_FW
// units the fp32 sums go by plain stores to the block's partial slot for
// that window and are cleared; the slots are summed in fp64 in a fixed order
// after the kernel.  Each label / mask word is stored once, by one lane
// (ghost rows write a dummy word).
typedef float kfs_f2 __attribute__((ext_vector_type(2)));
typedef int kfs_i2 __attribute__((ext_vector_type(2)));
__host__ __device__ constexpr int kfs_rs(int D) { return 2 * D + 16; }  // fp16 row stride: +16 B keeps ds_read_b128 conflict-free
constexpr int KP_WAVES = 8;
constexpr int KP_U = 32;     // rows per unit (one 32-row MFMA tile)
constexpr int KP_NR = 4;     // units per group in the register ring (load -> stage -> MFMA -> decide -> add)
constexpr int KP_AHEAD = 4;  // unit t + 4 is loaded in slot t (its stage is in slot t + 3)
constexpr int KP_LAG = 4;    // unit t - 4 is added in slot t
constexpr int KP_UNR = 8;    // slots per unrolled loop body: ring entries (unit >> 1) % 4 are compile-time
constexpr int KP_FW = 504;   // units per flush window (16128 rows)
constexpr int KP_XS = 48;    // exv / p2p row stride (bytes): 12 dwords, spreads a lane group's rows over the banks
static_assert(KP_FW % KP_UNR == 0 && KP_UNR == 2 * KP_NR && KP_AHEAD + KP_LAG == 2 * KP_NR,
              "flush points fall on the unrolled body's first slot; the ring cycles once per body");
static size_t kp_lds_bytes(int D) {
  return (size_t)256 * D * 4 + 256 * 4 + (size_t)2 * KP_U * kfs_rs(D) + (size_t)2 * KP_U * KP_XS +
         (size_t)4 * KP_U * KP_XS + (size_t)4 * KP_U * 4 + 256 * 4 + (size_t)8 * 2 * 16 * 4 + (size_t)D * 4 +
         (size_t)4 * KP_U * 4;
}

template <int KS, int NCT>
struct KpStep {
  static constexpr int D = 16 * KS, CPW = D / 4, CPL = D / 8, NQ = CPL / 4, RS = kfs_rs(D), U = KP_U,
                       NR = KP_NR;
  static_assert(CPL % 8 == 0, "D = 64 or 128");
};

template <int KS, int NCT>
__global__ __launch_bounds__(KP_WAVES * 64, 1) void k_kmeans_pp(
    i64 N, i64 K, const float* __restrict__ P, i64 ldp, const __bf16* __restrict__ CBh,
    const __bf16* __restrict__ CBl, const float* __restrict__ cnf2, const double* cmax_p,
    const float* __restrict__ muf, i64* __restrict__ labels, unsigned long long* __restrict__ und_mask,
    float* __restrict__ part, int nwin, unsigned long long* __restrict__ pcnt, unsigned long long* __restrict__ dummy) {
  typedef KpStep<KS, NCT> C;
  constexpr int D = C::D, CPW = C::CPW, CPL = C::CPL, NQ = C::NQ, RS = C::RS, U = C::U, NR = C::NR;
  extern __shared__ __attribute__((aligned(16))) unsigned char kp_lds[];
  float* sums = (float*)kp_lds;                          // [256][D] fp32
  unsigned int* cnts = (unsigned int*)(sums + 256 * D);  // [256] decided rows per centre
  unsigned char* xh = (unsigned char*)(cnts + 256);      // [2][U][RS] fp16 x' (by unit parity)
  unsigned char* exv = xh + (size_t)2 * U * RS;          // [2][U][KP_XS]: (b1, b2) of waves 0-3, then their 4 indices
  unsigned char* p2p = exv + (size_t)2 * U * KP_XS;      // [4][U][KP_XS]: 8 |x'|^2 column partials (by unit mod 4)
  int* dres = (int*)(p2p + (size_t)4 * U * KP_XS);       // [4][U]: label (low 16 bits, -1: undecided) | add round << 16
  unsigned int* rcnt = (unsigned int*)(dres + 4 * U);    // [256] rows per centre so far in the unit (rank counters)
  float* cci = (float*)(rcnt + 256);                     // [8 tiles][2 halves][16]: -cc/2 of a lane's accumulator centres
  float* mus = cci + 8 * 2 * 16;                         // [D] the centring vector mu
  float* ebuf = mus + D;                                 // [4][U]: a row's bound e (NaN: no decision), by unit mod 4
  // (j, h): the MFMA / fold / decision lanes (row j = lane & 31, k-half or
  // centre half h = lane >> 5).  (jr, hr): the raw-column lanes (row jr =
  // lane >> 1, column half hr = lane & 1) of the loads, the staging and the
  // sums adds: lane (jr, hr) of wave s holds columns col0 .. col0 + D/8 of
  // row jr as NQ 4-column quads, rotated by the row: register q holds quad
  // (q + jr) mod NQ.  So the 8 lanes of one
  // ds_write_b128 group (4 rows x 2 halves) store 8 different quads -- 8
  // distinct bank groups whatever the rows' centres -- and a ds_read_b128
  // group meets at most 2-way conflicts (a random centre-dependent swizzle
  // cost ~3x on both).
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, grp = w >> 2, s = w & 3, j = lane & 31, h = lane >> 5;
  const int jr = lane >> 1, hr = lane & 1;
  const int col0 = CPW * s + CPL * hr;
  for (int i = t; i < 256 * D + 256; i += KP_WAVES * 64) sums[i] = 0.f;  // (cnts: the same bits)
  for (int i = t; i < 256; i += KP_WAVES * 64) rcnt[i] = 0u;
  auto qof = [&](int q) __attribute__((always_inline)) { return (q + jr) & (NQ - 1); };
  for (int i = t; i < D; i += KP_WAVES * 64) mus[i] = muf[i];

  // A operands: wave s screens centre tiles 2s and 2s + 1 (lane (j, h):
  // centre 32 ct + j, dims 16 ks + 8 h .. + 8 of k-step ks)
  // (with 8 centre tiles every wave screens two: compile-time true, so the
  // MFMA chain and the fold carry no per-pair branches)
  const bool scr0 = NCT >= 8 || 2 * s < NCT, scr1 = NCT >= 8 || 2 * s + 1 < NCT;
  kh_f8 ca[2][KS];
#pragma unroll
  for (int tl = 0; tl < 2; ++tl) {
    const int ct = 2 * s + tl;
    const i64 c = 32 * (i64)(ct < NCT ? ct : 0) + j;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const i64 d = 16 * ks + 8 * h + e;
        ca[tl][ks][e] = (_Float16)((float)CBh[c * D + d] + (float)CBl[c * D + d]);
      }
    // the chain's initial accumulator (round 5; was a bf16 MFMA pair adding
    // -cc/2 as three pieces after the chain): register q of lane (j, h) is
    // centre 32 ct + (q & 3) + 8 (q >> 2) + 4 h, so the 16 values depend on
    // (ct, h) only -- lanes j < 16 write them once, the chain's lanes read
    // them back as four broadcast ds_read_b128 per tile
    if (j < 16) {
      const i64 m = 32 * (i64)ct + (j & 3) + 8 * (j >> 2) + 4 * h;
      cci[(ct * 2 + h) * 16 + j] = ct < NCT ? -0.5f * cnf2[m] : 0.f;
    }
  }

  // the certified bound of k_kmeans_filter_as MODE 1 (same arithmetic)
  const double cmax = cmax_p[0], mcoef = cmax_p[1], mun = cmax_p[2], dcmax = cmax_p[3];
  const double u32 = 5.9604644775390625e-08;
  const double chain = 16.0 * (double)KS;
  const double eS = (u32 * cmax + 4.8828125e-04 * cmax + 1.001 * dcmax +
                     2.0 * (chain + 3.0) * u32 * 1.001 * (cmax + dcmax)) * 1.01;
  double xk1 = 64.0 * u32 * cmax, xk0 = 32.0 * u32 * (cmax * cmax + 2.0 * mun * cmax);
  // -cc/2 enters the chain as its initial accumulator: every one of the
  // chain's roundings also sees |cc/2| <= cmax^2 / 2 (x 2 for the MFMA's
  // directed rounding, x 2 for the best and the second value)
  xk0 += 2.0 * (chain + 3.0) * u32 * 1.001 * 1.01 * cmax * cmax;
  xk0 += sqrt((double)D) * 1.1920928955078125e-07 * (cmax + dcmax) + (double)D * 3.552713678800501e-15;
  xk1 += 14.0 * 1.1920928955078125e-07 * cmax;
  xk0 += 7.0 * 1.1920928955078125e-07 * (cmax * cmax + 2.0 * mun * cmax);
  float kq[3];
  kc_coef(eS, cmax, mun, mcoef, D, kq, xk1, xk0);
  const bool cok = cmax * cmax < 1e36 && mun * cmax < 1e36 && cmax < 3.0e4 && dcmax == dcmax;
  // rows with |x'| >= pn_lim (the fp32 range limit) are left undecided and
  // not added (label code -1): the list passes label them exactly and the
  // gathered accumulation adds them in fp64.  A FAR row (|x'| >= pn_far =
  // 4 (cmax + |mu|)) that the screen cannot decide is not added
  // provisionally either: if its label moved afterwards, the fp32 rounding
  // of its own add would stay in p's window chain (the test with
  // far undecided outliers).  A far row the screen DOES decide is added as
  // any other -- its label is final, so nothing moves (round 6, ADVICE r05:
  // the far cut on every row left most rows of zero-mean data, where |x'|
  // is the data's scale and cmax + |mu| may be far smaller, to the list
  // passes).  Wave 1 hands the far flag to the decision as the sign of e.
  const float pn_lim = (float)(cmax > 0.0 ? 1e36 / cmax : 1e36);
  const float pn_far = (float)(4.0 * (cmax + mun) + 1e-30);

  const int G = gridDim.x, bk = blockIdx.x;
  // block bk takes units bk, bk + G, ...: in every slot the grid reads one
  // contiguous stretch of G units (G x 16 KiB).  (Round 5: one contiguous
  // range of units per block -- 256 streams far apart -- ran 0.1-0.2 ms
  // SLOWER at cfg3, gpurun_out/r5f.)
  const i64 nunits = (N + U - 1) / U;
  const int nit = bk < nunits ? (int)((nunits - 1 - bk) / G + 1) : 0;
  // slots 0 .. nit + KP_LAG - 1 (unit nit - 1 is added in slot nit - 1 + KP_LAG), whole bodies
  const int nrun = nit > 0 ? (nit + KP_LAG + KP_UNR - 1) / KP_UNR * KP_UNR : 0;

  kb_f4 ring[NR][NQ];
  kb_acc acc0 = (kb_acc){}, acc1 = (kb_acc){};
  auto load = [&](kb_f4 (&r)[NQ], int u) __attribute__((always_inline)) {  // clamped: always a valid address
    const i64 un = bk + (i64)(u < nit ? u : nit - 1) * G;
    i64 row = un * U + jr;
    row = row < N ? row : N - 1;
    const float* p = P + row * ldp + col0;
#pragma unroll
    for (int q = 0; q < NQ; ++q) r[q] = *(const kb_f4*)(p + 4 * qof(q));
  };
  auto mu_load = [&](kb_f4 (&mu4)[NQ]) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) mu4[q] = *(const kb_f4*)(mus + col0 + 4 * qof(q));
  };
  // unit u -> xh[u & 1], p2p[u & 3]
  auto stage = [&](const kb_f4 (&r)[NQ], const kb_f4 (&mu4)[NQ], int u) __attribute__((always_inline)) {
    typedef _Float16 kh_4 __attribute__((ext_vector_type(4)));
    kfs_f2 p2v = (kfs_f2){0.f, 0.f};
    unsigned char* hrow = xh + ((size_t)(u & 1) * U + jr) * RS + 2 * col0;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      kh_4 hv;
#pragma unroll
      for (int e = 0; e < 4; e += 2) {
        const kfs_f2 x = (kfs_f2){r[q][e], r[q][e + 1]} - (kfs_f2){mu4[q][e], mu4[q][e + 1]};
        p2v = __builtin_elementwise_fma(x, x, p2v);
        hv[e] = (_Float16)x[0];
        hv[e + 1] = (_Float16)x[1];
      }
      *(kh_4*)(hrow + 8 * qof(q)) = hv;
    }
    *(float*)(p2p + ((size_t)(u & 3) * U + jr) * KP_XS + 4 * (2 * s + hr)) = p2v[0] + p2v[1];
  };
  // lane j and lane j + 32 exchange x: both get (x of lane j, x of lane j + 32)
  auto sw32 = [](float x, float& lo, float& hi) __attribute__((always_inline)) {
    const unsigned int b = __builtin_bit_cast(unsigned int, x);
    const auto r = __builtin_amdgcn_permlane32_swap(b, b, false, false);
    lo = __builtin_bit_cast(float, (unsigned int)r[0]);
    hi = __builtin_bit_cast(float, (unsigned int)r[1]);
  };
  auto fold16 = [&](const kb_acc& acc, int ct, float& lo, float& sec, int& il) __attribute__((always_inline)) {
    float tv[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const float a = acc[q];
      tv[q] = __builtin_bit_cast(float, (__builtin_bit_cast(unsigned int, a) & ~15u) | (unsigned int)q);
    }
    lo = ks_max(tv[0], tv[1]);
    sec = ks_med3(tv[0], tv[1], -INFINITY);
#pragma unroll
    for (int q = 2; q < 16; q += 2) {
      sec = ks_max(sec, ks_med3(lo, tv[q], tv[q + 1]));
      lo = ks_max3(lo, tv[q], tv[q + 1]);
    }
    const unsigned int qb = __builtin_bit_cast(unsigned int, lo) & 15u;
    il = 32 * ct + (int)((qb & 3) + 8 * (qb >> 2)) + 4 * h;
  };

  auto cc_init = [&]() __attribute__((always_inline)) {
    acc0 = *(const kb_acc*)(cci + (4 * s + h) * 16);
    acc1 = *(const kb_acc*)(cci + (4 * s + 2 + h) * 16);
  };

  // vector role of slot t: the decision of unit t - 2 and its add rounds
  // (dres[(t - 2) & 3]), the fold of unit t - 1 (exv[(t - 1) & 1]), the
  // staging of unit t + 1.  Wave 0 of the group computes the decision and
  // writes it (round 4: every wave computed the same bits; wave 0 alone is
  // -0.05-0.1 ms, the kernel being power-limited): its LDS round trips run
  // in the shadow of the fold's vector work, interleaved by hand (sched
  // barriers).
  auto vector_role = [&](int tt, const kb_f4 (&rs)[NQ]) __attribute__((always_inline)) {
    const int u2 = tt - 2, uf = tt - 1, us = tt + 1;
    const bool dv = u2 >= 0 && u2 < nit, fv = uf >= 0 && uf < nit;
    const i64 grow = (bk + (i64)(dv ? u2 : 0) * G) * U + j;
    const bool rlive = dv && grow < N;
    const unsigned char* er = exv + ((size_t)(u2 & 1) * U + j) * KP_XS;
    // (1) the decision's loads (wave 0 only: the other waves' decisions were
    // the same bits, computed for nothing); the rows' bounds e come ready
    // from wave 1 of the previous slot (step (2b))
    kb_f4 e4 = (kb_f4){0.f, 0.f, 0.f, 0.f};
    kfs_i2 i2 = (kfs_i2){0, 0};
    float er_e = 0.f;
    if (s == 0) {
      e4 = *(const kb_f4*)(er + 16 * h);
      i2 = *(const kfs_i2*)(er + 32 + 8 * h);
      er_e = ebuf[(u2 & 3) * U + j];
    }
    // (2) fold, first tile (its latency cover)
    float lo0 = -INFINITY, sec0 = -INFINITY, lo1 = -INFINITY, sec1 = -INFINITY;
    int il0 = 0, il1 = 0;
    if (scr0) fold16(acc0, 2 * s, lo0, sec0, il0);  // (unused when !fv: exv is written only if fv)
    __builtin_amdgcn_sched_barrier(0);
    // (2b) wave 1 (off the critical path: it makes no decision) prepares the
    // bound of the unit decided in the NEXT slot, t - 1 (staged in slot t - 2,
    // its |x'|^2 partials complete): the sum of the 8 column partials, |p|,
    // e(|p|) and the finiteness / range checks, exactly as the decision did
    // them (the same order: bit-identical decisions), NaN for a row the
    // screen cannot decide.  (Round 5: the decision wave is the slot's
    // critical path, ~400 cycles longer than the other waves' vector roles,
    // tools/kp_roles.py.)
    if (s == 1) {
      const int ue = tt - 1;
      const kb_f4 p4 = *(const kb_f4*)(p2p + ((size_t)(ue & 3) * U + j) * KP_XS + 16 * h);
      const float pp = (p4[0] + p4[1]) + (p4[2] + p4[3]);
      float pl, ph;
      sw32(pp, pl, ph);
      const float p2f = pl + ph;  // the same order in both lanes of the row
      const float pn = __builtin_amdgcn_sqrtf(__builtin_fmaf(p2f, 1.001f, 1e-37f)) * 1.0001f;
      const float e = __builtin_fmaf(__builtin_fmaf(kq[2], pn, kq[1]), pn, kq[0]) * 1.0001f;
      const bool ok = cok && isfinite(p2f) && isfinite(e) && pn < pn_lim;
      if (h == 0) ebuf[(ue & 3) * U + j] = ok ? (pn < pn_far ? e : -e) : __builtin_nanf("");
    }
    // (3) decide: top-2 over the 4 waves' candidates, the certified rule.
    // d: the centre the row is added to -- its label when decided, and,
    // PROVISIONALLY, the screen's best for a finite undecided row (the list
    // passes settle its label; the few whose label then differs are moved
    // by a correction pass, spx_kmeans_step).  dl: the label code stored
    // for the row: the label, -2 - d (provisional) or -1 (not added:
    // non-finite, or a ghost row).
    int d = -1, dl = -1;
    if (s == 0) {
      const float b1 = ks_max(e4[0], e4[2]), b2 = ks_med3(e4[0], e4[2], ks_max(e4[1], e4[3]));
      const int ib = e4[0] >= e4[2] ? i2[0] : i2[1];
      float b1l, b1h, b2l, b2h, fl, fh;
      sw32(b1, b1l, b1h);
      sw32(b2, b2l, b2h);
      sw32(__builtin_bit_cast(float, ib), fl, fh);
      const float B1 = ks_max(b1l, b1h), B2 = ks_med3(b1l, b1h, ks_max(b2l, b2h));
      const int IB = b1l >= b1h ? __builtin_bit_cast(int, fl) : __builtin_bit_cast(int, fh);
      const float e = __builtin_fabsf(er_e);  // NaN: not finite, out of range, or cok false (2b)
      const bool far = er_e < 0.f;            // |x'| >= pn_far: added only when decided
      const bool fin = isfinite(e) && isfinite(B1) && isfinite(B2);
      const bool dec = fin && B1 - B2 > 1.0001f * e;
      const bool add = rlive && fin && IB < (int)K && (dec || !far);
      d = add ? IB : -1;
      dl = !add ? -1 : dec ? IB : -2 - IB;
    }
    // (4) each decided row's rank among the unit's rows of its centre (its
    // add round): one LDS atomic increment per row on wave 0's counter table
    // (lanes j < 32: one per row; the lanes of one instruction that hit one
    // address are ordered the same way every time, so the add order -- and
    // the sums -- are deterministic), the counters reset right behind it;
    // fold of the second tile beside the round trip.  The row is counted here
    // too, by an LDS atomic add with no return (integers: any order gives the
    // same count; a read-modify-write per add round cost a round trip each)
    const bool act = d >= 0;
    unsigned int rk = 0;
    if (s == 0 && h == 0 && act) {
      rk = __hip_atomic_fetch_add(rcnt + d, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_add(cnts + d, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (scr1) fold16(acc1, 2 * s + 1, lo1, sec1, il1);
    __builtin_amdgcn_sched_barrier(0);
    if (s == 0 && h == 0 && act) __hip_atomic_store(rcnt + d, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    // (5) merge the fold's tiles and halves, the candidates out (mu's reads
    // for the stage first)
    const float fb1 = ks_max(lo0, lo1), fb2 = ks_med3(lo0, lo1, ks_max(sec0, sec1));
    const int fib = lo0 >= lo1 ? il0 : il1;
    float c1l, c1h, c2l, c2h, cfl, cfh;
    sw32(fb1, c1l, c1h);
    sw32(fb2, c2l, c2h);
    sw32(__builtin_bit_cast(float, fib), cfl, cfh);
    const float FB1 = ks_max(c1l, c1h), FB2 = ks_med3(c1l, c1h, ks_max(c2l, c2h));
    const int FIB = c1l >= c1h ? __builtin_bit_cast(int, cfl) : __builtin_bit_cast(int, cfh);
    if (fv) {
      unsigned char* ew = exv + ((size_t)(uf & 1) * U + j) * KP_XS;
      if (h == 0)
        *(kfs_f2*)(ew + 8 * s) = (kfs_f2){FB1, FB2};
      else
        *(int*)(ew + 32 + 4 * s) = FIB;
    }
    __builtin_amdgcn_sched_barrier(0);
    // (6) stage of unit t + 1
    if (us < nit) {
      kb_f4 mu4[NQ];
      mu_load(mu4);
      stage(rs, mu4, us);
    }
    const int rnd = act ? (int)rk : 0xffff;  // add round (0xffff: no add)
    if (s == 0 && h == 0) dres[(u2 & 3) * U + j] = (dl & 0xffff) | (rnd << 16);
  };

  // matrix role of slot t: the MFMAs of unit t (if t < nit) with, woven
  // between them, the add rounds of unit t - 4 (raw columns in r, label and
  // round from dres), that unit's labels and undecided bits and the loads of
  // unit t + 4 into the ring entry unit t - 4 leaves.  Each MFMA pair holds
  // the matrix pipe for 64 cycles; an LDS read-add-write round, the stores
  // and the loads issue in those shadows instead of after the chain (round 5:
  // the chain, then the rounds, the stores and the loads made this role the
  // slot's critical path).
  auto matrix_role = [&](int tt, kb_f4 (&r)[NQ]) __attribute__((always_inline)) {
    // the matrix role is the slot's critical path: its wave issues first when
    // both waves of a SIMD are ready (-0.3 ms per cfg3 pass; the vector role
    // first: +0.2 ms, profiles/r04_kp_ablate_v4.txt)
    __builtin_amdgcn_s_setprio(1);
    const int ua = tt - KP_LAG;
    const bool av = ua >= 0 && ua < nit;
    const i64 una = bk + (i64)(av ? ua : 0) * G;
    const i64 grow = una * U + j;
    const bool rlive = av && grow < N;
    const int dr = dres[(ua & 3) * U + jr];  // the add lanes' rows
    const int dlv = dres[(ua & 3) * U + j];  // the label lanes' rows
    // the chain's initial accumulators (-cc/2), read first: the matrix role
    // has the slack for their latency, the vector role (the slot's critical
    // path, tools/kp_roles.py) does not
    cc_init();
    const unsigned char* bp = xh + ((size_t)(tt & 1) * U + j) * RS + 16 * h;
    // B fragments three k-steps ahead: under load an LDS read takes longer
    // than one MFMA pair, and a read issued one step ahead stalled every pair
    constexpr int PF = KS < 2 ? KS : 2, NB = PF + 1;
    kh_f8 bq[NB];
#pragma unroll
    for (int p = 0; p < PF; ++p) bq[p] = *(const kh_f8*)(bp + 32 * p);
    // the MFMAs run in every slot, also in the few drain slots past the
    // block's last unit (stale operands, results never folded into exv):
    // no per-pair branches in the chain; acc0 / acc1 hold -cc/2 (cc_init)
    const int dcode = av ? (int)(short)(dr & 0xffff) : -1;
    const int d = dcode >= 0 ? dcode : dcode <= -2 ? -2 - dcode : -1;  // the centre the row is added to
    const int rnd = av ? (int)((unsigned int)dr >> 16) : 0xffff;
    float* const srow = sums + (d >= 0 ? d : 0) * D + col0;
    // the add rounds (a wave's LDS operations run in issue order: round k + 1
    // reads what round k wrote); a row's round is its rank, so round k has
    // work only if some row of the unit has rank >= k.  Rounds 0 .. NRU - 1
    // are straight-line steps between the MFMA pairs: the reads of round k at
    // step RDk, its read-add-writes at step WRk; rounds NRU and later
    // (a unit with NRU + 1 rows of one centre: rare) run in a loop after the
    // chain's last k-step.
    constexpr int NRU = KS >= 8 ? 3 : 2;
    constexpr int WR0 = 1, RD1 = 2, WR1 = KS >= 8 ? 4 : 3, RD2 = 5, WR2 = 7;
    kb_f4 v[NQ];
    auto rd = [&]() __attribute__((always_inline)) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) v[q] = *(kb_f4*)(srow + 4 * qof(q));
    };
    auto wr = [&]() __attribute__((always_inline)) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) *(kb_f4*)(srow + 4 * qof(q)) = v[q] + r[q];
    };
    if (rnd == 0) rd();
    // labels (-1 for an undecided row: the list passes write it) and the
    // unit's undecided-row mask, each word stored ONCE: row j's label by lane
    // j of wave j / 8, the mask by lane 0 of wave 0 (round 5: every wave's 64
    // lanes stored every word, 8 label and 256 mask stores per word: -0.25 ms
    // without them, profiles/r05_kp_redundant_ab.txt -- the kernel is power-
    // limited).  The dummy word takes only ghost rows / units (a few per
    // block).  (With the idle lanes of every store aimed at ONE dummy word,
    // all CUs' stores met on one L2 line; the vmcnt waits that count those
    // stores cost ~3.7 ms per cfg3 pass -- profiles/r04_kp_ablate_v4.txt.)
    auto stores = [&]() __attribute__((always_inline)) {
      const int dlab = av ? (int)(short)(dlv & 0xffff) : -1;
      i64* la = rlive ? labels + grow : (i64*)dummy;
      if ((j >> 3) == s && h == 0) *la = (i64)dlab;
      const unsigned long long m = __ballot(dlab < 0 && rlive) & 0xffffffffull;
      unsigned long long* ma = av ? und_mask + una : dummy + 1;
      if (s == 0 && lane == 0) *ma = m;
    };
    auto mk = [&](auto kc) __attribute__((always_inline)) {
      constexpr int ks = decltype(kc)::value;
      if constexpr (ks + PF < KS) bq[(ks + PF) % NB] = *(const kh_f8*)(bp + 32 * (ks + PF));
      if (scr0) acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ca[0][ks], bq[ks % NB], acc0, 0, 0, 0);
      if (scr1) acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ca[1][ks], bq[ks % NB], acc1, 0, 0, 0);
      if constexpr (ks == WR0) { if (rnd == 0) wr(); }
      if constexpr (ks == RD1) { if (rnd == 1) rd(); }
      if constexpr (ks == WR1) { if (rnd == 1) wr(); }
      if constexpr (NRU > 2 && ks == RD2) { if (rnd == 2) rd(); }
      if constexpr (NRU > 2 && ks == WR2) { if (rnd == 2) wr(); }
      if constexpr (ks == KS - 2) stores();
      __builtin_amdgcn_sched_barrier(0);
    };
    ks_unroll(mk, std::make_integer_sequence<int, KS>{});
    // (a rank is < U by construction -- at most U rows per unit -- so the
    // cap k < U never binds; it bounds the loop whatever dres holds)
    for (int k = NRU; k < U && __ballot(rnd >= k && rnd != 0xffff) != 0ull; ++k)
      if (rnd == k) {
        rd();
        wr();
      }
    load(r, tt + KP_AHEAD);
    __builtin_amdgcn_s_setprio(0);
  };

  // one slot of the unrolled body (compile-time copy c of KP_UNR, group GR)
  auto slot = [&](auto gc, auto cc, int tt) __attribute__((always_inline)) {
    constexpr int GR = decltype(gc)::value, c = decltype(cc)::value;
    __syncthreads();
    if constexpr (c == 0)
      if (tt > 0 && tt % KP_FW == 0) {
        // window tt / KP_FW - 1 of the block's fp32 sums into its partial
        // slot (plain 16-byte stores), then cleared; summed in fp64 later
        float* pb = part + ((i64)bk * nwin + tt / KP_FW - 1) * K * D;
        for (int i = 4 * t; i < K * D; i += 4 * KP_WAVES * 64) {
          const int dd = i / D, cl = i % D;
          kb_f4* src = (kb_f4*)(sums + dd * D + cl);
          *(kb_f4*)(pb + i) = *src;
          *src = (kb_f4){0.f, 0.f, 0.f, 0.f};
        }
        __syncthreads();
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
      }
    if constexpr ((c & 1) == GR)
      matrix_role(tt, ring[((c + KP_UNR - KP_LAG) >> 1) % NR]);
    else
      vector_role(tt, ring[((c + 1) >> 1) % NR]);
  };

  auto body = [&](auto gc) __attribute__((always_inline)) {
    constexpr int GR = decltype(gc)::value;
    if (nit > 0) {
      // the loads in the order the loop keeps them in flight (two stores
      // before each unit's loads, as a matrix slot issues them), so the
      // compiler's count of outstanding operations is the same at the loop
      // head on entry and on the back edge
#pragma unroll
      for (int k = 0; k < KP_AHEAD / 2; ++k) {
        __builtin_nontemporal_store(0ull, dummy + (lane & 1) + 4 * k);
        __builtin_nontemporal_store(0ull, dummy + 2 + (lane & 1) + 4 * k);
        load(ring[k], GR + 2 * k);
      }
      if constexpr (GR == 0) {
        kb_f4 mu4[NQ];
        mu_load(mu4);
        stage(ring[0], mu4, 0);
      }
    }
    for (int t0 = 0; t0 < nrun; t0 += KP_UNR) {
      ks_unroll([&](auto cc) __attribute__((always_inline)) {
        slot(gc, cc, t0 + decltype(cc)::value);
      }, std::make_integer_sequence<int, KP_UNR>{});
    }
  };
  // the set-up loads (centres, mu, bound inputs) complete here, so the loop's
  // waits count only the ring's loads and the slots' stores
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  __syncthreads();  // sums, rcnt, cci
  cc_init();
  if (grp == 0)
    body(std::integral_constant<int, 0>{});
  else
    body(std::integral_constant<int, 1>{});

  __syncthreads();
  {
    // the last window, then zero slots for windows this block does not have
    const int wdone = nrun > 0 ? (nrun - 1) / KP_FW : 0;
    float* pb = part + ((i64)bk * nwin + wdone) * K * D;
    for (int i = 4 * t; i < K * D; i += 4 * KP_WAVES * 64) {
      const int dd = i / D, cl = i % D;
      *(kb_f4*)(pb + i) = *(kb_f4*)(sums + dd * D + cl);
    }
    for (int win = wdone + 1; win < nwin; ++win)
      for (int i = 4 * t; i < K * D; i += 4 * KP_WAVES * 64)
        *(kb_f4*)(part + ((i64)bk * nwin + win) * K * D + i) = (kb_f4){0.f, 0.f, 0.f, 0.f};
  }
  if (t < K) pcnt[(i64)bk * K + t] = cnts[t];
}

template <int KS, int NCT>
static void kp_launch(hipStream_t s, int grid, i64 N, i64 K, const float* P, i64 ldp, const __bf16* CBh,
                      const __bf16* CBl, const float* cnf2, const double* cmax, const float* muf, i64* labels,
                      unsigned long long* und_mask, float* part, int nwin, unsigned long long* pcnt,
                      unsigned long long* dummy) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_kmeans_pp<KS, NCT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)kp_lds_bytes(16 * KS));
    attr = true;
  }
  k_kmeans_pp<KS, NCT><<<grid, KP_WAVES * 64, kp_lds_bytes(16 * KS), s>>>(
      N, K, P, ldp, CBh, CBl, cnf2, cmax, muf, labels, und_mask, part, nwin, pcnt, dummy);
}

static void kp_launch_n(int nct, int KS, hipStream_t s, int grid, i64 N, i64 K, const float* P, i64 ldp,
                        const __bf16* CBh, const __bf16* CBl, const float* cnf2, const double* cmax, const float* muf,
                        i64* labels, unsigned long long* und_mask, float* part, int nwin, unsigned long long* pcnt,
                        unsigned long long* dummy) {
#define KP_CASE(KSV, NC)                                                                                         \
  if (KS == KSV && nct == NC) {                                                                                  \
    kp_launch<KSV, NC>(s, grid, N, K, P, ldp, CBh, CBl, cnf2, cmax, muf, labels, und_mask, part, nwin, pcnt, dummy); \
    return;                                                                                                      \
  }
  KP_CASE(8, 8) KP_CASE(8, 4) KP_CASE(8, 2) KP_CASE(8, 1)
  KP_CASE(4, 8) KP_CASE(4, 4) KP_CASE(4, 2) KP_CASE(4, 1)
#undef KP_CASE
}

// Deterministic compaction of lane masks (LAYOUT 2: bit j <-> row 32 tile + j)
// into an index-ordered row list: per-block counts, one exclusive scan, then
// k_ks_compact at the scanned bases (the summation order of the gathered
// accumulation depends on the list order, so it must not follow atomics).
template <int KC_TPT>
__global__ __launch_bounds__(256) void k_ks_count(i64 N, const unsigned long long* __restrict__ mask,
                                                  unsigned int* __restrict__ bcnt) {
  __shared__ unsigned int ws[4];
  const i64 ntiles = (N + 31) / 32;
  const i64 t0 = (i64)blockIdx.x * 256 * KC_TPT;
  unsigned int n = 0;
#pragma unroll
  for (int jj = 0; jj < KC_TPT; ++jj) {
    const i64 tl = t0 + jj * 256 + threadIdx.x;
    n += tl < ntiles ? (unsigned int)__popcll(mask[tl]) : 0u;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = n;
  __syncthreads();
  if (threadIdx.x == 0) bcnt[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// exclusive scan of n block counts in place (one block), the total into *total
__global__ __launch_bounds__(1024) void k_exscan_u32(unsigned int* __restrict__ v, i64 n, unsigned int* __restrict__ total) {
  // thread t owns a run of `per` entries; the run totals are scanned by a
  // wave scan + the 16 wave totals (the first version scanned all 1024 run
  // totals serially in thread 0: ~19 us of LDS round trips)
  __shared__ unsigned int wsum[16];
  const i64 per = (n + 1023) / 1024;
  const i64 a = threadIdx.x * per, b = a + per < n ? a + per : n;
  unsigned int s = 0;
  for (i64 i = a; i < b; ++i) s += v[i];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned int inc = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned int y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  unsigned int base = 0;
  for (int k = 0; k < w; ++k) base += wsum[k];
  if (threadIdx.x == 1023) *total = base + inc;
  unsigned int run = base + inc - s;
  for (i64 i = a; i < b; ++i) {
    const unsigned int x = v[i];
    v[i] = run;
    run += x;
  }
}

// Exact-order labels of the undecided points from their candidate masks
// (K <= 256); equal distances go to the lower index (= first occurrence).
// KC_LPP lanes per point: in round j lane s takes the (KC_LPP j + s)-th
// candidate (undecided points keep ~2 candidates: 99 % have <= 3, measured
// at cfg3, tools/km_undecided.py), and a (distance, index) min over the
// point's lanes.  The sequential fp64 d-loop reads the point and the centre
// in 16-dim chunks through a 2-deep register ring (16-byte loads, the next
// chunk in flight while this one is summed): the per-element loads of the
// first version paid an L2 / HBM latency per dim.
// NATURAL: bit k of word w <-> centre 32 w + k (bf16x3 filter); else centre
// w + 8 k (fp32 filter).
#define KC_LPP 4
#define KC_DC 16
template <typename TP>
__device__ __forceinline__ void kc_chunk(const TP* __restrict__ x, const double* __restrict__ cc, i64 d, bool vec,
                                         TP (&xv)[KC_DC], double (&cv)[KC_DC]) {
  if (vec) {
    typedef TP V4 __attribute__((ext_vector_type(16 / sizeof(TP))));
    constexpr int E = 16 / sizeof(TP);
#pragma unroll
    for (int k = 0; k < KC_DC; k += E) {
      const V4 v = *(const V4*)(x + d + k);
#pragma unroll
      for (int e = 0; e < E; ++e) xv[k + e] = v[e];
    }
#pragma unroll
    for (int k = 0; k < KC_DC; k += 2) {
      const double2 v = *(const double2*)(cc + d + k);
      cv[k] = v.x;
      cv[k + 1] = v.y;
    }
  } else {
#pragma unroll
    for (int k = 0; k < KC_DC; ++k) {
      xv[k] = x[d + k];
      cv[k] = cc[d + k];
    }
  }
}

template <typename TP, bool NATURAL>
__global__ __launch_bounds__(256) void k_kmeans_cand(i64 D, const TP* __restrict__ P, i64 ldp,
                                                     const double* __restrict__ C, i64* __restrict__ labels,
                                                     const unsigned int* __restrict__ counters,
                                                     const KfCand* __restrict__ cand_list, int r32) {
  const i64 n = counters[1];
  const int sub = threadIdx.x % KC_LPP;
  const i64 step = ((i64)gridDim.x * 256) / KC_LPP;
  const i64 Dc = D / KC_DC * KC_DC;  // chunked part of the d-loop
  for (i64 q = ((i64)blockIdx.x * 256 + threadIdx.x) / KC_LPP; q < n; q += step) {  // uniform per point lanes
    const i64 row = cand_list[q].row;
    unsigned int mw[8];
    int tot = 0;
#pragma unroll
    for (int wd = 0; wd < 8; ++wd) {
      mw[wd] = cand_list[q].mask[wd];
      tot += __popc(mw[wd]);
    }
    const TP* x = P + row * ldp;
    double best = 0.0;
    int bi = -1;
    for (int j = 0; KC_LPP * j < tot; ++j) {  // uniform per point lanes
      int nth = KC_LPP * j + sub, c = -1;
#pragma unroll
      for (int wd = 0; wd < 8; ++wd) {
        const int pc = __popc(mw[wd]);
        if (c < 0 && nth < pc) {
          unsigned int m = mw[wd];
          for (int k = 0; k < nth; ++k) m &= m - 1;
          const int b = __ffs(m) - 1;
          c = NATURAL ? 32 * wd + b : wd + 8 * b;
        } else if (c < 0) {
          nth -= pc;
        }
      }
      const double* cc = C + (i64)(c < 0 ? 0 : c) * D;
      const bool vec = ((uintptr_t)x % 16) == 0 && ((uintptr_t)cc % 16) == 0;
      double acc = 0.0;
      TP xv[2][KC_DC];
      double cv[2][KC_DC];
      if (Dc > 0) kc_chunk<TP>(x, cc, 0, vec, xv[0], cv[0]);
      for (i64 d0 = 0; d0 < Dc; d0 += 2 * KC_DC) {
        if (d0 + KC_DC < Dc) kc_chunk<TP>(x, cc, d0 + KC_DC, vec, xv[1], cv[1]);
#pragma unroll
        for (int k = 0; k < KC_DC; ++k) {
          const double df = (double)xv[0][k] - cv[0][k];
          const double sq = df * df;
          acc = acc + sq;
        }
        if (d0 + KC_DC >= Dc) break;
        if (d0 + 2 * KC_DC < Dc) kc_chunk<TP>(x, cc, d0 + 2 * KC_DC, vec, xv[0], cv[0]);
#pragma unroll
        for (int k = 0; k < KC_DC; ++k) {
          const double df = (double)xv[1][k] - cv[1][k];
          const double sq = df * df;
          acc = acc + sq;
        }
      }
      for (i64 d = Dc; d < D; ++d) {
        const double df = (double)x[d] - cc[d];
        const double sq = df * df;
        acc = acc + sq;
      }
      double dist = sqrt(acc);
      if (r32) dist = (double)(float)dist;  // fp32-rounded distances: equal values tie, first index wins
      if (c >= 0 && (bi < 0 || dist < best || (dist == best && c < bi))) {
        best = dist;
        bi = c;
      }
    }
#pragma unroll
    for (int o = 1; o < KC_LPP; o <<= 1) {
      const double ob = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (oi >= 0 && (bi < 0 || ob < best || (ob == best && oi < bi))) {
        best = ob;
        bi = oi;
      }
    }
    if (sub == 0) km_label(labels, counters, row, bi);
  }
}

// The same exact-order candidate distances with 16 lanes per point (fp32
// points, D = 16 DPL, 16-byte aligned rows and centres -- the bf16x3 path's
// shapes): lane s loads dims [s DPL, (s + 1) DPL) of the point once and of each
// candidate centre in one go and squares its differences in parallel; the
// sum keeps scipy's order ((0 + sq_0) + sq_1) + ... by passing the running
// fp64 sum from lane to lane (16 shuffles per candidate).  The 4-lane kernel
// above walked each 128-dim row through a 2-deep register ring: one memory
// round trip per 32 dims per candidate (0.46 ms for cfg3's ~0.6 M rows).
template <int DPL>
__global__ __launch_bounds__(256) void k_kmeans_cand16(const float* __restrict__ P, i64 ldp,
                                                       const double* __restrict__ C, i64* __restrict__ labels,
                                                       const unsigned int* __restrict__ counters,
                                                       const KfCand* __restrict__ cand_list, int r32) {
  constexpr int D = 16 * DPL;
  const i64 n = counters[1];
  const int g = threadIdx.x >> 4, s = threadIdx.x & 15;
  const i64 step = (i64)gridDim.x * 16;
  for (i64 q = (i64)blockIdx.x * 16 + g; q < n; q += step) {  // uniform per 16-lane group
    const i64 row = cand_list[q].row;
    float xv[DPL];
    {
      const float* x = P + row * ldp + s * DPL;
#pragma unroll
      for (int j = 0; j < DPL; j += 4) {
        const kb_f4 v = *(const kb_f4*)(x + j);
#pragma unroll
        for (int e = 0; e < 4; ++e) xv[j + e] = v[e];
      }
    }
    double best = 0.0;
    int bi = -1;
#pragma unroll 1
    for (int wd = 0; wd < 8; ++wd) {
      unsigned int m = cand_list[q].mask[wd];
      while (m) {  // uniform per group
        const int c = 32 * wd + __builtin_ctz(m);
        m &= m - 1;
        const double* cc = C + (i64)c * D + s * DPL;
        double sq[DPL];
#pragma unroll
        for (int j = 0; j < DPL; j += 2) {
          const double2 v = *(const double2*)(cc + j);
          const double d0 = (double)xv[j] - v.x, d1 = (double)xv[j + 1] - v.y;
          sq[j] = d0 * d0;
          sq[j + 1] = d1 * d1;
        }
        // lane t's dims follow lane t - 1's: the running sum goes round the
        // group by DPP row_newbcast (a VALU move; the ds_bpermute of __shfl put
        // an LDS round trip into each of the chain's 16 steps: 0.52 -> 0.46 ms
        // at cfg3; two candidates' chains interleaved measured slower)
        double acc = 0.0;
        ks_unroll([&](auto tc) __attribute__((always_inline)) {
          constexpr int t = decltype(tc)::value;
          double a = acc;
#pragma unroll
          for (int j = 0; j < DPL; ++j) a = a + sq[j];
          const unsigned long long u = __builtin_bit_cast(unsigned long long, a);
          const unsigned int lo = (unsigned int)__builtin_amdgcn_update_dpp(0, (int)(unsigned int)u, 0x150 + t, 0xF, 0xF, false);
          const unsigned int hi = (unsigned int)__builtin_amdgcn_update_dpp(0, (int)(unsigned int)(u >> 32), 0x150 + t, 0xF, 0xF, false);
          acc = __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
        }, std::make_integer_sequence<int, 16>{});
        double dist = sqrt(acc);
        if (r32) dist = (double)(float)dist;  // fp32-rounded distances: equal values tie, first index wins
        if (bi < 0 || dist < best || (dist == best && c < bi)) {
          best = dist;
          bi = c;
        }
      }
    }
    if (s == 0) km_label(labels, counters, row, bi);
  }
}

// CT[d][c] = (float)C[c][d] (zero-padded to Kp centres), cn[c] = |C[c]|^2 in
// fp64 (+inf for padding), *cmax = max_c |C[c]| (one block).
__global__ __launch_bounds__(256) void k_kmeans_prep(i64 D, i64 K, i64 Kp, const double* __restrict__ C,
                                                     float* __restrict__ CT, double* __restrict__ cn,
                                                     double* __restrict__ cmax, double mcoef) {
  __shared__ double red[256];
  double mx = 0.0;
  for (i64 c = threadIdx.x; c < Kp; c += 256) {
    double s = 0.0;
    for (i64 d = 0; d < D; ++d) {
      const double v = c < K ? C[c * D + d] : 0.0;
      CT[d * Kp + c] = (float)v;
      s += v * v;
    }
    cn[c] = c < K ? s : INFINITY;
    if (c < K) mx = (s > mx || s != s) ? s : mx;
  }
  red[threadIdx.x] = mx;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      const double a = red[threadIdx.x], b = red[threadIdx.x + o];
      red[threadIdx.x] = (b > a || b != b) ? b : a;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    cmax[0] = sqrt(red[0]) * 1.001;
    cmax[1] = mcoef;
    cmax[2] = 0.0;  // uncentred
  }
}

// Accumulation: sums[c][:] += P[p][:] and counts[c] += 1 for labels[p] == c,
// replacing kmeans_center_mapper / kmeans_count_mapper (k_means_.py:61-89,
// which sum in fp32; fp64 here is at least as exact).  No float atomics and a
// fixed summation order, so the result is deterministic:
//   k_kmeans_accum    persistent 1024-lane blocks; block (x, y) covers the
//                     centre tile of KA_CB = 16 waves x KA_CPW centres and the
//                     64 columns picked by y, over the point chunks x, x+G, ...
//                     Wave w owns the centres c == w (mod 16) of the tile and
//                     keeps their fp64 sums in registers (lane = column): the
//                     centre of a point is wave-uniform, so adding a row is an
//                     indexed-register add (s_set_gpr_idx), no LDS
//                     read-modify-write (fp64 LDS RMW traffic bounded the
//                     LDS-accumulator design at ~16 ms for cfg3,
//                     tools/ka_tune.hip).  Chunks are prefetched with 16-byte
//                     loads (one per lane: dword loads cap a 1-block-per-CU
//                     stream at ~2.2 TB/s) into a register ring KA_STAGES deep
//                     and staged in LDS, double-buffered (one barrier per
//                     chunk).  Every wave adds its own points in point order:
//                     the sums are deterministic, no atomics.  The tile is
//                     written once to the block's partial slot.
//   k_kmeans_reduce   out[i] (+)= sum over g of part[g][i]: four fixed g
//                     slices per output, combined in a fixed order.
constexpr int KA_THREADS = 1024;
constexpr int KA_CPL = 2;                  // columns per lane: 2 -> every point is visited once per wave at D = 128
constexpr int KA_DB = 64 * KA_CPL;         // columns per tile
constexpr int KA_WAVES = KA_THREADS / 64;  // centre owners per tile
constexpr int KA_CPW = 16;                 // centres per wave (register sums)
constexpr int KA_CB = KA_WAVES * KA_CPW;   // centres per tile
constexpr int KA_STAGES = 3;               // register prefetch ring depth (chunks per barrier): 3 -> 10.1 ms, 2 -> 10.2, 4 -> 10.7, 1 -> 11.8 at cfg3 (profiles/r01_ka_variants.txt)
constexpr int KA_BPC = 1;                  // resident blocks per CU (LDS: 2 KA_STAGES x 16 KiB per block)

// rows / nrows (optional): accumulate only the rows rows[0 .. *nrows) (a
// row list in row order, gathered row by row; the count is read on the device).
template <typename TP>
__global__ __launch_bounds__(KA_THREADS) __attribute__((amdgpu_waves_per_eu(4 * KA_BPC, 8))) void k_kmeans_accum(i64 N, i64 D, i64 K, const TP* __restrict__ P, i64 ldp,
                                                             const i64* __restrict__ labels, double* __restrict__ psum,
                                                             unsigned long long* __restrict__ pcnt, int ndb,
                                                             const i64* __restrict__ rows = nullptr,
                                                             const unsigned int* __restrict__ nrows = nullptr,
                                                             const i64* __restrict__ lab_list = nullptr) {
  // lab_list (with a row list): entry i's label is lab_list[i], not labels[row]
  if (rows) N = (i64)*nrows;
  constexpr int VE = 16 / (int)sizeof(TP);                // elements per 16-byte load
  constexpr int CH = KA_THREADS * VE / KA_DB;             // points per chunk (64 f32 / 32 f64)
  constexpr int LPR = KA_DB / VE;                         // lanes per row slice
  constexpr int ST = KA_STAGES;
  typedef TP V __attribute__((ext_vector_type(VE)));
  __shared__ __attribute__((aligned(16))) TP xs[2][ST][CH * KA_DB];
  __shared__ int lab_s[2][ST][CH];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int cb = blockIdx.y / ndb, db = blockIdx.y % ndb;
  const i64 c0 = (i64)cb * KA_CB, d0 = (i64)db * KA_DB;
  const i64 nch = (N + CH - 1) / CH;
  const i64 G = gridDim.x;
  // this lane's slice of a chunk: point lp, columns d0 + lc .. + VE
  const int lp = t / LPR, lc = (t % LPR) * VE;
  // 16-byte loads need the slice inside the row and aligned; else per element
  const bool vec = d0 + lc + VE <= D && (ldp % VE) == 0 && ((uintptr_t)P % 16) == 0;
  static_assert(KA_CPL == 1 || KA_CPL == 2, "one or two columns per lane");
  typedef TP XV __attribute__((ext_vector_type(2)));
  // one flat register array per column (a vector-of-pairs array indexed at
  // run time is not promoted to registers: it went to scratch)
  double acc0[KA_CPW], acc1[KA_CPW];
#pragma unroll
  for (int j = 0; j < KA_CPW; ++j) acc0[j] = acc1[j] = 0.0;
  // counts: integer LDS atomics at staging time (order-free, hence exact and
  // deterministic), kept by the db == 0 blocks
  __shared__ unsigned int cnt_s[KA_CB];
  for (int i = t; i < KA_CB; i += KA_THREADS) cnt_s[i] = 0u;
  // Prefetch ring: loads use clamped (always valid) addresses and nothing
  // consumes them until the stage comes round again -- a use right after the
  // issue would make the compiler wait for the whole ring (vmcnt(0)).
  // A row list's indices are loaded one round ahead of the rows themselves
  // (ridx / lidx: chunk ch + ST G's), so a round waits for one load latency,
  // not for the index load and then the dependent row load.
  V pf[ST];
  i64 plab[ST], ridx[ST], lidx[ST];
  auto load_idx = [&](int s, i64 ch) {
    const i64 p0 = (ch < nch ? ch : nch - 1) * CH;
    ridx[s] = rows[p0 + lp < N ? p0 + lp : N - 1];
    if (t < CH) lidx[s] = rows[p0 + t < N ? p0 + t : N - 1];
  };
  auto load = [&](int s, i64 ch) {
    if (N == 0) return;  // an empty row list: nothing to load
    const i64 p0 = (ch < nch ? ch : nch - 1) * CH;
    const i64 pr = rows ? ridx[s] : (p0 + lp < N ? p0 + lp : N - 1);
    if (vec) {
      pf[s] = ld_stream((const V*)(P + pr * ldp + d0 + lc));  // read once: nt
    } else {
#pragma unroll
      for (int j = 0; j < VE; ++j) {
        const i64 d = d0 + lc + j < D ? d0 + lc + j : D - 1;
        pf[s][j] = P[pr * ldp + d];
      }
    }
    if (t < CH)
      plab[s] = lab_list ? lab_list[p0 + t < N ? p0 + t : N - 1] : labels[rows ? lidx[s] : (p0 + t < N ? p0 + t : N - 1)];
    if (rows) load_idx(s, ch + ST * G);
  };
#pragma unroll
  for (int s = 0; s < ST; ++s) {
    ridx[s] = lidx[s] = 0;
    if (rows && N > 0) load_idx(s, blockIdx.x + s * G);
  }
#pragma unroll
  for (int s = 0; s < ST; ++s) load(s, blockIdx.x + s * G);
  int buf = 0;
  // one barrier per ST chunks: the waves' uneven shares of a chunk's points
  // (labels mod 16) even out over ST chunks
  for (i64 base = blockIdx.x; base < nch; base += ST * G) {
    // stage into xs[buf]: its last reads (ST chunks ago) happened before
    // every wave passed the previous barrier
#pragma unroll
    for (int s = 0; s < ST; ++s) {
      const i64 p0 = (base + s * G) * CH;
      const bool prow = p0 + lp < N;
#pragma unroll
      for (int j = 0; j < VE; ++j)
        xs[buf][s][lp * KA_DB + lc + j] = (prow && d0 + lc + j < D) ? pf[s][j] : TP(0);
      if (t < CH) {
        const i64 l = plab[s];
        const int lr = (p0 + t < N && l >= c0 && l < K && l - c0 < KA_CB) ? (int)(l - c0) : -1;
        lab_s[buf][s][t] = lr;
        if (db == 0 && lr >= 0) atomicAdd(&cnt_s[lr], 1u);
      }
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < ST; ++s) load(s, base + (s + ST) * G);  // the next ST chunks fly meanwhile
#pragma unroll
    for (int s = 0; s < ST; ++s) {
      const int r = lane < CH ? lab_s[buf][s][lane] : -1;
      const int jl = (int)((unsigned)r / (unsigned)KA_WAVES);  // this lane's point's register slot
      unsigned long long m = __ballot(r >= 0 && (r % KA_WAVES) == w);
      // one point per step, in point order: the loop is issue-bound, so no
      // padded slots (unrolled variants that batch the LDS reads measured
      // slower: 2 -> 13.9 ms, 4 -> 16.6 ms vs 12.3 ms at cfg3); the LDS
      // latency is hidden by the other waves of the SIMD
      while (m) {  // wave-uniform
        const int p = __ffsll((long long)m) - 1;
        m &= m - 1;
        const int j = __builtin_amdgcn_readlane(jl, p);
        if constexpr (KA_CPL == 2) {
          const XV x = *(const XV*)&xs[buf][s][p * KA_DB + 2 * lane];
          acc0[j] += (double)x[0];
          acc1[j] += (double)x[1];
        } else {
          acc0[j] += (double)xs[buf][s][p * KA_DB + lane];
        }
      }
    }
    buf ^= 1;
  }
  const i64 g = blockIdx.x;
#pragma unroll
  for (int j = 0; j < KA_CPW; ++j) {
    const i64 c = c0 + (i64)j * KA_WAVES + w;
#pragma unroll
    for (int cc = 0; cc < KA_CPL; ++cc) {
      const i64 d = d0 + KA_CPL * lane + cc;
      if (c < K && d < D) psum[(g * K + c) * D + d] = cc ? acc1[j] : acc0[j];
    }
  }
  __syncthreads();
  if (db == 0)
    for (int i = t; i < KA_CB; i += KA_THREADS)
      if (c0 + i < K) pcnt[g * K + c0 + i] = cnt_s[i];
}

// 256 lanes = 64 outputs x 4 g-slices; slice s sums g = s, s+4, ... in order,
// then the four slice sums are added in order 0..3 (deterministic).
template <typename T, typename P = T>
__global__ __launch_bounds__(256) void k_kmeans_reduce(i64 n, i64 G, const P* __restrict__ part, T* __restrict__ out,
                                                       int add) {
  __shared__ T red[4][64];
  const int j = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const i64 i = (i64)blockIdx.x * 64 + j;
  T s = T(0);
  // unrolled: the loads of 8 g's in flight (one at a time, each L2 / HBM
  // latency was paid in series: ~20 us for K = 256 counts); the adds keep
  // their order
  if (i < n)
#pragma unroll 8
    for (i64 g = sl; g < G; g += 4) s += (T)part[g * n + i];
  red[sl][j] = s;
  __syncthreads();
  if (sl == 0 && i < n) {
    if (add == 2) {  // out -= the sum (the provisional adds' correction)
      T q = red[0][j];
      q += red[1][j];
      q += red[2][j];
      q += red[3][j];
      out[i] = out[i] - q;
    } else {
      T v = add ? out[i] : T(0);
      v += red[0][j];
      v += red[1][j];
      v += red[2][j];
      v += red[3][j];
      out[i] = v;
    }
  }
}

// Many fp32 partial slots (k_kmeans_pp's windows: G x nwin = 6144 at cfg3,
// 805 MB) -> KR_S fp64 slice sums: slice s adds slots s, s + KR_S, ... in
// order, 4 consecutive elements per thread (16-byte loads, a wave reads 1 KiB
// of one slot), so ~1 K blocks keep the stream busy where one thread per
// output of k_kmeans_reduce ran latency-bound (0.63 ms at cfg3); the slices
// then go through k_kmeans_reduce in a fixed order.  n % 4 == 0.
constexpr int KR_S = 32;
__global__ __launch_bounds__(256) void k_kmeans_slices(i64 n, i64 P, const float* __restrict__ part,
                                                       double* __restrict__ out) {
  const i64 e = ((i64)blockIdx.x * 256 + threadIdx.x) * 4;
  const int sl = blockIdx.y;
  if (e >= n) return;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
#pragma unroll 8
  for (i64 p = sl; p < P; p += KR_S) {
    const kb_f4 v = ld_stream((const kb_f4*)(part + p * n + e));
    a0 += (double)v[0];
    a1 += (double)v[1];
    a2 += (double)v[2];
    a3 += (double)v[3];
  }
  double* o = out + (i64)sl * n + e;
  o[0] = a0;
  o[1] = a1;
  o[2] = a2;
  o[3] = a3;
}

// Grid of the accumulation for (N, D, K): x = G point-chunk streams, y = tiles.
static void ka_grid(int dtype, i64 N, i64 D, i64 K, i64* G, i64* ndb, i64* ncb) {
  const i64 ch = KA_THREADS * (dtype == SPX_F32 ? 4 : 2) / KA_DB;  // points per chunk (k_kmeans_accum CH)
  *ndb = (D + KA_DB - 1) / KA_DB;
  *ncb = (K + KA_CB - 1) / KA_CB;
  const i64 nch = (N + ch - 1) / ch;
  i64 g = 256 * KA_BPC / (*ndb * *ncb);  // KA_BPC blocks per CU over all tiles
  if (g < 1) g = 1;
  if (g > nch) g = nch;
  *G = g < 1 ? 1 : g;
}

static i64 kf_kp(i64 K) { return (K + KF_BN - 1) / KF_BN * KF_BN; }

static int kf_persistent_grid(i64 N) {
  const i64 g = (N + 255) / 256;
  return (int)(g < 2048 ? (g < 1 ? 1 : g) : 2048);
}

extern "C" int64_t spx_kmeans_assign_workspace(int dtype, int64_t N, int64_t D, int64_t K) {
  if ((dtype != SPX_F32 && dtype != SPX_F64) || N < 0 || D < 1 || K < 1) return -1;
  const i64 Kp = kf_kp(K);
  // CT (D x Kp f32) | cn (Kp f64) | cmax | counters | full list (N i64) | candidate list (N KfCand, K <= 256)
  // | undecided-row list (N i64, K <= 256) | screen's undecided-row list (N i64, K <= 256)
  // | per-tile undecided lane masks (ceil(N / 32) u64, K <= 256) | centre mean (D f32, K <= 256)
  return (D * Kp * 4 + 15) / 16 * 16 + Kp * 8 + 32 + 64 + N * 8 +
         (Kp == KF_BN ? N * (i64)sizeof(KfCand) + 2 * N * 8 + (N + 31) / 32 * 8 + D * 4 : 0);
}

// spx_kmeans_assign's workspace, carved: CT (D x Kp f32, reused for the
// bf16 split of the centres) | cn (Kp f64; the cnf / cnf2 floats of the
// centred filters) | cmax | counters | full list (N i64) | candidate list (N
// KfCand) | undecided-row list (N i64) | screen's undecided-row list (N i64) |
// per-tile undecided lane masks (ceil(N / 32) u64) | centre mean (D f32); the
// last five only for K <= 256.
struct KmWs {
  float* CT;
  double* cn;
  double* cmax;  // [0] max |c'|, [1] fp32 tie margin coefficient, [2] |mu|, [3] max |c' - fp16(c')|
  unsigned int* counters;  // [0] full-list rows, [1] candidate rows, [2] undecided rows, [3] screen-undecided rows
  i64* full_list;
  KfCand* cand_list;
  i64* und_list;
  i64* scr_list;
  unsigned long long* und_mask;
  float* muf;
};

static KmWs km_carve(void* workspace, i64 N, i64 D, i64 Kp) {
  KmWs w;
  unsigned char* ws = (unsigned char*)workspace;
  w.CT = (float*)ws;
  ws += (D * Kp * 4 + 15) / 16 * 16;
  w.cn = (double*)ws;
  ws += Kp * 8;
  w.cmax = (double*)ws;
  ws += 32;
  w.counters = (unsigned int*)ws;  // 4 counters, then a KmMove at counters + 4
  ws += 64;
  w.full_list = (i64*)ws;
  ws += N * 8;
  w.cand_list = (KfCand*)ws;
  w.und_list = (i64*)(ws + (Kp == KF_BN ? N * (i64)sizeof(KfCand) : 0));
  w.scr_list = w.und_list + N;
  w.und_mask = (unsigned long long*)(w.scr_list + N);
  w.muf = (float*)(w.und_mask + (N + 31) / 32);
  return w;
}

static int num_cus() {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 1)
      ncu = 256;
  }
  return ncu;
}

// The passes after a certified screen left its undecided rows in
// w.scr_list (count in counters[3]): the A-stationary bf16x3 filter in list
// mode over them, the all-accumulator filter in list mode over what is still
// undecided (candidate masks), the exact recompute of the candidates in
// scipy's order, and the all-centre exact kernel for the rows no filter could
// evaluate (non-finite / overflowing).  Labels of every row are final after it.
static int km_resolve(hipStream_t s, i64 N, i64 D, i64 K, const float* Pf, i64 ldp, const double* centers,
                      i64* labels, const KmWs& w, int nct, int r32) {
  const int ncu = num_cus();
  const i64 ntiles = (N + 31) / 32;
  __bf16* CBh = (__bf16*)w.CT;
  __bf16* CBl = CBh + (i64)32 * nct * D;
  const float* cnf = (const float*)w.cn;
  const i64 need_as = (ntiles + KS_WAVES - 1) / KS_WAVES;
  const int grid_as = (int)(need_as < ncu ? need_as : ncu);
  const unsigned int cgrid1 = (unsigned int)((ntiles + 255) / 256);
  // the bf16x3 list pass centres the points as the screen does: it ranks by
  // |c'|^2 - 2 x'.c' (cnf2 of the prep) with x' = fl(x - mu)
  ks_launch_n<0>(nct, s, N, D, Pf, ldp, CBh, CBl, cnf + KF_BN, w.cmax, labels, w.counters, w.full_list, w.und_mask,
                 w.scr_list, w.counters + 3, w.muf, grid_as);
  LAUNCH_CHECK("spx_kmeans_assign(filter A-stationary, list)");
  k_ks_compact<1><<<cgrid1, 256, 0, s>>>(N, w.und_mask, w.scr_list, w.counters + 3, w.und_list, w.counters + 2);
  LAUNCH_CHECK("spx_kmeans_assign(compact)");
  switch (nct) {
    case 1: kb_launch<1>(s, N, D, Pf, ldp, CBh, CBl, cnf + KF_BN, w.cmax, labels, w.counters, w.full_list, w.cand_list, ncu, w.und_list, w.counters + 2, w.muf); break;
    case 2: kb_launch<2>(s, N, D, Pf, ldp, CBh, CBl, cnf + KF_BN, w.cmax, labels, w.counters, w.full_list, w.cand_list, ncu, w.und_list, w.counters + 2, w.muf); break;
    case 4: kb_launch<4>(s, N, D, Pf, ldp, CBh, CBl, cnf + KF_BN, w.cmax, labels, w.counters, w.full_list, w.cand_list, ncu, w.und_list, w.counters + 2, w.muf); break;
    default: kb_launch<8>(s, N, D, Pf, ldp, CBh, CBl, cnf + KF_BN, w.cmax, labels, w.counters, w.full_list, w.cand_list, ncu, w.und_list, w.counters + 2, w.muf); break;
  }
  LAUNCH_CHECK("spx_kmeans_assign(filter bf16x3, undecided rows)");
  const int gp = kf_persistent_grid(N);
  if ((D == 64 || D == 128) && ((uintptr_t)centers % 16) == 0) {
    if (D == 64) k_kmeans_cand16<4><<<gp, 256, 0, s>>>(Pf, ldp, centers, labels, w.counters, w.cand_list, r32);
    else k_kmeans_cand16<8><<<gp, 256, 0, s>>>(Pf, ldp, centers, labels, w.counters, w.cand_list, r32);
  } else {
    k_kmeans_cand<float, true><<<gp, 256, 0, s>>>(D, Pf, ldp, centers, labels, w.counters, w.cand_list, r32);
  }
  LAUNCH_CHECK("spx_kmeans_assign(candidates)");
  k_kmeans_assign<float><<<gp, 256, 0, s>>>(N, D, K, Pf, ldp, centers, labels, nullptr, w.full_list, w.counters, r32);
  LAUNCH_CHECK("spx_kmeans_assign(exact)");
  return SPX_OK;
}

// the certified screens' domain: fp32 points, K <= 256, D in {64, 128}, 16-byte rows
static bool km_screen_ok(int dtype, i64 K, i64 D, const void* points, i64 ldp) {
  return dtype == SPX_F32 && kf_kp(K) == KF_BN && (D == 64 || D == 128) && ldp % 4 == 0 &&
         ((uintptr_t)points % 16) == 0;
}

static int km_nct(i64 K) { return K <= 32 ? 1 : K <= 64 ? 2 : K <= 128 ? 4 : 8; }

extern "C" int spx_kmeans_assign(int dtype, int64_t N, int64_t D, int64_t K, const void* points, int64_t ldp,
                                 const double* centers, int64_t* labels, double* mindist, void* workspace,
                                 size_t workspace_bytes, int dist_dtype, void* stream) {
  if (dtype != SPX_F32 && dtype != SPX_F64) return set_err(SPX_ENOTSUP, "spx_kmeans_assign: points must be F32/F64");
  if (N < 0 || D < 1 || K < 1 || (N > 0 && ldp < D)) return set_err(SPX_EINVAL, "spx_kmeans_assign: bad N/D/K/ldp");
  if (dist_dtype != SPX_F64 && dist_dtype != SPX_F32)
    return set_err(SPX_EINVAL, "spx_kmeans_assign: dist_dtype must be F64 or F32");
  if (N == 0) return SPX_OK;
  if (!points || !centers || !labels) return set_err(SPX_EINVAL, "spx_kmeans_assign: null pointer");
  const int r32 = dist_dtype == SPX_F32;
  const double mcoef = r32 ? 4.76837158203125e-07 : 0.0;  // 2^-21
  const i64 g = (N + 255) / 256;
  if (g > 0x7fffffffLL) return set_err(SPX_EINVAL, "spx_kmeans_assign: too many points");
  if (mindist || !workspace) {  // all points through the exact-order kernel
    if (dtype == SPX_F32)
      k_kmeans_assign<float><<<(unsigned)g, 256, 0, S(stream)>>>(N, D, K, (const float*)points, ldp, centers, labels,
                                                                  mindist, nullptr, nullptr, r32);
    else
      k_kmeans_assign<double><<<(unsigned)g, 256, 0, S(stream)>>>(N, D, K, (const double*)points, ldp, centers,
                                                                   labels, mindist, nullptr, nullptr, r32);
    LAUNCH_CHECK("spx_kmeans_assign");
    return SPX_OK;
  }
  const int64_t need = spx_kmeans_assign_workspace(dtype, N, D, K);
  if ((int64_t)workspace_bytes < need)
    return set_err(SPX_EINVAL, "spx_kmeans_assign: workspace %zu < %lld bytes", workspace_bytes, (long long)need);
  const i64 Kp = kf_kp(K);
  const KmWs w = km_carve(workspace, N, D, Kp);
  HIP_TRY(hipMemsetAsync(w.counters, 0, 64, S(stream)));  // the counters and a null KmMove
  const int gp = kf_persistent_grid(N);
  if (km_screen_ok(dtype, K, D, points, ldp)) {
    // fp16 screen (A-stationary, k_kmeans_filter_as MODE 1) over every row,
    // then km_resolve over the rows it leaves undecided
    const int nct = km_nct(K);
    __bf16* CBh = (__bf16*)w.CT;
    __bf16* CBl = CBh + (i64)32 * nct * D;
    float* cnf = (float*)w.cn;
    float* cnf2 = cnf + KF_BN;  // |c'|^2 for the screen (the cn area holds 2 KF_BN floats)
    k_kmeans_prep_b3<<<1, 1024, 0, S(stream)>>>(D, K, 32 * nct, centers, CBh, CBl, cnf, w.cmax, mcoef, cnf2, w.muf);
    LAUNCH_CHECK("spx_kmeans_assign(prep)");
    const int ncu = num_cus();
    const i64 ntiles = (N + 31) / 32;
    const i64 need_scr = (ntiles + ks_waves(1) - 1) / ks_waves(1);
    const int grid_scr = (int)(need_scr < ncu ? need_scr : ncu);
    const unsigned int cgrid = (unsigned int)((ntiles + 256 * 16 - 1) / (256 * 16));
    ks_launch_n<1>(nct, S(stream), N, D, (const float*)points, ldp, CBh, CBl, cnf2, w.cmax, labels, w.counters,
                   w.full_list, w.und_mask, nullptr, nullptr, w.muf, grid_scr);
    LAUNCH_CHECK("spx_kmeans_assign(fp16 screen)");
    k_ks_compact<16><<<cgrid, 256, 0, S(stream)>>>(N, w.und_mask, nullptr, nullptr, w.scr_list, w.counters + 3);
    LAUNCH_CHECK("spx_kmeans_assign(compact)");
    return km_resolve(S(stream), N, D, K, (const float*)points, ldp, centers, labels, w, nct, r32);
  }
  k_kmeans_prep<<<1, 256, 0, S(stream)>>>(D, K, Kp, centers, w.CT, w.cn, w.cmax, mcoef);
  LAUNCH_CHECK("spx_kmeans_assign(prep)");
  const i64 gf = (N + KfProd::BM - 1) / KfProd::BM;
  const bool al = D % KF_BK == 0 && ldp % 4 == 0 && ((uintptr_t)points % 16) == 0;
  if (dtype == SPX_F32) {
    if (al) KfProd::launch<float, true>(gf, S(stream), N, D, K, Kp, points, ldp, w.CT, w.cn, w.cmax, labels,
                                        w.counters, w.full_list, w.cand_list);
    else KfProd::launch<float, false>(gf, S(stream), N, D, K, Kp, points, ldp, w.CT, w.cn, w.cmax, labels, w.counters,
                                      w.full_list, w.cand_list);
  } else {
    KfProd::launch<double, false>(gf, S(stream), N, D, K, Kp, points, ldp, w.CT, w.cn, w.cmax, labels, w.counters,
                                  w.full_list, w.cand_list);
  }
  LAUNCH_CHECK("spx_kmeans_assign(filter)");
  if (Kp == KF_BN) {
    if (dtype == SPX_F32)
      k_kmeans_cand<float, false><<<gp, 256, 0, S(stream)>>>(D, (const float*)points, ldp, centers, labels,
                                                             w.counters, w.cand_list, r32);
    else
      k_kmeans_cand<double, false><<<gp, 256, 0, S(stream)>>>(D, (const double*)points, ldp, centers, labels,
                                                              w.counters, w.cand_list, r32);
    LAUNCH_CHECK("spx_kmeans_assign(candidates)");
  }
  if (dtype == SPX_F32)
    k_kmeans_assign<float><<<gp, 256, 0, S(stream)>>>(N, D, K, (const float*)points, ldp, centers, labels, nullptr,
                                                       w.full_list, w.counters, r32);
  else
    k_kmeans_assign<double><<<gp, 256, 0, S(stream)>>>(N, D, K, (const double*)points, ldp, centers, labels,
                                                        nullptr, w.full_list, w.counters, r32);
  LAUNCH_CHECK("spx_kmeans_assign(exact)");
  return SPX_OK;
}

extern "C" int64_t spx_kmeans_accumulate_workspace(int dtype, int64_t N, int64_t D, int64_t K) {
  if ((dtype != SPX_F32 && dtype != SPX_F64) || N < 0 || D < 1 || K < 1) return -1;
  i64 G, ndb, ncb;
  ka_grid(dtype, N, D, K, &G, &ndb, &ncb);
  return G * K * D * (int64_t)sizeof(double) + G * K * (int64_t)sizeof(uint64_t);
}

extern "C" int spx_kmeans_accumulate(int dtype, int64_t N, int64_t D, int64_t K, const void* points, int64_t ldp,
                                     const int64_t* labels, double* sums, uint64_t* counts, int zero_first,
                                     void* workspace, size_t workspace_bytes, void* stream) {
  if (dtype != SPX_F32 && dtype != SPX_F64)
    return set_err(SPX_ENOTSUP, "spx_kmeans_accumulate: points must be F32/F64");
  if (N < 0 || D < 1 || K < 1 || (N > 0 && ldp < D)) return set_err(SPX_EINVAL, "spx_kmeans_accumulate: bad N/D/K/ldp");
  if (!sums || !counts) return set_err(SPX_EINVAL, "spx_kmeans_accumulate: null pointer");
  if (N == 0) {
    if (zero_first) {
      HIP_TRY(hipMemsetAsync(sums, 0, (size_t)K * D * sizeof(double), S(stream)));
      HIP_TRY(hipMemsetAsync(counts, 0, (size_t)K * sizeof(uint64_t), S(stream)));
    }
    return SPX_OK;
  }
  if (!points || !labels || !workspace) return set_err(SPX_EINVAL, "spx_kmeans_accumulate: null pointer");
  const int64_t need = spx_kmeans_accumulate_workspace(dtype, N, D, K);
  if ((int64_t)workspace_bytes < need)
    return set_err(SPX_EINVAL, "spx_kmeans_accumulate: workspace %zu < %lld bytes", workspace_bytes, (long long)need);
  i64 G, ndb, ncb;
  ka_grid(dtype, N, D, K, &G, &ndb, &ncb);
  if (ndb * ncb > 65535) return set_err(SPX_ENOTSUP, "spx_kmeans_accumulate: K*D too large");
  double* psum = (double*)workspace;
  unsigned long long* pcnt = (unsigned long long*)(psum + G * K * D);
  dim3 grid((unsigned)G, (unsigned)(ndb * ncb));
  if (dtype == SPX_F32)
    k_kmeans_accum<float><<<grid, KA_THREADS, 0, S(stream)>>>(N, D, K, (const float*)points, ldp, labels, psum, pcnt,
                                                              (int)ndb);
  else
    k_kmeans_accum<double><<<grid, KA_THREADS, 0, S(stream)>>>(N, D, K, (const double*)points, ldp, labels, psum,
                                                               pcnt, (int)ndb);
  LAUNCH_CHECK("spx_kmeans_accumulate");
  const int add = zero_first ? 0 : 1;
  const i64 n = K * D;
  k_kmeans_reduce<double><<<(unsigned)((n + 63) / 64), 256, 0, S(stream)>>>(n, G, psum, sums, add);
  LAUNCH_CHECK("spx_kmeans_accumulate(reduce sums)");
  k_kmeans_reduce<unsigned long long><<<(unsigned)((K + 63) / 64), 256, 0, S(stream)>>>(
      K, G, pcnt, (unsigned long long*)counts, add);
  LAUNCH_CHECK("spx_kmeans_accumulate(reduce counts)");
  return SPX_OK;
}

// ------------------------------------------------------- fused k-means step
// spx_kmeans_step = spx_kmeans_assign + spx_kmeans_accumulate with the same
// results (labels bit for bit; counts exact; sums deterministic, within the
// fp32-chain bound below of the fp64 sums) and, in the certified screen's
// domain, ONE pass over the points: k_kmeans_pp labels and accumulates the
// rows it decides, and accumulates the finite rows it leaves undecided (a
// few %) PROVISIONALLY under their screen-best centre; those are listed in
// row order and resolved by km_resolve, whose label writes mark the rows that
// moved (and the non-finite ones, which were not added); k_kmeans_accum then
// adds them under their final label and takes the movers out of their
// provisional centre (two short gathered passes).  Partials are combined in a
// fixed order.  Workspace: spx_kmeans_assign's | spx_kmeans_accumulate's |
// fused partial sums (G x K x D f64) | fused partial counts (G x K u64) |
// compaction block counts | slice sums | provisional centres of the movers
// (N i64) | two row masks | two list counters.
static i64 kfs_grid(i64 N) {  // one block per CU, at most one per 32-row unit
  const i64 nunits = (N + KP_U - 1) / KP_U, ncu = num_cus();
  return nunits < ncu ? (nunits < 1 ? 1 : nunits) : ncu;
}

// the step's mask compactions: one 32-row mask word per thread (KFS_TPT), so
// the gathers beside the list (label codes, k_ks_compact vals) have one or two
// rows per thread in flight, not a thread's 16 words' worth in a row (234 us
// for the list's codes at cfg3 with 16)
constexpr int KFS_TPT = 1;
static i64 kfs_nblk(i64 N) { return ((N + 31) / 32 + 256 * KFS_TPT - 1) / (256 * KFS_TPT); }

// windows of k_kmeans_pp's fp32 partials per block (the block with the most units)
static i64 kp_nwin(i64 N) {
  const i64 nunits = (N + KP_U - 1) / KP_U, G = kfs_grid(N);
  const i64 nit = (nunits + G - 1) / G, nrun = (nit + KP_LAG + KP_UNR - 1) / KP_UNR * KP_UNR;
  return (nrun - 1) / KP_FW + 1;
}

// bytes of the fused step's block partials (k_kmeans_pp's fp32 windows)
static i64 kfs_part_bytes(i64 N, i64 D, i64 K) { return kfs_grid(N) * kp_nwin(N) * K * D * 4; }

// Optional timing of the fused step (spx_kmeans_timing): HIP events around
// k_kmeans_pp and around the whole step, recorded on the caller's stream for
// up to KT_CAP calls and read back (after the timed region) by
// spx_kmeans_times -- bench.py's per-kernel roofline of the k-means leg.
constexpr int KT_CAP = 256;
// the state is process-global: one mutex serialises enable / read-back /
// record, the events belong to the device that was current at enable time
// (a step on another device records nothing and is counted in g_kt_skipped,
// reported by spx_kmeans_times as an error), and a failed event creation
// destroys the events already made
static std::mutex g_kt_mu;
static bool g_kt_on = false;
static int g_kt_n = 0, g_kt_dev = -1, g_kt_skipped = 0;
static hipEvent_t g_kt_ev[KT_CAP][4];
static void kt_destroy(int upto) {
  for (int i = 0; i < upto; ++i)
    for (int k = 0; k < 4; ++k) (void)hipEventDestroy(g_kt_ev[i][k]);
}
extern "C" int spx_kmeans_timing(int enable) {
  std::lock_guard<std::mutex> lk(g_kt_mu);
  if (enable && !g_kt_on) {
    int dev = -1;
    HIP_TRY(hipGetDevice(&dev));
    for (int i = 0; i < KT_CAP; ++i)
      for (int k = 0; k < 4; ++k) {
        const hipError_t e = hipEventCreate(&g_kt_ev[i][k]);
        if (e != hipSuccess) {
          for (int kk = 0; kk < k; ++kk) (void)hipEventDestroy(g_kt_ev[i][kk]);
          kt_destroy(i);
          return set_err(SPX_EHIP, "spx_kmeans_timing: hipEventCreate: %s", hipGetErrorString(e));
        }
      }
    g_kt_on = true;
    g_kt_dev = dev;
  } else if (!enable && g_kt_on) {
    kt_destroy(KT_CAP);
    g_kt_on = false;
    g_kt_dev = -1;
  }
  g_kt_n = 0;
  g_kt_skipped = 0;
  return SPX_OK;
}
extern "C" int spx_kmeans_times(double* fused_ms, double* step_ms, int max) {
  std::lock_guard<std::mutex> lk(g_kt_mu);
  if (!g_kt_on) return set_err(SPX_EINVAL, "spx_kmeans_times: timing is off (spx_kmeans_timing(1))");
  if (g_kt_skipped) {
    const int sk = g_kt_skipped;
    g_kt_n = 0;
    g_kt_skipped = 0;
    return set_err(SPX_EINVAL, "spx_kmeans_times: %d step(s) ran on another device than the one timing was "
                   "enabled on (%d) and were not timed", sk, g_kt_dev);
  }
  const int n = g_kt_n < max ? g_kt_n : max;
  for (int i = 0; i < n; ++i) {
    float a = 0.f, b = 0.f;
    HIP_TRY(hipEventSynchronize(g_kt_ev[i][3]));
    HIP_TRY(hipEventElapsedTime(&a, g_kt_ev[i][1], g_kt_ev[i][2]));
    HIP_TRY(hipEventElapsedTime(&b, g_kt_ev[i][0], g_kt_ev[i][3]));
    fused_ms[i] = a;
    step_ms[i] = b;
  }
  g_kt_n = 0;
  return n;
}
// k = 0 opens a step's record (on the enabling device only), 3 closes it
static void kt_record(int k, void* stream) {
  std::lock_guard<std::mutex> lk(g_kt_mu);
  if (!g_kt_on || g_kt_n >= KT_CAP) return;
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev != g_kt_dev) {
    if (k == 0) ++g_kt_skipped;
    return;
  }
  (void)hipEventRecord(g_kt_ev[g_kt_n][k], S(stream));
  if (k == 3) ++g_kt_n;
}

extern "C" int64_t spx_kmeans_step_workspace(int dtype, int64_t N, int64_t D, int64_t K) {
  const int64_t a = spx_kmeans_assign_workspace(dtype, N, D, K);
  const int64_t c = spx_kmeans_accumulate_workspace(dtype, N, D, K);
  if (a < 0 || c < 0) return -1;
  const i64 G = kfs_grid(N);
  // ... | slice sums | the moved rows' provisional centres (N i64) | 2 row
  // masks ((N / 32 + 2) u64 each) | 2 list counters
  return (a + 255) / 256 * 256 + (c + 255) / 256 * 256 + kfs_part_bytes(N, D, K) + G * K * 8 + (kfs_nblk(N) + 1) * 4 + 512 +
         (int64_t)KR_S * K * D * 8 + 256 + N * 8 + 2 * ((N + 31) / 32 + 2) * 8 + 64;
}

extern "C" int spx_kmeans_step(int dtype, int64_t N, int64_t D, int64_t K, const void* points, int64_t ldp,
                               const double* centers, int64_t* labels, double* sums, uint64_t* counts, int zero_first,
                               void* workspace, size_t workspace_bytes, int dist_dtype, void* stream) {
  if (dtype != SPX_F32 && dtype != SPX_F64) return set_err(SPX_ENOTSUP, "spx_kmeans_step: points must be F32/F64");
  if (N < 0 || D < 1 || K < 1 || (N > 0 && ldp < D)) return set_err(SPX_EINVAL, "spx_kmeans_step: bad N/D/K/ldp");
  if (dist_dtype != SPX_F64 && dist_dtype != SPX_F32)
    return set_err(SPX_EINVAL, "spx_kmeans_step: dist_dtype must be F64 or F32");
  if (!sums || !counts || !centers || (N > 0 && (!points || !labels)) || !workspace)
    return set_err(SPX_EINVAL, "spx_kmeans_step: null pointer");
  const int64_t need = spx_kmeans_step_workspace(dtype, N, D, K);
  if (need < 0 || (int64_t)workspace_bytes < need)
    return set_err(SPX_EINVAL, "spx_kmeans_step: workspace %zu < %lld bytes", workspace_bytes, (long long)need);
  const int64_t na = spx_kmeans_assign_workspace(dtype, N, D, K);
  const int64_t nc = spx_kmeans_accumulate_workspace(dtype, N, D, K);
  unsigned char* wa = (unsigned char*)workspace;
  unsigned char* wc = wa + (na + 255) / 256 * 256;
  if (N == 0 || !km_screen_ok(dtype, K, D, points, ldp)) {  // two passes: assign, then accumulate
    int rc = spx_kmeans_assign(dtype, N, D, K, points, ldp, centers, labels, nullptr, wa, (size_t)na, dist_dtype,
                               stream);
    if (rc) return rc;
    return spx_kmeans_accumulate(dtype, N, D, K, points, ldp, labels, sums, counts, zero_first, wc, (size_t)nc, stream);
  }
  const i64 Kp = kf_kp(K), G = kfs_grid(N), nb = kfs_nblk(N), ntiles = (N + 31) / 32;
  float* partF = (float*)(wc + (nc + 255) / 256 * 256);
  unsigned long long* pcntF = (unsigned long long*)((unsigned char*)partF + kfs_part_bytes(N, D, K));
  unsigned int* bcnt = (unsigned int*)(pcntF + G * K);
  const KmWs w = km_carve(wa, N, D, Kp);
  const int r32 = dist_dtype == SPX_F32;
  const double mcoef = r32 ? 4.76837158203125e-07 : 0.0;  // 2^-21
  const int nct = km_nct(K);
  const float* Pf = (const float*)points;
  __bf16* CBh = (__bf16*)w.CT;
  __bf16* CBl = CBh + (i64)32 * nct * D;
  float* cnf = (float*)w.cn;
  float* cnf2 = cnf + KF_BN;
  kt_record(0, stream);
  HIP_TRY(hipMemsetAsync(w.counters, 0, 64, S(stream)));  // the counters and a null KmMove
  k_kmeans_prep_b3<<<1, 1024, 0, S(stream)>>>(D, K, 32 * nct, centers, CBh, CBl, cnf, w.cmax, mcoef, cnf2, w.muf);
  LAUNCH_CHECK("spx_kmeans_step(prep)");
  unsigned long long* dummy = (unsigned long long*)(((uintptr_t)(bcnt + nb + 1) + 63) & ~(uintptr_t)63);
  const i64 nwin = kp_nwin(N);
  kt_record(1, stream);
  kp_launch_n(nct, (int)(D / 16), S(stream), (int)G, N, K, Pf, ldp, CBh, CBl, cnf2, w.cmax, w.muf, labels,
               w.und_mask, partF, (int)nwin, pcntF, dummy);
  LAUNCH_CHECK("spx_kmeans_step(fused screen + accumulate)");
  kt_record(2, stream);
  // the screen's undecided rows, in row order (the gathered accumulation's order)
  k_ks_count<KFS_TPT><<<(unsigned)nb, 256, 0, S(stream)>>>(N, w.und_mask, bcnt);
  k_exscan_u32<<<1, 1024, 0, S(stream)>>>(bcnt, nb, w.counters + 3);
  // the slice sums live past the compaction counts and the dummy word; the
  // moved rows' provisional centres, the two row masks and two list counters
  // past them
  const i64 n = K * D;
  double* slices = (double*)(((uintptr_t)(bcnt + nb + 1) + 64 + 255) & ~(uintptr_t)255);
  i64* pside = (i64*)(((uintptr_t)(slices + (i64)KR_S * n) + 255) & ~(uintptr_t)255);
  const i64 nw = (N + 31) / 32 + 2;
  unsigned long long* add_rows = (unsigned long long*)(pside + N);
  unsigned long long* sub_rows = add_rows + nw;
  unsigned int* mcnt = (unsigned int*)(sub_rows + nw);
  k_ks_compact<KFS_TPT, 2><<<(unsigned)nb, 256, 0, S(stream)>>>(N, w.und_mask, nullptr, nullptr, w.scr_list, nullptr, bcnt);
  LAUNCH_CHECK("spx_kmeans_step(compact)");
  (void)ntiles;
  // the list passes mark, as they write final labels, the rows to add
  // under them and the rows to take out of their provisional centre
  HIP_TRY(hipMemsetAsync(add_rows, 0, (size_t)2 * nw * 8, S(stream)));
  k_km_setmove<<<1, 64, 0, S(stream)>>>((KmMove*)(w.counters + 4), add_rows, sub_rows, pside);
  LAUNCH_CHECK("spx_kmeans_step(move bookkeeping)");
  int rc = km_resolve(S(stream), N, D, K, Pf, ldp, centers, labels, w, nct, r32);
  if (rc) return rc;
  // The list rows' sums and counts: k_kmeans_pp added every finite undecided
  // row provisionally under its screen-best centre; now that the labels are
  // final, the rows it did not add (non-finite) and the ones whose label
  // moved are added under the final label, and the movers subtracted from
  // the provisional centre -- two gathered passes over the movers instead of
  // one over the whole list (6.2 % of cfg3's rows; ~0.6 % move).  Lists in
  // slot order (count, scan, compact), partials combined in a fixed order.
  i64 G2, ndb, ncb;
  ka_grid(dtype, N, D, K, &G2, &ndb, &ncb);
  if (ndb * ncb > 65535) return set_err(SPX_ENOTSUP, "spx_kmeans_step: K*D too large");
  double* psum2 = (double*)wc;
  unsigned long long* pcnt2 = (unsigned long long*)(psum2 + G2 * K * D);
  auto listed = [&](const unsigned long long* mask, i64* out, unsigned int* cnt, const i64* vin, i64* vout) {
    k_ks_count<KFS_TPT><<<(unsigned)nb, 256, 0, S(stream)>>>(N, mask, bcnt);
    k_exscan_u32<<<1, 1024, 0, S(stream)>>>(bcnt, nb, cnt);
    k_ks_compact<KFS_TPT, 2><<<(unsigned)nb, 256, 0, S(stream)>>>(N, mask, nullptr, nullptr, out, nullptr, bcnt, vin, vout);
  };
  listed(add_rows, w.und_list, mcnt, nullptr, nullptr);
  LAUNCH_CHECK("spx_kmeans_step(compact adds)");
  k_kmeans_accum<float><<<dim3((unsigned)G2, (unsigned)(ndb * ncb)), KA_THREADS, 0, S(stream)>>>(
      N, D, K, Pf, ldp, labels, psum2, pcnt2, (int)ndb, w.und_list, mcnt);
  LAUNCH_CHECK("spx_kmeans_step(accumulate list adds)");
  if (n % 4 == 0) {
    k_kmeans_slices<<<dim3((unsigned)((n / 4 + 255) / 256), KR_S), 256, 0, S(stream)>>>(n, G * nwin, partF, slices);
    k_kmeans_reduce<double><<<(unsigned)((n + 63) / 64), 256, 0, S(stream)>>>(n, KR_S, slices, sums,
                                                                              zero_first ? 0 : 1);
  } else {
    k_kmeans_reduce<double, float><<<(unsigned)((n + 63) / 64), 256, 0, S(stream)>>>(n, G * nwin, partF, sums,
                                                                                     zero_first ? 0 : 1);
  }
  k_kmeans_reduce<double><<<(unsigned)((n + 63) / 64), 256, 0, S(stream)>>>(n, G2, psum2, sums, 1);
  k_kmeans_reduce<unsigned long long><<<(unsigned)((K + 63) / 64), 256, 0, S(stream)>>>(
      K, G, pcntF, (unsigned long long*)counts, zero_first ? 0 : 1);
  k_kmeans_reduce<unsigned long long><<<(unsigned)((K + 63) / 64), 256, 0, S(stream)>>>(
      K, G2, pcnt2, (unsigned long long*)counts, 1);
  LAUNCH_CHECK("spx_kmeans_step(reduce)");
  // the movers out of their provisional centres (the same partial buffers,
  // reused after the adds' reduce)
  i64* subp = (i64*)w.cand_list;  // the list passes are done with the candidate list
  listed(sub_rows, w.full_list, mcnt + 1, pside, subp);
  LAUNCH_CHECK("spx_kmeans_step(compact subtractions)");
  k_kmeans_accum<float><<<dim3((unsigned)G2, (unsigned)(ndb * ncb)), KA_THREADS, 0, S(stream)>>>(
      N, D, K, Pf, ldp, labels, psum2, pcnt2, (int)ndb, w.full_list, mcnt + 1, subp);
  LAUNCH_CHECK("spx_kmeans_step(accumulate list subtractions)");
  k_kmeans_reduce<double><<<(unsigned)((n + 63) / 64), 256, 0, S(stream)>>>(n, G2, psum2, sums, 2);
  k_kmeans_reduce<unsigned long long><<<(unsigned)((K + 63) / 64), 256, 0, S(stream)>>>(
      K, G2, pcnt2, (unsigned long long*)counts, 2);
  LAUNCH_CHECK("spx_kmeans_step(reduce subtractions)");
  kt_record(3, stream);
  return SPX_OK;
}

// ----------------------------------------------------- full distance matrix
// out[p * ldo + c] = cdist(P, C)[p, c] (the materialised result of
// outer((X, C), (0, 0), kmeans_dist_mapper), k_means_.py:52-58) in scipy's
// exact order as in k_kmeans_assign (sequential fp64 over d, separately
// rounded, then sqrt), rounded once to the output dtype as the reference's
// target.update does.  A block owns a 64-point x 64-centre tile; each lane
// 4 x 4 pairs, operands staged through LDS in 16-dim chunks (zero padding
// past D adds exact +0.0 terms).  Only the unfused path uses it: argmin over
// it is fused into spx_kmeans_assign (expr/optimize.py OuterArgminFusion).
#define CD_T 64
#define CD_DC 16
template <typename TP, typename TO>
__global__ __launch_bounds__(256) void k_cdist(i64 N, i64 D, i64 K, const TP* __restrict__ P, i64 ldp,
                                               const double* __restrict__ C, TO* __restrict__ out, i64 ldo) {
  __shared__ double Ps[CD_T][CD_DC + 1];
  __shared__ double Cs[CD_T][CD_DC + 1];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const i64 c0 = (i64)blockIdx.x * CD_T;
  for (i64 p0 = (i64)blockIdx.y * CD_T; p0 < N; p0 += (i64)gridDim.y * CD_T) {  // block-uniform
    double s[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) s[i][j] = 0.0;
    for (i64 d0 = 0; d0 < D; d0 += CD_DC) {
      __syncthreads();
      for (int e = threadIdx.x; e < CD_T * CD_DC; e += 256) {
        const int r = e / CD_DC, dd = e % CD_DC;
        Ps[r][dd] = (p0 + r < N && d0 + dd < D) ? (double)P[(p0 + r) * ldp + d0 + dd] : 0.0;
        Cs[r][dd] = (c0 + r < K && d0 + dd < D) ? C[(c0 + r) * D + d0 + dd] : 0.0;
      }
      __syncthreads();
#pragma unroll 4
      for (int dd = 0; dd < CD_DC; ++dd) {
        double x[4], c[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          x[i] = Ps[ty + 16 * i][dd];
          c[i] = Cs[tx + 16 * i][dd];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const double df = x[i] - c[j];
            const double sq = df * df;
            s[i][j] = s[i][j] + sq;
          }
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const i64 p = p0 + ty + 16 * i, c = c0 + tx + 16 * j;
        if (p < N && c < K) out[p * ldo + c] = (TO)sqrt(s[i][j]);
      }
  }
}

extern "C" int spx_cdist(int dtype, int out_dtype, int64_t N, int64_t D, int64_t K, const void* points, int64_t ldp,
                         const double* centers, void* out, int64_t ldo, void* stream) {
  if (dtype != SPX_F32 && dtype != SPX_F64) return set_err(SPX_ENOTSUP, "spx_cdist: points must be F32/F64");
  if (out_dtype != SPX_F32 && out_dtype != SPX_F64) return set_err(SPX_ENOTSUP, "spx_cdist: out must be F32/F64");
  if (N < 0 || D < 1 || K < 1 || (N > 0 && (ldp < D || ldo < K))) return set_err(SPX_EINVAL, "spx_cdist: bad sizes");
  if (N == 0) return SPX_OK;
  if (!points || !centers || !out) return set_err(SPX_EINVAL, "spx_cdist: null pointer");
  const i64 cb = (K + CD_T - 1) / CD_T;
  if (cb > 65535) return set_err(SPX_ENOTSUP, "spx_cdist: K too large");
  i64 pb = (N + CD_T - 1) / CD_T;
  if (pb > 65535) pb = 65535;
  dim3 grid((unsigned)cb, (unsigned)pb);
  if (dtype == SPX_F32 && out_dtype == SPX_F32)
    k_cdist<float, float><<<grid, 256, 0, S(stream)>>>(N, D, K, (const float*)points, ldp, centers, (float*)out, ldo);
  else if (dtype == SPX_F32)
    k_cdist<float, double><<<grid, 256, 0, S(stream)>>>(N, D, K, (const float*)points, ldp, centers, (double*)out, ldo);
  else if (out_dtype == SPX_F32)
    k_cdist<double, float><<<grid, 256, 0, S(stream)>>>(N, D, K, (const double*)points, ldp, centers, (float*)out, ldo);
  else
    k_cdist<double, double><<<grid, 256, 0, S(stream)>>>(N, D, K, (const double*)points, ldp, centers, (double*)out,
                                                         ldo);
  LAUNCH_CHECK("spx_cdist");
  return SPX_OK;
}

// ----------------------------------------------------------------- bincount
// counts[k] (+)= #{i : labels[i] == k}, labels outside [0, K) skipped
// (np.bincount(labels, minlength=K) of kmeans_count_mapper, k_means_.py:
// 61-64).  Integer atomics, so the result is exact and order-free: per-block
// LDS histograms when K fits (K <= BC_LDS), else global atomics.
#define BC_LDS 16384
__global__ __launch_bounds__(256) void k_bincount(i64 N, const i64* __restrict__ labels, i64 K,
                                                  unsigned long long* __restrict__ counts, int use_lds) {
  extern __shared__ unsigned int hist[];
  if (use_lds) {
    for (i64 k = threadIdx.x; k < K; k += 256) hist[k] = 0u;
    __syncthreads();
  }
  for (i64 i = (i64)blockIdx.x * 256 + threadIdx.x; i < N; i += (i64)gridDim.x * 256) {
    const i64 v = labels[i];
    if (v >= 0 && v < K) {
      if (use_lds) atomicAdd(&hist[v], 1u);
      else atomicAdd(&counts[v], 1ull);
    }
  }
  if (use_lds) {
    __syncthreads();
    for (i64 k = threadIdx.x; k < K; k += 256)
      if (hist[k]) atomicAdd(&counts[k], (unsigned long long)hist[k]);
  }
}

extern "C" int spx_bincount(const int64_t* labels, int64_t N, int64_t K, uint64_t* counts, int zero_first,
                            void* stream) {
  if (N < 0 || K < 1) return set_err(SPX_EINVAL, "spx_bincount: bad N/K");
  if (!counts || (N > 0 && !labels)) return set_err(SPX_EINVAL, "spx_bincount: null pointer");
  if (zero_first) HIP_TRY(hipMemsetAsync(counts, 0, (size_t)K * sizeof(uint64_t), S(stream)));
  if (N == 0) return SPX_OK;
  const int use_lds = K <= BC_LDS;
  int g = grid_for(N, 16);
  if (g > 4096) g = 4096;
  k_bincount<<<g, 256, use_lds ? (size_t)K * sizeof(unsigned int) : 0, S(stream)>>>(
      N, labels, K, (unsigned long long*)counts, use_lds);
  LAUNCH_CHECK("spx_bincount");
  return SPX_OK;
}

// ============================================================ JIT modules
extern "C" int spx_module_load(const void* image, size_t nbytes, void** module_out) {
  if (!image || nbytes == 0 || !module_out) return set_err(SPX_EINVAL, "spx_module_load: bad args");
  hipModule_t m = nullptr;
  HIP_TRY(hipModuleLoadData(&m, image));
  *module_out = (void*)m;
  return SPX_OK;
}

extern "C" int spx_module_unload(void* module) {
  if (!module) return SPX_OK;
  HIP_TRY(hipModuleUnload((hipModule_t)module));
  return SPX_OK;
}

extern "C" int spx_module_function(void* module, const char* name, void** fn_out) {
  if (!module || !name || !fn_out) return set_err(SPX_EINVAL, "spx_module_function: bad args");
  hipFunction_t f = nullptr;
  hipError_t e = hipModuleGetFunction(&f, (hipModule_t)module, name);
  if (e != hipSuccess)
    return set_err(SPX_EHIP, "hipModuleGetFunction(%s): %s", name, hipGetErrorString(e));
  *fn_out = (void*)f;
  return SPX_OK;
}

extern "C" int spx_launch(void* fn, uint32_t gx, uint32_t gy, uint32_t gz, uint32_t block_x,
                          uint32_t shared_bytes, const void* args, size_t args_bytes, void* stream) {
  if (!fn) return set_err(SPX_EINVAL, "spx_launch: null function");
  if (gx == 0 || gy == 0 || gz == 0) return SPX_OK;
  if (block_x == 0 || block_x > 1024) return set_err(SPX_EINVAL, "spx_launch: bad block %u", block_x);
  size_t sz = args_bytes;
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, const_cast<void*>(args), HIP_LAUNCH_PARAM_BUFFER_SIZE,
                 &sz, HIP_LAUNCH_PARAM_END};
  HIP_TRY(hipModuleLaunchKernel((hipFunction_t)fn, gx, gy, gz, block_x, 1, 1, shared_bytes, S(stream),
                                nullptr, cfg));
  return SPX_OK;
}
