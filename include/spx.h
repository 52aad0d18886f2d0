/*
 * spx.h -- C ABI of libspx.so, the MI355X (gfx950) tile-execution backend
 * underneath spartan_amd.expr.
 *
 * The reference (sdutheone/spartan) has no native boundary on its hot path:
 * every tile operation is a NumPy/BLAS call made from a Python worker
 * (spartan/expr/local.py:110-122, spartan/expr/dot.py:195-212) and tiles move
 * over pickled ZeroMQ RPC.  Each entry point below replaces one of those
 * per-tile call sites; the reference interface it replaces is cited on it.
 *
 * Conventions
 *   - Every function returns 0 on success and a negative SPX_E* code on error;
 *     spx_last_error() returns the message of the calling thread's last error.
 *   - All device memory is owned by the caller (allocated through PyTorch-ROCm
 *     on the GPU of this rank).  The library never frees caller buffers.
 *   - Every compute call is asynchronous on the given hipStream_t (passed as
 *     void*; NULL = the null stream).  Nothing here synchronises the host.
 *   - Shapes, offsets and strides are in ELEMENTS, int64, row-major.
 *   - No torch types cross this boundary: plain pointers and sizes only.
 */
#ifndef SPX_H
#define SPX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPX_ABI_VERSION 3  /* 2: spx_kmeans_assign dist_dtype; collectives; 3: spx_kmeans_step */

/* error codes */
#define SPX_OK 0
#define SPX_EINVAL -1   /* bad argument (shape / dtype / null pointer)      */
#define SPX_EHIP -2     /* HIP runtime error (message has hipGetErrorString) */
#define SPX_ENOTSUP -3  /* combination not supported by this build           */

/* element types (NumPy dtype on the Python side) */
#define SPX_BOOL 0 /* numpy.bool_  stored as uint8 0/1 */
#define SPX_I32 1  /* numpy.int32  */
#define SPX_I64 2  /* numpy.int64  */
#define SPX_F32 3  /* numpy.float32 */
#define SPX_F64 4  /* numpy.float64 */

/* reduction / merge operators (reference accumulate_fn / reducer) */
#define SPX_OP_SUM 0     /* np.add     */
#define SPX_OP_MIN 1     /* np.minimum */
#define SPX_OP_MAX 2     /* np.maximum */
#define SPX_OP_ARGMIN 3  /* (value, first index) min */
#define SPX_OP_ARGMAX 4  /* (value, first index) max */
#define SPX_OP_REPLACE 5 /* reducer None: last write wins */

/* fill kinds */
#define SPX_FILL_CONST 0   /* value a                                   */
#define SPX_FILL_ARANGE 1  /* a + b * global_flat_index                 */
#define SPX_FILL_UNIFORM 2 /* a + (b-a) * U[0,1) from splitmix64(seed,i) */
#define SPX_FILL_NORMAL 3  /* a + b * N(0,1), Box-Muller of streams 2i, 2i+1 */

/* ---------------------------------------------------------------- basics */
int spx_abi_version(void);
const char* spx_last_error(void);

/* ------------------------------------------------------------------- JIT
 * Fused map / map+reduce kernels are generated from the LocalExpr tree by
 * spartan_amd/codegen.py, compiled to a gfx950 code object, and launched
 * through these three calls.  Replaces FnCallExpr.evaluate
 * (spartan/expr/local.py:110-122) driven by tile_mapper (spartan/expr/map.py:48-88)
 * and _reduce_mapper (spartan/expr/reduce.py:19-68); the reference's own
 * codegen hook is ParakeetExpr (spartan/expr/local.py:154-200).
 */
int spx_module_load(const void* image, size_t nbytes, void** module_out);
int spx_module_unload(void* module);
int spx_module_function(void* module, const char* name, void** fn_out);
/* args points to the packed kernel-argument struct (copied by the runtime). */
int spx_launch(void* fn, uint32_t grid_x, uint32_t grid_y, uint32_t grid_z,
               uint32_t block_x, uint32_t shared_bytes, const void* args,
               size_t args_bytes, void* stream);

/* ------------------------------------------------------------------ fills
 * Replaces builtins._make_ones/_make_zeros (spartan/expr/builtins.py:370-375),
 * _arange_mapper (:404-411) and np.random.rand per tile (:29-31; the
 * reference RNG is not reproducible, ours is counter-based on the GLOBAL flat
 * index, so values do not depend on the tiling).
 * The tile is dense row-major with tile_shape; it sits at ul inside an array
 * of array_shape (ndim <= 8).
 */
int spx_fill(int dtype, int kind, void* out, int ndim, const int64_t* tile_shape,
             const int64_t* ul, const int64_t* array_shape, double a, double b,
             uint64_t seed, void* stream);

/* -------------------------------------------------------- reduce finalize
 * Combines P partial rows (part_val[P][n], accumulator dtype acc_dtype, and
 * for ARGMIN/ARGMAX part_idx[P][n] int64) into out[n] of out_dtype
 * (for ARG* ops out is int64 indices and out_val may receive the values).
 * Partials are combined in index order p = 0..P-1, so results are
 * deterministic.  Replaces the per-tile partial merge of
 * _reduce_mapper -> DistArray.update -> tile.merge
 * (spartan/expr/reduce.py:53-67, spartan/array/tile.pyx:201-298).
 */
int spx_reduce_finalize(int op, int acc_dtype, int out_dtype, const void* part_val,
                        const int64_t* part_idx, int64_t P, int64_t n, void* out,
                        void* out_val, void* stream);

/* ------------------------------------------------------------------ merge
 * dst[region] = reducer(dst[region], src) with the reference's mask rule:
 * elements whose mask byte is 0 are replaced (first write), others reduced;
 * afterwards the region's mask bytes are 1.  With full_tile_fastpath != 0 and
 * the region equal to the whole tile, the reference's fast path is used: the
 * whole tile is reduced iff mask[0] is set, else replaced
 * (spartan/array/tile.pyx:264-284).  mask may be NULL (treated as all-set
 * for op != REPLACE).  src has src_dtype and is dense with region_shape.
 */
int spx_merge(int op, int dtype, void* dst, uint8_t* mask, int ndim,
              const int64_t* dst_shape, const int64_t* region_ul,
              const int64_t* region_shape, const void* src, int src_dtype,
              int full_tile_fastpath, void* stream);

/* ------------------------------------------------------------ copy region
 * Strided N-d copy with dtype conversion: dst[dst_ul + i] = src[src_ul + i]
 * for i in copy_shape.  Replaces the stitch loop of DistArrayImpl.fetch
 * (spartan/array/distarray.py:315-365) and Tile.get (tile.pyx:69-114).
 */
int spx_copy_region(int dst_dtype, void* dst, const int64_t* dst_shape,
                    const int64_t* dst_ul, int src_dtype, const void* src,
                    const int64_t* src_shape, const int64_t* src_ul, int ndim,
                    const int64_t* copy_shape, void* stream);

/* ------------------------------------------------------------------- gemm
 * C[M,N] = alpha * A[M,K] @ B[K,N] + beta * C, row-major with leading
 * dimensions lda/ldb/ldc, dtype F32 (v_mfma_f32_32x32x2_f32) or F64
 * (v_mfma_f64_16x16x4_f64).  Replaces tiles[0].dot(tiles[1]) in
 * dot_map2_mapper (spartan/expr/dot.py:195-212), dot_outer_mapper (:217-233)
 * and dot_map2_np_mapper (:172-187).
 * Memory: C must be coarse-grained device memory (hipMalloc / a torch CUDA
 * tensor).  The fp32 kernel flushes its accumulators into C every 512
 * K-tiles (fp32 chains of <= 4096 MFMA steps at any K): with K > 8192, or
 * with beta != 0, C is updated by no-return fp32 atomic adds, which are not
 * reliably performed on fine-grained or host-coherent allocations.  One wave
 * owns each element of C, so the adds land in program order (deterministic).
 */
int spx_gemm(int dtype, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
             const void* B, int64_t ldb, void* C, int64_t ldc, double alpha,
             double beta, void* stream);

/* ------------------------------------------------- arg-reduction combine
 * Element-wise combine of R (value, index) partial sets, e.g. gathered from
 * all ranks: out_idx[n] / out_val[n] = best over r of (vals[r][n], idx[r][n]);
 * smaller (ARGMIN) / larger (ARGMAX) value wins, ties go to the smaller
 * index (first occurrence), matching the sentinel-min of _arg_mapper
 * (spartan/expr/builtins.py:610-666).
 */
int spx_argreduce_combine(int op, int dtype, const void* vals, const int64_t* idx,
                          int64_t R, int64_t n, void* out_val, int64_t* out_idx,
                          void* stream);

/* ---------------------------------------------------------------- k-means
 * Assignment step of KMeans.fit (spartan/examples/sklearn/cluster/k_means_.py:
 * 126-128): labels[p] = first argmin over c of cdist(P[p], C[c]) computed
 * exactly as scipy's fp64 euclidean cdist (sequential sum of squared
 * differences, separately rounded, then sqrt) -> bit-exact labels.  points
 * F32/F64 (N, D) with row stride ldp; centers fp64 (K, D).
 * With a workspace (>= spx_kmeans_assign_workspace(dtype, N, D, K) bytes) and
 * mindist == NULL, MFMA passes first certify the points whose nearest centre
 * is separated from the runner-up by more than a rigorous error bound (fp32
 * points, K <= 256, D % 64 == 0: an fp16 screen over every point, then a
 * bf16x3 pass over the points it leaves undecided; other shapes: one fp32
 * MFMA pass); only the remaining points run the exact-order kernel.  The
 * labels are the same bits either way.  With mindist != NULL (receives the fp64 distance)
 * or workspace == NULL every point takes the exact-order kernel.
 * dist_dtype SPX_F64: argmin of the fp64 distances; SPX_F32: argmin of the
 * distances rounded to fp32, first index on equal rounded values -- the
 * outer product's target is fp32 when the points are (map2 / outer dtype
 * None -> arrays[0].dtype, k_means_.py:126-127), and the reference rounds the
 * cdist values into it before argmin.  The certified gap then also covers
 * the rounding (exact distances more than 2 fp32 ulps apart).
 */
int64_t spx_kmeans_assign_workspace(int dtype, int64_t N, int64_t D, int64_t K);
int spx_kmeans_assign(int dtype, int64_t N, int64_t D, int64_t K, const void* points, int64_t ldp,
                      const double* centers, int64_t* labels, double* mindist, void* workspace,
                      size_t workspace_bytes, int dist_dtype, void* stream);
/* Per-centre sums (fp64, K x D) and counts (K) of the points carrying each
 * label (labels outside [0, K) are skipped), ADDED into sums/counts (which are
 * overwritten instead when zero_first != 0): replaces kmeans_center_mapper /
 * kmeans_count_mapper (k_means_.py:61-89).  No float atomics: per-block fp64
 * partials go to the caller's workspace and are summed in a fixed order, so
 * the result is deterministic.  workspace_bytes must be at least
 * spx_kmeans_accumulate_workspace(dtype, N, D, K) (< 0 on bad arguments). */
int64_t spx_kmeans_accumulate_workspace(int dtype, int64_t N, int64_t D, int64_t K);
int spx_kmeans_accumulate(int dtype, int64_t N, int64_t D, int64_t K, const void* points, int64_t ldp,
                          const int64_t* labels, double* sums, uint64_t* counts, int zero_first,
                          void* workspace, size_t workspace_bytes, void* stream);
/* One k-means iteration's device work, fused: spx_kmeans_assign (labels, bit
 * for bit the same) followed by spx_kmeans_accumulate (counts exact, sums
 * deterministic) -- the argmin of outer((X, C), kmeans_dist_mapper) plus
 * kmeans_count_mapper / kmeans_center_mapper of one KMeans.fit iteration
 * (k_means_.py:126-136).  For fp32 points with K <= 256 and D in {64, 128}
 * the decided rows are labelled AND accumulated in one pass over the points
 * (k_kmeans_pp); their sums run in fp32 per block and window of 504 32-row
 * units -- one centre's chain is as long as that centre's rows in the window,
 * ~63 on average at K = 256 on uniform data and up to 16128 when one centre
 * takes every row (K = 1 or 2, skewed data) -- and the window sums are added
 * in fp64 in a fixed order.  A row the screen cannot decide is added
 * PROVISIONALLY to its screen-best centre p when its centred norm |x - mu| is
 * at most 4 (max_c |c - mu| + |mu|), and moved in fp64 afterwards if its final
 * label differs (farther rows are gathered in fp64 instead).  So a window
 * chain holds the centre's own rows plus at most a few such movers of the
 * data's own scale, and its a-priori bound is that of an fp32 sum of <= 16128
 * terms of that scale (<= 16128 u (sum |x| + |movers|), u = 2^-24); the
 * reference's own kmeans_center_mapper sums ALL of a centre's rows in one fp32
 * chain (k_means_.py:67-89).  Measured within 1e-5 of sum |x| in every test,
 * including the long-chain cases and far undecided outliers.
 * Other shapes run the two calls.  workspace_bytes >=
 * spx_kmeans_step_workspace(dtype, N, D, K). */
int64_t spx_kmeans_step_workspace(int dtype, int64_t N, int64_t D, int64_t K);
/* Timing aid (bench / profiling): spx_kmeans_timing(1) makes every later
 * fused spx_kmeans_step record HIP events on its stream around its one-pass
 * kernel and around the whole step (up to 256 calls; 0 turns it off and frees
 * the events).  spx_kmeans_times waits for the recorded calls and writes their
 * kernel / whole-step device times (ms) in call order, clears the record and
 * returns how many it wrote (< 0 on error). */
int spx_kmeans_timing(int enable);
int spx_kmeans_times(double* fused_ms, double* step_ms, int max);
int spx_kmeans_step(int dtype, int64_t N, int64_t D, int64_t K, const void* points, int64_t ldp,
                    const double* centers, int64_t* labels, double* sums, uint64_t* counts, int zero_first,
                    void* workspace, size_t workspace_bytes, int dist_dtype, void* stream);

/* Full distance matrix out[p * ldo + c] = cdist(points, centers)[p, c] in
 * the exact order above, rounded once to out_dtype (F32/F64): the
 * materialised outer((X, C), (0, 0), kmeans_dist_mapper) (k_means_.py:52-58,
 * outer.py:14-61).  points F32/F64 (N, D) row stride ldp; centers fp64. */
int spx_cdist(int dtype, int out_dtype, int64_t N, int64_t D, int64_t K, const void* points, int64_t ldp,
              const double* centers, void* out, int64_t ldo, void* stream);
/* counts[k] (+)= number of labels equal to k (labels outside [0, K)
 * skipped; overwritten when zero_first != 0): np.bincount(labels,
 * minlength=K) of kmeans_count_mapper (k_means_.py:61-64).  Exact. */
int spx_bincount(const int64_t* labels, int64_t N, int64_t K, uint64_t* counts, int zero_first, void* stream);

/* ------------------------------------------------------ automatic tiling */
/* Host-only (no device work, callable without a GPU): the node choice on the
 * AutomaticTiling cost graph (spartan/expr/optimize.py:454-890), replacing
 * the reference's native `tiling.mincost_tiling` (spartan/expr/tiling.cc:
 * 94-132, choice procedure :31-92).  Nodes 0..t, 0 = source, t = sink;
 * edge i is eu[i] -> ev[i] with cost ecost[i] (elements moved), in insertion
 * order; split pair k = {su[k], sv[k]} (the row / column alternatives of one
 * expression).  On return chosen[u] (u < t) is 1 for the chosen nodes and
 * *total_cost (may be NULL) holds the cost.  -1 on a malformed graph. */
int spx_mincost_tiling(int32_t t, int64_t n_edges, const int32_t* eu, const int32_t* ev, const int64_t* ecost,
                       int64_t n_split, const int32_t* su, const int32_t* sv, uint8_t* chosen,
                       int64_t* total_cost);

/* ----------------------------------------------------------- collectives
 * RCCL over xGMI, one communicator per process (one process per GPU).  The
 * reference has no collectives: every exchange below replaces a pattern of
 * pickled ZeroMQ point-to-point messages merged at an owner tile --
 *   partials of an axis reduction sent to the output tiles' owners and merged
 *     with np.add / np.minimum / np.maximum (reduce.py:53-67 ->
 *     distarray.py:384-421 -> tile.pyx:201-298): spx_reduce_scatter (row-slab
 *     outputs), spx_allreduce (others);
 *   dot partials reduced to the target tile's owner (map.py:326-328 with
 *     target reducer np.add, dot.py:268-283): spx_reduce / spx_reduce_scatter;
 *   argmin / argmax (value, index) partials gathered for the device combine
 *     (builtins.py:610-666): spx_allgather;
 *   a replicated small operand (the NumPy array2 pickled into every
 *     RunKernelReq, dot.py:249-257; k-means centres, k_means_.py:150-151):
 *     spx_broadcast;
 *   DistArray.fetch / update of remote regions (distarray.py:290-421 over
 *     blob_ctx.get / update): spx_sendrecv (one grouped point-to-point batch).
 * RCCL is opened at run time: spx_comm_load(path) dlopens it (NULL path:
 * "librccl.so.1"); the compute entry points never need it.  Counts are in
 * elements of dtype; ops are SPX_OP_SUM / MIN / MAX; all calls are enqueued
 * on `stream` (in-place send == recv allowed as in RCCL). */
int spx_comm_load(const char* rccl_path);
int spx_comm_unique_id(uint8_t* out, int64_t nbytes);          /* nbytes >= 128 */
int spx_comm_init(const uint8_t* unique_id, int64_t nbytes, int rank, int world, void** comm_out);
int spx_comm_destroy(void* comm);
int spx_allreduce(void* comm, const void* send, void* recv, int64_t count, int dtype, int op, void* stream);
int spx_reduce_scatter(void* comm, const void* send, void* recv, int64_t recvcount, int dtype, int op,
                       void* stream);
int spx_allgather(void* comm, const void* send, void* recv, int64_t sendcount, int dtype, void* stream);
int spx_broadcast(void* comm, const void* send, void* recv, int64_t count, int dtype, int root, void* stream);
int spx_reduce(void* comm, const void* send, void* recv, int64_t count, int dtype, int op, int root, void* stream);
/* grouped point-to-point: nsend byte buffers to speers[i], nrecv from rpeers[i] */
int spx_sendrecv(void* comm, int nsend, const void* const* sbufs, const int64_t* sbytes, const int* speers,
                 int nrecv, void* const* rbufs, const int64_t* rbytes, const int* rpeers, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* SPX_H */
