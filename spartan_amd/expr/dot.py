"""``dot`` on MFMA (restates the decomposition of spartan/expr/dot.py:238-283).

The reference builds a ``map2`` K-split join (square / wide A): every worker
computes a full-size partial ``A[:, K_i] @ B[K_i, :]`` with BLAS
(dot_map2_mapper, dot.py:195-212) and ships it to one owner tile where the
partials are summed with ``np.add`` (map.py:326-328, tile.pyx:264-284).  Here
that contraction is one ``DotExpr`` node:

  * the rank owning B's K-block j gets A[:, K_j] (``gather_regions``: the
    reference's A column-strip fetch, distarray.py:315-365, done as one P2P
    exchange), and accumulates C_partial += A[:, K_j] @ B_j with spx_gemm
    (v_mfma_f32_32x32x2_f32 / v_mfma_f64_16x16x4_f64);
  * partials are summed across ranks by RCCL (reduce_scatter onto row-strip
    output tiles, all_reduce otherwise) instead of a serial merge at one owner.

Host NumPy operands (``dot(X, w)`` with ``w`` an ndarray, dot_map2_np_mapper
dot.py:172-187) are replicated to every GPU; each rank multiplies its own A
row strips, so the partials land on local output tiles with no exchange.
Output tiling: ``tile_hint`` if given, else the default row strips (the
reference forces a single (M, N) tile on worker 0; values are identical).
"""
import numpy as np

from .. import backend, comm, runtime
from ..config import FLAGS
from ..array import distarray, extent as ext
from ..array.distarray import LocalWrapper
from .base import Expr, as_array


def _shape(a, b):
  if len(a.shape) == 1 and len(b.shape) == 1:
    if a.shape[0] != b.shape[0]:
      raise ValueError('objects are not aligned')
    return (1,)
  if len(a.shape) > 1 and len(b.shape) == 1:
    if a.shape[1] != b.shape[0]:
      raise ValueError('objects are not aligned')
    return (a.shape[0],)
  if len(a.shape) > 1 and len(b.shape) > 1:
    if a.shape[1] != b.shape[0]:
      raise ValueError('objects are not aligned')
    return (a.shape[0], b.shape[1])
  raise ValueError('objects are not aligned')


class DotExpr(Expr):
  _members = ('matrix_a', 'matrix_b')

  def compute_shape(self):
    return _shape(self.matrix_a, self.matrix_b)

  def compute_dtype(self):
    return np.result_type(self.matrix_a.dtype, self.matrix_b.dtype)

  def pretty_str(self):
    return 'Dot[%d](%s, %s)' % (self.expr_id, self.matrix_a, self.matrix_b)

  def _evaluate(self, deps):
    a, b = deps['matrix_a'], deps['matrix_b']
    if isinstance(a, np.ndarray):
      a = LocalWrapper(a)
    if isinstance(b, np.ndarray):
      b = LocalWrapper(b)
    return run_dot(a, b, getattr(self, 'tile_hint', None))


def dot(a, b, tile_hint=None):
  """Matrix / vector product of two arrays (dot.py:238-283)."""
  from ..array.distarray import DistArray
  if not isinstance(b, (Expr, np.ndarray, DistArray)):  # forced DistArrays stay device operands
    b = np.asarray(b)
  e = DotExpr(matrix_a=as_array(a), matrix_b=as_array(b) if not isinstance(b, np.ndarray) else b)
  e.tile_hint = tile_hint
  e.compute_shape()  # raises ValueError early on misalignment, as the reference
  return e


# ---------------------------------------------------------------- engine
class _As2D:
  """2-d view of a 1-d array: 'row' (1, K) for the left operand, 'col' (K, 1) for the right."""

  def __init__(self, arr, kind):
    self.arr, self.kind = arr, kind
    if len(arr.shape) == 2:
      self.shape = tuple(arr.shape)
    elif kind == 'row':
      self.shape = (1, arr.shape[0])
    else:
      self.shape = (arr.shape[0], 1)

  def to_base(self, region2):
    if len(self.arr.shape) == 2:
      return region2
    d = 1 if self.kind == 'row' else 0
    return ext.create((region2.ul[d],), (region2.lr[d],), self.arr.shape)

  def tiles2(self):
    """{2-d extent: worker} of the underlying array."""
    out = {}
    for ex, w in self.arr.tiles.items():
      if len(self.arr.shape) == 2:
        out[ex] = w
      elif self.kind == 'row':
        out[ext.create((0, ex.ul[0]), (1, ex.lr[0]), self.shape)] = w
      else:
        out[ext.create((ex.ul[0], 0), (ex.lr[0], 1), self.shape)] = w
    return out


def _as_dtype(t, dt):
  """Dense ``dt`` tensor of ``t`` (a strided view, e.g. a transpose, is made
  dense by the identity-map kernel; GEMM operands are row-major)."""
  return backend.get().contiguous(t, dt)


SKINNY_N = 4


def _skinny(at, bk, dtype):
  """A (R, K) @ B (K, n) for n <= 4: per column, a generated fused
  multiply + row-sum (packed-rows reduce), which streams A at HBM rate instead
  of padding an MFMA tile to 128 columns."""
  import torch
  from .. import codegen
  R, K = at.shape
  n = bk.shape[1]
  dt = np.dtype(dtype)
  root = codegen.Op('multiply', [codegen.In(0, dt), codegen.In(1, dt)])
  be = backend.get()
  cols = []
  for j in range(n):
    bj = bk[:, j].reshape(1, K)  # a strided column: the kernel reads it in place
    cols.append(be.reduce(root, 'sum', {0: at, 1: bj}, (R, K), 1, (R,), dt))
  if n == 1:
    return cols[0].reshape(R, 1)
  out = torch.empty((R, n), dtype=backend.torch_dtype(dt), device=at.device)
  for j, c in enumerate(cols):
    be.copy_region(out, (0, j), c.reshape(R, 1), (0, 0), (R, 1))
  return out


def run_dot(a, b, tile_hint=None):
  import torch
  ctx = runtime.get()
  be = backend.get()
  out_shape = _shape(a, b)
  dtype = np.result_type(a.dtype, b.dtype)
  A, B = _As2D(a, 'row'), _As2D(b, 'col')
  M, K = A.shape
  N = B.shape[1]
  C = None
  if b.replicated and not a.replicated:
    # X @ w with w on every GPU: local row strips of X -> local output rows
    Bd = _as_dtype(b.fetch(ext.from_shape(b.shape)).reshape(K, N), dtype)
    partials = {}
    for ex2, w in A.tiles2().items():
      if not ctx.is_local(w):
        continue
      at = _as_dtype(a.fetch(A.to_base(ex2)).reshape(ex2.shape), dtype)
      bk = Bd[ex2.ul[1]:ex2.lr[1]]
      if N <= SKINNY_N and np.dtype(dtype).kind == 'f':
        partials[ex2] = _skinny(at, bk, dtype)
      else:
        ct = torch.empty((ex2.shape[0], N), dtype=backend.torch_dtype(dtype), device=ctx.device)
        be.gemm(at, be.contiguous(bk), ct, 1.0, 0.0)
        partials[ex2] = ct
    return _combine_rows(partials, A, M, N, out_shape, dtype, tile_hint, k_split=any(
        ex.ul[1] != 0 or ex.lr[1] != K for ex in A.tiles2()))
  btiles = B.tiles2() if not b.replicated else {ext.from_shape((K, N)): -1}
  # no zero fill of the (M, N) partial: the first GEMM into each column
  # block runs with beta = 0, and only column blocks this rank computes
  # nothing for are zeroed (a rank without local B blocks)
  col_blocks = sorted({(bex.ul[1], bex.lr[1]) for bex in btiles})
  if _blocks_disjoint(col_blocks):
    C = torch.empty((M, N), dtype=backend.torch_dtype(dtype), device=ctx.device)
    started = set()
  else:
    # B's column splits differ between K bands: a later block's beta = 0
    # would overwrite an overlapping earlier one -- accumulate into zeros
    C = torch.zeros((M, N), dtype=backend.torch_dtype(dtype), device=ctx.device)
    started = _ALWAYS_STARTED
  requests, plan = [], []
  for bex, w in btiles.items():
    dst = ctx.owner(w) if w != -1 else None
    a_region = ext.create((0, bex.ul[0]), (M, bex.lr[0]), (M, K))
    if dst is None:  # replicated B and A: rank 0 computes
      dst = 0
    requests.append((A.to_base(a_region), dst))
    plan.append((bex, dst))
  output = distarray.create(out_shape, dtype, reducer=np.add, tile_hint=tile_hint)
  if ctx.distributed and len(out_shape) == 2 and FLAGS.dot_overlap and _owner_slabs(output, ctx, M):
    return _dot_overlapped(output, a, A, plan, b, B, K, M, N, dtype, C, col_blocks)
  got = distarray.gather_regions(a, requests)
  for qi, (bex, dst) in enumerate(plan):
    if dst != ctx.rank:
      continue
    at = _as_dtype(got[qi].reshape(M, bex.shape[0]), dtype)
    if b.replicated:
      bt = b.fetch(ext.from_shape(b.shape)).reshape(K, N)
    else:
      bt = b.fetch(B.to_base(bex)).reshape(bex.shape)
    bt = _as_dtype(bt, dtype)
    cview = C[:, bex.ul[1]:bex.lr[1]]
    key = (bex.ul[1], bex.lr[1])
    beta = 0.0 if key not in started else 1.0
    started.add(key)
    be.gemm(at, bt, cview, 1.0, beta)
  for c0, c1 in col_blocks:
    if (c0, c1) not in started:
      C[:, c0:c1].zero_()
  _scatter_full(output, C.reshape(out_shape), 'sum')
  return output


OVERLAPPED_CALLS = 0  # how often the overlapped path ran (tests check it is taken)


class _AlwaysStarted(set):
  """'Every column block already started': beta = 1 for every GEMM (C zeroed)."""

  def __contains__(self, key):
    return True

  def add(self, key):
    pass


_ALWAYS_STARTED = _AlwaysStarted()


def _blocks_disjoint(col_blocks):
  """True when the distinct (c0, c1) column ranges do not overlap (sorted input):
  then the first GEMM into each range may run with beta = 0."""
  return all(col_blocks[i][1] <= col_blocks[i + 1][0] for i in range(len(col_blocks) - 1))


def _owner_slabs(output, ctx, M):
  from .engine import _rank_slabs
  return _rank_slabs(output, ctx) and M % ctx.world_size == 0


# slab gathers in flight ahead of the GEMM that consumes them (_dot_overlapped)
GATHER_AHEAD = 2


def _dot_overlapped(output, a, A, plan, b, B, K, M, N, dtype, C, col_blocks):
  """K-split partials reduced slab by slab while the next slab computes, the
  A column strip gathered slab by slab ahead of its GEMM.

  The output is one row slab per rank.  For every slab j (in the same order
  on every rank) the rank needs rows j of its A column strip A[:, K_g]: the
  piece that the owner of A's rows j holds.  The slab gathers run
  GATHER_AHEAD slabs ahead of the GEMMs on the side stream
  (comm.exchange_async; a piece of whole rows is received straight into its
  buffer): slabs 0 .. GATHER_AHEAD - 1 are posted first, and the gather of
  slab j + GATHER_AHEAD right after the reduce of slab j, so slab j + 1's
  rows travel while slab j's GEMM runs and -- on one communication stream,
  where collectives run in posting order -- the reduce of slab j is not
  queued behind the gathers of every later slab (round-6 advisor).  The
  local piece needs no transfer at all when A is row-strip tiled.  After the
  partial of slab j is computed (MFMA GEMM into C[slab j]) an RCCL reduce of
  it to its owner j starts on the side stream, under the GEMM of slab j + 1.
  The bytes moved equal the gather + reduce-scatter's, but the xGMI time
  hides behind the GEMMs (measured per-rank GEMMs, predicted N = 8
  time).  Reference: dot.py:268-283 (map2 K-split, partials summed at the
  target tile), map.py:326-328."""
  global OVERLAPPED_CALLS
  OVERLAPPED_CALLS += 1
  ctx = runtime.get()
  be = backend.get()
  slab = M // ctx.world_size
  W = ctx.world_size
  # slab j's request list: the rows of slab j of every K block's A strip
  reqs = [[(A.to_base(ext.create((j * slab, bex.ul[0]), ((j + 1) * slab, bex.lr[0]), (M, K))), dst)
           for bex, dst in plan] for j in range(W)]
  pending = [None] * W
  for j in range(min(GATHER_AHEAD, W)):
    pending[j] = distarray.gather_regions_async(a, reqs[j])
  local_b = []
  for qi, (bex, dst) in enumerate(plan):
    if dst != ctx.rank:
      continue
    if b.replicated:
      bt = b.fetch(ext.from_shape(b.shape)).reshape(K, N)
    else:
      bt = b.fetch(B.to_base(bex)).reshape(bex.shape)
    local_b.append((qi, bex, _as_dtype(bt, dtype)))
  handles = []
  disjoint = _blocks_disjoint(col_blocks)  # (else the caller made C zeros)
  for j in range(W):
    r0, r1 = j * slab, (j + 1) * slab
    got = pending[j].finish()
    pending[j] = None
    started = set() if disjoint else _ALWAYS_STARTED
    for qi, bex, bt in local_b:
      at = _as_dtype(got[qi].reshape(slab, bex.shape[0]), dtype)
      key = (bex.ul[1], bex.lr[1])
      be.gemm(at, bt, C[r0:r1, key[0]:key[1]], 1.0, 0.0 if key not in started else 1.0)
      started.add(key)
    del got
    for c0, c1 in col_blocks:
      if (c0, c1) not in started:
        C[r0:r1, c0:c1].zero_()
    handles.append(comm.reduce_async(C[r0:r1], j, 'sum'))
    if j + GATHER_AHEAD < W:
      pending[j + GATHER_AHEAD] = distarray.gather_regions_async(a, reqs[j + GATHER_AHEAD])
  comm.wait_all(handles)
  (d, t), = output.local.items()
  t.data = C[ctx.rank * slab:(ctx.rank + 1) * slab].clone()  # free the full-size partial buffer
  t.written = [d]
  return output


def _scatter_full(output, full, op):
  """Sum the per-rank full buffers and deliver each output tile to its owner."""
  from .engine import _copy_out, _rank_slabs
  ctx = runtime.get()
  be = backend.get()
  if not ctx.distributed and len(output.local) == 1:
    (d, t), = output.local.items()
    if tuple(d.ul) == (0,) * len(output.shape) and tuple(t.shape) == tuple(output.shape):
      t.data = full.reshape(t.shape) if full.is_contiguous() else full.contiguous().reshape(t.shape)
      t.written = [d]
      return
  if ctx.distributed:
    if _rank_slabs(output, ctx):
      from .engine import COMBINE_CALLS
      COMBINE_CALLS['reduce_scatter'] += 1
      (d, t), = output.local.items()
      comm.reduce_scatter_rows(t.data, full.contiguous(), op)
      t.written = [d]
      return
    comm.all_reduce(full, op)
  for d, t in output.local.items():
    _copy_out(be, t, full.contiguous(), d)


def _combine_rows(partials, A, M, N, out_shape, dtype, tile_hint, k_split):
  """Row-block partials {A extent: (rows, N) tensor} -> output DistArray."""
  import torch
  ctx = runtime.get()
  be = backend.get()
  output = distarray.create(out_shape, dtype, reducer=np.add, tile_hint=tile_hint)
  two_d = len(out_shape) == 2
  # aligned: every A row block is exactly an output tile of the same rank, no K split
  aligned = not k_split
  if aligned:
    for ex2, w in A.tiles2().items():
      d = ext.create((ex2.ul[0], 0), (ex2.lr[0], N), (M, N)) if two_d else \
          ext.create((ex2.ul[0],), (ex2.lr[0],), out_shape)
      if d not in output.tiles or ctx.owner(output.tiles[d]) != ctx.owner(w):
        aligned = False
        break
  if aligned:
    for ex2, ct in partials.items():
      d = ext.create((ex2.ul[0], 0), (ex2.lr[0], N), (M, N)) if two_d else \
          ext.create((ex2.ul[0],), (ex2.lr[0],), out_shape)
      t = output.local[d]
      t.data = ct.reshape(t.shape)
      t.written = [d]
    return output
  full = torch.zeros((M, N), dtype=backend.torch_dtype(dtype), device=ctx.device)
  for ex2, ct in partials.items():
    be.merge(full, None, (ex2.ul[0], 0), ct, 'sum', fastpath=False)
  _scatter_full(output, full.reshape(out_shape), 'sum')
  return output
