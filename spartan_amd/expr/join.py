"""``map2`` and ``outer``: tile joins (restate spartan/expr/map.py:285-402 and
spartan/expr/outer.py:14-120).

The reference runs a user mapper on every join instance (a tile of
``arrays[0]`` with the matching tiles of the other arrays) with NumPy on a
worker and merges what it yields, ``(extent, value)`` pairs, into the target
with the target's reducer.  Here a mapper becomes device work in one of two
ways, never a host fallback:

  * registered joins (``register_join``): mappers whose job is a known
    kernel -- the k-means distance / count / centre mappers
    (examples/kmeans.py), ``bincount`` and ``concatenate`` (builtins) -- run
    as one kernel per local tile plus an RCCL combine;
  * any other mapper is TRACED once per join instance with symbolic tiles
    (expr/local.py Sym): each yielded value must be an elementwise
    expression of the fetched tiles (or a host constant), which becomes one
    generated gfx950 kernel; a mapper that does anything else raises
    ``CodegenError``.

Join instances follow the reference: for ``map2`` one per tile of
``arrays[0]`` with the other arrays' extents re-partitioned along ``axes``
(``join_mapper``); for ``outer`` one per (tile of ``arrays[0]``, distinct
re-partitioned tile of ``arrays[1]``) pair (``outer_mapper``).  The
instance's inputs reach the owner of the ``arrays[0]`` tile by one
``gather_regions`` exchange per array; yielded pieces travel to the owners
of the target tiles they overlap by one point-to-point batch and are merged
there in instance order (tile merge rule, tile.pyx:201-298).
"""
import numpy as np

from .. import backend, codegen, comm, runtime
from ..array import distarray, extent as ext
from .base import Expr, TupleExpr, as_array
from .local import CodegenError, LowerEnv, Sym

_JOINS = {}


def register_join(fn, impl):
  """``impl(kind, arrays, axes, fn_kw, target) -> None`` fills ``target``
  (a fresh DistArray of the join's shape / dtype / reducer) for mapper ``fn``."""
  _JOINS[fn] = impl
  return fn


class _JoinExpr(Expr):
  _members = ('arrays',)
  kind = None

  def compute_shape(self):
    return tuple(self.out_shape)

  def compute_dtype(self):
    return np.dtype(self.out_dtype) if self.out_dtype is not None else np.dtype(self.arrays.vals[0].dtype)

  def pretty_str(self):
    return '%s[%d](%s)' % (type(self).__name__, self.expr_id, getattr(self.fn, '__name__', self.fn))

  def _evaluate(self, deps):
    arrays = [distarray.as_array(a) for a in deps['arrays']]
    target = distarray.create(self.out_shape, self.compute_dtype(), reducer=self.reducer, tile_hint=self.tile_hint)
    impl = _JOINS.get(self.fn)
    if impl is not None:
      impl(self.kind, arrays, self.axes, dict(self.fn_kw or {}), target)
    else:
      run_traced_join(self.kind, arrays, self.axes, self.fn, dict(self.fn_kw or {}), target)
    return target


_ARGMIN_FUSIONS = {}


def register_argmin_fusion(fn, impl, dtypes=(np.float64,)):
  """``argmin(outer(arrays, (0, 0), fn), axis=1)`` may run as
  ``impl(arrays, fn_kw, labels_target, dist_dtype)`` without materialising
  the outer product, when the outer's result dtype is one of ``dtypes`` (the
  fused kernel must give the argmin of exactly those values, i.e. of the
  mapper's values rounded to ``dist_dtype``)."""
  _ARGMIN_FUSIONS[fn] = (impl, tuple(np.dtype(d) for d in dtypes))


def argmin_fusion_for(outer_expr):
  entry = _ARGMIN_FUSIONS.get(outer_expr.fn)
  if entry is None or tuple(outer_expr.axes) != (0, 0) or len(outer_expr.out_shape) != 2:
    return None
  impl, dtypes = entry
  return impl if outer_expr.compute_dtype() in dtypes else None


class ArgminJoinExpr(Expr):
  """argmin over axis 1 of an outer product, evaluated by a fused
  registered kernel (OuterArgminFusion); keeps the argmin node's expr_id."""
  _members = ('arrays',)

  def compute_shape(self):
    return (self.outer.out_shape[0],)

  def compute_dtype(self):
    return np.dtype(np.int64)

  def pretty_str(self):
    return 'ArgminJoin[%d](%s)' % (self.expr_id, getattr(self.outer.fn, '__name__', self.outer.fn))

  def _evaluate(self, deps):
    arrays = [distarray.as_array(a) for a in deps['arrays']]
    target = distarray.create(self.compute_shape(), np.int64, reducer=np.minimum, tile_hint=self.tile_hint)
    self.impl(arrays, dict(self.outer.fn_kw or {}), target, self.outer.compute_dtype())
    return target


class Map2Expr(_JoinExpr):
  kind = 'map2'


class OuterProductExpr(_JoinExpr):
  kind = 'outer'


def _iterable(v):
  return isinstance(v, (list, tuple))


def map2(arrays, axes=(), fn=None, fn_kw=None, shape=None, tile_hint=None, dtype=None, reducer=None):
  """Join ``arrays`` tile by tile along ``axes`` and merge what ``fn`` yields
  into a new array of ``shape`` (map.py:373-402)."""
  if not _iterable(arrays):
    arrays = [arrays]
  if not _iterable(axes):
    axes = [axes]
  assert fn is not None
  assert len(axes) == 0 or len(arrays) == len(axes)
  assert shape is not None
  return Map2Expr(arrays=TupleExpr(vals=tuple(as_array(a) for a in arrays)), axes=tuple(axes), fn=fn,
                  fn_kw=fn_kw, out_shape=tuple(shape), tile_hint=tile_hint, out_dtype=dtype, reducer=reducer)


def outer(arrays, axes, fn, fn_kw=None, shape=None, tile_hint=None, reducer=None, dtype=None):
  """Cartesian join of the tiles of ``arrays[0]`` and ``arrays[1]``
  (outer.py:104-120)."""
  assert fn is not None
  assert shape is not None
  return OuterProductExpr(arrays=TupleExpr(vals=tuple(as_array(a) for a in arrays)), axes=tuple(axes), fn=fn,
                          fn_kw=fn_kw, out_shape=tuple(shape), tile_hint=tile_hint, out_dtype=dtype, reducer=reducer)


# ------------------------------------------------------------ instances
def _sorted_tiles(array):
  return sorted(array.tiles.items(), key=lambda kv: tuple(kv[0].ul))


def join_instances(kind, arrays, axes):
  """[(owner worker, [extent per input])] -- the reference's join_mapper /
  outer_mapper enumeration, identical on every rank."""
  out = []
  if kind == 'map2':
    for ex, w in _sorted_tiles(arrays[0]):
      if len(axes) == 0:
        out.append((w, [ext.create(ex.ul, ex.lr, a.shape) for a in arrays], ex))
        continue
      first = ext.change_partition_axis(ex, axes[0])
      if first is None:
        continue
      k0, k1 = first.ul[axes[0]], first.lr[axes[0]]
      exs = [first]
      for a, ax in zip(arrays[1:], axes[1:]):
        ul = [0] * len(a.shape)
        lr = list(a.shape)
        ul[ax], lr[ax] = k0, k1
        exs.append(ext.create(ul, lr, a.shape))
      out.append((w, exs, exs))
    return out
  for ex, w in _sorted_tiles(arrays[0]):
    first = ext.change_partition_axis(ex, axes[0])
    if axes[1] is None:
      out.append((w, [first, ext.from_shape(arrays[1].shape)], None))
      continue
    done = set()
    for key, _ in _sorted_tiles(arrays[1]):
      oex = ext.change_partition_axis(key, axes[1])
      if oex is None or (oex.ul, oex.lr) in done:
        continue
      done.add((oex.ul, oex.lr))
      out.append((w, [first, oex], None))
  return out


# --------------------------------------------------------------- tracing
def _trace(kind, fn, exs, join_arg, dtypes, fn_kw):
  """Run ``fn`` on symbolic tiles; returns (env, [(target extent, value)])
  with value an IR root, a host ndarray or a scalar."""
  env = LowerEnv({})
  syms = []
  for i, (e, dt) in enumerate(zip(exs, dtypes)):
    s = Sym(codegen.In(i, dt), env)
    s.shape = tuple(e.shape)
    syms.append(s)
  try:
    if kind == 'map2':
      res = fn(join_arg, syms, **fn_kw)
    else:
      res = fn(exs[0], syms[0], exs[1], syms[1], **fn_kw)
    pieces = list(res) if res is not None else []
  except CodegenError:
    raise
  except Exception as e:
    raise CodegenError('join mapper %s cannot be lowered to a gfx950 kernel (%s: %s)'
                       % (getattr(fn, '__name__', fn), type(e).__name__, e))
  out = []
  for tex, v in pieces:
    if isinstance(v, Sym):
      want = tuple(tex.shape) if tex.ndim else ()
      if v.shape is not None and tuple(v.shape) != want:
        raise CodegenError('join mapper %s yielded a %s value for a %s extent'
                           % (getattr(fn, '__name__', fn), tuple(v.shape), want))
      out.append((tex, v.node))
    elif isinstance(v, (np.ndarray, np.generic, int, float, bool)):
      out.append((tex, np.asarray(v)))
    else:
      raise CodegenError('join mapper %s yielded %s' % (getattr(fn, '__name__', fn), type(v).__name__))
  return env, out


def _compact(root):
  """Renumber the array leaves of ``root`` to 0..n-1; returns {new: old}."""
  used = sorted({n.slot for n in codegen.walk(root) if isinstance(n, codegen.In)})
  remap = {old: i for i, old in enumerate(used)}
  for n in codegen.unique_nodes(root):
    if isinstance(n, codegen.In):
      n.slot = remap[n.slot]
  return {i: old for old, i in remap.items()}


def run_traced_join(kind, arrays, axes, fn, fn_kw, target):
  import torch
  ctx = runtime.get()
  be = backend.get()
  insts = join_instances(kind, arrays, axes)
  dtypes = [np.dtype(a.dtype) for a in arrays]
  traced = [_trace(kind, fn, exs, join_arg if kind == 'map2' else None, dtypes, fn_kw)
            for (w, exs, join_arg) in insts]
  # inputs of the local instances: one collective exchange per array
  got = []
  for i, a in enumerate(arrays):
    got.append(distarray.gather_regions(a, [(exs[i], ctx.owner(w) if w != -1 else ctx.rank)
                                            for (w, exs, _) in insts]))
  # updates: (instance, piece) -> target tiles; computed on the instance owner
  updates = []  # (order, target region, src rank, tensor or None)
  for qi, ((w, exs, _), (env, pieces)) in enumerate(zip(insts, traced)):
    src = ctx.owner(w) if w != -1 else ctx.rank
    for k, (tex, val) in enumerate(pieces):
      if tex.array_shape is not None and tuple(tex.array_shape) != tuple(target.shape):
        raise CodegenError('join mapper yielded an extent of shape %s for a %s target'
                           % (tex.array_shape, target.shape))
      t = None
      if src == ctx.rank:
        shape = tex.shape if tex.ndim else ()
        if isinstance(val, np.ndarray):
          from ..array import transfer
          t = transfer.upload(np.broadcast_to(val.astype(target.dtype), shape), ctx.device)
        else:
          slots = _compact(val)
          inputs = {new: got[old][qi] for new, old in slots.items()}
          t = torch.empty(shape, dtype=backend.torch_dtype(val.dtype), device=ctx.device)
          be.map(val, inputs, t)
      updates.append(((qi, k), tex, src, t))
  _scatter_updates(target, updates)


def _scatter_updates(target, updates):
  """Deliver every yielded piece to the owners of the target tiles it
  overlaps and merge them there in instance order.  Collective."""
  import torch
  ctx = runtime.get()
  be = backend.get()
  tdt = backend.torch_dtype(target.dtype)
  sends, recvs, merges = [], [], []
  for order, tex, src, t in updates:
    if t is not None and t.dtype != tdt:  # pieces travel in the target dtype (the merge casts anyway)
      conv = torch.empty(t.shape, dtype=tdt, device=t.device)
      be.copy_region(conv, (0,) * t.dim(), t, (0,) * t.dim(), tuple(t.shape))
      t = conv
    if not tex.ndim:
      pairs = [(tile_ex, tex) for tile_ex in target.tiles]
    else:
      pairs = list(ext.find_overlapping(target.tiles, tex))
    for tile_ex, region in pairs:
      dst = ctx.owner(target.tiles[tile_ex])
      if src == ctx.rank:
        piece = t
        if tex.ndim and region != tex:
          rel = tuple(u - o for u, o in zip(region.ul, tex.ul))
          piece = torch.empty(region.shape, dtype=tdt, device=t.device)
          be.copy_region(piece, (0,) * region.ndim, t, rel, region.shape)
        if dst == ctx.rank:
          merges.append((order, tile_ex, region, piece))
        else:
          sends.append((piece, dst))
      elif dst == ctx.rank:
        buf = torch.empty(region.shape if region.ndim else (), dtype=tdt, device=ctx.device)
        recvs.append((buf, src))
        merges.append((order, tile_ex, region, buf))
  comm.exchange(sends, recvs)
  for order, tile_ex, region, piece in sorted(merges, key=lambda m: m[0]):
    tile = target.local[tile_ex]
    if not tile.written and region == tile_ex and tuple(region.lr) == tuple(tile_ex.lr) \
        and piece.is_contiguous() and tuple(piece.shape) == tuple(tile.shape):
      tile.data = piece  # first write of a whole tile: adopt the piece, no copy
      tile.written = [tile_ex]
      continue
    target.update(region, piece)
