"""NumPy-style builtins (the hot-path subset of spartan/expr/builtins.py).

Creation: ``ones`` / ``zeros`` (:378-401), ``rand`` / ``randn`` (:72-104), ``arange``
(:404-463) -- each a map over an ``ndarray`` placeholder whose mapper has a
registered lowering (constants, or a generator leaf filled by spx_fill).
Reductions: ``sum`` / ``max`` / ``min`` / ``mean`` (:466-539), ``argmin`` /
``argmax`` (:610-666), ``count_nonzero`` / ``count_zero`` (:669-711).
Elementwise: ``add`` ... ``abs`` (:779-812), ``astype`` (:732-747).

``rand`` differs from the reference on purpose: the reference draws from
np.random per tile with per-worker seeds (not reproducible, worker.py:55);
here every element is splitmix64(seed, global flat index) -> U[0,1), so values
are independent of tiling and device and are reproduced bit-exactly by the
oracle.

``argmin`` / ``argmax`` are a single fused (value, first-index) reduction
instead of the reference's min -> location-map -> min composition; the result
(int64 global index of the first occurrence, global flat index for
axis=None) is the same for the row-strip tilings the reference produces.
"""
import itertools

import numpy as np

from .. import backend, codegen
from ..config import FLAGS
from . import engine
from .local import CodegenError, Pre, register_lowering
from .map import map
from .ndarray import ndarray
from .optimize import not_idempotent
from .reduce import reduce

_seed_counter = itertools.count(1)


def _leaf_of(op, env, i=0):
  from .local import lower
  return lower(op.deps[i], env)


# ---------------------------------------------------------------- creation
def _make_ones(input):
  return np.ones(input.shape, input.dtype)


def _make_zeros(input):
  return np.zeros(input.shape, input.dtype)


register_lowering(_make_ones, lambda op, env: codegen.Const(1, _leaf_of(op, env).dtype))
register_lowering(_make_zeros, lambda op, env: codegen.Const(0, _leaf_of(op, env).dtype))


def zeros(shape, dtype=np.float64, tile_hint=None):
  return map(ndarray(shape, dtype=dtype, tile_hint=tile_hint), fn=_make_zeros)


def ones(shape, dtype=np.float64, tile_hint=None):
  return map(ndarray(shape, dtype=dtype, tile_hint=tile_hint), fn=_make_ones)


def _make_rand(input, seed=0, low=0.0, high=1.0):
  raise CodegenError('_make_rand is lowered to spx_fill, never called')


def _lower_rand(op, env):
  leaf = _leaf_of(op, env)
  kw = op.kw
  return Pre('uniform', leaf.dtype, (backend.FILL_UNIFORM, float(kw.get('low', 0.0)),
                                     float(kw.get('high', 1.0)), int(kw['seed'])), None)


register_lowering(_make_rand, _lower_rand)


def _new_seed(seed):
  if seed is not None:
    return int(seed)
  return (int(FLAGS.rng_seed) * 1000003 + next(_seed_counter)) & 0xFFFFFFFFFFFF


@not_idempotent
def rand(*shape, **kw):
  """U[0,1) array (default float64).  Extra keywords of this build: ``dtype``,
  ``seed``, ``low``, ``high``."""
  tile_hint = kw.pop('tile_hint', None)
  dtype = kw.pop('dtype', np.float64)
  seed = _new_seed(kw.pop('seed', None))
  low = kw.pop('low', 0.0)
  high = kw.pop('high', 1.0)
  assert not kw, 'Unknown keywords %s' % kw
  for s in shape:
    assert isinstance(s, (int, np.integer))
  return map(ndarray(shape, dtype=dtype, tile_hint=tile_hint), fn=_make_rand,
             fn_kw={'seed': seed, 'low': low, 'high': high})


def _make_randn(input, seed=0):
  raise CodegenError('_make_randn is lowered to spx_fill, never called')


register_lowering(_make_randn, lambda op, env: Pre('normal', _leaf_of(op, env).dtype,
                                                   (backend.FILL_NORMAL, 0.0, 1.0, int(op.kw['seed'])), None))


@not_idempotent
def randn(*shape, **kw):
  """Standard normal array (float64; builtins.py:92-104).  Like ``rand``,
  values come from the counter-based splitmix64 stream (Box-Muller of the
  draws 2i and 2i+1), so they do not depend on tiling or device.  Extra
  keywords of this build: ``dtype``, ``seed``."""
  tile_hint = kw.pop('tile_hint', None)
  dtype = kw.pop('dtype', np.float64)
  seed = _new_seed(kw.pop('seed', None))
  assert not kw, 'Unknown keywords %s' % kw
  for s in shape:
    assert isinstance(s, (int, np.integer))
  return map(ndarray(shape, dtype=dtype, tile_hint=tile_hint), fn=_make_randn, fn_kw={'seed': seed})


def _arange_mapper(tile, ex, start, stop, step, dtype=None):
  raise CodegenError('_arange_mapper is lowered to spx_fill, never called')


def _lower_arange(op, env):
  leaf = _leaf_of(op, env)
  kw = op.kw
  dt = np.dtype(kw.get('dtype') or leaf.dtype)
  return Pre('arange', dt, (backend.FILL_ARANGE, kw['start'], kw['step'], 0), None)


register_lowering(_arange_mapper, _lower_arange)


def arange(shape=None, start=0, stop=None, step=1, dtype=np.float64, tile_hint=None):
  """Extended np.arange (builtins.py:414-463)."""
  from .map import MapExpr
  from .base import ListExpr
  from .local import LocalInput, LocalMapLocationExpr, make_var
  if shape is None and stop is None:
    raise ValueError('Shape or stop expected, none supplied.')
  if shape is not None and stop is not None:
    raise ValueError('Only shape OR stop can be supplied, not both.')
  if shape is None:
    shape = (int(np.ceil((stop - start) / float(step))),)
  if stop is None:
    stop = step * (int(np.prod(shape)) + start)
  if isinstance(shape, (int, np.integer)):
    shape = (int(shape),)
  var = make_var()
  op = LocalMapLocationExpr(fn=_arange_mapper, deps=[LocalInput(var), LocalInput('extent')],
                            kw={'start': start, 'stop': stop, 'step': step, 'dtype': dtype})
  return MapExpr(children=ListExpr(vals=[ndarray(shape, dtype, tile_hint)]), child_to_var=[var], op=op)


# --------------------------------------------------------------- reductions
def _sum_local(ex, data, axis):
  return data.sum(axis)


def _max_local(ex, data, axis):
  return data.max(axis)


def _min_local(ex, data, axis):
  return data.min(axis)


def _argmin_local(ex, data, axis):
  return data.argmin(axis)


def _argmax_local(ex, data, axis):
  return data.argmax(axis)


def _countnonzero_local(ex, data, axis):
  return (data != 0).sum(axis)


def _countzero_local(ex, data, axis):
  return (data == 0).sum(axis)


engine.register_reduce(_sum_local, 'sum')
engine.register_reduce(_max_local, 'max')
engine.register_reduce(_min_local, 'min')
engine.register_reduce(_argmin_local, 'argmin')
engine.register_reduce(_argmax_local, 'argmax')
engine.register_reduce(_countnonzero_local, 'sum',
                       lambda r: codegen.Op('not_equal', [r, codegen.Const(0, r.dtype)]))
engine.register_reduce(_countzero_local, 'sum',
                       lambda r: codegen.Op('equal', [r, codegen.Const(0, r.dtype)]))


def _same_dtype(input):
  return input.dtype


def sum(x, axis=None, tile_hint=None):
  return reduce(x, axis=axis, dtype_fn=_same_dtype, local_reduce_fn=_sum_local, accumulate_fn=np.add,
                tile_hint=tile_hint)


def max(x, axis=None, tile_hint=None):
  return reduce(x, axis=axis, dtype_fn=_same_dtype, local_reduce_fn=_max_local, accumulate_fn=np.maximum,
                tile_hint=tile_hint)


def min(x, axis=None, tile_hint=None):
  return reduce(x, axis=axis, dtype_fn=_same_dtype, local_reduce_fn=_min_local, accumulate_fn=np.minimum,
                tile_hint=tile_hint)


def mean(x, axis=None):
  """sum / count; integer inputs floor-divide as Python-2 ``np.divide`` did
  (builtins.py:527-539, SURVEY.md Appendix A pin 8)."""
  n = int(np.prod(x.shape)) if axis is None else x.shape[axis]
  s = sum(x, axis)
  if np.dtype(x.dtype).kind in 'biu':
    return map((s, n), fn=np.floor_divide)
  return map((s, n), fn=np.true_divide)


def std(a, axis=None):
  """Standard deviation (builtins.py:549-565): sqrt(mean(a^2) - mean(a)^2) in
  fp64, i.e. two fused map+reduce passes (x*x summed, x summed) and one
  elementwise map over the two partial results."""
  a64 = astype(a, np.float64)
  return sqrt(mean(a64 ** 2, axis) - mean(a64, axis) ** 2)


def _int64(input):
  return np.dtype(np.int64)


def argmin(x, axis=None):
  return reduce(x, axis=axis, dtype_fn=_int64, local_reduce_fn=_argmin_local, accumulate_fn=np.minimum)


def argmax(x, axis=None):
  return reduce(x, axis=axis, dtype_fn=_int64, local_reduce_fn=_argmax_local, accumulate_fn=np.minimum)


def count_nonzero(array, axis=None, tile_hint=None):
  return reduce(array, axis, dtype_fn=_int64, local_reduce_fn=_countnonzero_local, accumulate_fn=np.add,
                tile_hint=tile_hint)


def count_zero(array, axis=None):
  return reduce(array, axis, dtype_fn=_int64, local_reduce_fn=_countzero_local, accumulate_fn=np.add)


def size(x, axis=None):
  if axis is None:
    return int(np.prod(x.shape))
  return x.shape[axis]


# --------------------------------------------------------------- elementwise
def _astype_mapper(t, dtype):
  return t.astype(dtype)


register_lowering(_astype_mapper, lambda op, env: codegen.Cast(_leaf_of(op, env), np.dtype(op.kw['dtype'])))


def astype(x, dtype):
  assert x is not None
  return map(x, _astype_mapper, fn_kw={'dtype': np.dtype(dtype).str})


def add(a, b):
  return map((a, b), fn=np.add)


def sub(a, b):
  return map((a, b), fn=np.subtract)


def multiply(a, b):
  return map((a, b), fn=np.multiply)


def power(a, b):
  return map((a, b), fn=np.power)


def maximum(a, b):
  return map((a, b), np.maximum)


def minimum(a, b):
  return map((a, b), np.minimum)


def ln(v):
  return map(v, fn=np.log)


def log(v):
  return map(v, fn=np.log)


def exp(v):
  return map(v, fn=np.exp)


def square(v):
  return map(v, fn=np.square)


def sqrt(v):
  return map(v, fn=np.sqrt)


def abs(v):
  return map(v, fn=np.abs)


# ------------------------------------------------------- join builtins
def _bincount_mapper(ex, tiles, minlength=None):
  """builtins.py:815-821: per-tile np.bincount (host meaning; lowered to
  spx_bincount / spx_kmeans_accumulate by the registered join below)."""
  if len(tiles) > 1:
    result = np.bincount(tiles[0], weights=tiles[1], minlength=minlength)
  else:
    result = np.bincount(tiles[0], minlength=minlength)
  from ..array import extent as ext
  yield ext.from_shape(result.shape), result


def _bincount_join(kind, arrays, axes, fn_kw, target):
  import torch
  from .. import comm, runtime
  from ..examples.kmeans import _deliver_full
  ctx = runtime.get()
  be = backend.get()
  K = target.shape[0]
  v = arrays[0]
  if len(arrays) == 1:
    acc = torch.zeros((K,), dtype=torch.int64, device=ctx.device)
    for ex, tile in v.local.items():
      be.bincount(be.contiguous(tile.data, np.int64).reshape(-1), acc, zero_first=False)
  else:
    from ..array import distarray
    w = arrays[1]
    acc = torch.zeros((K, 1), dtype=torch.float64, device=ctx.device)
    counts = torch.zeros((K,), dtype=torch.int64, device=ctx.device)
    exs = sorted(v.tiles.items(), key=lambda kv: kv[0].ul)
    got = distarray.gather_regions(w, [(ex, ctx.owner(o)) for ex, o in exs])
    for qi, (ex, o) in enumerate(exs):
      if ctx.owner(o) != ctx.rank:
        continue
      lab = be.contiguous(v.local[ex].data, np.int64).reshape(-1)
      wt = got[qi]
      if np.dtype(w.dtype).kind != 'f':
        wt = be.contiguous(wt, np.float64)
      be.kmeans_accumulate(be.contiguous(wt).reshape(-1, 1), lab, acc, counts, zero_first=False)
  comm.all_reduce(acc, 'sum')
  _deliver_full(target, acc.reshape(K))


def bincount(v, weights=None, minlength=None):
  """Count occurrences of each value in a 1-d non-negative int array
  (builtins.py:824-846): per-tile counts (weighted sums with ``weights``)
  summed across tiles.  As in the reference the result has the input's
  dtype (int64), so weighted sums are truncated toward zero.  The reference
  asserts min(v) > 0, which rejects the value 0 its own mapper counts; here
  min(v) >= 0 is required."""
  import builtins as _b
  from .join import map2
  minval = int(min(v).glom())
  maxval = int(max(v).glom())
  assert minval >= 0, 'bincount: negative values'
  minlength = maxval + 1 if minlength is None else _b.max(maxval + 1, minlength)
  arrays = (v, weights) if weights is not None else v
  return map2(arrays, fn=_bincount_mapper, fn_kw={'minlength': minlength}, shape=(minlength,), reducer=np.add)


def _concatenate_mapper(extents, tiles, shape=None, axis=0):
  """builtins.py:871-884 (host meaning; data movement by the registered join)."""
  raise CodegenError('_concatenate_mapper is lowered to a tile copy, never called')


def _concatenate_join(kind, arrays, axes, fn_kw, target):
  """Every tile of ``a`` lands at its own offset in the target, every tile of
  ``b`` shifted by a.shape[axis] along ``axis``: one point-to-point batch."""
  from .. import runtime
  from ..array import extent as ext
  from .join import _scatter_updates
  ctx = runtime.get()
  axis = fn_kw.get('axis', 0)
  shape = tuple(target.shape)
  updates = []
  off = arrays[0].shape[axis]
  for ai, arr in enumerate(arrays):
    for ex, w in sorted(arr.tiles.items(), key=lambda kv: kv[0].ul):
      ul, lr = list(ex.ul), list(ex.lr)
      if ai == 1:
        ul[axis] += off
        lr[axis] += off
      src = ctx.owner(w)
      t = arr.local[ex].data if src == ctx.rank else None
      updates.append(((ai, tuple(ex.ul)), ext.create(ul, lr, shape), src, t))
  _scatter_updates(target, updates)


def concatenate(a, b, axis=0):
  """Join two arrays along ``axis`` (builtins.py:887-905)."""
  from .join import map2
  from ..array import extent as ext
  new_shape = [0] * len(a.shape)
  for index, (dim1, dim2) in enumerate(zip(a.shape, b.shape)):
    if index == axis:
      new_shape[index] = dim1 + dim2
      continue
    new_shape[index] = dim1
    if dim1 != dim2:
      raise ValueError('all the input array dimensions except for the concatenation axis must match exactly')
  partition_axis = ext.largest_dim_axis(a.shape, exclude_axes=[axis]) if len(a.shape) > 1 else 0
  return map2((a, b), (partition_axis, partition_axis), fn=_concatenate_mapper,
              fn_kw={'axis': axis, 'shape': new_shape}, shape=new_shape)


def _register_joins():
  from .join import register_join
  register_join(_bincount_mapper, _bincount_join)
  register_join(_concatenate_mapper, _concatenate_join)


_register_joins()
