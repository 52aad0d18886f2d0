"""Indexing ``x[idx]`` (restates spartan/expr/slice.py:87-136).

``SliceExpr`` evaluates to a zero-copy ``Slice`` view (array/views.py): maps,
reductions and dot iterate over the base tiles' intersections with the slice
and fetch the corresponding base regions, so ``x[200:300, :].sum()``
(tests/benchmark_slice.py:11-14) reads only the sliced rows.  Only basic
indexing (ints, slices, tuples of them) is on this path; boolean / integer
array indexing (FilterExpr, filter.py) is out of scope.
"""
import numpy as np

from ..array import extent as ext
from ..array.views import Slice
from .base import Expr, NotShapeable


def _basic(idx):
  items = idx if isinstance(idx, tuple) else (idx,)
  return all(isinstance(i, (slice, int, np.integer)) for i in items)


class SliceExpr(Expr):
  _members = ('src',)

  def compute_shape(self):
    if not _basic(self.idx):
      raise NotShapeable
    return tuple(ext.compute_slice(ext.from_shape(self.src.shape), self.idx).shape)

  def compute_dtype(self):
    return self.src.dtype

  def pretty_str(self):
    return 'Slice[%d](%s, %s)' % (self.expr_id, self.src, self.idx)

  def _evaluate(self, deps):
    return Slice(deps['src'], self.idx)


def slice_expr(src, idx):
  if not _basic(idx):
    raise NotImplementedError('only basic indexing (ints and slices) has a gfx950 path; got %r' % (idx,))
  e = SliceExpr(src=src)
  e.idx = idx
  return e


class UnitDimsExpr(Expr):
  """Drop / insert length-1 dims of ``array`` without a copy (the reference
  wraps int / newaxis indexing in a ReshapeExpr, base.py:402-430)."""
  _members = ('array',)

  def compute_shape(self):
    return self.new_shape

  def compute_dtype(self):
    return self.array.dtype

  def pretty_str(self):
    return 'UnitDims[%d](%s, %s)' % (self.expr_id, self.array, self.new_shape)

  def _evaluate(self, deps):
    from ..array.distarray import LocalWrapper, ReplicatedArray
    from ..array.views import unit_dims_of
    a = deps['array']
    if isinstance(a, ReplicatedArray):
      return ReplicatedArray(a.device_data().reshape(self.new_shape))
    if isinstance(a, LocalWrapper):
      return LocalWrapper(np.asarray(a.value).reshape(self.new_shape))
    return unit_dims_of(a, self.new_shape)


def unit_dims(array, new_shape):
  e = UnitDimsExpr(array=array)
  e.new_shape = tuple(int(s) for s in new_shape)
  return e
