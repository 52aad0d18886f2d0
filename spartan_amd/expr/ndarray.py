"""Lazily created empty arrays (restates spartan/expr/ndarray.py:9-58)."""
import numpy as np

from ..array import distarray
from .base import Expr, expr_like


class NdArrayExpr(Expr):
  _members = ()

  def __init__(self, _shape=None, dtype=np.float64, tile_hint=None, reduce_fn=None, sparse=False, **kw):
    super().__init__(**kw)
    self._shape = tuple(int(s) for s in _shape)
    self._dtype = np.dtype(dtype)
    self.tile_hint = tile_hint
    self.reduce_fn = reduce_fn
    self.sparse = sparse

  def visit(self, visitor):
    return expr_like(self)

  def dependencies(self):
    return {}

  def compute_shape(self):
    return self._shape

  def compute_dtype(self):
    return self._dtype

  def pretty_str(self):
    return 'DistArray[%d](%s, %s, hint=%s)' % (self.expr_id, self._shape, self._dtype.name, self.tile_hint)

  def _evaluate(self, deps):
    return distarray.create(self._shape, self._dtype, reducer=self.reduce_fn, tile_hint=self.tile_hint,
                            sparse=self.sparse)


def ndarray(shape, dtype=np.float64, tile_hint=None, reduce_fn=None, sparse=False):
  return NdArrayExpr(_shape=shape, dtype=dtype, tile_hint=tile_hint, reduce_fn=reduce_fn, sparse=sparse)
