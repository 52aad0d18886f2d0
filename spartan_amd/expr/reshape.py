"""reshape: only the size-preserving re-view of a single-tile (or replicated)
array is supported in this round; general reshape is a later-round item
(spartan/expr/reshape.py)."""
from .base import Expr


class ReshapeExpr(Expr):
  _members = ('array',)

  def compute_shape(self):
    return tuple(self.new_shape)

  def compute_dtype(self):
    return self.array.dtype

  def _evaluate(self, deps):
    raise NotImplementedError('reshape is a later-round item')


def reshape(array, new_shape):
  e = ReshapeExpr(array=array)
  e.new_shape = tuple(new_shape)
  return e
