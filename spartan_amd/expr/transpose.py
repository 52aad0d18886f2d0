"""``transpose(x)`` (restates spartan/expr/transpose.py:68-98): a zero-copy
``Transpose`` view (array/views.py) whose fetched pieces are strided device
views, consumed in place by the generated kernels."""
from ..array.views import transpose_of
from .base import Expr, lazify


class TransposeExpr(Expr):
  _members = ('array',)

  def compute_shape(self):
    return tuple(reversed(self.array.shape))

  def compute_dtype(self):
    return self.array.dtype

  def pretty_str(self):
    return 'Transpose[%d](%s)' % (self.expr_id, self.array)

  def _evaluate(self, deps):
    return transpose_of(deps['array'])


def transpose(array, tile_hint=None):
  e = TransposeExpr(array=lazify(array))
  e.tile_hint = tile_hint
  return e
