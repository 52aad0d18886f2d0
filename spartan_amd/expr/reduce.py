"""``reduce`` over an axis (restates spartan/expr/reduce.py:70-166).

The per-tile ``local_reduce_fn`` must be one of the registered builtin local
reducers (sum/min/max/argmin/argmax/count_*); with ReduceMapFusion the mapped
tree in front of it is fused into the same generated kernel.
"""
from . import engine
from .base import Expr, ListExpr
from .broadcast import broadcast
from .local import LocalInput, LocalReduceExpr, make_var
from ..array import extent as ext


class ReduceExpr(Expr):
  _members = ('children', 'child_to_var', 'axis', 'dtype_fn', 'op', 'accumulate_fn', 'tile_hint')

  def compute_shape(self):
    shapes = [c.shape for c in self.children]
    nd = max(len(s) for s in shapes)
    out = [0] * nd
    for s in shapes:
      for i, v in enumerate(s):
        out[i] = max(out[i], v)
    return tuple(ext.shape_for_reduction(tuple(out), self.axis))

  def pretty_str(self):
    return 'Reduce(%s, axis=%s, %s)' % (getattr(self.op.fn, '__name__', self.op.fn), self.axis,
                                        self.children.pretty_str())

  def _evaluate(self, deps):
    children = broadcast(list(deps['children']))
    dtype = self.dtype_fn(children[0])
    return engine.run_reduce(children, list(self.child_to_var), self.op, self.axis, dtype,
                             self.accumulate_fn, self.tile_hint)


def reduce(v, axis, dtype_fn, local_reduce_fn, accumulate_fn, fn_kw=None, tile_hint=None):
  """Reduce ``v`` over ``axis`` (reduce.py:127-166)."""
  fn_kw = dict(fn_kw or {})
  assert 'axis' not in fn_kw, '"axis" argument is reserved.'
  fn_kw['axis'] = axis
  var = make_var()
  op = LocalReduceExpr(fn=local_reduce_fn, deps=[LocalInput('extent'), LocalInput(var)], kw=fn_kw)
  return ReduceExpr(children=ListExpr(vals=[v]), child_to_var=[var], axis=axis, dtype_fn=dtype_fn,
                    op=op, accumulate_fn=accumulate_fn, tile_hint=tile_hint)
