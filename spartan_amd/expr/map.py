"""``map`` over tiles (restates spartan/expr/map.py:91-205).

MapExpr keeps the reference's fields (children, child_to_var, op) so the
fusion passes rewrite it exactly as MapMapFusion does; evaluation hands the
(fused) LocalExpr tree to the engine, which runs ONE generated gfx950 kernel
per output tile instead of one NumPy call per tree node.
"""
from .. import util
from . import engine
from .base import Expr, ListExpr, as_array
from .broadcast import broadcast
from .local import LocalInput, LocalMapExpr, make_var


class MapExpr(Expr):
  _members = ('children', 'child_to_var', 'op')

  def pretty_str(self):
    return 'Map[%d](%s, %s)' % (self.expr_id, self.op.pretty_str(), self.children.pretty_str())

  def compute_shape(self):
    """Right-aligned broadcast of the children's shapes (map.py:105-128)."""
    shapes = [list(c.shape) for c in self.children]
    nd = max(len(s) for s in shapes)
    out = [0] * nd
    for s in shapes:
      s = [1] * (nd - len(s)) + s
      for i, v in enumerate(s):
        out[i] = max(out[i], v)
    return tuple(out)

  def compute_dtype(self):
    import numpy as np
    from .. import codegen
    from .base import AsArray
    from .local import LowerEnv, lower
    env = LowerEnv({})
    for c, v in zip(self.children, self.child_to_var):
      if isinstance(c, AsArray) and np.ndim(c.val) == 0:
        env.leaves[v] = env.new_scalar(np.asarray(c.val).item())
      else:
        env.leaves[v] = codegen.In(0, c.dtype)
    return lower(self.op, env).dtype

  def _evaluate(self, deps):
    children = broadcast(list(deps['children']))
    child_to_var = list(self.child_to_var)
    largest = max(children, key=lambda v: v.real_size())
    i = [id(c) for c in children].index(id(largest))
    children[0], children[i] = children[i], children[0]
    child_to_var[0], child_to_var[i] = child_to_var[i], child_to_var[0]
    return engine.run_map(children, child_to_var, self.op)


def map(inputs, fn, numpy_expr=None, fn_kw=None):
  """Evaluate ``fn`` over each tile of the (broadcast) inputs (map.py:172-205)."""
  assert fn is not None
  if not util.is_iterable(inputs) or isinstance(inputs, Expr):
    inputs = [inputs]
  children, child_to_var, op_deps = [], [], []
  for v in inputs:
    v = as_array(v)
    var = make_var()
    children.append(v)
    child_to_var.append(var)
    op_deps.append(LocalInput(var))
  op = LocalMapExpr(fn=fn, kw=fn_kw, pretty_fn=numpy_expr, deps=op_deps)
  return MapExpr(children=ListExpr(vals=children), child_to_var=child_to_var, op=op)
