"""DAG rewrite passes run by ``Expr.optimized()`` (spartan/expr/optimize.py).

Kept: CollapsedCachedExpressions (:225-242), MapMapFusion (:128-182),
ReduceMapFusion (:185-222), in the reference's registration order
(:929-937), each switchable with its ``opt_*`` flag.  The passes fuse the
*DAG*; the fused LocalExpr tree they produce is what codegen turns into one
kernel.  ParakeetGeneration is replaced by that codegen; AutomaticTiling and
RotateSlice are later-round items.
"""
from ..config import FLAGS
from .base import AsArray, Expr, ListExpr, Val, expr_like, lazify
from .local import LocalInput, LocalMapLocationExpr, LocalReduceExpr, make_var
from .map import MapExpr
from .ndarray import NdArrayExpr
from .reduce import ReduceExpr


def not_idempotent(fn):
  """Results of ``fn`` are evaluated at once and never fused into
  (optimize.py:56-64)."""
  def wrapped(*args, **kw):
    r = fn(*args, **kw)
    if isinstance(r, Expr):
      r.needs_cache = True
      r.not_idempotent = True
    return r
  wrapped.__name__ = fn.__name__
  wrapped.__doc__ = fn.__doc__
  return wrapped


def fusable(v):
  return isinstance(v, (MapExpr, ReduceExpr, NdArrayExpr, Val, AsArray))


def merge_var(children, child_to_var, k, v):
  if k in child_to_var:
    assert children[child_to_var.index(k)] is v or \
        children[child_to_var.index(k)].expr_id == v.expr_id
  else:
    children.append(v)
    child_to_var.append(k)


class OptimizePass:
  name = None

  def __init__(self):
    self.visited = {}

  def visit(self, op):
    if not isinstance(op, Expr):
      return op
    if op.expr_id in self.visited:
      return self.visited[op.expr_id]
    handler = getattr(self, 'visit_default', None) or getattr(self, 'visit_' + op.typename(), None)
    new = handler(op) if handler is not None else op.visit(self)
    self.visited[new.expr_id] = new
    return new


class MapMapFusion(OptimizePass):
  """map(f, map(g, x)) -> map(f . g, x)."""
  name = 'map_fusion'

  def visit_MapExpr(self, expr):
    children = self.visit(expr.children)
    if not all(fusable(c) for c in children) or getattr(expr, 'not_idempotent', False):
      return expr.visit(self)
    new_children, new_vars = [], []
    op = expr.op
    combined = op.__class__(fn=op.fn, kw=op.kw, pretty_fn=op.pretty_fn)
    for child in children:
      if isinstance(child, MapExpr):
        for k, v in zip(child.child_to_var, child.children):
          merge_var(new_children, new_vars, k, v)
        combined.add_dep(child.op)
      else:
        key = make_var()
        new_children.append(child)
        new_vars.append(key)
        combined.add_dep(LocalInput(key))
    if isinstance(combined, LocalMapLocationExpr):
      combined.add_dep(LocalInput('extent'))
    return expr_like(expr, children=ListExpr(vals=new_children), child_to_var=new_vars, op=combined)


class ReduceMapFusion(OptimizePass):
  """reduce(f, map(g, X)) -> reduce(f . g, X)."""
  name = 'reduce_fusion'

  def visit_ReduceExpr(self, expr):
    children = self.visit(expr.children)
    for c in children:
      if not isinstance(c, MapExpr) or getattr(c, 'not_idempotent', False):
        return expr.visit(self)
    combined = LocalReduceExpr(fn=expr.op.fn, kw=expr.op.kw, deps=[expr.op.deps[0]])
    new_children, new_vars = [], []
    for c in children:
      for k, v in zip(c.child_to_var, c.children):
        merge_var(new_children, new_vars, k, v)
      combined.add_dep(c.op)
    return expr_like(expr, children=ListExpr(vals=new_children), child_to_var=new_vars, op=combined)


class CollapsedCachedExpressions(OptimizePass):
  """Replace already-evaluated nodes by their value."""
  name = 'collapse_cached'

  def visit_default(self, expr):
    c = expr.cache()
    if c is not None:
      return lazify(c)
    return expr.visit(self)


PASSES = [CollapsedCachedExpressions, MapMapFusion, ReduceMapFusion]


def optimize(dag):
  if not FLAGS.optimization:
    return dag
  for p in PASSES:
    if getattr(FLAGS, 'opt_' + p.name):
      dag = p().visit(dag)
  return dag
