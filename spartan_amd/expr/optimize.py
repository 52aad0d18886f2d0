"""DAG rewrite passes run by ``Expr.optimized()`` (spartan/expr/optimize.py).

Kept: CollapsedCachedExpressions (:225-242), MapMapFusion (:128-182),
ReduceMapFusion (:185-222), in the reference's registration order
(:929-937), each switchable with its ``opt_*`` flag.  The passes fuse the
*DAG*; the fused LocalExpr tree they produce is what codegen turns into one
kernel.  ParakeetGeneration is replaced by that codegen; AutomaticTiling and
RotateSlice are later-round items.
"""
import numpy as np

from ..config import FLAGS
from .base import AsArray, Expr, ListExpr, Val, expr_like, lazify
from .local import FnCallExpr, LocalInput, LocalMapLocationExpr, LocalReduceExpr, LocalRowDot, make_var
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


ROWDOT_MAX_K = 64  # one lane group of the column-reduce kernel holds a whole row


def _subst(op, var, repl):
  """Copy of a LocalExpr tree with every LocalInput(var) replaced by ``repl``."""
  if isinstance(op, LocalInput):
    return repl if op.idx == var else op
  new = op.__class__.__new__(op.__class__)
  new.__dict__.update(op.__dict__)
  new.deps = [_subst(d, var, repl) for d in op.deps]
  return new


class DotReduceFusion(OptimizePass):
  """reduce(f(x, dot(x, w)), axis=0) with a small host (K, 1) operand ``w``
  -> one fused kernel that reads ``x`` once.

  The reference evaluates ``dot(x, w)`` as its own pass (dot_map2_np_mapper,
  spartan/expr/dot.py:172-187), materialising yp, and the map+reduce that
  consumes it reads ``x`` again (linear_regression.py:10-16: ``x * (yp - y)``
  summed over axis 0).  When the DotExpr feeds a fused axis-0 reduction over
  an (N, K) iteration space and its left operand is that same (N, K) array,
  the dot is replaced by a ``rowdot(x, w)`` leaf evaluated row by row inside
  the reduction kernel (codegen.RowDot).  Applied only when every row fits one
  lane group (2 <= K <= 64) and x, w share a float dtype; otherwise the DAG is
  left unchanged."""
  name = 'dot_fusion'

  def visit_ReduceExpr(self, expr):
    from .dot import DotExpr
    children = self.visit(expr.children)
    expr = expr_like(expr, children=children)
    if expr.axis not in (0, -2) or not isinstance(expr.op, LocalReduceExpr):
      return expr
    shapes = [tuple(c.shape) for c in children]
    if any(len(s) > 2 for s in shapes) or max(len(s) for s in shapes) != 2:
      return expr
    it_shape = tuple(max(s[i - 2 + len(s)] if i - 2 + len(s) >= 0 else 1 for s in shapes) for i in range(2))
    vals, vars_ = list(children), list(expr.child_to_var)
    op = expr.op
    changed = False
    for i in range(len(vals)):
      d = vals[i]
      if not isinstance(d, DotExpr) or getattr(d, 'tile_hint', None) is not None:
        continue
      w, a = d.matrix_b, d.matrix_a
      if not isinstance(w, np.ndarray) or w.ndim != 2 or w.shape[1] != 1:
        continue
      K = w.shape[0]
      if not (2 <= K <= ROWDOT_MAX_K) or tuple(a.shape) != it_shape or it_shape[1] != K:
        continue
      if w.dtype.kind != 'f' or np.dtype(a.dtype) != w.dtype:
        continue
      var_a = None
      for c, v in zip(vals, vars_):
        if c is a or (isinstance(c, Expr) and c.expr_id == a.expr_id):
          var_a = v
          break
      if var_a is None:
        var_a = make_var()
        vals.append(a)
        vars_.append(var_a)
      var_w = make_var()
      vals.append(AsArray(val=np.ascontiguousarray(w.reshape(1, K))))
      vars_.append(var_w)
      op = _subst(op, vars_[i], LocalRowDot(deps=[LocalInput(var_a), LocalInput(var_w)]))
      vals[i] = None
      changed = True
    if not changed:
      return expr
    keep = [(c, v) for c, v in zip(vals, vars_) if c is not None]
    # the driving (N, K) input first: dtype_fn reads children[0]
    keep.sort(key=lambda cv: tuple(cv[0].shape) != it_shape)
    return expr_like(expr, children=ListExpr(vals=[c for c, _ in keep]),
                     child_to_var=[v for _, v in keep], op=op)


class CollapsedCachedExpressions(OptimizePass):
  """Replace already-evaluated nodes by their value."""
  name = 'collapse_cached'

  def visit_default(self, expr):
    c = expr.cache()
    if c is not None:
      return lazify(c)
    return expr.visit(self)


PASSES = [CollapsedCachedExpressions, MapMapFusion, ReduceMapFusion, DotReduceFusion]


def optimize(dag):
  if not FLAGS.optimization:
    return dag
  for p in PASSES:
    if getattr(FLAGS, 'opt_' + p.name):
      dag = p().visit(dag)
  return dag
