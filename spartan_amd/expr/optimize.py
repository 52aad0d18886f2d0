"""DAG rewrite passes run by ``Expr.optimized()`` (spartan/expr/optimize.py).

Kept: CollapsedCachedExpressions (:225-242), AutomaticTiling (:454-890,
solver in libspx.so), MapMapFusion (:128-182), ReduceMapFusion (:185-222),
in the reference's registration order (:929-937), each switchable with its
``opt_*`` flag; DotReduceFusion is new (after the reference's passes).  The
passes fuse the *DAG*; the fused LocalExpr tree they produce is what codegen
turns into one kernel.  ParakeetGeneration is replaced by that codegen;
RotateSlice (default off in the reference) is not built.
"""
import numpy as np

from ..config import FLAGS
from .base import AsArray, CollectionExpr, Expr, ListExpr, Val, expr_like, lazify
from .local import (FnCallExpr, LocalInput, LocalMapLocationExpr, LocalReduceExpr, LocalRowDot, has_location,
                    make_var)
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
      if not isinstance(c, MapExpr) or getattr(c, 'not_idempotent', False) or has_location(c.op):
        return expr.visit(self)  # location maps lower per tile: kept out of the fused reduce
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
  """reduce(f(x, dot(x, w)), axis=0) with a small (K, 1) operand ``w`` (a
  host array, or a device-resident array / expression) -> one fused kernel
  that reads ``x`` once.

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
      if not isinstance(d, DotExpr):  # (its tile_hint is moot: a fused dot has no output array)
        continue
      w, a = d.matrix_b, d.matrix_a
      # w: a host (K, 1) array, or a device-resident (K, 1) array / expression
      # (an iterative driver that keeps w on the GPU: no host round trip)
      host = isinstance(w, np.ndarray)
      wshape = tuple(w.shape) if host or isinstance(w, Expr) else None
      if wshape is None or len(wshape) != 2 or wshape[1] != 1:
        continue
      K = wshape[0]
      if not (2 <= K <= ROWDOT_MAX_K) or tuple(a.shape) != it_shape or it_shape[1] != K:
        continue
      if np.dtype(w.dtype).kind != 'f' or np.dtype(a.dtype) != np.dtype(w.dtype):
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
      if host:
        vals.append(AsArray(val=np.ascontiguousarray(w.reshape(1, K))))
      else:
        from .reshape import reshape
        vals.append(reshape(w, (1, K)))
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


class OuterArgminFusion(OptimizePass):
  """argmin(outer((X, C), (0, 0), mapper), axis=1) -> one fused kernel.

  The reference materialises the (N, K) outer product (k_means_.py:126-128:
  cdist per row strip into an N x K target, 204.8 GB fp64 at cfg3) and then
  runs argmin over it.  When the outer's mapper has a registered argmin
  fusion (examples/kmeans.py: kmeans_dist_mapper -> spx_kmeans_assign) and
  the argmin reads the outer product directly, the pair becomes an
  ArgminJoinExpr with the argmin's expr_id; its labels are the same bits."""
  name = 'outer_argmin_fusion'

  def visit_ReduceExpr(self, expr):
    from .builtins import _argmin_local
    from .join import ArgminJoinExpr, OuterProductExpr, argmin_fusion_for
    children = self.visit(expr.children)
    expr = expr_like(expr, children=children)
    op = expr.op
    if not isinstance(op, LocalReduceExpr) or op.fn is not _argmin_local or expr.axis not in (1, -1):
      return expr
    if len(children.vals) != 1 or not isinstance(children.vals[0], OuterProductExpr):
      return expr
    tree = op.deps[1]
    if not (isinstance(tree, LocalInput) and tree.idx == expr.child_to_var[0]):
      return expr
    outer = children.vals[0]
    impl = argmin_fusion_for(outer)
    if impl is None:
      return expr
    return ArgminJoinExpr(expr_id=expr.expr_id, arrays=outer.arrays, outer=outer, impl=impl,
                          tile_hint=expr.tile_hint)


class CollapsedCachedExpressions(OptimizePass):
  """Replace already-evaluated nodes by their value."""
  name = 'collapse_cached'

  def visit_default(self, expr):
    c = expr.cache()
    if c is not None:
      return lazify(c)
    return expr.visit(self)


# ---------------------------------------------------------- AutomaticTiling
# expr_id -> tiling chosen by an earlier optimisation (optimize.py _tiled_exprlist)
_tiled_exprs = {}


def _size(shape):
  n = 1
  for s in shape:
    n *= int(s)
  return n


class AutomaticTiling:
  """Row (0) or column (1) partitioning for every new array and result of a
  DAG (spartan/expr/optimize.py:454-890).

  A cost graph is built over (expression, tiling) nodes -- node 0 the
  source, one node per possible tiling of each expression, split pairs for
  the expressions that can go either way, edge costs in elements that would
  move if a consumer's tiling differs from its producer's -- exactly as the
  reference's visit_* methods do for the node types of this path (NdArrayExpr,
  MapExpr, ReduceExpr, DotExpr, DistArray values, collections, reshape).  The
  choice is made by the native solver (``spx_mincost_tiling`` in libspx.so,
  the reference's tiling.cc) and written back as ``tile_hint`` on
  NdArrayExpr / ReduceExpr / DotExpr: the chosen dim is divided into
  ``num_workers`` pieces (tile_expr, :793-796)."""
  name = 'auto_tiling'

  def __init__(self):
    self.cur = 1
    self.edges = {}
    self.nodes = {0: ([], -1, [], [])}  # id -> (exprs, tiling, children, parents)
    self.expr_to_nodes = {}
    self.split = {}
    self.root = None

  # -- graph -----------------------------------------------------------------
  def _node(self, exprs, tiling):
    nid = self.cur
    self.nodes[nid] = (list(exprs), tiling, [], [])
    self.cur += 1
    return nid

  def add_edge(self, u, v, cost=0):
    if (u, v) not in self.edges:
      self.nodes[u][3].append(v)
      self.nodes[v][2].append(u)
    self.edges[(u, v)] = int(cost)

  def add_split(self, a, b):
    self.split[a] = b
    self.split[b] = a

  def tiling(self, nid):
    return self.nodes[nid][1]

  def first_expr(self, nid):
    return self.nodes[nid][0][0]

  def visit_children(self, children, except_child=None):
    from ..array.distarray import DistArray
    ids = []
    for c in children:
      if isinstance(c, (Expr, DistArray)) and c is not except_child:
        ids.extend(self.visit_node(c))
    return ids

  def _alternatives(self, child_ids):
    """Node ids for an expression that follows its driving child's tiling:
    both tilings (a new split pair) if the child is split, else its tiling."""
    if child_ids and child_ids[0] in self.split:
      self.add_split(self.cur, self.cur + 1)
      return (0, 1)
    return (self.tiling(child_ids[0]),)

  # -- per node type (optimize.py:514-781) ----------------------------------
  def visit_NdArrayExpr(self, expr):
    shape = expr.shape
    if len(shape) > 1 and shape[1] > 1:
      a = self._node([expr], 0)
      self.add_edge(0, a, 0)
      b = self._node([expr], 1)
      self.add_edge(0, b, 0)
      self.add_split(a, b)
      return [a, b]
    a = self._node([expr], 0)
    self.add_edge(0, a, 0)
    return [a]

  def visit_MapExpr(self, expr):
    vals = list(expr.children.vals)
    largest = max(vals, key=lambda v: _size(v.shape))
    child_ids = self.visit_children([largest])
    other_ids = self.visit_children(vals, largest)
    kw = expr.op.kw if isinstance(getattr(expr.op, 'kw', None), dict) else {}
    kw_ids = self.visit_children(list(kw.values()))
    if not other_ids or not child_ids:  # one input: the map reuses its child's nodes
      ids = child_ids or other_ids
      for cid in ids:
        self.nodes[cid][0].append(expr)
      return ids
    out = []
    for i, tiling in enumerate(self._alternatives(child_ids)):
      nid = self._node([expr], tiling)
      out.append(nid)
      self.add_edge(child_ids[i], nid, 0)
      for cid in other_ids:
        cost = _size(self.first_expr(cid).shape) if self.tiling(cid) != tiling else 0
        self.add_edge(cid, nid, cost)
      for cid in kw_ids:
        self.add_edge(cid, nid, _size(self.first_expr(cid).shape))
    return out

  def visit_ReduceExpr(self, expr):
    child_ids = self.visit_children(list(expr.children.vals))
    cost = _size(expr.shape)
    nid = self._node([expr], 0)
    for cid in child_ids:
      free = expr.axis is None or (1 - expr.axis) == self.tiling(cid)
      self.add_edge(cid, nid, 0 if free else cost)
    return [nid]

  def visit_DotExpr(self, expr):
    child_ids = self.visit_children([expr.matrix_a])
    other_ids = self.visit_children([expr.matrix_b])
    if other_ids and child_ids:  # copy cost of B against A's tiling
      ids = []
      for i, tiling in enumerate(self._alternatives(child_ids)):
        nid = self._node([expr], tiling)
        ids.append(nid)
        self.add_edge(child_ids[i], nid, 0)
        for cid in other_ids:
          cost = _size(self.first_expr(cid).shape) if tiling == 0 or self.tiling(cid) == tiling else 0
          self.add_edge(cid, nid, cost)
      child_ids = ids
    shape = expr.shape
    if len(shape) == 1 or shape[1] == 1:
      tilings = (0,)
    else:
      tilings = (0, 1)
      self.add_split(self.cur, self.cur + 1)
    out = []
    for tiling in tilings:  # update cost of the result
      nid = self._node([expr], tiling)
      out.append(nid)
      for cid in child_ids:
        self.add_edge(cid, nid, _size(shape) if self.tiling(cid) != tiling else 0)
    return out

  def visit_WriteArrayExpr(self, expr):  # :716-740
    child_ids = self.visit_children([expr.array])
    data_ids = self.visit_children([expr.data])
    if not child_ids:
      return []
    if not data_ids:  # host data: the write keeps the target's nodes
      for cid in child_ids:
        self.nodes[cid][0].append(expr)
      return child_ids
    out = []
    for i, tiling in enumerate(self._alternatives(child_ids)):
      nid = self._node([expr], tiling)
      out.append(nid)
      self.add_edge(child_ids[i], nid, 0)
      for cid in data_ids:
        self.add_edge(cid, nid, _size(self.first_expr(cid).shape) if self.tiling(cid) != tiling else 0)
    return out

  def visit_ReshapeExpr(self, expr):  # visit_aligned_nodes(reverse_cost=True), :742-763
    child_ids = self.visit_children([expr.array])
    if not child_ids:
      return []
    if child_ids[0] in self.split:
      self.add_split(self.cur, self.cur + 1)
      tilings = (0, 1)
    else:
      tilings = (1 ^ int(self.tiling(child_ids[0])),)
    out = []
    for i, tiling in enumerate(tilings):
      nid = self._node([expr], tiling)
      out.append(nid)
      self.add_edge(child_ids[-(1 ^ i)], nid, 0)
    return out

  def visit_node(self, expr):
    from ..array.distarray import DistArray
    if self.root is None:
      self.root = expr
    key = getattr(expr, 'expr_id', None)
    if key is not None and key in _tiled_exprs:
      self.tile_cached(expr)
      nid = self._node([expr], _tiled_exprs[key])
      self.add_edge(0, nid, 0)
      ids = [nid]
    elif key is not None and key in self.expr_to_nodes:
      ids = self.expr_to_nodes[key]
      for nid in ids:
        self.nodes[nid][0].append(expr)
    elif isinstance(expr, DistArray) or (isinstance(expr, (Val, AsArray)) and isinstance(expr.val, DistArray)):
      arr = expr if isinstance(expr, DistArray) else expr.val
      if arr.replicated or not hasattr(arr, 'tile_shape'):
        ids = []  # a host / replicated value: no partitioning to choose (the reference's NumPy operands)
      else:
        tiling = 1 if (len(arr.shape) > 0 and arr.tile_shape()[0] == arr.shape[0]) else 0
        nid = self._node([expr], tiling)
        self.add_edge(0, nid, 0)
        ids = [nid]
    elif isinstance(expr, CollectionExpr):
      vals = list(expr.vals.values()) if isinstance(expr.vals, dict) else list(expr.vals)
      child_ids = self.visit_children(vals)
      nid = self._node([expr], -1)
      for cid in child_ids:
        self.add_edge(cid, nid, 0)
      ids = [nid]
    elif hasattr(self, 'visit_' + type(expr).__name__):
      ids = getattr(self, 'visit_' + type(expr).__name__)(expr)
    else:
      ids = []  # host values and view types outside this path: no node
    if key is not None:
      self.expr_to_nodes[key] = ids
    return ids

  # -- solve + write back (:783-840) ----------------------------------------
  def generate_edges(self, s, visited, out):
    parents = sorted(self.nodes[s][3], key=lambda p: _size(self.first_expr(p).shape))
    self.nodes[s][3][:] = parents
    for p in parents:
      out.append((s, p, self.edges[(s, p)]))
      if p not in visited:
        self.generate_edges(p, visited, out)
        visited.add(p)
    return out

  @staticmethod
  def tile_expr(expr, tiling):
    from .dot import DotExpr
    if isinstance(expr, (NdArrayExpr, ReduceExpr, DotExpr)) and len(expr.shape) > 0 and tiling in (0, 1):
      hint = list(expr.shape)
      if tiling < len(hint):
        W = max(1, int(FLAGS.num_workers or _world_workers()))
        hint[tiling] = -(-int(hint[tiling]) // W)
        expr.tile_hint = hint

  def tile_cached(self, expr):
    from .dot import DotExpr
    if not isinstance(expr, Expr) or isinstance(expr, (Val, AsArray)):
      return
    if expr.expr_id in _tiled_exprs:
      self.tile_expr(expr, _tiled_exprs[expr.expr_id])
    subs = []
    if isinstance(expr, DotExpr):
      subs += [expr.matrix_a, expr.matrix_b]
    for attr in ('array',):
      if hasattr(expr, attr):
        subs.append(getattr(expr, attr))
    if isinstance(getattr(expr, 'children', None), CollectionExpr):
      subs += list(expr.children.vals)
    for c in subs:
      self.tile_cached(c)

  def visit(self, dag):
    if not isinstance(dag, Expr):
      return dag
    ids = self.visit_node(dag)
    if not ids:
      return dag
    t = self._node([dag], -1)  # the sink
    self.add_edge(t - 1, t, 0)
    if t - 1 in self.split:
      self.add_edge(t - 2, t, 0)
    edges = self.generate_edges(0, set(), [])
    from .. import backend
    chosen, _ = backend.mincost_tiling(t, edges, sorted((a, b) for a, b in self.split.items() if a < b))
    for nid in chosen:
      exprs, tiling = self.nodes[nid][0], self.nodes[nid][1]
      for e in exprs:
        key = getattr(e, 'expr_id', None)
        if key is not None:
          _tiled_exprs[key] = tiling
        self.tile_expr(e, tiling)
    return dag


def _world_workers():
  from .. import runtime
  ctx = runtime.get()
  return ctx.num_workers if ctx is not None else 1


PASSES = [CollapsedCachedExpressions, AutomaticTiling, MapMapFusion, ReduceMapFusion, DotReduceFusion,
          OuterArgminFusion]


def _run_passes(dag):
  for p in PASSES:
    if getattr(FLAGS, 'opt_' + p.name):
      dag = p().visit(dag)
  return dag


def optimize(dag):
  if not FLAGS.optimization:
    return dag
  if FLAGS.opt_plan_cache:
    from . import plan_cache
    return plan_cache.optimize_cached(dag, _run_passes)
  return _run_passes(dag)
