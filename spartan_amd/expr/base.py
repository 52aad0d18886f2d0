"""Lazy expression DAG (restates spartan/expr/base.py).

Semantics kept from the reference:
  * expressions are identified by ``expr_id``; copies made by optimisation
    passes keep the id, and results are cached per id with reference counting
    (EvalCache, base.py:67-104);
  * ``evaluate`` is recursive and bottom-up with a cache hit short-cut
    (base.py:259-300); ``force`` never optimises (base.py:462-465);
  * ``optimized`` runs the optimiser once and caches the rewritten DAG on the
    node (base.py:467-480);
  * arithmetic operators build ``map`` nodes with the NumPy ufunc
    (base.py:318-375).  Python 3 ``/`` maps to ``np.true_divide``; ``//`` to
    ``np.floor_divide``.
"""
import itertools

import numpy as np

from ..array import distarray
from ..config import FLAGS
from ..util import log

_ids = itertools.count()


def _new_id():
  return next(_ids)


class newaxis(object):
  """Marks a new unit dimension in ``x[...]`` (reference base.py:23-26;
  NumPy's ``None`` / ``np.newaxis`` is accepted too)."""


class NotShapeable(Exception):
  pass


class EvalCache:
  def __init__(self):
    self.refs = {}
    self.cache = {}

  def set(self, exprid, value):
    self.cache[exprid] = value

  def get(self, exprid):
    return self.cache.get(exprid)

  def register(self, exprid):
    self.refs[exprid] = self.refs.get(exprid, 0) + 1

  def deregister(self, exprid):
    n = self.refs.get(exprid, 0) - 1
    if n <= 0:
      self.refs.pop(exprid, None)
      self.cache.pop(exprid, None)
    else:
      self.refs[exprid] = n

  def clear(self):
    self.cache.clear()


eval_cache = EvalCache()


class Expr:
  """Base node.  Subclasses list their dependency fields in ``_members``."""
  _members = ()
  needs_cache = True
  optimized_expr = None

  def __init__(self, expr_id=None, **kw):
    for k in self._members:
      setattr(self, k, kw.pop(k, None))
    for k, v in kw.items():
      setattr(self, k, v)
    self.expr_id = next(_ids) if expr_id is None else expr_id
    eval_cache.register(self.expr_id)
    self.needs_cache = self.needs_cache and FLAGS.opt_expression_cache

  def __del__(self):
    try:
      eval_cache.deregister(self.expr_id)
    except Exception:
      pass

  # -- structure ----------------------------------------------------------
  def dependencies(self):
    return {k: getattr(self, k) for k in self._members}

  def visit(self, visitor):
    return expr_like(self, **{k: visitor.visit(getattr(self, k)) for k in self._members})

  def typename(self):
    return type(self).__name__

  def __hash__(self):
    return self.expr_id

  # -- evaluation ---------------------------------------------------------
  def cache(self):
    r = eval_cache.get(self.expr_id)
    if r is not None and not getattr(r, 'bad_tiles', []):
      return r
    return None

  def evaluate(self):
    c = self.cache()
    if c is not None:
      return c
    deps = {}
    for k, v in self.dependencies().items():
      deps[k] = v.evaluate() if isinstance(v, Expr) else v
    value = self._evaluate(deps)
    if self.needs_cache:
      eval_cache.set(self.expr_id, value)
    return value

  def _evaluate(self, deps):
    raise NotImplementedError

  def force(self):
    return self.evaluate()

  def optimized(self):
    if self.optimized_expr is None:
      self.optimized_expr = optimized_dag(self)
      self.optimized_expr.optimized_expr = self.optimized_expr
    return self.optimized_expr

  def glom(self):
    return glom(self)

  # -- shape --------------------------------------------------------------
  def compute_shape(self):
    raise NotShapeable

  @property
  def shape(self):
    # a node's shape never changes (rewrites that keep the id keep the
    # shape), so the first answer is memoised: the optimiser asks for it
    # thousands of times per DAG
    s = self.__dict__.get('_shape_memo')
    if s is not None:
      return s
    c = self.cache()
    if c is not None:
      s = tuple(c.shape)
    else:
      try:
        s = tuple(self.compute_shape())
      except NotShapeable:
        s = tuple(evaluate(self).shape)
    self.__dict__['_shape_memo'] = s
    return s

  @property
  def ndim(self):
    return len(self.shape)

  @property
  def size(self):
    return int(np.prod(self.shape))

  @property
  def dtype(self):
    c = self.cache()
    if c is not None:
      return c.dtype
    return self.compute_dtype()

  def compute_dtype(self):
    return evaluate(self).dtype

  def __repr__(self):
    return self.pretty_str()

  def pretty_str(self):
    return '%s[%d]' % (self.typename(), self.expr_id)

  # -- operators (base.py:318-375) -----------------------------------------
  def __add__(self, o): return _map(self, o, fn=np.add)
  def __radd__(self, o): return _map(o, self, fn=np.add)
  def __sub__(self, o): return _map(self, o, fn=np.subtract)
  def __rsub__(self, o): return _map(o, self, fn=np.subtract)
  def __mul__(self, o): return _map(self, o, fn=np.multiply)
  def __rmul__(self, o): return _map(o, self, fn=np.multiply)
  def __truediv__(self, o): return _map(self, o, fn=np.true_divide)
  def __rtruediv__(self, o): return _map(o, self, fn=np.true_divide)
  def __floordiv__(self, o): return _map(self, o, fn=np.floor_divide)
  def __rfloordiv__(self, o): return _map(o, self, fn=np.floor_divide)
  def __mod__(self, o): return _map(self, o, fn=np.mod)
  def __pow__(self, o): return _map(self, o, fn=np.power)
  def __neg__(self): return _map(self, fn=np.negative)
  def __eq__(self, o): return _map(self, o, fn=np.equal)
  def __ne__(self, o): return _map(self, o, fn=np.not_equal)
  def __lt__(self, o): return _map(self, o, fn=np.less)
  def __gt__(self, o): return _map(self, o, fn=np.greater)
  def __le__(self, o): return _map(self, o, fn=np.less_equal)
  def __ge__(self, o): return _map(self, o, fn=np.greater_equal)
  def __and__(self, o): return _map(self, o, fn=np.logical_and)
  def __or__(self, o): return _map(self, o, fn=np.logical_or)
  def __xor__(self, o): return _map(self, o, fn=np.logical_xor)

  def __getitem__(self, idx):
    """Basic indexing (reference base.py:388-430): slices give a zero-copy
    slice view; an int index drops its dimension and ``newaxis`` inserts a
    unit dimension -- the reference's ReshapeExpr over the SliceExpr, here a
    zero-copy UnitDims view."""
    from .slice import slice_expr, unit_dims
    items = idx if isinstance(idx, tuple) else (idx,)
    if not any(_is_newaxis(i) or isinstance(i, (int, np.integer)) for i in items):
      return slice_expr(self, idx)
    core = tuple(i for i in items if not _is_newaxis(i))
    sl = slice_expr(self, core) if core else self
    kept = iter(sl.shape)
    new_shape = []
    for i in items:
      if _is_newaxis(i):
        new_shape.append(1)
      elif isinstance(i, (int, np.integer)):
        next(kept)  # an int index drops its (length-1) dimension
      else:
        new_shape.append(next(kept))
    new_shape.extend(kept)  # trailing dims the index did not name
    return unit_dims(sl, tuple(new_shape))

  @property
  def T(self):
    from .transpose import transpose
    return transpose(self)

  def __setitem__(self, k, v):
    raise Exception('Expressions are read-only.')

  def reshape(self, new_shape):
    from .reshape import reshape
    return reshape(self, new_shape)


def _is_newaxis(i):
  return i is None or i is newaxis


def _map(*args, fn):
  from .map import map as _m
  return _m(list(args), fn)


def expr_like(expr, **kw):
  """Copy of ``expr`` with new fields and the SAME expr_id (base.py:53-70)."""
  new = expr.__class__.__new__(expr.__class__)
  for k, v in expr.__dict__.items():
    if k not in ('expr_id', 'optimized_expr'):
      new.__dict__[k] = v
  for k, v in kw.items():
    new.__dict__[k] = v
  new.expr_id = expr.expr_id
  eval_cache.register(new.expr_id)
  return new


class AsArray(Expr):
  """Promote a host value to be array-like (base.py:498-523)."""
  _members = ()

  def __init__(self, val=None, **kw):
    super().__init__(**kw)
    self.val = val

  def visit(self, visitor):
    return self

  def dependencies(self):
    return {}

  def compute_shape(self):
    return np.shape(self.val)

  def compute_dtype(self):
    dt = getattr(self.val, 'dtype', None)  # DistArray / ndarray: no host materialisation
    return np.dtype(dt) if dt is not None else np.asarray(self.val).dtype

  def _evaluate(self, deps):
    return distarray.as_array(self.val)

  def pretty_str(self):
    return str(self.val)


class Val(Expr):
  """An already-computed value as an expression (base.py:526-547)."""
  _members = ()
  needs_cache = False

  def __init__(self, val=None, **kw):
    super().__init__(**kw)
    self.val = val

  def visit(self, visitor):
    return self

  def dependencies(self):
    return {}

  def compute_shape(self):
    return self.val.shape

  def compute_dtype(self):
    return self.val.dtype

  def _evaluate(self, deps):
    return self.val

  def pretty_str(self):
    return 'Val(%s)' % (self.val,)


class CollectionExpr(Expr):
  needs_cache = False

  def __init__(self, vals=None, **kw):
    super().__init__(**kw)
    self.vals = vals

  def __getitem__(self, idx):
    return self.vals[idx]

  def __iter__(self):
    return iter(self.vals)

  def __len__(self):
    return len(self.vals)


class ListExpr(CollectionExpr):
  def dependencies(self):
    return {'v%d' % i: v for i, v in enumerate(self.vals)}

  def _evaluate(self, deps):
    return [deps['v%d' % i] for i in range(len(self.vals))]

  def visit(self, visitor):
    return ListExpr(vals=[visitor.visit(v) for v in self.vals])

  def pretty_str(self):
    return '[%s]' % ', '.join(repr(v) for v in self.vals)


class TupleExpr(CollectionExpr):
  def dependencies(self):
    return {'v%d' % i: v for i, v in enumerate(self.vals)}

  def _evaluate(self, deps):
    return tuple(deps['v%d' % i] for i in range(len(self.vals)))

  def visit(self, visitor):
    return TupleExpr(vals=tuple(visitor.visit(v) for v in self.vals))


class DictExpr(CollectionExpr):
  def dependencies(self):
    return dict(self.vals)

  def _evaluate(self, deps):
    return deps

  def visit(self, visitor):
    return DictExpr(vals={k: visitor.visit(v) for k, v in self.vals.items()})


def glom(value):
  """Evaluate and return a NumPy array (base.py:630-640)."""
  if isinstance(value, Expr):
    value = evaluate(value)
  if isinstance(value, np.ndarray):
    return value
  return value.glom()


def optimized_dag(node):
  if not isinstance(node, Expr):
    raise TypeError
  from . import optimize
  return optimize.optimize(node)


def force(node):
  return evaluate(node)


def evaluate(node):
  if isinstance(node, Expr):
    return node.force()
  assert isinstance(node, (np.ndarray, distarray.DistArray)), type(node)
  return node


def eager(node):
  return Val(val=force(node))


def lazify(val):
  if isinstance(val, Expr):
    return val
  if isinstance(val, dict):
    return DictExpr(vals=val)
  if isinstance(val, list):
    return ListExpr(vals=val)
  if isinstance(val, tuple):
    return TupleExpr(vals=val)
  return Val(val=val)


def as_array(v):
  if isinstance(v, Expr):
    return v
  return AsArray(val=v)
