"""Replay of optimised DAGs whose structure repeats (Expr.optimized()).

Iterative drivers rebuild the same DAG every iteration with new host values:
the reference's linear regression (spartan/examples/linear_regression.py:
10-16, driven by sgd.py:34-39) builds ``sum(x * (dot(x, w) - y), axis=0)``
with a new host ``w`` each step and calls ``.optimized()`` on it, which
re-runs every rewrite pass (CollapsedCachedExpressions, AutomaticTiling,
the fusions) on an identical structure -- at cfg5 that host work is ~10 % of
an iteration next to a 4 ms kernel.

Here the first optimisation of a structure is kept as a *template*: a copy
of the optimised DAG that has never been evaluated, in which every leaf
object of the input DAG (host arrays, forced DistArrays, cached values) is
replaced by a numbered slot.  A later DAG with the same signature is
optimised by instantiating the template with its own leaf objects.  Node
ids follow what the passes do: a template node that kept the id of an input
node (passes rewrite with expr_like, which keeps ids) takes the id of the
corresponding node of the NEW input, so the evaluation cache sees exactly
what a fresh optimisation would give it (a value evaluated through this DAG
is found again by the next DAG that shares the node -- the reference's
KMeans loop forces ``labels`` through ``counts`` and reuses it for the
centres); nodes the passes created get fresh ids.  The fused LocalExpr trees
are copied as they are, so codegen finds the kernels it already built.

The signature is the DAG's structure with leaves abstracted:
  * Expr / LocalExpr nodes: class and every attribute except the id and the
    memoised shape / optimised-DAG fields;
  * generated variable names (``key_N``) and leaf objects are numbered by
    first appearance, so sharing patterns must match too;
  * host arrays: shape and dtype (the values are what changes);
  * DistArrays: type, shape, dtype and tile layout (the value is a slot:
    replay substitutes the new DAG's own array), views excluded;
  * functions / ufuncs: identity -- the cache entry keeps them alive, so an
    id cannot be reused by another function while the entry exists;
    plain scalars, strings, dtypes: value;
  * whether a node's value is already in the evaluation cache (the template
    then holds that value as a slot, as CollapsedCachedExpressions made it a
    Val), the tiling an earlier AutomaticTiling pinned on a node, and the
    optimisation flags / worker count the passes read.
Replay also repeats AutomaticTiling's side effect: each instantiated node
gets the tiling the template's node was given (optimize._tiled_exprs).
A structure whose optimised form holds a host array that is neither a leaf
of the input nor a contiguous same-size view of one (a pass derived new
values) is not cached: it is optimised every time, as before.
"""
import numpy as np

from ..config import FLAGS

_SKIP = ('expr_id', 'optimized_expr', '_shape_memo')
_PLANS = {}
_MAX_PLANS = 256
STATS = {'hits': 0, 'misses': 0, 'uncacheable': 0}


class _Slot:
  __slots__ = ('i',)

  def __init__(self, i):
    self.i = i


class _View:
  """A reshaped, contiguous view of host-array slot i."""
  __slots__ = ('i', 'shape')

  def __init__(self, i, shape):
    self.i = i
    self.shape = shape


class _Uncacheable(Exception):
  pass


def _is_leaf_obj(v):
  from ..array.distarray import DistArray
  return isinstance(v, (np.ndarray, DistArray))


_CLASSES = None


def _classes():
  global _CLASSES
  if _CLASSES is None:
    from ..array.distarray import DistArray
    from .base import Expr, eval_cache
    from .local import LocalExpr
    _CLASSES = (Expr, LocalExpr, DistArray, eval_cache)
  return _CLASSES


_SCALARS = (bool, int, float, complex, type(None))


class _Sig:
  def __init__(self):
    self.vars = {}
    self.slots = []       # leaf objects in first-appearance order
    self.slot_ids = {}    # id(obj) -> slot index
    self.memo = {}        # id(node) -> back-reference
    self.nodes = []       # input Expr nodes in memo order
    self.keep = []        # objects whose identity is part of the key
    self.Expr, self.LocalExpr, self.DistArray, self.cache = _classes()
    from .optimize import _tiled_exprs
    self.tiled = _tiled_exprs

  def slot(self, obj):
    k = id(obj)
    i = self.slot_ids.get(k)
    if i is not None:
      return ('S', i)
    self.slot_ids[k] = len(self.slots)
    self.slots.append(obj)
    return None

  def walk(self, v):
    t = type(v)
    if t in _SCALARS:
      return v if t is not float else ('f', repr(v))
    if t is str:
      if v.startswith('key_'):
        n = self.vars.get(v)
        if n is None:
          n = self.vars[v] = len(self.vars)
        return ('var', n)
      return v
    if t is list or t is tuple:
      return (t is list,) + tuple([self.walk(e) for e in v])
    if isinstance(v, self.Expr):
      k = id(v)
      m = self.memo.get(k)
      if m is not None:
        return ('ref', m)
      self.memo[k] = len(self.memo)
      self.nodes.append(v)
      cached = self.cache.cache.get(v.expr_id)
      if cached is not None:  # CollapsedCachedExpressions turns it into a Val of this value
        return ('cached', t, self.slot(cached) or self._obj_sig(cached))
      # attributes in insertion order: a node built another way only misses
      # (the names are part of the key), never collides; plus the tiling an
      # earlier optimisation pinned on this node (AutomaticTiling reads it)
      return (t, self.tiled.get(v.expr_id)) + tuple(
          [(a, self.walk(b)) for a, b in v.__dict__.items() if a not in _SKIP])
    if isinstance(v, self.LocalExpr):
      return (t,) + tuple([(a, self.walk(b)) for a, b in v.__dict__.items()])
    if t is np.ndarray:
      return self.slot(v) or ('np', v.shape, v.dtype.str, v.flags.c_contiguous)
    if isinstance(v, self.DistArray):
      return self.slot(v) or self._obj_sig(v)
    if t is dict:
      return ('d',) + tuple([(a, self.walk(v[a])) for a in sorted(v, key=repr)])
    if isinstance(v, np.generic):
      return ('g', v.dtype.str, repr(v.item()))
    if isinstance(v, np.dtype):
      return ('dt', v.str)
    if callable(v):  # functions, ufuncs, classes: identity (kept alive by the entry)
      self.keep.append(v)
      return ('f', id(v))
    raise _Uncacheable(t.__name__)

  def _obj_sig(self, v):
    # an array's layout never changes after it is built: memoised on the object
    sig = getattr(v, '_plan_sig', None)
    if sig is not None:
      return sig
    sig = self._obj_sig_new(v)
    try:
      v._plan_sig = sig
    except AttributeError:
      pass
    return sig

  def _obj_sig_new(self, v):
    from ..array.distarray import DistArrayImpl, LocalWrapper
    if not isinstance(v, (DistArrayImpl, LocalWrapper)):
      if isinstance(v, np.ndarray):
        return ('np', v.shape, v.dtype.str, v.flags.c_contiguous)
      raise _Uncacheable(type(v).__name__)  # views, scalars in the cache, ...
    tiles = getattr(v, 'tiles', None)
    layout = None
    if isinstance(tiles, dict):
      layout = tuple(sorted((tuple(ex.ul), tuple(ex.lr), w) for ex, w in tiles.items())) if len(tiles) <= 64 \
          else (len(tiles), hash(tuple(sorted((tuple(ex.ul), tuple(ex.lr), w) for ex, w in tiles.items()))))
    return ('o', type(v).__name__, tuple(getattr(v, 'shape', ())), str(getattr(v, 'dtype', '')), layout,
            getattr(v, 'replicated', None))


_FLAGS_KEY = [None, None]  # (FLAGS.version, key)


def _flags_key():
  if _FLAGS_KEY[0] != FLAGS.version:
    _FLAGS_KEY[1] = tuple(sorted((k, repr(v)) for k, v in FLAGS.items().items()
                                 if k.startswith('opt') or k == 'optimization'))
    _FLAGS_KEY[0] = FLAGS.version
  return _FLAGS_KEY[1]


def signature(dag):
  """(key, walk state: .slots leaf objects, .nodes Expr nodes, .keep) of
  ``dag``, or (None, None) if it has a part the signature does not
  understand."""
  from .. import runtime
  s = _Sig()
  try:
    body = s.walk(dag)
  except _Uncacheable:
    return None, None
  ctx = runtime.get() if runtime._ctx is not None else None
  key = (body, _flags_key(), ctx.num_workers if ctx else None, ctx.world_size if ctx else None)
  return key, s


def _template(v, slot_ids, slots, memo, id2pos=None):
  """Copy of optimised value ``v`` with leaf objects replaced by slots and
  never-evaluated expression nodes; ``_tpl_pos`` on a node is the position
  of the input node whose id it kept (None: a node the passes created)."""
  from .base import Expr
  from .local import LocalExpr
  k = id(v)
  if k in slot_ids:
    return _Slot(slot_ids[k])
  if isinstance(v, np.ndarray):
    # a pass's reshape of a host leaf: same bytes, both C-contiguous
    if v.flags.c_contiguous:
      for i, o in enumerate(slots):
        if isinstance(o, np.ndarray) and o.flags.c_contiguous and o.dtype == v.dtype and o.size == v.size \
            and o.__array_interface__['data'][0] == v.__array_interface__['data'][0]:
          return _View(i, v.shape)
    raise _Uncacheable('derived host array')
  if isinstance(v, (list, tuple)):
    return type(v)(_template(e, slot_ids, slots, memo, id2pos) for e in v)
  if isinstance(v, dict):
    return {a: _template(b, slot_ids, slots, memo, id2pos) for a, b in v.items()}
  if isinstance(v, (Expr, LocalExpr)):
    if k in memo:
      return memo[k]
    new = v.__class__.__new__(v.__class__)
    memo[k] = new
    for a, b in v.__dict__.items():
      if a in ('expr_id', 'optimized_expr'):
        continue
      new.__dict__[a] = _template(b, slot_ids, slots, memo, id2pos)
    if isinstance(v, Expr):
      new.__dict__['_tpl_pos'] = id2pos.get(v.expr_id)
      # the tiling AutomaticTiling chose for this node: replay pins it on the
      # instance's node too, as a fresh optimisation would have
      from .optimize import _tiled_exprs
      new.__dict__['_tpl_tiling'] = _tiled_exprs.get(v.expr_id)
    elif _pure(new.__dict__):
      # no slot, view or expression inside: every instantiation shares this
      # tree object (engine.bind lowers it once per binding pattern)
      new.__dict__['_tpl_pure'] = True
    return new
  if _is_leaf_obj(v):
    raise _Uncacheable('leaf object outside the input DAG')
  return v


def _pure(v):
  """True iff template value ``v`` holds no slot, view or expression node."""
  from .base import Expr
  from .local import LocalExpr
  t = type(v)
  if t is _Slot or t is _View or isinstance(v, Expr):
    return False
  if t in (list, tuple):
    return all(_pure(e) for e in v)
  if t is dict:
    return all(_pure(e) for e in v.values())
  if isinstance(v, LocalExpr):
    return bool(v.__dict__.get('_tpl_pure'))
  return True


def _instantiate(v, slots, nodes):
  Expr, LocalExpr, _, cache = _classes()
  from .base import _new_id
  return _Inst(Expr, LocalExpr, cache, _new_id, slots, nodes).run(v)


class _Inst:
  def __init__(self, Expr, LocalExpr, cache, new_id, slots, nodes):
    self.Expr, self.LocalExpr, self.cache, self.new_id, self.slots = Expr, LocalExpr, cache, new_id, slots
    self.nodes = nodes
    from .optimize import _tiled_exprs
    self.tiled = _tiled_exprs
    self.memo = {}

  def run(self, v):
    t = type(v)
    if t is _Slot:
      return self.slots[v.i]
    if t is _View:
      return self.slots[v.i].reshape(v.shape)
    if t is list:
      return [self.run(e) for e in v]
    if t is tuple:
      return tuple([self.run(e) for e in v])
    if t is dict:
      return {a: self.run(b) for a, b in v.items()}
    if isinstance(v, (self.Expr, self.LocalExpr)):
      if v.__dict__.get('_tpl_pure'):
        return v
      k = id(v)
      new = self.memo.get(k)
      if new is not None:
        return new
      new = t.__new__(t)
      self.memo[k] = new
      nd = new.__dict__
      for a, b in v.__dict__.items():
        if a != '_tpl_pos' and a != '_tpl_tiling':
          nd[a] = self.run(b)
      if isinstance(v, self.Expr):
        pos = v.__dict__.get('_tpl_pos')
        new.expr_id = self.nodes[pos].expr_id if pos is not None else self.new_id()
        self.cache.register(new.expr_id)
        tiling = v.__dict__.get('_tpl_tiling')
        if tiling is not None:
          self.tiled[new.expr_id] = tiling
      return new
    return v


def optimize_cached(dag, run_passes):
  """``run_passes(dag)``, or the replay of an earlier identical structure."""
  from .. import comm
  key, st = signature(dag)
  if key is None:
    STATS['uncacheable'] += 1
    comm.spmd_note('plan', 'uncacheable')
    return run_passes(dag)
  entry = _PLANS.get(key)
  if entry is not None:
    STATS['hits'] += 1
    comm.spmd_note('plan', 'hit')
    return _instantiate(entry[0], st.slots, st.nodes)
  STATS['misses'] += 1
  comm.spmd_note('plan', 'miss')
  opt = run_passes(dag)
  try:
    tpl = _template(opt, {id(o): i for i, o in enumerate(st.slots)}, st.slots, {},
                    {n.expr_id: i for i, n in enumerate(st.nodes)})
  except _Uncacheable as e:
    STATS['last_uncacheable'] = str(e)
    return opt
  if len(_PLANS) >= _MAX_PLANS:
    _PLANS.pop(next(iter(_PLANS)))
  _PLANS[key] = (tpl, st.keep)
  return opt


def clear():
  _PLANS.clear()
