"""Local (tile-level) expressions and their lowering to the kernel IR.

Restates the tree of spartan/expr/local.py (LocalInput :54-69, FnCallExpr
:72-122, LocalMapExpr :127-128, LocalMapLocationExpr :130-142,
LocalReduceExpr :144-145).  The reference *evaluates* this tree with one NumPy
call per node per tile; here the tree is only ever *lowered* -- to the IR of
``spartan_amd.codegen`` -- and executed as one generated gfx950 kernel.

Lowering rules (``lower``):
  * NumPy ufuncs                      -> ``codegen.Op`` (NumPy dtype resolution);
  * registered builtin mappers        -> their IR (``ones``/``zeros`` constants,
                                         ``astype`` casts, ``rand``/``arange``
                                         generator leaves materialised by spx_fill);
  * any other Python callable         -> traced once with symbolic proxies
                                         (operators and ufuncs on the proxies
                                         record IR); if tracing fails
                                         (``UntraceableMapper``) the tree is
                                         evaluated per tile on the host exactly
                                         as the reference does
                                         (``host_evaluate``; counted in
                                         engine.HOST_MAPPER_CALLS, warned once).
                                         Trees of ufuncs / builtins never take
                                         that path.
"""
import itertools

import numpy as np

from .. import codegen

_var_ids = itertools.count()


class CodegenError(NotImplementedError):
  pass


class UntraceableMapper(CodegenError):
  """A USER mapper whose body cannot be traced into a kernel (data-dependent
  control flow, NumPy calls other than ufuncs on the tile, ...).  The engine
  then evaluates the tree on the host exactly as the reference does
  (engine.run_host_map); builtin ufunc trees never raise this."""

  def __init__(self, msg, fn=None):
    super().__init__(msg)
    self.fn = fn


def make_var():
  """Unique variable name for a tile input (reference local.py:27-29)."""
  return 'key_%d' % next(_var_ids)


class LocalExpr:
  def __init__(self, deps=None):
    self.deps = list(deps or [])

  def add_dep(self, v):
    self.deps.append(v)

  def input_names(self):
    out = []
    for d in self.deps:
      for n in d.input_names():
        if n not in out:
          out.append(n)
    return out

  def __repr__(self):
    return self.pretty_str()


class LocalInput(LocalExpr):
  def __init__(self, idx):
    super().__init__()
    assert idx
    self.idx = idx

  def pretty_str(self):
    return self.idx

  def input_names(self):
    return [self.idx]


class FnCallExpr(LocalExpr):
  def __init__(self, fn=None, deps=None, kw=None, pretty_fn=None):
    super().__init__(deps)
    assert fn is not None
    self.fn = fn
    self.kw = dict(kw or {})
    self.pretty_fn = pretty_fn

  def fn_name(self):
    if self.pretty_fn:
      return self.pretty_fn
    return getattr(self.fn, '__name__', repr(self.fn))

  def pretty_str(self):
    args = ','.join(d.pretty_str() for d in self.deps)
    return '%s(%s)' % (self.fn_name().split('.')[-1], args)


class LocalMapExpr(FnCallExpr):
  _op_type = 'map'


class LocalMapLocationExpr(LocalMapExpr):
  _op_type = 'map_location'


class LocalReduceExpr(FnCallExpr):
  _op_type = 'reduce'


def rowdot(a, w):
  """Host meaning of a fused ``dot(x, w)`` leaf (dot_map2_np_mapper,
  spartan/expr/dot.py:172-187): ``a`` an (n, K) tile, ``w`` the (1, K) row
  vector of the host (K, 1) operand.  Only ever lowered, never called on the
  product path."""
  return a.dot(w.reshape(-1, 1))


class LocalRowDot(LocalMapExpr):
  """``dot(x, w)`` with a small host ``w`` folded into a fused tree
  (DotReduceFusion): deps = [x input, (1, K) w input]."""

  def __init__(self, deps=None):
    super().__init__(fn=rowdot, deps=deps, pretty_fn='rowdot')


# ---------------------------------------------------------------- lowering
class Pre(codegen.In):
  """A generator leaf (rand / arange ...) materialised into a tile by spx_fill
  before the fused kernel runs; it then becomes an ordinary array input."""
  __slots__ = ('kind', 'params', 'src_var')

  def __init__(self, kind, dtype, params, src_var):
    super().__init__(-1, dtype)
    self.kind, self.params, self.src_var = kind, params, src_var

  def sig(self):
    return 'i%d:%s' % (self.slot, self.dtype.str)


# builtin mapper registry: fn -> (lowering callable(fn_expr, lowered_deps, env) -> IR)
_BUILTIN_LOWERINGS = {}


def register_lowering(fn, lowering):
  _BUILTIN_LOWERINGS[fn] = lowering
  return fn


class LowerEnv:
  """Maps LocalInput names to IR leaves while lowering one tree."""

  def __init__(self, leaves, extent=None):
    self.leaves = leaves  # var name -> IR leaf (In / Sc / Const) or ('array', dtype) placeholders
    self.pres = []        # Pre leaves created
    self.scalars = []     # Sc leaves created
    self.extent = extent  # the tile's TileExtent when lowering a location map per tile

  def new_scalar(self, value):
    sc = codegen.Sc(len(self.scalars), value)
    if len(self.scalars) >= codegen.MAX_IN:
      raise CodegenError('too many scalar constants in one fused expression')
    self.scalars.append(sc)
    return sc


def lower(op, env):
  """Lower a LocalExpr tree to codegen IR."""
  if isinstance(op, LocalInput):
    if op.idx not in env.leaves:
      raise CodegenError('unbound tile input %s' % op.idx)
    return env.leaves[op.idx]
  if not isinstance(op, FnCallExpr):
    raise CodegenError('cannot lower %r' % (op,))
  fn = op.fn
  if isinstance(op, LocalRowDot):
    a, w = (lower(d, env) for d in op.deps)
    if not isinstance(a, codegen.In) or not isinstance(w, codegen.In):
      raise CodegenError('row dot operands must be tile inputs')
    return codegen.RowDot(a, w)
  if fn in _BUILTIN_LOWERINGS:
    return _BUILTIN_LOWERINGS[fn](op, env)
  deps = [d for d in op.deps if not (isinstance(d, LocalInput) and d.idx == 'extent')]
  args = [lower(d, env) for d in deps]
  if isinstance(op, LocalMapLocationExpr):
    # map_with_location: fn(*tiles, (ul, lr, array_shape), **kw), traced once
    # per tile with that tile's location as plain Python values
    # (local.py:130-142); the location enters the IR as kernel-argument
    # scalars, so tiles whose traces agree share one compiled kernel
    if env.extent is None:
      raise CodegenError('location map %s lowered without a tile extent' % op.fn_name())
    return trace_callable(fn, args, op.kw, env, extra=(env.extent.to_tuple(),))
  if isinstance(fn, np.ufunc):
    if op.kw:
      raise CodegenError('ufunc %s with keywords %s' % (fn.__name__, op.kw))
    if fn.nout != 1 or fn.nin != len(args):
      raise CodegenError('ufunc %s arity' % fn.__name__)
    return codegen.Op(fn.__name__, args)
  return trace_callable(fn, args, op.kw, env)


# ------------------------------------------------------------------ tracing
class Sym:
  """Symbolic tile value used to trace user mapper functions into IR."""
  __array_priority__ = 1000

  def __init__(self, node, env, shape=None):
    self.node, self.env = node, env
    self.shape = shape  # tile shape when known (join mappers read tiles[i].shape)

  @property
  def ndim(self):
    return None if self.shape is None else len(self.shape)

  @property
  def dtype(self):
    return self.node.dtype

  def _wrap(self, v):
    if isinstance(v, Sym):
      return v.node
    if isinstance(v, (bool, int, float, np.generic)) and np.ndim(v) == 0:
      return self.env.new_scalar(v.item() if isinstance(v, np.generic) else v)
    raise CodegenError('cannot trace operand of type %s' % type(v).__name__)

  @staticmethod
  def _shape_of(vals):
    """Broadcast shape of the operands whose shapes are known (else None)."""
    shapes = [v.shape for v in vals if isinstance(v, Sym) and v.shape is not None]
    if not shapes:
      return None
    try:
      return tuple(np.broadcast_shapes(*shapes))
    except ValueError:
      raise CodegenError('operands of shapes %s do not broadcast' % (shapes,))

  def __array_ufunc__(self, ufunc, method, *inputs, **kw):
    if method != '__call__' or kw:
      raise CodegenError('unsupported ufunc use %s.%s %s' % (ufunc.__name__, method, kw))
    return Sym(codegen.Op(ufunc.__name__, [self._wrap(x) for x in inputs]), self.env, self._shape_of(inputs))

  def _bin(name, rev=False):
    def f(self, other):
      a, b = (other, self) if rev else (self, other)
      return Sym(codegen.Op(name, [self._wrap(a), self._wrap(b)]), self.env, self._shape_of((a, b)))
    return f

  __add__, __radd__ = _bin('add'), _bin('add', True)
  __sub__, __rsub__ = _bin('subtract'), _bin('subtract', True)
  __mul__, __rmul__ = _bin('multiply'), _bin('multiply', True)
  __truediv__, __rtruediv__ = _bin('true_divide'), _bin('true_divide', True)
  __floordiv__, __rfloordiv__ = _bin('floor_divide'), _bin('floor_divide', True)
  __mod__, __rmod__ = _bin('remainder'), _bin('remainder', True)
  __pow__, __rpow__ = _bin('power'), _bin('power', True)
  __lt__, __le__ = _bin('less'), _bin('less_equal')
  __gt__, __ge__ = _bin('greater'), _bin('greater_equal')
  __eq__, __ne__ = _bin('equal'), _bin('not_equal')
  __and__, __or__, __xor__ = _bin('logical_and'), _bin('logical_or'), _bin('logical_xor')
  del _bin

  def __neg__(self):
    return Sym(codegen.Op('negative', [self.node]), self.env, self.shape)

  def __abs__(self):
    return Sym(codegen.Op('absolute', [self.node]), self.env, self.shape)

  def astype(self, dtype):
    return Sym(codegen.Cast(self.node, np.dtype(dtype)), self.env, self.shape)

  def __bool__(self):
    raise CodegenError('data-dependent control flow cannot be traced')

  __hash__ = object.__hash__


def has_location(op):
  """True iff a LocalExpr tree contains a map_with_location call."""
  if isinstance(op, LocalMapLocationExpr):
    return True
  return any(has_location(d) for d in getattr(op, 'deps', ()))


def trace_callable(fn, args, kw, env, extra=()):
  syms = [Sym(a, env) for a in args]
  try:
    out = fn(*syms, *extra, **kw)
  except Exception as e:
    raise UntraceableMapper('mapper %s cannot be lowered to a gfx950 kernel (%s: %s)'
                            % (getattr(fn, '__name__', fn), type(e).__name__, e), fn)
  if isinstance(out, Sym):
    return out.node
  if extra and args and isinstance(out, (bool, int, float, np.generic)) and np.ndim(out) == 0:
    # a location mapper returning a scalar for a whole tile (e.g. nbody.py:30-40
    # _set_diagonal_mapper): the tile is filled with it, in the input's dtype
    return codegen.Const(out.item() if isinstance(out, np.generic) else out, args[0].dtype)
  raise UntraceableMapper('mapper %s did not return a traced tile value' % getattr(fn, '__name__', fn), fn)


def host_evaluate(op, env):
  """The reference's per-tile evaluation of a LocalExpr tree
  (FnCallExpr.evaluate, spartan/expr/local.py:110-122, and
  LocalMapLocationExpr.evaluate, :133-142): ``fn(*deps, **kw)`` on host NumPy
  tiles, recursively.  ``env``: var name -> NumPy tile / scalar, 'extent' ->
  the TileExtent.  Used only for trees holding an untraceable USER mapper."""
  if isinstance(op, LocalInput):
    return env[op.idx]
  deps = []
  for d in op.deps:
    if isinstance(d, LocalInput) and d.idx == 'extent' and isinstance(op, LocalMapLocationExpr):
      deps.append(env['extent'].to_tuple())
    else:
      deps.append(host_evaluate(d, env))
  return op.fn(*deps, **op.kw)
