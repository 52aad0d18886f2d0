"""LocalExpr tree -> generated gfx950 HIP kernels.

The reference evaluates a fused map as a tree of NumPy ufunc calls per tile,
materialising one full-tile temporary per node (FnCallExpr.evaluate,
spartan/expr/local.py:110-122); its only codegen hook is the default-off
Parakeet pass (spartan/expr/optimize.py:260-365).  Here the tree that
MapMapFusion / ReduceMapFusion build is lowered to a small IR (``In``, ``Sc``,
``Const``, ``Op``, ``Cast``) with NumPy's own dtype resolution
(``ufunc.resolve_dtypes``), and the IR is emitted as straight-line HIP C++
inside one of three streaming kernel skeletons:

  * ``map``      -- elementwise; a dense fast path (flat index, 16-byte vector
                    loads/stores) and a general N-d strided/broadcast path;
  * ``rows``     -- reduce over a contiguous axis, (O, R) view, one or more
                    256-thread blocks per segment, wave/LDS tree at the end;
  * ``cols``     -- reduce over a strided axis, (O, R, I) view, lanes along the
                    contiguous I dim (coalesced 1 KiB per wave-instruction),
                    waves interleaved over R, LDS combine.

Reductions write partials [P][...] in the accumulator type; P > 1 partials are
combined deterministically by spx_reduce_finalize.

The source is compiled by ``backend.compile_kernel`` (device-only clang,
code object cached on disk by source hash) and launched through the C ABI
(spx_launch).  Nothing here executes on the CPU.
"""
import ctypes

import numpy as np

MAX_IN = 16
MAX_DIM = 8
# streamed contiguous vector loads carry the non-temporal hint (global_load
# ... nt): the inputs of a fused map / reduce are read exactly once
NT_LOADS = True


def _vstore(vtype, ptr_expr, val, nt):
  """Source of one contiguous vector store: non-temporal for large streamed
  outputs (backend.map picks the variant by output size; a runtime branch
  between the two forms is folded into one plain store by the compiler),
  plain otherwise (a small output stays in L2 / MALL for its next reader)."""
  if nt:
    return '__builtin_nontemporal_store(%s, (GLOBAL %s*)(%s));' % (val, vtype, ptr_expr)
  return '*(GLOBAL %s*)(%s) = %s;' % (vtype, ptr_expr, val)


def _vload(vtype, ptr_expr):
  """Source of one contiguous vector load of type ``vtype`` at ``ptr_expr``."""
  if NT_LOADS:
    return '__builtin_nontemporal_load((const GLOBAL %s*)(%s))' % (vtype, ptr_expr)
  return '*(const GLOBAL %s*)(%s)' % (vtype, ptr_expr)

# --------------------------------------------------------------------- IR

class In:
  """Array input ``slot`` (a device tile, possibly broadcast)."""
  __slots__ = ('slot', 'dtype')

  def __init__(self, slot, dtype):
    self.slot, self.dtype = slot, np.dtype(dtype)

  def sig(self):
    return 'i%d:%s' % (self.slot, self.dtype.str)


class Sc:
  """Scalar constant passed through the kernel arguments (NumPy 'weak' scalar)."""
  __slots__ = ('slot', 'pytype', 'dtype', 'value')

  def __init__(self, slot, value):
    if isinstance(value, (bool, np.bool_)):
      self.pytype, self.dtype, self.value = bool, np.dtype(np.bool_), bool(value)
    elif isinstance(value, (int, np.integer)):
      self.pytype, self.dtype, self.value = int, np.dtype(np.int64), int(value)
    else:
      self.pytype, self.dtype, self.value = float, np.dtype(np.float64), float(value)
    self.slot = slot

  def sig(self):
    return 's%d:%s' % (self.slot, self.pytype.__name__)


class Const:
  """Array-valued constant (``ones``/``zeros`` tiles): strong dtype, no memory."""
  __slots__ = ('value', 'dtype')

  def __init__(self, value, dtype):
    self.value, self.dtype = value, np.dtype(dtype)

  def sig(self):
    return 'c%r:%s' % (self.value, self.dtype.str)


class Op:
  __slots__ = ('name', 'args', 'in_dtypes', 'dtype')

  def __init__(self, name, args):
    self.name = name
    self.args = list(args)
    uf = getattr(np, name)
    keys = tuple(a.pytype if isinstance(a, Sc) else a.dtype for a in self.args)
    try:
      res = uf.resolve_dtypes(keys + (None,) * uf.nout)
    except Exception as e:  # pragma: no cover - numpy raises for invalid combos
      raise TypeError('ufunc %s has no loop for %s: %s' % (name, keys, e))
    self.in_dtypes = tuple(np.dtype(d) for d in res[:uf.nin])
    self.dtype = np.dtype(res[uf.nin])

  def sig(self):
    return '%s(%s)' % (self.name, ','.join(a.sig() for a in self.args))


class Cast:
  __slots__ = ('arg', 'dtype')

  def __init__(self, arg, dtype):
    self.arg, self.dtype = arg, np.dtype(dtype)

  def sig(self):
    return 'cast<%s>(%s)' % (self.dtype.str, self.arg.sig())


class RowDot:
  """Per-row dot product ``a[i, :] . w`` of a fused ``dot(x, w)`` whose right
  operand is a small host (K, 1) vector (DotReduceFusion): the value of
  ``dot_map2_np_mapper`` (spartan/expr/dot.py:172-187) for row i, broadcast
  along the row.  ``a`` is the (N, K) input itself, ``w`` a (1, K) broadcast
  input; the row's K products are summed inside the lane group that holds the
  row (only the 'cols' reduce skeleton with one column tile supports it)."""
  __slots__ = ('a', 'w', 'dtype', 'rid')

  def __init__(self, a, w):
    self.a, self.w = a, w
    self.dtype = np.result_type(a.dtype, w.dtype)
    self.rid = 0

  def sig(self):
    return 'rowdot(%s,%s)' % (self.a.sig(), self.w.sig())


def walk(node):
  yield node
  if isinstance(node, Op):
    for a in node.args:
      yield from walk(a)
  elif isinstance(node, Cast):
    yield from walk(node.arg)
  elif isinstance(node, RowDot):
    yield from walk(node.a)
    yield from walk(node.w)


def unique_nodes(root):
  """Nodes of a tree (a DAG when leaves are shared), each object once."""
  seen, out = set(), []
  for n in walk(root):
    if id(n) not in seen:
      seen.add(id(n))
      out.append(n)
  return out


def rowdots(root):
  """Unique RowDot nodes of a tree, numbered (rid) in first-visit order."""
  out = []
  for n in walk(root):
    if isinstance(n, RowDot) and not any(n is m for m in out):
      n.rid = len(out)
      out.append(n)
  return out


# ------------------------------------------------------------ C emission

CTYPE = {'?': 'u8', 'i1': 'signed char', 'u1': 'u8', 'i2': 'short', 'i4': 'int', 'i8': 'i64',
         'f4': 'float', 'f8': 'double'}


def ctype(dt):
  dt = np.dtype(dt)
  key = '?' if dt.kind == 'b' else dt.str[1:]
  if key not in CTYPE:
    raise TypeError('dtype %s not supported by the gfx950 codegen' % dt)
  return CTYPE[key]


def is_float(dt):
  return np.dtype(dt).kind == 'f'


def is_bool(dt):
  return np.dtype(dt).kind == 'b'


OCML_1 = {  # name -> ocml suffix (f32/f64 variants)
    'exp': 'exp', 'log': 'log', 'sqrt': 'sqrt', 'sin': 'sin', 'cos': 'cos', 'tan': 'tan',
    'tanh': 'tanh', 'sinh': 'sinh', 'cosh': 'cosh', 'arcsin': 'asin', 'arccos': 'acos',
    'arctan': 'atan', 'exp2': 'exp2', 'log2': 'log2', 'log10': 'log10', 'expm1': 'expm1',
    'log1p': 'log1p', 'floor': 'floor', 'ceil': 'ceil', 'trunc': 'trunc', 'rint': 'rint',
    'cbrt': 'cbrt', 'fabs': 'fabs',
}
OCML_2 = {'power': 'pow', 'arctan2': 'atan2', 'fmod': 'fmod', 'hypot': 'hypot'}


class Emitter:
  """Emits the statements computing one element of the IR tree."""

  def __init__(self):
    self.ocml = set()
    self.lines = []
    self.n = 0

  def tmp(self, ct, expr):
    name = 't%d' % self.n
    self.n += 1
    self.lines.append('%s %s = %s;' % (ct, name, expr))
    return name

  def conv(self, val, src_dt, dst_dt):
    src_dt, dst_dt = np.dtype(src_dt), np.dtype(dst_dt)
    if src_dt == dst_dt:
      return val
    if is_bool(dst_dt):
      return '(u8)((%s) != 0)' % val
    return '(%s)(%s)' % (ctype(dst_dt), val)

  def ocml_call(self, fname, dt, args):
    suf = 'f32' if np.dtype(dt) == np.float32 else 'f64'
    full = '__ocml_%s_%s' % (fname, suf)
    self.ocml.add((full, ctype(dt), len(args)))
    return '%s(%s)' % (full, ', '.join(args))

  def emit(self, node, leaf):
    """Return a C expression (usually a temporary) of node.dtype."""
    if isinstance(node, In):
      return leaf(node)
    if isinstance(node, (Sc, RowDot)):
      return leaf(node)
    if isinstance(node, Const):
      if is_float(node.dtype):
        return '(%s)%r' % (ctype(node.dtype), float(node.value))
      return '(%s)%d' % (ctype(node.dtype), int(node.value))
    if isinstance(node, Cast):
      v = self.emit(node.arg, leaf)
      return self.tmp(ctype(node.dtype), self.conv(v, node.arg.dtype, node.dtype))
    assert isinstance(node, Op)
    args = [self.conv(self.emit(a, leaf), a.dtype, t) for a, t in zip(node.args, node.in_dtypes)]
    return self.tmp(ctype(node.dtype), self.op_expr(node, args))

  def op_expr(self, node, a):
    name = node.name
    T = node.in_dtypes[0] if node.in_dtypes else node.dtype
    fl = is_float(T)
    bl = is_bool(T)
    ct = ctype(T)
    if name == 'add':
      return '(u8)(%s | %s)' % (a[0], a[1]) if bl else '%s + %s' % (a[0], a[1])
    if name == 'subtract':
      return '%s - %s' % (a[0], a[1])
    if name == 'multiply':
      return '(u8)(%s & %s)' % (a[0], a[1]) if bl else '%s * %s' % (a[0], a[1])
    if name in ('true_divide', 'divide'):
      return '%s / %s' % (a[0], a[1])
    if name == 'floor_divide':
      if fl:
        return self.ocml_call('floor', T, ['%s / %s' % (a[0], a[1])])
      return 'fdiv_i(%s, %s)' % (a[0], a[1])
    if name in ('remainder', 'mod'):
      if fl:
        return 'fmod_py(%s, %s)' % (a[0], a[1]) if self.ocml_call('fmod', T, [a[0], a[1]]) else ''
      return 'fmod_i(%s, %s)' % (a[0], a[1])
    if name == 'negative':
      return '-%s' % a[0]
    if name == 'positive':
      return a[0]
    if name == 'absolute':
      if fl:
        return self.ocml_call('fabs', T, [a[0]])
      return '(%s < 0 ? -%s : %s)' % (a[0], a[0], a[0]) if not bl else a[0]
    if name == 'square':
      return '%s * %s' % (a[0], a[0])
    if name == 'reciprocal':
      return '(%s)1 / %s' % (ct, a[0])
    if name == 'sign':
      return '(%s)((%s > 0) - (%s < 0))' % (ct, a[0], a[0]) if not fl else \
             '(%s != %s ? %s : (%s)((%s > 0) - (%s < 0)))' % (a[0], a[0], a[0], ct, a[0], a[0])
    if name in ('maximum', 'minimum'):
      cmp = '>' if name == 'maximum' else '<'
      if fl:  # NaN propagates like np.maximum / np.minimum
        return '((%s != %s) ? %s : ((%s != %s) ? %s : (%s %s %s ? %s : %s)))' % (
            a[0], a[0], a[0], a[1], a[1], a[1], a[0], cmp, a[1], a[0], a[1])
      return '(%s %s %s ? %s : %s)' % (a[0], cmp, a[1], a[0], a[1])
    if name in ('fmax', 'fmin'):
      return self.ocml_call(name, T, [a[0], a[1]])
    cmps = {'equal': '==', 'not_equal': '!=', 'less': '<', 'less_equal': '<=', 'greater': '>',
            'greater_equal': '>='}
    if name in cmps:
      return '(u8)(%s %s %s)' % (a[0], cmps[name], a[1])
    if name == 'logical_and':
      return '(u8)((%s != 0) && (%s != 0))' % (a[0], a[1])
    if name == 'logical_or':
      return '(u8)((%s != 0) || (%s != 0))' % (a[0], a[1])
    if name == 'logical_xor':
      return '(u8)((%s != 0) != (%s != 0))' % (a[0], a[1])
    if name == 'logical_not':
      return '(u8)(%s == 0)' % a[0]
    if name == 'isnan':
      return '(u8)(%s != %s)' % (a[0], a[0])
    if name == 'isinf':
      return '(u8)(%s == (%s)__builtin_inf() || %s == -(%s)__builtin_inf())' % (a[0], ct, a[0], ct)
    if name == 'isfinite':
      return '(u8)(%s - %s == (%s)0)' % (a[0], a[0], ct)
    if name == 'power':
      if fl:
        return self.ocml_call('pow', T, [a[0], a[1]])
      return 'ipow(%s, %s)' % (a[0], a[1])
    if name in OCML_1 and fl:
      return self.ocml_call(OCML_1[name], T, [a[0]])
    if name in OCML_2 and fl:
      return self.ocml_call(OCML_2[name], T, [a[0], a[1]])
    raise NotImplementedError('ufunc %s has no gfx950 lowering' % name)


PRELUDE = r'''
typedef long long i64;
typedef unsigned long long u64;
typedef unsigned int u32;
typedef unsigned char u8;
#define DEV static __attribute__((device)) inline __attribute__((always_inline))
#define KERN extern "C" __attribute__((global)) __attribute__((amdgpu_flat_work_group_size(256, 256)))
#define SHARED __attribute__((shared))
#define GLOBAL __attribute__((address_space(1)))
DEV u32 tid() { return __builtin_amdgcn_workitem_id_x(); }
DEV u32 bidx() { return __builtin_amdgcn_workgroup_id_x(); }
DEV void bsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
DEV i64 fdiv_i(i64 a, i64 b) { if (b == 0) return 0; i64 q = a / b; if ((a % b != 0) && ((a < 0) != (b < 0))) q -= 1; return q; }
DEV i64 fmod_i(i64 a, i64 b) { if (b == 0) return 0; i64 r = a % b; if (r != 0 && ((r < 0) != (b < 0))) r += b; return r; }
DEV i64 ipow(i64 a, i64 b) { i64 r = 1; while (b > 0) { if (b & 1) r *= a; a *= a; b >>= 1; } return r; }
struct KArgs {
  u64 ptr[16];
  u64 out0, out1;
  i64 dim[8];
  i64 str[16][8];
  double fsc[16];
  i64 isc[16];
  i64 n;
  i64 aux[8];
  i64 tshape[8], tul[8], ashape[8];
  u32 flags, grid;
};
'''


class KArgs(ctypes.Structure):
  _fields_ = [
      ('ptr', ctypes.c_uint64 * 16),
      ('out0', ctypes.c_uint64),
      ('out1', ctypes.c_uint64),
      ('dim', ctypes.c_int64 * 8),
      ('str', (ctypes.c_int64 * 8) * 16),
      ('fsc', ctypes.c_double * 16),
      ('isc', ctypes.c_int64 * 16),
      ('n', ctypes.c_int64),
      ('aux', ctypes.c_int64 * 8),
      ('tshape', ctypes.c_int64 * 8),
      ('tul', ctypes.c_int64 * 8),
      ('ashape', ctypes.c_int64 * 8),
      ('flags', ctypes.c_uint32),
      ('grid', ctypes.c_uint32),
  ]


def _ocml_decls(ocml):
  out = []
  for full, ct, nargs in sorted(ocml):
    out.append('extern "C" __attribute__((device)) %s %s(%s);' % (ct, full, ', '.join([ct] * nargs)))
  if any(f.startswith('__ocml_fmod') for f, _, _ in ocml):
    for full, ct, nargs in sorted(ocml):
      if full.startswith('__ocml_fmod'):
        out.append('DEV %s fmod_py(%s a, %s b) { %s r = %s(a, b); if (r != 0 && ((r < 0) != (b < 0))) r += b; return r; }'
                   % (ct, ct, ct, ct, full))
  return '\n'.join(out)


# ---------------------------------------------------------- input classes
# Per array input, how its innermost iteration dim is addressed:
#   'c' contiguous (stride 1, vector loads), 'b' broadcast (stride 0),
#   'g' gather (any other stride).

def _load_vec(slot, dt, cls, off, V):
  """Statements loading V consecutive elements (along the innermost dim) into x<slot>[V]."""
  ct = ctype(dt)
  p = '((const GLOBAL %s*)a.ptr[%d])' % (ct, slot)
  if V == 1:
    return ['%s x%d_0 = %s[%s];' % (ct, slot, p, off)]
  if cls == 'c':
    vt = '%s __attribute__((ext_vector_type(%d)))' % (ct, V)
    lines = ['typedef %s vt%d;' % (vt, slot),
             'vt%d xv%d = %s;' % (slot, slot, _vload('vt%d' % slot, '%s + %s' % (p, off)))]
    lines += ['%s x%d_%d = xv%d[%d];' % (ct, slot, j, slot, j) for j in range(V)]
    return lines
  if cls == 'b':
    lines = ['%s x%d_0 = %s[%s];' % (ct, slot, p, off)]
    lines += ['%s x%d_%d = x%d_0;' % (ct, slot, j, slot) for j in range(1, V)]
    return lines
  return ['%s x%d_%d = %s[%s + %d * s%d_in];' % (ct, slot, j, p, off, j, slot) for j in range(V)]


def _expr_fn(root, n_in, name='fexpr'):
  """Device function computing the tree for one element from x<slot> scalars."""
  em = Emitter()

  def leaf(node):
    if isinstance(node, In):
      return 'x%d' % node.slot
    if isinstance(node, RowDot):
      return 'rd%d' % node.rid
    if node.pytype is float:
      return 'a.fsc[%d]' % node.slot
    return 'a.isc[%d]' % node.slot

  val = em.emit(root, leaf)
  params = ', '.join(['const KArgs& a'] + ['%s x%d' % (ctype(dt), s) for s, dt in n_in] +
                     ['%s rd%d' % (ctype(r.dtype), r.rid) for r in rowdots(root)])
  body = '\n  '.join(em.lines + ['return %s;' % val])
  fn = 'DEV %s %s(%s) {\n  %s\n}' % (ctype(root.dtype), name, params, body)
  return fn, em.ocml


def _call_expr(inputs, j, name='fexpr', n_rd=0, sfx=''):
  return '%s(a%s%s)' % (name, ''.join(', x%d_%d%s' % (s, j, sfx) for s, _ in inputs),
                        ''.join(', rd%d%s' % (k, sfx) for k in range(n_rd)))


_NAME_RE = None


def _suffix_names(line, sfx):
  """Rename the per-load identifiers of a _load_vec / loads() line."""
  global _NAME_RE
  import re
  if _NAME_RE is None:
    _NAME_RE = re.compile(r'\b(off\d+|s\d+_in|vt\d+|xv\d+|x\d+_\d+)\b')
  return _NAME_RE.sub(lambda m: m.group(1) + sfx, line)


def rows_unroll(inputs, classes):
  """Unrolled steps of the row-reduce loop: 4 for one streamed input, 2 for
  two, 1 from three on (cfg2's x*y+exp(z) already streams 3 KiB per wave)."""
  streamed = sum(1 for c in classes if c != 'b')
  return 4 if streamed <= 1 else 2 if streamed == 2 else 1


def cols_unroll(inputs, classes, vec, row_strides=None):
  """Rows per lane group per iteration of the column-reduce loop: enough that
  each wave keeps >= ~3 KiB of streamed loads in flight (Little's law at
  ~8 TB/s over 256 CUs needs ~32-64 KiB per CU).  Inputs broadcast along the
  columns ('b') or along the reduced rows (row stride 0, e.g. the (1, K) row
  vector of a fused row dot) cost no HBM stream; one row of 3 contiguous
  fp32x4 inputs is 3 KiB per wave."""
  streamed = 0
  for k, ((s, dt), cls) in enumerate(zip(inputs, classes)):
    if cls != 'b' and not (row_strides is not None and row_strides[k] == 0):
      streamed += np.dtype(dt).itemsize * vec
  if streamed >= 48:
    return 1
  if streamed >= 24:
    return 2
  return 4


def named(src, base, kind):
  """Give a generated kernel a distinct entry name: ``<base>_<kind>_<h>``,
  h = 8 hex digits of the source's SHA-1 (e.g. spx_reduce_cols_1a2b3c4d), so
  rocprofv3 reports every generated kernel on its own row instead of folding
  all of them into one 'spx_reduce' line.  Returns (source, name)."""
  import hashlib
  h = hashlib.sha1(src.encode()).hexdigest()[:8]
  name = '%s_%s_%s' % (base, kind, h)
  old = 'KERN void %s(' % base
  assert src.count(old) == 1, 'generated source has no single %s entry' % base
  return src.replace(old, 'KERN void %s(' % name), name


# ---------------------------------------------------------------- map
def gen_map(root, inputs, classes, ndim, vec, dense, nt_store=False, unroll=1):
  """Elementwise kernel.  inputs: [(slot, dtype)], classes: per-input 'c'/'b'/'g'.

  dense=True: every input is contiguous with the output's shape (flat index).
  Otherwise the N-d path: offsets from the iteration index via dim[] / str[][].
  unroll: grid steps per lane (dense vector path), all loads first; the
  launch's grid is n / (256 vec unroll) (backend.MAP_UNROLL).
  """
  if rowdots(root):
    raise NotImplementedError('a fused row dot needs the column-reduce skeleton')
  fn, ocml = _expr_fn(root, inputs)
  out_ct = ctype(root.dtype)
  L = []

  def body(V, dense_):
    b = []
    if dense_:
      offs = {s: 'e' for s, _ in inputs}
    else:
      b.append('i64 rem = e;')
      for s, _ in inputs:
        b.append('i64 o%d = 0;' % s)
      for d in range(ndim - 1, -1, -1):
        b.append('{ i64 q = rem / a.dim[%d]; i64 ix = rem - q * a.dim[%d]; rem = q;' % (d, d))
        for s, _ in inputs:
          b.append('  o%d += ix * a.str[%d][%d];' % (s, s, d))
        b.append('}')
      offs = {s: 'o%d' % s for s, _ in inputs}
    for (s, dt), cls in zip(inputs, classes):
      if not dense_ and cls == 'g' and V > 1:
        b.append('const i64 s%d_in = a.str[%d][%d];' % (s, s, ndim - 1))
      b += _load_vec(s, dt, 'c' if dense_ else cls, offs[s], V)
    outp = '((GLOBAL %s*)a.out0)' % out_ct
    if V == 1:
      b.append('%s[e] = %s;' % (outp, _call_expr(inputs, 0)))
    else:
      b.append('typedef %s __attribute__((ext_vector_type(%d))) vo;' % (out_ct, V))
      b.append('vo r;')
      for j in range(V):
        b.append('r[%d] = %s;' % (j, _call_expr(inputs, j)))
      b.append(_vstore('vo', '%s + e' % outp, 'r', nt_store))
    return b

  L.append('KERN void spx_map(KArgs a) {')
  L.append('  const i64 n = a.n;')
  L.append('  if (a.flags & 1) {')
  L.append('    const i64 step = (i64)a.grid * 256 * %d;' % vec)
  L.append('    i64 e = ((i64)bidx() * 256 + tid()) * %d;' % vec)
  # dense maps: U grid steps per lane, all loads first (with the full grid,
  # U = 1, every lane has one vector: profiles/r02_map_grid.txt)
  U = unroll if dense and vec > 1 else 1
  if U > 1:
    L.append('    for (; e + %d * step < n; e += %d * step) {' % (U - 1, U))
    lines = []
    for u in range(U):
      for s_, dt in inputs:
        lines += [_suffix_names(x, '_u%d' % u) for x in _load_vec(s_, dt, 'c', '(e + %d * step)' % u, vec)]
    lines.append('typedef %s __attribute__((ext_vector_type(%d))) vo;' % (out_ct, vec))
    for u in range(U):
      lines.append('{ vo r;')
      for j in range(vec):
        lines.append('  r[%d] = %s;' % (j, _call_expr(inputs, j, sfx='_u%d' % u)))
      lines.append('  %s }' % _vstore('vo', '((GLOBAL %s*)a.out0) + (e + %d * step)' % (out_ct, u), 'r', nt_store))
    L += ['      ' + x for x in lines]
    L.append('    }')
  L.append('    for (; e < n; e += step) {')
  L += ['      ' + x for x in body(vec, dense)]
  L.append('    }')
  L.append('  } else {')
  L.append('    const i64 step = (i64)a.grid * 256;')
  L.append('    for (i64 e = (i64)bidx() * 256 + tid(); e < n; e += step) {')
  L += ['      ' + x for x in body(1, dense)]
  L.append('    }')
  L.append('  }')
  L.append('}')
  src = '\n'.join([PRELUDE, _ocml_decls(ocml), fn, '\n'.join(L)])
  return src


# -------------------------------------------------------------- reduce
REDOPS = ('sum', 'min', 'max', 'argmin', 'argmax')


def acc_dtype(op, dt):
  dt = np.dtype(dt)
  if op == 'sum':
    if dt.kind in 'biu':
      return np.dtype(np.int64)
    return dt
  if op in ('min', 'max'):
    if dt.kind == 'b':
      return np.dtype(np.int64)
    return dt
  # arg ops keep the value type
  if dt.kind == 'b':
    return np.dtype(np.int64)
  return dt


def partial_dtype(op, adt, interleave):
  """dtype of a column reduction's per-block partials: fp64 for an
  interleaved fp32 sum (its lane totals are fp64, codegen 'cols'), else the
  accumulator dtype."""
  if interleave and op == 'sum' and np.dtype(adt) == np.float32:
    return np.dtype(np.float64)
  return np.dtype(adt)


def _ident(op, dt):
  ct = ctype(dt)
  if op == 'sum':
    return '(%s)0' % ct
  if is_float(dt):
    return '(%s)__builtin_inf()' % ct if op in ('min', 'argmin') else '-(%s)__builtin_inf()' % ct
  # the value type's own extremes (a truncated int64 extreme would be -1 / 0)
  ii = np.iinfo(dt)
  v = int(ii.max) if op in ('min', 'argmin') else int(ii.min)
  if v == -(1 << 63):
    return '(%s)(-0x7fffffffffffffffLL - 1)' % ct
  return '(%s)%dULL' % (ct, v) if v >= 0 else '(%s)(%dLL)' % (ct, v)


def _comb_fns(op, adt):
  """Device helpers: comb(acc, v) and for arg ops better(v, vi, b, bi)."""
  ct = ctype(adt)
  fl = is_float(adt)
  if op == 'sum':
    return 'DEV %s comb(%s x, %s y) { return x + y; }' % (ct, ct, ct)
  if op in ('min', 'max'):
    c = '<' if op == 'min' else '>'
    if fl:
      # NaN-propagating: y wins if it is NaN or strictly better; a NaN x is
      # never displaced by a number (one compare + one select fewer)
      return ('DEV %s comb(%s x, %s y) { return ((y %s x) | (y != y)) ? y : x; }'
              % (ct, ct, ct, c))
    return 'DEV %s comb(%s x, %s y) { return (y %s x) ? y : x; }' % (ct, ct, ct, c)
  c = '<' if op == 'argmin' else '>'
  # better_seq: the in-loop form, for a thread's own elements in increasing
  # index order -- a held NaN is never displaced and a tie only displaces the
  # identity (acci still the sentinel), so no 64-bit index compare
  if fl:
    return ('DEV bool better(%s v, i64 vi, %s b, i64 bi) {\n'
            '  bool vn = v != v, bn = b != b;\n'
            '  if (vn || bn) { if (vn && !bn) return true; if (!vn && bn) return false; return vi < bi; }\n'
            '  if (v == b) return vi < bi;\n'
            '  return v %s b;\n}\n'
            'DEV bool better_seq(%s v, %s b, i64 bi) {\n'
            '  return (b == b) & ((v != v) | (v %s b) | ((v == b) & (bi == 0x7fffffffffffffffLL)));\n}'
            % (ct, ct, c, ct, ct, c))
  return ('DEV bool better(%s v, i64 vi, %s b, i64 bi) { if (v == b) return vi < bi; return v %s b; }\n'
          'DEV bool better_seq(%s v, %s b, i64 bi) { return (v %s b) | ((v == b) & (bi == 0x7fffffffffffffffLL)); }'
          % (ct, ct, c, ct, ct, c))


def _acc_update(op, j, val, idx_expr):
  if op in ('argmin', 'argmax'):
    return ('{ auto v_ = %s; if (better_seq(v_, acc%d, acci%d)) { acc%d = v_; acci%d = %s; } }'
            % (val, j, j, j, j, idx_expr))
  return 'acc%d = comb(acc%d, %s);' % (j, j, val)


def gen_reduce(root, inputs, classes, kind, op, vec, unroll=None, rowinv=(), lpr=None, full=False, interleave=False):
  """Fused map+reduce.  kind 'rows' (reduce over contiguous R of (O, R), one
  or more blocks per segment), 'rowsp' (the same for short R: several
  segments per wave, LPR lanes each, butterfly combine) or 'cols' (reduce over
  R of (O, R, I), I contiguous).

  classes: per-input addressing class of the vectorised dimension (R for rows,
  I for cols): 'c', 'b' or 'g'.

  'cols' only: ``lpr`` fixes the lanes per row group at compile time (else
  the launch's aux[2]); ``full`` (with ``lpr``) promises I == lpr * vec, so
  the vector path needs no column mask.  A fused row dot's per-row lane sum
  then compiles to 4 straight DPP adds: with a run-time LPR every row paid
  6 uniform branches, and the column masks a select per element -- cfg5's
  loop body was 641 instructions per 8 rows, issue-bound beside the loads.
  """
  assert op in REDOPS and kind in ('rows', 'rowsp', 'cols')
  rds = rowdots(root)
  if rds and kind != 'cols':
    raise NotImplementedError('a fused row dot needs the column-reduce skeleton')
  fn, ocml = _expr_fn(root, inputs)
  adt = acc_dtype(op, root.dtype)
  act = ctype(adt)
  arg = op in ('argmin', 'argmax')
  L = [PRELUDE, _ocml_decls(ocml), fn, _comb_fns(op, adt)]
  if rds or kind == 'rows':
    L.append(SHFL)
    L.append(ROW_ALLSUM)

  def val_j(j):
    return '(%s)%s' % (act, _call_expr(inputs, j, n_rd=len(rds)))

  def loads(V, base_expr, vdim):
    b = []
    for (s, dt), cls in zip(inputs, classes):
      b.append('const i64 off%d = %s;' % (s, base_expr(s)))
      if cls == 'g' and V > 1:
        b.append('const i64 s%d_in = a.str[%d][%d];' % (s, s, vdim))
      b += _load_vec(s, dt, cls, 'off%d' % s, V)
    return b

  def to_global():
    # tile-local indices of the per-thread arg accumulators -> global ones
    return ['if (acci%d != 0x7fffffffffffffffLL) acci%d = %s;' % (j, j, gidx('acci%d' % j)) for j in range(vec)]

  def gidx(r_expr):
    # global index of element r along the reduced dim (axis) or flat (axis None)
    return ('(a.aux[5] ? gflat(a, %s) : a.aux[4] + %s)' % (r_expr, r_expr))

  if arg:
    L.append('''DEV i64 gflat(const KArgs& a, i64 r) {
  i64 rem = r, g = 0, mul = 1;
  for (int d = (int)a.aux[6] - 1; d >= 0; --d) {
    i64 q = rem / a.tshape[d]; i64 li = rem - q * a.tshape[d]; rem = q;
    g += (li + a.tul[d]) * mul; mul *= a.ashape[d];
  }
  return g;
}''')

  if kind == 'rows':
    # U steps of the block's row loop per iteration, every load first: with
    # one or two streamed inputs a single vector load per lane cannot keep
    # enough bytes in flight (x.sum(axis=1) at cfg2 size: 4.1 TB/s with U=1).
    # Each accumulator still takes its elements in the same order: results
    # are unchanged.
    U = rows_unroll(inputs, classes)

    def body(V):
      b = []
      b.append('i64 r = r0 + (i64)tid() * %d;' % V)
      if U > 1:
        b.append('for (; r + %d * 256 * %d < r1; r += %d * 256 * %d) {' % (U - 1, V, U, V))
        for u in range(U):
          step = '(r + %d * 256 * %d)' % (u, V)
          lines = loads(V, lambda s: 'o * a.str[%d][0] + %s * a.str[%d][1]' % (s, step, s), 1)
          b += ['  ' + _suffix_names(x, '_u%d' % u) for x in lines]
        for u in range(U):
          for j in range(V):
            call = '(%s)%s' % (act, _call_expr(inputs, j, n_rd=len(rds), sfx='_u%d' % u))
            b.append('  ' + _acc_update(op, j, call, '(r + %d * 256 * %d + %d)' % (u, V, j)))
        b.append('}')
      b.append('for (; r < r1; r += 256 * %d) {' % V)
      b += ['  ' + x for x in loads(V, lambda s: 'o * a.str[%d][0] + r * a.str[%d][1]' % (s, s), 1)]
      for j in range(V):
        b.append('  ' + _acc_update(op, j, val_j(j), '(r + %d)' % j))
      b.append('}')
      return b

    L.append('KERN void spx_reduce(KArgs a) {')
    L.append('  const i64 O = a.dim[0], R = a.dim[1], P = a.aux[0], chunk = a.aux[1];')
    # grid-stride over the O * P segments (the launch may cap the grid)
    L.append('  for (i64 blk = bidx(); blk < O * P; blk += (i64)a.grid) {')
    L.append('  const i64 o = blk / P, p = blk - o * P;')
    L.append('  const i64 r0 = p * chunk; i64 r1 = r0 + chunk; if (r1 > R) r1 = R;')
    for j in range(vec):
      L.append('  %s acc%d = %s;' % (act, j, _ident(op, adt)))
      if arg:
        L.append('  i64 acci%d = 0x7fffffffffffffffLL;' % j)
    L.append('  if (a.flags & 1) {')
    L += ['    ' + x for x in body(vec)]
    L.append('  } else {')
    L += ['    ' + x for x in body(1)]
    L.append('  }')
    # in the loop the indices are tile-local (monotonic in the global index,
    # so first-occurrence ties resolve the same); converted once here
    if arg:
      L += ['  ' + x for x in to_global()]
    # fold the V slots in index order, then block tree
    L.append('  %s accv = acc0;' % act)
    if arg:
      L.append('  i64 acci = acci0;')
    for j in range(1, vec):
      if arg:
        L.append('  if (better(acc%d, acci%d, accv, acci)) { accv = acc%d; acci = acci%d; }' % (j, j, j, j))
      else:
        L.append('  accv = comb(accv, acc%d);' % j)
    # wave level first: DPP within each 16-lane row (quad_perm [1,0,3,2],
    # [2,3,0,1], row_half_mirror, row_mirror -- each lane meets a partner
    # holding its mirror group's partial, and comb / better are symmetric, so
    # every lane ends with the wave's value), ds_bpermute across rows; then
    # the 4 wave results through LDS with one barrier (was an 8-barrier tree)
    L.append('  const u32 t = tid();')
    steps = ['dpp_mov<0xB1>(%s)', 'dpp_mov<0x4E>(%s)', 'dpp_mov<0x141>(%s)', 'dpp_mov<0x140>(%s)',
             'shfl_xor(%s, 16)', 'shfl_xor(%s, 32)']
    for st in steps:
      if arg:
        L.append('  { %s ov = %s; i64 oi = %s;' % (act, st % 'accv', st % 'acci'))
        L.append('    if (better(ov, oi, accv, acci)) { accv = ov; acci = oi; } }')
      else:
        L.append('  accv = comb(accv, %s);' % (st % 'accv'))
    L.append('  SHARED %s sv[4];' % act)
    if arg:
      L.append('  SHARED i64 si[4];')
    L.append('  if ((t & 63) == 0) { sv[t >> 6] = accv;' + (' si[t >> 6] = acci;' if arg else '') + ' }')
    L.append('  bsync();')
    L.append('  if (t == 0) {')
    L.append('    %s v = sv[0];' % act)
    if arg:
      L.append('    i64 vi = si[0];')
    L.append('    for (int k = 1; k < 4; ++k) {')
    if arg:
      L.append('      if (better(sv[k], si[k], v, vi)) { v = sv[k]; vi = si[k]; }')
    else:
      L.append('      v = comb(v, sv[k]);')
    L.append('    }')
    L.append('    ((GLOBAL %s*)a.out0)[p * O + o] = v;' % act)
    if arg:
      L.append('    ((GLOBAL i64*)a.out1)[p * O + o] = vi;')
    L.append('  }')
    L.append('  bsync();  // sv is rewritten by the next segment')
    L.append('  }')
    L.append('}')
  elif kind == 'rowsp':
    def body(V):
      b = []
      b.append('if (o < O) {')
      b.append('  for (i64 r = cl * %d; r < R; r += LPR * %d) {' % (V, V))
      b += ['    ' + x for x in loads(V, lambda s: 'o * a.str[%d][0] + r * a.str[%d][1]' % (s, s), 1)]
      for j in range(V):
        b.append('    ' + _acc_update(op, j, val_j(j), '(r + %d)' % j))
      b.append('  }')
      b.append('}')
      return b

    L.append(SHFL)
    L.append('KERN void spx_reduce(KArgs a) {')
    L.append('  const i64 O = a.dim[0], R = a.dim[1];')
    L.append('  const i64 lpr_log = a.aux[2], LPR = (i64)1 << lpr_log, SPW = 64 >> lpr_log;')
    L.append('  const u32 t = tid(); const i64 lane = t & 63, w = t >> 6;')
    L.append('  const i64 sub = lane >> lpr_log, cl = lane & (LPR - 1);')
    L.append('  const i64 step = (i64)a.grid * 4 * SPW;')
    L.append('  for (i64 sb = (i64)bidx() * 4 * SPW; sb < O; sb += step) {')
    L.append('    const i64 o = sb + w * SPW + sub;')
    for j in range(vec):
      L.append('    %s acc%d = %s;' % (act, j, _ident(op, adt)))
      if arg:
        L.append('    i64 acci%d = 0x7fffffffffffffffLL;' % j)
    L.append('    if (a.flags & 1) {')
    L += ['      ' + x for x in body(vec)]
    L.append('    } else {')
    L += ['      ' + x for x in body(1)]
    L.append('    }')
    if arg:
      L += ['    ' + x for x in to_global()]
    L.append('    %s accv = acc0;' % act)
    if arg:
      L.append('    i64 acci = acci0;')
    for j in range(1, vec):
      if arg:
        L.append('    if (better(acc%d, acci%d, accv, acci)) { accv = acc%d; acci = acci%d; }' % (j, j, j, j))
      else:
        L.append('    accv = comb(accv, acc%d);' % j)
    L.append('    for (i64 m = 1; m < LPR; m <<= 1) {')
    L.append('      %s ov = shfl_xor(accv, (int)m);' % act)
    if arg:
      L.append('      i64 oi = shfl_xor(acci, (int)m);')
      L.append('      if (better(ov, oi, accv, acci)) { accv = ov; acci = oi; }')
    else:
      L.append('      accv = (cl & m) ? comb(ov, accv) : comb(accv, ov);')
    L.append('    }')
    L.append('    if (cl == 0 && o < O) {')
    L.append('      ((GLOBAL %s*)a.out0)[o] = accv;' % act)
    if arg:
      L.append('      ((GLOBAL i64*)a.out1)[o] = acci;')
    L.append('    }')
    L.append('  }')
    L.append('}')
  else:
    U = unroll or cols_unroll(inputs, classes, vec)
    lv = interleave and op == 'sum'
    pact = ctype(partial_dtype(op, adt, interleave))
    kahan = lv and pact == 'double' and act == 'double'

    def one_row(V, rv, sfx, masked, bcu=None):
      """Loads + (row dots) + accumulator updates of row ``rv`` into names
      suffixed ``sfx``; split in (load lines, compute lines) so an unrolled
      body issues every row's loads before the first use.  ``bcu``: this
      row's index u in an unrolled step whose per-row ('b') inputs were loaded
      once, row u by lane u of the 16-lane group (``yb<s>``): the value comes
      by DPP row_newbcast:u instead of a load per row."""
      ld, cp = [], []
      base = lambda s, c: 'o * a.str[%d][0] + %s * a.str[%d][1] + %s * a.str[%d][2]' % (s, rv, s, c, s)
      for (s, dt), cls in zip(inputs, classes):
        ct = ctype(dt)
        names = ['x%d_%d%s' % (s, j, sfx) for j in range(V)]
        if s in rowinv:
          ld += ['%s %s = x%d_%d_ri;' % (ct, n, s, j) for j, n in enumerate(names)]
          continue
        if bcu is not None and s in bcast:
          # (with the compute lines: the broadcast waits for the one load,
          # which must not hold back the rows' loads)
          v = 'dpp_mov<%d>(yb%d)' % (0x150 + bcu, s)
          cp.append('const %s xbb%d%s = %s;' % (ct, s, sfx, v))
          cp += ['%s %s = %s;' % (ct, n, ('colok ? xbb%d%s : (%s)0' % (s, sfx, ct)) if masked else 'xbb%d%s' % (s, sfx))
                 for n in names]
          continue
        srcs, pre = load_srcs(s, dt, cls, V, base(s, 'cc' if masked else 'col'))
        ld.append('%s %s;' % (ct, ' '.join(names).replace(' ', ', ')))
        ld.append('{')
        ld += ['  ' + x for x in pre]
        # masked lanes load column 0 (always in bounds) and select zero at use
        ld += ['  %s = %s;' % (n, ('colok ? %s : (%s)0' % (v, ct)) if masked else v) for n, v in zip(names, srcs)]
        ld.append('}')
      for rd in rds:
        ct = ctype(rd.dtype)
        n = 'rd%d%s' % (rd.rid, sfx)
        cp.append('%s %s = (%s)0;' % (ct, n, ct))
        for j in range(V):
          cp.append('%s = %s + (%s)x%d_%d%s * (%s)x%d_%d%s;' % (n, n, ct, rd.a.slot, j, sfx, ct, rd.w.slot, j, sfx))
        cp.append('%s = row_allsum(%s, LPR);' % (n, n))
      upd = []
      for j in range(V):
        call = '(%s)%s' % (act, _call_expr(inputs, j, n_rd=len(rds), sfx=sfx))
        upd.append(_acc_update(op, j, call, '(%s)' % rv))
      if masked:
        cp.append('if (colok) {')
        cp += ['  ' + x for x in upd]
        cp.append('}')
      else:
        cp += upd
      return ld, cp

    def load_srcs(s, dt, cls, V, off):
      """(per-element source expressions, preamble lines) of one vector load."""
      ct = ctype(dt)
      p = '((const GLOBAL %s*)a.ptr[%d])' % (ct, s)
      pre = ['const i64 off = %s;' % off]
      if V > 1 and cls == 'c':
        pre.append('typedef %s __attribute__((ext_vector_type(%d))) vt;' % (ct, V))
        pre.append('const vt xv = %s;' % _vload('vt', '%s + off' % p))
        return ['xv[%d]' % j for j in range(V)], pre
      if V > 1 and cls == 'b':
        pre.append('const %s xb = %s[off];' % (ct, p))
        return ['xb'] * V, pre
      if V > 1:
        pre.append('const i64 s_in = a.str[%d][2];' % s)
        return ['%s[off + %d * s_in]' % (p, j) for j in range(V)], pre
      return ['%s[off]' % p], pre

    # per-row inputs of a row-dot kernel with 16-lane row groups: one load per
    # unrolled step (lane u of the group fetches row u), DPP broadcasts --
    # for 4- and 8-byte values only (dpp_mov moves one or two dwords; a bool,
    # int8 or fp16 row input keeps its per-row load)
    bcast = ()
    if rds and lpr == 16 and U > 1 and U <= 16:
      bcast = tuple(s for (s, dt), cls in zip(inputs, classes)
                    if cls == 'b' and s not in rowinv and np.dtype(dt).itemsize in (4, 8))

    def body(V):
      masked = bool(rds)
      b = []
      # row-dot kernels: every lane of a row group takes part in the DPP row
      # sum, so lanes past the last column read column 0 and use zeros
      b.append('{' if masked else 'if (col < I) {')
      b.append('  const bool colok = %s; (void)colok;' % ('true' if (full and lpr and V == vec) else 'col < I'))
      b.append('  const i64 cc = colok ? col : 0; (void)cc;')
      for (s, dt), cls in zip(inputs, classes):
        if s in rowinv:  # row stride 0: loaded once, outside the row loop
          ct = ctype(dt)
          srcs, pre = load_srcs(s, dt, cls, V, 'o * a.str[%d][0] + %s * a.str[%d][2]'
                                % (s, 'cc' if masked else 'col', s))
          b.append('  %s %s;' % (ct, ', '.join('x%d_%d_ri' % (s, j) for j in range(V))))
          b.append('  {')
          b += ['    ' + x for x in pre]
          b += ['    x%d_%d_ri = %s;' % (s, j, (('colok ? %s : (%s)0' % (v, ct)) if masked else v))
                for j, v in enumerate(srcs)]
          b.append('  }')
      b.append('  const i64 STEP = 4 * RPW;')
      if interleave:
        # block p takes the U-step super-chunks p, p + P, p + 2P, ...: at any
        # moment the grid streams one contiguous stretch of X instead of P
        # streams far apart (one chunk per block).  A block then covers R / P
        # rows, so (sums) each super-chunk's U rows go into a fresh
        # accumulator (in the input's precision: U additions) that is folded
        # into a middle one, and every 32 chunks the middle one into the
        # block's total.  Middle and total are fp64 (round 6; fp32 inputs:
        # only the U-row chunk sums round to fp32, everything above them --
        # lane total, LDS combine, partials, finalize -- is fp64), and for
        # fp64 inputs the total is Kahan-compensated (topc)
        if lv:
          b.append('  %s %s;' % (pact, ', '.join('mid%d = 0.0, top%d = 0.0' % (j, j) for j in range(V))))
          if kahan:
            b.append('  double %s;' % ', '.join('topc%d = 0.0' % j for j in range(V)))
          b.append('  int nsc = 0;')
        b.append('  for (i64 sb = p * (%d * STEP); sb < R; sb += P * (%d * STEP)) {' % (U, U))
        b.append('  const i64 r0 = sb; i64 r1 = sb + %d * STEP; if (r1 > R) r1 = R;' % U)
      b.append('  i64 r = r0 + w * RPW + sub;')
      if U > 1:
        b.append('  for (; r + %d * STEP < r1; r += %d * STEP) {' % (U - 1, U))
        lds, cps = [], []
        for s_ in bcast:
          ct = ctype(dict(inputs)[s_])
          b.append('    %s yb%d;' % (ct, s_))
          b.append('    { const i64 rb = r + (cl < %d ? cl : 0) * STEP;' % U)
          b.append('      yb%d = ((const GLOBAL %s*)a.ptr[%d])[o * a.str[%d][0] + rb * a.str[%d][1]]; }'
                   % (s_, ct, s_, s_, s_))
        for u in range(U):
          b.append('    const i64 r_%d = r + %d * STEP;' % (u, u))
          ld, cp = one_row(V, 'r_%d' % u, '_u%d' % u, masked, u if bcast else None)
          lds += ld
          cps += cp
        b += ['    ' + x for x in lds + cps]
        b.append('  }')
      b.append('  for (; r < r1; r += STEP) {')
      ld, cp = one_row(V, 'r', '', masked)
      b += ['    ' + x for x in ld + cp]
      b.append('  }')
      if interleave:
        if lv:
          for j in range(V):
            b.append('  mid%d = mid%d + (%s)acc%d; acc%d = (%s)0;' % (j, j, pact, j, j, act))
          b.append('  if (++nsc == 32) {')
          for j in range(V):
            if kahan:
              b.append('    { const double y_ = mid%d - topc%d, t_ = top%d + y_; topc%d = (t_ - top%d) - y_; '
                       'top%d = t_; } mid%d = 0.0;' % (j, j, j, j, j, j, j))
            else:
              b.append('    top%d = top%d + mid%d; mid%d = 0.0;' % (j, j, j, j))
          b.append('    nsc = 0;')
          b.append('  }')
        b.append('  }')
        if lv:
          for j in range(V):
            if kahan:
              b.append('  fin%d = top%d + (mid%d - topc%d);' % (j, j, j, j))
            else:
              b.append('  fin%d = top%d + mid%d;' % (j, j, j))
      b.append('}')
      return b

    L.append('KERN void spx_reduce(KArgs a) {')
    L.append('  const i64 O = a.dim[0], R = a.dim[1], I = a.dim[2];')
    if lpr:
      assert lpr & (lpr - 1) == 0 and 1 <= lpr <= 64
      L.append('  const i64 P = a.aux[0], chunk = a.aux[1], CT = a.aux[3];')
      L.append('  constexpr i64 lpr_log = %d, LPR = %d, RPW = %d;' % (lpr.bit_length() - 1, lpr, 64 // lpr))
    else:
      L.append('  const i64 P = a.aux[0], chunk = a.aux[1], lpr_log = a.aux[2], CT = a.aux[3];')
      L.append('  const i64 LPR = (i64)1 << lpr_log, RPW = 64 >> lpr_log;')
    L.append('  const i64 blk = bidx(); const i64 ct = blk % CT; const i64 rest = blk / CT;')
    L.append('  const i64 o = rest % O, p = rest / O;')
    L.append('  const u32 t = tid(); const i64 lane = t & 63, w = t >> 6;')
    L.append('  const i64 sub = lane >> lpr_log, cl = lane & (LPR - 1);')
    L.append('  const i64 V = (a.flags & 1) ? %d : 1;' % vec)
    L.append('  const i64 col = ct * (LPR * V) + cl * V;')
    L.append('  const i64 r0 = p * chunk; i64 r1 = r0 + chunk; if (r1 > R) r1 = R;')
    for j in range(vec):
      L.append('  %s acc%d = %s;' % (act, j, _ident(op, adt)))
      if arg:
        L.append('  i64 acci%d = 0x7fffffffffffffffLL;' % j)
      if lv:
        L.append('  %s fin%d = 0.0;' % (pact, j))
    L.append('  if (a.flags & 1) {')
    L += ['    ' + x for x in body(vec)]
    L.append('  } else {')
    L += ['    ' + x for x in body(1)]
    L.append('  }')
    if arg:
      L += ['  ' + x for x in to_global()]
    # LDS combine over the 4*RPW row groups sharing a column, in row-group
    # order (in the partials' type: fp64 for an interleaved fp32 sum)
    L.append('  SHARED %s sv[256 * %d];' % (pact, vec))
    if arg:
      L.append('  SHARED i64 si[256 * %d];' % vec)
    L.append('  const i64 grp = w * RPW + sub;')
    L.append('  const i64 W = LPR * V;')
    for j in range(vec):
      L.append('  if (%d < V) { sv[grp * W + cl * V + %d] = %s%d;%s }'
               % (j, j, 'fin' if lv else 'acc', j, (' si[grp * W + cl * V + %d] = acci%d;' % (j, j)) if arg else ''))
    L.append('  bsync();')
    L.append('  if ((i64)t < W) {')
    L.append('    %s b = sv[t];' % pact)
    if arg:
      L.append('    i64 bi = si[t];')
    L.append('    for (i64 g = 1; g < 4 * RPW; ++g) {')
    if arg:
      L.append('      if (better(sv[g * W + t], si[g * W + t], b, bi)) { b = sv[g * W + t]; bi = si[g * W + t]; }')
    elif lv:
      L.append('      b = b + sv[g * W + t];')
    else:
      L.append('      b = comb(b, sv[g * W + t]);')
    L.append('    }')
    L.append('    const i64 gc = ct * W + t;')
    L.append('    if (gc < I) {')
    L.append('      ((GLOBAL %s*)a.out0)[(p * O + o) * I + gc] = b;' % pact)
    if arg:
      L.append('      ((GLOBAL i64*)a.out1)[(p * O + o) * I + gc] = bi;')
    L.append('    }')
    L.append('  }')
    L.append('}')
  return '\n'.join(L)


SHFL = r'''
DEV u32 shfl_u32(u32 v, int m) {
  const int lane = (int)(tid() & 63);
  return (u32)__builtin_amdgcn_ds_bpermute((lane ^ m) << 2, (int)v);
}
template <typename T> DEV T shfl_xor(T v, int m) {
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "shfl size");
  if constexpr (sizeof(T) == 4) {
    u32 u = __builtin_bit_cast(u32, v);
    return __builtin_bit_cast(T, shfl_u32(u, m));
  } else {
    u64 u = __builtin_bit_cast(u64, v);
    u32 lo = shfl_u32((u32)u, m), hi = shfl_u32((u32)(u >> 32), m);
    return __builtin_bit_cast(T, ((u64)hi << 32) | lo);
  }
}
'''


ROW_ALLSUM = r'''
// Sum over aligned groups of LPR lanes (LPR a power of two <= 64), result in
// every lane of the group.  Within a 16-lane DPP row: quad_perm [1,0,3,2],
// quad_perm [2,3,0,1], row_half_mirror, row_mirror (each step adds a partner
// holding the mirror-group's equal partial, so all lanes of a group end with
// the bit-identical sum); across rows: ds_bpermute xor 16 / 32.
template <int CTRL> DEV u32 dpp_u32(u32 v) {
  return (u32)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL, typename T> DEV T dpp_mov(T v) {
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, dpp_u32<CTRL>(__builtin_bit_cast(u32, v)));
  } else {
    u64 u = __builtin_bit_cast(u64, v);
    u32 lo = dpp_u32<CTRL>((u32)u), hi = dpp_u32<CTRL>((u32)(u >> 32));
    return __builtin_bit_cast(T, ((u64)hi << 32) | lo);
  }
}
template <typename T> DEV T row_allsum(T v, i64 LPR) {
  if (LPR > 1) v = v + dpp_mov<0xB1>(v);
  if (LPR > 2) v = v + dpp_mov<0x4E>(v);
  if (LPR > 4) v = v + dpp_mov<0x141>(v);
  if (LPR > 8) v = v + dpp_mov<0x140>(v);
  if (LPR > 16) v = v + shfl_xor(v, 16);
  if (LPR > 32) v = v + shfl_xor(v, 32);
  return v;
}
'''


def vec_width(dtypes):
  m = max(np.dtype(d).itemsize for d in dtypes)
  return max(1, 16 // m)
