"""Kernel backend: libspx.so (C ABI, include/spx.h) + generated-kernel JIT.

This is the only module that touches the GPU compute path.  It loads the
in-tree ``libspx.so`` (built by ``__graft_entry__.build()`` with hipcc for
gfx950) and fails loudly if it is missing -- there is no CPU fallback.  Tests
may install a different backend object with ``set_backend`` to exercise the
host logic without a GPU; product code never does.

Tensors are PyTorch-ROCm device tensors (allocation and streams only); every
call passes raw pointers and the current HIP stream to the C ABI.
"""
import ctypes
import hashlib
import os
import subprocess
import tempfile
import threading

import numpy as np

from . import codegen
from .config import FLAGS
from .layout import broadcast_strides, coalesce, reduce_view, contiguous_strides
from .util import prod

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, 'libspx.so')
SRC_PATH = os.path.join(_HERE, 'csrc', 'spx.hip')

SPX_BOOL, SPX_I32, SPX_I64, SPX_F32, SPX_F64 = 0, 1, 2, 3, 4
OP_CODE = {'sum': 0, 'min': 1, 'max': 2, 'argmin': 3, 'argmax': 4, 'replace': 5}
FILL_CONST, FILL_ARANGE, FILL_UNIFORM, FILL_NORMAL = 0, 1, 2, 3

_DT = {np.dtype(np.bool_): SPX_BOOL, np.dtype(np.int32): SPX_I32, np.dtype(np.int64): SPX_I64,
       np.dtype(np.float32): SPX_F32, np.dtype(np.float64): SPX_F64}


def spx_dtype(dt):
  dt = np.dtype(dt)
  if dt not in _DT:
    raise TypeError('dtype %s is not supported by the MI355X backend '
                    '(bool, int32, int64, float32, float64)' % dt)
  return _DT[dt]


def torch_dtype(dt):
  import torch
  return {np.dtype(np.bool_): torch.bool, np.dtype(np.int32): torch.int32,
          np.dtype(np.int64): torch.int64, np.dtype(np.float32): torch.float32,
          np.dtype(np.float64): torch.float64}[np.dtype(dt)]


def np_dtype(tdt):
  import torch
  return {torch.bool: np.dtype(np.bool_), torch.int32: np.dtype(np.int32),
          torch.int64: np.dtype(np.int64), torch.float32: np.dtype(np.float32),
          torch.float64: np.dtype(np.float64)}[tdt]


# ------------------------------------------------------------------ library
_lib = None
_lib_lock = threading.Lock()

_I64P = ctypes.POINTER(ctypes.c_int64)
_SIGS = {
    'spx_abi_version': ([], ctypes.c_int),
    'spx_last_error': ([], ctypes.c_char_p),
    'spx_module_load': ([ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
    'spx_module_unload': ([ctypes.c_void_p], ctypes.c_int),
    'spx_module_function': ([ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
    'spx_launch': ([ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                    ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p], ctypes.c_int),
    'spx_fill': ([ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, _I64P, _I64P, _I64P,
                  ctypes.c_double, ctypes.c_double, ctypes.c_uint64, ctypes.c_void_p], ctypes.c_int),
    'spx_reduce_finalize': ([ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_void_p], ctypes.c_int),
    'spx_merge': ([ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, _I64P, _I64P,
                   _I64P, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p], ctypes.c_int),
    'spx_copy_region': ([ctypes.c_int, ctypes.c_void_p, _I64P, _I64P, ctypes.c_int, ctypes.c_void_p, _I64P,
                         _I64P, ctypes.c_int, _I64P, ctypes.c_void_p], ctypes.c_int),
    'spx_gemm': ([ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                  ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                  ctypes.c_double, ctypes.c_double, ctypes.c_void_p], ctypes.c_int),
    'spx_argreduce_combine': ([ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                               ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    'spx_kmeans_assign_workspace': ([ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64],
                                     ctypes.c_int64),
    'spx_kmeans_assign': ([ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                           ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p], ctypes.c_int),
    'spx_kmeans_accumulate_workspace': ([ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64],
                                         ctypes.c_int64),
    'spx_kmeans_accumulate': ([ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                               ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                               ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p], ctypes.c_int),
    'spx_kmeans_step_workspace': ([ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64], ctypes.c_int64),
    'spx_kmeans_step': ([ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                         ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                         ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p], ctypes.c_int),
    'spx_kmeans_timing': ([ctypes.c_int], ctypes.c_int),
    'spx_kmeans_times': ([ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double), ctypes.c_int],
                         ctypes.c_int),
    'spx_cdist': ([ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                   ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p], ctypes.c_int),
    'spx_bincount': ([ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int,
                      ctypes.c_void_p], ctypes.c_int),
    'spx_comm_load': ([ctypes.c_char_p], ctypes.c_int),
    'spx_comm_unique_id': ([ctypes.c_void_p, ctypes.c_int64], ctypes.c_int),
    'spx_comm_init': ([ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)],
                      ctypes.c_int),
    'spx_comm_destroy': ([ctypes.c_void_p], ctypes.c_int),
    'spx_allreduce': ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                       ctypes.c_void_p], ctypes.c_int),
    'spx_reduce_scatter': ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                            ctypes.c_int, ctypes.c_void_p], ctypes.c_int),
    'spx_allgather': ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                       ctypes.c_void_p], ctypes.c_int),
    'spx_broadcast': ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                       ctypes.c_void_p], ctypes.c_int),
    'spx_reduce': ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                    ctypes.c_int, ctypes.c_void_p], ctypes.c_int),
    'spx_sendrecv': ([ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), _I64P,
                      ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), _I64P,
                      ctypes.POINTER(ctypes.c_int), ctypes.c_void_p], ctypes.c_int),
    'spx_mincost_tiling': ([ctypes.c_int32, ctypes.c_int64, ctypes.POINTER(ctypes.c_int32),
                            ctypes.POINTER(ctypes.c_int32), _I64P, ctypes.c_int64, ctypes.POINTER(ctypes.c_int32),
                            ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_uint8), _I64P], ctypes.c_int),
}
EXPORTED = tuple(_SIGS)


def load_library(path=LIB_PATH):
  """Load libspx.so (importing torch first so its HIP runtime is the one used)."""
  global _lib
  with _lib_lock:
    if _lib is not None:
      return _lib
    import torch  # noqa: F401  (torch's libamdhip64.so.7 must be the loaded runtime)
    if not os.path.exists(path):
      raise RuntimeError('libspx.so not found at %s: run __graft_entry__.build() '
                         '(hipcc --offload-arch=gfx950); there is no CPU fallback' % path)
    lib = ctypes.CDLL(path)
    for name, (args, res) in _SIGS.items():
      fn = getattr(lib, name)
      fn.argtypes = args
      fn.restype = res
    _lib = lib
    return lib


def mincost_tiling(t, edges, split_pairs):
  """spx_mincost_tiling (host code in libspx.so, no GPU needed): the node
  choice of the AutomaticTiling cost graph.  edges: [(u, v, cost)] in
  insertion order; split_pairs: [(a, b)].  Returns (chosen node ids < t,
  total cost)."""
  lib = load_library()
  n = len(edges)
  I32 = ctypes.c_int32
  eu = (I32 * max(n, 1))(*[int(e[0]) for e in edges])
  ev = (I32 * max(n, 1))(*[int(e[1]) for e in edges])
  ec = (ctypes.c_int64 * max(n, 1))(*[int(e[2]) for e in edges])
  m = len(split_pairs)
  su = (I32 * max(m, 1))(*[int(p[0]) for p in split_pairs])
  sv = (I32 * max(m, 1))(*[int(p[1]) for p in split_pairs])
  chosen = (ctypes.c_uint8 * max(int(t), 1))()
  total = ctypes.c_int64(0)
  rc = lib.spx_mincost_tiling(int(t), n, eu, ev, ec, m, su, sv, chosen, ctypes.byref(total))
  if rc != 0:
    raise ValueError('spx_mincost_tiling: malformed tiling graph')
  return [u for u in range(int(t)) if chosen[u]], int(total.value)


def _arr(vals):
  vals = [int(v) for v in vals] or [0]
  return (ctypes.c_int64 * len(vals))(*vals)


def _check(rc, what):
  if rc != 0:
    raise RuntimeError('%s failed (%d): %s' % (what, rc, _lib.spx_last_error().decode()))


# ------------------------------------------------------------ JIT compile
def clang_path():
  rocm = os.environ.get('ROCM_PATH', '/opt/rocm')
  p = os.path.join(rocm, 'lib', 'llvm', 'bin', 'clang++')
  if not os.path.exists(p):
    raise RuntimeError('device compiler %s not found' % p)
  return p


COMPILE_FLAGS = ['-x', 'hip', '--offload-arch=gfx950', '--cuda-device-only', '--no-gpu-bundle-output',
                 '-nogpuinc', '-O3', '-ffp-contract=off', '-std=c++17']


def cache_dir():
  d = FLAGS.kernel_cache_dir or os.path.join(_HERE, '_kcache')
  try:
    os.makedirs(d, exist_ok=True)
    if os.access(d, os.W_OK):
      return d
  except OSError:
    pass
  d = os.path.join(tempfile.gettempdir(), 'spartan_amd_kcache')
  os.makedirs(d, exist_ok=True)
  return d


def source_key(src):
  h = hashlib.sha1()
  h.update(' '.join(COMPILE_FLAGS).encode())
  h.update(src.encode())
  return h.hexdigest()[:24]


def compile_code_object(src):
  """Compile generated HIP source to a gfx950 code object (cached on disk)."""
  key = source_key(src)
  d = cache_dir()
  path = os.path.join(d, key + '.hsaco')
  if os.path.exists(path):
    with open(path, 'rb') as f:
      return f.read()
  # also look in the in-tree cache when an override dir is used
  intree = os.path.join(_HERE, '_kcache', key + '.hsaco')
  if os.path.exists(intree):
    with open(intree, 'rb') as f:
      return f.read()
  with tempfile.TemporaryDirectory() as td:
    sp = os.path.join(td, 'k.hip')
    op = os.path.join(td, 'k.hsaco')
    with open(sp, 'w') as f:
      f.write(src)
    r = subprocess.run([clang_path()] + COMPILE_FLAGS + ['-o', op, sp], capture_output=True, text=True)
    if r.returncode != 0:
      raise RuntimeError('gfx950 codegen compile failed:\n%s\n--- source ---\n%s' % (r.stderr, src))
    with open(op, 'rb') as f:
      img = f.read()
  tmp = path + '.%d.tmp' % os.getpid()
  with open(tmp, 'wb') as f:
    f.write(img)
  os.replace(tmp, path)
  return img


_NCU = []
MAP_UNROLL = 1  # vectors per lane of a dense map (grid = n / (256 V MAP_UNROLL))
NT_STORE_BYTES = 64 << 20  # map outputs at least this large: non-temporal stores
ROWS_GRID_PER_CU = 2  # rows reductions: 1.824 ms vs 1.836 uncapped at cfg2 axis 1 (profiles/r02_cfg2_grid.txt)
# fused row-dot column reductions (cfg5's gradient): blocks per CU, rows
# unrolled per lane group, and the row order.  Round 5: the blocks take
# interleaved super-chunks of U x 16 rows (block p: chunks p, p + P, ...;
# codegen.gen_reduce interleave) instead of one contiguous chunk each, so the
# grid streams one stretch of X at a time -- and then ONE block per CU is
# best: 3.600 ms per lreg iteration against 3.811 for the round-4 form (16
# contiguous chunks per CU, U 8) on one box; interleaved with 2 / 4 / 8 / 16
# blocks per CU 3.69-3.88, U 4 / 6 / 10 / 12 at one block 5.11 / 3.97 / 3.62
# / 3.71 (tools/lreg_il.py, profiles/r05_lreg_interleave.txt)
ROWDOT_BLOCKS_PER_CU = 1
ROWDOT_UNROLL = 8
ROWDOT_INTERLEAVE = True
# wide column sums (several column tiles: cfg2 axis 0): resident blocks per
# CU and whether their row segments are interleaved super-chunks.  The lreg
# kernel's interleaving does NOT carry over: cfg2 axis 0 ran 1.80 ms
# contiguous at 2 blocks per CU against 1.95-2.00 interleaved at 2 / 4 and
# 2.8-3.1 at one block (tools/cfg2_il.py, profiles/r05_cfg2_interleave.txt)
COLS_BLOCKS_PER_CU = 2
COLS_INTERLEAVE = False


def _num_cus():
  if not _NCU:
    import torch
    _NCU.append(torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count)
  return _NCU[0]


class HipBackend:
  """Launches libspx.so / generated kernels on the current HIP stream."""
  name = 'hip'

  def __init__(self):
    self.lib = load_library()
    self._fns = {}
    self._modules = []
    self._lock = threading.Lock()
    self.launch_log = None   # optional list collecting grids (tests)
    self.kernel_events = None  # optional list of (name, start, end) HIP events (bench)
    self._names = {}
    self._sig_fns = {}
    self._reduce_plans = {}  # backend.reduce launch plans (see reduce)

  # ---------------------------------------------------------------- utils
  def stream(self):
    # the raw pointer of the current stream, without building a torch Stream
    # object (torch.cuda.current_stream() cost ~10 us per call, three calls
    # per lreg iteration)
    import torch
    return ctypes.c_void_p(torch._C._cuda_getCurrentRawStream(torch.cuda.current_device()))

  def kernel(self, src, name):
    key = source_key(src)
    with self._lock:
      fn = self._fns.get(key)
      if fn is not None:
        return fn
      img = compile_code_object(src)
      mod = ctypes.c_void_p()
      _check(self.lib.spx_module_load(img, len(img), ctypes.byref(mod)), 'spx_module_load')
      self._modules.append(mod)
      f = ctypes.c_void_p()
      _check(self.lib.spx_module_function(mod, name.encode(), ctypes.byref(f)), 'spx_module_function')
      self._fns[key] = f
      self._names[f.value] = name
      return f

  def _aot_events(self, name):
    """(start, end) HIP events around one ahead-of-time libspx call on the
    current stream when bench timing is on (kernel_events), else None."""
    if self.kernel_events is None:
      return None
    import torch
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    ev[0].record()
    self.kernel_events.append((name, ev[0], ev[1]))
    return ev

  def kmeans_timing(self, enable):
    """Record HIP events around the one-pass kernel of every later fused
    spx_kmeans_step (bench.py's k-means kernel roofline)."""
    _check(self.lib.spx_kmeans_timing(1 if enable else 0), 'spx_kmeans_timing')

  def kmeans_times(self, max_calls=256):
    """[(fused kernel ms, whole step ms)] of the steps recorded since
    kmeans_timing(True) or the last call (waits for them)."""
    a = (ctypes.c_double * max_calls)()
    b = (ctypes.c_double * max_calls)()
    n = self.lib.spx_kmeans_times(a, b, max_calls)
    if n < 0:
      _check(n, 'spx_kmeans_times')
    return [(a[i], b[i]) for i in range(n)]

  def launch(self, fn, grid, args):
    if self.launch_log is not None:
      self.launch_log.append(grid)
    args.grid = grid
    ev = None
    if self.kernel_events is not None:
      import torch
      ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
      ev[0].record()
    _check(self.lib.spx_launch(fn, grid, 1, 1, 256, 0, ctypes.byref(args), ctypes.sizeof(args),
                               self.stream()), 'spx_launch')
    if ev is not None:
      ev[1].record()
      self.kernel_events.append((self._names.get(fn.value, '?'), ev[0], ev[1]))

  # ---------------------------------------------------------------- fills
  def fill(self, out, kind, a, b, seed, ul, array_shape):
    shape = tuple(out.shape)
    nd = len(shape)
    _check(self.lib.spx_fill(spx_dtype(np_dtype(out.dtype)), kind, ctypes.c_void_p(out.data_ptr()), nd,
                             _arr(shape), _arr(ul), _arr(array_shape), float(a), float(b),
                             int(seed) & 0xFFFFFFFFFFFFFFFF, self.stream()), 'spx_fill')

  # ------------------------------------------------------------------ map
  def map(self, root, inputs, out):
    """out[...] = root(inputs) elementwise.  inputs: {slot: tensor} (contiguous,
    broadcastable to out.shape); scalar slots come from the IR's Sc leaves."""
    shape = tuple(out.shape)
    n = prod(shape)
    if n == 0:
      return
    slots = sorted(inputs)
    ins = [(s, np_dtype(inputs[s].dtype)) for s in slots]
    strides = [broadcast_strides(tuple(inputs[s].shape), shape, inputs[s].stride()) for s in slots]
    dense = all(tuple(inputs[s].shape) == shape and inputs[s].is_contiguous() for s in slots)
    V = codegen.vec_width([dt for _, dt in ins] + [root.dtype])
    args = codegen.KArgs()
    _scalars_into(root, args)
    for s in slots:
      args.ptr[s] = inputs[s].data_ptr()
    args.out0 = out.data_ptr()
    args.n = n
    if dense:
      classes = ['c'] * len(slots)
      ndim = 1
      vec_ok = (n % V == 0) and all(inputs[s].data_ptr() % 16 == 0 for s in slots) and out.data_ptr() % 16 == 0
    else:
      cshape, cstr = coalesce(shape, strides)
      ndim = len(cshape)
      if ndim > codegen.MAX_DIM:
        raise NotImplementedError('map over %d non-coalescible dims' % ndim)
      for d in range(ndim):
        args.dim[d] = cshape[d]
      for k, s in enumerate(slots):
        for d in range(ndim):
          args.str[s][d] = cstr[k][d]
      classes = [_cls(cstr[k][ndim - 1]) for k in range(len(slots))]
      vec_ok = (cshape[-1] % V == 0) and out.data_ptr() % 16 == 0 and all(
          _vec_aligned(inputs[s], cstr[k], classes[k], V) for k, s in enumerate(slots))
    args.flags = 1 if (vec_ok and V > 1) else 0
    # streamed outputs: non-temporal stores (x*y+exp(z) map at 2^30 fp32:
    # 2.75 -> 2.57 ms, profiles/r02_stream_ceiling_maps.txt)
    nt = n * out.element_size() >= NT_STORE_BYTES
    mu = MAP_UNROLL if (dense and args.flags & 1) else 1
    sig = ('map', root.sig(), tuple(ins), tuple(classes), ndim, V, dense, nt, mu)
    fn = self._sig_fns.get(sig)
    if fn is None:
      src, kname = codegen.named(codegen.gen_map(root, ins, classes, ndim, V, dense, nt, mu), 'spx_map',
                                 'dense' if dense else 'nd')
      fn = self._sig_fns[sig] = self.kernel(src, kname)
    per = V if args.flags & 1 else 1
    # MAP_UNROLL vectors per lane and no grid-stride loop: x + 1 / x * y at
    # 2^30 fp32 1.75 / 2.58 ms with a 4096-block grid-stride loop, 1.34 / 2.01
    # ms with the full grid (6.4 TB/s read+write; profiles/r02_map_grid.txt)
    grid = max(1, -(-n // (256 * per * mu)))
    self.launch(fn, grid, args)

  # --------------------------------------------------------------- reduce
  def reduce(self, root, op, inputs, in_shape, axis, out_shape, out_dtype, idx_geom=None):
    """Fused map+reduce over one tile -> the tile's partial, a device tensor of
    out_shape and out_dtype; for argmin/argmax a (values, int64 indices) pair."""
    import torch
    slots = sorted(inputs)
    # launch plan of an identical call (same IR signature, operand layouts and
    # shapes: an iterative driver's replayed DAG): everything below up to the
    # kernel arguments is a function of this key
    # (the pointer's residue mod 16, not just 16-byte alignment: the vector
    # width of narrow types needs only 8 or 4 bytes, so two pointers with the
    # same 16-alignment verdict can still differ in what V they allow)
    pkey = (root.sig(), op, tuple((s, inputs[s].dtype, tuple(inputs[s].shape), inputs[s].stride(),
                                   inputs[s].data_ptr() % 16) for s in slots),
            tuple(in_shape), axis, tuple(out_shape), np.dtype(out_dtype).str,
            None if idx_geom is None else repr(sorted(idx_geom.items())),
            # the module's grid / layout knobs shape the plan too
            (ROWS_GRID_PER_CU, COLS_BLOCKS_PER_CU, COLS_INTERLEAVE, ROWDOT_BLOCKS_PER_CU, ROWDOT_UNROLL,
             ROWDOT_INTERLEAVE))
    plan = self._reduce_plans.get(pkey)
    if plan is not None:
      return self._replay_reduce(plan, root, inputs, slots, out_shape, out_dtype)
    ins = [(s, np_dtype(inputs[s].dtype)) for s in slots]
    strides = [broadcast_strides(tuple(inputs[s].shape), in_shape, inputs[s].stride()) for s in slots]
    view = reduce_view(in_shape, strides, axis)
    if view is None and any(not inputs[s].is_contiguous() for s in slots):
      # a strided view whose dims do not collapse to (O, R, I): make the
      # views dense (identity-map kernel) and take the plain path
      inputs = {s: self.contiguous(t) for s, t in inputs.items()}
      strides = [broadcast_strides(tuple(inputs[s].shape), in_shape) for s in slots]
      view = reduce_view(in_shape, strides, axis)
    if view is None:
      # inputs broadcast along different dims of an N-d iteration space (e.g.
      # (N, 1, D) - (1, K, D) reduced over the last axis): the rows of the
      # (O, R, I) form have no single stride.  Materialise the mapped values
      # with the N-d map kernel, then reduce that dense array -- in slabs of a
      # kept dim when the whole iteration space exceeds MATERIALISE_LIMIT bytes.
      if codegen.rowdots(root):
        raise NotImplementedError('row-dot reduction over a non-coalescible view')
      dev = out_device(inputs, slots)
      esize = np.dtype(root.dtype).itemsize
      total = prod(in_shape) * esize
      if axis is not None and total > self.MATERIALISE_LIMIT:
        kept = [d for d in range(len(in_shape)) if d != axis and in_shape[d] > 1]
        if kept:
          return self._reduce_slabs(root, op, inputs, tuple(in_shape), axis, tuple(out_shape), out_dtype,
                                    idx_geom, kept[0], dev)
      tmp = torch.empty(tuple(in_shape), dtype=torch_dtype(root.dtype), device=dev)
      self.map(root, inputs, tmp)
      return self.reduce(codegen.In(0, root.dtype), op, {0: tmp}, in_shape, axis, out_shape, out_dtype, idx_geom)
    O, R, I, vstr = view
    dev = out_device(inputs, slots)
    n_out = O * I
    arg = op in ('argmin', 'argmax')
    adt = codegen.acc_dtype(op, root.dtype)
    if arg:
      res_v = torch.empty(tuple(out_shape), dtype=torch_dtype(adt), device=dev)
      result = torch.empty(tuple(out_shape), dtype=torch.int64, device=dev)
    else:
      result = torch.empty(tuple(out_shape), dtype=torch_dtype(out_dtype), device=dev)
    if n_out == 0:
      return (res_v, result) if arg else result
    if R == 0:
      raise ValueError('zero-size reduction')
    V = codegen.vec_width([dt for _, dt in ins] + [adt])
    args = codegen.KArgs()
    _scalars_into(root, args)
    for k, s in enumerate(slots):
      args.ptr[s] = inputs[s].data_ptr()
      for d in range(3):
        args.str[s][d] = vstr[k][d]
    args.dim[0], args.dim[1], args.dim[2] = O, R, I
    target_blocks = 2048
    if I == 1 and R <= 64 * V * 16:
      # short segments: several per wave (LPR lanes each), grid-stride over O
      kind = 'rowsp'
      classes = [_cls(vstr[k][1]) for k in range(len(slots))]
      vec_ok = V > 1 and R % V == 0 and all(
          _aligned_ptr(inputs[s], V) and (vstr[k][0] % V == 0 if classes[k] == 'c' else True)
          for k, s in enumerate(slots))
      per = V if vec_ok else 1
      need = -(-R // per)
      lpr = 1
      while lpr < need and lpr < 64:
        lpr *= 2
      seg_per_block = 4 * (64 // lpr)
      P = 1
      nblk = max(1, min(-(-O // seg_per_block), 256 * 16))
      args.aux[0], args.aux[1], args.aux[2] = 1, R, lpr.bit_length() - 1
    elif I == 1:
      kind = 'rows'
      classes = [_cls(vstr[k][1]) for k in range(len(slots))]
      vec_ok = V > 1 and R % V == 0 and all(
          _aligned_ptr(inputs[s], V) and (vstr[k][0] % V == 0 if classes[k] == 'c' else True)
          for k, s in enumerate(slots))
      per = V if vec_ok else 1
      P = 1
      if O < target_blocks:
        P = max(1, min(-(-target_blocks // O), -(-R // (256 * per * 4))))
      chunk = -(-R // P)
      chunk = -(-chunk // per) * per
      P = -(-R // chunk)
      nblk = O * P
      # grid-stride kernel: at most ROWS_GRID_PER_CU resident blocks per CU
      # stream the segments
      nblk = min(nblk, ROWS_GRID_PER_CU * _num_cus())
      args.aux[0], args.aux[1] = P, chunk
    else:
      kind = 'cols'
      classes = [_cls(vstr[k][2]) for k in range(len(slots))]
      vec_ok = V > 1 and I % V == 0 and all(
          _aligned_ptr(inputs[s], V) and ((vstr[k][0] % V == 0 and vstr[k][1] % V == 0)
                                          if classes[k] == 'c' else True)
          for k, s in enumerate(slots))
      per = V if vec_ok else 1
      need = -(-I // per)
      lpr = 1
      while lpr < need and lpr < 64:
        lpr *= 2
      CT = -(-I // (lpr * per))
      rows_per_step = 4 * (64 // lpr)
      base = CT * O
      P = 1
      # wide column reductions (several column tiles) stream best with
      # exactly two resident blocks per CU (cfg2 axis 0: 512 blocks 1.80 ms,
      # 1024 1.87, 2048 1.87, 4096 1.90); one narrow column tile (cfg5's 64
      # columns) with eight (2048: 4.06 ms per lreg iteration, 512: 4.15)
      # -- profiles/r02_cfg2_grid.txt; a fused row dot (cfg5's gradient, one
      # 64-column tile) with ROWDOT_BLOCKS_PER_CU (one, its rows interleaved
      # over the blocks: see ROWDOT_INTERLEAVE)
      rowdot = bool(codegen.rowdots(root))
      tb = (COLS_BLOCKS_PER_CU if CT > 1 else ROWDOT_BLOCKS_PER_CU if rowdot else 8) * _num_cus()
      if base < tb:
        P = max(1, min(-(-tb // base), -(-R // (rows_per_step * 4))))
      chunk = -(-R // P)
      P = -(-R // chunk)
      nblk = base * P
      args.aux[0], args.aux[1], args.aux[2], args.aux[3] = P, chunk, lpr.bit_length() - 1, CT
    if codegen.rowdots(root) and (kind != 'cols' or CT != 1):
      raise NotImplementedError('fused row dot needs each row in one lane group (K <= 64 * vector width)')
    if nblk > 0x7fffffff:
      raise NotImplementedError('reduction grid too large')
    args.flags = 1 if vec_ok else 0
    if arg:
      g = idx_geom or {}
      args.aux[4] = g.get('offset', 0)
      args.aux[5] = 1 if g.get('decompose') else 0
      if g.get('decompose'):
        tshape, tul, ashape = g['tshape'], g['tul'], g['ashape']
        args.aux[6] = len(tshape)
        for d in range(len(tshape)):
          args.tshape[d], args.tul[d], args.ashape[d] = tshape[d], tul[d], ashape[d]
    # a fused row dot's lane group width (and whether the vector path covers
    # the columns exactly) is compiled in: its per-row lane sum is then
    # straight-line DPP (codegen.gen_reduce)
    klpr, kfull = None, False
    if kind == 'cols' and codegen.rowdots(root):
      klpr, kfull = lpr, bool(vec_ok and CT == 1 and I == lpr * per)
    kint = bool((klpr and ROWDOT_INTERLEAVE) or (kind == 'cols' and CT > 1 and op == 'sum' and COLS_INTERLEAVE))
    # partials' dtype: fp64 for an interleaved fp32 sum (codegen.partial_dtype)
    pdt = codegen.partial_dtype(op, adt, kint) if kind == 'cols' else adt
    if arg:
      direct = P == 1
      part_v = res_v if direct else torch.empty((P * n_out,), dtype=torch_dtype(adt), device=dev)
      part_i = result if direct else torch.empty((P * n_out,), dtype=torch.int64, device=dev)
    else:
      direct = (P == 1 and pdt == np.dtype(out_dtype))
      part_v = result if direct else torch.empty((P * n_out,), dtype=torch_dtype(pdt), device=dev)
      part_i = None
    args.out0 = part_v.data_ptr()
    args.out1 = part_i.data_ptr() if arg else 0
    U, rowinv = None, ()
    if kind == 'cols':
      U = codegen.cols_unroll(ins, classes, V, [vstr[k][1] for k in range(len(slots))])
      if codegen.rowdots(root):
        U = ROWDOT_UNROLL
      rowinv = tuple(s for k, s in enumerate(slots) if vstr[k][1] == 0)
    sig = ('reduce', root.sig(), tuple(ins), tuple(classes), kind, op, V, U, rowinv, klpr, kfull, kint)
    fn = self._sig_fns.get(sig)
    if fn is None:
      src, kname = codegen.named(codegen.gen_reduce(root, ins, classes, kind, op, V, U, rowinv, klpr, kfull,
                                                    kint), 'spx_reduce', kind)
      fn = self._sig_fns[sig] = self.kernel(src, kname)
    self.launch(fn, nblk, args)
    if not direct:
      _check(self.lib.spx_reduce_finalize(
          OP_CODE[op], spx_dtype(pdt), spx_dtype(np.int64 if arg else out_dtype),
          ctypes.c_void_p(part_v.data_ptr()), ctypes.c_void_p(part_i.data_ptr() if arg else 0), P, n_out,
          ctypes.c_void_p(result.data_ptr()), ctypes.c_void_p(res_v.data_ptr() if arg else 0),
          self.stream()), 'spx_reduce_finalize')
    if len(self._reduce_plans) >= 512:
      self._reduce_plans.clear()
    self._reduce_plans[pkey] = (fn, nblk, bytes(args), arg, direct, pdt, P, n_out, dev, OP_CODE[op])
    return (res_v, result) if arg else result

  def _replay_reduce(self, plan, root, inputs, slots, out_shape, out_dtype):
    """backend.reduce from a recorded launch plan: the same kernel, grid and
    argument block, with this call's scalars, pointers and output buffers."""
    import torch
    fn, nblk, blob, arg, direct, adt, P, n_out, dev, opc = plan
    args = codegen.KArgs.from_buffer_copy(blob)
    _scalars_into(root, args)
    for s in slots:
      args.ptr[s] = inputs[s].data_ptr()
    if arg:
      res_v = torch.empty(tuple(out_shape), dtype=torch_dtype(adt), device=dev)
      result = torch.empty(tuple(out_shape), dtype=torch.int64, device=dev)
      part_v = res_v if direct else torch.empty((P * n_out,), dtype=torch_dtype(adt), device=dev)
      part_i = result if direct else torch.empty((P * n_out,), dtype=torch.int64, device=dev)
    else:
      result = torch.empty(tuple(out_shape), dtype=torch_dtype(out_dtype), device=dev)
      part_v = result if direct else torch.empty((P * n_out,), dtype=torch_dtype(adt), device=dev)
      part_i = None
    args.out0 = part_v.data_ptr()
    args.out1 = part_i.data_ptr() if arg else 0
    self.launch(fn, nblk, args)
    if not direct:
      _check(self.lib.spx_reduce_finalize(
          opc, spx_dtype(adt),
          spx_dtype(np.int64 if arg else out_dtype),
          ctypes.c_void_p(part_v.data_ptr()), ctypes.c_void_p(part_i.data_ptr() if arg else 0), P, n_out,
          ctypes.c_void_p(result.data_ptr()), ctypes.c_void_p(res_v.data_ptr() if arg else 0),
          self.stream()), 'spx_reduce_finalize')
    return (res_v, result) if arg else result

  def contiguous(self, t, dtype=None):
    """Dense copy of a strided view (and/or dtype conversion) by the generated
    identity-map kernel; ``t`` itself when nothing is to be done."""
    import torch
    src_dt = np_dtype(t.dtype)
    dst_dt = np.dtype(dtype) if dtype is not None else src_dt
    if t.is_contiguous() and dst_dt == src_dt:
      return t
    out = torch.empty(tuple(t.shape), dtype=torch_dtype(dst_dt), device=t.device)
    if t.numel() == 0:
      return out
    root = codegen.In(0, src_dt)
    if dst_dt != src_dt:
      root = codegen.Cast(root, dst_dt)
    self.map(root, {0: t}, out)
    return out

  # ------------------------------------------------------------ finalize
  def finalize(self, op, parts, P, n, out):
    """out[i] = fold over p < P of parts[p * n + i] in p order (sum / min /
    max; NaN propagates for min / max like np.minimum / np.maximum)."""
    dt = spx_dtype(np_dtype(parts.dtype))
    _check(self.lib.spx_reduce_finalize(OP_CODE[op], dt, spx_dtype(np_dtype(out.dtype)),
                                        ctypes.c_void_p(parts.data_ptr()), ctypes.c_void_p(0), P, n,
                                        ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(0), self.stream()),
           'spx_reduce_finalize')

  def argcombine(self, op, vals, idx):
    """vals/idx: [R, n] -> (val[n], idx[n]) best-of-R with first-index ties."""
    import torch
    R, n = vals.shape[0], vals.shape[1] if vals.dim() > 1 else 1
    out_i = torch.empty((n,), dtype=torch.int64, device=vals.device)
    out_v = torch.empty((n,), dtype=vals.dtype, device=vals.device)
    _check(self.lib.spx_argreduce_combine(OP_CODE[op], spx_dtype(np_dtype(vals.dtype)),
                                          ctypes.c_void_p(vals.data_ptr()), ctypes.c_void_p(idx.data_ptr()),
                                          R, n, ctypes.c_void_p(out_v.data_ptr()),
                                          ctypes.c_void_p(out_i.data_ptr()), self.stream()),
           'spx_argreduce_combine')
    return out_v, out_i

  # ---------------------------------------------------------------- merge
  def merge(self, dst, mask, region_ul, src, op, fastpath=True):
    shape = tuple(dst.shape)
    _check(self.lib.spx_merge(OP_CODE[op], spx_dtype(np_dtype(dst.dtype)), ctypes.c_void_p(dst.data_ptr()),
                              ctypes.c_void_p(mask.data_ptr() if mask is not None else 0), len(shape),
                              _arr(shape), _arr(region_ul), _arr(tuple(src.shape) if src.dim() else ()),
                              ctypes.c_void_p(src.data_ptr()), spx_dtype(np_dtype(src.dtype)),
                              1 if fastpath else 0, self.stream()), 'spx_merge')

  def copy_region(self, dst, dst_ul, src, src_ul, shape):
    nd = len(shape)
    _check(self.lib.spx_copy_region(spx_dtype(np_dtype(dst.dtype)), ctypes.c_void_p(dst.data_ptr()),
                                    _arr(tuple(dst.shape)), _arr(dst_ul), spx_dtype(np_dtype(src.dtype)),
                                    ctypes.c_void_p(src.data_ptr()), _arr(tuple(src.shape)), _arr(src_ul), nd,
                                    _arr(shape), self.stream()), 'spx_copy_region')

  MATERIALISE_LIMIT = 2 << 30  # bytes of one materialised slab (non-coalescible reductions)

  def _reduce_slabs(self, root, op, inputs, in_shape, axis, out_shape, out_dtype, idx_geom, d, dev):
    """reduce() over slabs of the kept dim ``d`` (each slab materialised and
    reduced on its own), results copied into place."""
    import torch
    nd = len(in_shape)
    per = prod(in_shape) // in_shape[d] * np.dtype(root.dtype).itemsize
    nc = max(1, self.MATERIALISE_LIMIT // max(1, per))
    od = d if d < axis else d - 1  # the same dim in the output
    arg = op in ('argmin', 'argmax')
    res_v = res_i = None
    for c0 in range(0, in_shape[d], nc):
      c1 = min(in_shape[d], c0 + nc)
      sub = {}
      for sl, t in inputs.items():
        td = d - (nd - t.dim())  # inputs broadcast from the right
        sub[sl] = t.narrow(td, c0, c1 - c0) if td >= 0 and t.shape[td] == in_shape[d] else t
      sshape = in_shape[:d] + (c1 - c0,) + in_shape[d + 1:]
      soshape = out_shape[:od] + (c1 - c0,) + out_shape[od + 1:]
      got = self.reduce(root, op, sub, sshape, axis, soshape, out_dtype, idx_geom)
      ul = tuple(c0 if k == od else 0 for k in range(len(out_shape)))
      parts = got if arg else (got,)
      if res_v is None:
        res_v = torch.empty(out_shape, dtype=parts[0].dtype, device=dev)
        if arg:
          res_i = torch.empty(out_shape, dtype=parts[1].dtype, device=dev)
      self.copy_region(res_v, ul, parts[0], (0,) * len(out_shape), soshape)
      if arg:
        self.copy_region(res_i, ul, parts[1], (0,) * len(out_shape), soshape)
    return (res_v, res_i) if arg else res_v

  # ----------------------------------------------------------------- gemm
  def gemm(self, A, B, C, alpha=1.0, beta=0.0):
    """C = alpha * A @ B + beta * C for 2-d contiguous row-major tensors."""
    M, K = A.shape
    K2, N = B.shape
    assert K == K2 and tuple(C.shape) == (M, N)
    dt = np_dtype(A.dtype)
    ev = self._aot_events('spx_gemm')
    _check(self.lib.spx_gemm(spx_dtype(dt), M, N, K, ctypes.c_void_p(A.data_ptr()), A.stride(0),
                             ctypes.c_void_p(B.data_ptr()), B.stride(0), ctypes.c_void_p(C.data_ptr()),
                             C.stride(0), float(alpha), float(beta), self.stream()), 'spx_gemm')
    if ev is not None:
      ev[1].record()


  # --------------------------------------------------------------- k-means
  def kmeans_assign(self, points, centers, labels, mindist=None, exact_only=False, dist_dtype=np.float64):
    """labels[p] = first argmin_c cdist(points[p], centers[c]) (exact fp64
    order; dist_dtype float32: of the distances rounded to fp32).  Default:
    MFMA-certified fast path + exact-order kernel for the undecided points;
    exact_only=True (or mindist) runs every point exactly."""
    N, D = points.shape
    K = centers.shape[0]
    assert centers.dtype == self._f64() and tuple(centers.shape) == (K, D) and labels.shape[0] == N
    dt = spx_dtype(np_dtype(points.dtype))
    ws, nws = None, 0
    if mindist is None and not exact_only and N > 0:
      need = self.lib.spx_kmeans_assign_workspace(dt, N, D, K)
      if need < 0:
        raise RuntimeError('spx_kmeans_assign_workspace: bad arguments')
      ws = self._workspace(int(need), points.device)
      nws = ws.numel()
    _check(self.lib.spx_kmeans_assign(dt, N, D, K, ctypes.c_void_p(points.data_ptr()), points.stride(0),
                                      ctypes.c_void_p(centers.data_ptr()), ctypes.c_void_p(labels.data_ptr()),
                                      ctypes.c_void_p(mindist.data_ptr() if mindist is not None else 0),
                                      ctypes.c_void_p(ws.data_ptr() if ws is not None else 0), nws,
                                      spx_dtype(dist_dtype), self.stream()), 'spx_kmeans_assign')

  def kmeans_accumulate(self, points, labels, sums, counts, zero_first=True):
    N, D = points.shape
    K = sums.shape[0]
    dt = spx_dtype(np_dtype(points.dtype))
    need = self.lib.spx_kmeans_accumulate_workspace(dt, N, D, K)
    if need < 0:
      raise RuntimeError('spx_kmeans_accumulate_workspace: bad arguments')
    ws = self._workspace(max(int(need), 8), points.device)
    _check(self.lib.spx_kmeans_accumulate(dt, N, D, K, ctypes.c_void_p(points.data_ptr()), points.stride(0),
                                          ctypes.c_void_p(labels.data_ptr()), ctypes.c_void_p(sums.data_ptr()),
                                          ctypes.c_void_p(counts.data_ptr()), 1 if zero_first else 0,
                                          ctypes.c_void_p(ws.data_ptr()), ws.numel(), self.stream()),
           'spx_kmeans_accumulate')

  def kmeans_step(self, points, centers, labels, sums, counts, zero_first=True, dist_dtype=np.float64):
    """kmeans_assign + kmeans_accumulate in one call (spx_kmeans_step): the
    certified screen labels and accumulates the decided rows in one pass."""
    N, D = points.shape
    K = centers.shape[0]
    assert centers.dtype == self._f64() and tuple(centers.shape) == (K, D) and labels.shape[0] == N
    assert tuple(sums.shape) == (K, D) and counts.shape[0] == K and sums.is_contiguous() and counts.is_contiguous()
    dt = spx_dtype(np_dtype(points.dtype))
    need = self.lib.spx_kmeans_step_workspace(dt, N, D, K)
    if need < 0:
      raise RuntimeError('spx_kmeans_step_workspace: bad arguments')
    ws = self._workspace(max(int(need), 8), points.device)
    _check(self.lib.spx_kmeans_step(dt, N, D, K, ctypes.c_void_p(points.data_ptr()), points.stride(0),
                                    ctypes.c_void_p(centers.data_ptr()), ctypes.c_void_p(labels.data_ptr()),
                                    ctypes.c_void_p(sums.data_ptr()), ctypes.c_void_p(counts.data_ptr()),
                                    1 if zero_first else 0, ctypes.c_void_p(ws.data_ptr()), ws.numel(),
                                    spx_dtype(dist_dtype), self.stream()), 'spx_kmeans_step')

  def cdist(self, points, centers, out):
    """out (N, K) = exact-order cdist(points, centers), rounded to out's dtype."""
    N, D = points.shape
    K = centers.shape[0]
    assert centers.dtype == self._f64() and tuple(centers.shape) == (K, D) and tuple(out.shape) == (N, K)
    assert centers.is_contiguous() and points.stride(1) == 1 and out.stride(1) == 1
    _check(self.lib.spx_cdist(spx_dtype(np_dtype(points.dtype)), spx_dtype(np_dtype(out.dtype)), N, D, K,
                              ctypes.c_void_p(points.data_ptr()), points.stride(0),
                              ctypes.c_void_p(centers.data_ptr()), ctypes.c_void_p(out.data_ptr()), out.stride(0),
                              self.stream()), 'spx_cdist')

  def bincount(self, labels, counts, zero_first=True):
    """counts (K,) int64 (+)= bincount of int64 ``labels`` (out-of-range skipped)."""
    assert labels.dtype == counts.dtype and labels.is_contiguous() and counts.is_contiguous()
    _check(self.lib.spx_bincount(ctypes.c_void_p(labels.data_ptr()), labels.numel(), counts.numel(),
                                 ctypes.c_void_p(counts.data_ptr()), 1 if zero_first else 0, self.stream()),
           'spx_bincount')

  def kmeans_counters(self, D):
    """Diagnostic (tests, tools): the four u32 counters of the last
    spx_kmeans_assign / spx_kmeans_step workspace in the certified screens'
    layout (K <= 256; spx.hip KmWs): [rows sent to the all-centre exact
    kernel, candidate rows, rows left undecided by the bf16x3 pass, rows left
    undecided by the fp16 screen]."""
    import torch
    off = (D * 256 * 4 + 15) // 16 * 16 + 256 * 8 + 32
    return self._ws[off:off + 16].view(torch.int32).cpu().tolist()

  def _workspace(self, nbytes, device):
    """Grow-only scratch buffer on ``device`` (reuse is stream-ordered)."""
    import torch
    ws = getattr(self, '_ws', None)
    if ws is None or ws.numel() < nbytes or ws.device != device:
      ws = torch.empty((nbytes,), dtype=torch.uint8, device=device)
      self._ws = ws
    return ws

  @staticmethod
  def _f64():
    import torch
    return torch.float64


def out_device(inputs, slots):
  import torch
  if slots:
    return inputs[slots[0]].device
  return torch.device('cuda', torch.cuda.current_device())


def _cls(stride):
  return 'c' if stride == 1 else ('b' if stride == 0 else 'g')


def _aligned_ptr(t, V):
  return t.data_ptr() % (V * t.element_size()) == 0


def _vec_aligned(t, strides, cls, V):
  if cls == 'c':
    return _aligned_ptr(t, V) and all(s % V == 0 for s in strides[:-1])
  return True


def _scalars_into(root, args):
  for node in codegen.walk(root):
    if isinstance(node, codegen.Sc):
      if node.pytype is float:
        args.fsc[node.slot] = node.value
      else:
        args.isc[node.slot] = int(node.value)


# ----------------------------------------------------------- active backend
_backend = None


def get():
  global _backend
  if _backend is None:
    _backend = HipBackend()
  return _backend


def set_backend(b):
  """Install a backend object (tests only); returns the previous one."""
  global _backend
  prev = _backend
  _backend = b
  return prev
