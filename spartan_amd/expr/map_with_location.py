"""``map_with_location`` and ``region_map`` (restate
spartan/expr/map_with_location.py:22-60 and spartan/expr/region_map.py:9-80).

``map_with_location(inputs, fn)`` calls ``fn(*tiles, (ul, lr, array_shape),
**fn_kw)``.  It is a MapExpr whose LocalMapLocationExpr is lowered once PER
TILE with that tile's location as plain Python values (engine
run_location_map): the trace of a mapper that only does arithmetic on the
location (``tile + ex[0][0]``) differs between tiles only in kernel-argument
scalars, so the tiles share one compiled kernel; a mapper that branches on
the location (nbody.py:30-40 ``_set_diagonal_mapper``) gets one kernel per
distinct trace.  Such maps fuse with other maps (MapMapFusion) but stay out
of fused reductions.

``region_map(array, region, fn)`` keeps every element outside ``region``
and replaces each tile's part inside the FIRST region extent that meets the
tile by ``fn(part, tile_extent, **fn_kw)`` (region.py:9-39): a copy of the
tile, the traced ``fn`` over the sub-block, and a copy back into the tile's
offset -- per tile, no host round trip.
"""
import numpy as np

from .. import backend, codegen, runtime
from ..array import distarray, extent as ext
from .base import Expr, ListExpr, as_array, lazify
from .local import CodegenError, LocalInput, LocalMapLocationExpr, LowerEnv, make_var, trace_callable
from .map import MapExpr


def map_with_location(inputs, fn, numpy_expr=None, fn_kw=None):
  """Like ``map``, with the tile's location as an extra argument."""
  assert fn is not None
  if not isinstance(inputs, (list, tuple)):
    inputs = [inputs]
  children, child_to_var, op_deps = [], [], []
  for v in inputs:
    v = as_array(v)
    var = make_var()
    children.append(v)
    child_to_var.append(var)
    op_deps.append(LocalInput(var))
  op_deps.append(LocalInput('extent'))
  op = LocalMapLocationExpr(fn=fn, kw=fn_kw, pretty_fn=numpy_expr, deps=op_deps)
  return MapExpr(children=ListExpr(vals=children), child_to_var=child_to_var, op=op)


class RegionMapExpr(Expr):
  _members = ('array',)

  def compute_shape(self):
    return self.array.shape

  def compute_dtype(self):
    return self.array.dtype

  def pretty_str(self):
    return 'RegionMap[%d](%s)' % (self.expr_id, getattr(self.fn, '__name__', self.fn))

  def _evaluate(self, deps):
    return region_map_array(distarray.as_array(deps['array']), self.region, self.fn, self.fn_kw)


def region_map_array(arr, region, fn, fn_kw):
  import torch
  ctx = runtime.get()
  be = backend.get()
  dt = np.dtype(arr.dtype)
  tdt = backend.torch_dtype(dt)
  out_local = {}
  for ex, w in arr.tiles.items():
    if not ctx.is_local(w):
      continue
    src = arr.fetch(ex)
    out = torch.empty(ex.shape, dtype=tdt, device=ctx.device)
    be.copy_region(out, (0,) * ex.ndim, src, (0,) * ex.ndim, ex.shape)
    for area in region:
      inter = ext.intersection(area, ex)
      if inter is None:
        continue
      rel = tuple(u - o for u, o in zip(inter.ul, ex.ul))
      sub = torch.empty(inter.shape, dtype=tdt, device=ctx.device)
      be.copy_region(sub, (0,) * ex.ndim, out, rel, inter.shape)
      env = LowerEnv({}, ex)
      leaf = codegen.In(0, dt)
      try:
        from .local import Sym
        s = Sym(leaf, env, tuple(inter.shape))
        res = fn(s, ex, **(fn_kw or {}))
      except CodegenError:
        raise
      except Exception as e:
        raise CodegenError('region mapper %s cannot be lowered to a gfx950 kernel (%s: %s)'
                           % (getattr(fn, '__name__', fn), type(e).__name__, e))
      new = torch.empty(inter.shape, dtype=tdt, device=ctx.device)
      if isinstance(res, Sym):
        if res.shape is not None and tuple(res.shape) != tuple(inter.shape):
          raise CodegenError('region mapper yielded a %s value for a %s region' % (res.shape, inter.shape))
        root = res.node if np.dtype(res.node.dtype) == dt else codegen.Cast(res.node, dt)
        be.map(root, {0: sub} if any(isinstance(n, codegen.In) for n in codegen.walk(root)) else {}, new)
      elif isinstance(res, (np.ndarray, np.generic, int, float, bool)):
        from ..array import transfer
        new = transfer.upload(np.ascontiguousarray(np.broadcast_to(np.asarray(res, dtype=dt), inter.shape)),
                              ctx.device)
      else:
        raise CodegenError('region mapper returned %s' % type(res).__name__)
      be.copy_region(out, rel, new, (0,) * ex.ndim, inter.shape)
      break  # only the first region extent that meets the tile (region_map.py:31-37)
    out_local[ex] = out
  return distarray.from_tiles(arr.shape, dt, arr.tiles, out_local)


def region_map(array, region, fn, fn_kw=None):
  """Map ``fn`` over ``region`` (a TileExtent or a list of them) of ``array``;
  elements outside keep their values (region_map.py:42-80)."""
  if isinstance(region, ext.TileExtent):
    region = [region]
  e = RegionMapExpr(array=lazify(array))
  e.region = list(region)
  e.fn = fn
  e.fn_kw = dict(fn_kw or {})
  return e
