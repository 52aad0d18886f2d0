"""``reshape(x, shape)`` (restates spartan/expr/reshape.py:45-229).

The reference's ``Reshape`` is a lazy view whose fetch ravels the requested
extent, finds the enclosing base rectangle, fetches it and trims it
(reshape.py:153-191); its own comment notes it cannot serve column fetches.
Here the reshape is materialised once, with the same values: the result
gets the default tiling of the new shape -- row strips, each a contiguous
range of the row-major flat index -- and every output tile's flat range is
cut into base rectangles that are themselves contiguous in flat order
(``flat_rects``), moved by ONE ``gather_regions`` exchange and packed into the
tile with ``spx_copy_region``.  Strided base pieces (a transposed input) are
made dense by the identity-map kernel first.
"""
import numpy as np

from .. import backend, runtime
from ..array import distarray, extent as ext
from ..array.distarray import LocalWrapper, ReplicatedArray
from ..util import prod
from .base import Expr, lazify


def flat_rects(a, b, shape):
  """Rectangles (ul, lr) covering flat indices [a, b) of a row-major
  ``shape`` in order, each contiguous in flat order."""
  if a >= b:
    return []
  shape = tuple(int(s) for s in shape)
  if len(shape) == 1:
    return [((a,), (b,))]
  inner = prod(shape[1:])
  r0, o0 = divmod(a, inner)
  r1, o1 = divmod(b, inner)
  if r0 == r1:
    return [((r0,) + ul, (r0 + 1,) + lr) for ul, lr in flat_rects(o0, o1, shape[1:])]
  out = []
  if o0:
    out += [((r0,) + ul, (r0 + 1,) + lr) for ul, lr in flat_rects(o0, inner, shape[1:])]
    r0 += 1
  if r1 > r0:
    out.append(((r0,) + (0,) * (len(shape) - 1), (r1,) + shape[1:]))
  if o1:
    out += [((r1,) + ul, (r1 + 1,) + lr) for ul, lr in flat_rects(0, o1, shape[1:])]
  return out


def _flat_range(ex, shape):
  """[a, b) of a tile that is contiguous in flat order, else None."""
  a = ext.ravelled_pos(ex.ul, shape)
  n = prod(ex.shape)
  lead = [d for d in range(len(shape)) if ex.lr[d] - ex.ul[d] != shape[d]]
  # contiguous iff every dim after the first partial one is whole, and the
  # partial dims before the last one have extent 1
  if lead and any(ex.lr[d] - ex.ul[d] != 1 for d in lead[:-1]):
    return None
  if lead and any(ex.lr[d] - ex.ul[d] != shape[d] for d in range(lead[-1] + 1, len(shape))):
    return None
  return a, a + n


def reshape_array(base, shape):
  import torch
  shape = tuple(int(s) for s in shape)
  if isinstance(base, np.ndarray):
    base = LocalWrapper(base)
  if prod(shape) != prod(base.shape):
    raise ValueError('cannot reshape array of size %d into shape %s' % (prod(base.shape), shape))
  if isinstance(base, ReplicatedArray):
    return ReplicatedArray(backend.get().contiguous(base.device_data()).reshape(shape))
  if isinstance(base, LocalWrapper):
    return LocalWrapper(np.asarray(base.value).reshape(shape))
  ctx = runtime.get()
  be = backend.get()
  tiles = distarray.compute_extents(shape, None, ctx.num_workers)
  requests, plan = [], []
  for ex, w in tiles.items():
    fr = _flat_range(ex, shape) if len(shape) else (0, 1)
    assert fr is not None, 'default tiles are flat-contiguous'
    off = 0
    for ul, lr in flat_rects(fr[0], fr[1], base.shape) if len(base.shape) else [((), ())]:
      region = ext.create(ul, lr, base.shape)
      n = prod(region.shape) if len(base.shape) else 1
      requests.append((region, ctx.owner(w)))
      plan.append((ex, w, off, n))
      off += n
  got = distarray.gather_regions(base, requests)
  local = {}
  for qi, (ex, w, off, n) in enumerate(plan):
    if not ctx.is_local(w):
      continue
    if ex not in local:
      local[ex] = torch.empty(ex.shape if len(shape) else (), dtype=backend.torch_dtype(base.dtype),
                              device=ctx.device)
    piece = be.contiguous(got[qi]).reshape(-1)
    be.copy_region(local[ex].reshape(-1), (off,), piece, (0,), (n,))
  return distarray.from_tiles(shape, base.dtype, tiles, local)


class ReshapeExpr(Expr):
  _members = ('array',)

  def compute_shape(self):
    return tuple(self.new_shape)

  def compute_dtype(self):
    return self.array.dtype

  def pretty_str(self):
    return 'Reshape[%d](%s, %s)' % (self.expr_id, self.array, self.new_shape)

  def _evaluate(self, deps):
    return reshape_array(deps['array'], self.new_shape)


def reshape(array, new_shape, tile_hint=None):
  e = ReshapeExpr(array=lazify(array))
  e.new_shape = tuple(int(s) for s in new_shape)
  e.tile_hint = tile_hint
  return e
