"""HBM-resident dense tiles and the reference's merge rule.

Restates spartan/array/tile.pyx (Tile :25-143, from_shape :163-177,
merge :201-298) for dense tiles whose data is a PyTorch-ROCm device tensor.
The per-element "already written" mask of the reference is tracked on the
host as a list of written extents, so the common cases (first write, a
re-write of a fully written region, the full-tile fast path) need no device
mask and no host synchronisation; only irregular partial overlaps
materialise a device mask and use spx_merge's masked path.
"""
import numpy as np

from .. import backend
from . import extent as ext


class Tile:
  __slots__ = ('_data', '_spec', 'ex', 'written', 'mask')

  def __init__(self, data, ex, written=False, spec=None):
    self._data = data         # torch tensor, shape == ex.shape (0-d for scalar tiles)
    self._spec = spec         # (shape, torch dtype, device) when allocation is deferred
    self.ex = ex              # the tile's extent (coordinates in its array)
    self.written = [ex] if written else []
    self.mask = None          # device uint8 mask, only for irregular partial merges

  @classmethod
  def deferred(cls, shape, tdtype, device, ex):
    """Tile whose HBM is allocated on first access (reference Tile.data is
    None until _initialize, tile.pyx:116-128)."""
    return cls(None, ex, spec=(tuple(shape), tdtype, device))

  @property
  def data(self):
    if self._data is None:
      import torch
      shape, tdt, dev = self._spec
      self._data = torch.empty(shape, dtype=tdt, device=dev)
    return self._data

  @data.setter
  def data(self, t):
    self._data = t

  @property
  def dtype(self):
    if self._data is None:
      return backend.np_dtype(self._spec[1])
    return backend.np_dtype(self._data.dtype)

  @property
  def shape(self):
    if self._data is None:
      return self._spec[0]
    return tuple(self._data.shape)

  def origin_written(self):
    o = tuple(self.ex.ul)
    for w in self.written:
      if all(u <= x < l or (u == l and x == u) for u, l, x in zip(w.ul, w.lr, o)):
        return True
    return False


def _covered(region, regions):
  """True iff some single written region contains ``region``."""
  for w in regions:
    if all(wu <= ru and rl <= wl for wu, wl, ru, rl in zip(w.ul, w.lr, region.ul, region.lr)):
      return True
  return False


def _disjoint(region, regions):
  for w in regions:
    if ext.intersection(w, region) is not None:
      return False
  return True


def merge(tile, region, update, reducer_op):
  """tile[region] = reducer(tile[region], update) with first-write-replaces.

  ``region`` is an extent in the tile's array; ``update`` a device tensor of
  region.shape.  reducer_op in {'sum','min','max', None} (None = replace)."""
  be = backend.get()
  t_ex = tile.ex
  if len(tile.shape) == 0:  # 0-d tiles (tile.pyx:213-218)
    if not tile.written or reducer_op is None:
      be.copy_region(tile.data, (), update, (), ())
    else:
      be.merge(tile.data, None, (), update, reducer_op, fastpath=False)
    tile.written = [t_ex]
    return tile
  local_ul = tuple(r - u for r, u in zip(region.ul, t_ex.ul))
  full = tuple(region.ul) == tuple(t_ex.ul) and tuple(region.lr) == tuple(t_ex.lr)
  if full:
    # reference fast path: reduce iff mask[0] is set, else replace (tile.pyx:264-269)
    if reducer_op is not None and tile.origin_written():
      be.merge(tile.data, None, local_ul, update, reducer_op, fastpath=False)
    else:
      be.copy_region(tile.data, (0,) * len(local_ul), update, (0,) * len(local_ul), tile.shape)
    tile.written = [t_ex]
    tile.mask = None
    return tile
  if reducer_op is None or _disjoint(region, tile.written):
    be.copy_region(tile.data, local_ul, update, (0,) * len(local_ul), region.shape)
    tile.mask = None  # these branches do not set mask bits: rebuild from `written` when next needed
  elif _covered(region, tile.written):
    be.merge(tile.data, None, local_ul, update, reducer_op, fastpath=False)
    tile.mask = None
  else:
    if tile.mask is None:
      import torch
      tile.mask = torch.zeros(tile.shape, dtype=torch.bool, device=tile.data.device)
      for w in tile.written:
        wl = tuple(a - b for a, b in zip(w.ul, t_ex.ul))
        ones = torch.ones(w.shape, dtype=torch.bool, device=tile.data.device)
        be.copy_region(tile.mask, wl, ones, (0,) * len(wl), w.shape)
    be.merge(tile.data, tile.mask, local_ul, update, reducer_op, fastpath=False)
  tile.written.append(region)
  return tile


REDUCER_NAMES = {np.add: 'sum', np.minimum: 'min', np.maximum: 'max'}


def reducer_name(fn):
  if fn is None:
    return None
  if fn in REDUCER_NAMES:
    return REDUCER_NAMES[fn]
  raise NotImplementedError('reducer %r has no device merge (np.add / np.minimum / np.maximum)' % (fn,))
