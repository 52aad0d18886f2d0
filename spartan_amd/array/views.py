"""Zero-copy views over a DistArray: Slice and Transpose.

Restate spartan/expr/slice.py:41-84 (``Slice``) and
spartan/expr/transpose.py:25-65 (``Transpose``): a view reports tiles in its
own coordinates, owned by the workers that own the base tiles, and a fetch is
a fetch of the corresponding base region.  Here a fetched piece of a
Transpose is a strided device view (``permute``): the generated kernels read
it in place with the transposed strides (backend.map / reduce pass each
input's own strides), so no transposed copy is made unless a GEMM operand
needs row-major data.  ``gather_regions`` of a view is the same collective on
the base array.  A Slice of a Slice or Transpose of a Transpose collapses.
"""
import numpy as np

from . import extent as ext
from .distarray import DistArray, gather_regions, glom_region


class Slice(DistArray):
  """``base[idx]`` without a copy (slice.py:41-84).  Integer indices keep
  their dimension with length 1, as the reference's extent slicing does."""

  def __init__(self, base, idx):
    if isinstance(base, Slice):  # slice of a slice: one slice of the base
      inner = idx if isinstance(idx, ext.TileExtent) else ext.from_slice(idx, base.shape)
      idx = ext.create(tuple(u + o for u, o in zip(inner.ul, base.slice.ul)),
                       tuple(l + o for l, o in zip(inner.lr, base.slice.ul)), base.base.shape)
      base = base.base
    self.base = base
    self.slice = idx if isinstance(idx, ext.TileExtent) else ext.from_slice(idx, base.shape)
    self.shape = tuple(int(s) for s in self.slice.shape)
    self.dtype = base.dtype
    self.bad_tiles = []
    tiles = {}
    for bex, w in base.tiles.items():
      inter = ext.intersection(bex, self.slice)
      if inter is None or any(l <= u for u, l in zip(inter.ul, inter.lr)):
        continue
      tiles[self.from_base(inter)] = w
    self.tiles = tiles

  def from_base(self, region):
    return ext.create(tuple(u - o for u, o in zip(region.ul, self.slice.ul)),
                      tuple(l - o for l, o in zip(region.lr, self.slice.ul)), self.shape)

  def to_base(self, region):
    return ext.create(tuple(u + o for u, o in zip(region.ul, self.slice.ul)),
                      tuple(l + o for l, o in zip(region.lr, self.slice.ul)), self.base.shape)

  def tile_shape(self):
    counts = {}
    for ex in self.tiles:
      counts[ex.shape] = counts.get(ex.shape, 0) + 1
    return sorted(counts.items(), key=lambda kv: (kv[1], kv[0]))[-1][0]

  def fetch(self, region):
    return self.base.fetch(self.to_base(region))

  def owner_of_region(self, region):
    return self.base.owner_of_region(self.to_base(region))

  def gather(self, requests):
    return gather_regions(self.base, [(self.to_base(r), d) for r, d in requests])

  def glom(self):
    return glom_region(self.base, self.slice).reshape(self.shape)


def _rev(ex, shape):
  return ext.create(tuple(reversed(ex.ul)), tuple(reversed(ex.lr)), shape)


class Transpose(DistArray):
  """All axes reversed without a copy (transpose.py:25-65)."""

  def __init__(self, base):
    self.base = base
    self.shape = tuple(reversed(base.shape))
    self.dtype = base.dtype
    self.bad_tiles = []
    self.tiles = {_rev(ex, self.shape): w for ex, w in base.tiles.items()}

  def to_base(self, region):
    return _rev(region, self.base.shape)

  def tile_shape(self):
    return tuple(reversed(self.base.tile_shape()))

  def _t(self, t):
    return t.permute(*reversed(range(t.dim()))) if t.dim() > 1 else t

  def fetch(self, region):
    return self._t(self.base.fetch(self.to_base(region)))

  def owner_of_region(self, region):
    return self.base.owner_of_region(self.to_base(region))

  def gather(self, requests):
    got = gather_regions(self.base, [(self.to_base(r), d) for r, d in requests])
    return {k: self._t(v) for k, v in got.items()}

  def glom(self):
    return np.ascontiguousarray(np.transpose(self.base.glom()))


def slice_of(array, idx):
  return Slice(array, idx)


def transpose_of(array):
  if isinstance(array, Transpose):
    return array.base
  return Transpose(array)


def is_view(array):
  return isinstance(array, (Slice, Transpose))

