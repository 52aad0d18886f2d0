"""Zero-copy views over a DistArray: Slice, Transpose and UnitDims.

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


class UnitDims(DistArray):
  """``base`` with length-1 dimensions dropped and / or inserted, without a
  copy: the reference's ReshapeExpr after an int / newaxis index
  (base.py:388-430).  Non-unit dims keep their order; every region maps to
  the base region with the unit dims set to [0, 1), and a fetched piece is a
  reshaped (still strided) view of the base piece."""

  def __init__(self, base, shape):
    shape = tuple(int(s) for s in shape)
    nb = [i for i, s in enumerate(base.shape) if s != 1]
    nn = [j for j, s in enumerate(shape) if s != 1]
    if [base.shape[i] for i in nb] != [shape[j] for j in nn]:
      raise ValueError('UnitDims: %s -> %s changes a non-unit dimension' % (base.shape, shape))
    self.base = base
    self.shape = shape
    self.dtype = base.dtype
    self.bad_tiles = []
    self._b2n = dict(zip(nb, nn))   # base dim -> view dim (non-unit dims)
    self._n2b = dict(zip(nn, nb))
    self.tiles = {self.from_base(ex): w for ex, w in base.tiles.items()}

  def from_base(self, region):
    ul = [0] * len(self.shape)
    lr = [1] * len(self.shape)
    for i, j in self._b2n.items():
      ul[j], lr[j] = region.ul[i], region.lr[i]
    return ext.create(tuple(ul), tuple(lr), self.shape)

  def to_base(self, region):
    ul = [0] * len(self.base.shape)
    lr = [1] * len(self.base.shape)
    for j, i in self._n2b.items():
      ul[i], lr[i] = region.ul[j], region.lr[j]
    return ext.create(tuple(ul), tuple(lr), self.base.shape)

  def tile_shape(self):
    counts = {}
    for ex in self.tiles:
      counts[ex.shape] = counts.get(ex.shape, 0) + 1
    return sorted(counts.items(), key=lambda kv: (kv[1], kv[0]))[-1][0]

  def _v(self, t, region):
    return t.reshape(tuple(region.shape) if region.ndim else ())

  def fetch(self, region):
    return self._v(self.base.fetch(self.to_base(region)), region)

  def owner_of_region(self, region):
    return self.base.owner_of_region(self.to_base(region))

  def gather(self, requests):
    got = gather_regions(self.base, [(self.to_base(r), d) for r, d in requests])
    return {k: self._v(v, requests[k][0]) for k, v in got.items()}

  def glom(self):
    return np.asarray(self.base.glom()).reshape(self.shape)


def unit_dims_of(array, shape):
  if tuple(shape) == tuple(array.shape):
    return array
  if isinstance(array, UnitDims):
    array = array.base
  return UnitDims(array, shape)


def slice_of(array, idx):
  return Slice(array, idx)


def transpose_of(array):
  if isinstance(array, Transpose):
    return array.base
  return Transpose(array)


def is_view(array):
  return isinstance(array, (Slice, Transpose, UnitDims))

