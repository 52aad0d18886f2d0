"""Rectangular tile extents -- restated from spartan/array/extent.pyx.

A ``TileExtent`` is ``[ul, lr)`` inside an array of ``array_shape``, int64
coordinates.  Every function here keeps the reference's integer semantics
bit-exactly; where the Cython source relied on Python-2 ``/`` on ints
(floor division) this module uses ``//`` explicitly
(e.g. ``unravelled_pos``, extent.pyx:192-205).

Quirks kept on purpose (SURVEY.md Appendix A pin 1):
  * ``shape`` reports 0-length dims as 1 (extent.pyx:66-72);
  * ``create`` returns None when any ``ul >= lr`` (extent.pyx:141-153);
  * ``intersection`` returns None when empty (extent.pyx:363-383).
"""
import numpy as np

from ..util import divup, prod


class TileExtent:
  __slots__ = ('_ul', '_lr', 'array_shape')

  def __init__(self, ul=(), lr=(), array_shape=None):
    self._ul = tuple(int(x) for x in ul)
    self._lr = tuple(int(x) for x in lr)
    self.array_shape = None if array_shape is None else tuple(int(x) for x in array_shape)

  @property
  def ul(self):
    return self._ul

  @property
  def lr(self):
    return self._lr

  @property
  def shape(self):  # extent.pyx:66-72
    return tuple((l - u) if (l - u) != 0 else 1 for u, l in zip(self._ul, self._lr))

  @property
  def size(self):
    return prod(self.shape)

  @property
  def ndim(self):
    return len(self._ul)

  def to_slice(self):
    return tuple(slice(u, l) for u, l in zip(self._ul, self._lr))

  def to_tuple(self):
    return (self._ul, self._lr, self.array_shape)

  def __repr__(self):
    return 'extent(' + ','.join('%s:%s' % (a, b) for a, b in zip(self._ul, self._lr)) + ')'

  def __getitem__(self, idx):
    return create((self._ul[idx],), (self._lr[idx],), (self.array_shape[idx],))

  def __hash__(self):
    return hash(self._ul)

  def __eq__(self, other):
    return isinstance(other, TileExtent) and self._ul == other._ul and self._lr == other._lr

  def __ne__(self, other):
    return not self.__eq__(other)

  def __lt__(self, other):  # lexicographic on ul (extent.pyx:96-106)
    return self._ul < other._ul

  def __gt__(self, other):
    return self._ul > other._ul

  def __reduce__(self):
    return (create, (self._ul, self._lr, self.array_shape))

  def ravelled_pos(self):
    return ravelled_pos(self._ul, self.array_shape)

  def to_global(self, idx, axis):
    """Local offset in this tile -> global offset (extent.pyx:117-123)."""
    if axis is not None:
      return idx + self._ul[axis]
    local_idx = unravelled_pos(idx, self.shape)
    return ravelled_pos(np.asarray(self._ul) + np.asarray(local_idx), self.array_shape)

  def add_dim(self):
    return create(self._ul + (0,), self._lr + (1,), self.array_shape + (1,))

  def clone(self):
    return TileExtent(self._ul, self._lr, self.array_shape)


def create(ul, lr, array_shape):
  """New extent, or None if any ``ul >= lr`` (extent.pyx:141-178)."""
  ul = tuple(int(x) for x in ul)
  lr = tuple(int(x) for x in lr)
  for u, l in zip(ul, lr):
    if u >= l:
      return None
  return TileExtent(ul, lr, array_shape)


def from_shape(shp):
  return create((0,) * len(shp), tuple(shp), tuple(shp))


def unravelled_pos(idx, array_shape):
  """Unravel a flat index (py2 floor division made explicit, extent.pyx:192-205)."""
  out = []
  idx = int(idx)
  for dim in reversed(array_shape):
    out.append(idx % dim)
    idx //= dim
  return tuple(reversed(out))


def ravelled_pos(idx, array_shape):
  rpos = 0
  mul = 1
  for i in range(len(array_shape) - 1, -1, -1):
    rpos += mul * int(idx[i])
    mul *= int(array_shape[i])
  return rpos


def all_nonzero_shape(shape):
  return all(int(s) != 0 for s in shape)


def find_rect(ravelled_ul, ravelled_lr, shape):
  if shape[-1] == 1 or ravelled_ul // shape[-1] == ravelled_lr // shape[-1]:
    return (ravelled_ul, ravelled_lr)
  div = 1
  for i in shape[1:]:
    div *= i
  return (ravelled_ul - (ravelled_ul % div), ravelled_lr + (div - ravelled_lr % div) % div - 1)


def find_overlapping(extents, region):
  for ex in extents:
    overlap = intersection(ex, region)
    if overlap is not None:
      yield (ex, overlap)


def compute_slice(base, idx):
  """Extent for ``base[idx]`` (extent.pyx:262-292)."""
  if np.isscalar(idx):
    idx = slice(int(idx), int(idx) + 1)
  if not isinstance(idx, tuple):
    idx = (idx,)
  ul, lr = [], []
  bshape = base.shape
  for i in range(base.ndim):
    if i >= len(idx):
      ul.append(base.ul[i])
      lr.append(base.lr[i])
    else:
      a = idx[i]
      if np.isscalar(a):
        a = slice(int(a), int(a) + 1)
      start, stop, _ = a.indices(bshape[i])
      ul.append(base.ul[i] + start)
      lr.append(base.ul[i] + stop)
  return create(ul, lr, base.array_shape)


def offset_from(base, other):
  ul, lr = [], []
  for i in range(base.ndim):
    assert not (other.ul[i] < base.ul[i] or other.lr[i] > base.lr[i])
    ul.append(other.ul[i] - base.ul[i])
    lr.append(other.lr[i] - base.ul[i])
  return create(ul, lr, other.array_shape)


def offset_slice(base, other):
  return tuple(slice(other.ul[i] - base.ul[i], other.lr[i] - base.ul[i], None)
               for i in range(base.ndim))


def from_slice(idx, shape):
  """Extent from a slice / tuple of slices (extent.pyx:322-357; None bounds allowed)."""
  if not isinstance(idx, tuple):
    idx = (idx,)
  if len(idx) < len(shape):
    idx = tuple(list(idx) + [slice(None)] * (len(shape) - len(idx)))
  ul, lr = [], []
  for dim, slc in zip(shape, idx):
    if np.isscalar(slc):
      slc = slice(int(slc), int(slc) + 1)
    if slc.start is not None and slc.start > 0:
      assert slc.start <= dim
    if slc.stop is not None and slc.stop > 0:
      assert slc.stop <= dim
    start, stop, _ = slc.indices(dim)
    ul.append(start)
    lr.append(stop)
  return create(ul, lr, shape)


def from_tuple(tup):
  return create(tup[0], tup[1], tup[2])


def intersection(a, b):
  """Intersection or None (extent.pyx:363-383)."""
  if a is None:
    return None
  assert a.array_shape == b.array_shape, 'Tiles must have compatible shapes! %s %s' % (
      a.array_shape, b.array_shape)
  ul, lr = [], []
  for i in range(a.ndim):
    if b.lr[i] < a.ul[i]:
      return None
    if a.lr[i] < b.ul[i]:
      return None
    ul.append(max(a.ul[i], b.ul[i]))
    lr.append(min(a.lr[i], b.lr[i]))
  return create(ul, lr, a.array_shape)


def shape_for_reduction(input_shape, axis):
  if axis is None:
    return ()
  s = list(input_shape)
  del s[axis]
  return tuple(s)


def shapes_match(offset, data):
  return tuple(offset.shape) == tuple(data.shape)


def drop_axis(ex, axis):
  if axis is None:
    return TileExtent((), (), ())
  if axis < 0:
    axis += ex.ndim
  shape = list(ex.array_shape)
  del shape[axis]
  ul = ex.ul[:axis] + ex.ul[axis + 1:]
  lr = ex.lr[:axis] + ex.lr[axis + 1:]
  return create(ul, lr, shape)


def index_for_reduction(index, axis):
  return drop_axis(index, axis)


def find_shape(extents):
  shape = np.max([ex.lr for ex in extents], axis=0)
  shape[shape == 0] = 1
  return tuple(int(s) for s in shape)


def is_complete(shape, slices):
  if len(shape) != len(slices):
    return False
  for dim, s in zip(shape, slices):
    if s.start > 0:
      return False
    if s.stop < dim:
      return False
  return True


def largest_dim_axis(shape, exclude_axes=None):
  largest_dim, largest_axis = 0, 0
  for i in range(len(shape)):
    if exclude_axes is not None and i in exclude_axes:
      continue
    if largest_dim < shape[i]:
      largest_dim, largest_axis = shape[i], i
  return largest_axis


def change_partition_axis(ex, axis):
  """Re-express a partition along another axis (extent.pyx:489-539)."""
  if axis < 0:
    axis += len(ex.array_shape)
  if len(ex.shape) == 1:
    if axis == 1:
      return create((0,), ex.array_shape, ex.array_shape)
    return ex
  old_axes = [i for i in range(len(ex.shape)) if ex.shape[i] != ex.array_shape[i]]
  if len(old_axes) > 1:
    raise NotImplementedError('change_partition_axis: block partition %s' % (ex,))
  if len(old_axes) == 0 or old_axes[0] == axis:
    return ex
  old = old_axes[0]
  ul, lr = list(ex.ul), list(ex.lr)
  ul[axis] = divup(ul[old] * ex.array_shape[axis], ex.array_shape[old])
  ul[old] = 0
  lr[axis] = divup(lr[old] * ex.array_shape[axis], ex.array_shape[old])
  lr[old] = ex.array_shape[old]
  return create(ul, lr, ex.array_shape)
