"""NumPy-style broadcasting of DistArrays (restates spartan/expr/broadcast.py).

A ``Broadcast`` is a view: it reports the broadcast shape and maps an extent of
that shape back to the region of its base array (``_base_ex``,
broadcast.py:69-88).  The generated kernels then broadcast inside the tile with
zero strides, the device analogue of the reference letting NumPy broadcast
``fetch_base_tile`` results (broadcast.py:104-109).
"""
from ..array import distarray, extent as ext
from ..util import prod


class Broadcast(distarray.DistArray):
  def __init__(self, base, shape):
    if isinstance(base, Broadcast):
      base = base.base
    self.base = base
    self.shape = tuple(shape)
    self.dtype = base.dtype
    self.bad_tiles = []
    self.prepend_dim = len(self.shape) - len(base.shape)

  @property
  def tiles(self):
    return self.base.tiles

  @property
  def replicated(self):
    return self.base.replicated

  def __repr__(self):
    return 'Broadcast(%s -> %s)' % (self.base, self.shape)

  def real_size(self):
    """Underlying size minus one: prefer real arrays as the driver (broadcast.py:54-59)."""
    return prod(self.base.shape) - 1

  def _base_ex(self, ex):
    while ex.ndim > len(self.base.shape):
      ex = ext.drop_axis(ex, 0)
    ul, lr = [], []
    for i, size in enumerate(self.base.shape):
      if size == 1:
        ul.append(0)
        lr.append(1)
      else:
        ul.append(ex.ul[i])
        lr.append(ex.lr[i])
    if not self.base.shape:
      return ext.create((), (), ())
    return ext.create(ul, lr, self.base.shape)

  def fetch_base_tile(self, ex):
    return self.base.fetch(self._base_ex(ex))

  def owner_of_region(self, region):
    return self.base.owner_of_region(self._base_ex(region))


def broadcast(args):
  """Lift every array to the common broadcast shape (broadcast.py:111-158)."""
  if len(args) == 1:
    return list(args)
  orig = [list(x.shape) for x in args]
  nd = max(len(s) for s in orig)
  new = [[1] * (nd - len(s)) + s for s in orig]
  for axis in range(nd):
    sizes = set(s[axis] for s in new)
    assert len(sizes) <= 2, 'Mismatched shapes for broadcast: %s' % orig
    if len(sizes) == 2:
      assert 1 in sizes, 'Mismatched shapes for broadcast: %s' % orig
    m = max(s[axis] for s in new)
    for s in new:
      s[axis] = m
  out = []
  for a, o, n in zip(args, orig, new):
    out.append(a if n == o else Broadcast(a, tuple(n)))
  return out
