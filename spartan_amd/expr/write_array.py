"""Writes into arrays and host ingest (restates spartan/expr/write_array.py).

``write(array, src_slices, data, dst_slices)`` is ``array[src_slices] =
data[dst_slices]`` (write_array.py:72-90), in place like the reference's
(:1-8 note that it mutates).  The written region is merged into the target
tiles with the array's reducer (tile merge rule: the first write to an
element replaces, later writes reduce; tile.pyx:201-298):

  * ``data`` a NumPy array (or ``np.load(..., mmap_mode='r')`` memmap): each
    rank uploads only the pieces that land on its own tiles, through the
    pinned double-buffered staging pipeline of array/transfer.py;
  * ``data`` a DistArray / Expr: the source region is a zero-copy ``Slice``
    view of ``data`` and every target tile's piece is moved to the tile's
    owner by ONE ``gather_regions`` exchange (the reference fetches it per
    tile in ``_write_mapper``, :30-41), then merged on the device.

``from_numpy`` (:411-433) and ``from_file`` (.npy / .npz, dense; :380-409)
build on the same path.  Matrix Market / sparse inputs are out of scope
(sparse tiles are not on the MI355X path).
"""
import numpy as np

from .. import backend, runtime
from ..array import distarray, extent as ext
from ..array.views import Slice
from .base import Expr, Val, lazify


def from_numpy(a, tile_hint=None):
  """Upload a NumPy array into HBM tiles (each rank copies the tiles it owns)."""
  if not isinstance(a, np.ndarray):
    raise TypeError('Expected ndarray, got: %s' % type(a))
  return Val(val=distarray.from_numpy(a, tile_hint=tile_hint))


def from_file(fn, sparse=False, tile_hint=None):
  """Load a dense ``.npy`` / ``.npz`` file (write_array.py:380-409).

  ``.npy`` files are memory-mapped, so each rank reads only the pages of the
  tiles it owns; ``.npz`` members are read whole (the reference's ``arr_0``,
  or the single member).  Nothing is unpickled (``allow_pickle=False``)."""
  if sparse:
    raise NotImplementedError('sparse inputs are not on the MI355X path')
  if fn.endswith('.npy'):
    npa = np.load(fn, mmap_mode='r', allow_pickle=False)
  elif fn.endswith('.npz'):
    with np.load(fn, allow_pickle=False) as f:
      name = 'arr_0' if 'arr_0' in f.files else f.files[0]
      npa = f[name]
  else:
    raise NotImplementedError('Only .npy / .npz are supported, got %s' % fn)
  return from_numpy(npa, tile_hint)


def write_array(array, src_slices, data, dst_slices):
  """Eager body of WriteArrayExpr: merge data[dst_slices] into
  array[src_slices] in place and return ``array``."""
  sregion = ext.from_slice(src_slices, array.shape)
  if isinstance(data, (np.ndarray, np.generic)):
    data = np.asarray(data)
    if tuple(sregion.shape) != data.shape:
      data = data[dst_slices]
    array.update(sregion, data)
    return array
  if not isinstance(data, distarray.DistArray):
    raise TypeError('write: data must be an ndarray or a DistArray, got %s' % type(data))
  src = Slice(data, dst_slices)
  if tuple(src.shape) != tuple(sregion.shape):
    raise ValueError('write: region %s does not match source %s' % (sregion.shape, src.shape))
  ctx = runtime.get()
  requests, plan = [], []
  for ex, w in array.tiles.items():
    inter = ext.intersection(ex, sregion)
    if inter is None:
      continue
    ul = tuple(u - o for u, o in zip(inter.ul, sregion.ul))
    lr = tuple(l - o for l, o in zip(inter.lr, sregion.ul))
    requests.append((ext.create(ul, lr, src.shape), ctx.owner(w)))
    plan.append(inter)
  got = distarray.gather_regions(src, requests)
  aliased = _base(data) is array
  be = backend.get()
  pieces = {}
  for qi in got:
    piece = be.contiguous(got[qi])
    if aliased and piece.data_ptr() == got[qi].data_ptr():
      piece = piece.clone()  # source and target share tiles: snapshot before any merge writes
    pieces[qi] = piece
  for qi, piece in sorted(pieces.items()):
    array.update(plan[qi], piece)
  return array


def _base(a):
  while hasattr(a, 'base') and isinstance(getattr(a, 'base'), distarray.DistArray):
    a = a.base
  return a


class WriteArrayExpr(Expr):
  _members = ('array', 'data')

  def compute_shape(self):
    return self.array.shape

  def compute_dtype(self):
    return self.array.dtype

  def pretty_str(self):
    return 'WriteArrayExpr[%d] %s %s' % (self.expr_id, self.array, type(self.data).__name__)

  def _evaluate(self, deps):
    return write_array(deps['array'], self.src_slices, deps['data'], self.dst_slices)


def write(array, src_slices, data, dst_slices):
  """array[src_slices] = data[dst_slices] (write_array.py:72-90).

  ``array``: Expr or DistArray (mutated in place); ``data``: NumPy array,
  Expr or DistArray."""
  if not isinstance(data, (np.ndarray, np.generic)):
    data = lazify(data)
  e = WriteArrayExpr(array=lazify(array), data=data)
  e.src_slices = src_slices
  e.dst_slices = dst_slices
  return e
