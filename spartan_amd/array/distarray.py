"""Distributed arrays whose tiles live in HBM, one process per GPU.

Restates the placement and data-access contract of spartan/array/distarray.py:
  * ``good_tile_shape`` / ``compute_splits`` / ``compute_extents`` (:24-106)
    with the reference's Python-2 integer division made explicit;
  * round-robin placement tile i -> worker i % num_workers (:438-442);
  * ``fetch`` / ``update`` / ``glom`` / ``tile_shape`` / ``real_size``.

SPMD rules: every rank holds the full ``tiles`` map (extent -> worker) and the
device data only for tiles whose worker it owns (``local``).  ``fetch`` and
``update`` act on local data; data of other ranks is moved by the collective
``gather_regions`` / ``glom`` that all ranks enter together.
"""
import itertools

import numpy as np

from .. import backend, comm, runtime
from ..util import prod
from . import extent as ext
from . import transfer
from .tile import Tile, merge, reducer_name

DEFAULT_TILE_SIZE = 100000


def good_tile_shape(shape, num_shards=-1):
  """Tile shape filled from the last axis (distarray.py:24-46, py2 int division)."""
  if num_shards != -1:
    tile_size = prod(shape) // num_shards
  else:
    tile_size = DEFAULT_TILE_SIZE
  tile_shape = [1] * len(shape)
  idx = len(shape) - 1
  while tile_size > 1 and idx >= 0:
    tile_shape[idx] = min(shape[idx], tile_size)
    tile_size //= shape[idx]
    idx -= 1
  return tile_shape


def compute_splits(shape, tile_hint):
  splits = []
  for dim in range(len(shape)):
    step = tile_hint[dim]
    splits.append([(i, min(shape[dim], i + step)) for i in range(0, shape[dim], step)])
  return splits


def compute_extents(shape, tile_hint=None, num_shards=-1):
  """{extent: worker} in itertools.product order (distarray.py:69-106)."""
  if len(shape) == 0:
    return {ext.create([], [], ()): 0}
  if any(int(d) == 0 for d in shape):
    # TileExtent has no empty extent (extent.pyx:141-153 returns None for ul >= lr)
    raise ValueError('zero-size arrays are not supported: shape %s' % (tuple(shape),))
  if tile_hint is None:
    tile_hint = good_tile_shape(shape, num_shards)
  else:
    assert len(tile_hint) == len(shape), (
        '#dimensions in tile hint does not match shape %s vs %s' % (tile_hint, shape))
  result = {}
  idx = 0
  for slc in itertools.product(*compute_splits(shape, tile_hint)):
    if num_shards != -1:
      idx = idx % num_shards
    ul, lr = zip(*slc)
    result[ext.create(ul, lr, shape)] = idx
    idx += 1
  return result


class DistArray:
  """Interface every array-like value of the expression layer provides."""
  sparse = False
  replicated = False

  @property
  def ndim(self):
    return len(self.shape)

  @property
  def size(self):
    return prod(self.shape)

  def real_size(self):
    return prod(self.shape)

  def __len__(self):
    return self.shape[0]

  def __repr__(self):
    return '%s(shape=%s, dtype=%s)' % (self.__class__.__name__, self.shape, self.dtype)

  def owner_of_region(self, region):
    """Rank that owns every tile overlapping ``region``, or None if several do."""
    ctx = runtime.get()
    owners = set()
    for ex, _ in ext.find_overlapping(self.tiles, region):
      owners.add(ctx.owner(self.tiles[ex]))
    return owners.pop() if len(owners) == 1 else None

  def select(self, idx):
    if isinstance(idx, ext.TileExtent):
      return glom_region(self, idx)
    if np.isscalar(idx):
      return self.select(slice(idx, idx + 1))[0]
    return glom_region(self, ext.from_slice(idx, self.shape))

  def __getitem__(self, idx):
    return self.select(idx)

  def glom(self):
    return glom(self)


class DistArrayImpl(DistArray):
  def __init__(self, shape, dtype, tiles, local, reducer_fn=None):
    self.shape = tuple(int(s) for s in shape)
    self.dtype = np.dtype(dtype)
    self.tiles = tiles            # {TileExtent: worker}, identical on every rank
    self.local = local            # {TileExtent: Tile} for tiles owned by this rank
    self.reducer_fn = reducer_fn
    self.bad_tiles = []

  def tile_shape(self):
    counts = {}
    for ex in self.tiles:
      counts[ex.shape] = counts.get(ex.shape, 0) + 1
    return sorted(counts.items(), key=lambda kv: (kv[1], kv[0]))[-1][0]

  def local_extents(self):
    return list(self.local.keys())

  def fetch(self, region):
    """Device tensor for ``region``; every overlapping tile must be local."""
    assert region.array_shape == self.shape or (region.ndim == 0 and self.shape == ()), (region, self.shape)
    t = self.local.get(region)
    if t is not None and tuple(t.ex.lr) == tuple(region.lr):
      return t.data
    pieces = list(ext.find_overlapping(self.tiles, region))
    if len(pieces) == 1:
      ex, inter = pieces[0]
      if ex not in self.local:
        raise RuntimeError('fetch of non-local region %s (rank %d); use gather_regions'
                           % (region, runtime.get().rank))
      return _sub_tensor(self.local[ex], inter)
    import torch
    be = backend.get()
    out = torch.empty(region.shape, dtype=backend.torch_dtype(self.dtype), device=runtime.get().device)
    for ex, inter in pieces:
      if ex not in self.local:
        raise RuntimeError('fetch of non-local region %s (rank %d); use gather_regions'
                           % (region, runtime.get().rank))
      tile = self.local[ex]
      be.copy_region(out, _rel(inter, region), tile.data, _rel(inter, ex), inter.shape)
    return out

  def update(self, region, data, reducer=None):
    """Merge ``data`` (device tensor or host array of region.shape) into the
    local tiles overlapping ``region`` with this array's reducer
    (DistArrayImpl.update, distarray.py:370-421)."""
    import torch
    ctx = runtime.get()
    op = reducer_name(reducer if reducer is not None else self.reducer_fn)
    if not isinstance(data, torch.Tensor):
      # host data: only the pieces that land on this rank's tiles cross PCIe
      host = np.asarray(data, dtype=self.dtype)
      assert host.shape == tuple(region.shape) or host.size == region.size, (host.shape, region)
      host = host.reshape(region.shape) if region.ndim else host.reshape(())
      for ex, inter in ext.find_overlapping(self.tiles, region):
        if ex in self.local:
          piece = host[_rel_slice(inter, region)] if region.ndim else host
          merge(self.local[ex], inter, transfer.upload(piece, ctx.device), op)
      return
    assert tuple(data.shape) == tuple(region.shape) or data.numel() == region.size, (data.shape, region)
    data = data.reshape(region.shape) if region.ndim else data.reshape(())
    be = backend.get()
    for ex, inter in ext.find_overlapping(self.tiles, region):
      if ex not in self.local:
        continue
      piece = data if inter == region and region.ndim else None
      if piece is None:
        if region.ndim == 0:
          piece = data
        else:
          piece = torch.empty(inter.shape, dtype=data.dtype, device=data.device)
          be.copy_region(piece, (0,) * inter.ndim, data, _rel(inter, region), inter.shape)
      merge(self.local[ex], inter, piece, op)

  def __setitem__(self, idx, value):
    region = ext.from_slice(idx, self.shape)
    if np.isscalar(value):
      value = np.full(region.shape, value, dtype=self.dtype)
    self.update(region, np.asarray(value))


class LocalWrapper(DistArray):
  """A host value (scalar or NumPy array) used in an array context
  (distarray.py:547-611).  Arrays are uploaded once to every rank's GPU and
  behave as a single replicated tile."""
  replicated = True

  def __init__(self, data):
    self._data = np.asarray(data)
    self._ex = ext.from_slice(np.index_exp[:], self._data.shape) if self._data.ndim else ext.create((), (), ())
    self._dev = None
    self.bad_tiles = []

  @property
  def dtype(self):
    return self._data.dtype

  @property
  def shape(self):
    return self._data.shape

  @property
  def tiles(self):
    return {self._ex: -1}

  @property
  def value(self):
    return self._data

  def device_data(self):
    if self._dev is None:
      import torch
      self._dev = transfer.upload(self._data, runtime.get().device)
    return self._dev

  def fetch(self, region):
    if region.ndim == 0 or tuple(region.ul) == (0,) * self.ndim and tuple(region.lr) == tuple(self.shape):
      return self.device_data()
    import torch
    out = torch.empty(region.shape, dtype=backend.torch_dtype(self.dtype), device=runtime.get().device)
    backend.get().copy_region(out, (0,) * region.ndim, self.device_data(), region.ul, region.shape)
    return out

  def owner_of_region(self, region):
    return runtime.get().rank  # replicated: always local

  def glom(self):
    return self._data


class ReplicatedArray(LocalWrapper):
  """A device array held in full by every rank (e.g. a map over a LocalWrapper)."""

  def __init__(self, dev_tensor):
    self._dev = dev_tensor
    self._shape = tuple(dev_tensor.shape)
    self._dtype = backend.np_dtype(dev_tensor.dtype)
    self._ex = ext.from_slice(np.index_exp[:], self._shape) if self._shape else ext.create((), (), ())
    self.bad_tiles = []

  @property
  def dtype(self):
    return self._dtype

  @property
  def shape(self):
    return self._shape

  def device_data(self):
    return self._dev

  @property
  def value(self):
    return self.glom()

  def glom(self):
    return transfer.download(self._dev)


def as_array(data):
  if isinstance(data, DistArray):
    return data
  return LocalWrapper(data)


def largest_value(vals):
  return max(vals, key=lambda v: v.real_size())


def create(shape, dtype=np.float64, reducer=None, tile_hint=None, sparse=False):
  """Empty DistArray with round-robin placement (distarray.py:423-483)."""
  if sparse:
    raise NotImplementedError('sparse tiles are out of scope for the MI355X backend')
  ctx = runtime.get()
  dtype = np.dtype(dtype)
  shape = tuple(int(s) for s in shape)
  extents = compute_extents(shape, tile_hint, ctx.num_workers)
  tiles, local = {}, {}
  tdt = backend.torch_dtype(dtype)
  for ex, w in extents.items():
    tiles[ex] = w
    if ctx.is_local(w):
      local[ex] = Tile.deferred(ex.shape if ex.ndim else (), tdt, ctx.device, ex)
  return DistArrayImpl(shape, dtype, tiles, local, reducer)


def from_tiles(shape, dtype, tiles, local_data, reducer=None):
  """DistArray from {extent: worker} and {extent: device tensor} (written tiles)."""
  local = {ex: Tile(t, ex, written=True) for ex, t in local_data.items()}
  return DistArrayImpl(shape, dtype, dict(tiles), local, reducer)


def from_numpy(arr, tile_hint=None):
  """Upload a host array; each rank copies its own tiles (write_array.py:411-433)."""
  arr = np.asarray(arr)
  backend.spx_dtype(arr.dtype)
  out = create(arr.shape, arr.dtype, tile_hint=tile_hint)
  dev = runtime.get().device
  for ex, tile in out.local.items():
    piece = arr[ex.to_slice()] if ex.ndim else arr
    tile.data = transfer.upload(piece, dev)
    tile.written = [ex]
  return out


# ---------------------------------------------------------------- movement
def _rel(inner, outer):
  return tuple(a - b for a, b in zip(inner.ul, outer.ul))


def _rel_slice(inner, outer):
  return tuple(slice(u - o, l - o) for u, l, o in zip(inner.ul, inner.lr, outer.ul))


def _sub_tensor(tile, region):
  """View or copy of ``region`` (inside the tile) as a contiguous tensor."""
  t_ex = tile.ex
  if region == t_ex and tuple(region.lr) == tuple(t_ex.lr):
    return tile.data
  rel = _rel(region, t_ex)
  shape = region.shape
  # a leading-dim range with every trailing dim whole is a contiguous view
  if all(rel[d] == 0 and shape[d] == tile.shape[d] for d in range(1, len(shape))):
    return tile.data.narrow(0, rel[0], shape[0])
  import torch
  out = torch.empty(shape, dtype=tile.data.dtype, device=tile.data.device)
  backend.get().copy_region(out, (0,) * len(shape), tile.data, rel, shape)
  return out


def gather_regions(array, requests):
  """Collective: deliver ``region`` of ``array`` to rank ``dst`` for every
  (region, dst) in ``requests`` (identical list on every rank).  Returns
  {request index: device tensor} for the requests addressed to this rank."""
  if hasattr(array, 'gather'):  # a view (array/views.py): the same exchange on its base
    return array.gather(requests)
  return _gather_plan(array, requests, False).finish()


class _Gather:
  """A gather in flight: ``finish`` makes the current stream wait for the
  messages, stitches the received pieces into their buffers and returns
  {request index: device tensor}."""

  def __init__(self, out, handle, post):
    self.out, self.handle, self.post = out, handle, post

  def finish(self):
    if self.handle is not None:
      comm.wait_all([self.handle])
      self.handle = None
    be = backend.get()
    for buf, rel, tmp, shape in self.post:
      be.copy_region(buf, rel, tmp, (0,) * len(shape), shape)
    self.post = []
    return self.out


def gather_regions_async(array, requests):
  """``gather_regions`` whose messages run beside the current stream
  (comm.exchange_async): returns a handle; its ``finish()`` (later, in the
  same order on every rank) yields the tensors.  Lets a caller start the next
  pieces' transfers while it computes on the pieces it already has (the
  overlapped K-split dot, expr/dot.py).  A received piece that covers whole
  rows of its request lands in the request's buffer directly (no staging
  copy)."""
  if hasattr(array, 'gather'):
    out = array.gather(requests)
    return _Gather(out, None, [])
  return _gather_plan(array, requests, True)


def _gather_plan(array, requests, asynchronous):
  import torch
  ctx = runtime.get()
  be = backend.get()
  out, sends, recvs, post = {}, [], [], []
  tdt = backend.torch_dtype(array.dtype)
  for qi, (region, dst) in enumerate(requests):
    if array.replicated:
      if dst == ctx.rank:
        out[qi] = array.fetch(region)
      continue
    if dst == ctx.rank and array.owner_of_region(region) == ctx.rank:
      out[qi] = array.fetch(region)  # all pieces local: a view when possible
      continue
    buf = None
    if dst == ctx.rank:
      buf = torch.empty(region.shape, dtype=tdt, device=ctx.device)
      out[qi] = buf
    for ex, inter in ext.find_overlapping(array.tiles, region):
      src = ctx.owner(array.tiles[ex])
      if src == ctx.rank and dst == ctx.rank:
        be.copy_region(buf, _rel(inter, region), array.local[ex].data, _rel(inter, ex), inter.shape)
      elif src == ctx.rank:
        sends.append((_sub_tensor(array.local[ex], inter).contiguous(), dst))
      elif dst == ctx.rank:
        rel = _rel(inter, region)
        if asynchronous and _whole_rows(rel, inter.shape, region.shape):
          # rows [r0, r1) of a row-major buffer: one contiguous slice, received in place
          recvs.append((buf.reshape(region.shape[0], -1)[rel[0]:rel[0] + inter.shape[0]], src))
          continue
        tmp = torch.empty(inter.shape, dtype=tdt, device=ctx.device)
        recvs.append((tmp, src))
        post.append((buf, rel, tmp, inter.shape))
  if asynchronous:
    return _Gather(out, comm.exchange_async(sends, recvs), post)
  comm.exchange(sends, recvs)
  return _Gather(out, None, post)


def _whole_rows(rel, shape, full):
  """True when a piece at offset ``rel`` (a tuple) of ``shape`` spans every
  trailing dim of the ``full`` buffer (so it is a contiguous row range)."""
  return len(full) >= 1 and tuple(shape[1:]) == tuple(full[1:]) and all(u == 0 for u in rel[1:])


def glom(array):
  """Collective: the whole array as a NumPy array on every rank."""
  if isinstance(array, LocalWrapper):
    return array.glom()
  ctx = runtime.get()
  result = np.empty(array.shape, dtype=array.dtype)
  if len(array.shape) == 0:
    (ex, w), = array.tiles.items()
    import torch
    owner = ctx.owner(w)
    t = array.local[ex].data if owner == ctx.rank else torch.empty((), dtype=backend.torch_dtype(array.dtype),
                                                                    device=ctx.device)
    comm.broadcast(t, owner)
    return np.asarray(t.cpu().numpy())
  import torch
  for ex, w in array.tiles.items():
    owner = ctx.owner(w)
    if owner == ctx.rank:
      t = array.local[ex].data
    else:
      t = torch.empty(ex.shape, dtype=backend.torch_dtype(array.dtype), device=ctx.device)
    if ctx.distributed:
      t = t.contiguous()
      comm.broadcast(t, owner)
    transfer.download(t, result[ex.to_slice()])
  return result


def glom_region(array, region):
  """Collective: ``region`` of ``array`` as a NumPy array on every rank; only
  the region's bytes move (one gather_regions exchange + one D2H copy)."""
  if isinstance(array, LocalWrapper) or region.ndim == 0:
    full = glom(array)
    return full[region.to_slice()] if region.ndim else full
  ctx = runtime.get()
  got = gather_regions(array, [(region, r) for r in range(ctx.world_size)])
  return transfer.download(got[ctx.rank]).reshape(region.shape)
