"""CPU restatement of Spartan's tile evaluation (ORACLE: test infrastructure).

Each function follows the reference's algorithm, tile by tile, with NumPy:

  tiling      distarray.good_tile_shape / compute_extents  (spartan/array/distarray.py:24-106)
  map         tile_mapper + FnCallExpr.evaluate             (spartan/expr/map.py:48-88,
                                                              spartan/expr/local.py:110-122):
              one NumPy ufunc per tree node, each materialising a temporary
  reduce      _reduce_mapper -> DistArray.update -> tile.merge
              (spartan/expr/reduce.py:19-68, distarray.py:370-421, tile.pyx:201-298):
              per-tile ``data.sum(axis)`` etc. merged into the output tiles,
              first write replaces, later writes apply accumulate_fn
  argmin/max  min -> _arg_mapper -> min  (spartan/expr/builtins.py:610-666)
  dot         map2 K-split (dot_map2_mapper, dot.py:195-212 + join_mapper
              map.py:285-330) for square/wide A, outer row-split
              (dot_outer_mapper dot.py:217-233, outer.py:14-61) for tall A,
              NumPy-operand GEMV (dot_map2_np_mapper dot.py:172-187)

Tiles are processed in tile order (the reference's arrival order is
nondeterministic; any fixed order is one of its legal outcomes).
"""
import itertools

import numpy as np


# ------------------------------------------------------------ extent math
def ext_create(ul, lr, array_shape):
  ul, lr = tuple(int(x) for x in ul), tuple(int(x) for x in lr)
  if any(u >= l for u, l in zip(ul, lr)):
    return None
  return (ul, lr, tuple(array_shape))


def ext_shape(ex):
  return tuple((l - u) or 1 for u, l in zip(ex[0], ex[1]))


def ext_slice(ex):
  return tuple(slice(u, l) for u, l in zip(ex[0], ex[1]))


def intersection(a, b):
  ul, lr = [], []
  for i in range(len(a[0])):
    if b[1][i] < a[0][i] or a[1][i] < b[0][i]:
      return None
    ul.append(max(a[0][i], b[0][i]))
    lr.append(min(a[1][i], b[1][i]))
  return ext_create(ul, lr, a[2])


def drop_axis(ex, axis):
  if axis is None:
    return ((), (), ())
  shape = list(ex[2])
  del shape[axis]
  return ext_create(ex[0][:axis] + ex[0][axis + 1:], ex[1][:axis] + ex[1][axis + 1:], shape)


def ravelled_pos(idx, shape):
  r, m = 0, 1
  for i in range(len(shape) - 1, -1, -1):
    r += m * int(idx[i])
    m *= int(shape[i])
  return r


def unravelled_pos(idx, shape):
  out = []
  idx = int(idx)
  for d in reversed(shape):
    out.append(idx % d)
    idx //= d
  return tuple(reversed(out))


def divup(a, b):
  return -(-int(a) // int(b))


def change_partition_axis(ex, axis):
  ul, lr, shp = ex
  if len(shp) == 1:
    return ext_create((0,), shp, shp) if axis == 1 else ex
  old = [i for i in range(len(shp)) if ((lr[i] - ul[i]) or 1) != shp[i]]
  if len(old) > 1:
    raise NotImplementedError
  if not old or old[0] == axis:
    return ex
  o = old[0]
  nul, nlr = list(ul), list(lr)
  nul[axis] = divup(ul[o] * shp[axis], shp[o])
  nul[o] = 0
  nlr[axis] = divup(lr[o] * shp[axis], shp[o])
  nlr[o] = shp[o]
  return ext_create(nul, nlr, shp)


def good_tile_shape(shape, num_shards):
  tile_size = int(np.prod(shape)) // num_shards
  ts = [1] * len(shape)
  idx = len(shape) - 1
  while tile_size > 1 and idx >= 0:
    ts[idx] = min(shape[idx], tile_size)
    tile_size //= shape[idx]
    idx -= 1
  return ts


def compute_extents(shape, num_workers, tile_hint=None):
  """[(extent, worker)] in itertools.product order."""
  if len(shape) == 0:
    return [(((), (), ()), 0)]
  hint = tile_hint or good_tile_shape(shape, num_workers)
  splits = [[(i, min(shape[d], i + hint[d])) for i in range(0, shape[d], hint[d])] for d in range(len(shape))]
  out = []
  for k, slc in enumerate(itertools.product(*splits)):
    ul, lr = zip(*slc)
    out.append((ext_create(ul, lr, shape), k % num_workers))
  return out


# ------------------------------------------------------------- tile store
class OArray:
  """An oracle DistArray: {extent: ndarray tile} plus the merge mask."""

  def __init__(self, shape, dtype, num_workers, tile_hint=None, reducer=None):
    self.shape, self.dtype, self.reducer = tuple(shape), np.dtype(dtype), reducer
    self.extents = compute_extents(self.shape, num_workers, tile_hint)
    self.data = {ex: None for ex, _ in self.extents}
    self.mask = {ex: np.zeros(ext_shape(ex) if ex[0] else (), dtype=bool) for ex, _ in self.extents}

  @classmethod
  def from_numpy(cls, arr, num_workers, tile_hint=None):
    a = cls(arr.shape, arr.dtype, num_workers, tile_hint)
    for ex, _ in a.extents:
      a.data[ex] = np.array(arr[ext_slice(ex)] if ex[0] else arr)
      a.mask[ex][...] = True
    return a

  def fetch(self, region):
    out = np.empty(ext_shape(region) if region[0] else (), dtype=self.dtype)
    if not region[0]:
      (ex, _), = self.extents
      return np.array(self.data[ex])
    for ex, _ in self.extents:
      inter = intersection(ex, region)
      if inter is None:
        continue
      src = tuple(slice(iu - eu, il - eu) for iu, il, eu in zip(inter[0], inter[1], ex[0]))
      dst = tuple(slice(iu - ru, il - ru) for iu, il, ru in zip(inter[0], inter[1], region[0]))
      out[dst] = self.data[ex][src]
    return out

  def update(self, region, upd):
    """DistArrayImpl.update -> tile.merge with this array's reducer."""
    for ex, _ in self.extents:
      if not region[0]:
        inter, sub_t, sub_u = ex, (), ()
      else:
        inter = intersection(ex, region)
        if inter is None:
          continue
        sub_t = tuple(slice(iu - eu, il - eu) for iu, il, eu in zip(inter[0], inter[1], ex[0]))
        sub_u = tuple(slice(iu - ru, il - ru) for iu, il, ru in zip(inter[0], inter[1], region[0]))
      piece = np.asarray(upd)[sub_u] if sub_u else np.asarray(upd)
      self._merge(ex, sub_t, piece)

  def _merge(self, ex, sub, upd):
    if self.data[ex] is None:
      self.data[ex] = np.zeros(ext_shape(ex) if ex[0] else (), dtype=self.dtype)
    t, m = self.data[ex], self.mask[ex]
    if t.ndim == 0:  # tile.pyx:213-218
      if not m[()] or self.reducer is None:
        self.data[ex] = np.asarray(upd).astype(self.dtype)
      else:
        self.data[ex] = np.asarray(self.reducer(t, upd)).astype(self.dtype)
      m[()] = True
      return
    if t.shape == np.shape(upd):  # full-tile fast path: only mask[0] is checked
      if self.reducer is not None and m.flat[0]:
        self.data[ex] = np.asarray(self.reducer(t, upd)).astype(self.dtype)
      else:
        self.data[ex] = np.asarray(upd).astype(self.dtype)
      m[...] = True
      return
    region = t[sub]
    msk = m[sub]
    upd = np.asarray(upd)
    region[~msk] = upd[~msk]
    if self.reducer is not None:
      region[msk] = self.reducer(region[msk], upd[msk])
    else:
      region[msk] = upd[msk]
    m[sub] = True

  def glom(self):
    if not self.shape:
      (ex, _), = self.extents
      return np.asarray(self.data[ex])
    out = np.empty(self.shape, dtype=self.dtype)
    for ex, _ in self.extents:
      out[ext_slice(ex)] = self.data[ex]
    return out


# ----------------------------------------------------------- evaluation
def map_tiles(fn, arrays, num_workers):
  """Reference tile_mapper: fn applied per tile of the largest input (NumPy
  broadcasting of smaller inputs, map.py:33-45)."""
  arrays = [np.asarray(a) for a in arrays]
  shape = np.broadcast_shapes(*[a.shape for a in arrays])
  big = max(range(len(arrays)), key=lambda i: arrays[i].size)
  drv = OArray(arrays[big].shape, arrays[big].dtype, num_workers)
  out = None
  for ex, _ in drv.extents:
    sl = ext_slice(ex) if ex[0] else ()
    local = []
    for a in arrays:
      if a.shape == shape:
        local.append(a[sl] if sl else a)
      else:  # Broadcast.fetch_base_tile: base region, NumPy broadcasts inside the tile
        pad = len(shape) - a.ndim
        bsl = tuple(slice(None) if a.shape[i] == 1 else sl[i + pad] for i in range(a.ndim))
        local.append(a[bsl] if a.ndim else a)
    r = np.asarray(fn(*local))
    if out is None:
      out = np.empty(shape, dtype=r.dtype)
    if sl:
      out[sl] = r
    else:
      out[...] = r
  return out


def reduce_tiles(arr, axis, local_fn, accumulate_fn, num_workers, out_dtype=None):
  """Reference ReduceExpr: per-tile local reduce merged into the output array."""
  arr = np.asarray(arr)
  dtype = np.dtype(out_dtype or arr.dtype)
  out_shape = () if axis is None else tuple(s for i, s in enumerate(arr.shape) if i != axis)
  out = OArray(out_shape, dtype, num_workers, reducer=accumulate_fn)
  src = OArray.from_numpy(arr, num_workers)
  for ex, _ in src.extents:
    part = np.asarray(local_fn(src.data[ex], axis))
    dst = drop_axis(ex, axis)
    out.update(dst, part.reshape(ext_shape(dst) if dst[0] else ()))
  return out.glom()


def sum_tiles(arr, axis, num_workers):
  return reduce_tiles(arr, axis, lambda d, ax: d.sum(ax), np.add, num_workers)


def max_tiles(arr, axis, num_workers):
  return reduce_tiles(arr, axis, lambda d, ax: d.max(ax), np.maximum, num_workers)


def min_tiles(arr, axis, num_workers):
  return reduce_tiles(arr, axis, lambda d, ax: d.min(ax), np.minimum, num_workers)


def arg_tiles(arr, axis, num_workers, kind='argmin'):
  """argmin / argmax exactly as builtins.py:610-666: m = min(x, axis) ->
  per-tile first match -> global index or sentinel prod(shape) -> min."""
  arr = np.asarray(arr)
  red = min_tiles if kind == 'argmin' else max_tiles
  m = red(arr, axis, num_workers)
  if axis is not None:
    m = m.reshape(tuple(1 if i == axis else s for i, s in enumerate(arr.shape)))
  src = OArray.from_numpy(arr, num_workers)
  idx_arr = np.empty(arr.shape, dtype=np.int64)
  sentinel = int(np.prod(arr.shape))
  for ex, _ in src.extents:
    a = src.data[ex]
    if axis is not None:
      msl = tuple(slice(None) if i == axis else slice(ex[0][i], ex[1][i]) for i in range(arr.ndim))
      b = m[msl]
    else:
      b = m
    c = np.zeros(a.shape)
    c[a == b] = 1
    mx = np.argmax(c, axis)
    if axis is not None:
      shp = list(a.shape)
      shp[axis] = 1
      gi = mx.reshape(shp) + ex[0][axis]
    else:
      exs = [((ex[1][i] - ex[0][i]) or 1) for i in range(arr.ndim)]
      loc = unravelled_pos(mx, exs)
      gi = ravelled_pos(np.asarray(ex[0]) + np.asarray(loc), exs)
    t = np.zeros(a.shape, dtype=np.int64) + gi
    t[a != b] = sentinel
    idx_arr[ext_slice(ex)] = t
  return min_tiles(idx_arr, axis, num_workers)


def dot_tiles(a, b, num_workers):
  """Reference dot: map2 K-split (square/wide A), outer (tall A), or NumPy operand."""
  a = np.asarray(a)
  b = np.asarray(b)
  if a.ndim == 1 and b.ndim == 1:
    out = OArray((1,), np.result_type(a, b), num_workers, reducer=np.add)
    src = OArray.from_numpy(a, num_workers)
    for ex, _ in src.extents:
      out.update(ext_create((0,), (1,), (1,)), np.asarray(src.data[ex].dot(b[ext_slice(ex)])).reshape(1))
    return out.glom()
  if a.ndim == 2 and b.ndim == 1:
    b2 = b.reshape(-1, 1)
    return dot_tiles(a, b2, num_workers).reshape(-1)
  M, K = a.shape
  N = b.shape[1]
  dt = np.result_type(a, b)
  out = OArray((M, N), dt, num_workers, tile_hint=(M, N), reducer=np.add)
  src = OArray.from_numpy(a, num_workers)
  if M > K:  # outer row-split over B column blocks
    bsrc = OArray.from_numpy(b, num_workers)
    for ex, _ in src.extents:
      fa = change_partition_axis(ex, 0)
      ta = a[ext_slice(fa)]
      done = set()
      for bex, _ in bsrc.extents:
        ob = change_partition_axis(bex, 1)
        if ob is None or ob in done:
          continue
        done.add(ob)
        tb = b[ext_slice(ob)]
        dst = ext_create((fa[0][0], ob[0][1]), (fa[1][0], ob[1][1]), (M, N))
        out.update(dst, ta.dot(tb))
    return out.glom()
  for ex, _ in src.extents:  # map2 join on axes (1, 0)
    fa = change_partition_axis(ex, 1)
    if fa is None:
      continue
    k0, k1 = fa[0][1], fa[1][1]
    part = a[ext_slice(fa)].dot(b[k0:k1, :])
    out.update(ext_create((0, 0), (fa[1][0], N), (M, N)), part)
  return out.glom()
