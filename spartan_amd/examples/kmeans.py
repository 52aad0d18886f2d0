"""The reference's k-means driver, runnable unmodified on the MI355X path
(spartan/examples/sklearn/cluster/k_means_.py).

``KMeans.fit(X, centers, implementation='outer')`` is the reference's loop
(k_means_.py:108-152) written against ``expr.outer`` / ``expr.argmin`` /
``expr.map2`` with the reference's three mapper functions.  Those mappers
are registered joins (expr/join.py), so each runs as device work:

  kmeans_dist_mapper    outer((X, C), (0, 0))  -> spx_cdist: exact-order fp64
                        distances (N, K), rounded to the target dtype;
  argmin(outer(...), axis=1)                   -> fused by OuterArgminFusion
                        (expr/optimize.py) into spx_kmeans_assign for fp64
                        or fp32 distances (the argmin of the values rounded to
                        the target dtype): certified bf16x3-MFMA filter +
                        exact recompute, no (N, K) matrix (102-205 GB at cfg3);
                        in spx_kmeans_step's domain the fused step, whose
                        centre sums / counts the two joins below then take
                        (one pass over X per iteration);
  kmeans_count_mapper   map2(labels, 0)        -> spx_bincount per label tile
                        + RCCL all-reduce;
  kmeans_center_mapper  map2((X, labels), (0, 0)) -> spx_kmeans_accumulate
                        per-centre fp64 sums + RCCL all-reduce.

The mapper bodies below are the host meaning of each join (the reference's
NumPy code, restated); they are never called on the product path.

Divergence kept from workloads.kmeans_fit: counts and
centre sums are SUMMED over tiles, where the reference's reducer-less map2
keeps the last tile's; empty clusters are reseeded from a
seeded generator instead of the global ``np.random``.
"""
import numpy as np

from .. import backend, comm, expr, runtime
from ..array import distarray, extent as ext
from ..expr.join import register_argmin_fusion, register_join


# ------------------------------------------------------ the three mappers
def kmeans_dist_mapper(ex_a, tile_a, ex_b, tile_b):
  """k_means_.py:52-58: cdist of a point tile against a centre tile."""
  from scipy.spatial.distance import cdist
  target_ex = ext.create((ex_a.ul[0], ex_b.ul[0]), (ex_a.lr[0], ex_b.lr[0]),
                         (ex_a.array_shape[0], ex_b.array_shape[0]))
  yield target_ex, cdist(tile_a, tile_b)


def kmeans_count_mapper(extents, tiles, centers_count):
  """k_means_.py:61-64: np.bincount of a label tile."""
  target_ex = ext.create((0,), (centers_count,), (centers_count,))
  yield target_ex, np.bincount(tiles[0].astype(np.int64), minlength=centers_count)


def kmeans_center_mapper(extents, tiles, centers_count):
  """k_means_.py:67-89: per-centre sums of the points carrying each label."""
  points, labels = tiles
  target_ex = ext.create((0, 0), (centers_count, points.shape[1]), (centers_count, points.shape[1]))
  new_centers = np.zeros((centers_count, points.shape[1]))
  for i in range(centers_count):
    new_centers[i] = points[labels == i].sum(axis=0)
  yield target_ex, new_centers


# -------------------------------------------------------- device joins
def _replicated_f64(array):
  """The whole ``array`` as a contiguous fp64 tensor on every rank (collective)."""
  ctx = runtime.get()
  full = ext.from_shape(array.shape)
  got = distarray.gather_regions(array, [(full, r) for r in range(ctx.world_size)])
  return backend.get().contiguous(got[ctx.rank], np.float64)


# X's row blocks for the joins, kept across iterations at world size 1 (an
# iterative driver passes the same forced X every time; with more ranks the
# gather is a collective every rank must enter, so nothing is cached): valid
# while X lives (a weak reference) and every local tile tensor is the same
# object -- the rows are views of the tiles.  One entry.
_ROWS = {}


def _row_blocks(X, ncols):
  """[(owner rank, row extent over all columns)] of X's row blocks, and
  {index: device tensor} of the local ones (gathered when X is column-split)."""
  import weakref
  ctx = runtime.get()
  local = getattr(X, 'local', None)
  stamp = None
  if ctx.world_size == 1 and isinstance(local, dict) and not getattr(X, 'replicated', False):
    stamp = (ncols,) + tuple((tuple(ex.ul), id(t._data)) for ex, t in local.items())
    hit = _ROWS.get('x')
    if hit is not None and hit[0]() is X and hit[1] == stamp:
      return hit[2], hit[3]
  rows = sorted({(ex.ul[0], ex.lr[0]): w for ex, w in X.tiles.items()}.items())
  blocks = [(ctx.owner(w) if w != -1 else ctx.rank,
             ext.create((r0, 0), (r1, ncols), X.shape) if len(X.shape) == 2 else ext.create((r0,), (r1,), X.shape))
            for (r0, r1), w in rows]
  got = distarray.gather_regions(X, [(region, dst) for dst, region in blocks])
  _ROWS.clear()
  if stamp is not None:
    try:
      ref = weakref.ref(X, lambda _r: _ROWS.clear())
    except TypeError:
      ref = None
    if ref is not None:
      _ROWS['x'] = (ref, stamp, blocks, got)
  return blocks, got


def _deliver_full(target, full):
  """Copy a full-size tensor, identical on every rank, into target's local
  tiles; a local tile that IS the whole array and was never written adopts
  the tensor instead (no copy: the join made it for this target alone)."""
  from ..expr.engine import _copy_out
  be = backend.get()
  if len(target.local) == 1:
    (d, t), = target.local.items()
    if (not t.written and tuple(d.ul) == (0,) * len(target.shape) and tuple(d.shape) == tuple(target.shape)
        and tuple(full.shape) == tuple(d.shape) and full.dtype == backend.torch_dtype(target.dtype)
        and full.is_contiguous()):
      t.data = full
      t.written = [d]
      return
  for d, t in target.local.items():
    _copy_out(be, t, full, d)


def _dist_join(kind, arrays, axes, fn_kw, target):
  import torch
  from ..expr.join import _scatter_updates
  if kind != 'outer' or tuple(axes) != (0, 0) or len(arrays[0].shape) != 2:
    raise NotImplementedError('kmeans_dist_mapper: outer((X, C), (0, 0)) over a 2-d X only')
  X, C = arrays
  ctx = runtime.get()
  be = backend.get()
  c = _replicated_f64(C)
  K, D = c.shape
  blocks, got = _row_blocks(X, D)
  updates = []
  for qi, (src, region) in enumerate(blocks):
    tex = ext.create((region.ul[0], 0), (region.lr[0], K), target.shape)
    t = None
    if src == ctx.rank:
      pts = got[qi]
      if pts.stride(-1) != 1:
        pts = be.contiguous(pts)
      t = torch.empty(tex.shape, dtype=backend.torch_dtype(target.dtype), device=ctx.device)
      be.cdist(pts, c, t)
    updates.append((qi, tex, src, t))
  _scatter_updates(target, updates)


def _count_join(kind, arrays, axes, fn_kw, target):
  import torch
  ctx = runtime.get()
  be = backend.get()
  K = int(fn_kw['centers_count'])
  labels = arrays[0]
  pre = _take_step(_STEP.get('X'), labels, K, 'counts')
  if pre is not None:
    comm.all_reduce(pre, 'sum')
    _deliver_full(target, pre)
    _DT['cdt'] = np.dtype(target.dtype)
    _early_shadow('counts', target)
    _RED.clear()
    if len(target.local) == 1:  # the counts as the host will read them, for _speculate
      (_ex, tile), = target.local.items()
      _RED.update(labels=labels, counts=tile.data)
    return
  counts = torch.zeros((K,), dtype=torch.int64, device=ctx.device)
  for ex, tile in labels.local.items():
    lab = be.contiguous(tile.data, np.int64).reshape(-1)
    be.bincount(lab, counts, zero_first=False)
  comm.all_reduce(counts, 'sum')
  _deliver_full(target, counts)


def _center_join(kind, arrays, axes, fn_kw, target):
  import torch
  ctx = runtime.get()
  be = backend.get()
  K = int(fn_kw['centers_count'])
  X, labels = arrays
  D = X.shape[1]
  pre = _take_step(X, labels, K, 'sums')
  if pre is not None:  # the fused step of this labels array already summed X
    comm.all_reduce(pre, 'sum')
    _deliver_full(target, pre)
    _DT['sdt'] = np.dtype(target.dtype)
    _early_shadow('sums', target)
    if _NEXT['on'] and not _SPEC:  # (not queued early, _speculate_early)
      _speculate(X, labels, K, target)
    return
  sums = torch.zeros((K, D), dtype=torch.float64, device=ctx.device)
  counts = torch.zeros((K,), dtype=torch.int64, device=ctx.device)
  blocks, got = _row_blocks(X, D)
  lab_blocks = distarray.gather_regions(labels, [(ext.create((r.ul[0],), (r.lr[0],), labels.shape)
                                                  if len(labels.shape) == 1 else
                                                  ext.create((r.ul[0], 0), (r.lr[0], labels.shape[1]), labels.shape),
                                                  dst) for dst, r in blocks])
  for qi, (src, region) in enumerate(blocks):
    if src != ctx.rank:
      continue
    pts = got[qi]
    if pts.stride(-1) != 1:
      pts = be.contiguous(pts)
    lab = be.contiguous(lab_blocks[qi], np.int64).reshape(-1)
    be.kmeans_accumulate(pts, lab, sums, counts, zero_first=False)
  comm.all_reduce(sums, 'sum')
  _deliver_full(target, sums)


# The last fused assignment's per-rank centre sums and counts (one entry):
# argmin(outer(X, C)) runs spx_kmeans_step, which produces the iteration's
# sums and counts from the same single pass over X, and the centre / count
# joins of THAT labels array over THAT X take them instead of reading X again.
_STEP = {}


def _step_domain(X, K):
  """True where spx_kmeans_step fuses (fp32 rows of 64 / 128 dims, K <= 256,
  row-strip tiles): decided from global metadata, so every rank agrees."""
  return (np.dtype(X.dtype) == np.float32 and len(X.shape) == 2 and X.shape[1] in (64, 128) and K <= 256
          and all(ex.ul[1] == 0 and ex.lr[1] == X.shape[1] for ex in X.tiles))


def _assign_fused(arrays, fn_kw, target, dist_dtype):
  """argmin(outer((X, C), (0, 0), kmeans_dist_mapper), axis=1): the outer's
  target holds the cdist values rounded to its dtype (fp64, or fp32 for fp32
  points: map2 / outer dtype None -> arrays[0].dtype); spx_kmeans_assign per
  X row block gives the argmin of exactly those values (first index on
  ties, first NaN wins) without materialising them.  In spx_kmeans_step's
  domain the same labels come from the fused step, which also leaves this
  rank's centre sums and counts in _STEP for _center_join / _count_join."""
  import torch
  from ..expr.join import _scatter_updates
  X, C = arrays
  ctx = runtime.get()
  be = backend.get()
  c = _replicated_f64(C)
  K, D = c.shape
  blocks, got = _row_blocks(X, D)
  fused = _step_domain(X, K)
  spec = _take_spec(X, K, c, dist_dtype) if fused else None
  _STEP.clear()
  if fused:  # the first local block's step writes them (zero_first), the others add
    sums = torch.empty((K, D), dtype=torch.float64, device=ctx.device)
    counts = torch.empty((K,), dtype=torch.int64, device=ctx.device)
    first = True
  updates = []
  for qi, (src, region) in enumerate(blocks):
    tex = ext.create((region.ul[0],), (region.lr[0],), target.shape)
    lab = None
    if src == ctx.rank:
      pts = got[qi]
      if pts.stride(-1) != 1:
        pts = be.contiguous(pts)
      if spec is not None:  # the step queued for these very centres (_speculate)
        lab = spec['labs'][qi]
        first = False
      elif fused:
        lab = torch.empty((tex.shape[0],), dtype=torch.int64, device=ctx.device)
        be.kmeans_step(pts, c, lab, sums, counts, zero_first=first, dist_dtype=dist_dtype)
        first = False
      else:
        lab = torch.empty((tex.shape[0],), dtype=torch.int64, device=ctx.device)
      if not fused:
        be.kmeans_assign(pts, c, lab, dist_dtype=dist_dtype)
    updates.append((qi, tex, src, lab))
  _scatter_updates(target, updates)
  if fused:
    if spec is not None:
      sums, counts = spec['sums'], spec['counts']
    elif first:  # no local row block on this rank
      sums.zero_()
      counts.zero_()
    _STEP.update(labels=target, X=X, K=K, sums=sums, counts=counts, dd=dist_dtype)
    _EARLY.clear()
    if spec is not None and _spec_on():
      # (the loop's last iteration queues nothing, but still stages the
      # copies: its gloms and the upload of the final centres then need no
      # round trip of their own)
      _speculate_early(X, K, sums, counts, dist_dtype, queue=_NEXT['on'])


# Speculation (world size 1; SPARTAN_KMEANS_SPECULATE, default on).  The
# reference's loop reads the counts and the centre sums back to the host,
# divides there and uploads the new centres (k_means_.py:140-150): the GPU
# idles for that round trip and for the building of the next iteration's
# expressions.  While KMeans.fit has an iteration to go (_NEXT), the centre
# join, once the sums are all-reduced and delivered, (1) computes the next
# centres on the device exactly as the host will (the sums and counts rounded
# to the joins' target dtypes, divided in NumPy's result dtype), (2) copies
# the delivered sums to pinned memory and attaches that copy as the host
# shadow of the target tile (array/transfer.py), so the host's glom does not
# wait behind (3), the next fused step queued on the same stream with those
# centres.  The next fused assignment adopts that step's labels, sums and
# counts only if ITS centres are bit-identical to the queued ones (compared
# on the device); an empty cluster (reseeded on the host) or any other
# centres run the step as usual, after the queued one.  Results are those of
# the sequential loop.  (A side stream cannot overlap: k_kmeans_pp holds every
# CU's register file and LDS, so any other kernel -- the runtime's copy
# kernels too -- waits for it.)
_RED = {}           # the last fused step's all-reduced counts (from _count_join)
_DT = {}            # the dtypes the count / centre joins delivered in (the host reads them so)
_EARLY = {}         # host copies staged by _speculate_early for this iteration's joins
_SPEC = {}          # the queued step (one entry)
_NEXT = {'on': False}
_PIN = {}           # pinned staging for the shadows
SPEC_STATS = {'queued': 0, 'adopted': 0, 'dropped': 0}


def _spec_on():
  import os
  ctx = runtime.get()
  return (ctx.world_size == 1 and ctx.device.type == 'cuda'
          and os.environ.get('SPARTAN_KMEANS_SPECULATE', '1') != '0')


def _pinned(key, shape, tdt):
  import torch
  hp = _PIN.get(key)
  if hp is None or tuple(hp.shape) != tuple(shape) or hp.dtype != tdt:
    hp = _PIN[key] = torch.empty(tuple(shape), dtype=tdt, pin_memory=True)
  return hp


def _queue(X, K, cn, dd):
  """Queue the fused step of X for centres cn (device fp64) on the current
  stream: labels, sums, counts in fresh buffers, recorded in _SPEC."""
  import torch
  ctx = runtime.get()
  be = backend.get()
  D = X.shape[1]
  blocks, got = _row_blocks(X, D)
  s2 = torch.empty((K, D), dtype=torch.float64, device=ctx.device)
  c2 = torch.empty((K,), dtype=torch.int64, device=ctx.device)
  labs = {}
  first = True
  for qi, (src, _r) in enumerate(blocks):
    if src != ctx.rank:
      continue
    pts = got[qi]
    if pts.stride(-1) != 1:
      pts = be.contiguous(pts)
    lab = torch.empty((pts.shape[0],), dtype=torch.int64, device=ctx.device)
    be.kmeans_step(pts, cn, lab, s2, c2, zero_first=first, dist_dtype=dd)
    first = False
    labs[qi] = lab
  if first:
    s2.zero_()
    c2.zero_()
  _SPEC.update(X=X, K=K, dd=dd, cn=cn, labs=labs, sums=s2, counts=c2)
  SPEC_STATS['queued'] += 1


def _speculate(X, labels, K, target):
  """At the centre join (no step queued yet: the loop's first iteration, or
  after a dropped one): queue the next step behind a pinned copy of the sums
  the host is about to glom (a host shadow of the target tile)."""
  import torch
  _SPEC.clear()
  if not _spec_on() or _RED.get('labels') is not labels or _STEP.get('labels') is not labels \
      or len(target.local) != 1:
    return
  from ..array import transfer
  counts = _RED.pop('counts')
  (_ex, tile), = target.local.items()
  tt = tile.data  # the centre sums as the host will read them (the target's dtype)
  if tuple(tt.shape) != (K, X.shape[1]) or tuple(counts.shape) != (K,):
    return
  rdt = backend.torch_dtype(np.result_type(backend.np_dtype(tt.dtype), backend.np_dtype(counts.dtype)))
  cn = (tt.to(rdt) / counts.to(rdt).view(K, 1)).to(torch.float64)
  hp = _pinned('sums', tt.shape, tt.dtype)
  hp.copy_(tt, non_blocking=True)
  # the centres the host will compute, to host too: its from_numpy of them
  # then takes cn itself instead of a synchronous upload queued behind the
  # step (transfer.register_upload_alias; bit-identical or not taken)
  hc = _pinned('cn', cn.shape, torch.float64)
  hc.copy_(cn, non_blocking=True)
  ev = torch.cuda.Event()
  ev.record()
  transfer.attach_shadow(tt, hp.numpy(), ev)
  transfer.register_upload_alias(hc.numpy(), cn, ev)
  _queue(X, K, cn, _STEP.get('dd'))


def _speculate_early(X, K, sums, counts, dd, queue=True):
  """At the adoption of a queued step (world size 1: its sums and counts ARE
  the values this iteration's joins deliver): queue the step after it right
  away, computing its centres as the host will (the joins' target dtypes of
  the last iteration, NumPy's result dtype), and stage pinned copies of what
  the host will glom -- the counts, the sums in the centre target's dtype --
  and of those centres, all before the step, so that neither the gloms nor
  the upload of the centres wait behind it.  The joins attach the copies as
  host shadows of their target tiles (_EARLY)."""
  import torch
  from ..array import transfer
  sdt, cdt = _DT.get('sdt'), _DT.get('cdt')
  if sdt is None or cdt is None:
    return
  tdt = backend.torch_dtype
  rdt = tdt(np.result_type(sdt, cdt))
  st = sums.to(tdt(sdt))
  ct = counts.to(tdt(cdt))
  cn = (st.to(rdt) / ct.to(rdt).view(K, 1)).to(torch.float64)
  hs = _pinned('e_sums', st.shape, st.dtype)
  hk = _pinned('e_counts', ct.shape, ct.dtype)
  hc = _pinned('cn', cn.shape, torch.float64)
  hs.copy_(st, non_blocking=True)
  hk.copy_(ct, non_blocking=True)
  hc.copy_(cn, non_blocking=True)
  ev = torch.cuda.Event()
  ev.record()
  _EARLY.clear()
  _EARLY.update(sums=(hs.numpy(), ev, sdt), counts=(hk.numpy(), ev, cdt))
  transfer.register_upload_alias(hc.numpy(), cn, ev)
  if queue:
    _queue(X, K, cn, dd)


def _early_shadow(what, target):
  """Attach the early-staged host copy of ``what`` to target's tile (if the
  dtype and shape match what was staged)."""
  from ..array import transfer
  e = _EARLY.pop(what, None)
  if e is None or len(target.local) != 1:
    return
  host, ev, dt = e
  (_ex, tile), = target.local.items()
  tt = tile.data
  if np.dtype(target.dtype) == dt and tuple(tt.shape) == tuple(host.shape):
    transfer.attach_shadow(tt, host, ev)


def _take_spec(X, K, c, dist_dtype):
  """The queued step if it ran for exactly these centres (bit for bit), X, K
  and distance dtype, else None."""
  import torch
  sp = dict(_SPEC)
  _SPEC.clear()
  if not sp:
    return None
  # (the comparison's host sync waits for the queued step: the GPU is busy)
  if not (sp['X'] is X and sp['K'] == K and sp['dd'] == dist_dtype and tuple(c.shape) == tuple(sp['cn'].shape)
          and torch.equal(c.contiguous().view(torch.int64), sp['cn'].view(torch.int64))):
    SPEC_STATS['dropped'] += 1
    return None
  SPEC_STATS['adopted'] += 1
  return sp


def _take_step(X, labels, K, what):
  """This rank's fused sums / counts for (X, labels), once each, or None."""
  if _STEP.get('labels') is labels and _STEP.get('X') is X and _STEP.get('K') == K and what in _STEP:
    return _STEP.pop(what)
  return None


register_join(kmeans_dist_mapper, _dist_join)
register_argmin_fusion(kmeans_dist_mapper, _assign_fused, dtypes=(np.float64, np.float32))
register_join(kmeans_count_mapper, _count_join)
register_join(kmeans_center_mapper, _center_join)


# --------------------------------------------------------------- KMeans
class KMeans(object):
  """k_means_.py:90-152."""

  def __init__(self, n_clusters=8, n_iter=100, seed=0):
    self.n_clusters = n_clusters
    self.n_iter = n_iter
    self.seed = seed

  def fit(self, X, centers=None, implementation='outer'):
    """X: (N, D) array tiled by rows; centers: (K, D) host array / Expr, or
    None (``expr.rand``).  Returns (centers (K, D) host fp64, labels)."""
    if implementation == 'broadcast':
      return self._fit_broadcast(X, centers)
    if implementation != 'outer':
      raise NotImplementedError('implementation %r: "outer" (default) and "broadcast" are on the path'
                                % implementation)
    num_dim = X.shape[1]
    rng = np.random.default_rng(self.seed)
    labels = expr.zeros((X.shape[0], 1), dtype=np.int64)
    if centers is None:
      centers = expr.rand(self.n_clusters, num_dim)
    elif isinstance(centers, np.ndarray):
      centers = expr.from_numpy(centers)
    for i in range(self.n_iter):
      self.assign_centers_ = centers  # the centres this iteration's labels are assigned against
      distances = expr.outer((X, centers), (0, 0), fn=kmeans_dist_mapper,
                             shape=(X.shape[0], centers.shape[0]))
      labels = expr.argmin(distances, axis=1)
      counts = expr.map2(labels, 0, fn=kmeans_count_mapper, fn_kw={'centers_count': self.n_clusters},
                         shape=(centers.shape[0],))
      new_centers = expr.map2((X, labels), (0, 0), fn=kmeans_center_mapper,
                              fn_kw={'centers_count': self.n_clusters},
                              shape=(centers.shape[0], centers.shape[1]))
      # (another iteration follows: the centre join may queue it, _speculate)
      _NEXT['on'] = i + 1 < self.n_iter
      try:
        counts = counts.optimized().glom()
        centers = new_centers.optimized().glom()
      finally:
        _NEXT['on'] = False
      zcount_indices = (counts == 0).reshape(self.n_clusters)
      if np.any(zcount_indices):
        n_points = np.count_nonzero(zcount_indices)
        counts[zcount_indices] = 1
        centers[zcount_indices, :] = rng.standard_normal((n_points, num_dim))
      centers = centers / counts.reshape(centers.shape[0], 1)
      centers = expr.from_numpy(centers)
    return centers.glom(), labels

  def _fit_broadcast(self, X, centers):
    """k_means_.py:153-187: the same iteration written with broadcasting
    only -- (N, 1, D) - (1, K, D) squared and summed over the last axis (one
    fused map+reduce over the (N, K, D) iteration space, never
    materialised), argmin, one-hot matches by ``==`` against an arange,
    counts and centre sums as axis-0 reductions of broadcast products.  The
    distances are squared sums in the points' dtype (no sqrt, no fp64
    cdist), so near-tie labels follow this float order, as in the reference."""
    num_dim = X.shape[1]
    rng = np.random.default_rng(self.seed)
    if centers is None:
      centers = expr.rand(self.n_clusters, num_dim)
    elif isinstance(centers, np.ndarray):
      centers = expr.from_numpy(centers)
    labels = None
    for i in range(self.n_iter):
      X_broadcast = expr.reshape(X, (X.shape[0], 1, X.shape[1]))
      centers_broadcast = expr.reshape(centers, (1, centers.shape[0], centers.shape[1]))
      distances = expr.sum(expr.square(X_broadcast - centers_broadcast), axis=2)
      labels = expr.argmin(distances, axis=1)
      center_idx = expr.arange((1, centers.shape[0]))
      matches = expr.reshape(labels, (labels.shape[0], 1)) == center_idx
      matches = matches.astype(np.int64)
      counts = expr.sum(matches, axis=0)
      centers = expr.sum(X_broadcast * expr.reshape(matches, (matches.shape[0], matches.shape[1], 1)), axis=0)
      counts = counts.optimized().glom()
      centers = centers.optimized().glom()
      zcount_indices = (counts == 0).reshape(self.n_clusters)
      if np.any(zcount_indices):
        n_points = np.count_nonzero(zcount_indices)
        counts[zcount_indices] = 1
        centers[zcount_indices, :] = rng.standard_normal((n_points, num_dim))
      centers = centers / counts.reshape(centers.shape[0], 1)
      centers = expr.from_numpy(centers)
    return centers.glom(), labels
