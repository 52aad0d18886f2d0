"""Callers of the path: the reference's application drivers that BASELINE.json
configs exercise, restated on the spartan_amd.expr API.

linear_regression_update -- LinearRegression.update
  (spartan/examples/linear_regression.py:10-16) as driven by
  SGDRegressor.train (spartan/examples/sgd.py:34-39):
      yp   = dot(x, w)                 # w a host (d, 1) array
      diff = x * (yp - y)
      grad = sum(diff, axis=0).optimized().glom().reshape((d, 1))
      w    = w - grad * alpha          # host update
  Here ReduceMapFusion fuses ``x * (yp - y)`` into the axis-0 reduction and
  DotReduceFusion folds ``dot(x, w)`` into the same kernel as a per-row dot
  product (``rowdot``), so one generated kernel reads x and y once; the
  optimised plan is replayed across iterations (expr/plan_cache.py).  Across
  GPUs the (d,) partials are combined with one RCCL all-reduce (spx_allreduce).
"""
import os

import numpy as np

from . import expr


def linear_regression_update(x, y, w, alpha):
  """One gradient step; x (N, d), y (N, 1) arrays/exprs, w (d, 1) host array."""
  w = np.asarray(w)
  yp = expr.dot(x, w)
  diff = x * (yp - y)
  grad = expr.sum(diff, axis=0).optimized().glom().reshape((w.shape[0], 1))
  return w - grad * alpha


def sgd_train(x, y, w, alpha, iterations, device_w=True):
  """SGDRegressor.train (sgd.py:34-39): repeated full-batch updates.

  ``device_w`` (default): w stays on the GPU between iterations -- the same
  update ``w - grad * alpha`` in the same fp32 operations (bit-identical to
  the host form, linear_regression_update), but as a device map, so no
  iteration waits for a device-to-host copy of the gradient and the host
  builds iteration i + 1 while the GPU runs iteration i.  w comes back to
  the host once, at the end.  ``device_w=False``: the reference's form, one
  host round trip per iteration."""
  if not device_w:
    for _ in range(iterations):
      w = linear_regression_update(x, y, w, alpha)
    return w
  w = np.asarray(w)
  W = expr.from_numpy(w)
  for _ in range(iterations):
    W = expr.lazify(W)
    grad = expr.sum(x * (expr.dot(x, W) - y), axis=0)
    W = (W - expr.reshape(grad, w.shape) * alpha).optimized().force()
  return expr.glom(W)


_PINNED = {}


def _pinned_f64(n):
  """A pinned host fp64 buffer of >= n elements, kept across calls (a fresh
  pinned allocation inside a timed loop costs far more than the copies it
  serves; every copy into it is waited for before kmeans_fit returns)."""
  import torch
  buf = _PINNED.get('f64')
  if buf is None or buf.numel() < n:
    buf = _PINNED['f64'] = torch.empty((n,), dtype=torch.float64, pin_memory=True)
  return buf[:n]


def kmeans_fit(X, n_clusters, n_iter, centers=None, seed=0, info=None):
  """KMeans.fit, 'outer' implementation (spartan/examples/sklearn/cluster/
  k_means_.py:108-152), one fused pass pair per iteration on every rank:

    step        spx_kmeans_step: cdist + argmin(axis=1) with scipy's exact
                fp64 operation order -> bit-exact int64 labels, no (N, k)
                distance matrix is ever materialised (the reference's is
                N x k fp64 = 204.8 GB at cfg3), and the per-centre sums +
                counts of the local row strips -- one pass over the points
                for the rows the certified screen decides; one RCCL
                all-reduce of K*D + K values;
    host        empty-cluster reseed and centers = sums / counts (fp64).

  Divergences, documented in DESIGN.md: counts / centre sums are SUMMED over
  tiles (the reference's map2 without a reducer keeps the last tile's,
  SURVEY.md 3.4); empty clusters are reseeded from a seeded generator instead
  of the global np.random.

  X: (N, D) expression or DistArray (row strips).  centers: (K, D) host array
  or None (first K rows of X).  Returns (centers (K, D) fp64 host array,
  labels DistArray (N,) int64 tiled like X's rows).  ``info`` (a dict, optional)
  receives 'assign_centers': the (K, D) centres the returned labels were
  assigned against, and 'sums' / 'counts': that iteration's all-reduced
  per-centre sums and counts (bench.py's post-timing checks)."""
  import torch
  from . import backend, comm, runtime
  from .array import distarray, extent as ext
  ctx = runtime.get()
  be = backend.get()
  Xa = expr.force(X) if isinstance(X, expr.Expr) else X
  N, D = Xa.shape
  if centers is None:
    centers = distarray.glom_region(Xa, ext.create((0, 0), (n_clusters, D), (N, D)))
  centers = np.ascontiguousarray(np.asarray(centers, dtype=np.float64))
  K = centers.shape[0]
  rng = np.random.default_rng(seed)
  for ex in Xa.tiles:
    assert ex.ul[1] == 0 and ex.lr[1] == D, 'k-means needs row-strip tiles (k_means_.py:116)'
  label_tiles = {}

  def run_step(cdev):
    """One iteration's kernels on every local tile + the all-reduce, queued
    on the stream (no host wait): the (K D + K) sums | counts buffer."""
    # sums and counts share one buffer: one D2H per iteration
    buf = torch.empty((K * D + K,), dtype=torch.float64, device=ctx.device)
    sums = buf[:K * D].view(K, D)
    counts = buf[K * D:].view(torch.int64)
    first = True
    for ex, tile in Xa.local.items():
      lab = torch.empty((ex.shape[0],), dtype=torch.int64, device=ctx.device)
      # assignment + accumulation in one call: in the certified screen's
      # domain one pass over the tile labels and accumulates the decided rows
      be.kmeans_step(tile.data, cdev, lab, sums, counts, zero_first=first)
      first = False
      label_tiles[ex] = lab
    if first:  # no local tiles
      sums.zero_()
      counts.zero_()
    comm.all_reduce(sums, 'sum')
    comm.all_reduce(counts, 'sum')
    return buf

  # Speculation (SPARTAN_KMEANS_SPECULATE, default on): the next iteration is
  # queued with centres divided on the device BEFORE the host has looked at
  # this iteration's counts, so the GPU never idles on the host round trip
  # (~0.25 ms per cfg3 iteration).  The host then computes the centres
  # exactly as before (fp64 numpy, empty-cluster reseed) and keeps the queued
  # step only if no cluster was empty AND the device quotients are
  # bit-identical to its own (both are IEEE fp64 divisions; compared, not
  # assumed); otherwise it queues the step again with its own centres, which
  # overwrites the speculative results.  Returned values are those of the
  # sequential loop either way.
  spec = ctx.device.type == 'cuda' and os.environ.get('SPARTAN_KMEANS_SPECULATE', '1') != '0'
  host_t = _pinned_f64(2 * K * D + K) if spec else None
  if info is not None:
    info['speculated'] = 0
    info['respun'] = 0
  buf = run_step(torch.as_tensor(centers).to(ctx.device)) if n_iter > 0 else None
  for it in range(n_iter):
    if info is not None:
      info['assign_centers'] = centers
    more = it + 1 < n_iter
    if spec:
      host_t[:K * D + K].copy_(buf, non_blocking=True)
      nbuf = None
      if more:
        cnext = buf[:K * D].view(K, D) / buf[K * D:].view(torch.int64).to(torch.float64).view(K, 1)
        host_t[K * D + K:].copy_(cnext.view(-1), non_blocking=True)
      ev = torch.cuda.Event()
      ev.record()
      if more:
        nbuf = run_step(cnext)
      ev.synchronize()
      host = host_t.numpy()
    else:
      host = buf.cpu().numpy()
    c_host = host[K * D:K * D + K].view(np.int64)
    s_host = host[:K * D].reshape(K, D)
    if info is not None:
      info['sums'], info['counts'] = s_host.copy(), c_host.copy()
    empty = c_host == 0
    if np.any(empty):
      c_host = c_host.copy()
      s_host = s_host.copy()
      c_host[empty] = 1
      s_host[empty, :] = rng.standard_normal((int(empty.sum()), D))
    centers = s_host / c_host.reshape(K, 1)
    if more:
      if spec and not np.any(empty) and np.array_equal(
          centers.view(np.int64), host[K * D + K:].reshape(K, D).view(np.int64)):
        buf = nbuf
        if info is not None:
          info['speculated'] += 1
      else:
        if spec and info is not None:
          info['respun'] += 1
        buf = run_step(torch.as_tensor(centers).to(ctx.device))
  ltiles = {ext.create((ex.ul[0],), (ex.lr[0],), (N,)): w for ex, w in Xa.tiles.items()}
  llocal = {ext.create((ex.ul[0],), (ex.lr[0],), (N,)): t for ex, t in label_tiles.items()}
  labels = distarray.from_tiles((N,), np.int64, ltiles, llocal)
  return centers, labels
