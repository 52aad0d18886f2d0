"""Oracle restatements of the application drivers (test infrastructure).

linear_regression_update: spartan/examples/linear_regression.py:10-16 with
the reference's tile evaluation -- dot_map2_np_mapper GEMV per row strip
(spartan/expr/dot.py:172-187), the broadcast map x * (yp - y), and the
axis-0 reduce merged at the owner tiles (spartan/expr/reduce.py:19-68).
"""
import numpy as np

from . import spartan_cpu as O


def linear_regression_update(X, Y, w, alpha, num_workers):
  X = np.asarray(X)
  w = np.asarray(w)
  yp = np.empty((X.shape[0], w.shape[1]), dtype=np.result_type(X, w))
  for ex, _ in O.compute_extents(X.shape, num_workers):
    rows = slice(ex[0][0], ex[1][0])
    cols = slice(ex[0][1], ex[1][1])
    yp[rows] = X[rows, cols].dot(w[cols])  # one tile: all columns (row strips)
  diff = O.map_tiles(lambda x, a, b: x * (a - b), [X, yp, Y], num_workers)
  grad = O.sum_tiles(diff, 0, num_workers).reshape((w.shape[0], 1))
  return w - grad * alpha


def kmeans_assign(points, centers):
  """distances = cdist(points, centers) (k_means_.py:52-58, fp64) ->
  argmin(axis=1), first occurrence (builtins.py:631-647)."""
  from scipy.spatial.distance import cdist
  return cdist(np.asarray(points), np.asarray(centers)).argmin(axis=1).astype(np.int64)


def kmeans_fit(X, n_clusters, n_iter, num_workers, centers=None, seed=0):
  """KMeans.fit 'outer' (k_means_.py:108-152) with the reference's per-tile
  mappers: cdist + argmin per row strip, np.bincount (kmeans_count_mapper
  :61-64) and per-centre fp32 ``points[matching].sum(axis=0)``
  (kmeans_center_mapper :67-89) -- SUMMED across tiles (the reference's
  reducer-less map2 keeps the last tile's), empty clusters
  reseeded from np.random.default_rng(seed) like the build."""
  X = np.asarray(X)
  N, D = X.shape
  centers = np.asarray(X[:n_clusters] if centers is None else centers, dtype=np.float64)
  K = centers.shape[0]
  rng = np.random.default_rng(seed)
  labels = None
  for _ in range(n_iter):
    labels = np.empty(N, np.int64)
    counts = np.zeros(K, np.int64)
    sums = np.zeros((K, D))
    for ex, _w in O.compute_extents(X.shape, num_workers):
      rows = slice(ex[0][0], ex[1][0])
      pts = X[rows]
      lab = kmeans_assign(pts, centers)
      labels[rows] = lab
      counts += np.bincount(lab, minlength=K)
      for i in range(K):
        sums[i] += pts[lab == i].sum(axis=0)
    empty = counts == 0
    if np.any(empty):
      counts[empty] = 1
      sums[empty, :] = rng.standard_normal((int(empty.sum()), D))
    centers = sums / counts.reshape(K, 1)
  return centers, labels
