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
