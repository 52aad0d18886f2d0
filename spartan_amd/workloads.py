"""Callers of the path: the reference's application drivers that BASELINE.json
configs exercise, restated on the spartan_amd.expr API.

linear_regression_update -- LinearRegression.update
  (spartan/examples/linear_regression.py:10-16) as driven by
  SGDRegressor.train (spartan/examples/sgd.py:34-39):
      yp   = dot(x, w)                 # w a host (d, 1) array
      diff = x * (yp - y)
      grad = sum(diff, axis=0).optimized().glom().reshape((d, 1))
      w    = w - grad * alpha          # host update
  Here ``dot(x, w)`` is a skinny GEMV (generated multiply + packed row-sum) and
  ReduceMapFusion fuses ``x * (yp - y)`` into the axis-0 reduction: one
  generated kernel reading x once more.  Across GPUs the (d,) partials are
  combined with one RCCL all-reduce.
"""
import numpy as np

from . import expr


def linear_regression_update(x, y, w, alpha):
  """One gradient step; x (N, d), y (N, 1) arrays/exprs, w (d, 1) host array."""
  w = np.asarray(w)
  yp = expr.dot(x, w)
  diff = x * (yp - y)
  grad = expr.sum(diff, axis=0).optimized().glom().reshape((w.shape[0], 1))
  return w - grad * alpha


def sgd_train(x, y, w, alpha, iterations):
  """SGDRegressor.train (sgd.py:34-39): repeated full-batch updates."""
  for _ in range(iterations):
    w = linear_regression_update(x, y, w, alpha)
  return w
