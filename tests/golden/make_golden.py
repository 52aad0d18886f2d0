"""Generate the committed golden fixtures under tests/golden/ (run once, by hand):

    python tests/golden/make_golden.py

Every expected output is the ORACLE's (oracle/, the CPU restatement of the
reference's tile evaluation, itself pinned by the reference's own KATs in
tests/test_oracle.py / tests/test_extent.py), frozen here so that a change
in the oracle, in NumPy / SciPy, or in the counter-based generator shows up
as a diff against data instead of silently moving both sides of a parity
test.  k-means labels come from scipy's fp64 ``cdist`` + first-index argmin
(k_means_.py:52-58, builtins.py:631-647).

Inputs are stored when small; larger ones are regenerated from their seed by
oracle/rng.py and pinned by a SHA-256 of their bytes (``*_sha``).

Fixture families (SURVEY.md 8(c) "golden vectors"):
  cfg2.npz    x*y+exp(z) on (96,80) fp32 (inputs stored) and (257,131) fp32
              (seeds), W = 1/2/3/8 row strips: sum/min/max/argmin/argmax over
              None/0/1 (reduce.py:19-68, builtins.py:466-666)
  ties.npz    int64 / fp32 arrays full of ties: arg-reductions, W = 1/3/8
  dot.npz     (128,96).(96,80) fp32 + fp64 random, K-split over W = 4
              (dot.py:195-212); 2000^2 f64 ones identity (configs[0])
  kmeans.npz  2048 x 16 fp32 points with constructed near-ties, k = 8:
              first-iteration labels, centres after 3 iterations (W = 2)
  lreg.npz    10000 x 64 fp32 (seeds): gradient and w after 3 updates,
              W = 1 and 3 (linear_regression.py:10-16)
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import rng  # noqa: E402
from oracle import spartan_cpu as O  # noqa: E402
from oracle import workloads as OW  # noqa: E402

AXES = {'N': None, '0': 0, '1': 1}


def sha(a):
  return np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest(), dtype=np.uint8)


def cfg2_inputs(shape):
  return (rng.rand(shape, 11, np.float32), rng.rand(shape, 12, np.float32),
          rng.rand(shape, 13, np.float32, -1.0, 1.0))


def reductions(out, tag, m, workers):
  for W in workers:
    for an, ax in AXES.items():
      k = '%s_W%d_ax%s' % (tag, W, an)
      out['sum_' + k] = np.asarray(O.sum_tiles(m, ax, W))
      out['min_' + k] = np.asarray(O.min_tiles(m, ax, W))
      out['max_' + k] = np.asarray(O.max_tiles(m, ax, W))
      out['argmin_' + k] = np.asarray(O.arg_tiles(m, ax, W, 'argmin'))
      out['argmax_' + k] = np.asarray(O.arg_tiles(m, ax, W, 'argmax'))


def make_cfg2():
  out = {}
  for tag, shape, store in [('s', (96, 80), True), ('m', (257, 131), False)]:
    x, y, z = cfg2_inputs(shape)
    if store:
      out['x_' + tag], out['y_' + tag], out['z_' + tag] = x, y, z
    else:
      out['xyz_sha_' + tag] = sha(np.concatenate([x.ravel(), y.ravel(), z.ravel()]))
    m = O.map_tiles(lambda a, b, c: a * b + np.exp(c), [x, y, z], 1)
    reductions(out, tag, m, (1, 2, 3, 8))
  return out


def make_ties():
  g = np.random.default_rng(2024)
  out = {'i': g.integers(0, 4, (40, 30)).astype(np.int64),
         'f': g.integers(-3, 3, (33, 17)).astype(np.float32)}
  reductions(out, 'i', out['i'], (1, 3, 8))
  reductions(out, 'f', out['f'], (1, 3, 8))
  return out


def make_dot():
  out = {}
  for dt, tag in [(np.float32, 'f32'), (np.float64, 'f64')]:
    a = rng.rand((128, 96), 31, dt)
    b = rng.rand((96, 80), 32, dt)
    out['ab_sha_' + tag] = sha(np.concatenate([a.ravel(), b.ravel()]))
    out['c_' + tag] = O.dot_tiles(a, b, 4)
  # configs[0] identity: sum(dot(ones, ones)) over 2000^2 f64 = 2000 * 2000^2
  out['ones_sum'] = np.asarray(8e9)
  return out


def make_kmeans():
  g = np.random.default_rng(77)
  C = g.random((8, 16)).astype(np.float32)
  pts = (C[g.integers(0, 8, 2048)] + 0.15 * g.standard_normal((2048, 16))).astype(np.float32)
  # constructed near-ties: midpoints of centre pairs (equidistant up to the
  # fp32 rounding of the midpoint)
  for i in range(0, 2048, 16):
    a, b = g.integers(0, 8, 2)
    pts[i] = ((C[a].astype(np.float64) + C[b]) / 2).astype(np.float32)
  pts[5::64] = C[g.integers(0, 8, len(pts[5::64]))]  # points exactly on a centre
  centres0 = C.astype(np.float64)
  out = {'points': pts, 'centres0': centres0,
         'labels1': OW.kmeans_assign(pts, centres0)}
  c3, l3 = OW.kmeans_fit(pts, 8, 3, 2, centers=centres0)
  out['centres3'], out['labels3'] = c3, l3
  return out


def make_lreg():
  n, d = 10000, 64
  X = rng.rand((n, d), 41, np.float32)
  Y = rng.rand((n, 1), 42, np.float32)
  w0 = rng.rand((d, 1), 43, np.float32)
  out = {'xy_sha': sha(np.concatenate([X.ravel(), Y.ravel()])), 'w0': w0}
  for W in (1, 3):
    yp = np.empty((n, 1), np.float32)
    for ex, _ in O.compute_extents(X.shape, W):  # dot_map2_np_mapper GEMV per row strip
      rows = slice(ex[0][0], ex[1][0])
      yp[rows] = X[rows].dot(w0)
    diff = O.map_tiles(lambda x, a, b: x * (a - b), [X, yp, Y], W)
    out['grad_W%d' % W] = O.sum_tiles(diff, 0, W)
    w = w0
    for _ in range(3):
      w = OW.linear_regression_update(X, Y, w, 1e-6, W)
    out['w3_W%d' % W] = w
  return out


FAMILIES = {'cfg2': make_cfg2, 'ties': make_ties, 'dot': make_dot, 'kmeans': make_kmeans, 'lreg': make_lreg}


def main():
  for name, fn in FAMILIES.items():
    path = os.path.join(HERE, name + '.npz')
    np.savez_compressed(path, **fn())
    print('%-12s %8d bytes' % (name + '.npz', os.path.getsize(path)))


if __name__ == '__main__':
  main()
