"""Dev tool (GPU box): host timeline of one steady-state iteration of the
drop-in KMeans.fit loop (examples/kmeans.py) at the cfg3 shape -- every
wrapped call's start / end relative to the previous fused step's launch.
  python tools/km_api_timeline.py [N] [iters]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spartan_amd  # noqa: E402
from spartan_amd import backend, expr  # noqa: E402
from spartan_amd.array import distarray, extent as ext, transfer  # noqa: E402
from spartan_amd.expr import base as ebase, join as ejoin  # noqa: E402
from spartan_amd.examples import kmeans as km  # noqa: E402

REC = []


def wrap(obj, name, label):
  orig = getattr(obj, name)

  def f(*a, **kw):
    t = time.perf_counter()
    r = orig(*a, **kw)
    REC.append((label, t, time.perf_counter()))
    return r
  setattr(obj, name, f)


def main():
  N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
  iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
  K, D = 256, 128
  spartan_amd.initialize()
  be = backend.get()
  X = expr.rand(N, D, dtype=np.float32, seed=21).force()
  c0 = distarray.glom_region(X, ext.create((0, 0), (K, D), X.shape)).astype(np.float64)
  km.KMeans(K, 3).fit(X, c0)
  torch.cuda.synchronize()
  for obj, name, label in ((type(be), 'kmeans_step', 'kmeans_step'), (ebase.Expr, 'glom', 'glom'),
                           (ebase.Expr, 'optimized', 'optimized'), (expr, 'from_numpy', 'from_numpy'),
                           (expr, 'outer', 'outer'), (expr, 'argmin', 'argmin'), (expr, 'map2', 'map2'),
                           (km, '_replicated_f64', '_replicated_f64'), (km, '_row_blocks', '_row_blocks'),
                           (km, '_assign_fused', '_assign_fused'), (km, '_center_join', '_center_join'),
                           (km, '_count_join', '_count_join'), (ejoin, '_scatter_updates', '_scatter_updates'),
                           (transfer, 'download', 'download'), (transfer, 'upload', 'upload'),
                           (km, '_step_domain', '_step_domain'), (km, '_take_step', '_take_step'),
                           (km, '_deliver_full', '_deliver_full'), (torch, 'empty', 'torch.empty')):
    wrap(obj, name, label)
  # the registered join functions were bound at import: re-register the wrapped ones
  ejoin.register_join(km.kmeans_count_mapper, km._count_join)
  ejoin.register_join(km.kmeans_center_mapper, km._center_join)
  ejoin.register_argmin_fusion(km.kmeans_dist_mapper, km._assign_fused, dtypes=(np.float64, np.float32))
  t0 = time.perf_counter()
  km.KMeans(K, iters).fit(X, c0)
  torch.cuda.synchronize()
  print('wall per iteration %.3f ms' % ((time.perf_counter() - t0) / iters * 1e3))
  steps = [r for r in REC if r[0] == 'kmeans_step']
  for i in range(1, len(steps)):
    a, b = steps[i - 1][2], steps[i][2]
    print('--- iteration %d (times in ms after the previous step launch returned)' % i)
    for lab, s, e in sorted((r for r in REC if a <= r[1] <= b), key=lambda r: r[1]):
      print('  %-18s %8.3f -> %8.3f  (%.3f)' % (lab, (s - a) * 1e3, (e - a) * 1e3, (e - s) * 1e3))


if __name__ == '__main__':
  main()
