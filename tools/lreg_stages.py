"""Dev tool (GPU box): host time of one lreg iteration by stage at a small N
(kernel negligible): DAG build, optimized() (plan replay), evaluation +
glom.  python tools/lreg_stages.py [N] [iters]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import spartan_amd  # noqa: E402
from spartan_amd import expr  # noqa: E402

spartan_amd.initialize()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 500
X = expr.lazify(expr.rand(n, 64, dtype=np.float32, seed=41).force())
Y = expr.lazify(expr.rand(n, 1, dtype=np.float32, seed=42).force())
w = np.random.default_rng(43).random((64, 1)).astype(np.float32)
T = np.zeros(4)
for it in range(iters + 20):
  t0 = time.perf_counter()
  g = expr.sum(X * (expr.dot(X, w) - Y), axis=0)
  t1 = time.perf_counter()
  o = g.optimized()
  t2 = time.perf_counter()
  v = o.glom()
  t3 = time.perf_counter()
  w = w - v.reshape((64, 1)) * 1e-9
  t4 = time.perf_counter()
  if it >= 20:
    T += [t1 - t0, t2 - t1, t3 - t2, t4 - t3]
T /= iters
print('us/iter build %.1f optimize %.1f eval+glom %.1f update %.1f total %.1f' % tuple(list(T * 1e6) + [T.sum() * 1e6]))
import cProfile, pstats  # noqa: E402,E401
pr = cProfile.Profile()
pr.enable()
for it in range(200):
  g = expr.sum(X * (expr.dot(X, w) - Y), axis=0)
  v = g.optimized().glom()
pr.disable()
pstats.Stats(pr).sort_stats('cumtime').print_stats(45)
