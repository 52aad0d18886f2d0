"""Dev tool (GPU box): wall time inside one lreg iteration's evaluation by
function (wrappers with perf_counter, no profiler), small N.
  python tools/lreg_stages2.py [N] [iters]"""
import collections
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import spartan_amd  # noqa: E402
from spartan_amd import backend, expr  # noqa: E402
from spartan_amd.expr import engine, plan_cache  # noqa: E402
from spartan_amd.array import distarray, transfer  # noqa: E402

spartan_amd.initialize()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 500
T = collections.Counter()


def wrap(mod, name, label=None):
  f = getattr(mod, name)

  def g(*a, **k):
    t = time.perf_counter()
    try:
      return f(*a, **k)
    finally:
      T[label or name] += time.perf_counter() - t
  setattr(mod, name, g)


be = backend.get()
for nm in ['bind', 'fetch_inputs', 'combine_partials', 'driving_tiles', 'materialise_pres']:
  wrap(engine, nm)
wrap(plan_cache, 'signature')
wrap(plan_cache, '_instantiate')
wrap(distarray, 'create', 'distarray.create')
wrap(transfer, 'upload', 'transfer.upload')
wrap(transfer, 'download', 'transfer.download')
wrap(be, 'reduce', 'backend.reduce')
wrap(be, 'launch', 'backend.launch')
X = expr.lazify(expr.rand(n, 64, dtype=np.float32, seed=41).force())
Y = expr.lazify(expr.rand(n, 1, dtype=np.float32, seed=42).force())
w = np.random.default_rng(43).random((64, 1)).astype(np.float32)
tot = 0.0
for it in range(iters + 20):
  if it == 20:
    T.clear()
    tot = 0.0
  t0 = time.perf_counter()
  g = expr.sum(X * (expr.dot(X, w) - Y), axis=0)
  t1 = time.perf_counter()
  o = g.optimized()
  t2 = time.perf_counter()
  v = o.glom()
  t3 = time.perf_counter()
  T['build'] += t1 - t0
  T['optimize'] += t2 - t1
  T['eval+glom'] += t3 - t2
  tot += t3 - t0
  w = w - v.reshape((64, 1)) * 1e-9
for k, v in sorted(T.items(), key=lambda kv: -kv[1]):
  print('%-20s %8.1f us' % (k, v / iters * 1e6))
print('total %.1f us' % (tot / iters * 1e6))
