"""Dev tool (GPU box): where the drop-in KMeans.fit loop (examples/kmeans.py)
spends the time between two fused steps at the cfg3 shape.  Wraps
HipBackend.kmeans_step to record torch events just before and after each
launch (GPU timeline) and host perf_counter stamps at the launch and at each
glom's return; prints per iteration: the step's GPU time, the GPU time from
one step's end to the next one's start, and the host time from the centres
glom's return to the next step's launch.
  python tools/km_api_gaps.py [N] [iters]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spartan_amd  # noqa: E402
from spartan_amd import backend, expr  # noqa: E402
from spartan_amd.array import distarray, extent as ext  # noqa: E402
from spartan_amd.expr import base as ebase  # noqa: E402
from spartan_amd.examples.kmeans import KMeans  # noqa: E402


def main():
  N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
  iters = int(sys.argv[2]) if len(sys.argv) > 2 else 6
  K, D = 256, 128
  spartan_amd.initialize()
  be = backend.get()
  X = expr.rand(N, D, dtype=np.float32, seed=21).force()
  c0 = distarray.glom_region(X, ext.create((0, 0), (K, D), X.shape)).astype(np.float64)
  KMeans(K, 1).fit(X, c0)
  torch.cuda.synchronize()
  rec = []
  orig = type(be).kmeans_step

  def step(self, *a, **kw):
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t = time.perf_counter()
    e0.record()
    r = orig(self, *a, **kw)
    e1.record()
    rec.append(('step', t, time.perf_counter(), e0, e1))
    return r

  oglom = ebase.Expr.glom

  def glom(self, *a, **kw):
    r = oglom(self, *a, **kw)
    rec.append(('glom', time.perf_counter()))
    return r

  type(be).kmeans_step = step
  ebase.Expr.glom = glom
  t0 = time.perf_counter()
  KMeans(K, iters).fit(X, c0)
  torch.cuda.synchronize()
  wall = (time.perf_counter() - t0) / iters
  type(be).kmeans_step = orig
  ebase.Expr.glom = oglom
  steps = [r for r in rec if r[0] == 'step']
  print('N=%d iters=%d: %.3f ms per iteration wall' % (N, iters, wall * 1e3))
  for i, s in enumerate(steps):
    gpu = s[3].elapsed_time(s[4])
    line = 'iter %d: step %.3f ms (launch call %.3f ms host)' % (i, gpu, (s[2] - s[1]) * 1e3)
    if i > 0:
      p = steps[i - 1]
      line += '; GPU end(i-1) -> start(i) %.3f ms' % p[4].elapsed_time(s[3])
      # host: the last glom before this step returned -> this step's launch
      gl = [r[1] for r in rec if r[0] == 'glom' and p[2] < r[1] < s[1]]
      if gl:
        line += '; host: first glom return -> launch %.3f ms, last glom return -> launch %.3f ms' % (
            (s[1] - gl[0]) * 1e3, (s[1] - gl[-1]) * 1e3)
    print(line, flush=True)


if __name__ == '__main__':
  main()
