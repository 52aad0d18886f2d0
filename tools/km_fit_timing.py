"""Dev tool (GPU box): workloads.kmeans_fit at the cfg3 shape as bench.py's
k-means leg runs it (first K points, 2 iterations after a 1-iteration
warm-up), with the number of fused-step launches and the wall time.
  python tools/km_fit_timing.py [N] [iters] [module of spartan_amd with a previous kmeans_fit, timed first]
(Round 4: a one-iteration-ahead loop with device-divided centres measured
18.6-18.8 ms against the sequential loop's 18.5-18.6 on one box -- the host
update between iterations costs the GPU ~nothing outside a profiler; the
~1 ms gaps of a rocprofv3 trace are the profiler's.)"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spartan_amd import backend, expr, runtime, workloads  # noqa: E402


def main():
  N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
  iters = int(sys.argv[2]) if len(sys.argv) > 2 else 2
  runtime.initialize()
  be = backend.get()
  calls = [0]
  orig = be.kmeans_step

  def counted(*a, **k):
    calls[0] += 1
    return orig(*a, **k)
  be.kmeans_step = counted
  X = expr.rand(N, 128, dtype=np.float32, seed=21).force()
  workloads.kmeans_fit(X, 256, 1)
  torch.cuda.synchronize()
  old = None
  if len(sys.argv) > 3:  # a module of the package holding a previous kmeans_fit, timed first
    import importlib
    old = importlib.import_module('spartan_amd.' + sys.argv[3])
    old.kmeans_fit(X, 256, iters)
    torch.cuda.synchronize()
    for rep in range(3):
      t0 = time.perf_counter()
      old.kmeans_fit(X, 256, iters)
      torch.cuda.synchronize()
      print('old rep %d: %.3f ms per iteration' % (rep, (time.perf_counter() - t0) * 1e3 / iters), flush=True)
  workloads.kmeans_fit(X, 256, iters)
  torch.cuda.synchronize()
  for rep in range(3):
    calls[0] = 0
    t0 = time.perf_counter()
    workloads.kmeans_fit(X, 256, iters)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print('rep %d: %.3f ms per iteration, %d fused-step launches for %d iterations' %
          (rep, el * 1e3 / iters, calls[0], iters), flush=True)


if __name__ == '__main__':
  main()
