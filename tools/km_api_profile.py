"""Dev tool (GPU box): host overhead of the drop-in KMeans.fit loop
(examples/kmeans.py) at the cfg3 shape -- wall time per iteration against
spx_kmeans_step's own HIP-event time, then a cProfile of a second fit.
  python tools/km_api_profile.py [N] [iters]"""
import cProfile
import os
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spartan_amd  # noqa: E402
from spartan_amd import backend, expr  # noqa: E402
from spartan_amd.array import distarray, extent as ext  # noqa: E402
from spartan_amd.examples.kmeans import KMeans  # noqa: E402


def main():
  N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
  iters = int(sys.argv[2]) if len(sys.argv) > 2 else 4
  K, D = 256, 128
  spartan_amd.initialize()
  be = backend.get()
  X = expr.rand(N, D, dtype=np.float32, seed=21).force()
  c0 = distarray.glom_region(X, ext.create((0, 0), (K, D), X.shape)).astype(np.float64)
  KMeans(K, 1).fit(X, c0)
  torch.cuda.synchronize()
  be.kmeans_timing(True)
  t0 = time.perf_counter()
  KMeans(K, iters).fit(X, c0)
  torch.cuda.synchronize()
  el = (time.perf_counter() - t0) / iters
  kt = be.kmeans_times()
  be.kmeans_timing(False)
  steps = [b for _, b in kt]
  print('N=%d: %.3f ms per iteration wall; spx_kmeans_step %s ms; wall - step = %.3f ms' % (
      N, el * 1e3, ['%.3f' % b for b in steps], el * 1e3 - float(np.mean(steps))), flush=True)
  pr = cProfile.Profile()
  pr.enable()
  KMeans(K, iters).fit(X, c0)
  torch.cuda.synchronize()
  pr.disable()
  st = pstats.Stats(pr)
  st.sort_stats('cumulative').print_stats(40)
  st.sort_stats('tottime').print_stats(25)


if __name__ == '__main__':
  main()
