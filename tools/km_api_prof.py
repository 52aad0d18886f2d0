"""Dev tool (GPU box): host profile of the drop-in KMeans.fit loop
(examples/kmeans.py) at a small N, so that the per-iteration Python work --
the expression building, optimisation / plan replay, joins, gloms and
from_numpy -- dominates.  Prints cProfile's top functions by total and by
cumulative time, and the wall time per iteration of the API loop beside the
direct loop (workloads.kmeans_fit).
  python tools/km_api_prof.py [N] [iters]"""
import cProfile
import os
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spartan_amd  # noqa: E402
from spartan_amd import expr, workloads  # noqa: E402
from spartan_amd.array import distarray, extent as ext  # noqa: E402
from spartan_amd.examples.kmeans import KMeans  # noqa: E402


def main():
  N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
  iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
  K, D = 256, 128
  spartan_amd.initialize()
  X = expr.rand(N, D, dtype=np.float32, seed=21).force()
  c0 = distarray.glom_region(X, ext.create((0, 0), (K, D), X.shape)).astype(np.float64)
  KMeans(K, 2).fit(X, c0)
  workloads.kmeans_fit(X, K, 2, centers=c0)
  torch.cuda.synchronize()
  from spartan_amd.examples import kmeans as KM
  info = {}
  for name, fn in (('direct', lambda: workloads.kmeans_fit(X, K, iters, centers=c0, info=info)),
                   ('api', lambda: KMeans(K, iters).fit(X, c0))):
    before = dict(KM.SPEC_STATS)
    t = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    print('%s: %.3f ms per iteration; direct speculated %s respun %s; api %s' % (
        name, (time.perf_counter() - t) / iters * 1e3, info.get('speculated'), info.get('respun'),
        {k: KM.SPEC_STATS[k] - before[k] for k in before}))
  pr = cProfile.Profile()
  pr.enable()
  KMeans(K, iters).fit(X, c0)
  torch.cuda.synchronize()
  pr.disable()
  st = pstats.Stats(pr)
  st.sort_stats('tottime').print_stats(35)
  st.sort_stats('cumulative').print_stats(45)


if __name__ == '__main__':
  main()
