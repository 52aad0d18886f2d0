"""Host overhead of one lreg iteration (cfg5 driver at a small N, so the
kernel is negligible): cProfile of workloads.sgd_train.  Dev tool:
  python tools/lreg_overhead.py [N] [iters]"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import spartan_amd  # noqa: E402
from spartan_amd import expr, workloads  # noqa: E402

spartan_amd.initialize()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 200
X = expr.lazify(expr.rand(n, 64, dtype=np.float32, seed=41).force())
Y = expr.lazify(expr.rand(n, 1, dtype=np.float32, seed=42).force())
w = np.random.default_rng(43).random((64, 1)).astype(np.float32)
workloads.sgd_train(X, Y, w, 1e-6, 5)
torch.cuda.synchronize()
t = time.perf_counter()
workloads.sgd_train(X, Y, w, 1e-6, iters)
torch.cuda.synchronize()
print('ms/iter %.3f' % ((time.perf_counter() - t) / iters * 1e3))
pr = cProfile.Profile()
pr.enable()
workloads.sgd_train(X, Y, w, 1e-6, iters)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(30)
