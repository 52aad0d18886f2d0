"""Dev tool (GPU box): cProfile of the lreg iteration's host path at small N
(the kernel is ~us, so the profile is the host work).
  python tools/lreg_cprofile.py [N] [iters]"""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import spartan_amd  # noqa: E402
from spartan_amd import expr  # noqa: E402

spartan_amd.initialize()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 500
X = expr.lazify(expr.rand(n, 64, dtype=np.float32, seed=41).force())
Y = expr.lazify(expr.rand(n, 1, dtype=np.float32, seed=42).force())
w = np.random.default_rng(43).random((64, 1)).astype(np.float32)


def run(k, w):
  for _ in range(k):
    g = expr.sum(X * (expr.dot(X, w) - Y), axis=0)
    v = g.optimized().glom()
    w = w - v.reshape((64, 1)) * 1e-9
  return w


w = run(30, w)
pr = cProfile.Profile()
pr.enable()
run(iters, w)
pr.disable()
st = pstats.Stats(pr)
st.sort_stats('tottime').print_stats(35)
