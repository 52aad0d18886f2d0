"""Profile driver for cfg5 (lreg): python tools/lreg_prof.py [N] [iters]
Run under rocprofv3 --kernel-trace --stats to get the fused kernel's time."""
import os
import sys
import time

sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import spartan_amd  # noqa: E402
from spartan_amd import expr, workloads  # noqa: E402

spartan_amd.initialize()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000000
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
X = expr.lazify(expr.rand(n, 64, dtype=np.float32, seed=41).force())
Y = expr.lazify(expr.rand(n, 1, dtype=np.float32, seed=42).force())
w = np.random.default_rng(43).random((64, 1)).astype(np.float32)
workloads.sgd_train(X, Y, w, 1e-6, 2)
torch.cuda.synchronize()
t = time.perf_counter()
workloads.sgd_train(X, Y, w, 1e-6, iters)
torch.cuda.synchronize()
el = (time.perf_counter() - t) / iters
print('lreg ms/iter %.3f  GB/s %.1f' % (el * 1e3, (4.0 * n * 64 + 4.0 * n) / el / 1e9))
