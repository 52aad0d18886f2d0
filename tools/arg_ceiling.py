"""Dev tool (GPU box): fused map + min / argmin / max reductions at cfg2
size next to sum (same streamed bytes).  python tools/arg_ceiling.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import spartan_amd  # noqa: E402
from spartan_amd import backend, expr  # noqa: E402

spartan_amd.initialize()
be = backend.get()
S = 32768
X, Y, Z = (expr.lazify(expr.rand(S, S, dtype=np.float32, seed=s).force()) for s in (11, 12, 13))
for name, fn in [('sum', expr.sum), ('min', expr.min), ('argmin', expr.argmin), ('argmax', expr.argmax)]:
  for ax in (0, 1):
    for _ in range(2):
      fn(X * Y + expr.exp(Z), axis=ax).optimized().force()
    torch.cuda.synchronize()
    be.kernel_events = []
    for _ in range(5):
      fn(X * Y + expr.exp(Z), axis=ax).optimized().force()
    torch.cuda.synchronize()
    t = [s.elapsed_time(e) for n, s, e in be.kernel_events if n.startswith('spx_reduce')]
    be.kernel_events = None
    ms = float(np.median(t))
    print('%-7s axis %d  %.4f ms  %.1f GB/s' % (name, ax, ms, 3 * 4 * S * S / ms / 1e6), flush=True)
