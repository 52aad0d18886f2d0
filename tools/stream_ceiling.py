"""Dev tool (GPU box): the generated reduce kernels on cfg2-sized inputs with
less arithmetic (x*y+z, x+y+z, x) -- how close the exp variant is to the
streaming ceiling.  python tools/stream_ceiling.py"""
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
cases = [('x*y+exp(z)', lambda: X * Y + expr.exp(Z), 3), ('x*y+z', lambda: X * Y + Z, 3),
         ('x+y+z', lambda: X + Y + Z, 3), ('x', lambda: X, 1), ('x*y', lambda: X * Y, 2)]
for name, f, nin in (cases if os.environ.get("SC_REDUCE", "1") == "1" else []):
  for ax in (0, 1):
    for _ in range(2):
      expr.sum(f(), axis=ax).optimized().force()
    torch.cuda.synchronize()
    be.kernel_events = []
    for _ in range(10):
      expr.sum(f(), axis=ax).optimized().force()
    torch.cuda.synchronize()
    t = [s.elapsed_time(e) for n, s, e in be.kernel_events if n.startswith('spx_reduce')]
    be.kernel_events = None
    ms = float(np.median(t))
    print('%-12s axis %d  %.4f ms  %.1f GB/s' % (name, ax, ms, (nin * 4 * S * S + 4 * S) / ms / 1e6), flush=True)

# elementwise maps (read n_in streams, write one)
for name, f, nin in [('x*y+exp(z)', lambda: X * Y + expr.exp(Z), 3), ('x+1', lambda: X + 1.0, 1),
                     ('x*y', lambda: X * Y, 2)]:
  for _ in range(2):
    f().optimized().force()
  torch.cuda.synchronize()
  be.kernel_events = []
  for _ in range(10):
    f().optimized().force()
  torch.cuda.synchronize()
  t = [s.elapsed_time(e) for n, s, e in be.kernel_events if n.startswith('spx_map')]
  be.kernel_events = None
  ms = float(np.median(t))
  print('map %-12s %.4f ms  %.1f GB/s (read+write)' % (name, ms, ((nin + 1) * 4 * S * S) / ms / 1e6), flush=True)
print('map kernels:', [k[-1] for k in be._sig_fns if k[0] == 'map'])
