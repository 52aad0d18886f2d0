"""Dev tool (GPU box): a full-grid cfg2-size map (x*y+exp(z)) checked
against torch on the device, timed with HIP events.  python tools/map_check.py"""
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
x, y, z = (expr.rand(S, S, dtype=np.float32, seed=s).force() for s in (11, 12, 13))
X, Y, Z = (expr.lazify(a) for a in (x, y, z))
out = (X * Y + expr.exp(Z)).force()
xt, yt, zt, ot = (next(iter(a.local.values())).data for a in (x, y, z, out))
ref = xt * yt + torch.exp(zt)
err = ((ot - ref).abs() / ref.abs()).max().item()
print('max rel err vs torch %.3g' % err, 'shape', tuple(ot.shape), flush=True)
assert err < 1e-6
for _ in range(2):
  (X * Y + expr.exp(Z)).force()
torch.cuda.synchronize()
be.kernel_events = []
outs = []
for _ in range(10):
  outs.append((X * Y + expr.exp(Z)).force())
torch.cuda.synchronize()
bad = [i for i, o in enumerate(outs) if not torch.equal(next(iter(o.local.values())).data, ot)]
print('calls differing from the first:', bad, flush=True)
t = [s.elapsed_time(e) for n, s, e in be.kernel_events if n.startswith('spx_map')]
print('map median %.4f ms  %.1f GB/s' % (np.median(t), 16 * S * S / np.median(t) / 1e6), flush=True)
