"""Dev tool (GPU box): cfg2 fused map+reduce kernel time per axis under the
dev knobs (SPX_REDUCE_BLOCKS target grid).  python tools/cfg2_knobs.py"""
import os
import sys

os.environ['SPX_REDUCE_PLANS'] = '0'  # the env knobs are read per call
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import spartan_amd  # noqa: E402
from spartan_amd import backend, expr  # noqa: E402

spartan_amd.initialize()
be = backend.get()
S = 32768
X, Y, Z = (expr.lazify(expr.rand(S, S, dtype=np.float32, seed=s).force()) for s in (11, 12, 13))
for blocks in os.environ.get('KNOB_BLOCKS', '512,1024,2048').split(','):
  os.environ['SPX_ROWS_GRID'] = os.environ.get('KNOB_ROWS', '0')
  os.environ['SPX_REDUCE_BLOCKS'] = blocks
  for ax in (0, 1):
    for _ in range(2):
      expr.sum(X * Y + expr.exp(Z), axis=ax).optimized().force()
    torch.cuda.synchronize()
    be.kernel_events = []
    for _ in range(10):
      expr.sum(X * Y + expr.exp(Z), axis=ax).optimized().force()
    torch.cuda.synchronize()
    t = [s.elapsed_time(e) for n, s, e in be.kernel_events if n.startswith('spx_reduce')]
    be.kernel_events = None
    ms = float(np.median(t))
    print('blocks %6s axis %d  %.4f ms  %.1f GB/s' % (blocks, ax, ms, (3 * 4 * S * S + 4 * S) / ms / 1e6), flush=True)
