"""Dev tool (GPU box): dense map kernels at 2^30 fp32 by vectors per lane
(backend.MAP_UNROLL: grid = n / (256 x 4 x U), all loads first); kernel
time by HIP events (backend.kernel_events), ROUNDS alternations; results
compared bit for bit with U = 1.
  python tools/map_sweep.py [S] [EVALS] [ROUNDS]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spartan_amd  # noqa: E402
from spartan_amd import backend, expr  # noqa: E402


def main():
  S = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
  evals = int(sys.argv[2]) if len(sys.argv) > 2 else 10
  rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
  spartan_amd.initialize()
  x = expr.rand(S, S, dtype=np.float32, seed=11).force()
  y = expr.rand(S, S, dtype=np.float32, seed=12).force()
  z = expr.rand(S, S, dtype=np.float32, seed=13, low=-1.0, high=1.0).force()
  X, Y, Z = expr.lazify(x), expr.lazify(y), expr.lazify(z)
  be = backend.get()
  maps = {'x*y+exp(z)': (lambda: X * Y + expr.exp(Z), 16), 'x*y': (lambda: X * Y, 12), 'x+1': (lambda: X + 1.0, 8)}
  unrolls = (1, 2, 4, 8)
  res = {(m, u): [] for m in maps for u in unrolls}
  real = backend.MAP_UNROLL
  from spartan_amd.expr import plan_cache
  from spartan_amd.array import distarray, extent as ext
  ref = {}
  for r in range(rounds):
    for m, (f, per) in maps.items():
      for u in unrolls:
        backend.MAP_UNROLL = u
        be._sig_fns.clear()
        plan_cache.clear()
        out = f().optimized().force()
        reg = ext.create((S // 2, 0), (S // 2 + 4, S), (S, S))
        g = distarray.glom_region(out, reg)
        del out
        if m not in ref:
          ref[m] = g
        same = bool(np.array_equal(g, ref[m]))
        torch.cuda.synchronize()
        be.kernel_events = []
        for _ in range(evals):
          o = f().optimized().force()
          del o
        torch.cuda.synchronize()
        ks = [s.elapsed_time(e) for (n, s, e) in be.kernel_events if n.startswith('spx_map')]
        be.kernel_events = None
        ms = float(np.mean(ks))
        res[(m, u)].append(ms)
        print('round %d %-11s U=%d: kernel %.4f ms = %.3f of 8 TB/s  same=%s' % (
            r, m, u, ms, per * S * S / (ms * 1e-3) / 8e12, same), flush=True)
  backend.MAP_UNROLL = real
  for m, (f, per) in maps.items():
    for u in unrolls:
      b = min(res[(m, u)])
      print('  %-11s U=%d  best %.4f ms  %.3f of 8 TB/s' % (m, u, b, per * S * S / (b * 1e-3) / 8e12))


if __name__ == '__main__':
  main()
