"""Dev tool (GPU box): the cfg2 axis-0 fused sum (the 'cols' skeleton, 128
column tiles) with contiguous row segments per block (default) vs
interleaved super-chunks (backend.COLS_INTERLEAVE), over resident blocks per
CU; kernel time by HIP events (backend.kernel_events), ROUNDS alternations.
  python tools/cfg2_il.py [S] [EVALS] [ROUNDS]"""
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
  confs = [(False, 2), (False, 3), (False, 4), (True, 4), (False, 1)]
  res = {c: [] for c in confs}
  ref = None
  real = (backend.COLS_INTERLEAVE, backend.COLS_BLOCKS_PER_CU)
  nbytes = 12.0 * S * S + 4 * S
  for r in range(rounds):
    for il, bpc in confs:
      backend.COLS_INTERLEAVE, backend.COLS_BLOCKS_PER_CU = il, bpc
      be._sig_fns.clear()
      be._reduce_plans.clear()
      from spartan_amd.expr import plan_cache
      plan_cache.clear()
      g = expr.sum(X * Y + expr.exp(Z), axis=0).optimized().glom().astype(np.float64)
      if ref is None:
        ref = g
      torch.cuda.synchronize()
      be.kernel_events = []
      for _ in range(evals):
        expr.sum(X * Y + expr.exp(Z), axis=0).optimized().force()
      torch.cuda.synchronize()
      ks = [s.elapsed_time(e) for (n, s, e) in be.kernel_events if n.startswith('spx_reduce_cols')]
      be.kernel_events = None
      ms = float(np.mean(ks))
      res[(il, bpc)].append(ms)
      print('round %d interleave=%d blocks/CU=%d: kernel %.4f ms = %.3f of 8 TB/s  max rel diff %.2e' % (
          r, il, bpc, ms, nbytes / (ms * 1e-3) / 8e12, float(np.max(np.abs(g - ref) / np.abs(ref)))), flush=True)
  backend.COLS_INTERLEAVE, backend.COLS_BLOCKS_PER_CU = real
  for c in confs:
    b = min(res[c])
    print('  interleave=%d blocks/CU=%d  best %.4f ms  %.3f of 8 TB/s' % (c[0], c[1], b, nbytes / (b * 1e-3) / 8e12))


if __name__ == '__main__':
  main()
