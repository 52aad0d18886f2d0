"""Dev tool (GPU box): the cfg2 fused kernels with ocml's expf (product) vs
a two-instruction exp (v_mul + v_exp_f32 on z * log2(e)); kernel HIP-event
time, ROUNDS alternations, and the max relative difference of the sums.
  python tools/exp_ab.py [S] [EVALS] [ROUNDS]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spartan_amd  # noqa: E402
from spartan_amd import backend, codegen, expr  # noqa: E402

_orig = codegen.Emitter.op_expr


def fast(self, node, a):
  if node.name == 'exp' and np.dtype(node.in_dtypes[0]) == np.float32:
    return '__builtin_amdgcn_exp2f((%s) * 1.44269504088896341f)' % a[0]
  return _orig(self, node, a)


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
  from spartan_amd.expr import plan_cache
  ref = {}
  res = {}
  for r in range(rounds):
    for mode in ('ocml', 'fast'):
      codegen.Emitter.op_expr = fast if mode == 'fast' else _orig
      be._sig_fns.clear()
      be._reduce_plans.clear()
      plan_cache.clear()
      for ax in (0, 1):
        g = expr.sum(X * Y + expr.exp(Z), axis=ax).optimized().glom().astype(np.float64)
        ref.setdefault(ax, g)
        torch.cuda.synchronize()
        be.kernel_events = []
        for _ in range(evals):
          expr.sum(X * Y + expr.exp(Z), axis=ax).optimized().force()
        torch.cuda.synchronize()
        ks = [s.elapsed_time(e) for (n, s, e) in be.kernel_events if n.startswith('spx_reduce')]
        be.kernel_events = None
        ms = float(np.mean(ks))
        res.setdefault((mode, ax), []).append(ms)
        print('round %d %-4s axis %d: kernel %.4f ms = %.3f of 8 TB/s  max rel diff vs ocml %.2e' % (
            r, mode, ax, ms, 12.0 * S * S / (ms * 1e-3) / 8e12, float(np.max(np.abs(g - ref[ax]) / np.abs(ref[ax])))),
            flush=True)
  codegen.Emitter.op_expr = _orig
  for k, v in sorted(res.items()):
    print('  %-4s axis %d best %.4f ms  %.3f of 8 TB/s' % (k[0], k[1], min(v), 12.0 * S * S / (min(v) * 1e-3) / 8e12))


if __name__ == '__main__':
  main()
