"""Dev tool (GPU box): the cfg5 gradient at a given w through the product
path (fused, plan-cached), the product path with the plan cache off, the
unfused two-pass path, and a chunked torch fp64 restatement; prints each
path's worst |g - ref| / sum |x||r| over the 64 columns.
  python tools/lreg_check.py [N]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
  N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
  import spartan_amd
  from spartan_amd import expr, workloads
  from spartan_amd.config import FLAGS
  ctx = spartan_amd.initialize()
  D = 64
  X = expr.rand(N, D, dtype=np.float32, seed=41).force()
  Y = expr.rand(N, 1, dtype=np.float32, seed=42).force()
  w = np.random.default_rng(43).random((D, 1)).astype(np.float32)
  Xe, Ye = expr.lazify(X), expr.lazify(Y)
  w = workloads.sgd_train(Xe, Ye, w, 1e-6, 3)
  wd = torch.as_tensor(np.asarray(w, np.float64).reshape(D)).to(ctx.device)
  acc = torch.zeros((2, D), dtype=torch.float64, device=ctx.device)
  for (ex, t), (ey, u) in zip(sorted(X.local.items(), key=lambda e: e[0].ul), sorted(Y.local.items(), key=lambda e: e[0].ul)):
    for r0 in range(0, ex.shape[0], 1 << 23):
      xc = t.data[r0:r0 + (1 << 23)].to(torch.float64)
      res = xc @ wd - u.data.reshape(-1)[r0:r0 + (1 << 23)].to(torch.float64)
      acc[0] += res @ xc
      acc[1] += res.abs() @ xc.abs()
  ref, cond = acc.cpu().numpy()

  def rep(name, g):
    g = np.asarray(g, np.float64).reshape(D)
    r = np.abs(g - ref) / cond
    print('%-22s worst %.3e (col %d) median %.3e  |g| %.4e' % (name, r.max(), r.argmax(), np.median(r), np.abs(ref).max()),
          flush=True)

  rep('fused, replayed', expr.sum(Xe * (expr.dot(Xe, w) - Ye), axis=0).optimized().glom())
  FLAGS.opt_plan_cache = False
  rep('fused, fresh', expr.sum(Xe * (expr.dot(Xe, w) - Ye), axis=0).optimized().glom())
  FLAGS.opt_dot_fusion = False
  rep('two passes', expr.sum(Xe * (expr.dot(Xe, w) - Ye), axis=0).optimized().glom())
  # fp32 on the host-like order: torch fp32 chunked
  g32 = torch.zeros((D,), dtype=torch.float32, device=ctx.device)
  for (ex, t), (ey, u) in zip(sorted(X.local.items(), key=lambda e: e[0].ul), sorted(Y.local.items(), key=lambda e: e[0].ul)):
    for r0 in range(0, ex.shape[0], 1 << 23):
      xc = t.data[r0:r0 + (1 << 23)]
      res = xc @ wd.float() - u.data.reshape(-1)[r0:r0 + (1 << 23)]
      g32 += res @ xc
  rep('torch fp32 chunked', g32.cpu().numpy())
  spartan_amd.shutdown()


if __name__ == '__main__':
  main()
