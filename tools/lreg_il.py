"""Dev tool (GPU box): the cfg5 fused gradient kernel with its rows in one
contiguous chunk per block (the round-4 form) vs interleaved super-chunks
(backend.ROWDOT_INTERLEAVE), over a few blocks-per-CU values; ms per sgd
iteration by wall time over REPS iterations, ROUNDS alternations; the
gradient of each form checked against the contiguous one (1e-5 of sum |x||r|
is the bench's rule; here max rel diff printed).
  python tools/lreg_il.py [N] [REPS] [ROUNDS]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spartan_amd  # noqa: E402
from spartan_amd import backend, expr, workloads  # noqa: E402


def main():
  N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
  reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
  rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
  spartan_amd.initialize()
  D = 64
  X = expr.rand(N, D, dtype=np.float32, seed=41).force()
  Y = expr.rand(N, 1, dtype=np.float32, seed=42).force()
  w = np.random.default_rng(43).random((D, 1)).astype(np.float32)
  Xe, Ye = expr.lazify(X), expr.lazify(Y)
  be = backend.get()
  confs = [(False, 16, 8), (True, 1, 8), (True, 1, 4), (True, 1, 6), (True, 1, 10), (True, 2, 4), (True, 1, 12)]
  res = {c: [] for c in confs}
  grads = {}
  real = (backend.ROWDOT_INTERLEAVE, backend.ROWDOT_BLOCKS_PER_CU, backend.ROWDOT_UNROLL)
  for r in range(rounds):
    for il, bpc, U in confs:
      backend.ROWDOT_INTERLEAVE, backend.ROWDOT_BLOCKS_PER_CU, backend.ROWDOT_UNROLL = il, bpc, U
      be._sig_fns.clear()
      be._reduce_plans.clear()
      from spartan_amd.expr import plan_cache
      plan_cache.clear() if hasattr(plan_cache, 'clear') else None
      if r == 0:
        grads[(il, bpc, U)] = expr.sum(Xe * (expr.dot(Xe, w) - Ye), axis=0).optimized().glom().astype(np.float64)
      workloads.sgd_train(Xe, Ye, w, 1e-6, 2)
      torch.cuda.synchronize()
      t0 = time.perf_counter()
      workloads.sgd_train(Xe, Ye, w, 1e-6, reps)
      torch.cuda.synchronize()
      ms = (time.perf_counter() - t0) / reps * 1e3
      res[(il, bpc, U)].append(ms)
      print('round %d interleave=%d blocks/CU=%d U=%d: %.3f ms per iteration' % (r, il, bpc, U, ms), flush=True)
  backend.ROWDOT_INTERLEAVE, backend.ROWDOT_BLOCKS_PER_CU, backend.ROWDOT_UNROLL = real
  g0 = grads[(False, 16, 8)]
  print('best of %d rounds (ms per sgd iteration, 26.0 GB each), gradient max rel diff vs contiguous:' % rounds)
  for c in confs:
    b = min(res[c])
    d = float(np.max(np.abs(grads[c] - g0) / np.abs(g0)))
    print('  interleave=%d blocks/CU=%2d U=%2d  %.3f ms  %.2f TB/s  diff %.2e' % (c[0], c[1], c[2], b, 4.0 * N * (D + 1) / b / 1e9, d))


if __name__ == '__main__':
  main()
