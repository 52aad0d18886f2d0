"""Dev tool (GPU box): the cfg5 fused gradient kernel (DotReduceFusion, the
'cols' skeleton with one 64-column tile) under different row unrolls and
resident blocks per CU, interleaved rounds, kernel time by HIP events around
REPS sgd iterations.  Patches backend / codegen knobs in-process only.
  python tools/lreg_sweep.py [N] [REPS] [ROUNDS]"""
import itertools
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spartan_amd  # noqa: E402
from spartan_amd import backend, codegen, expr, workloads  # noqa: E402


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
  real = (backend.ROWDOT_UNROLL, backend.ROWDOT_BLOCKS_PER_CU)
  confs = list(itertools.product([4, 8, 12], [7, 8, 14, 16, 21, 28]))  # (rows unrolled, blocks per CU)
  res = {c: [] for c in confs}
  be = backend.get()
  for r in range(rounds):
    for U, bpc in confs:
      backend.ROWDOT_UNROLL, backend.ROWDOT_BLOCKS_PER_CU = U, bpc
      be._sig_fns.clear()
      be._reduce_plans.clear()
      from spartan_amd.expr import plan_cache
      plan_cache.clear() if hasattr(plan_cache, 'clear') else None
      workloads.sgd_train(Xe, Ye, w, 1e-6, 2)
      torch.cuda.synchronize()
      t0 = time.perf_counter()
      workloads.sgd_train(Xe, Ye, w, 1e-6, reps)
      torch.cuda.synchronize()
      ms = (time.perf_counter() - t0) / reps * 1e3
      res[(U, bpc)].append(ms)
      print('round %d U=%d blocks/CU=%d: %.3f ms per iteration' % (r, U, bpc, ms), flush=True)
  backend.ROWDOT_UNROLL, backend.ROWDOT_BLOCKS_PER_CU = real
  print('best of %d rounds (ms per sgd iteration, 26.0 GB each):' % rounds)
  for c in confs:
    b = min(res[c])
    print('  U=%d blocks/CU=%2d  %.3f ms  %.2f TB/s' % (c[0], c[1], b, 4.0 * N * (D + 1) / b / 1e9))


if __name__ == '__main__':
  main()
