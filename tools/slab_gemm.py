"""Dev tool (GPU box): the per-rank GEMMs that expr/dot.py's _dot_overlapped
issues for the cfg4 dot (32768^2, K-split over N ranks) at N = 1 / 2 / 4 / 8,
timed on ONE GPU: per slab j, A_slab (M/N x K/N) @ B_g (K/N x 32768) into a
row slab of the (M x 32768) partial -- N such GEMMs per rank -- fp32 and fp64,
HIP events around each spx_gemm call (median of reps).  Prints the per-rank
GEMM time per dot and the fraction of the dense MFMA peak.
  python tools/slab_gemm.py [reps]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spartan_amd import backend  # noqa: E402

PEAK = {torch.float32: 157.3, torch.float64: 78.6}


def main():
  reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
  be = backend.get()
  S = 32768
  for dt in (torch.float32, torch.float64):
    for n in (1, 2, 4, 8):
      m, k = S // n, S // n
      A = torch.rand((S, k), dtype=dt, device='cuda')      # the gathered A column strip (all M rows)
      B = torch.rand((k, S), dtype=dt, device='cuda')      # this rank's B row strip
      C = torch.empty((S, S), dtype=dt, device='cuda')     # the full partial
      times = []
      for r in range(reps + 1):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
        ev[0].record()
        for j in range(n):
          be.gemm(A[j * m:(j + 1) * m], B, C[j * m:(j + 1) * m], 1.0, 0.0)
          ev[j + 1].record()
        torch.cuda.synchronize()
        if r:
          times.append([ev[j].elapsed_time(ev[j + 1]) for j in range(n)])
      t = np.median(np.array(times), axis=0)  # ms per slab GEMM
      flops = 2.0 * m * k * S
      tot = float(t.sum())
      print('%s N=%d: slab GEMM %dx%dx%d  %.3f ms each (min %.3f max %.3f), %d per rank = %.2f ms per dot, '
            '%.1f TF = %.3f of peak' % (str(dt).split('.')[-1], n, m, k, S, t.mean(), t.min(), t.max(), n, tot,
                                       flops * n / (tot * 1e-3) / 1e12, flops * n / (tot * 1e-3) / 1e12 / PEAK[dt]),
            flush=True)
      del A, B, C
      torch.cuda.empty_cache()


if __name__ == '__main__':
  main()
