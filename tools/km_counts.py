"""Dev tool (GPU box): the fused k-means step's row counts at the cfg3 shape
(second-iteration centres, or the first K points with 'first'): rows the
fp16 screen left undecided, rows the bf16x3 list pass left undecided,
candidate rows, rows sent to the all-centre exact kernel.
  python tools/km_counts.py [N] [first]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spartan_amd import backend  # noqa: E402


def main():
  N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
  first = len(sys.argv) > 2 and sys.argv[2] == 'first'
  be = backend.get()
  D, K = 128, 256
  pts = torch.empty((N, D), dtype=torch.float32, device='cuda')
  be.fill(pts, backend.FILL_UNIFORM, 0.0, 1.0, 21, (0, 0), (N, D))
  lab = torch.empty((N,), dtype=torch.int64, device='cuda')
  sums = torch.empty((K, D), dtype=torch.float64, device='cuda')
  cnt = torch.empty((K,), dtype=torch.int64, device='cuda')
  cen = pts[:K].to(torch.float64).contiguous()
  if not first:
    be.kmeans_assign(pts, cen, lab)
    be.kmeans_accumulate(pts, lab, sums, cnt)
    cen = (sums / cnt.clamp(min=1).to(torch.float64).reshape(K, 1)).contiguous()
  be.kmeans_step(pts, cen, lab, sums, cnt)
  torch.cuda.synchronize()
  exact, cand, und_b3, und_fp16 = be.kmeans_counters(D)
  print('N=%d (%s centres): fp16 screen undecided %d (%.2f %%), after the bf16x3 list pass %d (%.3f %%), '
        'candidate rows %d, all-centre exact rows %d' % (N, 'first' if first else 'second-iteration', und_fp16,
                                                          100.0 * und_fp16 / N, und_b3, 100.0 * und_b3 / N, cand, exact),
        flush=True)


if __name__ == '__main__':
  main()
