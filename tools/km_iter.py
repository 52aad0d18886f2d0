"""Dev tool (GPU box): REPS full k-means iterations (assign + accumulate) at
cfg3 shape, second-iteration centres, for rocprofv3 counter passes.
  python tools/km_iter.py [N] [REPS]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spartan_amd import backend  # noqa: E402


def main():
  N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
  reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
  be = backend.get()
  D, K = 128, 256
  dev = torch.device('cuda:0')
  pts = torch.empty((N, D), dtype=torch.float32, device=dev)
  be.fill(pts, backend.FILL_UNIFORM, 0.0, 1.0, 21, (0, 0), (N, D))
  lab = torch.empty((N,), dtype=torch.int64, device=dev)
  sums = torch.empty((K, D), dtype=torch.float64, device=dev)
  cnt = torch.empty((K,), dtype=torch.int64, device=dev)
  cen = pts[:K].to(torch.float64).contiguous()
  be.kmeans_assign(pts, cen, lab)
  be.kmeans_accumulate(pts, lab, sums, cnt)
  cen = (sums / cnt.clamp(min=1).to(torch.float64).reshape(K, 1)).contiguous()
  for _ in range(reps):
    be.kmeans_assign(pts, cen, lab)
    be.kmeans_accumulate(pts, lab, sums, cnt)
  torch.cuda.synchronize()
  print('done', flush=True)


if __name__ == '__main__':
  main()
