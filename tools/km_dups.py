"""Dev tool (GPU box): label multiplicities inside k_kmeans_fs2's 64-row
units at cfg3, for first-iteration centres (data points) and second-iteration
centres: how many rows need the add rounds 1, 2 and the tail loop.
  python tools/km_dups.py [N]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spartan_amd import backend  # noqa: E402


def stats(lab):
  L = lab.reshape(-1, 64)
  s = np.sort(L, axis=1)
  # rank of each row among equal labels in its unit (0 = first)
  rank = np.zeros_like(s)
  for j in range(1, 64):
    rank[:, j] = np.where(s[:, j] == s[:, j - 1], rank[:, j - 1] + 1, 0)
  n = rank.size
  return {'round0': (rank == 0).sum() / n, 'round1': (rank == 1).sum() / n, 'round2': (rank == 2).sum() / n,
          'tail': (rank >= 3).sum() / n, 'max_mult': int(rank.max()) + 1,
          'largest_cluster_frac': float(np.bincount(lab).max() / lab.size)}


def main():
  N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
  be = backend.get()
  D, K = 128, 256
  dev = torch.device('cuda:0')
  pts = torch.empty((N, D), dtype=torch.float32, device=dev)
  be.fill(pts, backend.FILL_UNIFORM, 0.0, 1.0, 21, (0, 0), (N, D))
  lab = torch.empty((N,), dtype=torch.int64, device=dev)
  sums = torch.empty((K, D), dtype=torch.float64, device=dev)
  cnt = torch.empty((K,), dtype=torch.int64, device=dev)
  cen = pts[:K].to(torch.float64).contiguous()
  for it in range(2):
    be.kmeans_step(pts, cen, lab, sums, cnt)
    torch.cuda.synchronize()
    print('iteration %d:' % (it + 1), stats(lab[:N // 64 * 64].cpu().numpy()), flush=True)
    cen = (sums / cnt.clamp(min=1).to(torch.float64).reshape(K, 1)).contiguous()


if __name__ == '__main__':
  main()
