"""Dev tool (GPU box): how many rows each certified screen leaves undecided
at the cfg3 shape, for the first-iteration centres (the first K points) and
the second-iteration ones: spx_kmeans_assign's A-stationary screen vs the
fused spx_kmeans_step screen (workspace counters[3]), plus the later list
passes' counts (counters[2] = rows left for candidates, [0] = all-centre rows).
  python tools/km_und.py [N]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spartan_amd import backend  # noqa: E402


def main():
  N = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
  be = backend.get()
  D, K = 128, 256
  dev = torch.device('cuda:0')
  pts = torch.empty((N, D), dtype=torch.float32, device=dev)
  be.fill(pts, backend.FILL_UNIFORM, 0.0, 1.0, 21, (0, 0), (N, D))
  lab = torch.empty((N,), dtype=torch.int64, device=dev)
  lab2 = torch.empty((N,), dtype=torch.int64, device=dev)
  sums = torch.empty((K, D), dtype=torch.float64, device=dev)
  cnt = torch.empty((K,), dtype=torch.int64, device=dev)
  off = (D * 256 * 4 + 15) // 16 * 16 + 256 * 8 + 32
  cen = pts[:K].to(torch.float64).contiguous()
  for itn in (1, 2, 3):
    be.kmeans_assign(pts, cen, lab)
    torch.cuda.synchronize()
    ca = be._ws[off:off + 16].view(torch.int32).cpu().tolist()
    be.kmeans_step(pts, cen, lab2, sums, cnt)
    torch.cuda.synchronize()
    cs = be._ws[off:off + 16].view(torch.int32).cpu().tolist()
    print('iteration %d: assign counters %s (screen undecided %.3f %%) | step counters %s (%.3f %%) | labels equal %s'
          % (itn, ca, 100.0 * ca[3] / N, cs, 100.0 * cs[3] / N, bool(torch.equal(lab, lab2))), flush=True)
    cen = (sums / cnt.clamp(min=1).to(torch.float64).reshape(K, 1)).contiguous()


if __name__ == '__main__':
  main()
