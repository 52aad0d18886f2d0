"""Time spx_kmeans_assign and spx_kmeans_accumulate separately at cfg3 size
(HIP events on the launch stream).  Dev tool for the GPU box:
  python tools/km_split.py [libspx.so path] [N]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spartan_amd import backend  # noqa: E402


def main():
  lib = sys.argv[1] if len(sys.argv) > 1 else backend.LIB_PATH
  N = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000_000
  backend.load_library(lib)
  be = backend.get()
  D, K = 128, 256
  dev = torch.device('cuda:0')
  pts = torch.empty((N, D), dtype=torch.float32, device=dev)
  be.fill(pts, backend.FILL_UNIFORM, 0.0, 1.0, 21, (0, 0), (N, D))
  cen = pts[:K].to(torch.float64).contiguous()
  lab = torch.empty((N,), dtype=torch.int64, device=dev)
  sums = torch.empty((K, D), dtype=torch.float64, device=dev)
  cnt = torch.empty((K,), dtype=torch.int64, device=dev)
  st = torch.cuda.current_stream()
  for name, fn in [('assign', lambda: be.kmeans_assign(pts, cen, lab)),
                   ('accumulate', lambda: be.kmeans_accumulate(pts, lab, sums, cnt))]:
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(5):
      fn()
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    print('%s %-10s %8.3f ms  %7.1f GB/s of points' % (os.path.basename(lib), name, ms, N * D * 4 / ms / 1e6))
    sys.stdout.flush()


if __name__ == '__main__':
  main()
