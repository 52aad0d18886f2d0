"""Dev tool (GPU box): the certified k-means assignment's two filter modes
at cfg3 shape -- A-stationary first pass + list-mode candidates (default)
vs the single all-accumulator pass (SPX_KMEANS_FILTER=b3) -- labels checked
bit for bit against the all-exact kernel on a prefix, then timed with HIP
events on the launch stream (assign and accumulate separately).
  python tools/km_modes.py [libspx.so path] [N] [N_exact]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spartan_amd import backend  # noqa: E402


def timed(fn, reps=5):
  st = torch.cuda.current_stream()
  fn()
  torch.cuda.synchronize()
  e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  e0.record(st)
  for _ in range(reps):
    fn()
  e1.record(st)
  torch.cuda.synchronize()
  return e0.elapsed_time(e1) / reps


def main():
  lib = sys.argv[1] if len(sys.argv) > 1 else backend.LIB_PATH
  N = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000_000
  NE = int(sys.argv[3]) if len(sys.argv) > 3 else 4_000_000
  backend.load_library(lib)
  be = backend.get()
  D, K = 128, 256
  dev = torch.device('cuda:0')
  pts = torch.empty((N, D), dtype=torch.float32, device=dev)
  be.fill(pts, backend.FILL_UNIFORM, 0.0, 1.0, 21, (0, 0), (N, D))
  lab = torch.empty((N,), dtype=torch.int64, device=dev)
  sums = torch.empty((K, D), dtype=torch.float64, device=dev)
  cnt = torch.empty((K,), dtype=torch.int64, device=dev)
  for it, cen in enumerate([pts[:K].to(torch.float64).contiguous(), None]):
    if cen is None:  # second iteration's centres: the means of the first assignment
      be.kmeans_assign(pts, cen0, lab)
      be.kmeans_accumulate(pts, lab, sums, cnt)
      cen = (sums / cnt.clamp(min=1).to(torch.float64).reshape(K, 1)).contiguous()
    cen0 = cen
    ref = torch.empty((NE,), dtype=torch.int64, device=dev)
    be.kmeans_assign(pts[:NE], cen, ref, exact_only=True)
    res = {}
    for mode in os.environ.get('KM_MODES', 'as,b3').split(','):
      os.environ['SPX_KMEANS_FILTER'] = mode
      l2 = torch.empty((NE,), dtype=torch.int64, device=dev)
      be.kmeans_assign(pts[:NE], cen, l2)
      bad = int((l2 != ref).sum().item())
      ms = timed(lambda: be.kmeans_assign(pts, cen, lab))
      res[mode] = (ms, bad)
      print('iter %d %-3s assign %8.3f ms  mismatches vs exact (first %d): %d' % (it, mode, ms, NE, bad), flush=True)
    os.environ.pop('SPX_KMEANS_FILTER')
    ms = timed(lambda: be.kmeans_accumulate(pts, lab, sums, cnt))
    print('iter %d accumulate %8.3f ms  (%.1f GB/s of points)' % (it, ms, N * D * 4 / ms / 1e6), flush=True)


if __name__ == '__main__':
  main()
