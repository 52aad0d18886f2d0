"""Dev tool (GPU box): per-wave cycles of each loop segment of k_kmeans_fs2
(a -DKF2_PROF=1 build: tools/build_variant.sh prof -DKF2_PROF=1) at cfg3
with second-iteration centres ('first': the first K points), averaged over
the waves, per 64-row unit.
  python tools/kf2_prof.py tools/bin/libspx_prof.so [N] [first]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spartan_amd import backend  # noqa: E402

# pacc[k] = cycles from marker k - 1 to marker k (marker 0 follows the loop's
# last segment, the ring loads)
SEG = ['loads', 'barrier A wait', 'flush + MFMA + table', 'labels out', 'fold', 'barrier B wait', 'decide',
       'adds', 'stage']


def main():
  lib = backend.load_library(sys.argv[1])
  N = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000_000
  be = backend.get()
  D, K = 128, 256
  dev = torch.device('cuda:0')
  pts = torch.empty((N, D), dtype=torch.float32, device=dev)
  be.fill(pts, backend.FILL_UNIFORM, 0.0, 1.0, 21, (0, 0), (N, D))
  lab = torch.empty((N,), dtype=torch.int64, device=dev)
  sums = torch.empty((K, D), dtype=torch.float64, device=dev)
  cnt = torch.empty((K,), dtype=torch.int64, device=dev)
  cen = pts[:K].to(torch.float64).contiguous()
  first = len(sys.argv) > 3 and sys.argv[3] == 'first'
  if not first:
    be.kmeans_assign(pts, cen, lab)
    be.kmeans_accumulate(pts, lab, sums, cnt)
    cen = (sums / cnt.clamp(min=1).to(torch.float64).reshape(K, 1)).contiguous()
  be.kmeans_step(pts, cen, lab, sums, cnt)
  torch.cuda.synchronize()
  buf = (ctypes.c_ulonglong * (256 * 8 * 9))()
  assert lib.spx_dev_kf2_prof(buf) == 0
  a = np.frombuffer(buf, dtype=np.uint64).reshape(256 * 8, 9).astype(np.float64)
  nunits = (N + 63) // 64 / 256.0
  tot = a.sum(axis=1).mean() / nunits
  print('cycles per unit (mean over waves): total %.0f' % tot)
  for k, name in enumerate(SEG):
    col = a[:, k] / nunits
    print('  %-16s %7.0f  (waves 0-3 %7.0f, 4-7 %7.0f)' % (name, col.mean(), col.reshape(256, 8)[:, :4].mean(),
                                                          col.reshape(256, 8)[:, 4:].mean()))


if __name__ == '__main__':
  main()
