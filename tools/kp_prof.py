"""Dev tool (GPU box): per-segment cycles of k_kmeans_pp from the
tools/kp_prof.sh build (s_memtime counters; the instrumentation itself costs
~10 % of the cycles).  cfg3 shape, second-iteration centres (or the first K
points with 'first').  python tools/kp_prof.py [N] [first]"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from spartan_amd import backend  # noqa: E402

SEG = ['barrier wait', 'matrix: MFMAs + add round 0', 'matrix: add rounds 1+', 'matrix: stores + loads',
       'vector: part 1 (v3: fold 0 + decide; v5: fold + exv)', 'vector: part 2 (v3: rank + fold 1)',
       'vector: stage',
       'pre-barrier (flush)']


def main():
  N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
  first = len(sys.argv) > 2 and sys.argv[2] == 'first'
  lib = backend.load_library(os.path.join(ROOT, 'tools', 'bin', 'libspx_kpprof.so'))
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
  be.kmeans_step(pts, cen, lab, sums, cnt)
  torch.cuda.synchronize()
  buf = (ctypes.c_ulonglong * (1024 * 8 * 8))()
  assert lib.spx_dev_kp_prof(buf) == 0
  a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 8, 8).astype(np.float64)
  ncu = int(torch.cuda.get_device_properties(0).multi_processor_count)
  G = min(ncu, (N + 31) // 32)
  a = a[:G]
  nit = ((N + 31) // 32 + G - 1) // G
  nrun = (nit + 4 + 7) // 8 * 8
  print('N=%d grid=%d slots per block=%d (%s centres)' % (N, G, nrun, 'first-iteration' if first else 'second-iteration'))
  tot = a.sum(axis=2).mean(axis=0)  # per wave, cycles over the kernel's loop
  print('cycles per slot (32 rows), mean over blocks; waves 0-3 | 4-7:')
  for k, name in enumerate(SEG):
    per = 2.0 / nrun if 1 <= k <= 6 else 1.0 / nrun  # role segments run every other slot
    g0 = a[:, 0:4, k].mean() * per
    g1 = a[:, 4:8, k].mean() * per
    print('  %-32s %8.0f | %8.0f' % (name, g0, g1))
  print('  total per slot (all segments)  %8.0f | %8.0f' % (tot[0:4].mean() / nrun, tot[4:8].mean() / nrun))


if __name__ == '__main__':
  main()
