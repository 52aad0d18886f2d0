"""Dev tool (GPU box): cycles per slot in each role of k_kmeans_pp (the
tools/kp_roles.sh build: s_memtime at role start / end; the end stamp waits
for the role's LDS operations, as the slot barrier does).  cfg3 shape.
  python tools/kp_roles.py [N] [first]"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from spartan_amd import backend  # noqa: E402


def main():
  N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
  first = len(sys.argv) > 2 and sys.argv[2] == 'first'
  name = sys.argv[3] if len(sys.argv) > 3 else 'kproles'
  lib = backend.load_library(os.path.join(ROOT, 'tools', 'bin', 'libspx_%s.so' % name))
  lib.spx_dev_kp_roles.argtypes = [ctypes.c_void_p]
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
  for _ in range(2):
    be.kmeans_step(pts, cen, lab, sums, cnt)
  torch.cuda.synchronize()
  buf = (ctypes.c_ulonglong * (1024 * 8 * 4))()
  assert lib.spx_dev_kp_roles(buf) == 0
  a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 8, 4).astype(np.float64)
  G = min(int(torch.cuda.get_device_properties(0).multi_processor_count), (N + 31) // 32)
  a = a[:G]
  slots = a[:, :, 3].mean()
  print('%s: N=%d grid=%d, %.0f slots per wave (%s centres); cycles per slot, mean over blocks:' % (
      name, N, G, slots, 'first-iteration' if first else 'second-iteration'))
  for w0, w1, name in ((0, 4, 'waves 0-3'), (4, 8, 'waves 4-7')):
    m = a[:, w0:w1, 0].mean() / (slots / 2)
    v = a[:, w0:w1, 1].mean() / (slots / 2)
    tot = a[:, w0:w1, 2].mean() / slots
    print('  %s: matrix role %6.0f  vector role %6.0f  slot (wall) %6.0f  => barrier wait %6.0f' % (
        name, m, v, tot, tot - (m + v) / 2))
  for w in range(8):
    print('    wave %d (SIMD %d): matrix role %6.0f  vector role %6.0f' % (
        w, w & 3, a[:, w, 0].mean() / (slots / 2), a[:, w, 1].mean() / (slots / 2)))


if __name__ == '__main__':
  main()
