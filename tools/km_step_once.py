"""Dev tool (GPU box): spx_kmeans_step REPS times at the cfg3 shape (second-
iteration centres) for rocprofv3 kernel traces / counter passes.
  python tools/km_step_once.py [N] [REPS] [assign|step|first] [libspx variant .so]
('assign': kmeans_assign + kmeans_accumulate instead of the fused step;
'first': the fused step on first-iteration centres, the first K points)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spartan_amd import backend  # noqa: E402


def main():
  N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
  reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
  mode = sys.argv[3] if len(sys.argv) > 3 else 'step'
  two = mode == 'assign'
  if len(sys.argv) > 4:  # a variant build of the library (tools/build_variant.sh)
    backend.load_library(sys.argv[4])
  be = backend.get()
  D, K = 128, 256
  dev = torch.device('cuda:0')
  pts = torch.empty((N, D), dtype=torch.float32, device=dev)
  be.fill(pts, backend.FILL_UNIFORM, 0.0, 1.0, 21, (0, 0), (N, D))
  lab = torch.empty((N,), dtype=torch.int64, device=dev)
  sums = torch.empty((K, D), dtype=torch.float64, device=dev)
  cnt = torch.empty((K,), dtype=torch.int64, device=dev)
  cen = pts[:K].to(torch.float64).contiguous()
  # second-iteration centres from the two-pass path, so that variant builds of
  # the fused step are timed on the same centres whatever their sums
  if mode != 'first':
    be.kmeans_assign(pts, cen, lab)
    be.kmeans_accumulate(pts, lab, sums, cnt)
    cen = (sums / cnt.clamp(min=1).to(torch.float64).reshape(K, 1)).contiguous()
  be.kmeans_step(pts, cen, lab, sums, cnt)
  torch.cuda.synchronize()
  ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
  ev[0].record()
  for _ in range(reps):
    if two:
      be.kmeans_assign(pts, cen, lab)
      be.kmeans_accumulate(pts, lab, sums, cnt)
    else:
      be.kmeans_step(pts, cen, lab, sums, cnt)
  ev[1].record()
  torch.cuda.synchronize()
  print('%s: %.3f ms per iteration' % ('assign+accumulate' if two else mode, ev[0].elapsed_time(ev[1]) / reps),
        flush=True)
  # checksums of the last step's results (A/B of variant builds: equal bits)
  import hashlib
  h = hashlib.sha256()
  for t in (lab, sums, cnt):
    h.update(t.cpu().numpy().tobytes())
  print('checksum labels+sums+counts: %s' % h.hexdigest()[:16], flush=True)


if __name__ == '__main__':
  main()
