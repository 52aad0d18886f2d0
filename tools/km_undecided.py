"""Dev probe: fraction of points the k-means certified filter leaves undecided
(candidate list) or sends to the all-centre exact path, per iteration.
python tools/km_undecided.py [N] [iters]"""
import os
import sys

sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import spartan_amd  # noqa: E402
from spartan_amd import backend, expr, workloads  # noqa: E402

spartan_amd.initialize()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000000
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 4
D, K = 128, 256
X = expr.rand(n, D, dtype=np.float32, seed=21).force()
be = backend.get()
(ex, tile), = X.local.items()
P = tile.data
c = P[:K].double()
lab = torch.empty(n, dtype=torch.int64, device=P.device)
for it in range(iters):
  be.kmeans_assign(P, c, lab)
  torch.cuda.synchronize()
  Kp = 256
  off = (D * Kp * 4 + 15) // 16 * 16 + Kp * 8 + 16
  cnt = be._ws[off:off + 8].view(torch.int32).cpu().numpy()
  print('iter %d: full %d (%.4f%%)  candidates %d (%.4f%%)' % (it, cnt[0], 100 * cnt[0] / n, cnt[1], 100 * cnt[1] / n),
        flush=True)
  # candidates per undecided point: KfCand = {i64 row; u32 mask[8]} (40 B)
  base = off + 16 + n * 8
  raw = be._ws[base:base + int(cnt[1]) * 40].cpu().numpy().reshape(-1, 40)
  pc = np.unpackbits(raw[:, 8:].copy(), axis=1).sum(1)
  if len(pc):
    print('  candidates per point: mean %.2f  p50 %d  p90 %d  max %d  hist(1..8,>8) %s'
          % (pc.mean(), np.percentile(pc, 50), np.percentile(pc, 90), pc.max(),
             [int((pc == k).sum()) for k in range(1, 9)] + [int((pc > 8).sum())]), flush=True)
  c, _ = workloads.kmeans_fit(X, K, 1, centers=c.cpu().numpy())
  c = torch.as_tensor(c).to(P.device)
