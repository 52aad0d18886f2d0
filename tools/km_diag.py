"""Dev tool (GPU box): the skewed long-chain k-means case of
tests/test_gpu_parity.py::test_kmeans_step_long_chains[256] stage by stage,
printing (flushed) the time of every stage, so a slow or stuck stage names
itself.  python tools/km_diag.py [N]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spartan_amd import backend  # noqa: E402


def stage(name, fn):
  t0 = time.perf_counter()
  r = fn()
  torch.cuda.synchronize()
  print('%-28s %8.1f ms' % (name, (time.perf_counter() - t0) * 1e3), flush=True)
  return r


def main():
  N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_200_000
  be = backend.get()
  D, K = 64, 256
  P = torch.empty((N, D), dtype=torch.float32, device='cuda')
  stage('fill', lambda: be.fill(P, backend.FILL_UNIFORM, 0.0, 1.0, 91, (0, 0), (N, D)))
  stage('skew', lambda: P[: N * 95 // 100].mul_(0.01))
  g = np.random.default_rng(5)
  C = g.random((K, D)) * 0.5 + 0.5
  C[0] = 0.005
  Cd = torch.as_tensor(C).cuda()
  lab = torch.empty((N,), dtype=torch.int64, device='cuda')
  sums = torch.empty((K, D), dtype=torch.float64, device='cuda')
  cnt = torch.empty((K,), dtype=torch.int64, device='cuda')
  stage('kmeans_step', lambda: be.kmeans_step(P, Cd, lab, sums, cnt))
  print('undecided after the screen:', be.kmeans_counters(D)[3], flush=True)
  stage('kmeans_step again', lambda: be.kmeans_step(P, Cd, lab, sums, cnt))
  exact = torch.empty_like(lab)
  stage('assign exact_only', lambda: be.kmeans_assign(P, Cd, exact, exact_only=True))
  print('labels equal:', bool(torch.equal(lab, exact)), 'count of centre 0:', int(cnt[0]), flush=True)
  ws = torch.zeros((K, D), dtype=torch.float64, device='cuda')
  stage('index_add check', lambda: ws.index_add_(0, lab[:N // 8], P[:N // 8].to(torch.float64)))
  ws2 = torch.zeros((K, D), dtype=torch.float64, device='cuda')

  def onehot():
    for r0 in range(0, N, 1 << 20):
      oh = torch.nn.functional.one_hot(lab[r0:r0 + (1 << 20)], K).to(torch.float64)
      ws2.add_(oh.t() @ P[r0:r0 + (1 << 20)].to(torch.float64))
  stage('one-hot GEMM check', onehot)
  ws = ws2
  print('max rel err of sums:', float(((sums - ws).abs() / ws.abs().clamp(min=1e-300)).max()), flush=True)


if __name__ == '__main__':
  main()
