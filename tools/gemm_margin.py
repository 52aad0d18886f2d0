"""Dev tool (GPU box): the cfg4 fp32 GEMM (32768^2, A/B ~ U[0,1) from the
bench's seeds 31/32) through spx_gemm of a given libspx build: median kernel
time of 3 (HIP events), TF/s, and the max |C - fp64| / |fp64| over EVERY
element (torch fp64 GEMMs on the device, 2048-row blocks: a checker).
  python tools/gemm_margin.py [libspx .so]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spartan_amd import backend  # noqa: E402


def main():
  lib = sys.argv[1] if len(sys.argv) > 1 else None
  if lib:
    backend.load_library(lib)
  be = backend.get()
  S = 32768
  A = torch.empty((S, S), dtype=torch.float32, device='cuda')
  B = torch.empty((S, S), dtype=torch.float32, device='cuda')
  be.fill(A, backend.FILL_UNIFORM, 0.0, 1.0, 31, (0, 0), (S, S))
  be.fill(B, backend.FILL_UNIFORM, 0.0, 1.0, 32, (0, 0), (S, S))
  C = torch.empty((S, S), dtype=torch.float32, device='cuda')
  ts = []
  for _ in range(4):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    be.gemm(A, B, C, 1.0, 0.0)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
  t = float(np.median(ts[1:]))
  b64 = B.to(torch.float64)
  m = 0.0
  for r0 in range(0, S, 2048):
    want = A[r0:r0 + 2048].to(torch.float64) @ b64
    m = max(m, ((C[r0:r0 + 2048].to(torch.float64) - want).abs_().div_(want.abs())).max().item())
    del want
  print('%s: %.2f ms = %.1f TF; max rel err over all elements %.4g' % (
      os.path.basename(lib) if lib else 'product', t, 2.0 * S ** 3 / (t * 1e-3) / 1e12, m), flush=True)


if __name__ == '__main__':
  main()
