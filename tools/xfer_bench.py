"""Host <-> HBM transfer rates: the staged pipeline (array/transfer.py)
against the plain pageable copies it replaces.  Dev tool; run on the GPU box:
  python tools/xfer_bench.py [MiB]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spartan_amd.array import transfer  # noqa: E402


def rate(fn, nbytes, reps=3):
  fn()
  torch.cuda.synchronize()
  best = 1e30
  for _ in range(reps):
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    best = min(best, time.perf_counter() - t0)
  return nbytes / best / 1e9


def main():
  mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
  n = int(np.sqrt(mib * (1 << 20) / 4))
  dev = torch.device('cuda:0')
  host = np.random.default_rng(0).random((n, n), dtype=np.float32)
  cases = [('whole', host), ('col-half', host[:, : n // 2]), ('row-half', host[: n // 2])]
  print('matrix %dx%d f32 (%.0f MiB)  CHUNK=%d MiB threads=%d' % (n, n, host.nbytes / 2**20, transfer.CHUNK >> 20,
                                                              transfer.THREADS))
  for name, piece in cases:
    nb = piece.nbytes
    up_plain = rate(lambda: torch.as_tensor(np.ascontiguousarray(piece)).to(dev), nb)
    t = torch.as_tensor(np.ascontiguousarray(piece)).to(dev)
    out = np.empty((n, n), np.float32)
    dst = out[: piece.shape[0], : piece.shape[1]]

    def down_plain():
      dst[...] = t.cpu().numpy()

    def down_direct():
      torch.from_numpy(dcont).copy_(t)

    dcont = np.empty(piece.shape, np.float32)
    transfer.DIRECT_H2D = False
    up_staged = rate(lambda: transfer.upload(piece, dev), nb)
    transfer.DIRECT_H2D = True
    transfer.DIRECT_D2H = False
    down_staged = rate(lambda: transfer.download(t, dst), nb)
    transfer.DIRECT_D2H = True
    dp = rate(down_plain, nb)
    dd = rate(down_direct, nb)
    print('%-9s  H2D plain %6.1f GB/s  staged %6.1f GB/s   D2H plain %6.1f GB/s  staged %6.1f GB/s'
          '  direct-into-contiguous %6.1f GB/s' % (name, up_plain, up_staged, dp, down_staged, dd))
    sys.stdout.flush()


if __name__ == '__main__':
  main()
