"""Dev tool (GPU box): the generated 'rows' reduction (reduced axis
contiguous, > 4096 elements per segment) over many segments -- the shape
where the per-block combine is a visible share of each block's work.
GB/s of algorithmic bytes, HIP events on the launch stream.
  python tools/rows_bench.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.environ.get('SPX_PKG_ROOT') or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spartan_amd  # noqa: E402
from spartan_amd import backend, expr  # noqa: E402


def main():
  spartan_amd.initialize()
  be = backend.get()
  for shape in [(262144, 8192), (131072, 16384), (32768, 32768), (524288, 4352)]:
    x = expr.lazify(expr.rand(*shape, dtype=np.float32, seed=5).force())
    for _ in range(2):
      expr.sum(x * 2.0, axis=1).optimized().force()
    torch.cuda.synchronize()
    be.kernel_events = []
    for _ in range(10):
      expr.sum(x * 2.0, axis=1).optimized().force()
    torch.cuda.synchronize()
    ms = [s.elapsed_time(e) for n, s, e in be.kernel_events if n.startswith('spx_reduce')]
    be.kernel_events = None
    t = float(np.median(ms)) * 1e-3
    nb = shape[0] * shape[1] * 4 + shape[0] * 4
    print('rows %-16s %8.3f ms  %7.1f GB/s' % (shape, t * 1e3, nb / t / 1e9), flush=True)
    del x
    torch.cuda.empty_cache()


if __name__ == '__main__':
  main()
