"""Profile driver for the dot GEMMs (configs[3] kernels at a smaller size):
python tools/dot_prof.py [S] -- run under rocprofv3 (--kernel-trace --stats,
or a --pmc pass such as SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE) to get the
MFMA utilisation of spx_mfma::gemm for fp32 and fp64."""
import os
import sys
import time

sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import spartan_amd  # noqa: E402
from spartan_amd import expr  # noqa: E402

spartan_amd.initialize()
S = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
for dt in (np.float32, np.float64):
  a = expr.rand(S, S, dtype=dt, seed=1).force()
  b = expr.rand(S, S, dtype=dt, seed=2).force()
  for _ in range(2):
    torch.cuda.synchronize()
    t = time.perf_counter()
    expr.dot(a, b).force()
    torch.cuda.synchronize()
    el = time.perf_counter() - t
  print('%s S=%d %.3f ms %.1f TF/s' % (np.dtype(dt).name, S, el * 1e3, 2.0 * S ** 3 / el / 1e12), flush=True)
  del a, b
  torch.cuda.empty_cache()
