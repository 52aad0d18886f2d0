"""Dev (GPU box): do libspx's RCCL collectives run with two ranks on the one
GPU of a test box?  torchrun --nproc-per-node 2 tools/rccl_probe.py
(RCCL normally refuses two ranks on one device; this records what it does)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import spartan_amd  # noqa: E402
from spartan_amd import comm, runtime  # noqa: E402

ctx = spartan_amd.initialize()
t = torch.full((1024,), float(ctx.rank + 1), device=ctx.device)
comm.all_reduce(t, 'sum')
torch.cuda.synchronize()
out = torch.empty((512,), device=ctx.device)
full = torch.arange(1024, dtype=torch.float32, device=ctx.device) * (ctx.rank + 1)
comm.reduce_scatter_rows(out, full, 'sum')
torch.cuda.synchronize()
print('rank %d backend %s allreduce %s rs[0:2] %s' % (ctx.rank, ctx.dist_backend, t[0].item(), out[:2].tolist()),
      flush=True)
runtime.shutdown()
