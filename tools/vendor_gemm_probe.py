"""Dev probe: time torch.matmul (the vendor GEMM) for fp32 / fp64 at a few
sizes, so rocprofv3 --kernel-trace names the library kernel it picks."""
import sys
import torch

torch.backends.cuda.matmul.allow_tf32 = False
for S in [int(s) for s in (sys.argv[1:] or ['8192', '32768'])]:
  for dt in (torch.float32, torch.float64):
    a = torch.rand((S, S), dtype=dt, device='cuda')
    b = torch.rand((S, S), dtype=dt, device='cuda')
    c = torch.empty((S, S), dtype=dt, device='cuda')
    for _ in range(3):
      torch.matmul(a, b, out=c)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
      torch.matmul(a, b, out=c)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / 3
    print('%s S=%d %.3f ms %.1f TF' % (dt, S, ms, 2 * S ** 3 / ms / 1e9), flush=True)
    del a, b, c
    torch.cuda.empty_cache()
