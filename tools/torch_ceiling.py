"""Dev tool (GPU box): PyTorch's own elementwise / reduction kernels on
cfg2-sized fp32 tensors, HIP-event timed -- a second opinion on the
achievable streaming rate.  python tools/torch_ceiling.py"""
import torch

S = 32768
dev = torch.device('cuda:0')
g = torch.Generator(device=dev)
g.manual_seed(0)
x = torch.rand((S, S), device=dev, generator=g)
y = torch.rand((S, S), device=dev, generator=g)
z = torch.rand((S, S), device=dev, generator=g)
out = torch.empty_like(x)


def tm(f, nbytes, name):
  for _ in range(2):
    f()
  torch.cuda.synchronize()
  ts = []
  for _ in range(10):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    f()
    b.record()
    b.synchronize()
    ts.append(a.elapsed_time(b))
  ts.sort()
  ms = ts[len(ts) // 2]
  print('%-28s %.4f ms  %.1f GB/s' % (name, ms, nbytes / ms / 1e6), flush=True)


E = S * S * 4
tm(lambda: torch.mul(x, y, out=out), 3 * E, 'mul(x,y) out=')
tm(lambda: torch.add(x, 1.0, out=out), 2 * E, 'add(x,1) out=')
tm(lambda: torch.exp(z, out=out), 2 * E, 'exp(z) out=')
tm(lambda: out.copy_(x), 2 * E, 'copy')
tm(lambda: x.sum(dim=1), E, 'sum(x, dim=1)')
tm(lambda: x.sum(dim=0), E, 'sum(x, dim=0)')
tm(lambda: torch.addcmul(torch.exp(z), x, y).sum(dim=1), 5 * E, 'addcmul(exp z) sum dim1 (unfused)')
