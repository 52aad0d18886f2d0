import sys, time
sys.path.insert(0, '.')
import numpy as np, torch
from spartan_amd.array import transfer
dev = torch.device('cuda:0')
w = np.random.rand(64, 1).astype(np.float32)
torch.zeros(1, device=dev); torch.cuda.synchronize()
def tm(f, n=2000):
    for _ in range(50): f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n): f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e6
print('transfer.upload %.1f us' % tm(lambda: transfer.upload(w, dev)))
print('as_tensor.to %.1f us' % tm(lambda: torch.as_tensor(w).to(dev)))
pin = torch.empty(4096, dtype=torch.uint8, pin_memory=True)
pv = pin.numpy()
def pinned():
    pv[:256] = w.reshape(-1).view(np.uint8)
    o = torch.empty((64, 1), dtype=torch.float32, device=dev)
    o.view(-1).view(torch.uint8).copy_(pin[:256], non_blocking=True)
    return o
print('pinned copy_ %.1f us' % tm(pinned))
print('torch.empty %.1f us' % tm(lambda: torch.empty((64, 1), dtype=torch.float32, device=dev)))
ev = torch.cuda.Event()
print('event.record %.1f us' % tm(lambda: ev.record()))
print('pin.numpy %.1f us' % tm(lambda: pin.numpy()))
t = torch.empty((64,), device=dev)
print('cpu() D2H %.1f us' % tm(lambda: t.cpu()))
print('cpu().numpy %.1f us' % tm(lambda: t.cpu().numpy()))
