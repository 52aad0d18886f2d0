"""Cross-rank data movement for tiles (torch.distributed: RCCL on GPU, gloo in tests).

With ``SPARTAN_DIST_BACKEND=gloo`` on GPUs (rehearsing N ranks on one
device, e.g. the 1-GPU box) device tensors are staged through host memory,
since gloo moves host buffers only; the RCCL path never stages.

Replaces the reference's pickled ZeroMQ point-to-point messages
(spartan/rpc/common.py:52-62, spartan/blob_ctx.py:127-179): every exchange here
is a collective that all ranks enter with identical arguments, because every
rank computes the same tile plan (SPMD).
"""
import numpy as np

from . import runtime

_OPS = {'sum': 'SUM', 'min': 'MIN', 'max': 'MAX'}


def _dist():
  import torch.distributed as dist
  return dist


def _staged(ctx, t):
  return ctx.dist_backend == 'gloo' and t.device.type != 'cpu'


def all_reduce(t, op):
  ctx = runtime.get()
  if not ctx.distributed:
    return t
  dist = _dist()
  if _staged(ctx, t):
    h = t.cpu()
    dist.all_reduce(h, op=getattr(dist.ReduceOp, _OPS[op]))
    t.copy_(h)
    return t
  dist.all_reduce(t, op=getattr(dist.ReduceOp, _OPS[op]))
  return t


def reduce_scatter_rows(out, full, op):
  """out = rank-th equal row slab of the element-wise reduction of ``full``."""
  ctx = runtime.get()
  dist = _dist()
  if ctx.dist_backend == 'gloo':  # gloo has no reduce_scatter: all_reduce + slice
    all_reduce(full, op)
    n = out.shape[0]
    out.copy_(full[ctx.rank * n:(ctx.rank + 1) * n])
    return out
  dist.reduce_scatter_tensor(out, full, op=getattr(dist.ReduceOp, _OPS[op]))
  return out


def all_gather_stack(t):
  """[world, *t.shape] stack of every rank's ``t`` (same shape on all ranks)."""
  import torch
  ctx = runtime.get()
  if not ctx.distributed:
    return t.unsqueeze(0)
  dist = _dist()
  out = torch.empty((ctx.world_size,) + tuple(t.shape), dtype=t.dtype, device=t.device)
  if _staged(ctx, t):
    h = torch.empty(out.shape, dtype=t.dtype)
    dist.all_gather(list(h.unbind(0)), t.contiguous().cpu())
    out.copy_(h)
  elif ctx.dist_backend == 'gloo':
    dist.all_gather(list(out.unbind(0)), t.contiguous())
  else:
    dist.all_gather_into_tensor(out, t.contiguous())
  return out


def broadcast(t, src_rank):
  ctx = runtime.get()
  if not ctx.distributed:
    return t
  if _staged(ctx, t):
    h = t.cpu()
    _dist().broadcast(h, src=src_rank)
    t.copy_(h)
    return t
  _dist().broadcast(t, src=src_rank)
  return t


def reduce_async(t, dst_rank, op):
  """Start reducing ``t`` (contiguous, same shape on every rank) into
  ``t`` on ``dst_rank``; returns a handle for ``wait_all``.  On RCCL the
  reduction runs on the process group's stream, after the work already
  queued on the current stream and concurrently with what follows it."""
  ctx = runtime.get()
  dist = _dist()
  if _staged(ctx, t):  # rehearsal: synchronous through the host
    h = t.cpu()
    dist.reduce(h, dst=dst_rank, op=getattr(dist.ReduceOp, _OPS[op]))
    if ctx.rank == dst_rank:
      t.copy_(h)
    return None
  return dist.reduce(t, dst=dst_rank, op=getattr(dist.ReduceOp, _OPS[op]), async_op=True)


def wait_all(handles):
  for h in handles:
    if h is not None:
      h.wait()


def all_to_all_single(out, inp, out_splits, in_splits):
  _dist().all_to_all_single(out, inp, output_split_sizes=out_splits, input_split_sizes=in_splits)
  return out


def exchange(sends, recvs):
  """Point-to-point batch.  sends: [(tensor, dst_rank)], recvs: [(tensor, src_rank)].

  Every rank passes the pairs it takes part in; messages between the same pair
  of ranks are matched in list order."""
  ctx = runtime.get()
  if not ctx.distributed or (not sends and not recvs):
    return
  import torch
  dist = _dist()
  post = []
  if ctx.dist_backend == 'gloo':  # host staging for device tensors (rehearsal mode)
    sends = [(t.contiguous().cpu() if _staged(ctx, t) else t, peer) for t, peer in sends]
    staged = []
    for t, peer in recvs:
      if _staged(ctx, t):
        h = torch.empty(t.shape, dtype=t.dtype)
        post.append((t, h))
        staged.append((h, peer))
      else:
        staged.append((t, peer))
    recvs = staged
  ops = [dist.P2POp(dist.isend, t.contiguous(), peer) for t, peer in sends]
  ops += [dist.P2POp(dist.irecv, t, peer) for t, peer in recvs]
  for req in dist.batch_isend_irecv(ops):
    req.wait()
  for t, h in post:
    t.copy_(h)


def barrier():
  ctx = runtime.get()
  if ctx.distributed:
    _dist().barrier()


def max_over_ranks(x):
  """Max of a host float over all ranks (bench timing)."""
  import torch
  ctx = runtime.get()
  if not ctx.distributed:
    return x
  t = torch.tensor([float(x)], dtype=torch.float64, device=ctx.device)
  all_reduce(t, 'max')
  return float(t.item())
