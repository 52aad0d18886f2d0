"""Cross-rank data movement for tiles.

Data plane, by ``ctx.dist_backend``:

* ``'nccl'`` (the GPU default at N > 1): torch.distributed's RCCL process
  group (PyTorch's librccl; 'nccl' is RCCL on ROCm), also the fallback when
  the libspx communicator cannot be created or fails its start-up self-test
  (``selftest``).  The control plane runs on a gloo group of its own.
* ``'rccl'`` (opt-in, ``SPARTAN_DIST_BACKEND=rccl``, until a multi-GPU run
  validates it): every collective is a libspx.so C-ABI call
  (``spx_allreduce`` / ``spx_reduce_scatter`` / ``spx_allgather`` /
  ``spx_broadcast`` / ``spx_reduce`` / ``spx_sendrecv``, include/spx.h) on
  the RCCL communicator the runtime created, enqueued on the current HIP
  stream.  torch.distributed (gloo) is the host control plane only: the
  unique-id hand-off, ``barrier``, the SPMD guard and ``max_over_ranks`` of
  host floats.
* ``'gloo'``: CPU tests, and the one-GPU multi-rank rehearsal
  (``SPARTAN_DIST_BACKEND=gloo``), where device tensors are staged through
  host memory.

Replaces the reference's pickled ZeroMQ point-to-point messages
(spartan/rpc/common.py:52-62, spartan/blob_ctx.py:127-179): every exchange
here is a collective that all ranks enter with identical arguments, because
every rank computes the same tile plan (SPMD).
"""
import ctypes
import os
import zlib

from . import runtime

_OPS = {'sum': 'SUM', 'min': 'MIN', 'max': 'MAX'}
_SPX_OP = {'sum': 0, 'min': 1, 'max': 2}


def _dist():
  import torch.distributed as dist
  return dist


def _grp():
  """The torch process group of the data plane: torch's own RCCL group when
  the runtime fell back to it, else the default group."""
  return getattr(runtime.get(), 'pg', None)


def _ctl(ctx):
  """(group, device) of the host control plane: the runtime's gloo group
  when the default group is nccl, else the default (gloo) group."""
  import torch
  if getattr(ctx, 'ctl', None) is not None:
    return ctx.ctl, torch.device('cpu')
  if _dist().get_backend() == 'nccl':  # a caller-made nccl default group and no gloo group
    return None, ctx.device
  return None, torch.device('cpu')


def _staged(ctx, t):
  return ctx.dist_backend == 'gloo' and t.device.type != 'cpu'


# ------------------------------------------------------- libspx RCCL plane
def _lib():
  from . import backend
  return backend.load_library()


def _check(rc, what):
  if rc != 0:
    raise RuntimeError('%s failed (%d): %s' % (what, rc, _lib().spx_last_error().decode()))


def _dt(t):
  from . import backend
  return backend.spx_dtype(backend.np_dtype(t.dtype))


def _stream():
  import torch
  return ctypes.c_void_p(torch._C._cuda_getCurrentRawStream(torch.cuda.current_device()))


def _p(t):
  return ctypes.c_void_p(t.data_ptr())


def rccl_path():
  """The RCCL PyTorch-ROCm itself loaded (one RCCL, one HIP runtime per
  process); /opt/rocm's librccl.so.1 otherwise."""
  import os
  import torch
  p = os.path.join(os.path.dirname(torch.__file__), 'lib', 'librccl.so')
  return p if os.path.exists(p) else 'librccl.so.1'


def rccl_init(rank, world, unique_id=None):
  """Create this rank's RCCL communicator through libspx.so.  ``unique_id``:
  the 128 bytes rank 0 made (``rccl_unique_id``); returns the handle."""
  lib = _lib()
  _check(lib.spx_comm_load(rccl_path().encode()), 'spx_comm_load')
  buf = (ctypes.c_uint8 * 128).from_buffer_copy(bytes(unique_id))
  comm = ctypes.c_void_p()
  _check(lib.spx_comm_init(buf, 128, int(rank), int(world), ctypes.byref(comm)), 'spx_comm_init')
  return comm


def rccl_unique_id():
  lib = _lib()
  _check(lib.spx_comm_load(rccl_path().encode()), 'spx_comm_load')
  buf = (ctypes.c_uint8 * 128)()
  _check(lib.spx_comm_unique_id(buf, 128), 'spx_comm_unique_id')
  return bytes(buf)


def rccl_destroy(comm):
  if comm is not None and comm.value:
    _check(_lib().spx_comm_destroy(comm), 'spx_comm_destroy')


def _contig(t, what):
  if not t.is_contiguous():
    raise ValueError('%s needs a contiguous tensor' % what)


# ---------------------------------------------------------------- SPMD guard
# Every rank must issue the same collectives in the same order (each rank
# computes the same tile plan); a divergence would otherwise show up as a hang
# inside RCCL / gloo.  Each collective (and each plan-cache decision) folds
# its name and shapes into a running CRC; the ranks compare it on the control
# plane -- before every collective with SPARTAN_SPMD_GUARD=strict (the tests),
# every N-th collective and at every barrier with SPARTAN_SPMD_GUARD=N (the
# default, 64), never with 0 -- and raise RuntimeError on a mismatch.
_GUARD = {'h': 0, 'n': 0, 'last': ()}


def _guard_every():
  v = os.environ.get('SPARTAN_SPMD_GUARD', '64').strip().lower()
  if v == 'strict':
    return 1
  try:
    return max(0, int(v))
  except ValueError:
    return 64


def spmd_note(*desc):
  """Fold ``desc`` (plain values) into this rank's running SPMD hash."""
  ctx = runtime._ctx
  if ctx is None or not ctx.distributed:
    return
  _GUARD['h'] = zlib.crc32(repr(desc).encode(), _GUARD['h'])
  _GUARD['n'] += 1
  _GUARD['last'] = desc


def spmd_check(where='check'):
  """Collective on the control plane: raise RuntimeError if the ranks'
  running hashes differ."""
  import torch
  ctx = runtime.get()
  if not ctx.distributed:
    return
  h = _GUARD['h']
  grp, dev = _ctl(ctx)
  t = torch.tensor([h, -h], dtype=torch.int64, device=dev)
  _dist().all_reduce(t, op=_dist().ReduceOp.MAX, group=grp)
  hi, lo = int(t[0].item()), -int(t[1].item())
  if hi != h or lo != h:
    raise RuntimeError('SPMD divergence at %s: rank %d issued a different sequence of collectives than '
                       'another rank (hash %08x, ranks span %08x..%08x after %d notes; last: %r)'
                       % (where, ctx.rank, h, lo, hi, _GUARD['n'], _GUARD['last']))


def _guard(*desc):
  spmd_note(*desc)
  every = _guard_every()
  if every and _GUARD['n'] % every == 0:
    spmd_check(desc[0])


def _tdesc(t):
  return (tuple(t.shape), str(t.dtype))


# ------------------------------------------------------------- collectives
def all_reduce(t, op):
  ctx = runtime.get()
  if not ctx.distributed:
    return t
  _guard('all_reduce', op, _tdesc(t))
  if ctx.dist_backend == 'rccl':
    _contig(t, 'all_reduce')
    _check(_lib().spx_allreduce(ctx.rccl, _p(t), _p(t), t.numel(), _dt(t), _SPX_OP[op], _stream()),
           'spx_allreduce')
    return t
  dist = _dist()
  if _staged(ctx, t):
    h = t.cpu()
    dist.all_reduce(h, op=getattr(dist.ReduceOp, _OPS[op]))
    t.copy_(h)
    return t
  dist.all_reduce(t, op=getattr(dist.ReduceOp, _OPS[op]), group=_grp())
  return t


def reduce_scatter_rows(out, full, op):
  """out = rank-th equal row slab of the element-wise reduction of ``full``."""
  ctx = runtime.get()
  _guard('reduce_scatter', op, _tdesc(out), _tdesc(full))
  if ctx.dist_backend == 'rccl':
    _contig(out, 'reduce_scatter')
    _contig(full, 'reduce_scatter')
    assert full.numel() == out.numel() * ctx.world_size
    _check(_lib().spx_reduce_scatter(ctx.rccl, _p(full), _p(out), out.numel(), _dt(out), _SPX_OP[op],
                                     _stream()), 'spx_reduce_scatter')
    return out
  dist = _dist()
  if ctx.dist_backend == 'gloo':  # gloo has no reduce_scatter: all_reduce + slice
    all_reduce(full, op)
    n = out.shape[0]
    out.copy_(full[ctx.rank * n:(ctx.rank + 1) * n])
    return out
  dist.reduce_scatter_tensor(out, full, op=getattr(dist.ReduceOp, _OPS[op]), group=_grp())
  return out


def all_gather_stack(t):
  """[world, *t.shape] stack of every rank's ``t`` (same shape on all ranks)."""
  import torch
  ctx = runtime.get()
  if not ctx.distributed:
    return t.unsqueeze(0)
  _guard('all_gather', _tdesc(t))
  out = torch.empty((ctx.world_size,) + tuple(t.shape), dtype=t.dtype, device=t.device)
  if ctx.dist_backend == 'rccl':
    t = t.contiguous()
    _check(_lib().spx_allgather(ctx.rccl, _p(t), _p(out), t.numel(), _dt(t), _stream()), 'spx_allgather')
    return out
  dist = _dist()
  if _staged(ctx, t):
    h = torch.empty(out.shape, dtype=t.dtype)
    dist.all_gather(list(h.unbind(0)), t.contiguous().cpu())
    out.copy_(h)
  elif ctx.dist_backend == 'gloo':
    dist.all_gather(list(out.unbind(0)), t.contiguous())
  else:
    dist.all_gather_into_tensor(out, t.contiguous(), group=_grp())
  return out


def broadcast(t, src_rank):
  ctx = runtime.get()
  if not ctx.distributed:
    return t
  _guard('broadcast', int(src_rank), _tdesc(t))
  if ctx.dist_backend == 'rccl':
    _contig(t, 'broadcast')
    _check(_lib().spx_broadcast(ctx.rccl, _p(t), _p(t), t.numel(), _dt(t), int(src_rank), _stream()),
           'spx_broadcast')
    return t
  if _staged(ctx, t):
    h = t.cpu()
    _dist().broadcast(h, src=src_rank)
    t.copy_(h)
    return t
  _dist().broadcast(t, src=src_rank, group=_grp())
  return t


class _Pending:
  """An RCCL reduce running on the side stream; ``wait`` makes the current
  stream wait for it (no host synchronisation)."""

  def __init__(self, event, keep):
    self.event = event
    self.keep = keep  # the tensor stays alive until the wait

  def wait(self):
    import torch
    torch.cuda.current_stream().wait_event(self.event)
    self.keep = None


def reduce_async(t, dst_rank, op):
  """Start reducing ``t`` (contiguous, same shape on every rank) into
  ``t`` on ``dst_rank``; returns a handle for ``wait_all``.  The reduction
  runs on a side stream, after the work already queued on the current
  stream and concurrently with what follows it."""
  ctx = runtime.get()
  _guard('reduce', int(dst_rank), op, _tdesc(t))
  if ctx.dist_backend == 'rccl':
    import torch
    _contig(t, 'reduce')
    cur = torch.cuda.current_stream()
    side = ctx.comm_stream()
    ready = torch.cuda.Event()
    ready.record(cur)
    side.wait_event(ready)
    _check(_lib().spx_reduce(ctx.rccl, _p(t), _p(t), t.numel(), _dt(t), _SPX_OP[op], int(dst_rank),
                             ctypes.c_void_p(side.cuda_stream)), 'spx_reduce')
    done = torch.cuda.Event()
    done.record(side)
    return _Pending(done, t)
  dist = _dist()
  if _staged(ctx, t):  # rehearsal: synchronous through the host
    h = t.cpu()
    dist.reduce(h, dst=dst_rank, op=getattr(dist.ReduceOp, _OPS[op]))
    if ctx.rank == dst_rank:
      t.copy_(h)
    return None
  return dist.reduce(t, dst=dst_rank, op=getattr(dist.ReduceOp, _OPS[op]), group=_grp(), async_op=True)


def wait_all(handles):
  for h in handles:
    if h is not None:
      h.wait()


class _Works:
  """torch.distributed async works; ``wait`` makes the current stream wait
  for them (NCCL works do not block the host)."""

  def __init__(self, works, keep):
    self.works = works
    self.keep = keep

  def wait(self):
    for w in self.works:
      w.wait()
    self.keep = None


def exchange_async(sends, recvs):
  """``exchange`` that runs beside the current stream: the messages start
  after the work already queued on it (the sends' producers) and run
  concurrently with what follows; returns a handle whose ``wait`` makes the
  current stream wait for the received tensors (``wait_all``), or None when
  the exchange already completed (gloo: host-staged, synchronous).  Same
  matching rules and SPMD contract as ``exchange``."""
  ctx = runtime.get()
  if not ctx.distributed:
    return None
  if ctx.dist_backend == 'gloo':
    exchange(sends, recvs)
    return None
  _guard('exchange')
  if not sends and not recvs:
    return None
  import torch
  sends = [(t.contiguous(), peer) for t, peer in sends]
  if ctx.dist_backend == 'rccl':
    cur = torch.cuda.current_stream()
    side = ctx.comm_stream()
    ready = torch.cuda.Event()
    ready.record(cur)
    side.wait_event(ready)
    with torch.cuda.stream(side):
      _exchange_rccl(sends, recvs)
    done = torch.cuda.Event()
    done.record(side)
    return _Pending(done, (sends, recvs))
  dist = _dist()
  g = _grp()
  ops = [dist.P2POp(dist.isend, t, peer, group=g) for t, peer in sends]
  ops += [dist.P2POp(dist.irecv, t, peer, group=g) for t, peer in recvs]
  return _Works(dist.batch_isend_irecv(ops), (sends, recvs))


def _exchange_rccl(sends, recvs):
  """spx_sendrecv of one batch on the current stream (libspx RCCL plane)."""
  ctx = runtime.get()
  for t, _ in recvs:
    _contig(t, 'exchange recv')
  ns, nr = len(sends), len(recvs)
  VP, I64, I32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
  sb = (VP * max(ns, 1))(*[t.data_ptr() for t, _ in sends])
  sn = (I64 * max(ns, 1))(*[t.numel() * t.element_size() for t, _ in sends])
  sp = (I32 * max(ns, 1))(*[int(p) for _, p in sends])
  rb = (VP * max(nr, 1))(*[t.data_ptr() for t, _ in recvs])
  rn = (I64 * max(nr, 1))(*[t.numel() * t.element_size() for t, _ in recvs])
  rp = (I32 * max(nr, 1))(*[int(p) for _, p in recvs])
  _check(_lib().spx_sendrecv(ctx.rccl, ns, sb, sn, sp, nr, rb, rn, rp, _stream()), 'spx_sendrecv')


def exchange(sends, recvs):
  """Point-to-point batch.  sends: [(tensor, dst_rank)], recvs: [(tensor, src_rank)].

  Every rank passes the pairs it takes part in; messages between the same pair
  of ranks are matched in list order."""
  ctx = runtime.get()
  if not ctx.distributed:
    return
  # every rank enters (the plans are identical); what each sends differs by
  # rank, so only the call itself is folded into the SPMD hash
  _guard('exchange')
  if not sends and not recvs:
    return
  import torch
  if ctx.dist_backend == 'rccl':
    _exchange_rccl([(t.contiguous(), peer) for t, peer in sends], recvs)
    return
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
  g = _grp()
  ops = [dist.P2POp(dist.isend, t.contiguous(), peer, group=g) for t, peer in sends]
  ops += [dist.P2POp(dist.irecv, t, peer, group=g) for t, peer in recvs]
  for req in dist.batch_isend_irecv(ops):
    req.wait()
  for t, h in post:
    t.copy_(h)


def _wait_device(dev, timeout):
  """Wait for the work queued on ``dev``'s current stream, at most ``timeout``
  s (an event polled from the host: a collective whose peer never arrives
  would block torch.cuda.synchronize for ever).  True when it finished."""
  import time
  import torch
  if dev.type != 'cuda':
    return True
  ev = torch.cuda.Event()
  ev.record(torch.cuda.current_stream(dev))
  end = time.monotonic() + timeout
  while not ev.query():
    if time.monotonic() > end:
      return False
    time.sleep(0.001)
  return True


def selftest(timeout=None):
  """Exercise every collective of the data plane once on small tensors and
  check the results on the host; returns None, or a description of the first
  wrong result / error.  All ranks call it (collective) and all get the same
  verdict (a max over ranks on the control plane).  runtime.initialize runs
  it on the libspx RCCL communicator before any tile data moves, and falls
  back to torch.distributed's own RCCL group if it fails.

  Every rank issues every collective even after one of its own calls raised
  (each call in its own try), so the ranks stay in step; the device wait is
  bounded (``SPARTAN_SELFTEST_TIMEOUT`` s, default 60); the SPMD guard's
  running hash is restored afterwards, so a rank that failed part-way does
  not leave the ranks' hashes different."""
  import torch
  ctx = runtime.get()
  if not ctx.distributed:
    return None
  if timeout is None:
    timeout = float(os.environ.get('SPARTAN_SELFTEST_TIMEOUT', '60'))
  W, r = ctx.world_size, ctx.rank
  dev = ctx.device
  saved = dict(_GUARD)
  errs = []
  checks = []

  def call(name, fn):
    try:
      fn()
    except Exception as e:  # noqa: BLE001  (reported to the caller, which decides)
      errs.append('%s: %s: %s' % (name, type(e).__name__, e))

  base = torch.arange(4 * W, dtype=torch.float32, device=dev)
  t = base + float(r)
  call('all_reduce(sum)', lambda: all_reduce(t, 'sum'))
  checks.append(('all_reduce(sum)', t, W * torch.arange(4 * W, dtype=torch.float64) + W * (W - 1) / 2.0))
  full = base.double() * (r + 1)
  out = torch.zeros((4,), dtype=torch.float64, device=dev)
  call('reduce_scatter(sum)', lambda: reduce_scatter_rows(out, full, 'sum'))
  checks.append(('reduce_scatter(sum)', out,
                 torch.arange(4 * W, dtype=torch.float64)[4 * r:4 * r + 4] * (W * (W + 1) / 2.0)))
  mx = torch.full((3,), float(r), dtype=torch.float64, device=dev)
  call('all_reduce(max)', lambda: all_reduce(mx, 'max'))
  checks.append(('all_reduce(max)', mx, torch.full((3,), float(W - 1), dtype=torch.float64)))
  g = [torch.zeros((W, 3), dtype=torch.int64, device=dev)]

  def gather():
    g[0] = all_gather_stack(torch.full((3,), r, dtype=torch.int64, device=dev))
  call('all_gather', gather)
  b = torch.full((5,), 7 * r + 1, dtype=torch.int64, device=dev)
  call('broadcast', lambda: broadcast(b, W - 1))
  checks.append(('broadcast', b, torch.full((5,), 7 * (W - 1) + 1, dtype=torch.int64)))
  src = torch.full((6,), 10 * r + 3, dtype=torch.int32, device=dev)
  dst = torch.zeros((6,), dtype=torch.int32, device=dev)
  call('send/recv', lambda: exchange([(src, (r + 1) % W)], [(dst, (r - 1) % W)]))
  checks.append(('send/recv', dst, torch.full((6,), 10 * ((r - 1) % W) + 3, dtype=torch.int32)))
  err = errs[0] if errs else None
  if not _wait_device(dev, timeout):
    err = err or 'the collectives did not complete within %g s' % timeout
  else:
    checks.insert(3, ('all_gather', g[0], torch.arange(W, dtype=torch.int64).repeat_interleave(3).view(W, 3)))
    for name, got, want in checks:
      if err is None and not torch.equal(got.cpu().to(want.dtype), want):
        err = '%s wrong' % name
  _GUARD.clear()
  _GUARD.update(saved)
  bad = max_over_ranks(1.0 if err else 0.0)
  if bad and err is None:
    err = 'another rank failed'
  return err


def barrier():
  """Host barrier over the control plane (callers synchronise their device
  streams around it)."""
  ctx = runtime.get()
  if ctx.distributed:
    if _guard_every():
      spmd_check('barrier')
    _dist().barrier()


def max_over_ranks(x):
  """Max of a host float over all ranks (bench timing), on the control plane."""
  import torch
  ctx = runtime.get()
  if not ctx.distributed:
    return x
  grp, dev = _ctl(ctx)
  t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
  _dist().all_reduce(t, op=_dist().ReduceOp.MAX, group=grp)
  return float(t.item())
