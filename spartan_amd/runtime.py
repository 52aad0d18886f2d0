"""Per-process runtime: which GPU this rank drives and who owns which worker.

Replaces the reference's master/worker cluster (spartan/cluster.py:120-164,
spartan/master.py, spartan/worker.py, spartan/blob_ctx.py) with the MI355X
execution model: ONE process per GPU, launched by torchrun, all processes
running the same (SPMD) program.  A tile *worker* index (the reference's
``TileId.worker``, spartan/core.pyx:16-41) is owned by rank ``worker % world``.
Every rank computes the same tile plan, runs the kernels for the tiles it owns
on its own GPU, and exchanges data only through RCCL collectives over xGMI
issued through libspx.so's C ABI (comm.py); torch.distributed (gloo) is the
host control plane, and gloo alone carries the CPU-only tests.
"""
import os

from .config import FLAGS

_ctx = None


class Context:
  def __init__(self, rank, world_size, local_rank, device, dist_backend, rccl=None):
    self.rank = rank
    self.world_size = world_size
    self.local_rank = local_rank
    self.device = device
    self.dist_backend = dist_backend   # data plane: 'rccl' (libspx), 'gloo' (tests / rehearsal), 'nccl' (torch)
    self.rccl = rccl                   # libspx RCCL communicator handle when dist_backend == 'rccl'
    self._comm_stream = None
    self.pg = None          # torch process group of the data plane when dist_backend == 'nccl' (None: default)
    self.selftest = None    # data-plane self-test verdict at start-up (multi-rank RCCL only)
    self.num_workers = int(FLAGS.num_workers or world_size)
    if self.num_workers < 1:
      raise ValueError('num_workers must be >= 1')

  def comm_stream(self):
    """Side HIP stream for collectives that overlap compute (dot slab reduces)."""
    if self._comm_stream is None:
      import torch
      self._comm_stream = torch.cuda.Stream(device=self.device)
    return self._comm_stream

  # reference blob_ctx.BlobCtx.num_workers semantics
  def owner(self, worker):
    return worker % self.world_size

  def is_local(self, worker):
    return self.owner(worker) == self.rank

  def is_master(self):
    return self.rank == 0

  @property
  def distributed(self):
    return self.world_size > 1

  def __repr__(self):
    return 'Context(rank=%d/%d, device=%s, workers=%d)' % (self.rank, self.world_size, self.device,
                                                            self.num_workers)


def initialize(argv=None, device=None):
  """Bring up this rank (reference spartan.initialize, spartan/__init__.py:42-56).

  Reads RANK / WORLD_SIZE / LOCAL_RANK from the torchrun environment and
  selects cuda:LOCAL_RANK.  With more than one rank on GPUs the data plane
  is, by default, torch.distributed's own RCCL process group ('nccl' -- the
  same librccl, the collective path PyTorch validates on every multi-GPU
  job).  ``SPARTAN_DIST_BACKEND=rccl`` opts in to the libspx.so C-ABI
  communicator instead (spx_comm_init; every device collective a C-ABI call,
  comm.py; torch.distributed then runs gloo as the host control plane: the
  unique-id hand-off, barriers, host maxima), checked by a start-up
  self-test that falls back to the torch group.  It stays opt-in until a
  multi-GPU run has validated it (so far it has run at world 1 only).
  ``SPARTAN_DIST_BACKEND=gloo`` rehearses N ranks on fewer GPUs (device
  tensors staged through the host).  ``device`` overrides the device (tests
  run the host logic on 'cpu' with a test backend and gloo)."""
  global _ctx
  import torch
  if argv is not None:
    FLAGS.parse(list(argv))
  world = int(os.environ.get('WORLD_SIZE', '1'))
  rank = int(os.environ.get('RANK', '0'))
  local_rank = int(os.environ.get('LOCAL_RANK', str(rank)))
  if device is None:
    if not torch.cuda.is_available():
      raise RuntimeError('spartan_amd needs a ROCm GPU (torch.cuda.is_available() is False)')
    device = torch.device('cuda', local_rank % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(device)
  device = torch.device(device)
  backend = None
  rccl = None
  if world > 1:
    import torch.distributed as dist
    backend = os.environ.get('SPARTAN_DIST_BACKEND', 'nccl' if device.type == 'cuda' else 'gloo')
    if backend not in ('nccl', 'rccl', 'gloo'):
      raise ValueError('SPARTAN_DIST_BACKEND must be nccl, rccl or gloo, not %r' % backend)
    if backend == 'rccl' and os.environ.get('SPARTAN_COMM') == 'torch':
      backend = 'nccl'
    pg = 'nccl' if backend == 'nccl' else 'gloo'   # torch.distributed: control plane (or the torch RCCL path)
    if not dist.is_initialized():
      os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
      kw = {}
      if device.type == 'cuda' and pg == 'nccl':
        kw['device_id'] = device
      dist.init_process_group(backend=pg, rank=rank, world_size=world, **kw)
    if backend == 'rccl':
      from . import comm
      obj = [comm.rccl_unique_id() if rank == 0 else None]
      dist.broadcast_object_list(obj, src=0)
      rccl = comm.rccl_init(rank, world, obj[0])
  _ctx = Context(rank, world, local_rank, device, backend, rccl)
  if backend == 'rccl' and os.environ.get('SPARTAN_RCCL_SELFTEST', '1') != '0':
    # every collective of the libspx data plane, once, on small tensors,
    # checked on the host before any tile moves; a wrong result or an error
    # moves the data plane to torch.distributed's own RCCL group (loudly)
    from . import comm
    err = comm.selftest()
    _ctx.selftest = err or 'ok'
    if err:
      import warnings
      warnings.warn('spartan_amd: the libspx RCCL data plane failed its self-test (%s); '
                    'using torch.distributed\'s RCCL process group instead' % err)
      import torch.distributed as dist
      _ctx.pg = dist.new_group(backend='nccl')
      _ctx.dist_backend = 'nccl'
      _ctx.rccl = None  # not destroyed: a communicator in an unknown state may block in ncclCommDestroy
      bad = comm.selftest()
      if bad:
        raise RuntimeError('spartan_amd: no working GPU data plane (libspx RCCL: %s; torch RCCL: %s)' % (err, bad))
  return _ctx


def shutdown():
  global _ctx
  if _ctx is not None and _ctx.distributed:
    import torch.distributed as dist
    if _ctx.rccl is not None:
      import torch
      from . import comm
      torch.cuda.synchronize(_ctx.device)
      comm.rccl_destroy(_ctx.rccl)
      _ctx.rccl = None
    if dist.is_initialized():
      dist.barrier()
      dist.destroy_process_group()
  _ctx = None


def get():
  if _ctx is None:
    initialize()
  return _ctx


def set_context(ctx):
  global _ctx
  prev = _ctx
  _ctx = ctx
  return prev
