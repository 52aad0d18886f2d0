"""Per-process runtime: which GPU this rank drives and who owns which worker.

Replaces the reference's master/worker cluster (spartan/cluster.py:120-164,
spartan/master.py, spartan/worker.py, spartan/blob_ctx.py) with the MI355X
execution model: ONE process per GPU, launched by torchrun, all processes
running the same (SPMD) program.  A tile *worker* index (the reference's
``TileId.worker``, spartan/core.pyx:16-41) is owned by rank ``worker % world``.
Every rank computes the same tile plan, runs the kernels for the tiles it owns
on its own GPU, and exchanges data through RCCL collectives over xGMI.  By
default (world > 1 on GPUs) they run on torch.distributed's RCCL process group
(backend 'nccl' = RCCL on ROCm); ``SPARTAN_DIST_BACKEND=rccl`` issues them
through libspx.so's C ABI instead (``spx_allreduce`` & co., comm.py) on a
communicator this module creates, with torch.distributed (gloo) as the host
control plane and a start-up self-test that falls back to torch's RCCL group
if that communicator cannot be created or computes a wrong result.  The libspx
communicator stays opt-in until a multi-GPU run has validated it (it has
completed collectives at world 1 only).  gloo alone carries the CPU-only
tests.
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
    self.selftest = None    # data-plane self-test verdict at start-up (every multi-rank data plane)
    self.ctl = None         # gloo group of the control plane when the default group is nccl (None: default)
    self.pg_timeout = None  # seconds: the process groups' collective timeout (world > 1)
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


def data_plane(device_type, env=None):
  """The device-collective backend a multi-rank run starts with: 'nccl'
  (torch.distributed's RCCL group) on GPUs unless SPARTAN_DIST_BACKEND names
  another ('rccl': the libspx C-ABI communicator, self-tested at start-up
  with a fallback to 'nccl'; 'gloo': host-staged rehearsal); 'gloo' for CPU
  devices (tests).  A collective that hangs on the libspx communicator keeps
  its HIP stream blocked, so no fallback can rescue it: that is why 'rccl'
  stays opt-in until a multi-GPU run has shown selftest='ok' with correct
  results."""
  env = os.environ if env is None else env
  backend = env.get('SPARTAN_DIST_BACKEND', 'nccl' if device_type == 'cuda' else 'gloo')
  if backend not in ('nccl', 'rccl', 'gloo'):
    raise ValueError('SPARTAN_DIST_BACKEND must be nccl, rccl or gloo, not %r' % backend)
  if backend == 'rccl' and (env.get('SPARTAN_COMM') == 'torch' or device_type != 'cuda'):
    backend = 'nccl' if device_type == 'cuda' else 'gloo'
  return backend


class DataPlaneError(RuntimeError):
  """The multi-rank data plane failed its start-up self-test (the message
  names the first failing collective)."""


def pg_timeout_s(env=None):
  """Timeout (s) of the torch.distributed process groups: a collective that
  never completes aborts the job after this long instead of torch's default
  (``SPARTAN_NCCL_TIMEOUT``, default 300)."""
  env = os.environ if env is None else env
  t = float(env.get('SPARTAN_NCCL_TIMEOUT', '300'))
  if not t > 0:
    raise ValueError('SPARTAN_NCCL_TIMEOUT must be > 0, not %r' % env.get('SPARTAN_NCCL_TIMEOUT'))
  return t


def _rccl_init_bounded(comm, rank, world, uid, device, timeout):
  """spx_comm_init on a helper thread, waited for at most ``timeout`` s.

  ncclCommInitRank blocks until every rank has joined; a rank that never
  arrives (or a transport that never connects) would block this process for
  ever.  The call releases the GIL (ctypes), so the main thread can give up
  and report instead; the helper thread is left behind (a daemon) -- the
  communicator it may still produce is never used.  Returns (handle, error)."""
  import threading
  box = {}

  def run():
    try:
      import torch
      if device.type == 'cuda':
        torch.cuda.set_device(device)  # RCCL binds the calling thread's current device
      box['comm'] = comm.rccl_init(rank, world, uid)
    except Exception as e:  # noqa: BLE001  (reported to the caller)
      box['err'] = '%s: %s' % (type(e).__name__, e)

  th = threading.Thread(target=run, name='spx_comm_init', daemon=True)
  th.start()
  th.join(timeout)
  if th.is_alive():
    return None, 'spx_comm_init did not return within %g s' % timeout
  return box.get('comm'), box.get('err')


def initialize(argv=None, device=None):
  """Bring up this rank (reference spartan.initialize, spartan/__init__.py:42-56).

  Reads RANK / WORLD_SIZE / LOCAL_RANK from the torchrun environment and
  selects cuda:LOCAL_RANK.  With more than one rank on GPUs the data plane
  is, by default, torch.distributed's RCCL process group (``'nccl'``; the
  control plane then gets its own gloo group).  ``SPARTAN_DIST_BACKEND=rccl``
  selects libspx.so's C-ABI RCCL communicator (spx_comm_init, every device
  collective an ``spx_*`` call, comm.py), with torch.distributed running gloo
  as the host control plane (the unique-id hand-off, barriers, host maxima,
  the SPMD guard).  That communicator's creation is bounded
  (``SPARTAN_RCCL_INIT_TIMEOUT`` s, default 120) and a start-up self-test
  checks every collective on every rank; if either fails on any rank, all
  ranks switch the device collectives to torch.distributed's own RCCL process
  group (loudly) and re-run the test on a fresh stream -- a collective that
  HANGS on the libspx communicator is fatal (its stream stays blocked).
  ``SPARTAN_DIST_BACKEND=gloo`` rehearses N ranks on fewer GPUs (device
  tensors staged through the host).
  ``device`` overrides the device (tests run the host logic on 'cpu' with a
  test backend and gloo)."""
  global _ctx
  import datetime
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
  init_err = None
  ctl = None
  pg_timeout = pg_timeout_s()
  if world > 1:
    import torch.distributed as dist
    backend = data_plane(device.type)
    pg = 'nccl' if backend == 'nccl' else 'gloo'   # torch.distributed: control plane (or the torch RCCL path)
    if not dist.is_initialized():
      os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
      kw = {'timeout': datetime.timedelta(seconds=pg_timeout)}
      if device.type == 'cuda' and pg == 'nccl':
        kw['device_id'] = device
      dist.init_process_group(backend=pg, rank=rank, world_size=world, **kw)
    if dist.get_backend() == 'nccl':
      # the SPMD guard and host maxima never share the data plane's communicator
      ctl = dist.new_group(backend='gloo', timeout=datetime.timedelta(seconds=pg_timeout))
    if backend == 'rccl':
      from . import comm
      obj = [None]
      if rank == 0:
        try:
          obj = [comm.rccl_unique_id()]
        except Exception as e:  # noqa: BLE001
          obj = ['error: %s' % e]
      dist.broadcast_object_list(obj, src=0)
      if isinstance(obj[0], bytes):
        rccl, init_err = _rccl_init_bounded(comm, rank, world, obj[0], device,
                                            float(os.environ.get('SPARTAN_RCCL_INIT_TIMEOUT', '120')))
      else:
        init_err = 'rank 0 could not make an RCCL unique id (%s)' % obj[0]
  _ctx = Context(rank, world, local_rank, device, backend, rccl)
  _ctx.ctl = ctl
  if world > 1:
    _ctx.pg_timeout = pg_timeout
  if world > 1 and backend != 'rccl' and os.environ.get('SPARTAN_SELFTEST', '1') != '0':
    # the default data plane (torch's RCCL group; gloo in the CPU tests) is
    # checked the same way before any tile moves: every collective once,
    # bounded, the verdict agreed over ranks -- a failure names the
    # collective and stops the run here instead of in the first tile
    # exchange (which would sit until the process group's timeout)
    from . import comm
    err = comm.selftest()
    _ctx.selftest = err or 'ok'
    if err:
      raise DataPlaneError('spartan_amd: the %s data plane failed its start-up self-test: %s' % (backend, err))
  if backend == 'rccl':
    from . import comm
    # every rank learns whether any rank's communicator failed to come up
    bad = comm.max_over_ranks(1.0 if init_err or rccl is None else 0.0)
    err = init_err or ('another rank could not create its RCCL communicator' if bad else None)
    if err is None and os.environ.get('SPARTAN_RCCL_SELFTEST', '1') != '0':
      # every collective of the libspx data plane, once, on small tensors,
      # checked on the host before any tile moves
      err = comm.selftest()
    _ctx.selftest = err or 'ok'
    if err:
      _fall_back_to_torch_rccl(err)
  return _ctx


def _fall_back_to_torch_rccl(err):
  """Move the device collectives to torch.distributed's own RCCL group after
  the libspx communicator failed (``err``); raise if that group fails too."""
  import warnings
  import torch.distributed as dist
  from . import comm
  warnings.warn('spartan_amd: the libspx RCCL data plane failed (%s); using torch.distributed\'s RCCL '
                'process group instead' % err)
  _ctx.pg = dist.new_group(backend='nccl')
  _ctx.dist_backend = 'nccl'
  _ctx.rccl = None  # not destroyed: a communicator in an unknown state may block in ncclCommDestroy
  import torch
  if _ctx.device.type == 'cuda':
    # a fresh stream: the failed test's work may still sit on the current one
    with torch.cuda.stream(torch.cuda.Stream(device=_ctx.device)):
      bad = comm.selftest()
  else:
    bad = comm.selftest()
  _ctx.selftest = 'fallback (%s)' % err
  if bad:
    raise RuntimeError('spartan_amd: no working GPU data plane (libspx RCCL: %s; torch RCCL: %s)' % (err, bad))


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
