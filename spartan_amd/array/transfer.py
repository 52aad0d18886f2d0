"""Host <-> HBM movement for ingest (``from_numpy``, ``write``, ``update``)
and egress (``glom``).

The reference ships NumPy tiles to workers over its RPC layer
(write_array.py:411-433 -> distarray.py:370-421 -> worker update) and
pickles fetched tiles back to the master for ``glom`` (distarray.py:246-266).
Here the hop is PCIe between host memory and HBM.  Measured on MI355X
(tools/xfer_bench.py, 1 GiB fp32, profiles/r01_xfer.txt):

  * a C-contiguous piece moves straight from / into pageable memory at
    56 GB/s each way (the driver's direct path) -- used as is;
  * a strided piece (a column tile of a row-major matrix, a page range of an
    ``np.load(mmap_mode='r')`` file sliced by columns) packed by NumPy and
    then copied runs at 7.6 GB/s H2D, and ``.cpu()`` + a scatter into the
    ``glom`` result at 5.4 GB/s D2H.

Strided pieces therefore move in row blocks of ``CHUNK`` bytes through two
pinned staging buffers on a dedicated copy stream: the CPU gathers block
i+1 into one buffer (the only host copy, straight from the strided source,
split over ``THREADS`` host threads) while the DMA engine moves block i out
of the other (37.5 GB/s H2D).  ``download`` is the mirror image: block i+1's
D2H DMA is in flight while the CPU scatters block i into the destination
(38.7 GB/s).  The consuming stream waits on the copy stream with an event,
so kernels that read an uploaded tile are ordered after it without a host
synchronisation.  Pieces under ``SMALL`` bytes, and CPU runs of the
test-double backend, take the plain copy.
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

CHUNK = 16 << 20   # bytes per staging block
SMALL = 1 << 20    # below this a plain copy is cheaper than the pipeline
# C-contiguous pieces / destinations go straight between pageable memory and
# HBM: the driver's direct path measured 56 GB/s each way on MI355X against
# 42-46 GB/s staged (profiles/r01_xfer.txt); strided ones take the pipeline
DIRECT_H2D = True
DIRECT_D2H = True
THREADS = max(1, min(8, int(os.environ.get('OMP_NUM_THREADS', '8') or 8)))

_stages = {}
_pool = None


def _par_copy(dst, src):
  """np.copyto split over host threads along axis 0 (NumPy releases the GIL
  for plain dtypes, so the gathers of one block run in parallel)."""
  global _pool
  rows = dst.shape[0]
  if THREADS == 1 or rows < 2 or dst.nbytes < (2 << 20):
    np.copyto(dst, src, casting='no')
    return
  if _pool is None:
    _pool = ThreadPoolExecutor(THREADS)
  step = -(-rows // THREADS)
  futs = [_pool.submit(np.copyto, dst[r:r + step], src[r:r + step], casting='no')
          for r in range(0, rows, step)]
  for f in futs:
    f.result()


class _Stage:
  """Two pinned host blocks, their events and a copy stream for one device."""

  def __init__(self, device):
    import torch
    self.stream = torch.cuda.Stream(device=device)
    self.bufs = [torch.empty(CHUNK, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    self.views = [b.numpy() for b in self.bufs]
    self.events = [torch.cuda.Event() for _ in range(2)]
    self.used = [False, False]


def _stage(device):
  key = (device.type, device.index)
  st = _stages.get(key)
  if st is None:
    st = _stages[key] = _Stage(device)
  return st


def _blocks(shape, itemsize):
  """Row blocks (r0, r1) along axis 0 of at most CHUNK bytes, or None when a
  single row is larger than a block (then the piece is moved flat)."""
  rows = shape[0]
  row_bytes = itemsize * int(np.prod(shape[1:], dtype=np.int64))
  if row_bytes == 0 or row_bytes > CHUNK:
    return None
  per = max(1, CHUNK // row_bytes)
  return [(r, min(rows, r + per)) for r in range(0, rows, per)], row_bytes


# dtypes the pinned ring uploads (native byte order, the backend's own
# types); anything else (float16, int8, big-endian ...) takes the plain path
_TINY_DTYPES = tuple(np.dtype(t) for t in (np.bool_, np.int32, np.int64, np.float32, np.float64))


# Upload aliases: a producer that has already computed on the device the
# values the host is about to upload (examples/kmeans.py: the next k-means
# centres, divided on the device exactly as the host divides) registers that
# tensor with a host copy of it; the next upload of an array bit-identical to
# that copy returns the tensor instead of copying (a synchronous pageable H2D
# would wait behind the work already queued).  One-shot: the next upload of
# any array takes the entry.  The registered tensor must not be written
# afterwards (the producer hands it over).
_ALIAS = {}


def register_upload_alias(host, dev, event):
  """``host``: an ndarray holding ``dev``'s values once ``event`` completes."""
  _ALIAS['a'] = (host, dev, event)


def _take_alias(arr, device):
  host, dev, ev = _ALIAS.pop('a')
  if dev.device != device or arr.dtype != host.dtype or arr.size != host.size or tuple(dev.shape) != arr.shape:
    return None
  ev.synchronize()
  a = np.ascontiguousarray(arr)
  if not np.array_equal(a.reshape(-1).view(np.uint8), host.reshape(-1).view(np.uint8)):
    return None
  return dev


def upload(arr, device, dtype=None):
  """Device tensor holding ``arr`` (any strides, memmaps included)."""
  import torch
  from .. import backend
  arr = np.asarray(arr) if dtype is None else np.asarray(arr, dtype=dtype)
  if not arr.dtype.isnative:  # torch takes native byte order only
    arr = arr.astype(arr.dtype.newbyteorder('='))
  if _ALIAS and device.type == 'cuda':
    hit = _take_alias(arr, device)
    if hit is not None:
      return hit
  if device.type == 'cuda' and arr.nbytes <= TINY and arr.dtype in _TINY_DTYPES:
    return _tiny_upload(arr, device)
  if device.type != 'cuda' or arr.ndim == 0 or arr.nbytes < SMALL or (
      arr.flags.c_contiguous and DIRECT_H2D):
    host = np.ascontiguousarray(arr)
    if not host.flags.writeable or host is arr and device.type != 'cuda':
      host = host.copy()  # a read-only memmap, or a caller's array a CPU tile must not alias
    return torch.as_tensor(host).to(device)
  out = torch.empty(arr.shape, dtype=backend.torch_dtype(arr.dtype), device=device)
  plan = _blocks(arr.shape, arr.itemsize)
  if plan is None:  # rows wider than a block: move it as a flat vector
    arr = np.ascontiguousarray(arr).reshape(-1)
    plan = _blocks(arr.shape, arr.itemsize)
  blocks, row_bytes = plan
  dst = out.view(-1).view(torch.uint8)
  st = _stage(device)
  with torch.cuda.stream(st.stream):
    for i, (r0, r1) in enumerate(blocks):
      k = i & 1
      if st.used[k]:
        st.events[k].synchronize()  # the DMA that last read this block is done
      nb = (r1 - r0) * row_bytes
      _par_copy(st.views[k][:nb].view(arr.dtype).reshape((r1 - r0,) + arr.shape[1:]), arr[r0:r1])
      dst[r0 * row_bytes:r1 * row_bytes].copy_(st.bufs[k][:nb], non_blocking=True)
      st.events[k].record(st.stream)
      st.used[k] = True
  out.record_stream(st.stream)
  torch.cuda.current_stream(device).wait_stream(st.stream)
  return out


# host arrays up to this size go through a pinned ring (an iterative
# driver's w, 256 B at cfg5).  (Round 6: raised to 1 MiB for the k-means
# centres, the 256 KiB copy into the pinned slot took 0.13 ms against 0.04
# for the pageable upload -- gpurun_out/r6o -- so it stays at 4 KiB.)
TINY = 4096
_TINY_RING = 8
_tiny = {}


def _tiny_upload(arr, device):
  """Small host array -> device through a ring of pinned slots: an async
  copy on the current stream (a pageable copy blocks the host for the
  driver's staging round trip; lreg uploads its (64, 1) w every iteration).
  A slot is reused only after the copy that last read it has completed."""
  import torch
  from .. import backend
  key = (device.type, device.index)
  ring = _tiny.get(key)
  if ring is None:
    ring = _tiny[key] = {'pos': 0, 'slots': [(torch.empty(TINY, dtype=torch.uint8, pin_memory=True), torch.cuda.Event())
                                             for _ in range(_TINY_RING)], 'used': [False] * _TINY_RING}
  k = ring['pos']
  ring['pos'] = (k + 1) % _TINY_RING
  buf, ev = ring['slots'][k]
  if ring['used'][k]:
    ev.synchronize()
  host = np.ascontiguousarray(arr)
  nb = host.nbytes
  buf.numpy()[:nb] = host.reshape(-1).view(np.uint8)
  out = torch.empty(host.shape, dtype=backend.torch_dtype(host.dtype), device=device)
  if nb:
    out.view(-1).view(torch.uint8).copy_(buf[:nb], non_blocking=True)
  ev.record()
  ring['used'][k] = True
  return out


# Host shadows: a producer that knows the host will read a device tensor and
# is about to queue long work behind it (examples/kmeans.py: the next k-means
# step, queued before the host has read this iteration's centre sums) copies
# the tensor to pinned memory first and attaches the copy here; the next
# download of THAT tensor, unmodified since (same object, same torch version
# counter), waits for that copy instead of queueing its own behind the work.
# One-shot: the entry is taken by the first download that looks for it.
_SHADOWS = {}


def attach_shadow(t, host, event):
  """``host`` (an ndarray of t's shape and dtype) holds t's current values
  once ``event`` has completed."""
  import weakref
  _SHADOWS[id(t)] = (weakref.ref(t), t._version, host, event)


def _take_shadow(t):
  e = _SHADOWS.pop(id(t), None)
  if e is None:
    return None
  ref, ver, host, ev = e
  if ref() is not t or t._version != ver:
    return None
  ev.synchronize()
  return host


def download(t, out=None):
  """Copy device tensor ``t`` into host array ``out`` (any strides; a new
  C-order array when None) and return it."""
  import torch
  from .. import backend
  shape = tuple(t.shape)
  if out is None:
    out = np.empty(shape, dtype=backend.np_dtype(t.dtype))
  if _SHADOWS:
    h = _take_shadow(t)
    if h is not None:
      out[...] = h.reshape(out.shape)
      return out
  if t.device.type != 'cuda' or t.dim() == 0 or t.numel() * t.element_size() < SMALL:
    out[...] = t.cpu().numpy().reshape(out.shape)
    return out
  if not t.is_contiguous():
    t = backend.get().contiguous(t)
  if out.flags.c_contiguous and out.flags.writeable and DIRECT_D2H:
    torch.from_numpy(out).copy_(t.reshape(out.shape))  # straight into pageable memory (measured fastest)
    return out
  plan = _blocks(shape, t.element_size())
  view = out
  if plan is None:
    if not out.flags.c_contiguous:
      tmp = download(t.reshape(-1))
      out[...] = tmp.reshape(out.shape)
      return out
    view = out.reshape(-1)
    plan = _blocks(view.shape, t.element_size())
  blocks, row_bytes = plan
  src = t.reshape(-1).view(torch.uint8)
  dt = out.dtype
  st = _stage(t.device)
  st.stream.wait_stream(torch.cuda.current_stream(t.device))  # t is produced on the compute stream
  t.record_stream(st.stream)

  def issue(i):
    r0, r1 = blocks[i]
    k = i & 1
    with torch.cuda.stream(st.stream):
      st.bufs[k][:(r1 - r0) * row_bytes].copy_(src[r0 * row_bytes:r1 * row_bytes], non_blocking=True)
      st.events[k].record(st.stream)
      st.used[k] = True

  issue(0)
  if len(blocks) > 1:
    issue(1)
  for i, (r0, r1) in enumerate(blocks):
    k = i & 1
    st.events[k].synchronize()
    nb = (r1 - r0) * row_bytes
    _par_copy(view[r0:r1], st.views[k][:nb].view(dt).reshape((r1 - r0,) + view.shape[1:]))
    if i + 2 < len(blocks):
      issue(i + 2)
  return out
