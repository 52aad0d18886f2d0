"""CPU baseline (ORACLE, test/bench infrastructure): the reference's
multi-worker execution model restated with NumPy worker processes.

W worker processes each own one row-strip tile (good_tile_shape with
num_workers = W, spartan/array/distarray.py:24-46) that they generate
themselves and keep resident, like the reference's workers.  A step sends one
"run kernel" request per worker (BlobCtx.map, spartan/blob_ctx.py:256-275);
each worker evaluates the tile exactly as the reference's mappers do -- one
NumPy call per LocalExpr node with materialised temporaries
(spartan/expr/local.py:110-122) -- and the master merges the partials in tile
order with np.add (tile.merge, tile.pyx:201-298).  Input tiles never cross
process boundaries (no pickling of tiles, no ZeroMQ): a best case for the
reference; partials travel to the owner over a pipe (pickled), as the
reference's UpdateReqs do over ZeroMQ.

Workers are started with the 'spawn' method and OMP_NUM_THREADS /
OPENBLAS_NUM_THREADS / MKL_NUM_THREADS = 1 in their environment BEFORE they
import NumPy (one BLAS thread per worker, one worker per core: the
reference's worker.py:40-41 / cluster.py:54 model).  W is the host's
physical core count, capped by the CPU share this process may use (its
affinity mask and cgroup quota: on the shared GPU box a job's share is 16
CPUs of a much larger machine); ``host_info`` records every number that went
into it.  A single-process NumPy time (default BLAS threading) is reported
next to the W-worker time.

Legs (reference wall-clock anchors in
tests/test_performance.py:42-99):
  cfg2    sum(x*y+exp(z), axis 0) + (axis 1) on row strips;
  dot     K-split dot (dot.py:268-283, map.py:285-330): worker i multiplies
          A[:, K_i] by B[K_i, :] with NumPy BLAS, partials summed at the owner;
  lreg    linear_regression.py:10-16: GEMV per strip (dot_map2_np_mapper,
          dot.py:172-187), x * (yp - y), sum(axis=0), merged at the owner;
  kmeans  k_means_.py:125-152 'outer': cdist + argmin per strip (scipy fp64),
          bincount and per-centre sums per strip, merged at the owner.
"""
import multiprocessing as mp
import os
import time

import numpy as np

from . import rng

_ONE_THREAD = {'OMP_NUM_THREADS': '1', 'OPENBLAS_NUM_THREADS': '1', 'MKL_NUM_THREADS': '1'}


# ---------------------------------------------------------------- host facts
def _cgroup_cpus():
  try:
    with open('/sys/fs/cgroup/cpu.max') as f:
      q, p = f.read().split()[:2]
    if q != 'max':
      return max(1, int(int(q) // int(p)))
  except (OSError, ValueError):
    pass
  try:
    with open('/sys/fs/cgroup/cpu/cpu.cfs_quota_us') as f:
      q = int(f.read())
    with open('/sys/fs/cgroup/cpu/cpu.cfs_period_us') as f:
      p = int(f.read())
    if q > 0:
      return max(1, q // p)
  except (OSError, ValueError):
    pass
  return None


def host_info(share_cap=16):
  """nproc, affinity, cgroup quota, lscpu-style model / physical cores, and
  the worker count W derived from them."""
  model, phys = None, set()
  try:
    with open('/proc/cpuinfo') as f:
      pid = core = None
      for line in f:
        if line.startswith('model name') and model is None:
          model = line.split(':', 1)[1].strip()
        elif line.startswith('physical id'):
          pid = line.split(':', 1)[1].strip()
        elif line.startswith('core id'):
          core = line.split(':', 1)[1].strip()
          phys.add((pid, core))
  except OSError:
    pass
  nproc = os.cpu_count()
  try:
    aff = len(os.sched_getaffinity(0))
  except AttributeError:
    aff = nproc
  cg = _cgroup_cpus()
  physical = len(phys) or nproc
  w = min(physical, aff, cg or aff)
  cap_note = None
  if share_cap and w > share_cap and os.environ.get('GRAFT_REPO_ROOT'):
    # on the shared GPU box nproc / affinity show the whole machine; this
    # job's CPU share is 16 (the pool's rule), so more workers would time
    # other jobs' cores
    w = share_cap
    cap_note = 'capped to the GPU box CPU share (%d)' % share_cap
  return {'nproc': nproc, 'affinity_cpus': aff, 'cgroup_cpus': cg, 'physical_cores': physical,
          'model': model, 'workers': w, 'cap': cap_note}


# ------------------------------------------------------------------ workers
def _row_tiles(rows, W):
  """Row extents of good_tile_shape(shape, W) for a 2-d (rows, cols) array
  (distarray.py:24-46: tile_size = rows*cols // W, filled from the last axis)."""
  tr = max(1, rows // W)
  return [(r, min(rows, r + tr)) for r in range(0, rows, tr)]


def _gen(shape, r0, seed, dtype, lo=0.0, hi=1.0):
  rows, cols = shape
  g = np.arange(r0 * cols, (r0 + rows) * cols, dtype=np.uint64)
  return rng.uniform_values(g, seed, lo, hi, dtype).reshape(rows, cols)


def _worker(conn, kind, spec):
  """One reference worker: builds its tile(s), then serves run-kernel
  requests until None."""
  import numpy as np  # noqa: F811  (spawned: imported after OMP_NUM_THREADS=1)
  if kind == 'cfg2':
    r0, r1, cols = spec
    x = _gen((r1 - r0, cols), r0, 11, np.float32)
    y = _gen((r1 - r0, cols), r0, 12, np.float32)
    z = _gen((r1 - r0, cols), r0, 13, np.float32, -1.0, 1.0)
  elif kind == 'dot':
    M, k0, k1, N, K = spec
    # A[:, k0:k1] (the column strip change_partition_axis gives the worker,
    # extent.pyx:489-539) and B[k0:k1, :] of the (M, K) / (K, N) operands
    g = (np.arange(M, dtype=np.uint64)[:, None] * np.uint64(K) +
         np.arange(k0, k1, dtype=np.uint64)[None, :])
    a = rng.uniform_values(g.reshape(-1), 31, 0.0, 1.0, np.float32).reshape(M, k1 - k0)
    b = _gen((k1 - k0, N), k0, 32, np.float32)
  elif kind == 'lreg':
    r0, r1, D = spec
    x = _gen((r1 - r0, D), r0, 41, np.float32)
    yv = _gen((r1 - r0, 1), r0, 42, np.float32)
  elif kind == 'kmeans':
    r0, r1, D = spec
    pts = _gen((r1 - r0, D), r0, 21, np.float32)
  conn.send('ready')
  while True:
    msg = conn.recv()
    if msg is None:
      break
    if kind == 'cfg2':
      t = np.multiply(x, y)          # LocalMapExpr(np.multiply)
      e = np.exp(z)                  # LocalMapExpr(np.exp)
      v = np.add(t, e)               # LocalMapExpr(np.add)
      conn.send(v.sum(msg))          # _sum_local
    elif kind == 'dot':
      conn.send(a.dot(b))            # dot_map2_mapper: tiles[0].dot(tiles[1])
    elif kind == 'lreg':
      w = msg
      yp = x.dot(w)                  # dot_map2_np_mapper (GEMV)
      diff = x * (yp - yv)           # MapExpr (broadcast (N,1) against (N,D))
      conn.send(diff.sum(0))         # _sum_local(axis=0)
    elif kind == 'kmeans':
      from scipy.spatial.distance import cdist
      centers = msg
      dist = cdist(pts, centers)     # kmeans_dist_mapper (fp64)
      lab = dist.argmin(axis=1)      # argmin(distances, axis=1)
      K = centers.shape[0]
      cnt = np.bincount(lab, minlength=K)          # kmeans_count_mapper
      sums = np.zeros((K, pts.shape[1]))
      for i in range(K):                           # kmeans_center_mapper
        sums[i] = pts[lab == i].sum(axis=0)
      conn.send((cnt, sums))


class _Pool:
  def __init__(self, kind, specs):
    ctx = mp.get_context('spawn')
    saved = {k: os.environ.get(k) for k in _ONE_THREAD}
    os.environ.update(_ONE_THREAD)  # inherited by the spawned workers before they import NumPy
    try:
      self.procs, self.conns = [], []
      for spec in specs:
        a, b = ctx.Pipe()
        p = ctx.Process(target=_worker, args=(b, kind, spec), daemon=True)
        p.start()
        self.procs.append(p)
        self.conns.append(a)
    finally:
      for k, v in saved.items():
        if v is None:
          os.environ.pop(k, None)
        else:
          os.environ[k] = v
    for c in self.conns:
      assert c.recv() == 'ready'

  def run(self, msg):
    for c in self.conns:
      c.send(msg)
    return [c.recv() for c in self.conns]

  def close(self):
    for c in self.conns:
      c.send(None)
    for p in self.procs:
      p.join(timeout=60)


def _timed(fn, reps):
  fn()  # warm-up
  times = []
  for _ in range(reps):
    t0 = time.perf_counter()
    fn()
    times.append(time.perf_counter() - t0)
  return float(np.median(times))


# ---------------------------------------------------------------------- legs
def cfg2_cpu_baseline(rows=4096, cols=32768, workers=None, reps=5):
  """sum(x*y+exp(z), axis=0) + sum(..., axis=1) on a (rows, cols) fp32
  sample: W workers, and one process.  GB/s of algorithmic bytes."""
  info = host_info()
  W = workers or info['workers']
  tiles = _row_tiles(rows, W)
  pool = _Pool('cfg2', [(r0, r1, cols) for r0, r1 in tiles])

  def step():
    out0 = None
    for part in pool.run(0):  # merge at the owner in tile order (np.add)
      out0 = part if out0 is None else np.add(out0, part)
    return out0, np.concatenate(pool.run(1))
  try:
    t = _timed(step, reps)
  finally:
    pool.close()
  nbytes = 2 * (3 * 4 * rows * cols + 4 * cols)  # two evaluations, algorithmic bytes
  # one process, default threading, on a slice of the same sample
  srows = max(1, min(rows, 4096))
  x, y = _gen((srows, cols), 0, 11, np.float32), _gen((srows, cols), 0, 12, np.float32)
  z = _gen((srows, cols), 0, 13, np.float32, -1.0, 1.0)
  t1 = _timed(lambda: ((x * y + np.exp(z)).sum(0), (x * y + np.exp(z)).sum(1)), 3)
  sbytes = 2 * (3 * 4 * srows * cols + 4 * cols)
  return {'value': nbytes / t / 1e9, 'unit': 'GB/s', 'cores': len(tiles), 'kind': 'port',
          'seconds_per_step': t, 'host': info,
          'single_process': {'value': round(sbytes / t1 / 1e9, 3), 'unit': 'GB/s',
                             'sample': 'fp32 (%d, %d), one process, NumPy default threading' % (srows, cols)},
          'sample': 'fp32 (%d, %d) rows of cfg2 (%.1f%% of 2^30), %d row-strip worker processes (spawned, one '
                    'BLAS thread each), median of %d steps of sum axis0 + axis1' % (
                        rows, cols, 100.0 * rows * cols / 2 ** 30, len(tiles), reps)}


def dot_cpu_baseline(S=4096, workers=None, reps=3):
  """K-split dot (configs[3] shape class) on an S x S fp32 sample: worker i
  computes A[:, K_i] @ B[K_i, :] (NumPy BLAS, one thread), the owner sums
  the partials with np.add.  GFLOP/s."""
  W = workers or host_info()['workers']
  ks = _row_tiles(S, W)
  pool = _Pool('dot', [(S, k0, k1, S, S) for k0, k1 in ks])

  def step():
    out = None
    for part in pool.run(1):
      out = part if out is None else np.add(out, part)
    return out
  try:
    t = _timed(step, reps)
  finally:
    pool.close()
  a, b = _gen((S, S), 0, 31, np.float32), _gen((S, S), 0, 32, np.float32)
  t1 = _timed(lambda: a.dot(b), reps)
  flops = 2.0 * S ** 3
  return {'value': round(flops / t / 1e9, 2), 'unit': 'GFLOP/s', 'cores': len(ks), 'kind': 'port',
          'single_process_gflops': round(flops / t1 / 1e9, 2),
          'sample': 'dot of (%d, %d) fp32, K split over %d workers, partials merged at the owner; median of %d' % (
              S, S, len(ks), reps)}


def lreg_cpu_baseline(N=4_000_000, D=64, workers=None, reps=3):
  """One linear-regression gradient step (configs[4] shape class) on an
  (N, D) fp32 sample.  ms per iteration and GB/s of the single-pass bytes
  (4 N D + 4 N), the unit the GPU leg reports."""
  W = workers or host_info()['workers']
  tiles = _row_tiles(N, W)
  pool = _Pool('lreg', [(r0, r1, D) for r0, r1 in tiles])
  w = np.random.default_rng(43).random((D, 1)).astype(np.float32)

  def step():
    g = None
    for part in pool.run(w):
      g = part if g is None else np.add(g, part)
    return g
  try:
    t = _timed(step, reps)
  finally:
    pool.close()
  nbytes = 4.0 * N * D + 4.0 * N
  return {'ms_per_iter': round(t * 1e3, 3), 'value': round(nbytes / t / 1e9, 3), 'unit': 'GB/s', 'cores': len(tiles),
          'kind': 'port', 'sample': 'X (%d, %d) fp32, y (%d, 1): GEMV + x*(yp-y) + sum(axis=0) per strip, %d workers; '
                                    'median of %d' % (N, D, N, len(tiles), reps)}


def kmeans_cpu_baseline(N=400_000, D=128, K=256, workers=None, reps=2):
  """One k-means iteration (configs[2] shape class) on an (N, D) fp32
  sample: cdist (fp64) + argmin + bincount + per-centre sums per strip.
  ms per iteration and points per second."""
  W = workers or host_info()['workers']
  tiles = _row_tiles(N, W)
  pool = _Pool('kmeans', [(r0, r1, D) for r0, r1 in tiles])
  centers = _gen((K, D), 0, 21, np.float32).astype(np.float64)

  def step():
    cnt, sums = None, None
    for c, s in pool.run(centers):
      cnt = c if cnt is None else cnt + c
      sums = s if sums is None else sums + s
    return sums / np.maximum(cnt, 1).reshape(K, 1)
  try:
    t = _timed(step, reps)
  finally:
    pool.close()
  return {'ms_per_iter': round(t * 1e3, 2), 'value': round(N / t, 1), 'unit': 'points/s', 'cores': len(tiles),
          'kind': 'port', 'sample': '(%d, %d) fp32 points, k=%d, scipy cdist + argmin + bincount + per-centre sums per '
                                    'strip, %d workers; median of %d' % (N, D, K, len(tiles), reps)}
