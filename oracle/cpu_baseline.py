"""CPU baseline (ORACLE, test/bench infrastructure): the reference's
multi-worker execution model restated with NumPy worker processes.

W worker processes each own one row-strip tile (good_tile_shape with
num_workers = W, spartan/array/distarray.py:24-46) that they generate
themselves and keep resident, like the reference's workers.  A step sends one
"run kernel" request per worker (BlobCtx.map, spartan/blob_ctx.py:256-275);
each worker evaluates the fused tree exactly as FnCallExpr.evaluate does --
one NumPy call per node, materialising temporaries (spartan/expr/local.py:110-122)
-- reduces its tile (``data.sum(axis)``, builtins.py:466-470) and returns the
partial; the master merges partials into the output with np.add in tile order
(tile.merge, tile.pyx:201-298).  Tiles never cross process boundaries (no
pickling of tiles, no ZeroMQ): a best case for the reference.
"""
import multiprocessing as mp
import os
import time

import numpy as np

from . import rng


def _worker(conn, r0, r1, cols, seeds):
  os.environ['OMP_NUM_THREADS'] = '1'
  n = (r1 - r0) * cols
  g = np.arange(r0 * cols, r0 * cols + n, dtype=np.uint64)
  x = rng.uniform_values(g, seeds[0], 0.0, 1.0, np.float32).reshape(r1 - r0, cols)
  y = rng.uniform_values(g, seeds[1], 0.0, 1.0, np.float32).reshape(r1 - r0, cols)
  z = rng.uniform_values(g, seeds[2], -1.0, 1.0, np.float32).reshape(r1 - r0, cols)
  del g
  conn.send('ready')
  while True:
    msg = conn.recv()
    if msg is None:
      break
    axis = msg
    t = np.multiply(x, y)          # LocalMapExpr(np.multiply)
    e = np.exp(z)                  # LocalMapExpr(np.exp)
    v = np.add(t, e)               # LocalMapExpr(np.add)
    conn.send(v.sum(axis))         # _sum_local


def _row_tiles(rows, cols, W):
  tile_size = rows * cols // W
  tr = max(1, tile_size // cols) if tile_size >= cols else 1
  out = []
  for r in range(0, rows, tr):
    out.append((r, min(rows, r + tr)))
  return out


def cfg2_cpu_baseline(rows=4096, cols=32768, workers=None, reps=3, seeds=(11, 12, 13)):
  """Time sum(x*y+exp(z), axis=0) + sum(..., axis=1) on a (rows, cols) fp32
  sample.  Returns dict(value GB/s, seconds per step, cores, sample)."""
  if workers is None:
    try:
      workers = len(os.sched_getaffinity(0))
    except AttributeError:
      workers = os.cpu_count()
    workers = max(1, min(16, workers))
  tiles = _row_tiles(rows, cols, workers)
  ctx = mp.get_context('fork')
  procs, conns = [], []
  for (r0, r1) in tiles:
    a, b = ctx.Pipe()
    p = ctx.Process(target=_worker, args=(b, r0, r1, cols, seeds), daemon=True)
    p.start()
    procs.append(p)
    conns.append(a)
  for c in conns:
    assert c.recv() == 'ready'

  def step():
    out0 = None
    for c in conns:
      c.send(0)
    for c in conns:  # merge at the owner in tile order (np.add)
      part = c.recv()
      out0 = part if out0 is None else np.add(out0, part)
    for c in conns:
      c.send(1)
    out1 = np.concatenate([c.recv() for c in conns])
    return out0, out1

  step()  # warm-up
  times = []
  for _ in range(reps):
    t0 = time.perf_counter()
    step()
    times.append(time.perf_counter() - t0)
  for c in conns:
    c.send(None)
  for p in procs:
    p.join(timeout=30)
  t = float(np.median(times))
  nbytes = 2 * (3 * 4 * rows * cols + 4 * cols)  # two evaluations, algorithmic bytes
  return {'value': nbytes / t / 1e9, 'unit': 'GB/s', 'cores': workers, 'kind': 'port',
          'seconds_per_step': t,
          'sample': 'fp32 (%d, %d) rows of cfg2 (%.1f%% of 2^30), %d row-strip worker processes, '
                    'median of %d steps of sum axis0 + axis1' % (rows, cols, 100.0 * rows * cols / 2 ** 30,
                                                                len(tiles), reps)}
