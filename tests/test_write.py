"""Writes and ingest: the reference's tests/test_write.py
restated (from_file .npy / .npz, from_numpy 1-d / 2-d, write from NumPy and
from arrays), plus the merge rule on partial sub-region writes with a
reducer (tile.pyx:201-298: first write replaces, later writes reduce),
self-aliasing writes and writes from views.  ``_run_write_cases`` is shared
by the CPU test double here, the GPU parity test and the gloo world-2 test."""
import os

import numpy as np
import pytest

from oracle import rng

S1 = (slice(0, 50), slice(0, 50))
S2 = (slice(0, 50), slice(50, 100))
S3 = (slice(50, 100), slice(0, 50))
S4 = (slice(50, 100), slice(50, 100))


def _run_write_cases(expr, tmpdir):
  # test_from_np1d / test_from_np2d (test_write.py:9-31)
  for shape in [(100, 100), (10000,)]:
    npa = rng.rand(shape, 7, np.float64)
    base = os.path.join(tmpdir, 'w_%d' % len(shape))
    np.save(base + '.npy', npa)
    np.savez(base + '.npz', npa)
    for t in (expr.from_file(base + '.npy', sparse=False), expr.from_file(base + '.npz', sparse=False),
              expr.from_numpy(npa)):
      np.testing.assert_array_equal(t.glom(), npa)

  # test_slices_from_np (:33-45)
  npa = rng.rand((100, 100), 8, np.float64)
  t1 = expr.randn(100, 100)
  t5 = expr.write(expr.write(expr.write(expr.write(t1, S1, npa, S1), S2, npa, S2), S3, npa, S3), S4, npa, S4)
  np.testing.assert_array_equal(t5.glom(), npa)

  # test_slices_from_slices (:47-71)
  t1 = expr.randn(100, 100)
  t2 = expr.randn(100, 100)
  t6 = expr.write(expr.write(expr.write(expr.write(t2, S1, t1, S1), S2, t1, S2), S3, t1, S3), S4, t1, S4)
  np.testing.assert_array_equal(t1.glom(), t6.glom())
  dst = np.arange(0, 2500).reshape(50, 50)
  t14 = expr.write(expr.write(expr.write(expr.write(t1, S1, dst, S1), S2, dst, S1), S3, dst, S1), S4, dst, S1)
  tmp = expr.write(expr.randn(100, 100), S4, dst, S1)
  t24 = expr.write(expr.write(expr.write(expr.write(t2, S1, tmp, S4), S2, tmp, S4), S3, tmp, S4), S4, tmp, S4)
  want = np.tile(dst.astype(np.float64), (2, 2))
  np.testing.assert_array_equal(t14.glom(), want)
  np.testing.assert_array_equal(t24.glom(), want)

  # randn values: the counter-based stream's Box-Muller draws
  z = expr.randn(64, 48, seed=5).glom()
  np.testing.assert_allclose(z, rng.randn((64, 48), 5), rtol=1e-12, atol=1e-13)

  # merge rule on partial writes: first write replaces, later writes reduce
  a = rng.rand((20, 10), 9, np.float64)
  b = rng.rand((20, 15), 10, np.float64)
  for fn, red in [(np.add, lambda x, y: x + y), (np.minimum, np.minimum), (None, lambda x, y: y)]:
    t = expr.ndarray((30, 20), dtype=np.float64, reduce_fn=fn).force()
    expr.write(t, (slice(0, 20), slice(0, 10)), a, ()).force()
    expr.write(t, (slice(10, 30), slice(5, 20)), b, ()).force()
    got = t.glom()
    np.testing.assert_array_equal(got[0:10, 0:10], a[0:10])
    np.testing.assert_array_equal(got[10:20, 0:5], a[10:20, 0:5])
    np.testing.assert_array_equal(got[10:20, 5:10], red(a[10:20, 5:10], b[0:10, 0:5]))
    np.testing.assert_array_equal(got[10:20, 10:20], b[0:10, 5:15])
    np.testing.assert_array_equal(got[20:30, 5:20], b[10:20])

  # a longer sequence: irregular overlap (device mask built), then a disjoint
  # and an irregular write again -- the mask must still know every element
  # written since it was built (tile.pyx:284 sets mask[subslice] on every merge)
  # Model: per tile, a write covering the whole tile reduces everywhere iff
  # the tile's first element was written, else replaces (tile.pyx:264-269);
  # a partial write replaces unwritten and reduces written elements.
  # ``defined`` tracks elements whose value does not depend on uninitialised
  # memory (a reduce into a never-written element stays undefined).
  for fn in (np.add, np.maximum):
    t = expr.ndarray((12,), dtype=np.float64, reduce_fn=fn).force()
    tiles = sorted((ex.ul[0], ex.lr[0]) for ex in t.tiles)
    want = np.zeros(12)
    seen = np.zeros(12, bool)
    defined = np.zeros(12, bool)
    for k, (lo, hi) in enumerate([(0, 4), (2, 6), (7, 9), (5, 9), (0, 12), (10, 12), (4, 11)]):
      piece = np.arange(lo, hi, dtype=np.float64) * (k + 2) + 0.5
      expr.write(t, (slice(lo, hi),), piece, ()).force()
      full = np.zeros(12)
      full[lo:hi] = piece
      for tu, tl in tiles:
        a, b = max(lo, tu), min(hi, tl)
        if a >= b:
          continue
        idx = np.arange(a, b)
        if (a, b) == (tu, tl):
          red = np.full(b - a, seen[tu])
        else:
          red = seen[a:b].copy()
        want[idx[~red]] = full[idx[~red]]
        defined[idx[~red]] = True
        want[idx[red]] = fn(want[idx[red]], full[idx[red]])
        seen[a:b] = True
      np.testing.assert_array_equal(t.glom()[defined], want[defined], err_msg='%s write %d' % (fn.__name__, k))

  # write from a transposed view, and a write whose source is the target itself
  src = np.arange(40 * 30, dtype=np.float64).reshape(40, 30)
  t = expr.zeros((30, 40)).force()
  expr.write(t, (slice(0, 30), slice(0, 40)), expr.transpose(expr.from_numpy(src)), ()).force()
  np.testing.assert_array_equal(t.glom(), src.T)
  x = expr.from_numpy(src.copy()).force()
  expr.write(x, (slice(0, 24), slice(0, 30)), x, (slice(12, 36), slice(0, 30))).force()
  want = src.copy()
  want[0:24] = src[12:36]
  np.testing.assert_array_equal(x.glom(), want)

  # __setitem__ with a scalar and with an array (distarray.py:160-170)
  y = expr.zeros((12, 9), dtype=np.float32).force()
  y[2:5, 3:7] = 1.5
  y[8:12, :] = np.arange(36, dtype=np.float32).reshape(4, 9)
  want = np.zeros((12, 9), np.float32)
  want[2:5, 3:7] = 1.5
  want[8:12] = np.arange(36).reshape(4, 9)
  np.testing.assert_array_equal(y.glom(), want)


@pytest.mark.parametrize('W', [1, 3, 4])
def test_write_host(host_ctx, W, tmp_path):
  host_ctx(W)
  from spartan_amd import expr
  _run_write_cases(expr, str(tmp_path))


def test_write_errors(host_ctx):
  host_ctx(2)
  from spartan_amd import expr
  t = expr.zeros((10, 10)).force()
  with pytest.raises(ValueError):
    expr.write(t, (slice(0, 5), slice(0, 5)), expr.ones((10, 10)), (slice(0, 4), slice(0, 5))).force()
  with pytest.raises(TypeError):
    expr.from_numpy([1, 2, 3])
  with pytest.raises(NotImplementedError):
    expr.from_file('x.mtx')


def test_transfer_blocks():
  from spartan_amd.array import transfer
  blocks, rb = transfer._blocks((100000, 300), 8)
  assert rb == 2400 and blocks[0] == (0, transfer.CHUNK // 2400) and blocks[-1][1] == 100000
  assert all(a[1] == b[0] for a, b in zip(blocks, blocks[1:]))
  assert transfer._blocks((2, transfer.CHUNK), 8) is None  # rows wider than a block
