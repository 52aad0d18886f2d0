"""Body of the multi-rank GPU rehearsal (tests/test_gpu_parity.py::
test_multirank_rehearsal_gpu): launched by torchrun with every rank on the
same GPU and SPARTAN_DIST_BACKEND=gloo, so the N>1 tile plans, region
exchanges and partial combines run with the real gfx950 kernels (RCCL itself
is exercised only on a multi-GPU node).  Checks against NumPy / the oracle."""
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402


def main():
  import faulthandler
  faulthandler.dump_traceback_later(150, exit=True)  # a hang names its stack instead of timing out silently
  import spartan_amd
  from spartan_amd import expr
  from spartan_amd.config import FLAGS
  from oracle import rng
  from oracle import spartan_cpu as O
  W = int(os.environ.get('REHEARSAL_WORKERS', '3'))
  FLAGS.num_workers = W
  ctx = spartan_amd.initialize()
  assert ctx.world_size > 1 and ctx.dist_backend == 'gloo'
  x = expr.arange((40, 30), dtype=np.int64).force()
  nx = np.arange(1200).reshape(40, 30)
  X = expr.lazify(x)
  for axis in (None, 0, 1):
    np.testing.assert_array_equal(X.sum(axis).glom(), O.sum_tiles(nx, axis, W))
    np.testing.assert_array_equal(X.argmin(axis).glom(), nx.argmin(axis))
  # forced DistArrays as direct dot / map / fused-reduce operands
  xf = expr.arange((40, 30)).force()
  nxf = np.arange(1200.).reshape(40, 30)
  yf = expr.arange((30, 20)).force()
  np.testing.assert_array_equal(expr.dot(xf, yf).glom(), nxf @ np.arange(600.).reshape(30, 20))
  np.testing.assert_allclose(expr.map(xf, np.sqrt).glom(), np.sqrt(nxf), rtol=1e-15)
  np.testing.assert_allclose(expr.sum(expr.sqrt(xf), 0).glom(), O.sum_tiles(np.sqrt(nxf), 0, W), rtol=1e-12)
  shape = (64, 48)
  xs = expr.rand(*shape, dtype=np.float32, seed=11)
  ys = expr.rand(*shape, dtype=np.float32, seed=12)
  zs = expr.rand(*shape, dtype=np.float32, seed=13, low=-1.0, high=1.0)
  mapped = O.map_tiles(lambda a, b, c: a * b + np.exp(c),
                       [rng.rand(shape, 11, np.float32), rng.rand(shape, 12, np.float32),
                        rng.rand(shape, 13, np.float32, -1.0, 1.0)], W)
  for axis in (None, 0, 1):
    got = expr.sum(xs * ys + expr.exp(zs), axis=axis).optimized().glom()
    np.testing.assert_allclose(got, mapped.sum(axis), rtol=1e-5)
  a = rng.rand((96, 80), 1, np.float64)
  b = rng.rand((80, 72), 2, np.float64)
  np.testing.assert_allclose(expr.dot(expr.from_numpy(a), expr.from_numpy(b)).glom(), a @ b, rtol=1e-12)
  # one output row slab per rank: the overlapped slab-by-slab dot reduction
  ctx.num_workers = ctx.world_size  # (the context caches FLAGS.num_workers at initialize)
  dot_mod = sys.modules['spartan_amd.expr.dot']
  n0 = dot_mod.OVERLAPPED_CALLS
  a2 = rng.rand((128, 96), 3, np.float32)
  b2 = rng.rand((96, 80), 4, np.float32)
  np.testing.assert_allclose(expr.dot(expr.from_numpy(a2), expr.from_numpy(b2)).glom(), a2 @ b2, rtol=1e-5)
  assert dot_mod.OVERLAPPED_CALLS == n0 + 1
  ctx.num_workers = W
  from spartan_amd import workloads
  from oracle import workloads as OW
  pts = rng.rand((3000, 64), 21, np.float32)
  c, lab = workloads.kmeans_fit(expr.from_numpy(pts), 40, 2)
  c2, l2 = OW.kmeans_fit(pts, 40, 2, W)
  np.testing.assert_allclose(c, c2, rtol=1e-6)
  np.testing.assert_array_equal(lab.glom(), l2)
  from test_views import _views_cases
  for name, e, want in _views_cases(expr):
    np.testing.assert_allclose(np.asarray(e.glom()).reshape(np.shape(want)), want, rtol=1e-12, err_msg=name)
  from test_write import _run_write_cases
  _run_write_cases(expr, tempfile.mkdtemp())
  from test_join import _run_join_cases
  _run_join_cases(expr, FLAGS)
  from test_location import _run_location_cases
  _run_location_cases(expr, W)
  print('rehearsal ok rank %d of %d' % (ctx.rank, ctx.world_size), flush=True)
  spartan_amd.shutdown()


if __name__ == '__main__':
  main()
