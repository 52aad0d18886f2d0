"""map_with_location / region_map: the reference's
tests/test_optimization.py:166-185 and tests/test_tile_sharing.py cases, the
nbody.py set_diagonal mapper, a location-dependent mapper and the
cholesky.py zero-fill region mapper.  Shared by the CPU test double, the GPU
parity test and the gloo world-2 test."""
import numpy as np
import pytest


def _set_diagonal_mapper(tile, ex, scalar):  # nbody.py:30-40
  ul = ex[0]
  if ul[0] == ul[1]:
    return scalar
  return tile


def _run_location_cases(expr, num_workers):
  from spartan_amd.array import extent

  def plus10(tile, ex):
    return tile + 10

  a = expr.map_with_location(expr.ones((5, 5)), plus10) + expr.ones((5, 5))
  np.testing.assert_array_equal(a.optimized().glom(), np.full((5, 5), 12.0))   # test_optimization.py:166-173
  np.testing.assert_array_equal(a.glom(), np.full((5, 5), 12.0))

  x = expr.arange((12, 7), dtype=np.int64).force()

  def add_row_offset(tile, ex):
    return tile + ex[0][0] * 1000 + ex[0][1]

  got = expr.map_with_location(x, add_row_offset).glom()
  want = np.arange(84).reshape(12, 7)
  for ex in x.tiles:
    want[ex.to_slice()] += ex.ul[0] * 1000 + ex.ul[1]
  np.testing.assert_array_equal(got, want)
  np.testing.assert_array_equal(expr.sum(expr.map_with_location(x, add_row_offset), axis=0).glom(), want.sum(0))

  d = expr.ones((9, 9), tile_hint=(3, 3)).force()
  got = expr.map_with_location(d, _set_diagonal_mapper, fn_kw={'scalar': 5.0}).glom()
  want = np.ones((9, 9))
  for ex in d.tiles:
    if ex.ul[0] == ex.ul[1]:
      want[ex.to_slice()] = 5.0
  np.testing.assert_array_equal(got, want)

  n = 5 * num_workers                                                            # test_tile_sharing.py
  xs = expr.ones((n, 1), tile_hint=(n // num_workers, 1))
  y = expr.region_map(xs, extent.create((0, 0), (3, 1), (n, 1)), fn=lambda data, ex, a: data + a, fn_kw={'a': 1})
  npy = np.ones((n, 1))
  npy[0:3, 0] += 1
  np.testing.assert_array_equal(xs.glom(), np.ones((n, 1)))
  np.testing.assert_array_equal(y.glom(), npy)

  r = expr.region_map(expr.ones((5, 5)), extent.create((0, 0), (1, 5), (5, 5)), plus10) + expr.ones((5, 5)) * 10
  want = np.full((5, 5), 11.0)                                                   # test_optimization.py:175-182
  want[0] = 21.0
  np.testing.assert_array_equal(r.optimized().glom(), want)

  v = expr.arange((8, 6)).force()
  regs = [extent.create((2, 0), (6, 6), (8, 6)), extent.create((0, 0), (8, 6), (8, 6))]
  got = expr.region_map(v, regs, lambda inp, ex: np.zeros(inp.shape, inp.dtype)).glom()  # cholesky.py:64
  want = np.arange(48.).reshape(8, 6)
  for ex in v.tiles:  # only the first region meeting each tile applies
    inter = extent.intersection(regs[0], ex) or extent.intersection(regs[1], ex)
    want[inter.to_slice()] = 0.0
  np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize('W', [1, 3, 4])
def test_location_host(host_ctx, W):
  host_ctx(W)
  from spartan_amd import expr
  _run_location_cases(expr, W)
