"""GPU restatement of the reference's builtin / elementwise / broadcast /
stats tests on the hot path:

  tests/test_builtins.py:9-135   arange signatures, bincount, concatenate,
                                 max / min (the diag* cases are out of scope,
                                 SURVEY.md section 2 row 10)
  tests/test_elementwise.py:9-22 maximum of two arrays and with a scalar
  tests/test_broadcast.py:9-20   (100,1,100,100) +/- (10,100,1)
  tests/test_stats.py:9-47       std over None / 0 / 1 (fused mean / sum)

The reference draws unseeded np.random inputs; these use fixed seeds.  Each
case runs with 1 and 3 virtual workers (row strips, ragged for 3).
Tolerances: integer / index results and exact float identities bit-exact;
std against the same formula evaluated by NumPy within 1e-12 (fp64) and
against np.std within the reference's own allclose (rtol 1e-5).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

WORKERS = [1, 3]


@pytest.fixture
def ex(gpu_workers):
  from spartan_amd import expr
  return expr, gpu_workers


@pytest.mark.parametrize('W', WORKERS)
def test_arange_shape(ex, W):
  """test_builtins.py:9-44."""
  expr, setw = ex
  setw(W)
  with pytest.raises(ValueError):
    expr.arange()
  with pytest.raises(ValueError):
    expr.arange((0,), stop=0)
  eq = np.testing.assert_array_equal
  eq(expr.arange((10,)).glom(), np.arange(10))
  eq(expr.arange((3, 5)).glom(), np.arange(15).reshape((3, 5)))
  eq(expr.arange((10,), -1).glom(), np.arange(-1, 9))
  eq(expr.arange((10,), 1).glom(), np.arange(1, 11))
  eq(expr.arange((3, 5), -1).glom(), np.arange(-1, 14).reshape((3, 5)))
  eq(expr.arange((10,), step=2).glom(), np.arange(0, 20, 2))
  eq(expr.arange((3, 5), step=2).glom(), np.arange(0, 30, 2).reshape((3, 5)))
  eq(expr.arange((10,), -1, step=2).glom(), np.arange(-1, 19, 2))
  eq(expr.arange((10,), 1, step=2).glom(), np.arange(1, 21, 2))
  eq(expr.arange((3, 5), 1, step=2).glom(), np.arange(1, 31, 2).reshape((3, 5)))


@pytest.mark.parametrize('W', WORKERS)
def test_arange_stop(ex, W):
  """test_builtins.py:47-57."""
  expr, setw = ex
  setw(W)
  eq = np.testing.assert_array_equal
  eq(expr.arange(stop=10).glom(), np.arange(10))
  eq(expr.arange(None, -1, 10).glom(), np.arange(-1, 10))
  eq(expr.arange(None, 1, 10).glom(), np.arange(1, 10))
  eq(expr.arange(None, -1, 19, 2).glom(), np.arange(-1, 19, 2))
  eq(expr.arange(None, 1, 21, 2).glom(), np.arange(1, 21, 2))


@pytest.mark.parametrize('W', WORKERS)
def test_bincount_max_min(ex, W):
  """test_builtins.py:60-65, 121-135."""
  expr, setw = ex
  setw(W)
  src = np.asarray([1, 1, 1, 2, 2, 5, 5, 10])
  np.testing.assert_array_equal(expr.bincount(expr.from_numpy(src)).glom(), np.bincount(src))
  np.testing.assert_array_equal(expr.max(expr.from_numpy(src)).glom(), np.max(src))
  np.testing.assert_array_equal(expr.min(expr.from_numpy(src)).glom(), np.min(src))
  m = np.arange(100).reshape(10, 10)
  np.testing.assert_array_equal(expr.min(expr.from_numpy(m), axis=1).glom(), np.min(m, axis=1))


@pytest.mark.parametrize('W', WORKERS)
def test_concatenate(ex, W):
  """test_builtins.py:97-118."""
  expr, setw = ex
  setw(W)
  g = np.random.default_rng(5)
  n1 = g.standard_normal(10)
  s1 = expr.from_numpy(n1)
  np.testing.assert_array_equal(expr.concatenate(s1, s1).glom(), np.concatenate((n1, n1)))
  n2 = np.arange(1024).reshape(32, 32)
  s2 = expr.from_numpy(n2)
  np.testing.assert_array_equal(expr.concatenate(s2, s2).glom(), np.concatenate((n2, n2)))
  np.testing.assert_array_equal(expr.concatenate(s2, s2, 1).glom(), np.concatenate((n2, n2), 1))
  a, b = g.standard_normal((15, 5)), g.standard_normal((15, 7))
  np.testing.assert_array_equal(expr.concatenate(expr.from_numpy(a), expr.from_numpy(b), 1).glom(),
                                np.concatenate((a, b), 1))


@pytest.mark.parametrize('W', WORKERS)
def test_maximum(ex, W):
  """test_elementwise.py:9-22."""
  expr, setw = ex
  setw(W)
  g = np.random.default_rng(7)
  a, b = g.standard_normal((10, 10)), g.standard_normal((10, 10))
  sa, sb = expr.from_numpy(a), expr.from_numpy(b)
  np.testing.assert_array_equal(expr.maximum(sa, sb).glom(), np.maximum(a, b))
  np.testing.assert_array_equal(expr.maximum(sa, 0).glom(), np.maximum(a, 0))


@pytest.mark.parametrize('W', WORKERS)
def test_broadcast_4d(ex, W):
  """test_broadcast.py:9-20: (100,1,100,100) against (10,100,1)."""
  expr, setw = ex
  from spartan_amd.expr import broadcast
  setw(W)
  a = expr.ones((100, 1, 100, 100)).force()
  b = expr.ones((10, 100, 1)).force()
  a, b = broadcast.broadcast((a, b))
  c = expr.add(a, b).force()
  d = expr.sub(a, b).force()
  n = np.ones((100, 10, 100, 100))
  np.testing.assert_array_equal(c.glom(), n + n)
  np.testing.assert_array_equal(d.glom(), n - n)


def _std_formula(a, axis):
  a = a.astype(np.float64)
  return np.sqrt(np.mean(a ** 2, axis) - np.mean(a, axis) ** 2)


@pytest.mark.parametrize('W', WORKERS)
def test_std_no_axis(ex, W):
  """test_stats.py:9-26."""
  expr, setw = ex
  setw(W)
  g = np.random.default_rng(9)
  for shape in [(10,), (10, 10), (17, 17)]:
    a = g.standard_normal(shape)
    got = expr.std(expr.from_numpy(a)).glom()
    np.testing.assert_allclose(got, _std_formula(a, None), rtol=1e-12)
    np.testing.assert_allclose(got, np.std(a), rtol=1e-5)


@pytest.mark.parametrize('W', WORKERS)
def test_std_with_axis(ex, W):
  """test_stats.py:29-47, plus an fp32 input (std casts to fp64 first)."""
  expr, setw = ex
  setw(W)
  g = np.random.default_rng(10)
  for shape in [(10, 10), (15, 13), (13, 15)]:
    a = g.standard_normal(shape)
    s = expr.from_numpy(a)
    for axis in (0, 1):
      got = expr.std(s, axis).glom()
      np.testing.assert_allclose(got, _std_formula(a, axis), rtol=1e-12)
      np.testing.assert_allclose(got, np.std(a, axis), rtol=1e-5)
  a32 = g.random((33, 21), dtype=np.float32)
  got = expr.std(expr.from_numpy(a32), 0).glom()
  assert got.dtype == np.float64
  np.testing.assert_allclose(got, _std_formula(a32, 0), rtol=1e-12)
