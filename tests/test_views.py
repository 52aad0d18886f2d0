"""Views on the path: slicing, transpose, reshape --
the reference's tests/test_slice.py, test_transpose.py, test_reshape.py
restated.  Host logic runs on CPU with the test double (W workers on one
rank); the same cases run through the gfx950 kernels in test_gpu_parity.py."""
import numpy as np
import pytest

from oracle import rng

TEST_SIZE = 10


def _views_cases(expr):
  """(lazy expression, expected NumPy value) pairs shared with the GPU test."""
  cases = []
  x = expr.arange((TEST_SIZE, TEST_SIZE))
  nx = np.arange(TEST_SIZE * TEST_SIZE).reshape(TEST_SIZE, TEST_SIZE).astype(np.float64)
  cases.append(('slice_get', x[5:8, 5:8], nx[5:8, 5:8]))                               # test_slice.py:24-29
  cases.append(('slice_map', expr.map(x[5:8, 5:8], lambda t: t + 1), nx[5:8, 5:8] + 1))  # :31-38
  x3 = expr.arange((10, 10, 10), dtype=np.int64)
  nx3 = np.arange(1000, dtype=np.int64).reshape(10, 10, 10)
  cases.append(('slice_map2', expr.map(x3[:, :, 0], lambda t: t + 13), nx3[:, :, 0:1] + 13))  # :50-58
  cases.append(('slice_reduce', x3[:, :, 0].sum(), nx3[:, :, 0].sum()))                 # :63-69
  a = expr.arange((TEST_SIZE,), dtype=np.int64)
  na = np.arange(TEST_SIZE, dtype=np.int64)
  cases.append(('slice_sub', a[1:] - a[:-1], na[1:] - na[:-1]))                          # :71-80
  cases.append(('slice_rows_sum', x[2:7, :].sum(1), nx[2:7, :].sum(1)))                  # benchmark_slice.py
  cases.append(('slice_of_slice', x[1:9, 2:9][2:5, 1:4], nx[1:9, 2:9][2:5, 1:4]))
  t1 = expr.arange((37, 13))
  t2 = np.arange(37 * 13, dtype=np.float64).reshape(37, 13)
  cases.append(('transpose', expr.transpose(t1), t2.T))                                  # test_transpose.py:8-11
  t3 = expr.arange((11, 12, 13))
  cases.append(('transpose3', expr.transpose(t3), np.arange(11 * 12 * 13.).reshape(11, 12, 13).T))  # :13-16
  cases.append(('transpose_map', expr.transpose(t1) * 2 + 1, t2.T * 2 + 1))
  for ax in (None, 0, 1):
    cases.append(('transpose_sum%s' % ax, expr.transpose(t1).sum(ax), t2.T.sum(ax)))
  p1 = rng.rand((41, 9), 1, np.float64)
  p2 = rng.rand((41, 9), 2, np.float64)
  cases.append(('transpose_dot', expr.dot(expr.from_numpy(p1), expr.transpose(expr.from_numpy(p2))),
                p1 @ p2.T))                                                              # :26-36
  r = expr.arange((10, 10))
  cases.append(('reshape1', expr.reshape(r, (100,)), np.arange(100.)))                   # test_reshape.py:9-13
  cases.append(('reshape3', expr.reshape(expr.reshape(expr.reshape(expr.arange((20, 30)), (600,)), (600, 1)),
                                         (1, 600)), np.arange(600.).reshape(1, 600)))   # :20-26
  e = expr.arange((1200,))
  for s in [(10, 120), (120, 10), (24, 50), (50, 24), (1, 1200)]:
    cases.append(('reshape4_%s' % (s,), expr.reshape(e, s), np.arange(1200.).reshape(s)))  # :28-36
  a7 = expr.arange((10, 6, 12))
  for s in [(6, 12, 10), (3, 40, 6), (720, 1), (1, 720)]:
    cases.append(('reshape7_%s' % (s,), expr.reshape(a7, s), np.arange(720.).reshape(s)))  # :54-85
  q1 = rng.rand((35, 9), 3, np.float64)
  q2 = rng.rand((7, 35), 4, np.float64)
  cases.append(('reshape_dot', expr.dot(expr.reshape(expr.from_numpy(q1), (45, 7)), expr.from_numpy(q2)),
                q1.reshape(45, 7) @ q2))                                                 # :95-121
  cases.append(('reshape_transpose', expr.reshape(expr.transpose(t1), (13 * 37,)), t2.T.reshape(-1)))
  # newaxis indexing (reference base.py:23-30, 402-430) and Expr.outer (expr/__init__.py:47)
  na_ = expr.newaxis
  cases.append(('newaxis_front', x[na_, 2:5], nx[None, 2:5]))
  cases.append(('newaxis_mid', x[:, na_], nx[:, None]))
  cases.append(('newaxis_int', x[3, na_], nx[3, None]))
  cases.append(('newaxis_none', x[1:4, None, 2:6], nx[1:4, None, 2:6]))
  cases.append(('newaxis_bcast', (x[:, na_, 0:3] * x3[0:10, 0:1, 0:3]).sum(1),
                (nx[:, None, 0:3] * nx3[0:10, 0:1, 0:3]).sum(1)))
  return cases


@pytest.mark.parametrize('W', [1, 3, 4])
def test_views_host(host_ctx, W):
  host_ctx(W)
  from spartan_amd import expr
  for name, e, want in _views_cases(expr):
    got = e.glom()
    np.testing.assert_allclose(np.asarray(got).reshape(np.shape(want)), want, rtol=1e-12, err_msg=name)


def test_flat_rects_cover_in_order():
  from spartan_amd.expr.reshape import flat_rects
  r = np.random.default_rng(3)
  for _ in range(300):
    shape = tuple(int(v) for v in r.integers(1, 6, size=r.integers(1, 4)))
    n = int(np.prod(shape))
    a = int(r.integers(0, n))
    b = int(r.integers(a, n + 1))
    flat = np.arange(n).reshape(shape)
    got = np.concatenate([flat[tuple(slice(u, l) for u, l in zip(ul, lr))].reshape(-1)
                          for ul, lr in flat_rects(a, b, shape)] or [np.zeros(0, int)])
    np.testing.assert_array_equal(got, np.arange(a, b))


def test_fancy_indexing_is_refused(host_ctx):
  host_ctx(2)
  from spartan_amd import expr
  x = expr.arange((5, 5))
  with pytest.raises(NotImplementedError):
    x[np.array([1, 2])]


def _optimization_dag_cases(expr, n=1000):
  """The reference's tests/test_optimization.py:9-44 (nonordered) and
  :124-163 (reduced): maps, slices of maps, a dot of slices and a final sum,
  optimised as one DAG."""
  na = rng.rand((n, n), 91, np.float64)
  nb = rng.rand((n, n), 92, np.float64)
  a = expr.from_numpy(na)
  b = expr.from_numpy(nb)
  s1, s2, s3 = slice(n // 5, 9 * n // 10), slice(n // 10, n // 2), slice(n // 10, n // 5)
  c = a + b
  d = a + c
  f = c[s1, s1]
  g = d[s1, s1]
  h = f + g
  i = f + h
  j = h[s2, s2]
  k = i[s2, s2]
  l = expr.dot(j, k)
  m = j + k
  nn = k + l
  o = nn + m
  q = o[s3, s3]
  nc = na + nb
  nd = na + nc
  nf = nc[s1, s1]
  ng = nd[s1, s1]
  nh = nf + ng
  ni = nf + nh
  nj = nh[s2, s2]
  nk = ni[s2, s2]
  nl = nj @ nk
  nm = nj + nk
  nno = nk + nl
  no = nno + nm
  nq = no[s3, s3]
  out = [('nonordered', q, nq)]
  c = a - b
  d = a + c
  f = c[s1, s1]
  g = d[s1, s1]
  h = f - g
  i = f + h
  j = h[s2, s2]
  k = i[s2, s2]
  l = expr.dot(j, k)
  m = j + k
  nn = k - l
  o = nn - m
  q = nn + o
  r = q - m
  s = expr.sum(r)
  nc = na - nb
  nd = na + nc
  nf = nc[s1, s1]
  ng = nd[s1, s1]
  nh = nf - ng
  ni = nf + nh
  nj = nh[s2, s2]
  nk = ni[s2, s2]
  nl = nj @ nk
  nm = nj + nk
  nno = nk - nl
  no = nno - nm
  nq = nno + no
  nr = nq - nm
  out.append(('reduced', s, nr.sum()))
  return out


@pytest.mark.parametrize('W', [1, 3])
def test_optimization_dags_host(host_ctx, W):
  host_ctx(W)
  from spartan_amd import expr
  for name, e, want in _optimization_dag_cases(expr, 200):
    np.testing.assert_allclose(e.optimized().glom(), want, rtol=1e-10, err_msg=name)
