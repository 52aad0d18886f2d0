"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py).

CPU (not gpu): the oracle and the counter-based generator still reproduce
the frozen vectors -- input digests bit-exact, integer / index outputs
bit-exact, floating-point outputs within 1e-6 (fp32) / 1e-13 (fp64)
relative (NumPy's SIMD exp / summation kernels may differ by an ulp across
host CPUs).

GPU: the HIP path against the same frozen vectors with the parity rules of
tests/test_gpu_parity.py: indices bit-exact; fp32 reductions / dot within
1e-5 relative of the fixture OR at least as close to the fp64-exact value;
fp64 within 1e-12 by the same rule.
"""
import hashlib
import os

import numpy as np
import pytest

from oracle import rng
from oracle import spartan_cpu as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
AXES = {'N': None, '0': 0, '1': 1}


def load(name):
  with np.load(os.path.join(GOLDEN, name + '.npz')) as f:
    return {k: f[k] for k in f.files}


def sha(a):
  return np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest(), dtype=np.uint8)


def _make(name):
  import importlib.util
  spec = importlib.util.spec_from_file_location('make_golden', os.path.join(GOLDEN, 'make_golden.py'))
  mod = importlib.util.module_from_spec(spec)
  spec.loader.exec_module(mod)
  return mod.FAMILIES[name]()


def _same(got, want, key):
  got, want = np.asarray(got), np.asarray(want)
  assert got.shape == want.shape and got.dtype == want.dtype, key
  if want.dtype.kind in 'biu':
    np.testing.assert_array_equal(got, want, err_msg=key)
  else:
    rtol = 1e-6 if want.dtype == np.float32 else 1e-13
    np.testing.assert_allclose(got, want, rtol=rtol, atol=0, err_msg=key)


@pytest.mark.parametrize('name', ['cfg2', 'ties', 'dot', 'kmeans', 'lreg'])
def test_oracle_reproduces_golden(name):
  want = load(name)
  got = _make(name)
  assert sorted(got) == sorted(want)
  for k in want:
    _same(got[k], want[k], '%s:%s' % (name, k))


def test_golden_input_digests():
  """The generator's streams behind the seed-only fixtures are unchanged."""
  c = load('cfg2')
  x, y, z = (rng.rand((257, 131), 11, np.float32), rng.rand((257, 131), 12, np.float32),
             rng.rand((257, 131), 13, np.float32, -1.0, 1.0))
  np.testing.assert_array_equal(sha(np.concatenate([x.ravel(), y.ravel(), z.ravel()])), c['xyz_sha_m'])
  np.testing.assert_array_equal(c['x_s'], rng.rand((96, 80), 11, np.float32))
  d = load('dot')
  for dt, tag in [(np.float32, 'f32'), (np.float64, 'f64')]:
    a, b = rng.rand((128, 96), 31, dt), rng.rand((96, 80), 32, dt)
    np.testing.assert_array_equal(sha(np.concatenate([a.ravel(), b.ravel()])), d['ab_sha_' + tag])


def test_golden_arg_semantics():
  """Frozen arg-reductions are first-occurrence indices of the frozen min / max."""
  t = load('ties')
  for tag in ('i', 'f'):
    a = t[tag]
    for an, ax in AXES.items():
      for W in (1, 3, 8):
        k = '%s_W%d_ax%s' % (tag, W, an)
        np.testing.assert_array_equal(t['argmin_' + k], np.argmin(a, axis=ax))
        np.testing.assert_array_equal(t['argmax_' + k], np.argmax(a, axis=ax))
        np.testing.assert_array_equal(t['min_' + k], np.min(a, axis=ax))


# ------------------------------------------------------------------ GPU
@pytest.fixture
def ex(gpu_workers):
  from spartan_amd import expr
  return expr, gpu_workers


def check_fp(gpu, ref, exact, rtol):
  gpu, ref, exact = (np.asarray(v, dtype=np.float64) for v in (gpu, ref, exact))
  assert gpu.shape == ref.shape
  scale = np.maximum(np.abs(ref), 1e-30)
  close = np.abs(gpu - ref) <= rtol * scale
  better = np.abs(gpu - exact) <= np.abs(ref - exact) + rtol * 1e-3 * scale
  bad = ~(close | better)
  assert not bad.any(), 'max rel err %g' % (np.abs(gpu - ref) / scale).max()


@pytest.mark.gpu
@pytest.mark.parametrize('tag', ['s', 'm'])
@pytest.mark.parametrize('W', [1, 2, 3, 8])
def test_gpu_cfg2_golden(ex, tag, W):
  expr, setw = ex
  setw(W)
  g = load('cfg2')
  if tag == 's':
    nx, ny, nz = g['x_s'], g['y_s'], g['z_s']
    x, y, z = expr.from_numpy(nx), expr.from_numpy(ny), expr.from_numpy(nz)
  else:
    shape = (257, 131)
    nx, ny, nz = (rng.rand(shape, 11, np.float32), rng.rand(shape, 12, np.float32),
                  rng.rand(shape, 13, np.float32, -1.0, 1.0))
    x = expr.rand(*shape, dtype=np.float32, seed=11)
    y = expr.rand(*shape, dtype=np.float32, seed=12)
    z = expr.rand(*shape, dtype=np.float32, seed=13, low=-1.0, high=1.0)
  host_m = nx * ny + np.exp(nz)
  m = (x * y + expr.exp(z)).optimized().glom()
  agree = bool((m == host_m).all())  # indices are compared where the mapped values agree bit for bit
  for an, ax in AXES.items():
    k = '%s_W%d_ax%s' % (tag, W, an)
    got = expr.sum(x * y + expr.exp(z), axis=ax).optimized().glom()
    check_fp(got, g['sum_' + k], m.astype(np.float64).sum(ax), 1e-5)
    for red in ('min', 'max'):
      got = getattr(expr, red)(x * y + expr.exp(z), axis=ax).optimized().glom()
      # selections: bit-exact on the GPU's own map values, 1e-6 of the frozen vector
      np.testing.assert_array_equal(got, getattr(O, red + '_tiles')(m, ax, W))
      np.testing.assert_allclose(got, g['%s_%s' % (red, k)], rtol=1e-6)
    for kind in ('argmin', 'argmax'):
      got = getattr(expr, kind)(x * y + expr.exp(z), axis=ax).optimized().glom()
      assert got.dtype == np.int64
      # always: the reference's three-pass argmin over the GPU's own map values
      np.testing.assert_array_equal(got, O.arg_tiles(m, ax, W, kind))
      if agree:  # and the frozen vector where OCML's exp matches NumPy's bit for bit
        np.testing.assert_array_equal(got, g['%s_%s' % (kind, k)])


@pytest.mark.gpu
@pytest.mark.parametrize('W', [1, 3, 8])
def test_gpu_ties_golden(ex, W):
  expr, setw = ex
  setw(W)
  t = load('ties')
  for tag in ('i', 'f'):
    a = expr.from_numpy(t[tag])
    for an, ax in AXES.items():
      k = '%s_W%d_ax%s' % (tag, W, an)
      for red in ('sum', 'min', 'max', 'argmin', 'argmax'):
        got = getattr(expr, red)(a, axis=ax).glom()
        np.testing.assert_array_equal(got, t['%s_%s' % (red, k)], err_msg='%s %s' % (red, k))


@pytest.mark.gpu
def test_gpu_dot_golden(ex):
  expr, setw = ex
  setw(4)
  d = load('dot')
  for dt, tag, tol in [(np.float32, 'f32', 1e-5), (np.float64, 'f64', 1e-12)]:
    a = expr.rand(128, 96, dtype=dt, seed=31)
    b = expr.rand(96, 80, dtype=dt, seed=32)
    na, nb = rng.rand((128, 96), 31, dt), rng.rand((96, 80), 32, dt)
    got = expr.dot(a, b).glom()
    assert got.dtype == dt
    check_fp(got, d['c_' + tag], na.astype(np.float64) @ nb.astype(np.float64), tol)
  ones = expr.ones((2000, 2000))
  assert expr.sum(expr.dot(ones, ones)).glom() == d['ones_sum']


@pytest.mark.gpu
def test_gpu_kmeans_golden(ex):
  from spartan_amd import workloads
  expr, setw = ex
  setw(2)
  k = load('kmeans')
  pts = k['points']
  _, l1 = workloads.kmeans_fit(expr.from_numpy(pts), 8, 1, centers=k['centres0'])
  np.testing.assert_array_equal(l1.glom(), k['labels1'])
  c3, l3 = workloads.kmeans_fit(expr.from_numpy(pts), 8, 3, centers=k['centres0'])
  np.testing.assert_array_equal(l3.glom(), k['labels3'])
  # the centres after the third update are the means over the third
  # iteration's labels: their fp64-exact values decide between fixture and build
  exact = np.stack([pts[k['labels3'] == i].astype(np.float64).mean(0) for i in range(8)])
  check_fp(c3, k['centres3'], exact, 1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize('W', [1, 3])
def test_gpu_lreg_golden(ex, W):
  from spartan_amd import workloads
  expr, setw = ex
  setw(W)
  L = load('lreg')
  n, dim = 10000, 64
  x = expr.rand(n, dim, dtype=np.float32, seed=41)
  y = expr.rand(n, 1, dtype=np.float32, seed=42)
  w0 = L['w0']
  X, Y = rng.rand((n, dim), 41, np.float32), rng.rand((n, 1), 42, np.float32)
  g = expr.sum(x * (expr.dot(x, w0) - y), axis=0).optimized().glom()
  exact = (X.astype(np.float64) * (X.astype(np.float64) @ w0.astype(np.float64) - Y)).sum(0)
  check_fp(g, L['grad_W%d' % W], exact, 1e-5)
  w3 = workloads.sgd_train(x, y, w0, 1e-6, 3)
  gmax = np.abs(exact).max()
  np.testing.assert_allclose(w3, L['w3_W%d' % W], rtol=0, atol=3 * 1e-6 * 1e-5 * gmax + 1e-7)
