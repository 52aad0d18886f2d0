import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
  config.addinivalue_line('markers', 'gpu: needs a real MI355X (runs through libspx.so / generated kernels)')


@pytest.fixture
def host_ctx():
  """Single-rank CPU context with the TEST-DOUBLE backend (host logic only)."""
  import torch
  from spartan_amd import backend, runtime
  from spartan_amd.config import FLAGS
  from spartan_amd.expr.base import eval_cache
  from fake_backend import FakeBackend

  def make(num_workers=1):
    FLAGS.num_workers = num_workers
    ctx = runtime.Context(0, 1, 0, torch.device('cpu'), None)
    runtime.set_context(ctx)
    return ctx

  prev_b = backend.set_backend(FakeBackend())
  prev_c = runtime.set_context(None)
  yield make
  eval_cache.clear()
  FLAGS.num_workers = None
  backend.set_backend(prev_b)
  runtime.set_context(prev_c)


@pytest.fixture(scope='session')
def gpu_ctx():
  """Real MI355X context: libspx.so + generated kernels on cuda:0."""
  import torch
  if not torch.cuda.is_available():
    pytest.skip('no GPU')
  from spartan_amd import backend, runtime
  ctx = runtime.initialize()
  backend.set_backend(backend.HipBackend())
  return ctx


@pytest.fixture
def gpu_workers(gpu_ctx):
  """Set FLAGS.num_workers (virtual workers sharing the GPU) for one test."""
  from spartan_amd.config import FLAGS
  from spartan_amd.expr.base import eval_cache

  def setw(n):
    FLAGS.num_workers = n
    gpu_ctx.num_workers = n
    return gpu_ctx
  yield setw
  FLAGS.num_workers = None
  gpu_ctx.num_workers = 1
  eval_cache.clear()
