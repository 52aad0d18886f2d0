"""(f1) AutomaticTiling's solver pinned to the reference's OWN code: libspx's
spx_mincost_tiling against find_mincost_tiling compiled from
/root/reference/spartan/expr/tiling.cc:1-92 (oracle/build_ref.sh ->
oracle/_ref/libreftiling.so), on the AutomaticTiling graphs of the
configs[0] / configs[1] / configs[3] / configs[4] DAGs and on random graphs
with split pairs, repeated arcs and cost ties.  Identical chosen sets and
costs are required.  The library is built in this container by build() (it
needs the reference tree); where it is absent the tests skip."""
import random

import numpy as np
import pytest

from oracle import ref_tiling as RT
from oracle import tiling as OT

pytestmark = pytest.mark.skipif(not RT.available(), reason='oracle/_ref/libreftiling.so not built '
                                '(bash oracle/build_ref.sh needs /root/reference)')


def _random_graphs(seed, count, tie_heavy=False):
  rnd = random.Random(seed)
  for _ in range(count):
    t = rnd.randint(2, 18)
    edges = []
    for v in range(1, t + 1):
      for _ in range(rnd.randint(1, 3)):
        c = rnd.choice([0, 0, 1, 1, 2]) if tie_heavy else rnd.choice([0, 0, 1, 5, 10, rnd.randint(0, 100)])
        edges.append((rnd.randint(0, v - 1), v, c))
    nodes = list(range(1, t))
    rnd.shuffle(nodes)
    pairs = [(nodes[i], nodes[i + 1]) for i in range(0, rnd.randint(0, len(nodes) // 2) * 2, 2)]
    yield t, edges, pairs


def test_random_graphs_match_reference():
  from spartan_amd import backend
  n = 0
  for t, edges, pairs in _random_graphs(11, 2000):
    want = RT.mincost_tiling(t, edges, pairs)
    assert backend.mincost_tiling(t, edges, pairs) == want, (t, edges, pairs)
    assert OT.mincost_tiling(t, edges, pairs) == want
    n += 1
  assert n == 2000


def test_tie_heavy_graphs_match_reference():
  """Costs drawn from {0, 1, 2}: most split choices tie, which exercises the
  deferred-tie re-queue (tiling.cc:67-69) and its resolution."""
  from spartan_amd import backend
  for t, edges, pairs in _random_graphs(12, 2000, tie_heavy=True):
    assert backend.mincost_tiling(t, edges, pairs) == RT.mincost_tiling(t, edges, pairs), (t, edges, pairs)


def _captured_graphs(host_ctx, build):
  """Every (t, edges, split pairs) AutomaticTiling hands the solver while
  ``build()``'s expressions are optimised."""
  from spartan_amd import backend
  seen = []
  real = backend.mincost_tiling

  def spy(t, edges, pairs):
    seen.append((t, list(edges), list(pairs)))
    return real(t, edges, pairs)
  backend.mincost_tiling = spy
  try:
    build()
  finally:
    backend.mincost_tiling = real
  return seen


@pytest.mark.parametrize('W', [1, 3, 8])
def test_config_dags_match_reference(host_ctx, W):
  host_ctx(W)
  from spartan_amd import expr

  def build():
    # configs[0]: sum(dot(ones, ones)) (tests/benchmark_dot.py), configs[1]:
    # sum(x * y + exp(z), axis) on new arrays, configs[3]: dot of two new
    # arrays, configs[4]: the lreg gradient sum(x * (dot(x, w) - y), axis=0)
    n = 48
    expr.sum(expr.dot(expr.ones((n, n)), expr.ones((n, n)))).optimized()
    for ax in (0, 1, None):
      x, y, z = (expr.rand(n, 40, seed=s) for s in (1, 2, 3))
      expr.sum(x * y + expr.exp(z), axis=ax).optimized()
    expr.dot(expr.rand(n, 40, seed=4), expr.rand(40, 24, seed=5)).optimized()
    x = expr.rand(n, 8, seed=6)
    yv = expr.rand(n, 1, seed=7)
    w = np.full((8, 1), 0.5, np.float32)
    expr.sum(x * (expr.dot(x, w) - yv), axis=0).optimized()
  graphs = _captured_graphs(host_ctx, build)
  assert len(graphs) >= 6
  from spartan_amd import backend
  for t, edges, pairs in graphs:
    assert pairs, 'AutomaticTiling graphs carry split pairs'
    assert backend.mincost_tiling(t, edges, pairs) == RT.mincost_tiling(t, edges, pairs), (t, edges, pairs)
