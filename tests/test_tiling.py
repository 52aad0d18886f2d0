"""Placement KATs: good_tile_shape / compute_extents / round robin
(spartan/array/distarray.py:24-106, 438-442)."""
import pytest

from spartan_amd.array import distarray
from oracle import spartan_cpu as O


def test_good_tile_shape_row_strips():
  assert distarray.good_tile_shape((32768, 32768), 8) == [4096, 32768]
  assert distarray.good_tile_shape((32768, 32768), 1) == [32768, 32768]
  assert distarray.good_tile_shape((2000, 2000), 4) == [500, 2000]
  assert distarray.good_tile_shape((50, 50), 3) == [16, 50]
  assert distarray.good_tile_shape((50, 50, 50), 3) == [16, 50, 50]
  assert distarray.good_tile_shape((32768,), 8) == [4096]


def test_remainder_tile_quirk():
  # (1e8, 128) on 3 workers: 33,333,333-row tiles, 4 tiles, last has 1 row
  ex = distarray.compute_extents((100000000, 128), None, 3)
  rows = [e.lr[0] - e.ul[0] for e in ex]
  assert rows == [33333333, 33333333, 33333333, 1]
  assert list(ex.values()) == [0, 1, 2, 0]


def test_round_robin_matches_oracle():
  for shape, W in [((32768, 32768), 8), ((257, 131), 3), ((50, 50, 50), 3), ((7,), 3), ((5, 3), 8)]:
    got = [((e.ul, e.lr), w) for e, w in distarray.compute_extents(shape, None, W).items()]
    want = [((e[0], e[1]), w) for e, w in O.compute_extents(shape, W)]
    assert got == want


def test_scalar_array_single_tile():
  ex = distarray.compute_extents((), None, 4)
  (e, w), = ex.items()
  assert e.ndim == 0 and w == 0


def test_mincost_solver_matches_restatement():
  """libspx's spx_mincost_tiling (host C++) against the Python restatement of
  tiling.cc's find_mincost_tiling (oracle/tiling.py) on random DAGs with
  split pairs, repeated arcs and cost ties."""
  import random
  from spartan_amd import backend
  from oracle import tiling as OT
  rnd = random.Random(7)
  for _ in range(1500):
    t = rnd.randint(2, 15)
    edges = []
    for v in range(1, t + 1):
      for _ in range(rnd.randint(1, 3)):
        edges.append((rnd.randint(0, v - 1), v, rnd.choice([0, 0, 1, 5, 10, rnd.randint(0, 100)])))
    nodes = list(range(1, t))
    rnd.shuffle(nodes)
    pairs = [(nodes[i], nodes[i + 1]) for i in range(0, rnd.randint(0, len(nodes) // 2) * 2, 2)]
    assert backend.mincost_tiling(t, edges, pairs) == OT.mincost_tiling(t, edges, pairs)
  with pytest.raises(ValueError):
    backend.mincost_tiling(3, [(0, 9, 1)], [])


def test_mincost_solver_known_answer():
  """Source -> two tilings {1, 2} of one array; 1 -> 3 costs 100, 2 -> 3 costs
  0; 3 -> sink 4: tiling 2 must be chosen, total 0."""
  from spartan_amd import backend
  from oracle import tiling as OT
  edges = [(0, 1, 0), (0, 2, 0), (1, 3, 100), (2, 3, 0), (3, 4, 0)]
  assert backend.mincost_tiling(4, edges, [(1, 2)]) == ([2, 3], 0) == OT.mincost_tiling(4, edges, [(1, 2)])
