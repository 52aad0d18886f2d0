"""Placement KATs: good_tile_shape / compute_extents / round robin
(spartan/array/distarray.py:24-106, 438-442)."""
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
