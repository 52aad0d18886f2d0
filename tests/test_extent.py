"""Extent math KATs -- restated from the reference's tests/test_extent.py:6-50
plus the Appendix-A pins of SURVEY.md (bit-exact integer semantics)."""
import random

import numpy as np

from spartan_amd.array import extent


def test_intersection():
  a = extent.create((0, 0), (10, 10), None)
  b = extent.create((5, 5), (6, 6), None)
  assert extent.intersection(a, b) == extent.create((5, 5), (6, 6), None)
  assert extent.intersection(b, a) == extent.create((5, 5), (6, 6), None)
  a = extent.create((5, 5), (10, 10), None)
  b = extent.create((4, 6), (6, 8), None)
  assert extent.intersection(a, b) == extent.create((5, 6), (6, 8), None)
  a = extent.create((5, 5), (5, 5), None)  # empty -> None
  assert a is None
  b = extent.create((1, 1), (2, 2), None)
  assert extent.intersection(a, b) is None
  # touching extents do not intersect
  assert extent.intersection(extent.create((0,), (5,), (10,)), extent.create((5,), (10,), (10,))) is None


def test_local_offset():
  a = extent.create((0, 0), (5, 5), None)
  b = extent.create((2, 2), (3, 3), None)
  assert extent.offset_from(a, b) == extent.create((2, 2), (3, 3), None)
  assert extent.offset_slice(a, b) == (slice(2, 3, None), slice(2, 3, None))


def test_ravelled_pos():
  a = extent.create((2, 2), (7, 7), (10, 10))
  for i in range(10):
    for j in range(10):
      assert extent.ravelled_pos((i, j), a.array_shape) == 10 * i + j
  assert a.to_global(0, axis=None) == 22
  assert a.to_global(10, axis=None) == 42
  assert a.to_global(11, axis=None) == 43
  assert a.to_global(20, axis=None) == 62


def test_unravel():
  rnd = random.Random(0)
  for _ in range(100):
    shp = (20, 77)
    ul = (rnd.randint(0, 19), rnd.randint(0, 76))
    lr = (rnd.randint(ul[0] + 1, 20), rnd.randint(ul[1] + 1, 77))
    a = extent.create(ul, lr, shp)
    assert extent.unravelled_pos(a.ravelled_pos(), a.array_shape) == a.ul
  assert extent.unravelled_pos(11, (10, 10)) == (1, 1)  # py2 floor division pinned


def test_shape_zero_len_as_one_and_drop_axis():
  ex = extent.TileExtent((0, 3), (4, 3), (4, 8))
  assert ex.shape == (4, 1)
  d = extent.drop_axis(extent.create((0, 0), (4096, 32768), (32768, 32768)), 0)
  assert d == extent.create((0,), (32768,), (32768,)) and d.array_shape == (32768,)
  assert extent.drop_axis(d, None).ndim == 0
  assert extent.shape_for_reduction((3, 4, 5), 1) == (3, 5)
  assert extent.shape_for_reduction((3, 4), None) == ()


def test_change_partition_axis():
  ex = extent.create((500, 0), (1000, 2000), (2000, 2000))
  assert extent.change_partition_axis(ex, 1) == extent.create((0, 500), (2000, 1000), (2000, 2000))
  ex = extent.create((0, 0), (33, 100), (132, 100))
  got = extent.change_partition_axis(ex, 1)
  assert got.ul == (0, 0) and got.lr == (132, 25)
  v = extent.create((10,), (20,), (100,))
  assert extent.change_partition_axis(v, 1) == extent.create((0,), (100,), (100,))
  assert extent.change_partition_axis(v, 0) is v


def test_from_slice_and_compute_slice():
  ex = extent.from_slice(np.index_exp[:], (4, 6))
  assert ex.ul == (0, 0) and ex.lr == (4, 6)
  ex = extent.from_slice((slice(1, 3), 2), (4, 6))
  assert ex.ul == (1, 2) and ex.lr == (3, 3)
  base = extent.create((10, 0), (20, 6), (40, 6))
  sub = extent.compute_slice(base, (slice(2, 5),))
  assert sub.ul == (12, 0) and sub.lr == (15, 6)


def test_find_overlapping_and_shape():
  exs = [extent.create((i * 10,), ((i + 1) * 10,), (40,)) for i in range(4)]
  got = list(extent.find_overlapping(exs, extent.create((5,), (25,), (40,))))
  assert [g[1].ul for g in got] == [(5,), (10,), (20,)]
  assert extent.find_shape(exs) == (40,)
