"""Host ingest (restates from_numpy, spartan/expr/write_array.py:411-433)."""
import numpy as np

from ..array import distarray
from .base import Val


def from_numpy(a, tile_hint=None):
  """Upload a NumPy array into HBM tiles (each rank copies the tiles it owns)."""
  if not isinstance(a, np.ndarray):
    raise TypeError('Expected ndarray, got: %s' % type(a))
  return Val(val=distarray.from_numpy(a, tile_hint=tile_hint))
