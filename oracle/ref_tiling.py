"""Oracle (test infrastructure): ctypes access to the reference's own
min-cost tiling search, compiled from /root/reference/spartan/expr/tiling.cc
lines 1-92 by oracle/build_ref.sh into oracle/_ref/libreftiling.so
(see oracle/ref_tiling_harness.cpp).  Only tests load it; spartan_amd never
does."""
import ctypes
import os

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), '_ref', 'libreftiling.so')
_lib = None


def available():
  return os.path.exists(LIB)


def _load():
  global _lib
  if _lib is None:
    _lib = ctypes.CDLL(LIB)
    I32P, I64P = ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_long)
    _lib.ref_mincost_tiling.argtypes = [ctypes.c_int, ctypes.c_long, I32P, I32P, I64P, ctypes.c_long, I32P, I32P,
                                        ctypes.POINTER(ctypes.c_uint8), I64P]
    _lib.ref_mincost_tiling.restype = ctypes.c_long
  return _lib


def mincost_tiling(t, edges, split_pairs):
  """Same signature and result as oracle.tiling.mincost_tiling /
  backend.mincost_tiling: (sorted chosen node ids < t, total cost)."""
  lib = _load()
  n, m = len(edges), len(split_pairs)
  eu = (ctypes.c_int32 * max(n, 1))(*[u for u, _, _ in edges])
  ev = (ctypes.c_int32 * max(n, 1))(*[v for _, v, _ in edges])
  ec = (ctypes.c_long * max(n, 1))(*[c for _, _, c in edges])
  sa = (ctypes.c_int32 * max(m, 1))(*[a for a, _ in split_pairs])
  sb = (ctypes.c_int32 * max(m, 1))(*[b for _, b in split_pairs])
  chosen = (ctypes.c_uint8 * max(t, 1))()
  cost = ctypes.c_long()
  if lib.ref_mincost_tiling(int(t), n, eu, ev, ec, m, sa, sb, chosen, ctypes.byref(cost)) != 0:
    raise ValueError('ref_mincost_tiling: graph out of the reference tables\' range')
  return [u for u in range(t) if chosen[u]], int(cost.value)
