"""Iteration-space layout: NumPy broadcasting -> per-input element strides.

Host-side index bookkeeping shared by every backend.  Given the shape of the
tile being produced and the shapes of the (contiguous) input tiles, compute
each input's strides in the output index space (0 on broadcast dims, the
reference's ``Broadcast.fetch_base_tile`` + NumPy broadcasting,
spartan/expr/broadcast.py:98-109 / spartan/expr/map.py:33-45) and coalesce
adjacent dims that are contiguous for every input, so the generated kernels see
at most a handful of dims.
"""
from .util import prod


def contiguous_strides(shape):
  st = [0] * len(shape)
  acc = 1
  for d in range(len(shape) - 1, -1, -1):
    st[d] = acc
    acc *= int(shape[d])
  return st


def broadcast_strides(in_shape, out_shape, in_strides=None):
  """Strides (elements) of an ``in_shape`` tensor viewed as ``out_shape``.
  ``in_strides``: the tensor's own element strides (a strided view such as a
  transpose, consumed in place by the generated kernels); default contiguous."""
  in_shape = tuple(int(s) for s in in_shape)
  out_shape = tuple(int(s) for s in out_shape)
  own = list(in_strides) if in_strides is not None else contiguous_strides(in_shape)
  if len(in_shape) > len(out_shape):
    # leading size-1 dims may be dropped
    extra = len(in_shape) - len(out_shape)
    assert all(s == 1 for s in in_shape[:extra]), (in_shape, out_shape)
    in_shape = in_shape[extra:]
    own = own[extra:]
  pad = len(out_shape) - len(in_shape)
  full = (1,) * pad + in_shape
  cst = [0] * pad + [int(x) for x in own]
  out = []
  for d, (si, so) in enumerate(zip(full, out_shape)):
    if si == so:
      out.append(cst[d] if so != 1 else 0)
    elif si == 1:
      out.append(0)
    else:
      raise ValueError('shape %s does not broadcast to %s' % (in_shape, out_shape))
  return out


def coalesce(shape, strides_list):
  """Merge adjacent dims contiguous for every input; drop size-1 dims.

  Returns (shape', [strides'...]); shape' has at least one dim."""
  dims = [(int(s), [st[d] for st in strides_list]) for d, s in enumerate(shape) if int(s) != 1]
  if not dims:
    return [1], [[0] for _ in strides_list]
  merged = [dims[0]]
  for s, st in dims[1:]:
    ps, pst = merged[-1]
    if all(pst[k] == st[k] * s for k in range(len(st))):
      merged[-1] = (ps * s, st)
    else:
      merged.append((s, st))
  shape_out = [m[0] for m in merged]
  strides_out = [[m[1][k] for m in merged] for k in range(len(strides_list))]
  return shape_out, strides_out


def reduce_view(shape, strides_list, axis):
  """(O, R, I) view of a reduction over ``axis`` (None = all dims).

  Returns (O, R, I, [(so, sr, si)...]) or None when a group of dims cannot be
  collapsed to a single strided dim for every input."""
  nd = len(shape)
  if axis is None:
    groups = [list(range(0)), list(range(nd)), []]
  else:
    groups = [list(range(axis)), [axis], list(range(axis + 1, nd))]
  out_dims = []
  out_str = [[] for _ in strides_list]
  for g in groups:
    sub_shape = [shape[d] for d in g]
    sub_str = [[st[d] for d in g] for st in strides_list]
    if not g or prod(sub_shape) == 1:
      out_dims.append(1)
      for k in range(len(strides_list)):
        out_str[k].append(0)
      continue
    cs, cst = coalesce(sub_shape, sub_str)
    if len(cs) != 1:
      return None
    out_dims.append(cs[0])
    for k in range(len(strides_list)):
      out_str[k].append(cst[k][0])
  return out_dims[0], out_dims[1], out_dims[2], [tuple(s) for s in out_str]
