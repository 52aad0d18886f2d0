"""TEST DOUBLE of spartan_amd.backend.HipBackend for CPU-only host-logic tests.

It implements the same tensor-level interface with NumPy on CPU tensors so the
expression layer, tile placement, SPMD collectives (gloo) and partial-combine
logic can be exercised without a GPU.  It is installed only by tests through
``spartan_amd.backend.set_backend``; product code never selects it, and the
GPU tests (``-m gpu``) never use it.
"""
import numpy as np
import torch

from spartan_amd import backend as B
from spartan_amd import codegen
from spartan_amd.layout import broadcast_strides
from oracle import rng


def _np(t):
  return t.detach().cpu().numpy()


def _put(t, arr):
  t.copy_(torch.as_tensor(np.ascontiguousarray(arr)).reshape(t.shape))


def eval_ir(node, arrays, shape):
  if isinstance(node, codegen.In):
    a = arrays[node.slot]
    return np.broadcast_to(a.reshape(a.shape), shape) if a.ndim else np.full(shape, a[()], a.dtype)
  if isinstance(node, codegen.Sc):
    return node.value
  if isinstance(node, codegen.Const):
    return np.full(shape, node.value, dtype=node.dtype)
  if isinstance(node, codegen.Cast):
    v = eval_ir(node.arg, arrays, shape)
    return np.asarray(v).astype(node.dtype)
  if isinstance(node, codegen.RowDot):
    a = np.asarray(eval_ir(node.a, arrays, shape), dtype=node.dtype)
    w = np.asarray(eval_ir(node.w, arrays, shape), dtype=node.dtype)
    return np.broadcast_to(a.dot(w[0].reshape(-1, 1)), shape)
  args = []
  for a, dt in zip(node.args, node.in_dtypes):
    v = eval_ir(a, arrays, shape)
    args.append(np.asarray(v, dtype=dt) if not isinstance(a, codegen.Sc) else np.asarray(v).astype(dt))
  with np.errstate(all='ignore'):
    r = getattr(np, node.name)(*args)
  return np.asarray(r).astype(node.dtype)


class FakeBackend:
  name = 'fake'

  def __init__(self):
    self.calls = []

  def fill(self, out, kind, a, b, seed, ul, array_shape):
    dt = B.np_dtype(out.dtype)
    shape = tuple(out.shape)
    n = int(np.prod(shape))
    if len(shape):
      li = np.arange(n)
      idx = np.unravel_index(li, shape)
      g = np.ravel_multi_index(tuple(i + u for i, u in zip(idx, ul)), tuple(array_shape))
    else:
      g = np.zeros(1, dtype=np.int64)
    if kind == B.FILL_CONST:
      if dt.kind in 'iu':
        info = np.iinfo(dt)
        iv = info.max if a >= info.max else (info.min if a <= info.min else int(a))
        v = np.full(n, iv, dtype=dt)
      else:
        v = np.full(n, a, dtype=dt)
    elif kind == B.FILL_ARANGE:
      v = rng.arange_values(g, a, b, dt)
    elif kind == B.FILL_NORMAL:
      v = rng.normal_values(g, seed, a, b, dt)
    else:
      v = rng.uniform_values(g, seed, a, b, dt)
    _put(out, v.reshape(shape))
    self.calls.append('fill')

  def contiguous(self, t, dtype=None):
    out = t.contiguous()
    return out if dtype is None else out.to(B.torch_dtype(dtype))

  def map(self, root, inputs, out):
    shape = tuple(out.shape)
    arrays = {s: _np(t) for s, t in inputs.items()}
    r = eval_ir(root, arrays, shape)
    _put(out, np.asarray(r).astype(root.dtype).reshape(shape))
    self.calls.append('map')

  def reduce(self, root, op, inputs, in_shape, axis, out_shape, out_dtype, idx_geom=None):
    arrays = {s: _np(t) for s, t in inputs.items()}
    vals = np.asarray(eval_ir(root, arrays, tuple(in_shape))).reshape(in_shape)
    adt = codegen.acc_dtype(op, root.dtype)
    vals = vals.astype(adt)
    self.calls.append('reduce')
    if op in ('argmin', 'argmax'):
      f = np.argmin if op == 'argmin' else np.argmax
      idx = f(vals, axis=axis)
      v = (np.min if op == 'argmin' else np.max)(vals, axis=axis)
      g = idx_geom or {}
      if axis is None:
        if g.get('decompose'):
          loc = np.unravel_index(idx, g['tshape'])
          idx = np.ravel_multi_index(tuple(l + u for l, u in zip(loc, g['tul'])), g['ashape'])
        else:
          idx = idx + g.get('offset', 0)
      else:
        idx = idx + g.get('offset', 0)
      ti = torch.as_tensor(np.asarray(idx, dtype=np.int64).reshape(out_shape))
      tv = torch.as_tensor(np.asarray(v).reshape(out_shape))
      return tv, ti
    f = {'sum': np.sum, 'min': np.min, 'max': np.max}[op]
    r = f(vals, axis=axis)
    return torch.as_tensor(np.asarray(r).astype(out_dtype).reshape(out_shape))

  def finalize(self, op, parts, P, n, out):
    v = _np(parts).reshape(P, n)
    f = {'sum': np.add, 'min': np.minimum, 'max': np.maximum}[op]
    acc = v[0].copy()
    for p in range(1, P):
      acc = f(acc, v[p])
    _put(out, acc.astype(B.np_dtype(out.dtype)))
    self.calls.append('finalize')

  def argcombine(self, op, vals, idx):
    v = _np(vals)
    i = _np(idx)
    R, n = v.shape
    bv, bi = v[0].copy(), i[0].copy()
    EMPTY = np.iinfo(np.int64).max
    for r in range(1, R):
      for k in range(n):
        cv, ci = v[r, k], i[r, k]
        if ci == EMPTY:
          continue
        if bi[k] == EMPTY:
          better = True
        elif cv == bv[k]:
          better = ci < bi[k]
        else:
          better = cv < bv[k] if op == 'argmin' else cv > bv[k]
        if better:
          bv[k], bi[k] = cv, ci
    return torch.as_tensor(bv), torch.as_tensor(bi)

  def merge(self, dst, mask, region_ul, src, op, fastpath=True):
    d = _np(dst).copy()
    s = _np(src)
    sl = tuple(slice(u, u + n) for u, n in zip(region_ul, s.shape))
    if op == 'replace':
      d[sl] = s
    else:
      f = {'sum': np.add, 'min': np.minimum, 'max': np.maximum}[op]
      if mask is not None:
        m = _np(mask).astype(bool)[sl]
        reg = d[sl]
        reg[~m] = s[~m]
        reg[m] = f(reg[m], s[m])
        d[sl] = reg
        mm = _np(mask).copy()
        mm[sl] = 1
        _put(mask, mm)
      else:
        d[sl] = f(d[sl], s.astype(d.dtype))
    _put(dst, d)

  def copy_region(self, dst, dst_ul, src, src_ul, shape):
    d = _np(dst).copy()
    s = _np(src)
    dsl = tuple(slice(u, u + n) for u, n in zip(dst_ul, shape))
    ssl = tuple(slice(u, u + n) for u, n in zip(src_ul, shape))
    d[dsl] = s[ssl].astype(d.dtype)
    _put(dst, d)

  def gemm(self, A, Bm, C, alpha=1.0, beta=0.0):
    a, b = _np(A), _np(Bm)
    r = a @ b
    if alpha != 1.0:
      r = r * alpha
    if beta != 0.0:
      r = r + beta * _np(C)
    C.copy_(torch.as_tensor(np.ascontiguousarray(r.astype(_np(C).dtype))))

  def kmeans_assign(self, points, centers, labels, mindist=None, exact_only=False, dist_dtype=np.float64):
    from scipy.spatial.distance import cdist
    d = cdist(_np(points).astype(np.float64), _np(centers)).astype(dist_dtype)
    labels.copy_(torch.as_tensor(d.argmin(1).astype(np.int64)))

  def cdist(self, points, centers, out):
    from scipy.spatial.distance import cdist
    d = cdist(_np(points).astype(np.float64), _np(centers))
    out.copy_(torch.as_tensor(d.astype(B.np_dtype(out.dtype))))

  def bincount(self, labels, counts, zero_first=True):
    lab = _np(labels).reshape(-1)
    K = counts.numel()
    lab = lab[(lab >= 0) & (lab < K)]
    c = np.bincount(lab, minlength=K).astype(np.int64)
    if not zero_first:
      c = c + _np(counts)
    counts.copy_(torch.as_tensor(c))

  def kmeans_accumulate(self, points, labels, sums, counts, zero_first=True):
    p = _np(points).astype(np.float64)
    lab = _np(labels)
    K = sums.shape[0]
    s = np.zeros((K, p.shape[1])) if zero_first else _np(sums).copy()
    c = np.zeros(K, np.int64) if zero_first else _np(counts).copy()
    np.add.at(s, lab, p)
    np.add.at(c, lab, 1)
    sums.copy_(torch.as_tensor(s))
    counts.copy_(torch.as_tensor(c))

  def kmeans_step(self, points, centers, labels, sums, counts, zero_first=True, dist_dtype=np.float64):
    self.kmeans_assign(points, centers, labels, dist_dtype=dist_dtype)
    self.kmeans_accumulate(points, labels, sums, counts, zero_first=zero_first)
