"""Tile-loop engine behind MapExpr / ReduceExpr evaluation (SPMD, HBM tiles).

What the reference does per worker with NumPy (tile_mapper,
spartan/expr/map.py:48-88; _reduce_mapper, spartan/expr/reduce.py:19-68;
DistArray.update + tile.merge for the partials) is done here per rank:

 1. bind the children of the fused node to kernel inputs: host scalars become
    kernel-argument constants, arrays become device tiles;
 2. plan, on every rank identically, which child regions each output tile
    needs; regions not resident on the tile's rank are moved by one
    collective ``gather_regions`` (row-strip co-tiled inputs need none);
 3. lower the LocalExpr tree once and launch ONE generated kernel per local
    tile (map, or fused map+reduce);
 4. for reductions, combine the tile partials: written straight into the
    output tile when the partial lands exactly on a tile of the same rank,
    otherwise merged locally and combined across ranks with RCCL
    (reduce_scatter / all_reduce; all_gather + spx_argreduce_combine for
    argmin/argmax, which RCCL has no operator for).
"""
import numpy as np

from .. import backend, codegen, comm, runtime
from ..array import distarray, extent as ext
from ..array.distarray import DistArrayImpl, LocalWrapper, ReplicatedArray
from ..util import prod
from .broadcast import Broadcast
from .local import CodegenError, LowerEnv, Pre, UntraceableMapper, has_location, host_evaluate, lower


# --------------------------------------------------------------- binding
def _scalar_value(child):
  """Host scalar carried by a child, or None."""
  base = child.base if isinstance(child, Broadcast) else child
  if isinstance(base, LocalWrapper) and not isinstance(base, ReplicatedArray) and base.value.ndim == 0:
    v = base.value
    return v.item() if hasattr(v, 'item') else v
  return None


_BIND_MEMO = {}


def bind(children, child_to_var, op, extent=None):
  """Lower ``op`` with children bound to IR leaves (``extent``: the tile, for
  trees holding a location map).

  Returns (root, array_slots {slot: child index}, pres [Pre leaves]).

  A LocalExpr tree that a replayed plan shares between iterations
  (plan_cache marks it ``_tpl_pure``) is lowered once per binding pattern
  (which children are host scalars, their values, the array dtypes); the
  entry holds the tree, so its id cannot be reused while the entry lives."""
  key = None
  if extent is None and op.__dict__.get('_tpl_pure'):
    desc = []
    for child in children:
      sv = _scalar_value(child)
      # floats by their repr: 0.0 and -0.0 (and nan) must not share a lowering
      desc.append(('a', child.dtype.str) if sv is None else
                  (type(sv), repr(sv) if isinstance(sv, (float, np.floating)) else sv))
    key = (id(op), tuple(child_to_var), tuple(desc))
    hit = _BIND_MEMO.get(key)
    if hit is not None:
      return hit[1]
  out = _bind(children, child_to_var, op, extent)
  if key is not None:
    if len(_BIND_MEMO) >= 256:
      _BIND_MEMO.clear()
    _BIND_MEMO[key] = (op, out)
  return out


def _bind(children, child_to_var, op, extent=None):
  env = LowerEnv({}, extent)
  slots = {}
  for i, (child, var) in enumerate(zip(children, child_to_var)):
    sv = _scalar_value(child)
    if sv is not None:
      env.leaves[var] = env.new_scalar(sv)
    else:
      slot = len(slots)
      env.leaves[var] = codegen.In(slot, child.dtype)
      slots[slot] = i
  root = lower(op, env)
  used = {n.slot for n in codegen.walk(root) if isinstance(n, codegen.In) and not isinstance(n, Pre)}
  pres = [n for n in codegen.walk(root) if isinstance(n, Pre)]
  # compact slots: referenced array inputs first, then generator leaves
  remap = {}
  for old in sorted(used):
    remap[old] = len(remap)
  for n in codegen.unique_nodes(root):
    if isinstance(n, codegen.In) and not isinstance(n, Pre):
      n.slot = remap[n.slot]
  seen = {}
  for p in pres:
    if id(p) not in seen:
      seen[id(p)] = len(remap) + len(seen)
      p.slot = seen[id(p)]
  if len(remap) + len(seen) > codegen.MAX_IN:
    raise CodegenError('fused expression has more than %d array inputs' % codegen.MAX_IN)
  array_slots = {remap[s]: slots[s] for s in used}
  uniq_pres = []
  for p in pres:
    if p not in uniq_pres:
      uniq_pres.append(p)
  return root, array_slots, uniq_pres


# ------------------------------------------------------------ tile plan
def driving_tiles(largest):
  """{extent: worker} of the iteration space (broadcast drivers expand their base tiles)."""
  if isinstance(largest, Broadcast):
    out = {}
    for bex, w in largest.base.tiles.items():
      ul = [0] * len(largest.shape)
      lr = list(largest.shape)
      for i in range(len(bex.ul) - 1, -1, -1):
        bi = i + largest.prepend_dim
        if largest.base.shape[i] == largest.shape[bi]:
          ul[bi], lr[bi] = bex.ul[i], bex.lr[i]
      out[ext.create(ul, lr, largest.shape)] = w
    return out
  return dict(largest.tiles)


def _child_region(child, ex):
  if isinstance(child, Broadcast):
    return child.base, child._base_ex(ex)
  return child, ex


def fetch_inputs(children, slots_to_child, tiles):
  """For every local driving extent: {slot: device tensor}.  Collective."""
  ctx = runtime.get()
  per_ex = {ex: {} for ex, w in tiles.items() if ctx.is_local(w) or w == -1}
  for slot, ci in slots_to_child.items():
    arr, _ = _child_region(children[ci], next(iter(tiles)))
    requests, req_ex = [], []
    local_fetch = []
    for ex, w in tiles.items():
      dst = ctx.owner(w) if w != -1 else ctx.rank
      a, region = _child_region(children[ci], ex)
      owner = a.owner_of_region(region) if not a.replicated else dst
      if owner == dst or w == -1:
        if dst == ctx.rank:
          local_fetch.append((ex, a, region))
      else:
        requests.append((region, dst))
        req_ex.append(ex)
    for ex, a, region in local_fetch:
      per_ex[ex][slot] = a.fetch(region)
    if requests:
      got = distarray.gather_regions(arr, requests)
      for qi, t in got.items():
        per_ex[req_ex[qi]][slot] = t
  return per_ex


def materialise_pres(pres, children, child_to_var, ex, inputs):
  """Fill generator leaves (rand / arange) for extent ``ex`` into temp tiles."""
  import torch
  ctx = runtime.get()
  be = backend.get()
  for p in pres:
    t = torch.empty(ex.shape if ex.ndim else (), dtype=backend.torch_dtype(p.dtype), device=ctx.device)
    kind, a, b, seed = p.params
    be.fill(t, kind, a, b, seed, ex.ul, ex.array_shape if ex.array_shape is not None else ())
    inputs[p.slot] = t


# ----------------------------------------------------------------- map
def run_location_map(children, child_to_var, op):
  """A map whose tree holds a map_with_location call: lowered once per tile
  with that tile's extent (map_with_location.py:22-60), one kernel per tile.

  Tracing is per tile, so only ranks holding a tile that fails to trace would
  see UntraceableMapper, and only ranks holding tiles can see two result
  dtypes: both are decided over all ranks (control plane) before any rank
  branches, so every rank takes the same path and raises the same error."""
  import torch
  ctx = runtime.get()
  be = backend.get()
  largest = distarray.largest_value(children)
  tiles = driving_tiles(largest)
  arrays = {i: i for i, c in enumerate(children) if _scalar_value(c) is None}
  per_ex = fetch_inputs(children, arrays, tiles)
  bound, untraceable, dtypes = {}, None, set()
  for ex in per_ex:
    try:
      bound[ex] = bind(children, child_to_var, op, extent=ex)
    except UntraceableMapper as e:
      untraceable = e
      break
    dtypes.add(np.dtype(bound[ex][0].dtype))
  if ctx.distributed:
    if comm.max_over_ranks(1.0 if untraceable is not None else 0.0) and untraceable is None:
      untraceable = UntraceableMapper('map_with_location mapper could not be traced on another rank')
  if untraceable is not None:
    return run_host_map(children, child_to_var, op, untraceable)
  if len(dtypes) > 1:
    mine = None  # _agree_dtype raises on every rank
  else:
    mine = next(iter(dtypes)) if dtypes else None
  if ctx.distributed or len(dtypes) > 1:
    dtype = _agree_dtype(mine, conflict=len(dtypes) > 1, what='location map')
  elif mine is None:  # no local tile: the dtype of the first tile's trace
    root, _, _ = bind(children, child_to_var, op, extent=next(iter(tiles)))
    dtype = np.dtype(root.dtype)
  else:
    dtype = mine
  out_local = {}
  for ex, fetched in per_ex.items():
    root, slots, pres = bound[ex]
    inputs = {slot: fetched[ci] for slot, ci in slots.items()}
    materialise_pres(pres, children, child_to_var, ex, inputs)
    out = torch.empty(ex.shape if ex.ndim else (), dtype=backend.torch_dtype(root.dtype), device=ctx.device)
    if isinstance(root, codegen.In) and not isinstance(root, Pre):
      be.copy_region(out, (0,) * out.dim(), inputs[root.slot], (0,) * out.dim(), tuple(out.shape))
    elif isinstance(root, (codegen.Const, codegen.Sc)):
      be.fill(out, backend.FILL_CONST, root.value, 0.0, 0, ex.ul, ex.array_shape or ())
    else:
      be.map(root, inputs, out)
    out_local[ex] = out
  if all(w == -1 for w in tiles.values()):
    (ex, out), = out_local.items()
    return ReplicatedArray(out)
  return distarray.from_tiles(largest.shape, dtype, tiles, out_local)


# ------------------------------------------------ untraceable user mappers
HOST_MAPPER_CALLS = [0]   # tiles evaluated on the host (tests assert on it)
_HOST_WARNED = set()


def _agree_dtype(dt, conflict=False, what='mapper'):
  """The result dtype every rank uses: ranks without a local tile learn it
  from the others (control plane).  If any rank saw two dtypes among its own
  tiles (``conflict``) or the ranks' dtypes differ, EVERY rank raises (one
  agreed verdict, so no rank goes on to a collective the others skip)."""
  codes = [np.dtype(t) for t in (np.bool_, np.int32, np.int64, np.float32, np.float64)]
  bad_type = dt is not None and np.dtype(dt) not in codes
  mine = -1 if dt is None or bad_type else codes.index(np.dtype(dt))
  hi = int(comm.max_over_ranks(float(mine)))
  lo = -int(comm.max_over_ranks(float(-mine if mine >= 0 else -99)))
  flags = int(comm.max_over_ranks(float(2 * bool(bad_type) + bool(conflict))))
  if flags & 2:
    raise TypeError('%s result dtype %s is not supported by the MI355X backend' % (what, dt))
  if flags & 1 or (hi >= 0 and lo != hi):
    raise CodegenError('%s yields different dtypes on different tiles or ranks' % what)
  if hi < 0:
    raise ValueError('map over an array without tiles')
  return codes[hi]


def run_host_map(children, child_to_var, op, err):
  """A map whose tree holds an untraceable USER mapper, evaluated like the
  reference's tile_mapper (spartan/expr/map.py:48-88): per local tile, the
  inputs come to the host (broadcast children as their base tiles, so NumPy
  broadcasts inside the mapper, as fetch_base_tile does), the tree runs in
  NumPy (local.host_evaluate), the result is checked against the tile shape
  and uploaded.  Counted in HOST_MAPPER_CALLS; warns once per mapper."""
  import warnings
  from ..array import transfer
  ctx = runtime.get()
  key = getattr(err, 'fn', None)
  if key not in _HOST_WARNED:
    _HOST_WARNED.add(key)
    warnings.warn('spartan_amd: %s -- evaluating it per tile on the host (NumPy), as the reference does' % err,
                  RuntimeWarning, stacklevel=3)
  largest = distarray.largest_value(children)
  tiles = driving_tiles(largest)
  arrays = {i: i for i, c in enumerate(children) if _scalar_value(c) is None}
  per_ex = fetch_inputs(children, arrays, tiles)
  out_local, dtype, conflict = {}, None, False
  for ex, fetched in per_ex.items():
    env = {'extent': ex}
    for i, (c, var) in enumerate(zip(children, child_to_var)):
      sv = _scalar_value(c)
      env[var] = sv if sv is not None else transfer.download(fetched[i])
    res = np.asarray(host_evaluate(op, env))
    shape = ex.shape if ex.ndim else ()
    if tuple(res.shape) != tuple(shape):  # tile_mapper's Assert.eq (map.py:80-82)
      raise AssertionError('Bad shape -- tile %s, mapper result %s' % (shape, res.shape))
    conflict = conflict or (dtype is not None and res.dtype != dtype)
    dtype = res.dtype
    out_local[ex] = res
    HOST_MAPPER_CALLS[0] += 1
  dtype = _agree_dtype(None if conflict else dtype, conflict=conflict)
  out_local = {ex: transfer.upload(np.ascontiguousarray(res, dtype=dtype), ctx.device)
               for ex, res in out_local.items()}
  if all(w == -1 for w in tiles.values()):
    (ex, out), = out_local.items()
    return ReplicatedArray(out)
  return distarray.from_tiles(largest.shape, dtype, tiles, out_local)


def run_map(children, child_to_var, op):
  ctx = runtime.get()
  try:
    if has_location(op):
      return run_location_map(children, child_to_var, op)
    largest = distarray.largest_value(children)
    root, slots, pres = bind(children, child_to_var, op)
  except UntraceableMapper as e:
    return run_host_map(children, child_to_var, op, e)
  tiles = driving_tiles(largest)
  replicated = all(w == -1 for w in tiles.values())
  # identity map returns the driving input itself (map.py:76-77)
  if isinstance(root, codegen.In) and not isinstance(root, Pre) and slots.get(root.slot) == 0 \
      and not isinstance(children[0], Broadcast):
    return children[0]
  per_ex = fetch_inputs(children, slots, tiles)
  import torch
  be = backend.get()
  out_local = {}
  for ex, inputs in per_ex.items():
    shape = ex.shape if ex.ndim else ()
    if isinstance(root, Pre):
      out = torch.empty(shape, dtype=backend.torch_dtype(root.dtype), device=ctx.device)
      kind, a, b, seed = root.params
      be.fill(out, kind, a, b, seed, ex.ul, ex.array_shape)
    elif isinstance(root, (codegen.Const, codegen.Sc)):
      out = torch.empty(shape, dtype=backend.torch_dtype(root.dtype), device=ctx.device)
      be.fill(out, backend.FILL_CONST, root.value, 0.0, 0, ex.ul, ex.array_shape or ())
    else:
      materialise_pres(pres, children, child_to_var, ex, inputs)
      out = torch.empty(shape, dtype=backend.torch_dtype(root.dtype), device=ctx.device)
      be.map(root, inputs, out)
    out_local[ex] = out
  if replicated:
    (ex, out), = out_local.items()
    return ReplicatedArray(out)
  return distarray.from_tiles(largest.shape, root.dtype, tiles, out_local)


# -------------------------------------------------------------- reduce
REDUCE_FNS = {}  # local_reduce_fn -> (op name, pre-transform of the mapped value or None)


def register_reduce(fn, op, transform=None):
  REDUCE_FNS[fn] = (op, transform)
  return fn


def run_reduce(children, child_to_var, local_op, axis, dtype, accumulate_fn, tile_hint):
  """Fused map+reduce.  ``local_op`` is a LocalReduceExpr(fn, [extent, tree])."""
  ctx = runtime.get()
  fn = local_op.fn
  if fn not in REDUCE_FNS:
    raise CodegenError('local reduce function %r has no gfx950 lowering' % (fn,))
  opname, transform = REDUCE_FNS[fn]
  tree = local_op.deps[1]
  largest = distarray.largest_value(children)
  try:
    root, slots, pres = bind(children, child_to_var, tree)
  except UntraceableMapper as e:
    # the mapped values on the host (reference semantics), then the same
    # device reduction over the materialised tiles
    from .local import LocalInput, LocalReduceExpr
    m = run_host_map(children, child_to_var, tree, e)
    return run_reduce([m], ['_host0'], LocalReduceExpr(fn=fn, deps=[LocalInput('extent'), LocalInput('_host0')]),
                      axis, dtype, accumulate_fn, tile_hint)
  if transform is not None:
    root = transform(root)
  in_shape_full = largest.shape
  nd = len(in_shape_full)
  ax = None if axis is None else (axis + nd if axis < 0 else axis)
  out_shape = ext.shape_for_reduction(children[0].shape, axis)
  arg = opname in ('argmin', 'argmax')
  out_dtype = np.dtype(np.int64) if arg else np.dtype(dtype)
  tiles = driving_tiles(largest)
  per_ex = fetch_inputs(children, slots, tiles)
  be = backend.get()
  partials = {}
  for ex, inputs in per_ex.items():
    materialise_pres(pres, children, child_to_var, ex, inputs)
    dst = ext.index_for_reduction(ex, ax)
    geom = None
    if arg:
      if ax is not None:
        geom = {'offset': ex.ul[ax]}
      elif all(ex.ul[d] == 0 and ex.lr[d] == in_shape_full[d] for d in range(1, nd)):
        geom = {'offset': ext.ravelled_pos(ex.ul, in_shape_full) if nd else 0}
      else:
        geom = {'decompose': True, 'tshape': ex.shape, 'tul': ex.ul, 'ashape': in_shape_full}
    partials[ex] = (dst, be.reduce(root, opname, inputs, ex.shape if nd else (), ax,
                                   dst.shape if dst.ndim else (), out_dtype, geom))
  output = distarray.create(out_shape, out_dtype, reducer=accumulate_fn, tile_hint=tile_hint)
  combine_partials(output, partials, tiles, ax, opname,
                   value_dtype=codegen.acc_dtype(opname, root.dtype) if arg else None)
  return output


def _identity(op, dt):
  dt = np.dtype(dt)
  if op == 'sum':
    return 0.0
  if dt.kind == 'f':
    return float('inf') if op == 'min' else float('-inf')
  if dt.kind == 'b':
    return 1.0 if op == 'min' else 0.0
  info = np.iinfo(dt)
  return float(info.max) if op == 'min' else float(info.min)


# How many times each cross-rank combine ran (tests assert the branch taken).
COMBINE_CALLS = {'reduce_scatter': 0, 'all_reduce': 0, 'gather_combine': 0, 'arg_gather': 0}


def combine_partials(output, partials, tiles, ax, opname, value_dtype=None):
  """Merge tile partials into ``output`` (reference: _reduce_mapper ->
  output.update(dst, partial) -> tile.merge with accumulate_fn).

  ``value_dtype``: for argmin/argmax, the dtype of the partial values (the
  same on every rank, also on ranks without a local partial)."""
  import torch
  ctx = runtime.get()
  be = backend.get()
  arg = opname in ('argmin', 'argmax')
  # every rank computes the same alignment decision from the global tile map
  dsts = [(ext.index_for_reduction(ex, ax), w) for ex, w in tiles.items()]
  seen = set()
  aligned = True
  for d, w in dsts:
    if d not in output.tiles or (d.ul, d.lr) in seen or \
        (w != -1 and ctx.owner(output.tiles[d]) != ctx.owner(w)):
      aligned = False
      break
    seen.add((d.ul, d.lr))
  if aligned:
    for ex, (d, part) in partials.items():
      t = output.local.get(d)
      if t is None:
        continue
      data = part[1] if arg else part
      if data.dtype != t.data.dtype:
        conv = torch.empty(t.data.shape, dtype=t.data.dtype, device=t.data.device)
        be.copy_region(conv, (0,) * conv.dim(), data, (0,) * conv.dim(), tuple(conv.shape))
        data = conv
      t.data = data.reshape(t.data.shape)
      t.written = [d]
    return
  shape = output.shape
  if arg:
    # values keep their own dtype end to end: int64 compares as int64 (a
    # float64 detour would merge distinct values above 2^53)
    vdt = backend.torch_dtype(value_dtype) if value_dtype is not None else None
    for _, (d, (pv, pi)) in partials.items():
      vdt = pv.dtype
    if vdt is None:
      raise ValueError('combine_partials: value dtype of the arg-reduction unknown on this rank')
    full_v = torch.zeros(shape, dtype=vdt, device=ctx.device)
    full_i = torch.empty(shape, dtype=torch.int64, device=ctx.device)
    be.fill(full_i, backend.FILL_CONST, 9.3e18, 0.0, 0, (0,) * len(shape), shape)
    for ex, (d, (pv, pi)) in partials.items():
      _arg_merge_region(be, full_v, full_i, d, pv, pi, opname)
    if ctx.distributed:
      COMBINE_CALLS['arg_gather'] += 1
      vs = comm.all_gather_stack(full_v.reshape(-1))
      is_ = comm.all_gather_stack(full_i.reshape(-1))
      _, best_i = be.argcombine(opname, vs, is_)
      full_i = best_i.reshape(shape)
    for d, t in output.local.items():
      _copy_out(be, t, full_i, d)
    return
  full = torch.empty(shape, dtype=backend.torch_dtype(output.dtype), device=ctx.device)
  be.fill(full, backend.FILL_CONST, _identity(opname, output.dtype), 0.0, 0, (0,) * len(shape), shape)
  for ex, (d, part) in partials.items():
    be.merge(full, None, d.ul, part.reshape(d.shape if d.ndim else ()), opname, fastpath=False)
  if ctx.distributed:
    if opname != 'sum':
      # min / max across ranks: gather every rank's partial and fold them in
      # rank order with the local kernels' NaN rule (np.minimum / np.maximum
      # propagate NaN; the collective library's MIN / MAX need not)
      COMBINE_CALLS['gather_combine'] += 1
      stack = comm.all_gather_stack(full.reshape(-1))
      n = full.numel()
      folded = torch.empty((n,), dtype=full.dtype, device=full.device)
      be.finalize(opname, stack.reshape(-1), ctx.world_size, n, folded)
      full = folded.reshape(shape)
    elif _rank_slabs(output, ctx):
      COMBINE_CALLS['reduce_scatter'] += 1
      (d, t), = output.local.items()
      comm.reduce_scatter_rows(t.data, full, opname)
      t.written = [d]
      return
    else:
      COMBINE_CALLS['all_reduce'] += 1
      comm.all_reduce(full, opname)
  for d, t in output.local.items():
    _copy_out(be, t, full, d)


def _rank_slabs(output, ctx):
  """True iff output tiles are world_size equal row slabs, tile k on rank k."""
  if len(output.shape) == 0 or len(output.tiles) != ctx.world_size:
    return False
  exs = sorted(output.tiles.items(), key=lambda kv: kv[0].ul)
  n = exs[0][0].shape[0]
  for k, (ex, w) in enumerate(exs):
    if ctx.owner(w) != k or ex.ul[0] != k * n or ex.lr[0] - ex.ul[0] != n:
      return False
    if any(ex.ul[d] != 0 or ex.lr[d] != output.shape[d] for d in range(1, len(output.shape))):
      return False
  return True


def _copy_out(be, tile, full, d):
  if d.ndim == 0:
    be.copy_region(tile.data, (), full, (), ())
  else:
    be.copy_region(tile.data, (0,) * d.ndim, full, d.ul, d.shape)
  tile.written = [d]


def _arg_merge_region(be, full_v, full_i, d, pv, pi, opname):
  import torch
  shape = d.shape if d.ndim else ()
  n = prod(shape)
  old_v = torch.empty(shape, dtype=full_v.dtype, device=full_v.device)
  old_i = torch.empty(shape, dtype=torch.int64, device=full_v.device)
  ul = d.ul if d.ndim else ()
  be.copy_region(old_v, (0,) * len(shape), full_v, ul, shape)
  be.copy_region(old_i, (0,) * len(shape), full_i, ul, shape)
  pvc = pv.reshape(shape).to(full_v.dtype) if pv.dtype != full_v.dtype else pv.reshape(shape)
  vs = torch.stack([old_v.reshape(n), pvc.reshape(n)])
  is_ = torch.stack([old_i.reshape(n), pi.reshape(n)])
  bv, bi = be.argcombine(opname, vs, is_)
  be.copy_region(full_v, ul, bv.reshape(shape), (0,) * len(shape), shape)
  be.copy_region(full_i, ul, bi.reshape(shape), (0,) * len(shape), shape)
