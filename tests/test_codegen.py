"""Generated kernels: every lowered ufunc / dtype / skeleton compiles for
gfx950 (device-only clang, runs on CPU), and lowering follows NumPy's dtype
resolution."""
import numpy as np
import pytest

from spartan_amd import backend, codegen
from spartan_amd.codegen import Cast, Const, In, Op, Sc

F32, F64, I32, I64, B = (np.dtype(t) for t in (np.float32, np.float64, np.int32, np.int64, np.bool_))

UNARY_F = ['exp', 'log', 'sqrt', 'sin', 'cos', 'tanh', 'absolute', 'negative', 'square', 'floor', 'log1p']
BINARY = ['add', 'subtract', 'multiply', 'true_divide', 'maximum', 'minimum', 'power', 'floor_divide',
          'remainder', 'less', 'greater_equal', 'equal', 'logical_and']


def _compile(src):
  backend.compile_code_object(src)


def test_dtype_resolution_matches_numpy():
  assert Op('add', [In(0, F32), Sc(0, 2.0)]).dtype == F32
  assert Op('add', [In(0, I32), Sc(0, 2.0)]).dtype == F64
  assert Op('true_divide', [In(0, I64), In(1, I64)]).dtype == F64
  assert Op('less', [In(0, F32), In(1, F64)]).dtype == B
  assert Op('exp', [In(0, I32)]).dtype == F64
  assert Op('maximum', [In(0, B), In(1, B)]).dtype == B


@pytest.mark.parametrize('dt', [F32, F64])
def test_unary_float_compile(dt):
  root = In(0, dt)
  for name in UNARY_F:
    root = Op(name, [root]) if name not in ('log', 'sqrt', 'log1p') else Op(name, [Op('absolute', [root])])
  _compile(codegen.gen_map(root, [(0, dt)], ['c'], 1, codegen.vec_width([dt]), True))


@pytest.mark.parametrize('dt', [F32, F64, I32, I64])
def test_binary_compile_all_skeletons(dt):
  for name in BINARY:
    root = Op(name, [In(0, dt), In(1, dt)])
    if root.dtype == B:
      root = Cast(root, I64)
    ins = [(0, dt), (1, dt)]
    V = codegen.vec_width([dt, root.dtype])
    _compile(codegen.gen_map(root, ins, ['c', 'b'], 2, V, False))
    for op in ('sum', 'max', 'argmin'):
      _compile(codegen.gen_reduce(root, ins, ['c', 'g'], 'rows', op, codegen.vec_width([dt, codegen.acc_dtype(op, root.dtype)])))
      _compile(codegen.gen_reduce(root, ins, ['c', 'b'], 'cols', op, codegen.vec_width([dt, codegen.acc_dtype(op, root.dtype)])))


def test_scalars_consts_and_bools_compile():
  root = Op('logical_or', [Op('greater', [In(0, F32), Sc(0, 0.5)]), Op('isnan', [In(1, F64)])])
  root = Op('add', [Cast(root, I32), Const(1, I32)])
  _compile(codegen.gen_map(root, [(0, F32), (1, F64)], ['c', 'c'], 1, 2, True))
  _compile(codegen.gen_reduce(Op('not_equal', [In(0, B), Const(0, B)]), [(0, B)], ['c'], 'rows', 'sum', 2))


def test_generated_source_is_deterministic():
  root = Op('add', [Op('multiply', [In(0, F32), In(1, F32)]), Op('exp', [In(2, F32)])])
  ins = [(0, F32), (1, F32), (2, F32)]
  a = codegen.gen_reduce(root, ins, ['c'] * 3, 'cols', 'sum', 4)
  b = codegen.gen_reduce(root, ins, ['c'] * 3, 'cols', 'sum', 4)
  assert a == b and backend.source_key(a) == backend.source_key(b)


@pytest.mark.parametrize('dt', [F32, F64])
def test_rowdot_cols_compile(dt):
  """DotReduceFusion's row-dot leaf in the column-reduce skeleton (vector and
  scalar paths), and its refusal in the other skeletons."""
  from spartan_amd.codegen import RowDot
  x, yv, w = In(0, dt), In(1, dt), In(2, dt)
  root = Op('multiply', [x, Op('subtract', [RowDot(x, w), yv])])
  ins = [(0, dt), (1, dt), (2, dt)]
  for V in (codegen.vec_width([dt]), 1):
    src = codegen.gen_reduce(root, ins, ['c', 'b', 'c'], 'cols', 'sum', V)
    assert 'row_allsum(rd0' in src
    _compile(src)
  with pytest.raises(NotImplementedError):
    codegen.gen_reduce(root, ins, ['c', 'b', 'c'], 'rows', 'sum', 1)
  with pytest.raises(NotImplementedError):
    codegen.gen_map(root, ins, ['c', 'b', 'c'], 2, 1, False)


@pytest.mark.parametrize('dt', [F32, F64])
def test_rowdot_cols_fixed_lane_groups(dt):
  """The cfg5 form of the row-dot kernel: lanes per row group compiled in
  (LPR 16: the row sum is straight-line DPP, no run-time branches), no column
  mask on the vector path, and the per-row input (y) loaded once per unrolled
  step and handed to the step's rows by DPP row_newbcast (one load instead of
  U), in both the vector and the scalar path.  Compiles for both dtypes."""
  from spartan_amd.codegen import RowDot
  x, yv, w = In(0, dt), In(1, dt), In(2, dt)
  root = Op('multiply', [x, Op('subtract', [RowDot(x, w), yv])])
  ins = [(0, dt), (1, dt), (2, dt)]
  V = codegen.vec_width([dt])
  src = codegen.gen_reduce(root, ins, ['c', 'b', 'c'], 'cols', 'sum', V, 8, (2,), lpr=16, full=True)
  assert 'constexpr i64 lpr_log = 4, LPR = 16, RPW = 4;' in src
  assert 'const bool colok = true;' in src
  assert src.count('dpp_mov<%d>(yb1)' % 0x150) == 2 and 'dpp_mov<%d>(yb1)' % (0x150 + 7) in src
  _compile(src)
  # without a fixed width: the run-time form (aux[2]) and no broadcasts
  src = codegen.gen_reduce(root, ins, ['c', 'b', 'c'], 'cols', 'sum', V, 8, (2,))
  assert 'lpr_log = a.aux[2]' in src and 'yb1' not in src


@pytest.mark.parametrize("rdt", [B, np.dtype(np.int8), np.dtype(np.int16)])
def test_rowdot_narrow_row_input_compiles(rdt):
  """A per-row input narrower than 4 bytes (a bool row mask, int8, int16) in
  the fixed-width row-dot kernel keeps its per-row load: dpp_mov moves whole
  dwords, so only 4- and 8-byte row inputs are DPP-broadcast."""
  from spartan_amd.codegen import RowDot
  x, yv, w, m = In(0, F32), In(1, F32), In(2, F32), In(3, rdt)
  root = Op('multiply', [Op('multiply', [x, Op('subtract', [RowDot(x, w), yv])]), Cast(m, F32)])
  ins = [(0, F32), (1, F32), (2, F32), (3, rdt)]
  V = codegen.vec_width([F32])
  src = codegen.gen_reduce(root, ins, ['c', 'b', 'c', 'b'], 'cols', 'sum', V, 8, (2,), lpr=16, full=True)
  assert 'yb1' in src and 'yb3' not in src
  _compile(src)


def test_rowdot_interleaved_rows_compile():
  """The cfg5 kernel's interleaved row order (round 5): block p walks the
  U-step super-chunks p, p + P, ... (one loop around the unrolled and the
  tail loops), for both dtypes; the contiguous form has no such loop."""
  from spartan_amd.codegen import RowDot
  for dt in (F32, F64):
    x, yv, w = In(0, dt), In(1, dt), In(2, dt)
    root = Op('multiply', [x, Op('subtract', [RowDot(x, w), yv])])
    ins = [(0, dt), (1, dt), (2, dt)]
    V = codegen.vec_width([dt])
    src = codegen.gen_reduce(root, ins, ['c', 'b', 'c'], 'cols', 'sum', V, 8, (2,), lpr=16, full=True,
                             interleave=True)
    assert src.count('for (i64 sb = p * (8 * STEP); sb < R; sb += P * (8 * STEP))') == 2
    # round 6: the chunk sums fold into fp64 middle / total accumulators, the
    # LDS combine and the partials are fp64; fp64 inputs Kahan the total
    assert 'double mid0 = 0.0, top0 = 0.0' in src
    assert 'SHARED double sv[' in src and '((GLOBAL double*)a.out0)' in src
    assert ('topc0' in src) == (dt == F64)
    assert codegen.partial_dtype('sum', dt, True) == F64
    assert codegen.partial_dtype('sum', dt, False) == dt
    _compile(src)
    assert 'for (i64 sb' not in codegen.gen_reduce(root, ins, ['c', 'b', 'c'], 'cols', 'sum', V, 8, (2,),
                                                   lpr=16, full=True)


@pytest.mark.parametrize('unroll', [1, 2, 4])
def test_dense_map_unroll_compiles(unroll):
  """backend.MAP_UNROLL: U vectors per lane (all loads first) for the dense
  vector path; U = 1 has no unrolled loop at all (the full-grid default)."""
  root = Op('add', [Op('multiply', [In(0, F32), In(1, F32)]), Op('exp', [In(2, F32)])])
  ins = [(0, F32), (1, F32), (2, F32)]
  src = codegen.gen_map(root, ins, ['c'] * 3, 1, 4, True, True, unroll)
  assert ('e + %d * step < n' % (unroll - 1) in src) == (unroll > 1)
  _compile(src)
