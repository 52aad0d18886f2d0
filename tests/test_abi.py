"""The C-ABI library loads and exports every entry point include/spx.h declares
(no compute calls: those need a GPU)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, 'spartan_amd', 'libspx.so')


def declared():
  src = open(os.path.join(ROOT, 'include', 'spx.h')).read()
  return sorted(set(re.findall(r'\b(spx_[a-z_]+)\s*\(', src)))


def test_header_lists_the_boundary():
  names = declared()
  for n in ['spx_abi_version', 'spx_last_error', 'spx_module_load', 'spx_module_function', 'spx_launch',
            'spx_fill', 'spx_reduce_finalize', 'spx_merge', 'spx_copy_region', 'spx_gemm',
            'spx_argreduce_combine', 'spx_module_unload', 'spx_comm_load', 'spx_comm_unique_id',
            'spx_comm_init', 'spx_comm_destroy', 'spx_allreduce', 'spx_reduce_scatter', 'spx_allgather',
            'spx_broadcast', 'spx_reduce', 'spx_sendrecv']:
    assert n in names


@pytest.mark.skipif(not os.path.exists(LIB), reason='libspx.so not built')
def test_library_exports_every_declared_symbol():
  import torch  # noqa: F401  (torch's HIP runtime first)
  lib = ctypes.CDLL(LIB)
  for n in declared():
    assert hasattr(lib, n), n
  lib.spx_abi_version.restype = ctypes.c_int
  assert lib.spx_abi_version() == 3


@pytest.mark.skipif(not os.path.exists(LIB), reason='libspx.so not built')
def test_python_binding_signatures_cover_header():
  from spartan_amd import backend
  assert sorted(backend.EXPORTED) == declared()


@pytest.mark.skipif(not os.path.exists(LIB), reason='libspx.so not built')
def test_argument_validation_without_gpu():
  """Invalid arguments are rejected before any device work (error codes + message)."""
  import torch  # noqa: F401
  lib = ctypes.CDLL(LIB)
  lib.spx_last_error.restype = ctypes.c_char_p
  I64 = ctypes.c_int64 * 1
  rc = lib.spx_fill(ctypes.c_int(99), ctypes.c_int(0), None, ctypes.c_int(1), I64(4), I64(0), I64(4),
                    ctypes.c_double(0), ctypes.c_double(0), ctypes.c_uint64(0), None)
  assert rc == -1 and b'dtype' in lib.spx_last_error()
  rc = lib.spx_gemm(ctypes.c_int(0), ctypes.c_int64(4), ctypes.c_int64(4), ctypes.c_int64(4), None,
                    ctypes.c_int64(4), None, ctypes.c_int64(4), None, ctypes.c_int64(4),
                    ctypes.c_double(1), ctypes.c_double(0), None)
  assert rc == -3 and b'not supported' in lib.spx_last_error()
  rc = lib.spx_gemm(ctypes.c_int(3), ctypes.c_int64(4), ctypes.c_int64(4), ctypes.c_int64(8), None,
                    ctypes.c_int64(4), None, ctypes.c_int64(4), None, ctypes.c_int64(4),
                    ctypes.c_double(1), ctypes.c_double(0), None)
  assert rc == -1 and b'leading dimension' in lib.spx_last_error()


@pytest.mark.skipif(not os.path.exists(LIB), reason='libspx.so not built')
def test_collectives_boundary_without_gpu():
  """RCCL is opened at run time: before spx_comm_load every collective
  refuses; after it (PyTorch's own RCCL) a unique id can be made without a
  device; bad dtypes / ops are rejected before RCCL sees them."""
  import subprocess
  import sys
  code = r'''
import ctypes, sys
sys.path.insert(0, %r)
from spartan_amd import backend, comm
lib = backend.load_library()
assert lib.spx_allreduce(None, None, None, 4, 3, 0, None) == -1
assert b'spx_comm_load' in lib.spx_last_error()
uid = comm.rccl_unique_id()
assert len(uid) == 128 and any(uid)
assert lib.spx_allreduce(ctypes.c_void_p(1), None, None, 4, 9, 0, None) == -1
assert b'dtype' in lib.spx_last_error()
assert lib.spx_reduce_scatter(ctypes.c_void_p(1), None, None, 4, 3, 4, None) == -1
assert b'op' in lib.spx_last_error()
assert lib.spx_comm_init(uid, 128, 2, 2, ctypes.byref(ctypes.c_void_p())) == -1
assert lib.spx_comm_load(b'/nonexistent/librccl.so') == 0  # already loaded: a no-op
print('ok')
''' % ROOT
  r = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, timeout=120)
  assert r.returncode == 0 and r.stdout.strip().endswith('ok'), r.stderr[-2000:]
