"""Small helpers (reference: spartan/util.py).

``divup`` restates spartan/util.py:396-400 with integer arithmetic;
``Assert`` keeps the semantics of spartan/util.py:214-256 that tests use.
"""
import logging
import math
import time

import numpy as np

log = logging.getLogger('spartan_amd')


def divup(a, b):
  if isinstance(a, tuple):
    return tuple(divup(x, b) for x in a)
  return -(-int(a) // int(b))


def is_iterable(x):
  """util.py:412-413: an explicit ``__iter__`` (a DistArray, which only has
  ``__getitem__`` / ``__len__``, is ONE operand, not a sequence of rows;
  Python-2 ``str`` had no ``__iter__`` either)."""
  return hasattr(x, '__iter__') and not isinstance(x, (str, bytes))


def prod(shape):
  p = 1
  for s in shape:
    p *= int(s)
  return p


class Timer:
  def __init__(self):
    self.t0 = time.perf_counter()

  def elapsed(self):
    return time.perf_counter() - self.t0


class Assert:
  @staticmethod
  def eq(a, b, msg=''):
    assert a == b, '%s == %s failed %s' % (a, b, msg)

  @staticmethod
  def ne(a, b, msg=''):
    assert a != b, '%s != %s failed %s' % (a, b, msg)

  @staticmethod
  def isinstance(a, t, msg=''):
    assert isinstance(a, t), '%s is not %s %s' % (type(a), t, msg)

  @staticmethod
  def all_eq(a, b, tolerance=0):
    """Exact (or absolute-tolerance) equality, spartan/util.py:228-249."""
    a = np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape, 'Mismatched shapes: %s %s' % (a.shape, b.shape)
    if tolerance == 0:
      assert np.all(a == b), 'Failed: \n%s\n ==\n%s' % (a, b)
    else:
      assert np.all(np.abs(a - b) < tolerance), 'Failed: \n%s\n ==\n%s' % (a, b)

  @staticmethod
  def all_close(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape, 'Mismatched shapes: %s %s' % (a.shape, b.shape)
    assert np.allclose(a, b), 'Failed: \n%s close to \n%s' % (a, b)
