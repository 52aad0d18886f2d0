"""spartan_amd.expr -- the spartan.expr API (spartan/expr/__init__.py:26-53)
on the MI355X tile-execution backend."""
from .base import (Expr, NotShapeable, as_array, eager, evaluate, force, glom, lazify, newaxis,
                   optimized_dag)
from .builtins import (abs, add, arange, argmax, argmin, astype, bincount, concatenate, count_nonzero,
                       count_zero, exp,
                       ln, log, maximum, max, mean, min, minimum, multiply, ones, power, rand, randn,
                       size, sqrt, square, std, sub, sum, zeros)
from .dot import dot
from .join import map2, outer
from .map import map
from .map_with_location import map_with_location, region_map
from .ndarray import ndarray
from .reduce import reduce
from .reshape import reshape
from .slice import slice_expr
from .transpose import transpose
from .write_array import from_file, from_numpy, write

Expr.outer = outer
Expr.sum = sum
Expr.mean = mean
Expr.astype = astype
Expr.argmin = argmin
Expr.argmax = argmax
