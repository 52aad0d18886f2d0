"""spartan_amd -- MI355X-native tile-execution backend for Spartan's lazy
array expressions.

Drop-in for the reference's ``spartan.expr`` path (ones / map / reduce / dot /
force and the fused Map/Reduce/Dot DAG): forced tiles live in HBM, one process
per GPU, fused maps and reductions run as generated gfx950 kernels, dot on
MFMA, cross-tile combines over RCCL.  See DESIGN.md.
"""
from . import config
from .config import FLAGS
from .runtime import initialize, shutdown
from . import expr
from .expr import *  # noqa: F401,F403

__all__ = ['initialize', 'shutdown', 'expr', 'FLAGS']
