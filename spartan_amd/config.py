"""Global flags (reference: spartan/config.py:27-140).

The reference parses argv / an ini file / ``SPARTAN_OPTS`` into a global
``FLAGS`` registry.  Only the flags the tile-execution path reads are kept;
they can be set as attributes, through ``FLAGS.parse(argv)`` or through the
``SPARTAN_OPTS`` environment variable (``--name=value`` tokens).

MI355X meaning of the worker flags: a "worker" is a tile owner.  Workers are
dealt round-robin to ranks (one process per GPU); ``num_workers`` defaults to
the world size, so one worker == one GPU unless set higher (several workers
may then share a GPU, which is how the multi-tile paths are exercised on a
single device).
"""
import os
import shlex


class _Flag:
  def __init__(self, name, default, typ, help=''):
    self.name, self.default, self.typ, self.help = name, default, typ, help

  def parse(self, s):
    if self.typ is bool:
      return str(s).lower() in ('1', 'true', 'yes', 'on')
    if self.default is None and self.typ is int:
      return None if str(s).lower() in ('', 'none') else int(s)
    return self.typ(s)


class Flags:
  def __init__(self):
    object.__setattr__(self, '_flags', {})
    object.__setattr__(self, '_vals', {})
    object.__setattr__(self, 'version', 0)  # bumped on every change (plan-cache keys read it)

  def add(self, name, default, typ=None, help=''):
    typ = typ or type(default)
    self._flags[name] = _Flag(name, default, typ, help)
    self._vals.setdefault(name, default)
    object.__setattr__(self, 'version', self.version + 1)

  def __getattr__(self, name):
    vals = object.__getattribute__(self, '_vals')
    if name in vals:
      return vals[name]
    raise AttributeError('unknown flag %s' % name)

  def __setattr__(self, name, value):
    if name not in self._flags:
      raise AttributeError('unknown flag %s' % name)
    self._vals[name] = value
    object.__setattr__(self, 'version', self.version + 1)

  def reset(self):
    for k, f in self._flags.items():
      self._vals[k] = f.default
    object.__setattr__(self, 'version', self.version + 1)

  def parse(self, argv):
    """Consume ``--name=value`` / ``--name value`` tokens for known flags.

    Returns the remaining (unrecognised) arguments."""
    rest = []
    i = 0
    while i < len(argv):
      tok = argv[i]
      if tok.startswith('--'):
        body = tok[2:]
        if '=' in body:
          k, v = body.split('=', 1)
        else:
          k, v = body, None
        if k in self._flags:
          if v is None:
            if self._flags[k].typ is bool:
              v = 'true'
            else:
              i += 1
              v = argv[i]
          self._vals[k] = self._flags[k].parse(v)
          object.__setattr__(self, 'version', self.version + 1)
          i += 1
          continue
      rest.append(tok)
      i += 1
    return rest

  def items(self):
    return dict(self._vals)


FLAGS = Flags()
FLAGS.add('num_workers', None, int, 'tile owners; default = torch.distributed world size')
FLAGS.add('tile_assignment_strategy', 'round_robin', str, 'only round_robin is supported')
FLAGS.add('optimization', True, bool)
FLAGS.add('opt_collapse_cached', True, bool)
FLAGS.add('opt_map_fusion', True, bool)
FLAGS.add('opt_reduce_fusion', True, bool)
FLAGS.add('opt_dot_fusion', True, bool, 'fold dot(x, w_host) into a fused axis-0 reduction over x')
FLAGS.add('opt_auto_tiling', True, bool, 'row / column partitioning chosen by the min-cost tiling solver')
FLAGS.add('opt_outer_argmin_fusion', True, bool,
          'argmin(outer(X, C, registered distance mapper), axis=1) -> one fused assignment kernel')
FLAGS.add('opt_expression_cache', True, bool)
FLAGS.add('opt_plan_cache', True, bool, 'replay the optimised DAG of a structure seen before (expr/plan_cache.py)')
FLAGS.add('dot_overlap', True, bool, 'multi-rank dot: reduce each output row slab while the next one computes')
FLAGS.add('rng_seed', 0x5EED, int, 'base seed of the counter-based rand()')
FLAGS.add('kernel_cache_dir', '', str, 'override the JIT code-object cache directory')
FLAGS.add('log_level', 'WARNING', str)


def parse_env():
  opts = os.environ.get('SPARTAN_OPTS', '')
  if opts:
    FLAGS.parse(shlex.split(opts))


parse_env()
