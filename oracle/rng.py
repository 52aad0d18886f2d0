"""Counter-based input generator shared (bit for bit) with the HIP fill kernel.

value(g) for global flat index g: splitmix64 finaliser of
  seed * 0xD1B54A32D192ED03 + (g + 1) * 0x9E3779B97F4A7C15   (mod 2^64)
float32: (z >> 40) * 2^-24, then low + (high - low) * u in float32 steps;
float64: (z >> 11) * 2^-53, then low + (high - low) * u in float64.
Mirrors rng_at / fill_value in spartan_amd/csrc/spx.hip.
"""
import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def mix64(z):
  z = z.astype(np.uint64)
  with np.errstate(over='ignore'):
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
  return z ^ (z >> np.uint64(31))


def raw(g, seed):
  g = np.asarray(g, dtype=np.uint64)
  with np.errstate(over='ignore'):
    x = np.uint64(seed) * np.uint64(0xD1B54A32D192ED03) + (g + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
  return mix64(x)


def uniform_values(g, seed, low, high, dtype):
  dtype = np.dtype(dtype)
  z = raw(g, seed)
  if dtype == np.float32:
    u = (z >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24)
    return np.float32(low) + np.float32(high - low) * u
  if dtype == np.float64:
    u = (z >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)
    return np.float64(low) + (high - low) * u
  u = (z >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)
  return np.floor(low + (high - low) * u).astype(dtype)


def normal_values(g, seed, loc, scale, dtype):
  """loc + scale * N(0,1): Box-Muller over streams 2g (u1 in (0,1]) and
  2g+1, in fp64 (libm log/cos: within a few ulp of the device's, not bit-exact)."""
  g = np.asarray(g, dtype=np.uint64)
  u1 = ((raw(np.uint64(2) * g, seed) >> np.uint64(11)) + np.uint64(1)).astype(np.float64) * (2.0 ** -53)
  u2 = (raw(np.uint64(2) * g + np.uint64(1), seed) >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)
  z = np.sqrt(-2.0 * np.log(u1)) * np.cos(6.283185307179586 * u2)
  v = loc + scale * z
  dtype = np.dtype(dtype)
  return v.astype(dtype) if dtype.kind == 'f' else np.floor(v).astype(dtype)


def randn(shape, seed, dtype=np.float64):
  n = int(np.prod(shape))
  return normal_values(np.arange(n, dtype=np.uint64), seed, 0.0, 1.0, dtype).reshape(shape)


def arange_values(g, start, step, dtype):
  dtype = np.dtype(dtype)
  g = np.asarray(g, dtype=np.int64)
  if dtype.kind == 'f':
    return (float(start) + float(step) * g.astype(np.float64)).astype(dtype)
  return (int(start) + int(step) * g).astype(dtype)


def rand(shape, seed, dtype=np.float64, low=0.0, high=1.0):
  n = int(np.prod(shape))
  return uniform_values(np.arange(n, dtype=np.uint64), seed, low, high, dtype).reshape(shape)
