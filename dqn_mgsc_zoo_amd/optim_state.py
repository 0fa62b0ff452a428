"""Agent-state containers in the reference's optax / JAX shapes.

The reference checkpoints `get_state()` verbatim (dqn/agent.py:209-227,
dqn_mgsc_batched/agent.py:381-400), so its values are optax 0.1.2 states
(requirements_cc.txt:11) and a JAX key:

* `optax.rmsprop(centered=True)` (dqn/run_atari.py:208-213) is
  chain(scale_by_stddev, scale(-lr)): state
  `(ScaleByRStdDevState(mu, nu), EmptyState())`, mu / nu Haiku trees;
* `optax.adam` (dqn_mgsc_batched/run_atari.py:241-243) is
  chain(scale_by_adam, scale(-lr)): `(ScaleByAdamState(count, mu, nu),
  EmptyState())`, over the [meta_batch] logit vector;
* the key is an array of uint32.  Here the acting stream is Philox-4x32, so
  the key is uint32[4] = (seed lo, seed hi, counter lo, counter hi): the
  64-bit key and the 64-bit draw counter, JAX's uint32[2] threefry key
  widened by the counter JAX folds into its splits.

A reference-shaped uint32[2] key (a JAX PRNGKey, `jax.random.PRNGKey(seed)`
= [seed >> 32, seed & 0xFFFFFFFF]) restores as that 64-bit seed with the draw
counter at 0: JAX's threefry stream itself is not reproducible here, so the
acting stream restarts at the head of the Philox stream of that seed (a
documented deviation).

Loaders also take the round-2 forms (a {'seed', 'count'} dict, a (mu, nu)
pair, a {'count', 'mu', 'nu'} dict) so older checkpoints still restore.
"""

from typing import Any, NamedTuple, Tuple

import numpy as np


class ScaleByRStdDevState(NamedTuple):
  """optax.ScaleByRStdDevState (centered RMSProp moments)."""
  mu: Any
  nu: Any


class ScaleByAdamState(NamedTuple):
  """optax.ScaleByAdamState."""
  count: Any
  mu: Any
  nu: Any


class EmptyState(NamedTuple):
  """optax.EmptyState (the scale(-lr) stage)."""


_M32 = 0xFFFFFFFF


def pack_key(seed: int, count: int) -> np.ndarray:
  """(64-bit seed, 64-bit counter) -> uint32[4] key array."""
  seed, count = int(seed), int(count)
  if not (0 <= seed < 2**64 and 0 <= count < 2**64):
    raise ValueError('seed and count must be in [0, 2**64)')
  return np.array([seed & _M32, seed >> 32, count & _M32, count >> 32],
                  dtype=np.uint32)


def unpack_key(key) -> Tuple[int, int]:
  """uint32[4] key array, a JAX-shaped uint32[2] key (seed, counter 0) or
  the round-2 {'seed', 'count'} dict -> (seed, count)."""
  if isinstance(key, dict):
    return int(key['seed']), int(key['count'])
  a = np.asarray(key)
  if a.dtype != np.uint32 or a.shape not in ((4,), (2,)):
    raise ValueError('expected a uint32[4] or uint32[2] key, got %s%s' %
                     (a.dtype, a.shape))
  v = [int(x) for x in a.tolist()]
  if a.shape == (2,):  # jax.random.PRNGKey layout: [hi, lo]
    return (v[0] << 32) | v[1], 0
  return v[0] | (v[1] << 32), v[2] | (v[3] << 32)


def rmsprop_state(mu, nu):
  return (ScaleByRStdDevState(mu=mu, nu=nu), EmptyState())


def rmsprop_moments(opt_state):
  """(mu, nu) from a rmsprop state tuple (or the round-2 (mu, nu) pair)."""
  first = opt_state[0]
  if isinstance(first, ScaleByRStdDevState) or (
      hasattr(first, 'mu') and hasattr(first, 'nu')):
    return first.mu, first.nu
  mu, nu = opt_state
  return mu, nu


def adam_state(count, mu, nu):
  return (ScaleByAdamState(count=np.int32(count), mu=mu, nu=nu), EmptyState())


def adam_moments(opt_state):
  """(count, mu, nu) from an adam state tuple (or the round-2 dict)."""
  if isinstance(opt_state, dict):
    return int(opt_state['count']), opt_state['mu'], opt_state['nu']
  first = opt_state[0]
  return int(first.count), first.mu, first.nu
