"""Agent-state containers in the reference's optax / JAX shapes (CPU).

The reference checkpoints get_state() as is (dqn/agent.py:209-227): the
values are optax 0.1.2 states and a JAX uint32 key.  These tests pin the
container shapes, the key round trip and the round-2 forms the loaders
still accept.
"""

import pickle

import numpy as np
import pytest

from dqn_mgsc_zoo_amd import optim_state as os_


@pytest.mark.parametrize('seed,count', [(0, 0), (7, 1), (2**63 - 1, 2**40 + 3),
                                        (2**64 - 1, 2**64 - 1)])
def test_key_round_trip(seed, count):
  key = os_.pack_key(seed, count)
  assert key.dtype == np.uint32 and key.shape == (4,)
  assert os_.unpack_key(key) == (seed, count)


def test_key_rejects_out_of_range_and_wrong_shapes():
  with pytest.raises(ValueError):
    os_.pack_key(-1, 0)
  with pytest.raises(ValueError):
    os_.pack_key(0, 2**64)
  with pytest.raises(ValueError):
    os_.unpack_key(np.zeros(3, np.uint32))
  with pytest.raises(ValueError):
    os_.unpack_key(np.zeros(4, np.int64))


def test_jax_shaped_key_restores_as_seed_with_counter_zero():
  # jax.random.PRNGKey(seed) = uint32[2] [seed >> 32, seed & 0xFFFFFFFF]
  seed = (5 << 32) | 42
  assert os_.unpack_key(np.array([5, 42], np.uint32)) == (seed, 0)


def test_legacy_dict_key_still_restores():
  assert os_.unpack_key({'seed': 5, 'count': 9}) == (5, 9)


def test_rmsprop_state_is_optax_shaped_and_picklable():
  mu = {'conv1': {'w': np.ones(3), 'b': np.zeros(1)}}
  nu = {'conv1': {'w': np.full(3, 2.0), 'b': np.ones(1)}}
  st = os_.rmsprop_state(mu, nu)
  assert isinstance(st, tuple) and len(st) == 2
  assert type(st[0]).__name__ == 'ScaleByRStdDevState'
  assert st[0]._fields == ('mu', 'nu')
  assert st[1] == os_.EmptyState() and st[1]._fields == ()
  back = pickle.loads(pickle.dumps(st))
  got_mu, got_nu = os_.rmsprop_moments(back)
  np.testing.assert_array_equal(got_mu['conv1']['w'], mu['conv1']['w'])
  np.testing.assert_array_equal(got_nu['conv1']['b'], nu['conv1']['b'])
  # round 2's (mu, nu) pair
  assert os_.rmsprop_moments((mu, nu)) == (mu, nu)


def test_adam_state_is_optax_shaped():
  st = os_.adam_state(4, np.zeros(8, np.float32), np.ones(8, np.float32))
  assert type(st[0]).__name__ == 'ScaleByAdamState'
  assert st[0]._fields == ('count', 'mu', 'nu')
  assert st[0].count.dtype == np.int32
  count, mu, nu = os_.adam_moments(st)
  assert count == 4 and mu.shape == (8,) and nu[0] == 1.0
  # round 2's dict
  c2, m2, n2 = os_.adam_moments({'count': 3, 'mu': mu, 'nu': nu})
  assert c2 == 3 and m2 is mu and n2 is nu
