"""GPU: checkpoint save -> restore into fresh agents, and reservoir storage.

* `parts.Checkpoint` (the role of dqn_zoo/parts.py:517-561): a training agent
  runs, its state goes to a pickle file through `Checkpoint.save()`, a fresh
  agent built with a different seed is restored from that file, and both are
  driven with the same timesteps for 60 more frames.  Actions, online /
  target parameters, RMSProp moments and — for the MGSC agents — the device
  logits and the Adam meta-optimizer state must stay bit-identical.  Covers
  dqn, prioritized, MGSC-FIFO and MGSC-reservoir (second-order meta-grad).
* dqn_reservoir (replay.py:246-296, Algorithm R): after many replacements,
  every slot of the device frame store holds exactly the transition last
  written to it (frames are never aliased across slots).
"""

import numpy as np
import pytest
import torch

from tests import fake_env

pytestmark = pytest.mark.gpu

LR, DECAY, EPS, BOUND = 2.5e-4, 0.95, 0.01 / 32**2, 1.0 / 32


def _agent(kind, seed, capacity=160):
  from dqn_mgsc_zoo_amd import learner as learner_lib
  from dqn_mgsc_zoo_amd import networks
  from dqn_mgsc_zoo_amd import parts
  from dqn_mgsc_zoo_amd import replay as replay_lib
  from dqn_mgsc_zoo_amd import replay_circular as rc
  structure = replay_lib.Transition(None, None, None, None, None)
  extra = {}
  net = networks.dqn_atari_network(6)
  if kind == 'per':
    from dqn_mgsc_zoo_amd.prioritized import agent as agent_lib
    replay = replay_lib.PrioritizedTransitionReplay(
        capacity, structure, priority_exponent=0.6,
        importance_sampling_exponent=lambda t: 0.4,
        uniform_sample_probability=1e-3, normalize_weights=True,
        random_state=np.random.RandomState(seed))
    cls, net = agent_lib.PrioritizedDqn, networks.double_dqn_atari_network(6)
  elif kind == 'dqn':
    from dqn_mgsc_zoo_amd.dqn import agent as agent_lib
    replay = replay_lib.TransitionReplay(capacity, structure,
                                         np.random.RandomState(seed))
    cls = agent_lib.Dqn
  elif kind == 'reservoir':
    from dqn_mgsc_zoo_amd import dqn_reservoir
    replay = replay_lib.ReservoirTransitionReplay(capacity, structure,
                                                  np.random.RandomState(seed))
    cls = dqn_reservoir.Dqn
  else:
    if kind == 'mgsc_fifo':
      from dqn_mgsc_zoo_amd.dqn_mgsc_batched import agent as agent_lib
      replay = rc.MGSCFiFoTransitionReplay(capacity, structure,
                                           np.random.default_rng(seed))
    else:
      from dqn_mgsc_zoo_amd.dqn_mgsc_batched_reservoir import agent as agent_lib
      replay = rc.MGSCReservoirTransitionReplay(capacity, structure,
                                                np.random.default_rng(seed))
    cls = agent_lib.MGSCDqn
    extra = dict(meta_optimizer=learner_lib.adam(2.5e-4), meta_batch_size=16)
  agent = cls(
      preprocessor=fake_env.FrameStacker(),
      sample_network_input=np.zeros((84, 84, 4), np.uint8),
      network=net,
      optimizer=learner_lib.rmsprop(LR, DECAY, EPS, centered=True),
      transition_accumulator=replay_lib.TransitionAccumulator(),
      replay=replay, batch_size=32,
      exploration_epsilon=parts.LinearSchedule(
          begin_t=40, decay_steps=200, begin_value=1.0, end_value=0.1),
      min_replay_capacity_fraction=0.25, learn_period=4,
      target_network_update_period=40, grad_error_bound=BOUND,
      rng_key=np.array([0, seed], np.uint32), **extra)
  return agent, replay


def _timesteps(n, seed, episode_len):
  env = fake_env.FakeAtari(episode_len=episode_len, seed=seed)
  steps = [env.reset()]
  for t in range(n - 1):
    steps.append(env.step(t % 6) if not steps[-1].last() else env.reset())
  return steps


def _drive(agent, steps):
  actions = []
  for ts in steps:
    if ts.first():
      agent.reset()
    actions.append(agent.step(ts))
  return actions


def _replay_rng(replay):
  return getattr(replay, '_random_state', None)


@pytest.mark.parametrize('kind', ['dqn', 'per', 'mgsc_fifo', 'mgsc_reservoir'])
def test_checkpoint_save_restore_continues_bit_exactly(device, tmp_path, kind):
  from dqn_mgsc_zoo_amd import parts
  a1, r1 = _agent(kind, seed=4)
  _drive(a1, _timesteps(100, 5, 19))
  # the reference's state shapes (dqn/agent.py:209-217): a uint32 key array,
  # optax's (ScaleByRStdDevState(mu, nu), EmptyState()) over Haiku trees
  st = a1.get_state()
  assert st['rng_key'].dtype == np.uint32 and st['rng_key'].shape == (4,)
  rms, empty = st['opt_state']
  assert type(rms).__name__ == 'ScaleByRStdDevState' and empty._fields == ()
  assert set(rms.mu) == set(st['online_params']) == set(rms.nu)
  if kind.startswith('mgsc'):
    adam = st['meta_opt_state'][0]
    assert type(adam).__name__ == 'ScaleByAdamState' and adam.count > 0
  ck = parts.Checkpoint(str(tmp_path / 'run.chkpt'))
  ck.state.iteration = 3
  ck.state.train_agent = a1
  ck.state.random_state = _replay_rng(r1)
  ck.save()

  a2, r2 = _agent(kind, seed=99)
  ck2 = parts.Checkpoint(str(tmp_path / 'run.chkpt'))
  ck2.state.train_agent = a2
  ck2.state.random_state = None
  assert ck2.can_be_restored()
  ck2.restore()
  assert ck2.state.iteration == 3
  rs = ck2.state.random_state
  if isinstance(rs, np.random.RandomState):
    # the runner's RandomState is the replay's (dqn/run_atari.py:103,204)
    r2._random_state.set_state(rs.get_state())  # pylint: disable=protected-access
  # the restored agent is a different object graph: nothing is shared
  assert a2.learner.online.data_ptr() != a1.learner.online.data_ptr()

  more = _timesteps(60, 6, 17)
  assert _drive(a1, more) == _drive(a2, more)
  for which in ('online', 'target', 'mu', 'nu'):
    assert torch.equal(getattr(a1.learner, which), getattr(a2.learner, which)), which
  if kind.startswith('mgsc'):
    assert torch.equal(r1.logits, r2.logits)
    m1, m2 = a1.meta_learner.get_state()[0], a2.meta_learner.get_state()[0]
    assert m1.count == m2.count and m1.count > 0
    np.testing.assert_array_equal(m1.mu, m2.mu)
    np.testing.assert_array_equal(m1.nu, m2.nu)
  if kind == 'per':
    assert a1.max_seen_priority == a2.max_seen_priority


def test_reservoir_store_holds_last_write_per_slot(device):
  """dqn_reservoir run loop: 400 frames into 48 slots (many Algorithm-R
  replacements); every slot's device transition equals the item last
  written to it."""
  from dqn_mgsc_zoo_amd import replay as replay_lib
  agent, replay = _agent('reservoir', seed=8, capacity=48)
  last = {}
  orig_make = replay._make_backend  # pylint: disable=protected-access

  def make(use_device):
    backend = orig_make(use_device)
    put = backend.put

    def spy(slot, item, oldest_live_slot=None):
      last[int(slot)] = replay_lib.Transition(
          np.array(item.s_tm1), int(item.a_tm1), float(item.r_t),
          float(item.discount_t), np.array(item.s_t))
      return put(slot, item, oldest_live_slot)

    backend.put = spy
    return backend

  replay._make_backend = make  # pylint: disable=protected-access
  _drive(agent, _timesteps(400, 9, 29))
  assert replay.size == replay.capacity
  assert replay._t > 2 * replay.capacity  # pylint: disable=protected-access
  assert sorted(last) == list(range(replay.capacity))
  got = list(replay.get(range(replay.capacity)))
  for slot, g in enumerate(got):
    want = last[slot]
    np.testing.assert_array_equal(g.s_tm1, want.s_tm1, err_msg=str(slot))
    np.testing.assert_array_equal(g.s_t, want.s_t, err_msg=str(slot))
    assert int(g.a_tm1) == want.a_tm1
    assert float(g.r_t) == np.float32(want.r_t)
    assert float(g.discount_t) == np.float32(want.discount_t)
  assert torch.isfinite(agent.learner.online).all()


@pytest.mark.parametrize('kind', ['dqn', 'per', 'mgsc_fifo', 'mgsc_reservoir'])
def test_checkpoint_does_not_perturb_the_saver(device, tmp_path, kind):
  """Saving is observation-free: two agents with the same seed
  run the same 100 frames; one of them is checkpointed through
  parts.Checkpoint; over the next 60 frames both act, learn and (MGSC)
  sample / meta-update identically, bit for bit — the learned-logit
  buffer's running log-sum-exp is read out, not invalidated, by get_state
  (replay_circular.CircularLogitBuffer.get_state)."""
  from dqn_mgsc_zoo_amd import parts
  a1, r1 = _agent(kind, seed=4)
  a2, r2 = _agent(kind, seed=4)
  first = _timesteps(100, 5, 19)
  assert _drive(a1, first) == _drive(a2, first)
  ck = parts.Checkpoint(str(tmp_path / 'saver.chkpt'))
  ck.state.train_agent = a1
  ck.save()
  more = _timesteps(60, 6, 17)
  assert _drive(a1, more) == _drive(a2, more)
  for which in ('online', 'target', 'mu', 'nu'):
    assert torch.equal(getattr(a1.learner, which), getattr(a2.learner, which)), which
  if kind.startswith('mgsc'):
    d1, d2 = r1.device_logits, r2.device_logits
    assert torch.equal(d1.logits, d2.logits)
    assert d1.run_state() == d2.run_state()
    assert d1.run_state()['known'] == 1  # nothing forced a re-scan
    m1, m2 = a1.meta_learner.get_state()[0], a2.meta_learner.get_state()[0]
    np.testing.assert_array_equal(m1.mu, m2.mu)
  if kind == 'per':
    assert a1.max_seen_priority == a2.max_seen_priority
