"""Shared body of the device DQN agents (dqn/agent.py:40-229 glue).

`step()` follows the reference exactly (dqn/agent.py:133-158): preprocess;
repeat the previous action on a None timestep; otherwise act eps-greedily
and push the accumulator's transitions into the replay; learn every
`learn_period` frames once the replay holds `min_replay_capacity_fraction *
capacity` items; hard-copy the target network every
`target_network_update_period` frames, after learning.

The learner step itself is one libdqz call on device (learner.py); the
replay hands it device slot indices, never stacked frames.
"""

from typing import Any, Callable, Mapping
import warnings

import numpy as np
import torch

from dqn_mgsc_zoo_amd import learner as learner_lib
from dqn_mgsc_zoo_amd import networks as networks_lib
from dqn_mgsc_zoo_amd import optim_state
from dqn_mgsc_zoo_amd import parts


def seed_from_key(rng_key) -> int:
  """Integer seed from a JAX-style PRNGKey (uint32[2]) or an int."""
  a = np.asarray(rng_key)
  if a.ndim == 0:
    return int(a) & (2**63 - 1)
  v = 0
  for x in a.reshape(-1).tolist():
    v = (v * 1000003 + int(x)) & (2**63 - 1)
  return v


class DeviceDqnAgent(parts.Agent):
  """Common state, acting, target sync and (de)serialisation."""

  _ALGO = 'dqn'

  def __init__(self, preprocessor, sample_network_input,
               network: networks_lib.NetworkSpec, optimizer,
               transition_accumulator: Any, replay, batch_size: int,
               exploration_epsilon: Callable[[int], float],
               min_replay_capacity_fraction: float, learn_period: int,
               target_network_update_period: int, grad_error_bound: float,
               rng_key, device='cuda'):
    del sample_network_input  # shapes are fixed by the NatureQNetwork
    self._preprocessor = preprocessor
    self._replay = replay
    self._transition_accumulator = transition_accumulator
    self._batch_size = batch_size
    self._exploration_epsilon = exploration_epsilon
    self._min_replay_capacity = min_replay_capacity_fraction * replay.capacity
    self._learn_period = learn_period
    self._target_network_update_period = target_network_update_period
    seed = seed_from_key(rng_key)
    self._act_seed = seed
    self._act_count = 0
    self._network = network
    self._learner = learner_lib.Learner(network, batch_size, algo=self._ALGO,
                                        optimizer=optimizer,
                                        grad_error_bound=grad_error_bound,
                                        device=device)
    self._learner.set_params(network.init(seed))
    self._action = None
    self._frame_t = -1
    self._statistics = {'state_value': np.nan}
    self._learn_steps = 0
    self._last_health_check = 0  # learn steps done at the previous check
    self._nonfinite_loss_checks = 0

  # -- reference surface ----------------------------------------------------

  def step(self, timestep) -> parts.Action:
    self._frame_t += 1
    timestep = self._preprocessor(timestep)
    if timestep is None:
      if self._action is None:
        raise RuntimeError('Cannot repeat if action has never been selected.')
      action = self._action
    else:
      action = self._action = self._act(timestep)
      for transition in self._transition_accumulator.step(timestep, action):
        self._add(transition)
    if self._replay.size < self._min_replay_capacity:
      return action
    if self._frame_t % self._learn_period == 0:
      self._learn()
      self._after_learn()
    if self._frame_t % self._target_network_update_period == 0:
      self._learner.sync_target()
      self.check_learner_health()
    return action

  # Learn steps between reads of the learner's health word (each read
  # synchronises the device once; the acting path synchronises every frame
  # anyway).
  HEALTH_CHECK_PERIOD = 1000

  def _after_learn(self) -> None:
    self._learn_steps += 1
    if self._learn_steps % self.HEALTH_CHECK_PERIOD == 0:
      self.check_learner_health()

  def check_learner_health(self) -> int:
    """Reads the learner's health word (dqz_learner_sync_status).

    A hand-off wait that gave up (bit 0) makes every step since the previous
    check invalid: the online parameters and RMSProp moments may have been
    updated from partial payloads, so the learner state must be restored
    from a checkpoint (parts.Checkpoint); raises RuntimeError naming the
    learn steps since the previous check (reading the word has already reset
    the hand-off words, so a restored learner can continue).  A non-finite
    batch loss (bit 1) is counted and warned about; the update ran, as the
    reference's jitted update would.  Called every HEALTH_CHECK_PERIOD learn
    steps, at every target sync and from get_state.
    """
    status = self._health_word()
    first, last = self._last_health_check, self._learn_steps
    self._last_health_check = self._learn_steps
    if status & 2:
      self._nonfinite_loss_checks += 1
      warnings.warn('learner: a batch loss since the last check was NaN or '
                    'infinite (frame %d)' % self._frame_t, RuntimeWarning)
    if status & 1:
      raise RuntimeError(
          'learner hand-off wait timed out in learn steps %d..%d (frame %d): '
          'those updates are invalid; restore the agent from a checkpoint' % (
              first + 1, last, self._frame_t))
    return status

  def _health_word(self) -> int:
    """The device health word check_learner_health reads (agents with more
    device state, e.g. the MGSC meta-update, OR theirs in)."""
    return self._learner.sync_status()

  def reset(self) -> None:
    self._transition_accumulator.reset()
    parts.reset(self._preprocessor)
    self._action = None

  def _add(self, transition) -> None:
    self._replay.add(transition)

  def _act(self, timestep) -> parts.Action:
    """select_action + device_get (dqn/agent.py:169-177) as one device call:
    eps-greedy draw number `_act_count` of the Philox stream `_act_seed`
    (JAX's threefry keys are not reproducible here; the distribution is
    distrax.EpsilonGreedy's)."""
    a, v = self._learner.act(timestep.observation, self.exploration_epsilon,
                             self._act_seed, self._act_count)
    self._act_count += 1
    self._statistics['state_value'] = v
    return parts.Action(a)

  def _learn(self) -> None:
    raise NotImplementedError

  @property
  def learner(self) -> learner_lib.Learner:
    return self._learner

  @property
  def online_params(self):
    """Current online parameters as the reference returns them
    (dqn/agent.py:192-194): the Haiku tree {module: {'w', 'b'}}, each leaf a
    device view of the learner's live buffer (no copy).  The runners hand it
    to the eval actor (dqn/run_atari.py:264)."""
    return self._network.device_tree(self._learner.online)

  @property
  def online_params_flat(self):
    """The same parameters as one flat device tensor (dqz layout)."""
    return self._learner.online

  @property
  def statistics(self) -> Mapping[str, float]:
    return self._statistics

  @property
  def exploration_epsilon(self) -> float:
    return self._exploration_epsilon(self._frame_t)

  def get_state(self) -> Mapping[str, Any]:
    lrn = self._learner
    self.check_learner_health()
    return {
        'rng_key': optim_state.pack_key(self._act_seed, self._act_count),
        'frame_t': self._frame_t,
        'opt_state': optim_state.rmsprop_state(lrn.params_tree('mu'),
                                               lrn.params_tree('nu')),
        'online_params': lrn.params_tree('online'),
        'target_params': lrn.params_tree('target'),
        'replay': self._replay.get_state(),
    }

  def set_state(self, state: Mapping[str, Any]) -> None:
    self._act_seed, self._act_count = optim_state.unpack_key(state['rng_key'])
    self._frame_t = state['frame_t']
    self._learner.set_params(state['online_params'], state['target_params'])
    self._learner.set_opt_state(*optim_state.rmsprop_moments(state['opt_state']))
    self._replay.set_state(state['replay'])

  def _store(self):
    st = self._replay.frame_store
    if st is None:
      raise RuntimeError('the device learner needs frame transitions '
                         '(uint8 84x84x4 stacks) in its replay')
    return st


def to_device_f32(x, device):
  return torch.as_tensor(np.asarray(x, np.float32), device=device)
