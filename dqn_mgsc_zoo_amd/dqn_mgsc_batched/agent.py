"""MGSC DQN agent (drop-in for dqn_zoo/dqn_mgsc_batched/agent.py:42-403).

Step order follows the reference exactly (agent.py:237-280): act and
accumulate transitions; every `learn_period` frames, once the replay holds
max(meta_batch_size, min_replay_capacity) items, run one meta-update on the
newest accumulated transition (then clear the list); add the transitions to
replay; learn and sync the target as DQN does.

The meta-update (meta_loss_fn / meta_update, agent.py:104-220) is one libdqz
call (learner.MetaLearner); the learned logits live in the replay's device
logit buffer and are updated in place (update_priorities, agent.py:334).
"""

from typing import Any, Mapping

import numpy as np

from dqn_mgsc_zoo_amd import agent_base
from dqn_mgsc_zoo_amd import learner as learner_lib


class MGSCDqn(agent_base.DeviceDqnAgent):
  """Deep Q-Network agent with meta-learned replay logits."""

  _ALGO = 'dqn'
  _SECOND_ORDER = False  # theta'' = stop_gradient(...) (agent.py:191)

  def __init__(self, preprocessor, sample_network_input, network, optimizer,
               transition_accumulator, replay, batch_size: int,
               exploration_epsilon, min_replay_capacity_fraction: float,
               learn_period: int, target_network_update_period: int,
               grad_error_bound: float, rng_key, meta_optimizer=None,
               meta_batch_size: int = 100, device='cuda'):
    super().__init__(preprocessor, sample_network_input, network, optimizer,
                     transition_accumulator, replay, batch_size,
                     exploration_epsilon, min_replay_capacity_fraction,
                     learn_period, target_network_update_period,
                     grad_error_bound, rng_key, device=device)
    self._meta_batch_size = int(meta_batch_size)
    self._meta = learner_lib.MetaLearner(self._learner, self._meta_batch_size,
                                         meta_optimizer,
                                         second_order=self._SECOND_ORDER)
    self._last_transitions = []
    self._slots_cache = None
    self._upload = None  # pinned staging of the per-learn host draws

  def step(self, timestep):
    """agent.py:237-280."""
    self._frame_t += 1
    timestep = self._preprocessor(timestep)
    transitions = []
    if timestep is None:
      if self._action is None:
        raise RuntimeError('Cannot repeat if action has never been selected.')
      action = self._action
    else:
      action = self._action = self._act(timestep)
      transitions = list(self._transition_accumulator.step(timestep, action))
      self._last_transitions = self._last_transitions + transitions
    if (self._frame_t % self._learn_period == 0 and self._replay.size >= max(
        self._meta_batch_size, self._min_replay_capacity)):
      if self._last_transitions:
        self._meta_prioritization_learn(self._last_transitions[-1])
        self._last_transitions.clear()
      else:
        print('Skipping a META LEARNING train step because the '
              '_last_transitions buffer was empty on frame %d...' %
              self._frame_t)
    if timestep is not None:
      for transition in transitions:
        self._replay.add(transition)
    if self._replay.size < self._min_replay_capacity:
      return action
    if self._frame_t % self._learn_period == 0:
      self._learn()
      self._after_learn()
    if self._frame_t % self._target_network_update_period == 0:
      self._learner.sync_target()
      self.check_learner_health()
    return action

  def reset(self) -> None:
    super().reset()
    self._last_transitions = []

  def _meta_prioritization_learn(self, online_transition) -> None:
    """agent.py:302-334: meta batch, meta_update, update_priorities."""
    import torch  # pylint: disable=g-import-not-at-top
    _, slots, positions = self._replay.meta_batch_slots(self._meta_batch_size)
    pos = self._uploader()(torch.empty((len(positions),), dtype=torch.int32,
                                       device=self._learner.device),
                           np.asarray(positions, np.int32))
    self._meta.set_online_transition(online_transition)
    dl = self._replay.device_logits  # running log-sum-exp kept current
    self._meta.update(self._store(), slots, dl.logits, pos, logit_buffer=dl)

  def _learn(self) -> None:
    """agent.py:341-360: softmax(logits)-sampled batch, DQN update — one
    call: the replay Generator's uniforms are resolved into slots inside the
    learner's forward launch (Learner.step_logits)."""
    import torch  # pylint: disable=g-import-not-at-top
    if getattr(self._replay, 'exact_sampling', False):
      # the reference's own probabilities (dqz_logits_sample_exact), then the step
      self._learner.step(self._store(), self._replay.sample_slots(self._batch_size))
      return
    u = self._replay.draw_uniforms(self._batch_size)
    dev = self._learner.device
    if self._slots_cache is None:
      self._slots_cache = (torch.zeros((self._batch_size,), dtype=torch.int32, device=dev),
                           torch.zeros((self._batch_size,), dtype=torch.float64, device=dev))
    slots, u_dev = self._slots_cache
    self._uploader()(u_dev, np.asarray(u, np.float64))
    self._learner.step_logits(self._store(), self._replay.device_logits, slots,
                              uniforms=u_dev)

  def _uploader(self):
    """Host -> device copies without a host wait (store.Uploader): the meta
    batch's positions and the learn step's uniforms would otherwise block
    until the meta-update queued before them had finished."""
    if self._upload is None:
      from dqn_mgsc_zoo_amd import store as store_lib  # pylint: disable=g-import-not-at-top
      self._upload = store_lib.Uploader(8 * max(self._meta_batch_size, self._batch_size))
    return self._upload

  def _health_word(self) -> int:
    # the learner's word and the meta-update's (its two learners' hand-offs,
    # the HVP's ddot1 wait and the fused Adam's entry wait)
    return super()._health_word() | self._meta.sync_status()

  @property
  def meta_learner(self) -> learner_lib.MetaLearner:
    return self._meta

  def get_state(self) -> Mapping[str, Any]:
    state = dict(super().get_state())
    state['meta_opt_state'] = self._meta.get_state()
    return state

  def set_state(self, state: Mapping[str, Any]) -> None:
    super().set_state(state)
    self._meta.set_state(state['meta_opt_state'])
