"""Prioritized DQN agent (drop-in for dqn_zoo/prioritized/agent.py:40-258).

Double-Q loss weighted by importance-sampling weights, new transitions get
the running max priority, learned priorities are |td| (agent.py:187-206).
"""

import numpy as np
import torch

from dqn_mgsc_zoo_amd import agent_base


class PrioritizedDqn(agent_base.DeviceDqnAgent):
  """Prioritized Double DQN agent."""

  _ALGO = 'per'

  def __init__(self, *args, **kwargs):
    super().__init__(*args, **kwargs)
    self._max_seen_priority = 1.0
    self._w = torch.zeros((self._batch_size,), dtype=torch.float32,
                          device=self._learner.device)

  def _add(self, transition) -> None:
    self._replay.add(transition, priority=self._max_seen_priority)

  def _learn(self) -> None:
    ids, slots, weights = self._replay.sample_slots(self._batch_size)
    self._w.copy_(torch.from_numpy(np.asarray(weights, np.float32)))
    self._learner.step(self._store(), slots, self._w)
    _, td, _ = self._learner.fetch_outputs()
    priorities = np.abs(td.cpu().numpy().astype(np.float64))
    self._max_seen_priority = max(self._max_seen_priority, float(priorities.max()))
    self._replay.update_priorities(ids, priorities)

  @property
  def importance_sampling_exponent(self) -> float:
    return self._replay.importance_sampling_exponent

  @property
  def max_seen_priority(self) -> float:
    return self._max_seen_priority

  def get_state(self):
    state = dict(super().get_state())
    state['max_seen_priority'] = self._max_seen_priority
    return state

  def set_state(self, state) -> None:
    super().set_state(state)
    self._max_seen_priority = state['max_seen_priority']
