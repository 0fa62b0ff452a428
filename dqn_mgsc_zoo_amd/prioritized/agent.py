"""Prioritized DQN agent (drop-in for dqn_zoo/prioritized/agent.py:40-258).

Double-Q loss weighted by importance-sampling weights, new transitions get
the running max priority, learned priorities are |td| (agent.py:187-206).

With frame transitions the replay's sum tree lives in HBM and a learn is
two device calls with no host synchronisation: `sample_device` (the
replay's RandomState draws, resolved on device: tree indices, slots, IS
weights) and the learner step with the write-back (|td| ->
max_seen_priority -> p ** alpha into the tree) folded into its backward
launch (dqz_learner_step_per).  `max_seen_priority` is then a device scalar,
read back only when asked for.  Host-stored items keep the reference's host
path.
"""

import numpy as np
import torch

from dqn_mgsc_zoo_amd import agent_base


class PrioritizedDqn(agent_base.DeviceDqnAgent):
  """Prioritized Double DQN agent."""

  _ALGO = 'per'

  def __init__(self, *args, **kwargs):
    super().__init__(*args, **kwargs)
    dev = self._learner.device
    self._max_seen_priority = 1.0
    self._max_seen_dev = torch.ones((1,), dtype=torch.float64, device=dev)
    self._w = torch.zeros((self._batch_size,), dtype=torch.float32, device=dev)
    self._sample_out = (
        torch.zeros((self._batch_size,), dtype=torch.int32, device=dev),
        torch.zeros((self._batch_size,), dtype=torch.int32, device=dev),
        self._w)

  def _add(self, transition) -> None:
    if self._replay.stores_on_device(transition):
      self._replay.add(transition, priority=self._max_seen_dev)
    else:
      self._replay.add(transition, priority=self._max_seen_priority)

  def _learn(self) -> None:
    if self._replay.on_device:
      indices, slots, weights = self._replay.sample_device(
          self._batch_size, out=self._sample_out)
      wb = self._replay.write_back_args(indices, self._max_seen_dev)
      self._learner.step(self._store(), slots, weights, write_back=wb)
      if wb is None:
        self._replay.write_back(self._learner, indices, self._max_seen_dev)
      return
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
    if self._replay.on_device:
      return float(self._max_seen_dev.item())
    return self._max_seen_priority

  def get_state(self):
    state = dict(super().get_state())
    state['max_seen_priority'] = self.max_seen_priority
    return state

  def set_state(self, state) -> None:
    super().set_state(state)
    self._max_seen_priority = float(state['max_seen_priority'])
    self._max_seen_dev.fill_(self._max_seen_priority)
