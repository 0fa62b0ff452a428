"""Prioritized DQN agent (drop-in for dqn_zoo/prioritized/agent.py:40-258).

Double-Q loss weighted by importance-sampling weights, new transitions get
the running max priority, learned priorities are |td| (agent.py:187-206).

With frame transitions the replay's sum tree lives in HBM and a learn is
one device call with no host synchronisation (dqz_learner_step_per_draw):
the replay's RandomState draws are resolved into tree indices and slots by
the learner's conv1 workgroups, the head forms the IS weights, and the
write-back (|td| -> max_seen_priority -> p ** alpha into the tree) runs
inside the backward launch.  `max_seen_priority` is then a device scalar,
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
    self._draw_out = (
        torch.zeros((self._batch_size,), dtype=torch.int32, device=dev),
        torch.zeros((self._batch_size,), dtype=torch.int32, device=dev),
        torch.zeros((self._batch_size,), dtype=torch.float64, device=dev),
        self._w)

  def _add(self, transition) -> None:
    if self._replay.stores_on_device(transition):
      self._replay.add(transition, priority=self._max_seen_dev)
    else:
      self._replay.add(transition, priority=self._max_seen_priority)

  def _learn(self) -> None:
    if self._replay.on_device:
      pd = self._replay.per_draw(self._batch_size, self._max_seen_dev,
                                 out=self._draw_out)
      if pd is not None:  # draw, weights, step and write-back: one call
        self._learner.step_per_draw(self._store(), pd[0])
        return
      indices, slots, weights = self._replay.sample_device(
          self._batch_size, out=self._sample_out)
      self._learner.step(self._store(), slots, weights)
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
