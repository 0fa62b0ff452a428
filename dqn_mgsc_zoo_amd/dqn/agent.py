"""DQN agent class (drop-in for dqn_zoo/dqn/agent.py:40-229).

rlax.q_learning loss with clip_gradient, centered RMSProp; the jitted
`update` (agent.py:109-119) is one libdqz learner step on device.
"""

from dqn_mgsc_zoo_amd import agent_base


class Dqn(agent_base.DeviceDqnAgent):
  """Deep Q-Network agent."""

  _ALGO = 'dqn'

  def _learn(self) -> None:
    """Samples a batch of transitions from replay and learns from it."""
    _, slots = self._replay.sample_slots(self._batch_size)
    self._learner.step(self._store(), slots)
