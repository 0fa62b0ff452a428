"""Double DQN agent (drop-in for dqn_zoo/double_q/agent.py).

rlax.double_q_learning (online network selects, target evaluates) on the
shared-bias head of double_dqn_atari_network.
"""

from dqn_mgsc_zoo_amd import agent_base


class DoubleDqn(agent_base.DeviceDqnAgent):
  """Double DQN (tuned) agent."""

  _ALGO = 'double'

  def _learn(self) -> None:
    _, slots = self._replay.sample_slots(self._batch_size)
    self._learner.step(self._store(), slots)
