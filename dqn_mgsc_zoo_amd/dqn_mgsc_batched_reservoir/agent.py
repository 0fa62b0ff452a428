"""MGSC DQN agent over the learned-logit reservoir replay
(drop-in for dqn_zoo/dqn_mgsc_batched_reservoir/agent.py).

The reference file differs from dqn_mgsc_batched/agent.py in two places
only: the replay type hint (MGSCReservoirTransitionReplay, :52) and the
missing `jax.lax.stop_gradient` on theta'' (:191 of the batched agent),
which makes its meta-gradient second order (d theta''/d theta' involves the
Hessian of the online-transition loss).  The device meta-update implements
the stop-gradient form; the second-order form is not on device yet, so this
agent refuses to run it silently: pass meta_gradient='stop_gradient' to opt
into the first-order meta-gradient explicitly.
"""

from dqn_mgsc_zoo_amd.dqn_mgsc_batched import agent as batched


class MGSCDqn(batched.MGSCDqn):
  """MGSC DQN over MGSCReservoirTransitionReplay."""

  def __init__(self, *args, meta_gradient='second_order', **kwargs):
    if meta_gradient != 'stop_gradient':
      raise NotImplementedError(
          'dqn_mgsc_batched_reservoir differentiates through theta\'\' '
          '(no stop_gradient, second-order meta-gradient); the device '
          "meta-update implements the stop_gradient form only. Pass "
          "meta_gradient='stop_gradient' to use it.")
    super().__init__(*args, **kwargs)
