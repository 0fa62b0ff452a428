"""DQN with reservoir replay: the dqn agent over ReservoirTransitionReplay
(dqn_zoo/dqn_reservoir/agent.py is byte-identical to dqn/agent.py)."""
from dqn_mgsc_zoo_amd.dqn.agent import Dqn  # noqa: F401
