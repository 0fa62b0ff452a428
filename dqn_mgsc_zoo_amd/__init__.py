"""dqn_mgsc_zoo_amd — MI355X-native DQN learner step (drop-in for the hot
path of Stalfoes/dqn_mgsc_zoo: replay sample -> NatureQNetwork fwd/bwd ->
q_learning / double_q_learning TD loss -> RMSProp / Adam)."""

__version__ = '0.1.0'
