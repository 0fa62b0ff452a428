"""MGSC DQN agent over MGSCReservoirTransitionReplay
(drop-in for dqn_zoo/dqn_mgsc_batched_reservoir)."""
