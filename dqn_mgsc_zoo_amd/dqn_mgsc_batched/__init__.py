"""MGSC DQN agent (drop-in for dqn_zoo/dqn_mgsc_batched)."""
