"""Prioritized DQN agent (drop-in for dqn_zoo/prioritized)."""
