"""DQN agent (drop-in for dqn_zoo/dqn)."""
