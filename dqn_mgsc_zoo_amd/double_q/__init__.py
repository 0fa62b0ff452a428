"""Double DQN agent (drop-in for dqn_zoo/double_q)."""
