"""CPU: the agent protocol surface (parts.py) — run_loop interleaving,
schedules, trackers, eps-greedy probabilities."""

import numpy as np
import pytest

from dqn_mgsc_zoo_amd import parts


class TapeAgent(parts.Agent):

  def __init__(self, tape):
    self._tape = tape

  def reset(self):
    self._tape.append('Agent reset')

  def step(self, timestep):
    del timestep
    self._tape.append('Agent step')
    return 0

  def get_state(self):
    return {}

  def set_state(self, state):
    del state

  @property
  def statistics(self):
    return {}


class TapeEnv:

  def __init__(self, tape, episode_length):
    self._tape = tape
    self._len = episode_length

  def reset(self):
    self._t = 0
    self._tape.append('Environment reset')
    return parts.TimeStep(parts.StepType.FIRST, 0.0, 0.0, 1.0)

  def step(self, action):
    self._tape.append('Environment step (%s)' % action)
    self._t += 1
    if self._t == self._len:
      kind = parts.StepType.LAST
      self._t = -1
    else:
      kind = parts.StepType.MID
    return parts.TimeStep(kind, 2.0, 0.0 if kind == parts.StepType.LAST else 1.0, 1.0)


def _run(episode_length, n, max_steps=0, yield_before_reset=False):
  tape = []
  agent, env = TapeAgent(tape), TapeEnv(tape, episode_length)
  loop = parts.run_loop(agent, env, max_steps, yield_before_reset)
  for _ in range(n):
    next(loop)
  return tape


def test_run_loop_interleaving():
  tape = _run(episode_length=2, n=5)
  assert tape == [
      'Agent reset', 'Environment reset', 'Agent step',
      'Environment step (0)', 'Agent step',
      'Environment step (0)', 'Agent step',  # LAST: extra agent step
      'Agent reset', 'Environment reset', 'Agent step',
      'Environment step (0)', 'Agent step']


def test_run_loop_truncation():
  tape = _run(episode_length=10, n=4, max_steps=2)
  assert tape.count('Agent reset') == 2
  assert tape[:7] == ['Agent reset', 'Environment reset', 'Agent step',
                      'Environment step (0)', 'Agent step',
                      'Environment step (0)', 'Agent step']


def test_run_loop_yield_before_reset():
  tape = []
  loop = parts.run_loop(TapeAgent(tape), TapeEnv(tape, 3), 0, True)
  env, ts, agent, a = next(loop)
  assert ts is None and a is None and tape == []


def test_linear_schedule():
  s = parts.LinearSchedule(begin_value=1.0, end_value=0.1, begin_t=10,
                           decay_steps=90)
  assert s(0) == 1.0 and s(10) == 1.0 and s(100) == pytest.approx(0.1)
  assert s(55) == pytest.approx(0.55)
  with pytest.raises(ValueError, match='Exactly one of end_t, decay_steps'):
    parts.LinearSchedule(1.0, 0.0, 0)


def test_epsilon_greedy_probs_ties():
  p = parts.epsilon_greedy_probs([1.0, 3.0, 3.0, 0.0], 0.2)
  np.testing.assert_allclose(p, [0.05, 0.45, 0.45, 0.05])
  assert p.sum() == pytest.approx(1.0)
