"""Agent protocol and run loop of `dqn_zoo/parts.py`, unchanged in behaviour.

Kept so the device agents are drop-ins for the reference's runners:
`Agent` ABC (parts.py:43-68), `run_loop` (:71-123), `generate_statistics`
and trackers (:126-340), `EpsilonGreedyActor` (:343-412), `LinearSchedule`
(:415-431), `NullWriter`/`CsvWriter` (:434-494), `NullCheckpoint` /
`Checkpoint` (:497-561).  dm_env is not installed here, so a minimal
`StepType` / `TimeStep` with the same fields and methods is provided; any
dm_env.TimeStep works as well.
"""

import abc
import collections
import csv
import enum
import os
import pickle
import timeit
import typing
from typing import Any, Iterable, Mapping, Optional, Sequence, Tuple

import numpy as np

Action = int


class StepType(enum.IntEnum):
  FIRST = 0
  MID = 1
  LAST = 2


class TimeStep(typing.NamedTuple):
  step_type: Any
  reward: Any
  discount: Any
  observation: Any

  def first(self) -> bool:
    return self.step_type == StepType.FIRST

  def mid(self) -> bool:
    return self.step_type == StepType.MID

  def last(self) -> bool:
    return self.step_type == StepType.LAST


class Agent(abc.ABC):
  """Agent interface."""

  @abc.abstractmethod
  def step(self, timestep) -> Action:
    """Selects action given timestep and potentially learns."""

  @abc.abstractmethod
  def reset(self) -> None:
    """Resets the agent's episodic state (start of every episode)."""

  @abc.abstractmethod
  def get_state(self) -> Mapping[str, Any]:
    """Retrieves agent state as a dictionary (e.g. for serialization)."""

  @abc.abstractmethod
  def set_state(self, state: Mapping[str, Any]) -> None:
    """Sets agent state from a (potentially de-serialized) dictionary."""

  @property
  @abc.abstractmethod
  def statistics(self) -> Mapping[str, float]:
    """Returns current agent statistics as a dictionary."""


def _with_last(timestep):
  if hasattr(timestep, '_replace'):
    return timestep._replace(step_type=type(timestep.step_type)(2)
                             if isinstance(timestep.step_type, enum.Enum)
                             else StepType.LAST)
  raise TypeError('timestep must be a namedtuple')


def run_loop(agent: Agent, environment, max_steps_per_episode: int = 0,
             yield_before_reset: bool = False) -> Iterable[Tuple[Any, Optional[Any], Agent, Optional[Action]]]:
  """Alternates environment and agent steps; yields (env, timestep, agent, a).

  After the last timestep of an episode the agent takes one extra step whose
  action is ignored; an episode reaching `max_steps_per_episode` is
  truncated by relabelling its timestep LAST.
  """
  while True:
    if yield_before_reset:
      yield environment, None, agent, None
    t = 0
    agent.reset()
    timestep_t = environment.reset()
    while True:
      a_t = agent.step(timestep_t)
      yield environment, timestep_t, agent, a_t
      t += 1
      timestep_t = environment.step(a_t)
      if max_steps_per_episode > 0 and t >= max_steps_per_episode:
        assert t == max_steps_per_episode
        timestep_t = _with_last(timestep_t)
      if timestep_t.last():
        agent.step(timestep_t)  # extra step, action ignored
        yield environment, timestep_t, agent, None
        break


def generate_statistics(trackers: Sequence[Any], timestep_action_sequence) -> Mapping[str, Any]:
  for tracker in trackers:
    tracker.reset()
  for environment, timestep_t, agent, a_t in timestep_action_sequence:
    for tracker in trackers:
      tracker.step(environment, timestep_t, agent, a_t)
  return dict(collections.ChainMap(*(t.get() for t in trackers)))


class EpisodeTracker:
  """Episode returns; the reward of a FIRST timestep is ignored."""

  def __init__(self):
    self._num_steps_since_reset = None
    self._num_steps_over_episodes = None
    self._episode_returns = None
    self._current_episode_rewards = None
    self._current_episode_step = None

  def step(self, environment, timestep_t, agent, a_t) -> None:
    del environment, agent, a_t
    if self._episode_returns is None:
      raise RuntimeError('reset() must be called before first call to step().')
    if timestep_t.first():
      if self._current_episode_rewards:
        raise ValueError('Current episode reward list should be empty.')
      if self._current_episode_step != 0:
        raise ValueError('Current episode step should be zero.')
    else:
      self._current_episode_rewards.append(timestep_t.reward)
    self._num_steps_since_reset += 1
    self._current_episode_step += 1
    if timestep_t.last():
      self._episode_returns.append(sum(self._current_episode_rewards))
      self._current_episode_rewards = []
      self._num_steps_over_episodes += self._current_episode_step
      self._current_episode_step = 0

  def reset(self) -> None:
    self._num_steps_since_reset = 0
    self._num_steps_over_episodes = 0
    self._episode_returns = []
    self._current_episode_step = 0
    self._current_episode_rewards = []

  def get(self) -> Mapping[str, Any]:
    if self._episode_returns is None:
      raise RuntimeError('reset() must be called before first call to get().')
    if self._episode_returns:
      mean_return = np.array(self._episode_returns).mean()
      current = sum(self._current_episode_rewards)
      episode_return = mean_return
    else:
      mean_return = np.nan
      current = (sum(self._current_episode_rewards)
                 if self._num_steps_since_reset > 0 else np.nan)
      episode_return = current
    return {'mean_episode_return': mean_return,
            'current_episode_return': current,
            'episode_return': episode_return,
            'num_episodes': len(self._episode_returns),
            'num_steps_over_episodes': self._num_steps_over_episodes,
            'current_episode_step': self._current_episode_step,
            'num_steps_since_reset': self._num_steps_since_reset}


class StepRateTracker:
  """Steps per second since reset."""

  def __init__(self):
    self._num_steps_since_reset = None
    self._start = None

  def step(self, environment, timestep_t, agent, a_t) -> None:
    del environment, timestep_t, agent, a_t
    self._num_steps_since_reset += 1

  def reset(self) -> None:
    self._num_steps_since_reset = 0
    self._start = timeit.default_timer()

  def get(self) -> Mapping[str, float]:
    if self._start is None:
      raise RuntimeError('reset() must be called before first call to get().')
    duration = timeit.default_timer() - self._start
    rate = (self._num_steps_since_reset / duration
            if self._num_steps_since_reset > 0 else np.nan)
    return {'step_rate': rate, 'num_steps': self._num_steps_since_reset,
            'duration': duration}


class UnbiasedExponentialWeightedAverageAgentTracker:
  """Sutton & Barto's unbiased constant-step-size trick over agent stats."""

  def __init__(self, step_size: float, initial_agent: Agent):
    self._initial_statistics = dict(initial_agent.statistics)
    self._step_size = step_size
    self.trace = 0.0
    self._statistics = dict(self._initial_statistics)

  def step(self, environment, timestep_t, agent, a_t) -> None:
    del environment, timestep_t, a_t
    self.trace = (1 - self._step_size) * self.trace + self._step_size
    final = self._step_size / self.trace
    assert 0 <= final <= 1
    if final == 1:
      self._statistics = dict(agent.statistics)
    else:
      self._statistics = {k: (1 - final) * self._statistics[k] + final * v
                          for k, v in agent.statistics.items()}

  def reset(self) -> None:
    self.trace = 0.0
    self._statistics = dict(self._initial_statistics)

  def get(self) -> Mapping[str, float]:
    return self._statistics


def make_default_trackers(initial_agent: Agent):
  return [EpisodeTracker(), StepRateTracker(),
          UnbiasedExponentialWeightedAverageAgentTracker(1e-3, initial_agent)]


def epsilon_greedy_probs(q, epsilon):
  """distrax.EpsilonGreedy: (1-eps) spread over argmax ties + eps/A."""
  q = np.asarray(q, np.float64)
  greedy = (q == q.max()).astype(np.float64)
  greedy /= greedy.sum()
  return (1.0 - epsilon) * greedy + epsilon / q.shape[-1]


class EpsilonGreedyActor(Agent):
  """Acts eps-greedily with externally set network parameters on device."""

  def __init__(self, preprocessor, network, exploration_epsilon: float,
               rng_key, learner=None):
    from dqn_mgsc_zoo_amd import learner as learner_lib  # pylint: disable=g-import-not-at-top
    self._preprocessor = preprocessor
    key = np.asarray(rng_key).astype(np.uint64).reshape(-1).tolist()
    self._act_seed = 0
    for x in key:
      self._act_seed = (self._act_seed * 1000003 + int(x)) & (2**63 - 1)
    self._act_count = 0
    self._rng_key = rng_key
    self._action = None
    self._epsilon = exploration_epsilon
    self._learner = learner or learner_lib.Learner(
        network, 1, algo='dqn' if not network.shared_bias else 'double')
    self.network_params = None  # flat device tensor or a parameter tree

  def step(self, timestep) -> Action:
    timestep = self._preprocessor(timestep)
    if timestep is None:
      if self._action is None:
        raise RuntimeError('Cannot repeat if action has never been selected.')
      return self._action
    a, _ = self._learner.act(timestep.observation, self._epsilon,
                             self._act_seed, self._act_count,
                             params=self.network_params)
    self._act_count += 1
    self._action = Action(a)
    return self._action

  def reset(self) -> None:
    reset(self._preprocessor)
    self._action = None

  def get_state(self) -> Mapping[str, Any]:
    return {'rng_key': self._rng_key, 'network_params': self.network_params,
            'act_count': self._act_count}

  def set_state(self, state: Mapping[str, Any]) -> None:
    self._rng_key = state['rng_key']
    self.network_params = state['network_params']
    self._act_count = state.get('act_count', 0)

  @property
  def statistics(self) -> Mapping[str, float]:
    return {}


def reset(processor) -> None:
  """processors.reset: calls `reset()` on a processor if it has one."""
  if hasattr(processor, 'reset'):
    processor.reset()


def identity_preprocessor(timestep):
  return timestep


class LinearSchedule:
  """Linear transition from begin_value to end_value (exploration epsilon)."""

  def __init__(self, begin_value, end_value, begin_t, end_t=None, decay_steps=None):
    if (end_t is None) == (decay_steps is None):
      raise ValueError('Exactly one of end_t, decay_steps must be provided.')
    self._decay_steps = decay_steps if end_t is None else end_t - begin_t
    self._begin_t = begin_t
    self._begin_value = begin_value
    self._end_value = end_value

  def __call__(self, t):
    frac = min(max(t - self._begin_t, 0), self._decay_steps) / self._decay_steps
    return (1 - frac) * self._begin_value + frac * self._end_value


class NullWriter:

  def write(self, *args, **kwargs) -> None:
    pass

  def close(self) -> None:
    pass


class CsvWriter:
  """Appends OrderedDict rows to a CSV file with a fixed header."""

  def __init__(self, fname: str):
    dirname = os.path.dirname(fname)
    if dirname and not os.path.exists(dirname):
      os.makedirs(dirname)
    self._fname = fname
    self._header_written = False
    self._fieldnames = None

  def write(self, values) -> None:
    if self._fieldnames is None:
      self._fieldnames = list(values.keys())
    with open(self._fname, 'a') as f:
      writer = csv.DictWriter(f, fieldnames=self._fieldnames)
      if not self._header_written:
        writer.writeheader()
        self._header_written = True
      writer.writerow(values)

  def close(self) -> None:
    pass

  def get_state(self) -> Mapping[str, Any]:
    return {'header_written': self._header_written, 'fieldnames': self._fieldnames}

  def set_state(self, state: Mapping[str, Any]) -> None:
    self._header_written = state['header_written']
    self._fieldnames = state['fieldnames']


class AttributeDict(dict):

  def __getattr__(self, key):
    return self[key]

  def __setattr__(self, key, value):
    self[key] = value

  def __delattr__(self, key):
    del self[key]


class NullCheckpoint:

  def __init__(self):
    self.state = AttributeDict()

  def save(self) -> None:
    pass

  def can_be_restored(self) -> bool:
    return False

  def restore(self) -> None:
    pass


class Checkpoint:
  """Pickles {iteration, agents' get_state(), random_state, writer} next to
  the results CSV (parts.py:517-561).  Device tensors in agent states are
  converted to numpy by the agents' get_state()."""

  def __init__(self):
    self.state = AttributeDict()

  @property
  def filepath(self) -> str:
    return os.path.splitext(self.state.writer._fname)[0] + '.chkpt'  # pylint: disable=protected-access

  def save(self) -> None:
    payload = {'iteration': self.state.iteration,
               'train_agent': self.state.train_agent.get_state(),
               'eval_agent': self.state.eval_agent.get_state(),
               'random_state': self.state.random_state,
               'writer': self.state.writer.get_state()}
    try:
      with open(self.filepath, 'wb') as f:
        pickle.dump(payload, f)
    except Exception:
      if os.path.exists(self.filepath):
        os.remove(self.filepath)
      raise

  def can_be_restored(self) -> bool:
    return os.path.isfile(self.filepath)

  def restore(self) -> None:
    with open(self.filepath, 'rb') as f:  # our own file format
      payload = pickle.load(f)
    self.state.iteration = payload['iteration']
    self.state.train_agent.set_state(payload['train_agent'])
    self.state.eval_agent.set_state(payload['eval_agent'])
    self.state.random_state = payload['random_state']
    self.state.writer.set_state(payload['writer'])
    self.state.writer._header_written = True  # pylint: disable=protected-access
