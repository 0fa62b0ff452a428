"""Agent protocol and run loop of `dqn_zoo/parts.py`, unchanged in behaviour.

Kept so the device agents are drop-ins for the reference's runners:
`Agent` ABC (parts.py:43-68), `run_loop` (:71-123), `EpsilonGreedyActor`
(:343-412), `LinearSchedule` (:415-431) and a `Checkpoint` with the role of
:497-561.  The statistics trackers and CSV writers (:126-340, :434-494) are
outside the learner hot path and are not provided.  dm_env is not installed here, so a minimal
`StepType` / `TimeStep` with the same fields and methods is provided; any
dm_env.TimeStep works as well.
"""

import abc
import enum
import os
import pickle
import types
import typing
from typing import Any, Iterable, Mapping, Optional, Tuple

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


class Checkpoint:
  """Resume point of a training run (the role of parts.py:517-561).

  `state` is a namespace the runner fills (`iteration`, `train_agent`,
  `eval_agent`, `random_state`, optionally `writer`).  `save()` writes one
  pickle of the agents' `get_state()` dictionaries (device tensors come back
  as host numpy arrays) next to `path`; the file is written under a
  temporary name and renamed, so an interrupted save never leaves a
  truncated checkpoint behind.  `restore()` loads it and pushes every piece
  back through `set_state()`.  Only files this class wrote are read.
  """

  def __init__(self, path: Optional[str] = None):
    self.state = types.SimpleNamespace()
    self._path = path

  @property
  def filepath(self) -> str:
    if self._path is not None:
      return self._path
    writer = getattr(self.state, 'writer', None)
    fname = getattr(writer, 'fname', None) or getattr(writer, '_fname', None)
    if fname is None:
      raise ValueError('Checkpoint needs a path or a state.writer with a file name')
    return os.path.splitext(fname)[0] + '.chkpt'

  def _payload(self) -> Mapping[str, Any]:
    out = {}
    for key in ('iteration', 'random_state'):
      if hasattr(self.state, key):
        out[key] = getattr(self.state, key)
    for key in ('train_agent', 'eval_agent', 'writer'):
      obj = getattr(self.state, key, None)
      if obj is not None and hasattr(obj, 'get_state'):
        out[key] = obj.get_state()
    return out

  def save(self) -> None:
    path = self.filepath
    folder = os.path.dirname(path)
    if folder:
      os.makedirs(folder, exist_ok=True)
    tmp = path + '.tmp'
    with open(tmp, 'wb') as f:
      pickle.dump(self._payload(), f, protocol=pickle.HIGHEST_PROTOCOL)
    os.replace(tmp, path)

  def can_be_restored(self) -> bool:
    return os.path.isfile(self.filepath)

  def restore(self) -> None:
    with open(self.filepath, 'rb') as f:  # written by save() above
      payload = pickle.load(f)
    for key in ('iteration', 'random_state'):
      if key in payload:
        setattr(self.state, key, payload[key])
    for key in ('train_agent', 'eval_agent', 'writer'):
      obj = getattr(self.state, key, None)
      if key in payload and obj is not None and hasattr(obj, 'set_state'):
        obj.set_state(payload[key])


class NullCheckpoint(Checkpoint):
  """Checkpointing disabled: nothing is written or restored."""

  def save(self) -> None:
    pass

  def can_be_restored(self) -> bool:
    return False

  def restore(self) -> None:
    pass
