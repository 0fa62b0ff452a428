"""Atari timestep preprocessing (drop-in for dqn_zoo/processors.py).

The control flow is the reference's (processors.py:48-365, 390-508): action
repeats through a None-padded buffer that is passed on at FIRST, LAST and
every `num_action_repeats` steps; rewards summed then clipped; discounts
multiplied then scaled; zero discount on life loss; a 4-frame stack with
trailing zero padding.  The observation math of each emitted step — max
over the last `num_pooled_frames` RGB frames, rgb2y, PIL BILINEAR resize —
is one device launch (`dqz_atari_frame`, csrc/preprocess.hpp), bit-exact
with numpy + PIL (tests/test_preprocess*.py).
"""

import collections
import ctypes
from typing import Any, Callable, Iterable, List, Optional, Sequence

import numpy as np
import torch

from dqn_mgsc_zoo_amd import _native
from dqn_mgsc_zoo_amd import parts

StepType = parts.StepType
Processor = Callable
identity = lambda v: v  # noqa: E731


def reset(processor) -> None:
  """processors.reset: calls `reset()` when the processor has one."""
  if hasattr(processor, 'reset'):
    processor.reset()


def trailing_zero_pad(length: int):
  """Pads a list of arrays with zero arrays at the end up to `length`."""

  def pad(arrays):
    missing = length - len(arrays)
    if missing <= 0:
      return arrays
    return arrays + [np.zeros_like(arrays[0])] * missing

  return pad


def none_to_zero_pad(values):
  """Replaces None entries of a list of named tuples by all-zero tuples."""
  present = [v for v in values if v is not None]
  if not present:
    raise ValueError('Must have at least one value which is not None.')
  if len(present) == len(values):
    return values
  proto = present[0]
  zero = type(proto)(*(np.zeros_like(f) for f in proto))
  return [zero if v is None else v for v in values]


def named_tuple_sequence_stack(values):
  """[T(a1, b1), T(a2, b2)] -> T((a1, a2), (b1, b2))."""
  return type(values[0])(*zip(*values))


class Deque:
  """Bounded deque returned whole after every append."""

  def __init__(self, max_length: int, initial_values: Optional[Iterable[Any]] = None):
    self._items = collections.deque(maxlen=max_length)
    self._initial = list(initial_values or [])

  def reset(self) -> None:
    self._items.clear()
    self._items.extend(self._initial)

  def __call__(self, value):
    self._items.append(value)
    return self._items


class FixedPaddedBuffer:
  """A `length`-slot buffer of None-padded values, restarted once full.

  The first value lands at `initial_index`; after the last slot the next
  value starts a fresh all-None buffer (the action-repeat window)."""

  def __init__(self, length: int, initial_index: int):
    self._length = length
    self._start = initial_index % length
    self.reset()

  def reset(self) -> None:
    self._pos = self._start
    self._slots = [None] * self._length

  def __call__(self, value):
    if self._pos == self._length:
      self._pos = 0
      self._slots = [None] * self._length
    self._slots[self._pos] = value
    self._pos += 1
    return self._slots


class ConditionallySubsample:
  """Passes the value on when `condition(value)`, else returns None."""

  def __init__(self, condition):
    self._condition = condition

  def reset(self) -> None:
    reset(self._condition)

  def __call__(self, value):
    return value if self._condition(value) else None


class TimestepBufferCondition:
  """True for buffers holding a FIRST or a LAST, and every `period` steps."""

  def __init__(self, period: int):
    self._period = period
    self.reset()

  def reset(self) -> None:
    self._since_first = None
    self._needs_reset = False

  def __call__(self, timesteps) -> bool:
    if self._needs_reset:
      raise RuntimeError('Should have reset.')
    kind = StepType.MID
    for ts in timesteps:
      if ts is None or ts.step_type not in (StepType.FIRST, StepType.LAST):
        continue
      if kind != StepType.MID:
        raise RuntimeError('Expected at most one FIRST or LAST.')
      kind = ts.step_type
    if self._since_first is None and kind != StepType.FIRST:
      raise RuntimeError('After reset first timestep should be FIRST.')
    if kind == StepType.FIRST:
      self._since_first = 0
      return True
    if kind == StepType.LAST:
      self._since_first = None
      self._needs_reset = True
      return True
    self._since_first += 1
    return self._since_first % self._period == 0


class ApplyToNamedTupleField:
  """Runs `processors` in order on one field of a named tuple."""

  def __init__(self, field: str, *processors):
    self._field = field
    self._processors = processors

  def reset(self) -> None:
    for p in self._processors:
      reset(p)

  def __call__(self, value):
    x = getattr(value, self._field)
    for p in self._processors:
      x = p(x)
    return value._replace(**{self._field: x})


class Maybe:
  """None in, None out; otherwise the wrapped processor."""

  def __init__(self, processor):
    self._processor = processor

  def reset(self) -> None:
    reset(self._processor)

  def __call__(self, value):
    return None if value is None else self._processor(value)


class Sequential:
  """Chains processors."""

  def __init__(self, *processors):
    self._processors = processors

  def reset(self) -> None:
    for p in self._processors:
      reset(p)

  def __call__(self, value):
    for p in self._processors:
      value = p(value)
    return value


class ZeroDiscountOnLifeLoss:
  """Discount 0 on a MID timestep whose lives count (observation[1]) fell."""

  def __init__(self):
    self._prev_lives = None

  def reset(self) -> None:
    self._prev_lives = None

  def __call__(self, timestep):
    lives = timestep.observation[1]
    lost = timestep.mid() and lives < self._prev_lives
    self._prev_lives = lives
    return timestep._replace(discount=0.0) if lost else timestep


def reduce_step_type(step_types: Sequence[StepType], debug: bool = False) -> StepType:
  """FIRST if the (zero-padded) buffer holds a padded FIRST, LAST if it
  holds a LAST, else MID."""
  for i, st in enumerate(step_types):
    if st == 0:  # zero padding reads as FIRST: expected 000F
      if debug and not (np.array(step_types) == 0).all():
        raise ValueError('Expected zero padding followed by FIRST.')
      return StepType.FIRST
    if st == StepType.LAST:
      if debug and not (np.array(step_types)[i + 1:] == 0).all():
        raise ValueError('Expected LAST to be followed by zero padding.')
      return StepType.LAST
    if st != StepType.MID:
      raise ValueError('Expected MID if not FIRST or LAST.')
  return StepType.MID


def aggregate_rewards(rewards: Sequence[Optional[float]], debug: bool = False):
  """Sum of the buffered rewards (None at FIRST)."""
  if None in rewards:
    if debug:
      r = np.array(rewards)
      if not (r[-1] is None and (r[:-1] == 0).all()):
        raise ValueError('Should only have a None reward for FIRST.')
    return None
  total = 0
  for r in rewards:
    total = total + r
  return total


def aggregate_discounts(discounts: Sequence[Optional[float]], debug: bool = False):
  """Product of the buffered discounts (each 0 or 1; None at FIRST)."""
  if debug:
    d = np.array(discounts)
    if not np.isin(d, [0.0, 1.0, None]).all():
      raise ValueError('All discounts should be 0 or 1, got: %s.' % d)
  if None in discounts:
    if debug:
      d = np.array(discounts)
      if not (d[-1] is None and (d[:-1] == 0).all()):
        raise ValueError('Should only have a None discount for FIRST.')
    return None
  prod = 1
  for d in discounts:
    prod = prod * d
  return prod


def select_rgb_observation(timestep):
  """(rgb, lives) observation -> rgb."""
  return timestep._replace(observation=timestep.observation[0])


def apply_additional_discount(additional_discount: float):
  return lambda d: None if d is None else additional_discount * d


def clip_reward(bound: float):
  return lambda r: None if r is None else max(min(r, bound), -bound)


class DeviceAtariFrame:
  """max-pool + rgb2y + BILINEAR resize of the last pooled RGB frames, on
  device (dqz_atari_frame): returns the uint8 [out_h, out_w] frame.

  The RGB frames are staged in pinned host memory that the kernel reads in
  place, and the output lands in pinned memory: one launch and one stream
  synchronisation per emitted step."""

  def __init__(self, num_pooled_frames: int, resize_shape=(84, 84)):
    self._n = num_pooled_frames
    self._out_shape = tuple(resize_shape)
    self._plan = None
    self._in_shape = None

  def _prepare(self, shape):
    lib = _native.lib()
    if self._plan is not None:
      _native.check(lib.dqz_frame_plan_destroy(self._plan))
    h, w = int(shape[0]), int(shape[1])
    plan = ctypes.c_void_p()
    _native.check(lib.dqz_frame_plan_create(h, w, self._out_shape[0],
                                            self._out_shape[1],
                                            ctypes.byref(plan)))
    self._plan = plan
    self._in_shape = (h, w)
    self._stage = torch.empty((self._n, h, w, 3), dtype=torch.uint8, pin_memory=True)
    self._stage_np = self._stage.numpy()
    self._out = torch.empty(self._out_shape, dtype=torch.uint8, pin_memory=True)
    self._out_np = self._out.numpy()

  def __call__(self, observations):
    frames = list(observations)[-self._n:]
    if self._in_shape != frames[0].shape[:2]:
      self._prepare(frames[0].shape)
    for i, f in enumerate(frames):
      self._stage_np[i] = f
    _native.check(_native.lib().dqz_atari_frame(
        self._plan, ctypes.c_void_p(self._stage.data_ptr()), len(frames),
        ctypes.c_void_p(self._out.data_ptr()), _native.stream_handle()))
    torch.cuda.current_stream().synchronize()
    return self._out_np.copy()

  def __del__(self):
    if getattr(self, '_plan', None) is not None and _native is not None:
      try:
        _native.lib().dqz_frame_plan_destroy(self._plan)
      except Exception:  # pylint: disable=broad-except
        pass


def atari(additional_discount: float = 0.99,
          max_abs_reward: Optional[float] = 1.0,
          resize_shape=(84, 84),
          num_action_repeats: int = 4,
          num_pooled_frames: int = 2,
          zero_discount_on_life_loss: bool = True,
          num_stacked_frames: int = 4,
          grayscaling: bool = True,
          observation_frame: Optional[Callable] = None):
  """Standard DQN Atari preprocessing (processors.py:421-508).

  `observation_frame` maps the buffered RGB observations of an emitted step
  to its 2-D frame; by default the device kernel (DeviceAtariFrame).  Only
  grayscale + resize (the reference's defaults and every runner's setting)
  are on the device path."""
  if not grayscaling or resize_shape is None:
    raise ValueError('the device observation path takes grayscaling=True and a resize_shape')
  frame_fn = observation_frame or DeviceAtariFrame(num_pooled_frames, resize_shape)
  return Sequential(
      ZeroDiscountOnLifeLoss() if zero_discount_on_life_loss else identity,
      select_rgb_observation,
      FixedPaddedBuffer(length=num_action_repeats, initial_index=-1),
      ConditionallySubsample(TimestepBufferCondition(num_action_repeats)),
      Maybe(Sequential(
          none_to_zero_pad,
          named_tuple_sequence_stack,
          ApplyToNamedTupleField('step_type', reduce_step_type),
          ApplyToNamedTupleField(
              'reward', aggregate_rewards,
              clip_reward(max_abs_reward) if max_abs_reward else identity),
          ApplyToNamedTupleField(
              'discount', aggregate_discounts,
              apply_additional_discount(additional_discount)),
          ApplyToNamedTupleField(
              'observation', frame_fn,
              Deque(max_length=num_stacked_frames), list,
              trailing_zero_pad(length=num_stacked_frames),
              lambda frames: np.stack(frames, axis=-1)),
      )))
