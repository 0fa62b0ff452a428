"""Learned-logit replays of `dqn_zoo/replay_circular.py`, logits in HBM.

* `CircularLogitBuffer` (replay_circular.py:148-248): ring of f32 logits, -inf
  for empty slots; `add()` without a value writes log-mean-exp of all slots
  (a device reduction over the whole capacity, as the reference does);
  `sample(n)` = `Generator.choice(capacity, n, p=softmax(logits))` on device,
  fed with the caller Generator's own uniform draws so the indices match the
  reference (pinned in tests/golden).
* `MGSCFiFoTransitionReplay` (:1217-1312) and `MGSCReservoirDistribution` /
  `MGSCReservoirTransitionReplay` (:500-664) on top, with frame transitions in
  a device FrameStore; their slots are what the learner and the meta-update
  consume.  `TransitionReplay` / `ReservoirTransitionReplay` (Generator
  variants, :251-497) are re-exported from replay.py.
"""

import typing
from typing import Any, Iterable, Mapping, Optional, Sequence, Tuple
import weakref

import numpy as np

from dqn_mgsc_zoo_amd import replay as replay_lib

Transition = replay_lib.Transition
ReservoirTransitionReplay = replay_lib.ReservoirTransitionReplay
TransitionAccumulator = replay_lib.TransitionAccumulator  # :1432-1466
SumTree = replay_lib.SumTree
importance_sampling_weights = replay_lib.importance_sampling_weights
_power = replay_lib._power  # pylint: disable=protected-access


def TransitionReplay(capacity, structure, random_state, encoder=None,  # pylint: disable=invalid-name
                     decoder=None, device=None):
  """FIFO uniform replay drawing with `Generator.integers` (:325-407)."""
  return replay_lib.TransitionReplay(
      capacity, structure, random_state, encoder, decoder, device,
      distribution_cls=replay_lib.GeneratorUniformDistribution)


def probabilities_from_logits(logits: np.ndarray) -> np.ndarray:
  logits = np.asarray(logits)
  return np.exp(logits - logsumexp(logits))


def logsumexp(x: np.ndarray) -> np.ndarray:
  c = x.max()
  return c + np.log(np.sum(np.exp(x - c)))


# Live device logit buffers by the address of their logits tensor, so a
# writer handed only the raw tensor (MetaLearner.update without
# logit_buffer) can still find the running state it must keep current.
_LIVE_BUFFERS = weakref.WeakValueDictionary()


def logit_buffer_of(logits) -> Optional['_DeviceLogits']:
  """The live _DeviceLogits whose logits tensor is `logits`, or None."""
  buf = _LIVE_BUFFERS.get(logits.data_ptr())
  if buf is None or buf.logits.numel() != logits.numel():
    return None
  return buf


class _DeviceLogits:
  """f32 logits [capacity] in HBM plus the libdqz reduction scratch."""

  def __init__(self, capacity, device='cuda', max_queries=1024):
    import ctypes  # pylint: disable=g-import-not-at-top
    import torch  # pylint: disable=g-import-not-at-top
    from dqn_mgsc_zoo_amd import _native  # pylint: disable=g-import-not-at-top
    if not torch.cuda.is_available():
      raise _native.NativeLibraryError('learned-logit buffers live in HBM: a '
                                       'HIP device is required')
    self._torch, self._native = torch, _native
    self.device = torch.device(device)
    self.logits = torch.full((capacity,), -np.inf, dtype=torch.float32,
                             device=self.device)
    h = ctypes.c_void_p()
    _native.check(_native.lib().dqz_logit_buffer_create(
        int(capacity), int(max_queries), ctypes.byref(h)))
    self._h = h
    self._u = torch.zeros((max_queries,), dtype=torch.float64,
                          device=self.device)
    self._idx = torch.zeros((max_queries,), dtype=torch.int64,
                            device=self.device)
    _LIVE_BUFFERS[self.logits.data_ptr()] = self

  def __del__(self):
    h = getattr(self, '_h', None)
    if h is not None and h.value and self._native._lib is not None:  # pylint: disable=protected-access
      self._native.lib().dqz_logit_buffer_destroy(h)
      self._h = None

  def add_default(self, write_pos, size, clear_pos=-1):
    n = self._native
    n.check(n.lib().dqz_logits_add(self._h, n.ptr(self.logits), int(clear_pos),
                                   int(write_pos), int(size), None,
                                   n.stream_handle()))

  def add_default_exact(self, write_pos, size, clear_pos=-1):
    """The reference's default logit exactly (dqz_logits_add_exact)."""
    n = self._native
    n.check(n.lib().dqz_logits_add_exact(self._h, n.ptr(self.logits), int(clear_pos),
                                         int(write_pos), int(size), n.stream_handle()))

  def set(self, positions, values):
    """logits[positions] = values in order, keeping the running log-sum-exp."""
    pos = self._torch.as_tensor(np.asarray(positions, np.int64),
                                device=self.device)
    val = self._torch.as_tensor(np.asarray(values, np.float32),
                                device=self.device)
    n = self._native
    n.check(n.lib().dqz_logits_write(self._h, n.ptr(self.logits), n.ptr(pos),
                                     n.ptr(val), int(pos.numel()),
                                     n.stream_handle()))

  def put(self, position, value):
    """logits[position] = value (one write, no host->device copy)."""
    n = self._native
    n.check(n.lib().dqz_logits_put(self._h, n.ptr(self.logits), int(position),
                                   float(value), n.stream_handle()))

  @property
  def handle(self):
    """The dqz_logit_buffer handle (for dqz_meta_update's logit_buf)."""
    return self._h

  def run_state(self):
    """The running log-sum-exp state (dqz_logits_run_get; synchronises)."""
    import ctypes  # pylint: disable=g-import-not-at-top
    n = self._native
    S, c = ctypes.c_double(), ctypes.c_float()
    valid, known, adds = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    n.check(n.lib().dqz_logits_run_get(self._h, ctypes.byref(S), ctypes.byref(c),
                                       ctypes.byref(valid), ctypes.byref(known),
                                       ctypes.byref(adds), n.stream_handle()))
    return {'S': S.value, 'c': c.value, 'valid': valid.value,
            'known': known.value, 'adds': adds.value}

  def set_run_state(self, st):
    n = self._native
    n.check(n.lib().dqz_logits_run_set(self._h, n.ptr(self.logits),
                                       float(st['S']), float(st['c']),
                                       int(st['valid']), int(st['known']),
                                       int(st['adds']), n.stream_handle()))

  def invalidate(self):
    """The logits tensor was (or may be) written outside the library."""
    self._native.check(self._native.lib().dqz_logits_invalidate(self._h))

  def writable(self):
    """The logits tensor for an outside writer (the meta-update)."""
    self.invalidate()
    return self.logits

  def load(self, logits):
    self.logits.copy_(self._torch.from_numpy(np.asarray(logits, np.float32)))
    self.invalidate()

  def get(self, positions):
    pos = self._torch.as_tensor(np.asarray(positions, np.int64),
                                device=self.device)
    return self.logits[pos].cpu().numpy()

  def terms(self):
    """(t, csum, c): the f32 terms expf(x - c) a draw's CDF is built from,
    the float64 chunk sums and the shift (diagnostic; device tensors)."""
    t = self._torch.empty_like(self.logits)
    nb = (self.logits.numel() + 4095) // 4096
    csum = self._torch.empty((nb,), dtype=self._torch.float64, device=self.device)
    c = self._torch.empty((1,), dtype=self._torch.float32, device=self.device)
    nat = self._native
    nat.check(nat.lib().dqz_logits_terms(self._h, nat.ptr(self.logits), nat.ptr(t),
                                         nat.ptr(csum), nat.ptr(c),
                                         nat.stream_handle()))
    return t, csum, c

  def probs(self):
    """(p, lse): the sampling probabilities (f32) and the running
    log-sum-exp (diagnostic; device tensors)."""
    p = self._torch.empty_like(self.logits)
    lse = self._torch.empty((1,), dtype=self._torch.float32, device=self.device)
    nat = self._native
    nat.check(nat.lib().dqz_logits_probs(self._h, nat.ptr(self.logits),
                                         nat.ptr(p), nat.ptr(lse),
                                         nat.stream_handle()))
    return p, lse

  def sample_exact(self, uniforms, probs=False):
    """The reference's draw exactly (dqz_logits_sample_exact): absolute
    slots for host uniforms from the reference's own float32 probabilities
    (numpy's operations, bit for bit), and those probabilities as a device
    tensor when `probs`."""
    n = len(uniforms)
    nat = self._native
    p = self._torch.empty_like(self.logits) if probs else None
    if n:
      u = self._u[:n]
      u.copy_(self._torch.as_tensor(np.asarray(uniforms, np.float64)))
      out = self._idx[:n]
    nat.check(nat.lib().dqz_logits_sample_exact(
        self._h, nat.ptr(self.logits), nat.ptr(u) if n else None, n, nat.ptr(out) if n else None,
        nat.ptr(p) if probs else None, nat.stream_handle()))
    idx = out if n else None
    return (idx, p) if probs else idx

  def sample_slots_philox(self, seed, counter, out_slots, out_idx=None):
    """Learner batch in one launch (dqz_logits_sample_slots): Philox
    uniforms (seed, device int64 counter, advanced on device), softmax-CDF
    choice, int32 absolute slots into `out_slots` (and int64 into `out_idx`
    if given).  Draws what dqz_uniform_philox + sample_abs would."""
    nat = self._native
    nat.check(nat.lib().dqz_logits_sample_slots(
        self._h, nat.ptr(self.logits), int(seed) & (2**64 - 1),
        nat.ptr(counter), None, int(out_slots.numel()), nat.ptr(out_slots),
        nat.ptr(out_idx), nat.stream_handle()))
    return out_slots

  def sample_abs(self, uniforms):
    """Absolute slots for host uniforms (device int64 tensor)."""
    n = len(uniforms)
    u = self._u[:n]
    u.copy_(self._torch.as_tensor(np.asarray(uniforms, np.float64)))
    out = self._idx[:n]
    nat = self._native
    nat.check(nat.lib().dqz_logits_sample(self._h, nat.ptr(self.logits),
                                          nat.ptr(u), n, nat.ptr(out),
                                          nat.stream_handle()))
    return out


class CircularLogitBuffer:
  """Ring of learned logits; sampling probability = softmax over capacity."""

  def __init__(self, capacity: int, random_state: np.random.Generator,
               device='cuda', exact_sampling=False):
    """exact_sampling: draw from the reference's own float32 probabilities
    (dqz_logits_sample_exact: six passes over the buffer per draw) instead
    of the running-state terms (O(1) per write, a float32 ulp per term), and
    form default logits with its own logsumexp (dqz_logits_add_exact, four
    passes per add)."""
    self._dev = _DeviceLogits(capacity, device)
    self._capacity = capacity
    self._size = 0
    self._left_head = 0
    self._right_head = 0
    self._rng_state = random_state
    self._exact = bool(exact_sampling)

  @property
  def capacity(self) -> int:
    return self._capacity

  @property
  def size(self) -> int:
    return self._size

  @property
  def logits(self):
    """Device f32 logits [capacity] (absolute slot order).  Handed out for
    writing (the meta-update's Adam step), so the next add re-scans."""
    return self._dev.writable()

  def is_full(self) -> bool:
    return self._size == self._capacity

  def add(self, item: Optional[float] = None) -> None:
    if self.is_full():
      raise BufferError('Buffer is full and cannot be added to. Pop an item first.')
    if item is None:
      if self._exact:
        self._dev.add_default_exact(self._right_head, self._size)
      else:
        self._dev.add_default(self._right_head, self._size)
    else:
      self._dev.put(self._right_head, item)
    self._right_head = (self._right_head + 1) % self._capacity
    self._size += 1

  def popleft(self, return_value=True):
    if self._size == 0:
      raise BufferError('Buffer is empty and cannot be popped from. Add an item first.')
    item = self._dev.get([self._left_head])[0] if return_value else None
    self._dev.put(self._left_head, -np.inf)
    self._left_head = (self._left_head + 1) % self._capacity
    self._size -= 1
    return item

  def _abs(self, key):
    return (self._left_head + np.asarray(key)) % self._capacity

  def __getitem__(self, key):
    if self._size == 0:
      raise BufferError('Buffer is empty and cannot be indexed. Add an item first.')
    key = np.asarray(key)
    if (key >= self._size).any():
      raise KeyError('Buffer is not large enough to index at position %s. '
                     'Must be in [0,%d).' % (key, self.size - 1))
    return self._dev.get(np.atleast_1d(self._abs(key))).reshape(key.shape)

  def __setitem__(self, key, item):
    key = np.asarray(key)
    if (key >= self._size).any():
      raise KeyError('Buffer is not large enough to index at position %s. '
                     'Must be in [0,%d).' % (key, self.size - 1))
    self._dev.set(np.atleast_1d(self._abs(key)), np.atleast_1d(item))

  def as_probs(self):
    if self._exact:  # probabilities_from_logits bit for bit
      return self._dev.sample_exact([], probs=True)[1]
    t = self._dev.logits
    return (t - self._dev._torch.logsumexp(t, 0)).exp()  # pylint: disable=protected-access

  def draw_uniforms(self, size: int) -> np.ndarray:
    """The Generator draws sample(size) consumes (same checks), for a caller
    that resolves them on device itself (Learner.step_logits)."""
    if self._size < size:
      raise BufferError('Cannot sample from buffer with length %d when '
                        'requested sample size was %d.' % (self._size, size))
    return self._rng_state.random(size)

  def sample_slots(self, size: int):
    """Absolute slots (device int64), drawn like Generator.choice(p=softmax)."""
    u = self.draw_uniforms(size)
    return self._dev.sample_exact(u) if self._exact else self._dev.sample_abs(u)

  def sample(self, size: int) -> np.ndarray:
    """Relative indices, as the reference returns them."""
    absolute = self.sample_slots(size).cpu().numpy()
    return (absolute - self._left_head) % self._capacity

  def sample_uniform(self, size: int, replace: bool = True) -> np.ndarray:
    if self._size < size:
      raise BufferError('Cannot sample from buffer with length %d when '
                        'requested sample size was %d.' % (self._size, size))
    return self._rng_state.choice(self._size, size=size, replace=replace)

  @property
  def device_logits(self):
    """The device logit buffer (logits + running log-sum-exp), for writers
    that keep the running state current (the meta-update)."""
    return self._dev

  def get_state(self) -> Mapping[str, Any]:
    # The running log-sum-exp travels with the logits: saving does not
    # disturb the saver, and a restored copy continues with the same bits.
    return {'capacity': self._capacity,
            'logits': self._dev.logits.cpu().numpy(), 'size': self._size,
            'left_head': self._left_head, 'right_head': self._right_head,
            'rng_state': self._rng_state, 'logit_run': self._dev.run_state()}

  def set_state(self, state: Mapping[str, Any]) -> None:
    self._capacity = state['capacity']
    self._dev.load(state['logits'])
    if 'logit_run' in state:
      self._dev.set_run_state(state['logit_run'])
    self._size = state['size']
    self._left_head = state['left_head']
    self._right_head = state['right_head']
    self._rng_state = state['rng_state']

  def check_valid(self) -> Tuple[bool, str]:
    return True, ''


class CircularBuffer:
  """Ring of items with popleft (replay_circular.py:90-146)."""

  def __init__(self, capacity: int):
    self._list = [None] * capacity
    self._capacity = capacity
    self._size = 0
    self._left_head = 0
    self._right_head = 0

  @property
  def capacity(self) -> int:
    return self._capacity

  @property
  def size(self) -> int:
    return self._size

  def is_full(self) -> bool:
    return self._size == self._capacity

  def add(self, item) -> int:
    if self.is_full():
      raise BufferError('Buffer is full and cannot be added to. Pop an item first.')
    pos = self._right_head
    self._list[pos] = item
    self._right_head = (pos + 1) % self._capacity
    self._size += 1
    return pos

  def popleft(self):
    if self._size == 0:
      raise BufferError('Buffer is empty and cannot be popped from. Add an item first.')
    item = self._list[self._left_head]
    self._left_head = (self._left_head + 1) % self._capacity
    self._size -= 1
    return item

  def __getitem__(self, key: int):
    if self._size == 0:
      raise BufferError('Buffer is empty and cannot be indexed. Add an item first.')
    return self._list[(self._left_head + key) % self._capacity]

  def __len__(self):
    return self._size

  def get_state(self) -> Mapping[str, Any]:
    return {'list': self._list, 'capacity': self._capacity, 'size': self._size,
            'left_head': self._left_head, 'right_head': self._right_head}

  def set_state(self, state: Mapping[str, Any]) -> None:
    self._list = state['list']
    self._capacity = state['capacity']
    self._size = state['size']
    self._left_head = state['left_head']
    self._right_head = state['right_head']


class _SlotStorage:
  """Item storage of the MGSC replays: host list or device FrameStore."""

  def __init__(self, capacity, mode, device):
    self._capacity = capacity
    self._mode = mode
    self._device = device
    self._backend = None

  def _make(self, use_device):
    if use_device:
      return replay_lib._DeviceStorage(  # pylint: disable=protected-access
          self._capacity, self._mode, None, self._device)
    return replay_lib._HostStorage(None, None)  # pylint: disable=protected-access

  def put(self, slot, item, oldest_live_slot=None):
    if self._backend is None:
      self._backend = self._make(replay_lib.is_frame_transition(item))
    self._backend.put(slot, item, oldest_live_slot)

  def drop(self, slot):
    if self._backend is not None:
      self._backend.drop(slot)

  def stack(self, structure, slots):
    return self._backend.stack(structure, np.asarray(slots))

  def slots_tensor(self, slots):
    return self._backend.slots_tensor(slots)

  @property
  def on_device(self):
    return self._backend is not None and self._backend.device

  @property
  def frame_store(self):
    return self._backend.store if self.on_device else None

  def get_state(self):
    return None if self._backend is None else self._backend.get_state()

  def set_state(self, state):
    if state is not None:
      if self._backend is None:
        self._backend = self._make(state.get('kind') == 'device')
      self._backend.set_state(state)


class MGSCFiFoTransitionReplay:
  """FIFO replay sampled by softmax(learned logits) (:1217-1312)."""

  def __init__(self, capacity: int, structure, random_state: np.random.Generator,
               encoder=None, decoder=None, device='cuda', exact_sampling=False):
    del encoder, decoder  # frames live uncompressed in HBM
    self._capacity = capacity
    self._structure = structure
    self._distribution = CircularLogitBuffer(capacity, random_state, device, exact_sampling)
    self._ring = CircularBuffer(capacity)  # slot of each live item, FIFO order
    self._items = _SlotStorage(capacity, 'ring', device)
    self._t = 0

  def add(self, item) -> None:
    if self._ring.is_full():
      self._distribution.popleft(return_value=False)
      self._items.drop(self._ring.popleft())
    self._distribution.add()
    slot = self._ring._right_head  # pylint: disable=protected-access
    oldest = self._ring[0] if self._ring.size else None
    self._items.put(slot, item, oldest)
    self._ring.add(slot)
    self._t += 1

  def get(self, indices: Sequence[int]) -> Iterable[Any]:
    for i in indices:
      yield self._items.stack(self._structure, [self._ring[int(i)]])

  def _slots(self, relative):
    return (self._ring._left_head + np.asarray(relative)) % self._capacity  # pylint: disable=protected-access

  def sample(self, size: int):
    return self.stack_transitions(self._distribution.sample(size))

  def sample_slots(self, size: int):
    """Device int32 slots drawn by softmax(logits) for the learner."""
    return self._distribution.sample_slots(size).to(dtype=_torch().int32)

  @property
  def exact_sampling(self) -> bool:
    """Draws follow the reference's own float32 probabilities exactly."""
    return self._distribution._exact  # pylint: disable=protected-access

  def stack_transitions(self, indices: Sequence[int]):
    return self._items.stack(self._structure, self._slots(indices))

  def batch_of_ids_transitions_and_logits(self, size: int):
    """Uniform meta batch without replacement (:1270-1275)."""
    indices = self._distribution.sample_uniform(size, replace=False)
    transitions = self.stack_transitions(indices)
    logits = self._distribution[np.asarray(indices)]
    return indices, transitions, logits

  def meta_batch_slots(self, size: int):
    """(relative indices, device int32 slots, device logit positions)."""
    indices = self._distribution.sample_uniform(size, replace=False)
    slots = self._slots(indices)
    return indices, self._items.slots_tensor(slots), slots

  def update_priorities(self, indices: Sequence[int], priorities) -> None:
    self._distribution[np.asarray(indices)] = priorities

  @property
  def frame_store(self):
    return self._items.frame_store

  @property
  def logits(self):
    return self._distribution.logits

  @property
  def device_logits(self):
    return self._distribution.device_logits

  def draw_uniforms(self, size: int):
    """Host Generator draws of sample(size), resolved on device by
    Learner.step_logits (absolute slots = item slots)."""
    return self._distribution.draw_uniforms(size)

  @property
  def size(self) -> int:
    return self._ring.size

  @property
  def capacity(self) -> int:
    return self._capacity

  def get_state(self) -> Mapping[str, Any]:
    return {'storage': self._ring.get_state(), 't': self._t,
            'distribution': self._distribution.get_state(),
            'items': self._items.get_state()}

  def set_state(self, state: Mapping[str, Any]) -> None:
    self._ring.set_state(state['storage'])
    self._t = state['t']
    self._distribution.set_state(state['distribution'])
    self._items.set_state(state.get('items'))

  def check_valid(self) -> Tuple[bool, str]:
    if self._t < self._ring.size:
      return False, 't should be >= storage size.'
    return self._distribution.check_valid()


class MGSCReservoirDistribution:
  """Fixed-slot learned logits for the reservoir replay (:500-565)."""

  def __init__(self, rng_state: np.random.Generator, capacity: int,
               device='cuda', exact_sampling=False):
    self._capacity = capacity
    self._dev = _DeviceLogits(capacity, device)
    self._size = 0
    self._rng_state = rng_state
    self._exact = bool(exact_sampling)  # as CircularLogitBuffer's

  @property
  def capacity(self) -> int:
    return self._capacity

  @property
  def size(self) -> int:
    return self._size

  @property
  def logits(self):
    """Device f32 logits [capacity]; handed out for writing (next add re-scans)."""
    return self._dev.writable()

  def is_full(self) -> bool:
    return self._size == self._capacity

  def add(self, priority: Optional[float] = None) -> None:
    if self.is_full():
      raise BufferError('Buffer is full and cannot be added to. Pop an item first.')
    if priority is None:
      if self._exact:
        self._dev.add_default_exact(self._size, self._size)
      else:
        self._dev.add_default(self._size, self._size)
    else:
      self._dev.put(self._size, priority)
    self._size += 1

  def replace(self, idx: int, priority: Optional[float] = None) -> None:
    """Reset slot idx: -inf, then log-mean-exp over all slots / size."""
    if not self.is_full():
      raise BufferError('Buffer should be full before replacing. Current '
                        'size=%d while capacity=%d.' % (self._size, self._capacity))
    if priority is None:
      if self._exact:
        self._dev.add_default_exact(idx, self._size, clear_pos=idx)
      else:
        self._dev.add_default(idx, self._size, clear_pos=idx)
    else:
      self._dev.put(idx, priority)

  def __getitem__(self, key):
    key = np.asarray(key)
    return self._dev.get(np.atleast_1d(key)).reshape(key.shape)

  def __setitem__(self, key, priority):
    self._dev.set(np.atleast_1d(key), np.atleast_1d(priority))

  def as_probs(self):
    if self._exact:  # probabilities_from_logits bit for bit
      return self._dev.sample_exact([], probs=True)[1]
    t = self._dev.logits
    return (t - self._dev._torch.logsumexp(t, 0)).exp()  # pylint: disable=protected-access

  def draw_uniforms(self, size: int) -> np.ndarray:
    if self._size < size:
      raise BufferError('Cannot sample a batch of size %d from buffer with '
                        'size %d.' % (size, self._size))
    return self._rng_state.random(size)

  def sample_slots(self, size: int):
    u = self.draw_uniforms(size)
    return self._dev.sample_exact(u) if self._exact else self._dev.sample_abs(u)

  def sample(self, size: int) -> np.ndarray:
    return self.sample_slots(size).cpu().numpy()

  def sample_uniform(self, size: int, replace: bool = True) -> np.ndarray:
    if self._size < size:
      raise BufferError('Cannot sample a batch of size %d from buffer with '
                        'size %d.' % (size, self._size))
    return self._rng_state.choice(self._size, size=size, replace=replace)

  @property
  def device_logits(self):
    return self._dev

  def get_state(self) -> Mapping[str, Any]:
    return {'capacity': self._capacity, 'logits': self._dev.logits.cpu().numpy(),
            'size': self._size, 'rng_state': self._rng_state,
            'logit_run': self._dev.run_state()}

  def set_state(self, state: Mapping[str, Any]) -> None:
    self._capacity = state['capacity']
    self._dev.load(state['logits'])
    if 'logit_run' in state:
      self._dev.set_run_state(state['logit_run'])
    self._size = state['size']
    self._rng_state = state['rng_state']


class MGSCReservoirTransitionReplay:
  """Reservoir replay sampled by softmax(learned logits) (:568-664)."""

  def __init__(self, capacity: int, structure, random_state: np.random.Generator,
               encoder=None, decoder=None, device='cuda', exact_sampling=False):
    del encoder, decoder
    self._capacity = capacity
    self._structure = structure
    self._random_state = random_state
    self._distribution = MGSCReservoirDistribution(random_state, capacity, device, exact_sampling)
    self._items = _SlotStorage(capacity, 'slot', device)
    self._t = 0

  def add(self, item) -> None:
    if self.size == self._capacity:
      j = self._random_state.integers(0, self._t)
      if j < self.size:
        self._items.put(int(j), item)
        self._distribution.replace(int(j))
    else:
      self._distribution.add()
      self._items.put(self._t, item)
    self._t += 1

  def get(self, ids: Sequence[int]) -> Iterable[Any]:
    for i in ids:
      yield self._items.stack(self._structure, [int(i)])

  def sample(self, size: int):
    return self.stack_transitions(self._distribution.sample(size))

  def sample_slots(self, size: int):
    return self._distribution.sample_slots(size).to(dtype=_torch().int32)

  @property
  def exact_sampling(self) -> bool:
    return self._distribution._exact  # pylint: disable=protected-access

  def stack_transitions(self, indices: Sequence[int]):
    return self._items.stack(self._structure, np.asarray(indices))

  def batch_of_ids_transitions_and_logits(self, size: int):
    indices = self._distribution.sample_uniform(size, replace=False)
    transitions = self.stack_transitions(indices)
    logits = self._distribution[np.asarray(indices)]
    return indices, transitions, logits

  def meta_batch_slots(self, size: int):
    indices = self._distribution.sample_uniform(size, replace=False)
    return indices, self._items.slots_tensor(indices), np.asarray(indices)

  def update_priorities(self, indices: Sequence[int], priorities) -> None:
    self._distribution[np.asarray(indices)] = priorities

  @property
  def frame_store(self):
    return self._items.frame_store

  @property
  def logits(self):
    return self._distribution.logits

  @property
  def device_logits(self):
    return self._distribution.device_logits

  def draw_uniforms(self, size: int):
    """Host Generator draws of sample(size), resolved on device by
    Learner.step_logits (absolute slots = item slots)."""
    return self._distribution.draw_uniforms(size)

  @property
  def size(self) -> int:
    return self._distribution.size

  @property
  def capacity(self) -> int:
    return self._capacity

  def get_state(self) -> Mapping[str, Any]:
    return {'storage': self._items.get_state(), 't': self._t,
            'distribution': self._distribution.get_state(),
            'random_state': self._random_state, 'capacity': self._capacity}

  def set_state(self, state: Mapping[str, Any]) -> None:
    self._items.set_state(state['storage'])
    self._t = state['t']
    self._distribution.set_state(state['distribution'])
    self._random_state = state['random_state']
    self._capacity = state['capacity']

  def check_valid(self) -> Tuple[bool, str]:
    return True, ''


def _torch():
  import torch  # pylint: disable=g-import-not-at-top
  return torch
