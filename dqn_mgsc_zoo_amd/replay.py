"""Replay components with the API of `dqn_zoo/replay.py`, storage in HBM.

Drop-in for the reference's uniform FIFO (`TransitionReplay`,
replay.py:163-243), reservoir (`ReservoirTransitionReplay`, :246-333) and
prioritized (`PrioritizedTransitionReplay`, :1046-1160) replays.

* ID bookkeeping and sampling decisions run on the host with the caller's
  `np.random.RandomState`, in the reference's call order, so a replay seeded
  like the reference draws the same IDs (pinned by tests/golden).
* Frame transitions (`Transition` with uint8 [84,84,4] stacks) are stored in a
  device `FrameStore` (frame pool + transition table; store.py).  `sample()`
  returns a `Transition` of device tensors; the learner consumes
  `sample_slots()` and never materialises stacks.  Any other item structure
  (the reference's tests use scalar named tuples) is kept host-side exactly
  like the reference container.
* `SumTree` / `PrioritizedDistribution` keep the fp64 tree on the host;
  `device_sumtree.py` mirrors it in HBM for the on-device PER sampler.

Exception types and messages follow the reference.
"""

import collections
import typing
from typing import Any, Callable, Iterable, Mapping, Optional, Sequence, Tuple

import numpy as np

FRAME_SHAPE = (84, 84, 4)


class Transition(typing.NamedTuple):
  s_tm1: Optional[Any]
  a_tm1: Optional[Any]
  r_t: Optional[Any]
  discount_t: Optional[Any]
  s_t: Optional[Any]


def is_frame_transition(item) -> bool:
  """True for a Transition whose states are uint8 84x84x4 stacks."""
  if not (isinstance(item, tuple) and hasattr(item, '_fields')):
    return False
  if 's_tm1' not in item._fields or 's_t' not in item._fields:
    return False
  s0, s1 = getattr(item, 's_tm1'), getattr(item, 's_t')
  return (isinstance(s0, np.ndarray) and isinstance(s1, np.ndarray) and
          s0.shape == FRAME_SHAPE and s1.shape == FRAME_SHAPE and
          s0.dtype == np.uint8 and s1.dtype == np.uint8)


# ---------------------------------------------------------------------------
# uniform distribution over integer IDs (replay.py:87-160)


class UniformDistribution:
  """Uniform sampling of integer IDs; swap-remove keeps IDs contiguous."""

  def __init__(self, random_state: np.random.RandomState):
    self._random_state = random_state
    self._ids = []
    self._id_to_index = {}

  def add(self, ids: Sequence[int]) -> None:
    for i in ids:
      if i in self._id_to_index:
        raise IndexError('Cannot add ID %d, it already exists.' % i)
    for i in ids:
      self._id_to_index[i] = len(self._ids)
      self._ids.append(i)

  def remove(self, ids: Sequence[int]) -> None:
    for i in ids:
      if i not in self._id_to_index:
        raise IndexError('Cannot remove ID %d, it does not exist.' % i)
    for i in ids:
      pos = self._id_to_index[i]
      last = self._ids[-1]
      self._ids[pos] = last
      self._id_to_index[last] = pos
      self._ids.pop()
      del self._id_to_index[i]

  def _draw(self, size):
    return self._random_state.randint(self.size, size=size)

  def sample(self, size: int) -> np.ndarray:
    positions = self._draw(size)
    return np.array([self._ids[p] for p in positions], dtype=np.int64)

  def ids(self) -> Iterable[int]:
    return self._id_to_index.keys()

  @property
  def size(self) -> int:
    return len(self._ids)

  def get_state(self) -> Mapping[str, Any]:
    return {'ids': self._ids, 'id_to_index': self._id_to_index}

  def set_state(self, state: Mapping[str, Any]) -> None:
    self._ids = state['ids']
    self._id_to_index = state['id_to_index']

  def check_valid(self) -> Tuple[bool, str]:
    if len(self._ids) != len(self._id_to_index):
      return False, 'ids and id_to_index should be the same size.'
    if len(set(self._ids)) != len(self._ids):
      return False, 'IDs should be unique.'
    if len(set(self._id_to_index.values())) != len(self._id_to_index):
      return False, 'Indices should be unique.'
    for i in self._ids:
      if self._ids[self._id_to_index[i]] != i:
        return False, 'ID %d should map to itself.' % i
    return True, ''


class GeneratorUniformDistribution(UniformDistribution):
  """`np.random.Generator` twin (replay_circular.py:251-322)."""

  def _draw(self, size):
    return self._random_state.integers(self.size, size=size)


# ---------------------------------------------------------------------------
# storage backends


class _HostStorage:
  """Reference-style container for arbitrary item structures."""

  device = False

  def __init__(self, encoder, decoder):
    self._encoder = encoder or (lambda s: s)
    self._decoder = decoder or (lambda s: s)
    self.items = {}

  def put(self, slot, item, oldest_live_slot=None):
    del oldest_live_slot
    self.items[slot] = self._encoder(item)

  def get(self, slot):
    return self._decoder(self.items[slot])

  def drop(self, slot):
    self.items.pop(slot, None)

  def stack(self, structure, slots):
    samples = [self.get(s) for s in slots]
    stacked = [np.stack(xs, axis=0) for xs in zip(*samples)]
    return type(structure)(*stacked)

  def get_state(self):
    return {'kind': 'host', 'items': dict(self.items)}

  def set_state(self, state):
    self.items = dict(state['items'])


class _DeviceStorage:
  """Frame transitions in a device FrameStore (store.py)."""

  device = True

  def __init__(self, capacity, mode, num_frames=None, device='cuda',
               frames_per_slot=5):
    import torch  # pylint: disable=g-import-not-at-top
    from dqn_mgsc_zoo_amd import _native  # pylint: disable=g-import-not-at-top
    from dqn_mgsc_zoo_amd import store as store_lib  # pylint: disable=g-import-not-at-top
    if not torch.cuda.is_available():
      raise _native.NativeLibraryError(
          'frame transitions are stored in HBM: a HIP device is required')
    _native.lib()
    if mode == 'ring':
      nf = num_frames or 2 * capacity + 64
    else:
      nf = capacity * frames_per_slot
    self._torch = torch
    self._args = {'capacity': capacity, 'mode': mode, 'num_frames': nf,
                  'frames_per_slot': frames_per_slot}
    self.store = store_lib.FrameStore(capacity, nf, device=device)
    self.allocator = store_lib.FrameAllocator(self.store, mode,
                                              per_slot=frames_per_slot)
    self.device_name = device
    self._slots_upload = None  # pinned staging of slots_tensor

  def put(self, slot, item, oldest_live_slot=None):
    s_tm1 = np.asarray(item.s_tm1, np.uint8)
    s_t = np.asarray(item.s_t, np.uint8)
    fidx, new_frames = self.allocator.allocate(slot, s_tm1, s_t,
                                               oldest_live_slot)
    self.store.put(slot, fidx, item.a_tm1, item.r_t, item.discount_t,
                   new_frames)

  def get(self, slot):
    return self.host_batch(np.array([slot]), single=True)

  def drop(self, slot):
    self.allocator.forget(slot)

  def slots_tensor(self, slots):
    """Device int32 copy of host slots, uploaded without a host wait
    (store.Uploader; a fresh tensor per call, so callers may keep it)."""
    a = np.asarray(slots, np.int32)
    if self._slots_upload is None or self._slots_upload.nbytes < a.nbytes:
      from dqn_mgsc_zoo_amd import store as store_lib  # pylint: disable=g-import-not-at-top
      self._slots_upload = store_lib.Uploader(max(a.nbytes, 4096))
    return self._slots_upload(self._torch.empty(a.shape, dtype=self._torch.int32,
                                                device=self.store.device), a)

  def stack(self, structure, slots):
    """Device Transition: uint8 stacks gathered on device, int32/f32 rest."""
    del structure
    st = self.store
    sl = self.slots_tensor(slots)
    s_tm1 = st.gather_stacks(sl, 0)
    s_t = st.gather_stacks(sl, 1)
    idx = sl.long()
    return Transition(s_tm1=s_tm1, a_tm1=st.action[idx], r_t=st.reward[idx],
                      discount_t=st.discount[idx], s_t=s_t)

  def host_batch(self, slots, single=False):
    tr = self.stack(None, slots)
    host = [x.cpu().numpy() for x in tr]
    if single:
      host = [h[0] for h in host]
    return Transition(*host)

  def get_state(self):
    st = self.store
    return {'kind': 'device', 'args': dict(self._args),
            'frames': st.frames.cpu().numpy(), 'fidx': st.fidx.cpu().numpy(),
            'action': st.action.cpu().numpy(),
            'reward': st.reward.cpu().numpy(),
            'discount': st.discount.cpu().numpy(),
            'allocator': self.allocator.get_state()}

  def set_state(self, state):
    st = self.store
    t = self._torch
    st.frames.copy_(t.from_numpy(state['frames']))
    st.fidx.copy_(t.from_numpy(state['fidx']))
    st.action.copy_(t.from_numpy(state['action']))
    st.reward.copy_(t.from_numpy(state['reward']))
    st.discount.copy_(t.from_numpy(state['discount']))
    self.allocator.set_state(state['allocator'])


class _StorageMixin:
  """Picks host or device storage on the first add()."""

  def _init_storage(self, capacity, encoder, decoder, device, num_frames,
                    mode):
    self._backend = None
    self._backend_args = (capacity, encoder, decoder, device, num_frames, mode)

  def _make_backend(self, use_device):
    capacity, encoder, decoder, device, num_frames, mode = self._backend_args
    if use_device:
      return _DeviceStorage(capacity, mode, num_frames,
                            device if isinstance(device, str) else 'cuda',
                            frames_per_slot=getattr(self, '_frames_per_slot', 5))
    return _HostStorage(encoder, decoder)

  def _storage_for(self, item):
    if self._backend is None:
      device = self._backend_args[3]
      self._backend = self._make_backend(
          device if device is not None else is_frame_transition(item))
    return self._backend

  def _restore_backend(self, backend_state):
    """set_state(): re-creates the storage kind the checkpoint was made with."""
    if backend_state is None:
      return
    if self._backend is None:
      self._backend = self._make_backend(backend_state.get('kind') == 'device')
    self._backend.set_state(backend_state)

  def stores_on_device(self, item) -> bool:
    """Whether `item` is (or, on the first add, will be) stored in HBM."""
    if self._backend is not None:
      return self._backend.device
    device = self._backend_args[3]
    return bool(device) if device is not None else is_frame_transition(item)

  @property
  def on_device(self) -> bool:
    return self._backend is not None and self._backend.device

  @property
  def frame_store(self):
    """The device FrameStore (None for host-stored items)."""
    return self._backend.store if self.on_device else None


# ---------------------------------------------------------------------------
# FIFO uniform replay (replay.py:163-243)


class TransitionReplay(_StorageMixin):
  """Uniform replay with FIFO eviction; slot of ID i is i mod capacity."""

  def __init__(self, capacity: int, structure, random_state,
               encoder: Optional[Callable] = None,
               decoder: Optional[Callable] = None, device=None,
               num_frames: Optional[int] = None,
               distribution_cls=UniformDistribution):
    self._capacity = capacity
    self._structure = structure
    self._random_state = random_state
    self._distribution = distribution_cls(random_state=random_state)
    self._order = collections.OrderedDict()  # live IDs, oldest first
    self._t = 0
    self._init_storage(capacity, encoder, decoder, device, num_frames, 'ring')

  def _slot(self, item_id):
    return item_id % self._capacity

  def add(self, item) -> None:
    backend = self._storage_for(item)
    if self.size == self._capacity:
      oldest_id, _ = self._order.popitem(last=False)
      self._distribution.remove([oldest_id])
      backend.drop(self._slot(oldest_id))
    item_id = self._t
    self._distribution.add([item_id])
    oldest = next(iter(self._order)) if self._order else None
    backend.put(self._slot(item_id), item,
                None if oldest is None else self._slot(oldest))
    self._order[item_id] = None
    self._t += 1

  def get(self, ids: Sequence[int]) -> Iterable[Any]:
    for i in ids:
      if i not in self._order:
        raise KeyError(i)
      yield self._backend.get(self._slot(i))

  def sample_ids(self, size: int) -> np.ndarray:
    return self._distribution.sample(size)

  def slots_of(self, ids) -> np.ndarray:
    return np.asarray(ids, np.int64) % self._capacity

  def sample(self, size: int):
    """Batch of `size` items, uniformly with replacement."""
    ids = self.sample_ids(size)
    return self._backend.stack(self._structure, self.slots_of(ids))

  def sample_slots(self, size: int):
    """(ids, device int32 slots) for the learner; frame storage only."""
    ids = self.sample_ids(size)
    return ids, self._backend.slots_tensor(self.slots_of(ids))

  def ids(self) -> Iterable[int]:
    return self._order.keys()

  @property
  def size(self) -> int:
    return len(self._order)

  @property
  def capacity(self) -> int:
    return self._capacity

  @property
  def t(self) -> int:
    return self._t

  def get_state(self) -> Mapping[str, Any]:
    return {
        'storage': list(self._order.keys()),
        't': self._t,
        'distribution': self._distribution.get_state(),
        'backend': None if self._backend is None else self._backend.get_state(),
    }

  def set_state(self, state: Mapping[str, Any]) -> None:
    self._order = collections.OrderedDict((i, None) for i in state['storage'])
    self._t = state['t']
    self._distribution.set_state(state['distribution'])
    self._restore_backend(state.get('backend'))

  def check_valid(self) -> Tuple[bool, str]:
    if self._t < len(self._order):
      return False, 't should be >= storage size.'
    if set(self._order.keys()) != set(self._distribution.ids()):
      return False, 'IDs in storage and distribution do not match.'
    return self._distribution.check_valid()


# ---------------------------------------------------------------------------
# reservoir replay (replay.py:246-333; Generator twin replay_circular.py:410-497)


class ReservoirTransitionReplay(_StorageMixin):
  """Fill to capacity, then Algorithm R: j = randint(0, t) (exclusive upper
  bound, as replay.py:271) replaces slot j when j < size."""

  def __init__(self, capacity: int, structure, random_state,
               encoder: Optional[Callable] = None,
               decoder: Optional[Callable] = None, device=None,
               frames_per_slot: int = 5):
    self._capacity = capacity
    self._structure = structure
    self._random_state = random_state
    if isinstance(random_state, np.random.Generator):
      self._distribution = GeneratorUniformDistribution(random_state)
      self._randint = lambda hi: int(random_state.integers(0, hi))
    else:
      self._distribution = UniformDistribution(random_state)
      self._randint = lambda hi: int(random_state.randint(0, hi))
    self._slots = set()
    self._t = 0
    self._frames_per_slot = frames_per_slot
    self._init_storage(capacity, encoder, decoder, device, None, 'slot')

  def add(self, item) -> None:
    backend = self._storage_for(item)
    if self.size == self._capacity:
      j = self._randint(self._t)
      if j < self.size:
        backend.put(j, item)
    else:
      item_id = self._t
      self._distribution.add([item_id])
      backend.put(item_id, item)
      self._slots.add(item_id)
    self._t += 1

  def get(self, ids: Sequence[int]) -> Iterable[Any]:
    for i in ids:
      yield self._backend.get(i)

  def sample_ids(self, size: int) -> np.ndarray:
    return self._distribution.sample(size)

  def sample(self, size: int):
    return self._backend.stack(self._structure, self.sample_ids(size))

  def sample_slots(self, size: int):
    ids = self.sample_ids(size)
    return ids, self._backend.slots_tensor(ids)

  def ids(self) -> Iterable[int]:
    return sorted(self._slots)

  @property
  def size(self) -> int:
    return len(self._slots)

  @property
  def capacity(self) -> int:
    return self._capacity

  def get_state(self) -> Mapping[str, Any]:
    return {'storage': sorted(self._slots), 't': self._t,
            'distribution': self._distribution.get_state(),
            'backend': None if self._backend is None else self._backend.get_state()}

  def set_state(self, state: Mapping[str, Any]) -> None:
    self._slots = set(state['storage'])
    self._t = state['t']
    self._distribution.set_state(state['distribution'])
    self._restore_backend(state.get('backend'))

  def check_valid(self) -> Tuple[bool, str]:
    if self._t < len(self._slots):
      return False, 't should be >= storage size.'
    if set(self._slots) != set(self._distribution.ids()):
      return False, 'IDs in storage and distribution do not match.'
    return self._distribution.check_valid()


# ---------------------------------------------------------------------------
# prioritized replay (replay.py:336-784, 1046-1160)


def _power(base, exponent) -> np.ndarray:
  """base ** exponent with 0 ** e == 0 (zero priority is never sampled)."""
  base = np.asarray(base)
  return np.where(base == 0.0, 0.0, base**exponent)


def importance_sampling_weights(probabilities, uniform_probability: float,
                                exponent: float, normalize: bool) -> np.ndarray:
  """(uniform_probability / p) ** exponent, optionally divided by its max."""
  if not 0.0 <= exponent <= 1.0:
    raise ValueError('Require 0 <= exponent <= 1.')
  if not 0.0 <= uniform_probability <= 1.0:
    raise ValueError('Expected 0 <= uniform_probability <= 1.')
  weights = (uniform_probability / np.asarray(probabilities)) ** exponent
  if normalize:
    weights = weights / np.max(weights)
  if not np.isfinite(weights).all():
    raise ValueError('Weights are not finite: %s.' % weights)
  return weights


class SumTree:
  """Implicit binary tree of fp64 partial sums over non-negative leaves.

  storage[1] is the root, node i has children 2i and 2i+1, leaves occupy
  [first_leaf, first_leaf + size) with first_leaf = capacity (a power of two).
  Every internal node is recomputed as left + right, so the fp64 values are
  a deterministic function of the leaves (the device mirror relies on it).
  """

  def __init__(self):
    self._size = 0
    self._storage = np.zeros(0, dtype=np.float64)
    self._first_leaf = 0

  def resize(self, size: int) -> None:
    self._initialize(size, None)

  def get(self, indices: Sequence[int]) -> np.ndarray:
    indices = np.asarray(indices)
    if not ((0 <= indices) & (indices < self.size)).all():
      raise IndexError('index out of range, expect 0 <= index < %s' % self.size)
    return self.values[indices]

  def set(self, indices: Sequence[int], values: Sequence[float]) -> None:
    values = np.asarray(values)
    if not np.isfinite(values).all() or (values < 0.0).any():
      raise ValueError('value must be finite and positive.')
    self.values[indices] = values
    st = self._storage
    for leaf in np.asarray(indices) + self._first_leaf:
      node = int(leaf) >> 1
      while node > 0:
        st[node] = st[2 * node] + st[2 * node + 1]
        node >>= 1

  def set_all(self, values: Sequence[float]) -> None:
    values = np.asarray(values)
    if not np.isfinite(values).all() or (values < 0.0).any():
      raise ValueError('Values must be finite positive numbers.')
    self._initialize(len(values), values)

  def query(self, targets: Sequence[float]) -> Sequence[int]:
    """Smallest index whose inclusive prefix sum exceeds each target."""
    return [self._descend(t) for t in targets]

  def root(self) -> float:
    return self._storage[1] if self.size > 0 else np.nan

  @property
  def values(self) -> np.ndarray:
    return self._storage[self._first_leaf:self._first_leaf + self.size]

  @property
  def size(self) -> int:
    return self._size

  @property
  def capacity(self) -> int:
    return self._first_leaf

  @property
  def storage(self) -> np.ndarray:
    return self._storage

  def get_state(self) -> Mapping[str, Any]:
    return {'size': self._size, 'storage': self._storage,
            'first_leaf': self._first_leaf}

  def set_state(self, state: Mapping[str, Any]) -> None:
    self._size = state['size']
    self._storage = state['storage']
    self._first_leaf = state['first_leaf']

  def check_valid(self) -> Tuple[bool, str]:
    if len(self._storage) != 2 * self._first_leaf:
      return False, 'first_leaf should be half the size of storage.'
    if not 0 <= self.size <= self.capacity:
      return False, 'Require 0 <= self.size <= self.capacity.'
    if len(self.values) != self.size:
      return False, 'Number of values should be equal to the size.'
    st = self._storage
    for i in range(1, self._first_leaf):
      if st[i] != st[2 * i] + st[2 * i + 1]:
        return False, 'Non-leaf node %d should be sum of child nodes.' % i
    return True, ''

  def _initialize(self, size, values):
    assert size >= 0
    if size < self.size:
      new_values = self.values[:size] if values is None else values
      self._size = size
      self._rebuild(new_values)
    elif size <= self.capacity:
      self._size = size
      if values is not None:
        self._rebuild(values)
    else:
      cap = 1
      while cap < size:
        cap *= 2
      new_values = self.values if values is None else values
      self._storage = np.empty((2 * cap,), dtype=np.float64)
      self._first_leaf = cap
      self._size = size
      self._rebuild(new_values)

  def _rebuild(self, values):
    assert len(values) <= self.capacity
    st = self._storage
    fl = self._first_leaf
    st[fl:fl + len(values)] = values
    st[fl + len(values):] = 0
    for i in range(fl - 1, 0, -1):
      st[i] = st[2 * i] + st[2 * i + 1]
    st[0] = 0.0

  def _descend(self, target):
    if not 0.0 <= target < self.root():
      raise ValueError('Require 0 <= target < total sum.')
    st = self._storage
    node = 1
    while node < self._first_leaf:
      left = st[2 * node]
      if target < left:
        node = 2 * node
      else:
        target -= left
        node = 2 * node + 1
    return node - self._first_leaf


class _DeviceSumTree:
  """The SumTree's fp64 storage in HBM (same implicit layout: root at 1,
  leaves from `capacity`), for replays whose transitions live on device.

  Writes go through libdqz (`dqz_sumtree_set`, `dqz_per_add`,
  `dqz_per_write_back`: ancestors rebuilt as left + right, bit-identical to
  SumTree.set).  Host reads (`get`, `root`, `storage`, state) copy back and
  synchronise; the learner path never makes them.  Also owns the device map
  tree index -> replay slot the sampler uses.
  """

  def __init__(self, host_tree: SumTree, device):
    import torch  # pylint: disable=g-import-not-at-top
    from dqn_mgsc_zoo_amd import _native  # pylint: disable=g-import-not-at-top
    self._torch, self._native = torch, _native
    self._size = host_tree.size
    cap = max(host_tree.capacity, 1)
    self._first_leaf = cap
    st = np.zeros((2 * cap,), np.float64)
    st[:len(host_tree.storage)] = host_tree.storage
    self.tree = torch.from_numpy(st).to(device)
    self.index_to_slot = torch.zeros((cap,), dtype=torch.int32, device=device)

  def _check(self, rc):
    return self._native.check(rc)

  def resize(self, size: int) -> None:
    if size > self._first_leaf:
      raise ValueError('the device sum tree has a fixed capacity of %d leaves'
                       % self._first_leaf)
    if size < self._size:
      self.tree[self._first_leaf + size:] = 0.0
      self._rebuild()
    self._size = size

  def _rebuild(self):
    st = self.tree.cpu().numpy()
    fl = self._first_leaf
    for i in range(fl - 1, 0, -1):
      st[i] = st[2 * i] + st[2 * i + 1]
    self.tree.copy_(self._torch.from_numpy(st))

  def get(self, indices: Sequence[int]) -> np.ndarray:
    indices = np.asarray(indices)
    if not ((0 <= indices) & (indices < self.size)).all():
      raise IndexError('index out of range, expect 0 <= index < %s' % self.size)
    return self.values[indices]

  def set(self, indices: Sequence[int], values: Sequence[float]) -> None:
    values = np.asarray(values, np.float64)
    if not np.isfinite(values).all() or (values < 0.0).any():
      raise ValueError('value must be finite and positive.')
    indices = np.asarray(indices, np.int64).reshape(-1)
    if indices.size == 0:
      return
    last = {}
    for i, v in zip(indices.tolist(), np.broadcast_to(values, indices.shape).tolist()):
      last[i] = v  # numpy fancy assignment: the last write of an index wins
    t = self._torch
    idx = t.tensor(list(last.keys()), dtype=t.int64).to(self.tree.device, non_blocking=True)
    val = t.tensor(list(last.values()), dtype=t.float64).to(self.tree.device, non_blocking=True)
    n = self._native
    self._check(n.lib().dqz_sumtree_set(n.ptr(self.tree), self._first_leaf, n.ptr(idx),
                                        n.ptr(val), len(last), n.stream_handle()))

  def per_add(self, remove_index, add_index, priority, max_seen_dev, alpha, slot):
    n = self._native
    self._check(n.lib().dqz_per_add(
        n.ptr(self.tree), self._first_leaf, int(remove_index), int(add_index),
        float(priority), n.ptr(max_seen_dev), float(alpha),
        n.ptr(self.index_to_slot), int(slot), n.stream_handle()))

  def root(self) -> float:
    return float(self.tree[1].item()) if self.size > 0 else np.nan

  @property
  def values(self) -> np.ndarray:
    fl = self._first_leaf
    return self.tree[fl:fl + self.size].cpu().numpy()

  @property
  def size(self) -> int:
    return self._size

  @property
  def capacity(self) -> int:
    return self._first_leaf

  @property
  def storage(self) -> np.ndarray:
    return self.tree.cpu().numpy()

  def get_state(self) -> Mapping[str, Any]:
    return {'size': self._size, 'storage': self.storage,
            'first_leaf': self._first_leaf}

  def set_state(self, state: Mapping[str, Any]) -> None:
    if state['first_leaf'] != self._first_leaf:
      raise ValueError('sum tree capacity mismatch: %d vs %d' %
                       (state['first_leaf'], self._first_leaf))
    self._size = state['size']
    self.tree.copy_(self._torch.from_numpy(np.asarray(state['storage'], np.float64)))

  def check_valid(self) -> Tuple[bool, str]:
    host = SumTree()
    host.set_state(self.get_state())
    return host.check_valid()


class PrioritizedDistribution:
  """Proportional prioritized sampling of integer IDs (replay.py:562-784)."""

  def __init__(self, priority_exponent: float, uniform_sample_probability: float,
               random_state: np.random.RandomState, min_capacity: int = 0,
               max_capacity: Optional[int] = None):
    if priority_exponent < 0.0:
      raise ValueError('Require priority_exponent >= 0.')
    if not 0.0 <= uniform_sample_probability <= 1.0:
      raise ValueError('Require 0 <= uniform_sample_probability <= 1.')
    if max_capacity is not None and max_capacity < min_capacity:
      raise ValueError('Require max_capacity >= min_capacity.')
    if min_capacity < 0:
      raise ValueError('Require min_capacity >= 0.')
    self._priority_exponent = priority_exponent
    self._uniform_sample_probability = uniform_sample_probability
    self._max_capacity = max_capacity
    self._sum_tree = SumTree()
    self._sum_tree.resize(min_capacity)
    self._random_state = random_state
    self._id_to_index = {}
    self._index_to_id = {}
    self._inactive_indices = list(range(min_capacity))
    self._active_indices = []
    self._active_indices_location = {}
    self._positive_written = False

  @property
  def sum_tree(self) -> SumTree:
    return self._sum_tree

  @property
  def priority_exponent(self) -> float:
    return self._priority_exponent

  @property
  def uniform_sample_probability(self) -> float:
    return self._uniform_sample_probability

  @property
  def on_device(self) -> bool:
    return isinstance(self._sum_tree, _DeviceSumTree)

  def to_device(self, device) -> None:
    """Moves the tree into HBM (fixed capacity from here on)."""
    if not self.on_device:
      self._sum_tree = _DeviceSumTree(self._sum_tree, device)

  def draw(self, size: int):
    """The random streams of sample(), in the reference's order
    (replay.py:684-697): tree indices of the uniform picks, target
    fractions, usp-mix uniforms -> (uniform_idx, [targets, mix]).  The
    reference skips the target draw while the tree's root is 0; the host
    knows that without reading the device tree as long as no positive
    priority has been written (`_positive_written`), and then draws the mix
    stream only (targets 0: with root 0 every draw is its uniform pick).
    Once a positive priority was written the root is taken as positive: a
    tree whose positive leaves were all removed or written back as 0 again
    would draw the target stream where the reference does not (stated in
    INTEGRATION.md)."""
    if self.size == 0:
      raise RuntimeError('No IDs to sample.')
    rs = self._random_state
    uniform_idx = np.array([self._active_indices[j]
                            for j in rs.randint(self.size, size=size)], np.int32)
    if self.on_device:
      root_zero = not self._positive_written
    else:
      root_zero = self._sum_tree.root() == 0.0
    if root_zero:
      u = np.concatenate([np.zeros(size), rs.uniform(size=size)])
    else:
      u = np.concatenate([rs.uniform(size=size), rs.uniform(size=size)])
    return uniform_idx, u

  def note_priorities(self, priorities) -> None:
    """Host bookkeeping of draw(): a positive priority (or a device value,
    the agent's running max_seen_priority >= 1) makes the root positive."""
    if priorities is None or np.any(np.asarray(priorities) > 0.0):
      self._positive_written = True

  def index_to_id(self, indices) -> np.ndarray:
    return np.array([self._index_to_id[int(i)] for i in indices], dtype=np.int64)

  def ensure_capacity(self, capacity: int) -> None:
    if self._max_capacity is not None and capacity > self._max_capacity:
      raise ValueError('capacity %d cannot exceed max_capacity %d' %
                       (capacity, self._max_capacity))
    if capacity <= self._sum_tree.size:
      return
    self._inactive_indices.extend(range(self._sum_tree.size, capacity))
    self._sum_tree.resize(capacity)

  def _assign_indices(self, ids: Sequence[int]):
    """add_priorities' bookkeeping: checks, growth, tree indices for ids."""
    for i in ids:
      if i in self._id_to_index:
        raise IndexError('ID %d already exists.' % i)
    new_size = self.size + len(ids)
    if self._max_capacity is not None and new_size > self._max_capacity:
      raise ValueError('Cannot add IDs as max capacity would be exceeded.')
    if new_size > self.capacity:
      grow = max(new_size, 2 * self.capacity)
      if self._max_capacity is not None:
        grow = min(self._max_capacity, grow)
      self.ensure_capacity(grow)
    indices = []
    for i in ids:
      idx = self._inactive_indices.pop()
      self._active_indices_location[idx] = len(self._active_indices)
      self._active_indices.append(idx)
      self._id_to_index[i] = idx
      self._index_to_id[idx] = i
      indices.append(idx)
    return indices

  def _release_indices(self, ids: Sequence[int]):
    """remove_priorities' bookkeeping (swap-remove); the freed indices."""
    indices = [self._id_to_index[i] for i in ids]  # KeyError if absent
    for i, idx in zip(ids, indices):
      del self._id_to_index[i]
      del self._index_to_id[idx]
      loc = self._active_indices_location[idx]
      last = self._active_indices[-1]
      self._active_indices[loc] = last
      self._active_indices_location[last] = loc
      self._active_indices.pop()
      del self._active_indices_location[idx]
    self._inactive_indices.extend(indices)
    return indices

  def add_priorities(self, ids: Sequence[int], priorities: Sequence[float]) -> None:
    self.note_priorities(priorities)
    indices = self._assign_indices(ids)
    self._sum_tree.set(indices, _power(priorities, self._priority_exponent))
    return indices

  def remove_priorities(self, ids: Sequence[int]) -> None:
    indices = self._release_indices(ids)
    self._sum_tree.set(indices, np.zeros((len(indices),), dtype=np.float64))
    return indices

  def update_priorities(self, ids: Sequence[int], priorities: Sequence[float]) -> None:
    self.note_priorities(priorities)
    indices = []
    for i in ids:
      if i not in self._id_to_index:
        raise IndexError('ID %d does not exist.' % i)
      indices.append(self._id_to_index[i])
    self._sum_tree.set(indices, _power(priorities, self._priority_exponent))
    return indices

  def sample(self, size: int) -> Tuple[np.ndarray, np.ndarray]:
    """IDs and their sampling probabilities, in the reference's RNG order:
    randint (uniform picks), uniform*root (tree targets), uniform (< usp)."""
    if self.size == 0:
      raise RuntimeError('No IDs to sample.')
    rs = self._random_state
    uniform_idx = [self._active_indices[j] for j in rs.randint(self.size, size=size)]
    root = self._sum_tree.root()
    if root == 0.0:
      prio_idx = uniform_idx
    else:
      prio_idx = np.asarray(self._sum_tree.query(rs.uniform(size=size) * root))
    usp = self._uniform_sample_probability
    indices = np.where(rs.uniform(size=size) < usp, uniform_idx, prio_idx)
    uniform_prob = np.asarray(1.0 / self.size)
    leaves = self._sum_tree.get(indices)
    if root == 0.0:
      prio_probs = np.full_like(leaves, fill_value=uniform_prob)
    else:
      prio_probs = leaves / root
    probs = (1.0 - usp) * prio_probs + usp * uniform_prob
    ids = np.array([self._index_to_id[i] for i in indices], dtype=np.int64)
    return ids, probs

  def get_exponentiated_priorities(self, ids: Sequence[int]) -> Sequence[float]:
    idx = np.array([self._id_to_index[i] for i in ids], dtype=np.int64)
    return self._sum_tree.get(idx)

  def index_of(self, ids) -> np.ndarray:
    return np.array([self._id_to_index[i] for i in ids], dtype=np.int64)

  def ids(self) -> Iterable[int]:
    return self._id_to_index.keys()

  @property
  def capacity(self) -> int:
    return self._sum_tree.size

  @property
  def size(self) -> int:
    return len(self._id_to_index)

  def get_state(self) -> Mapping[str, Any]:
    return {'sum_tree': self._sum_tree.get_state(),
            'id_to_index': self._id_to_index, 'index_to_id': self._index_to_id,
            'inactive_indices': self._inactive_indices,
            'active_indices': self._active_indices,
            'active_indices_location': self._active_indices_location,
            'positive_written': self._positive_written}

  def set_state(self, state: Mapping[str, Any]) -> None:
    self._sum_tree.set_state(state['sum_tree'])
    self._id_to_index = state['id_to_index']
    self._index_to_id = state['index_to_id']
    self._inactive_indices = state['inactive_indices']
    self._active_indices = state['active_indices']
    self._active_indices_location = state['active_indices_location']
    self._positive_written = state.get(
        'positive_written', bool(self._sum_tree.root() > 0.0))

  def check_valid(self) -> Tuple[bool, str]:
    if len(self._id_to_index) != len(self._index_to_id):
      return False, 'ID to index maps are not the same size.'
    for i in self._id_to_index:
      if self._index_to_id[self._id_to_index[i]] != i:
        return False, 'ID %d should map to itself.' % i
    if len(set(self._inactive_indices)) != len(self._inactive_indices):
      return False, 'Inactive indices should be unique.'
    if len(set(self._active_indices)) != len(self._active_indices):
      return False, 'Active indices should be unique.'
    if set(self._active_indices) != set(self._index_to_id.keys()):
      return False, 'Active indices should match index to ID mapping keys.'
    if sorted(self._inactive_indices + self._active_indices) != list(
        range(self._sum_tree.size)):
      return False, 'Inactive and active indices should partition all indices.'
    if len(self._active_indices) != len(self._active_indices_location):
      return False, 'Active indices and their location should be the same size.'
    for j, i in enumerate(self._active_indices):
      if j != self._active_indices_location[i]:
        return False, 'Active index location %d not correct for index %d.' % (j, i)
    return self._sum_tree.check_valid()


class PrioritizedTransitionReplay(_StorageMixin):
  """Prioritized replay with FIFO eviction (replay.py:1046-1160)."""

  def __init__(self, capacity: int, structure, priority_exponent: float,
               importance_sampling_exponent: Callable[[int], float],
               uniform_sample_probability: float, normalize_weights: bool,
               random_state: np.random.RandomState,
               encoder: Optional[Callable] = None,
               decoder: Optional[Callable] = None, device=None,
               num_frames: Optional[int] = None):
    self._capacity = capacity
    self._structure = structure
    self._random_state = random_state
    self._distribution = PrioritizedDistribution(
        min_capacity=capacity, max_capacity=capacity,
        priority_exponent=priority_exponent,
        uniform_sample_probability=uniform_sample_probability,
        random_state=random_state)
    self._importance_sampling_exponent = importance_sampling_exponent
    self._normalize_weights = normalize_weights
    self._order = collections.OrderedDict()
    self._t = 0
    self._init_storage(capacity, encoder, decoder, device, num_frames, 'ring')

  def _slot(self, item_id):
    return item_id % self._capacity

  def add(self, item, priority) -> None:
    """`priority` is a float, or — for a device replay — a device f64 [1]
    tensor (the agent's running max_seen_priority, read on device)."""
    backend = self._storage_for(item)
    if backend.device:
      self._add_device(backend, item, priority)
      return
    if not isinstance(priority, (int, float, np.floating, np.integer)):
      priority = float(priority.item())
    if self.size == self._capacity:
      oldest_id, _ = self._order.popitem(last=False)
      self._distribution.remove_priorities([oldest_id])
      backend.drop(self._slot(oldest_id))
    item_id = self._t
    self._distribution.add_priorities([item_id], [priority])
    oldest = next(iter(self._order)) if self._order else None
    backend.put(self._slot(item_id), item,
                None if oldest is None else self._slot(oldest))
    self._order[item_id] = None
    self._t += 1

  def _device_tree(self):
    dist = self._distribution
    if not dist.on_device:
      dist.to_device(self._backend.store.device)
      self._sync_index_map()
    return dist.sum_tree

  def _sync_index_map(self):
    """index_to_slot of every live ID (after a restore)."""
    import torch  # pylint: disable=g-import-not-at-top
    dist = self._distribution
    ids = list(self._order)
    if not ids:
      return
    idx = torch.as_tensor(dist.index_of(ids), dtype=torch.int64)
    slots = torch.as_tensor(np.asarray(ids, np.int64) % self._capacity,
                            dtype=torch.int32)
    m = dist.sum_tree.index_to_slot
    m[idx.to(m.device)] = slots.to(m.device)

  def _add_device(self, backend, item, priority) -> None:
    """One dqz_per_add launch: evicted leaf -> 0, new leaf -> p ** alpha,
    tree index -> slot; ID bookkeeping stays on the host."""
    tree = self._device_tree()
    dist = self._distribution
    remove = -1
    if self.size == self._capacity:
      oldest_id, _ = self._order.popitem(last=False)
      remove = dist._release_indices([oldest_id])[0]  # pylint: disable=protected-access
      backend.drop(self._slot(oldest_id))
    item_id = self._t
    add = dist._assign_indices([item_id])[0]  # pylint: disable=protected-access
    dist.note_priorities(
        priority if isinstance(priority, (int, float, np.floating, np.integer))
        else None)
    if isinstance(priority, (int, float, np.floating, np.integer)):
      # host priority: exponentiated here with numpy, like the reference
      # (SumTree leaves bit-equal to the host path); the kernel's ** 1 is exact
      p = float(_power(float(priority), dist.priority_exponent))
      if not (np.isfinite(p) and p >= 0.0):
        raise ValueError('value must be finite and positive.')
      tree.per_add(remove, add, p, None, 1.0, self._slot(item_id))
    else:
      tree.per_add(remove, add, -1.0, priority, dist.priority_exponent,
                   self._slot(item_id))
    oldest = next(iter(self._order)) if self._order else None
    backend.put(self._slot(item_id), item,
                None if oldest is None else self._slot(oldest))
    self._order[item_id] = None
    self._t += 1

  def get(self, ids: Sequence[int]) -> Iterable[Any]:
    for i in ids:
      if i not in self._order:
        raise KeyError(i)
      yield self._backend.get(self._slot(i))

  def sample_device(self, size: int, out=None):
    """Device sample for the learner: (tree indices, slots, weights), device
    int32 / int32 / f32 [size], drawn with the caller's RandomState in the
    reference's order and resolved on device (dqz_per_sample) — no host
    synchronisation.  `out` may pass preallocated tensors."""
    import torch  # pylint: disable=g-import-not-at-top
    from dqn_mgsc_zoo_amd import _native  # pylint: disable=g-import-not-at-top
    tree = self._device_tree()
    dist = self._distribution
    dev = tree.tree.device
    uniform_idx, u = dist.draw(size)
    inj_i = torch.from_numpy(uniform_idx).pin_memory().to(dev, non_blocking=True)
    inj_u = torch.from_numpy(u).pin_memory().to(dev, non_blocking=True)
    if out is None:
      out = (torch.empty((size,), dtype=torch.int32, device=dev),
             torch.empty((size,), dtype=torch.int32, device=dev),
             torch.empty((size,), dtype=torch.float32, device=dev))
    indices, slots, weights = out
    beta = self.importance_sampling_exponent
    if not 0.0 <= beta <= 1.0:
      raise ValueError('Require 0 <= exponent <= 1.')
    _native.check(_native.lib().dqz_per_sample(
        _native.ptr(tree.tree), tree.capacity, 0, self.size, self._capacity,
        int(size), float(dist.uniform_sample_probability), float(beta),
        int(bool(self._normalize_weights)), 0, None, _native.ptr(inj_i),
        _native.ptr(inj_u), _native.ptr(tree.index_to_slot),
        _native.ptr(indices), _native.ptr(slots), _native.ptr(weights), None,
        _native.stream_handle()))
    return indices, slots, weights

  def write_back(self, learner, indices, max_seen_dev) -> None:
    """|td| of the learner's last step -> max_seen_priority -> priorities of
    the sampled tree indices (prioritized/agent.py:201-206), one launch."""
    from dqn_mgsc_zoo_amd import _native  # pylint: disable=g-import-not-at-top
    tree = self._device_tree()
    self._distribution.note_priorities(None)
    _native.check(_native.lib().dqz_per_write_back(
        learner._h, _native.ptr(tree.tree), tree.capacity, _native.ptr(indices),  # pylint: disable=protected-access
        float(self._distribution.priority_exponent), _native.ptr(max_seen_dev),
        _native.stream_handle()))

  def per_draw(self, size: int, max_seen_dev, out=None):
    """The DqzPerDraw of one learn (Learner.step_per_draw): this replay's
    RandomState draws for sample(size), in the reference's order, injected;
    the step resolves them on device, forms the IS weights and writes the
    priorities back.  Returns (draw, (indices, slots, probs, weights,
    inj_idx, inj_u)) — keep the tensors alive until the step has run.
    None when the batch or tree is past the fused step's limits."""
    import torch  # pylint: disable=g-import-not-at-top
    from dqn_mgsc_zoo_amd import _native  # pylint: disable=g-import-not-at-top
    tree = self._device_tree()
    if size > 64 or tree.capacity > (1 << 24):
      return None
    dist = self._distribution
    beta = self.importance_sampling_exponent
    if not 0.0 <= beta <= 1.0:
      raise ValueError('Require 0 <= exponent <= 1.')
    dev = tree.tree.device
    uniform_idx, u = dist.draw(size)
    inj_i = torch.from_numpy(uniform_idx).pin_memory().to(dev, non_blocking=True)
    inj_u = torch.from_numpy(u).pin_memory().to(dev, non_blocking=True)
    if out is None:
      out = (torch.empty((size,), dtype=torch.int32, device=dev),
             torch.empty((size,), dtype=torch.int32, device=dev),
             torch.empty((size,), dtype=torch.float64, device=dev),
             torch.empty((size,), dtype=torch.float32, device=dev))
    indices, slots, probs, weights = out
    dist.note_priorities(None)  # the write-back may write positive priorities
    p = _native.ptr
    d = _native.DqzPerDraw(
        p(tree.tree).value, tree.capacity, 0, self.size, self._capacity,
        float(dist.uniform_sample_probability), float(beta),
        int(bool(self._normalize_weights)), 0, None, p(inj_i).value,
        p(inj_u).value, p(tree.index_to_slot).value,
        float(dist.priority_exponent), p(max_seen_dev).value,
        p(indices).value, p(slots).value, p(probs).value, p(weights).value)
    return d, (indices, slots, probs, weights, inj_i, inj_u)

  def write_back_args(self, indices, max_seen_dev):
    """The write-back of `indices` as Learner.step(write_back=...) folds it
    into the learner's backward launch (dqz_learner_step_per), or None when
    the batch or the tree is past that path's limits (then call
    write_back after the step)."""
    tree = self._device_tree()
    if indices.numel() > 64 or tree.capacity > (1 << 24):
      return None
    self._distribution.note_priorities(None)
    return (tree.tree, tree.capacity, indices,
            float(self._distribution.priority_exponent), max_seen_dev)

  def sample_ids(self, size: int):
    """(ids, normalised importance weights) as the reference computes them."""
    if self._distribution.on_device:
      indices, _, weights = self.sample_device(size)
      ids = self._distribution.index_to_id(indices.cpu().numpy())
      return ids, weights.cpu().numpy().astype(np.float64)
    ids, probabilities = self._distribution.sample(size)
    weights = importance_sampling_weights(
        probabilities, uniform_probability=1.0 / self.size,
        exponent=self.importance_sampling_exponent,
        normalize=self._normalize_weights)
    return ids, weights

  def sample(self, size: int):
    ids, weights = self.sample_ids(size)
    stacked = self._backend.stack(self._structure, np.asarray(ids) % self._capacity)
    return stacked, ids, weights

  def sample_slots(self, size: int):
    ids, weights = self.sample_ids(size)
    return ids, self._backend.slots_tensor(np.asarray(ids) % self._capacity), weights

  def update_priorities(self, ids: Sequence[int], priorities: Sequence[float]) -> None:
    self._distribution.update_priorities(ids, np.asarray(priorities))

  @property
  def size(self) -> int:
    return len(self._order)

  @property
  def capacity(self) -> int:
    return self._capacity

  @property
  def importance_sampling_exponent(self):
    return self._importance_sampling_exponent(self._t)

  @property
  def distribution(self) -> PrioritizedDistribution:
    return self._distribution

  def get_state(self) -> Mapping[str, Any]:
    return {'storage': list(self._order.keys()), 't': self._t,
            'distribution': self._distribution.get_state(),
            'backend': None if self._backend is None else self._backend.get_state()}

  def set_state(self, state: Mapping[str, Any]) -> None:
    self._order = collections.OrderedDict((i, None) for i in state['storage'])
    self._t = state['t']
    self._distribution.set_state(state['distribution'])
    self._restore_backend(state.get('backend'))
    if self._distribution.on_device:
      self._sync_index_map()
    elif self.on_device:
      self._device_tree()

  def check_valid(self) -> Tuple[bool, str]:
    if self._t < len(self._order):
      return False, 't should be >= storage size.'
    if set(self._order.keys()) != set(self._distribution.ids()):
      return False, 'IDs in storage and distribution do not match.'
    return self._distribution.check_valid()


# ---------------------------------------------------------------------------
# timesteps -> transitions (replay.py:1163-1197)


class TransitionAccumulator:
  """Pairs consecutive timesteps of an episode into 1-step transitions."""

  def __init__(self):
    self.reset()

  def step(self, timestep_t, a_t) -> Iterable[Transition]:
    if timestep_t.first():
      self.reset()
    if self._timestep_tm1 is None:
      if not timestep_t.first():
        raise ValueError('Expected FIRST timestep, got %s.' % str(timestep_t))
      self._timestep_tm1 = timestep_t
      self._a_tm1 = a_t
      return
    transition = Transition(
        s_tm1=self._timestep_tm1.observation, a_tm1=self._a_tm1,
        r_t=timestep_t.reward, discount_t=timestep_t.discount,
        s_t=timestep_t.observation)
    self._timestep_tm1 = timestep_t
    self._a_tm1 = a_t
    yield transition

  def reset(self) -> None:
    self._timestep_tm1 = None
    self._a_tm1 = None
