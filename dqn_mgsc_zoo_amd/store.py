"""HBM replay storage: a uint8 frame pool plus an SoA transition table.

Replaces the reference's per-transition snappy-compressed host storage
(replay.py:163-206, :1287-1296; replay_circular.py:90-146).  A transition
lives in a *slot*; its two 84x84x4 stacks are described by eight frame
indices into the pool (channels 0..3 = s_tm1, 4..7 = s_t; -1 = the trailing
zero padding of processors.py:57-69), so consecutive transitions share
frames and a stack is assembled on device by the gather fused into conv1.

Layout in HBM (caller-owned torch tensors, borrowed by libdqz):
  frames   uint8 [num_frames][7056]
  fidx     int32 [capacity][8]
  action   int32 [capacity]  reward f32 [capacity]  discount f32 [capacity]
"""

import collections
import ctypes

import numpy as np
import torch

from dqn_mgsc_zoo_amd import _native

FRAME_BYTES = _native.FRAME_BYTES
STACK = _native.STACK


class FrameStore:
  """Device frame pool + transition table (see module docstring)."""

  def __init__(self, capacity, num_frames, device='cuda'):
    if capacity < 1 or num_frames < 1:
      raise ValueError('capacity and num_frames must be positive.')
    self.capacity = int(capacity)
    self.num_frames = int(num_frames)
    self.device = torch.device(device)
    self.frames = torch.zeros((self.num_frames, FRAME_BYTES), dtype=torch.uint8,
                              device=self.device)
    self.fidx = torch.full((self.capacity, 8), -1, dtype=torch.int32,
                           device=self.device)
    self.action = torch.zeros((self.capacity,), dtype=torch.int32,
                              device=self.device)
    self.reward = torch.zeros((self.capacity,), dtype=torch.float32,
                              device=self.device)
    self.discount = torch.zeros((self.capacity,), dtype=torch.float32,
                                device=self.device)
    self._c = _native.DqzStore(
        self.frames.data_ptr(), self.fidx.data_ptr(), self.action.data_ptr(),
        self.reward.data_ptr(), self.discount.data_ptr(), self.capacity,
        self.num_frames)

  @property
  def c_struct(self):
    return self._c

  def c_ref(self):
    return ctypes.byref(self._c)

  def write_frame(self, index, frame):
    """Copies one host [84,84] (or [7056]) uint8 frame into the pool."""
    self.frames[index].copy_(
        torch.from_numpy(np.ascontiguousarray(frame, np.uint8).reshape(-1)))

  def write_transition(self, slot, fidx8, a_tm1, r_t, discount_t):
    self.fidx[slot].copy_(torch.as_tensor(np.asarray(fidx8, np.int32)))
    self.action[slot] = int(a_tm1)
    self.reward[slot] = float(r_t)
    self.discount[slot] = float(discount_t)

  def gather_stacks(self, slots, which, stream=None):
    """uint8 [n,84,84,4] stacks of `which` (0 = s_tm1, 1 = s_t) on device."""
    slots = torch.as_tensor(slots, dtype=torch.int32, device=self.device)
    n = int(slots.numel())
    out = torch.empty((n, 84, 84, STACK), dtype=torch.uint8, device=self.device)
    _native.check(_native.lib().dqz_gather_stacks(
        self.c_ref(), _native.ptr(slots), n, int(which), _native.ptr(out),
        _native.stream_handle(stream)))
    return out


class FrameAllocator:
  """Host-side assignment of pool indices to the channels of added stacks.

  Byte-identical frames are shared between consecutive transitions (the
  overlap of s_tm1 and s_t, and of s_t with the next s_tm1), all-zero
  channels become -1.  Two modes:
    * 'ring': FIFO replays; frames are appended to a ring of `num_frames`.
      A frame may only be overwritten once no live transition references it;
      otherwise `allocate` raises (the pool is too small for the stream).
    * 'slot': reservoir replays; slot i owns pool indices
      [i*per_slot, (i+1)*per_slot) and only shares frames within itself.
  """

  def __init__(self, store, mode, per_slot=8, window=16):
    if mode not in ('ring', 'slot'):
      raise ValueError('mode must be ring or slot')
    self._store = store
    self._mode = mode
    self._per_slot = per_slot
    self._pos = 0  # ring: absolute position of the next frame
    self._recent = collections.OrderedDict()  # key -> absolute position
    self._window = window
    self._min_ref = {}  # slot -> oldest absolute frame position referenced

  def allocate(self, slot, s_tm1, s_t, oldest_live_slot=None):
    """Writes the unique frames of the two stacks; returns 8 pool indices."""
    channels = [s_tm1[..., c] for c in range(STACK)] + [
        s_t[..., c] for c in range(STACK)]
    if self._mode == 'slot':
      return self._allocate_slot(slot, channels)
    out = []
    refs = []
    for ch in channels:
      if not ch.any():
        out.append(-1)
        continue
      raw = ch.tobytes()
      key = hash(raw)
      hit = self._recent.get(key)
      if (hit is not None and hit[1] == raw and
          self._pos - hit[0] <= self._store.num_frames):
        pos = hit[0]
        self._recent.move_to_end(key)
      else:
        pos = self._append(ch, oldest_live_slot)
        self._recent[key] = (pos, raw)
        while len(self._recent) > self._window:
          self._recent.popitem(last=False)
      refs.append(pos)
      out.append(pos % self._store.num_frames)
    self._min_ref[slot] = min(refs) if refs else self._pos
    return out

  def _append(self, ch, oldest_live_slot):
    pos = self._pos
    victim = pos - self._store.num_frames
    if victim >= 0 and oldest_live_slot is not None:
      if self._min_ref.get(oldest_live_slot, victim + 1) <= victim:
        raise RuntimeError(
            'Frame pool of %d frames is too small for this transition stream: '
            'overwriting frame %d still referenced by a live transition. '
            'Increase num_frames.' % (self._store.num_frames, victim))
    self._store.write_frame(pos % self._store.num_frames, ch)
    self._pos += 1
    return pos

  def _allocate_slot(self, slot, channels):
    base = slot * self._per_slot
    seen = {}
    out = []
    used = 0
    for ch in channels:
      if not ch.any():
        out.append(-1)
        continue
      key = ch.tobytes()
      if key not in seen:
        if used == self._per_slot:
          raise RuntimeError(
              'transition has more than %d distinct frames; construct the '
              'replay with frames_per_slot=8.' % self._per_slot)
        self._store.write_frame(base + used, ch)
        seen[key] = base + used
        used += 1
      out.append(seen[key])
    return out

  def forget(self, slot):
    self._min_ref.pop(slot, None)

  def get_state(self):
    return {'mode': self._mode, 'per_slot': self._per_slot, 'pos': self._pos,
            'recent': list(self._recent.items()),
            'min_ref': dict(self._min_ref)}

  def set_state(self, state):
    self._mode = state['mode']
    self._per_slot = state['per_slot']
    self._pos = state['pos']
    self._recent = collections.OrderedDict(state['recent'])
    self._min_ref = dict(state['min_ref'])
