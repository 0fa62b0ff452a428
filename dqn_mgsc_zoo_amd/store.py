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
import xxhash

from dqn_mgsc_zoo_amd import _native

FRAME_BYTES = _native.FRAME_BYTES
STACK = _native.STACK
_STAGE_SLOTS = 64


class Uploader:
  """Host -> device copies that do not wait for the device.

  A pageable `tensor.copy_(host)` blocks the host until every launch queued
  before it has finished (in the MGSC agent: the whole meta-update before
  the learn step's 32 uniforms).  Here the host array is written into one of
  a ring of pinned staging buffers and copied with non_blocking=True on the
  current stream; a buffer is reused once the copy that read it has
  completed (one event per buffer), so a call returns at once."""

  def __init__(self, nbytes, slots=8):
    self.nbytes = int(nbytes)
    self._buf = torch.empty((slots, self.nbytes), dtype=torch.uint8, pin_memory=True)
    self._np = self._buf.numpy()
    self._ev = [None] * slots
    self._k = 0

  def __call__(self, dst, array):
    """dst (contiguous device tensor) <- array (same itemsize, dst.numel() items)."""
    a = np.ascontiguousarray(array)
    n = a.nbytes
    if (n > self.nbytes or not dst.is_contiguous() or a.dtype.itemsize != dst.element_size()
        or dst.numel() * dst.element_size() != n):
      raise ValueError('upload of %s %s into %s %s' % (a.dtype, a.shape, dst.dtype, tuple(dst.shape)))
    k = self._k
    self._k = (k + 1) % len(self._ev)
    if self._ev[k] is not None:
      self._ev[k].synchronize()
    self._np[k, :n] = a.view(np.uint8).reshape(-1)
    dst.view(-1).view(torch.uint8).copy_(self._buf[k, :n], non_blocking=True)
    if self._ev[k] is None:
      self._ev[k] = torch.cuda.Event()
    self._ev[k].record()
    return dst


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
    self._stage = None  # pinned staging slots of put(), allocated on first use
    self._stage_k = 0
    self._c = _native.DqzStore(
        self.frames.data_ptr(), self.fidx.data_ptr(), self.action.data_ptr(),
        self.reward.data_ptr(), self.discount.data_ptr(), self.capacity,
        self.num_frames)

  @property
  def c_struct(self):
    return self._c

  def c_ref(self):
    return ctypes.byref(self._c)

  def put(self, slot, fidx8, a_tm1, r_t, discount_t, new_frames=()):
    """One replay add in one launch (dqz_store_put): the new frames
    [(pool row, host [84,84] uint8), ...] go through a pinned staging slot
    that the kernel reads in place, then the record {fidx, a, r, d}.

    Staging slots are reused round-robin once the launch that read them has
    completed (one event per slot), so calls return without waiting."""
    if self._stage is None:
      self._stage = torch.empty((_STAGE_SLOTS, 8, FRAME_BYTES), dtype=torch.uint8,
                                pin_memory=True)
      self._stage_np = self._stage.numpy()
      self._stage_ev = [None] * _STAGE_SLOTS
    k = self._stage_k
    self._stage_k = (k + 1) % _STAGE_SLOTS
    if self._stage_ev[k] is not None:
      self._stage_ev[k].synchronize()
    t = _native.DqzTransitionPut()
    t.slot = int(slot)
    for i, f in enumerate(fidx8):
      t.fidx[i] = int(f)
    t.action = int(a_tm1)
    t.reward = float(r_t)
    t.discount = float(discount_t)
    t.num_frames = len(new_frames)
    for i, (row, frame) in enumerate(new_frames):
      self._stage_np[k, i] = np.asarray(frame, np.uint8).reshape(-1)
      t.frame_rows[i] = int(row)
    _native.check(_native.lib().dqz_store_put(
        self.c_ref(), ctypes.byref(t),
        ctypes.c_void_p(self._stage[k].data_ptr()), _native.stream_handle()))
    if self._stage_ev[k] is None:
      self._stage_ev[k] = torch.cuda.Event()
    self._stage_ev[k].record()

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

  Ring mode takes two byte-exact shortcuts before hashing a channel: the
  accumulator hands the previous transition's s_t object back as the next
  s_tm1 (replay.py:1183-1191), whose channels are then already placed; and
  the frame stack shifts by one frame per step (processors.py:497-504), so
  s_t channels 0..2 equal s_tm1 channels 1..3 whenever one vectorised
  compare of the two stacks' 32-bit pixels says so.  Every other channel is
  fingerprinted (xxh3 of the contiguous plane) against a window of recent
  frames and byte-compared before it is shared.
  """

  def __init__(self, store, mode, per_slot=8, window=16):
    if mode not in ('ring', 'slot'):
      raise ValueError('mode must be ring or slot')
    self._store = store
    self._mode = mode
    self._per_slot = per_slot
    self._pos = 0  # ring: absolute position of the next frame
    self._recent = collections.OrderedDict()  # fingerprint -> (absolute position, plane)
    self._window = window
    self._min_ref = {}  # slot -> oldest absolute frame position referenced
    self._new = []  # frames of the current allocate() still to be written
    self._prev = None  # (last s_t object, its 4 absolute positions / -1)

  def allocate(self, slot, s_tm1, s_t, oldest_live_slot=None):
    """Assigns pool rows to the channels of the two stacks.

    Returns (8 pool indices, [(pool row, frame plane), ...] of the frames
    that are new and still have to be written, in order)."""
    self._new = []
    if self._mode == 'slot':
      return self._allocate_slot(slot, s_tm1, s_t), self._new
    nf = self._store.num_frames
    prev = self._prev
    if (prev is not None and prev[0] is s_tm1 and
        all(p < 0 or self._pos - p <= nf for p in prev[1])):
      first = list(prev[1])
    else:
      first = [self._place(s_tm1, c, oldest_live_slot) for c in range(STACK)]
    second = [None] * STACK
    if (s_tm1.flags.c_contiguous and s_t.flags.c_contiguous and
        s_tm1.shape == (84, 84, STACK) and s_t.shape == (84, 84, STACK)):
      u_tm1 = s_tm1.view(np.uint32).reshape(-1)
      u_t = s_t.view(np.uint32).reshape(-1)
      if np.array_equal(u_t & np.uint32(0x00FFFFFF), u_tm1 >> np.uint32(8)):
        second[:STACK - 1] = first[1:]
    for c in range(STACK):
      if second[c] is None:
        second[c] = self._place(s_t, c, oldest_live_slot)
    self._prev = (s_t, second)
    positions = first + second
    refs = [p for p in positions if p >= 0]
    self._min_ref[slot] = min(refs) if refs else self._pos
    return [p % nf if p >= 0 else -1 for p in positions], self._new

  def _place(self, stack, c, oldest_live_slot):
    """Absolute pool position of channel c of `stack` (-1: all zero)."""
    ch = np.ascontiguousarray(stack[..., c]).reshape(-1)
    if not ch.any():
      return -1
    key = xxhash.xxh3_64_intdigest(ch)
    hit = self._recent.get(key)
    if (hit is not None and self._pos - hit[0] <= self._store.num_frames and
        np.array_equal(hit[1], ch)):
      self._recent.move_to_end(key)
      return hit[0]
    pos = self._append(ch, oldest_live_slot)
    self._recent[key] = (pos, ch)
    while len(self._recent) > self._window:
      self._recent.popitem(last=False)
    return pos

  def _append(self, ch, oldest_live_slot):
    pos = self._pos
    victim = pos - self._store.num_frames
    if victim >= 0 and oldest_live_slot is not None:
      if self._min_ref.get(oldest_live_slot, victim + 1) <= victim:
        raise RuntimeError(
            'Frame pool of %d frames is too small for this transition stream: '
            'overwriting frame %d still referenced by a live transition. '
            'Increase num_frames.' % (self._store.num_frames, victim))
    self._new.append((pos % self._store.num_frames, ch))
    self._pos += 1
    return pos

  def _allocate_slot(self, slot, s_tm1, s_t):
    base = slot * self._per_slot
    seen = {}
    out = []
    used = 0
    for stack in (s_tm1, s_t):
      for c in range(STACK):
        ch = np.ascontiguousarray(stack[..., c]).reshape(-1)
        if not ch.any():
          out.append(-1)
          continue
        key = ch.tobytes()
        if key not in seen:
          if used == self._per_slot:
            raise RuntimeError(
                'transition has more than %d distinct frames; construct the '
                'replay with frames_per_slot=8.' % self._per_slot)
          self._new.append((base + used, ch))
          seen[key] = base + used
          used += 1
        out.append(seen[key])
    return out

  def forget(self, slot):
    self._min_ref.pop(slot, None)

  def get_state(self):
    return {'mode': self._mode, 'per_slot': self._per_slot, 'pos': self._pos,
            'recent': [(k, (p, ch.tobytes())) for k, (p, ch) in self._recent.items()],
            'min_ref': dict(self._min_ref)}

  def set_state(self, state):
    self._mode = state['mode']
    self._per_slot = state['per_slot']
    self._pos = state['pos']
    self._recent = collections.OrderedDict(
        (k, (p, np.frombuffer(raw, np.uint8))) for k, (p, raw) in state['recent'])
    self._min_ref = dict(state['min_ref'])
    self._prev = None
