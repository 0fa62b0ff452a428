"""Shared test fixtures: seeded replay contents and parameter trees."""

import numpy as np

FRAME = 84 * 84


def random_store_contents(capacity, num_frames, num_actions, seed, pad_frac=0.2):
  """Random frame pool + transition table (host numpy).

  Each slot's stacks follow the processor layout: s_t = s_tm1 shifted by one
  frame, with trailing zero padding (-1) at the start of an episode.
  """
  rng = np.random.default_rng(seed)
  frames = rng.integers(0, 256, size=(num_frames, FRAME), dtype=np.uint8)
  fidx = np.empty((capacity, 8), np.int32)
  for i in range(capacity):
    k = int(rng.integers(1, 8))  # in-episode index of s_t
    if rng.random() > pad_frac:
      k = max(k, 4)
    newest = int(rng.integers(0, num_frames))
    def stack(kk, pos):
      n = min(kk, 3)
      ch = [-1] * 4
      for c in range(n + 1):
        ch[c] = (pos - n + c) % num_frames
      return ch
    fidx[i, :4] = stack(k - 1, newest - 1)
    fidx[i, 4:] = stack(k, newest)
  action = rng.integers(0, num_actions, size=capacity).astype(np.int32)
  reward = rng.choice([-1.0, 0.0, 1.0], size=capacity).astype(np.float32)
  discount = (0.99 * (rng.random(capacity) > 0.1)).astype(np.float32)
  return frames, fidx, action, reward, discount


def stacks_from(frames, fidx, slots, which):
  """Host reference of the device gather: uint8 [n,84,84,4]."""
  out = np.zeros((len(slots), 84, 84, 4), np.uint8)
  for b, s in enumerate(slots):
    for c in range(4):
      f = fidx[s, which * 4 + c]
      if f >= 0:
        out[b, :, :, c] = frames[f].reshape(84, 84)
  return out


def perturbed_tree(tree, seed, scale=0.02):
  rng = np.random.default_rng(seed)
  return {m: {n: (v + scale * rng.standard_normal(v.shape)).astype(np.float32)
              for n, v in d.items()} for m, d in tree.items()}


def kink_free_slots(params, host, capacity, batch, rng, margin=1e-6, tries=64):
  """Draws slots (rng.integers, as the tests did before) until the online
  forward on their s_tm1 stacks keeps every ReLU pre-activation at least
  `margin` x its layer's largest |value| away from 0 (oracle relu_margin):
  elementwise gradient / optimizer-state comparisons against fp64 are only
  meaningful away from the kink (seen: a conv2 pre-activation of 7.8e-8 at
  scale 0.54 flipped with a change of f32 summation order and moved the
  conv1 gradient by 2e-3 of its largest entry)."""
  from oracle import learner_ref
  for _ in range(tries):
    slots = rng.integers(0, capacity, size=batch).astype(np.int32)
    s = stacks_from(host['frames'], host['fidx'], slots, 0)
    if learner_ref.relu_margin(params, s) >= margin:
      return slots
  raise AssertionError('no kink-free batch in %d draws' % tries)


def canonical_chunk_sums(t):
  """Restatement of the device's chunk sums (sampling.hpp chunk_sum): per
  chunk of 4096 terms, lane l sums terms [16 l, 16 l + 16) in order, a
  Hillis-Steele scan inside each 64-lane wave, then the last wave's total
  plus the sum of the first three in order."""
  t = np.asarray(t, np.float32).astype(np.float64)
  nb = -(-len(t) // 4096)
  padded = np.zeros(nb * 4096)
  padded[:len(t)] = t
  terms = padded.reshape(nb, 256, 16)
  lane = terms[:, :, 0].copy()
  for i in range(1, 16):
    lane = lane + terms[:, :, i]
  incl = lane.reshape(nb, 4, 64)
  pos = np.arange(64)
  o = 1
  while o < 64:
    up = np.zeros_like(incl)
    up[..., o:] = incl[..., :-o]
    incl = np.where(pos >= o, incl + up, incl)
    o *= 2
  w = incl[..., 63]
  first3 = (w[:, 0] + w[:, 1]) + w[:, 2]
  return w[:, 3] + first3
