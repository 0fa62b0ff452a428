"""ORACLE — test infrastructure only.  Never imported by the product.

CPU restatement of the replay-side arithmetic that libdqz implements on
device, written independently of the product's host bookkeeping
(dqn_mgsc_zoo_amd/replay.py) so the two check each other.  Pinned against
the reference itself through tests/golden/replay_golden.json
(tests/golden/make_golden.py runs the reference's replay.py /
replay_circular.py in the build container).

  * SumTree query = first index whose inclusive prefix sum exceeds the
    target (replay.py:432-446, :539-559), here as a naive cumulative sum
    (the reference's own NaiveSumTree idea, replay_test.py:1048-1120).
  * logits_logmeanexp: the default logit of CircularLogitBuffer.add /
    MGSCReservoirDistribution.add / .replace (replay_circular.py:166-179,
    :518-533): logsumexp(all capacity slots, -inf for empty) - log(size),
    float32 like the reference's numpy call on a float32 array.
  * softmax_choice: Generator.choice(C, n, p=softmax(logits)) given the
    uniforms the Generator would draw (replay_circular.py:205-217): numpy
    forms cdf = cumsum(float64(p)), cdf /= cdf[-1], idx =
    searchsorted(cdf, u, side='right').
  * per_sample: PrioritizedDistribution.sample given its three random
    streams (replay.py:680-716).
"""

import numpy as np


class SumTree:
  """Naive restatement: values array, prefix-sum queries."""

  def __init__(self):
    self._values = np.zeros(0, np.float64)
    self._capacity = 0

  def resize(self, size):
    v = np.zeros(size, np.float64)
    n = min(size, len(self._values))
    v[:n] = self._values[:n]
    self._values = v
    cap = 1 if size > 0 else 0
    while cap < size:
      cap *= 2
    self._capacity = max(self._capacity, cap)

  def set(self, indices, values):
    values = np.asarray(values, np.float64)
    if not np.isfinite(values).all() or (values < 0).any():
      raise ValueError('value must be finite and positive.')
    self._values[np.asarray(indices)] = values

  def set_all(self, values):
    values = np.asarray(values, np.float64)
    self._values = np.zeros(0)
    self.resize(len(values))
    self._values[:] = values

  def root(self):
    return float(self._values.sum()) if len(self._values) else np.nan

  def query(self, targets):
    cum = np.cumsum(self._values)
    out = []
    for t in targets:
      if not 0.0 <= t < cum[-1]:
        raise ValueError('Require 0 <= target < total sum.')
      out.append(int(np.searchsorted(cum, t, side='right')))
    return out

  def check_valid(self):
    return True, ''

  @property
  def values(self):
    return self._values

  @property
  def capacity(self):
    return self._capacity


def logsumexp_f32(x):
  x = np.asarray(x, np.float32)
  c = x.max()
  return np.float32(c + np.log(np.sum(np.exp(x - c))))


def logits_logmeanexp(logits, size):
  """Default logit of a new item: 0 for an empty buffer."""
  if size == 0:
    return np.float32(0.0)
  return np.float32(logsumexp_f32(logits) - np.log(size))


def softmax_f32(logits):
  logits = np.asarray(logits, np.float32)
  return np.exp(logits - logsumexp_f32(logits))


def softmax_choice(logits, uniforms):
  p = softmax_f32(logits).astype(np.float64)
  cdf = np.cumsum(p)
  cdf /= cdf[-1]
  return np.searchsorted(cdf, np.asarray(uniforms, np.float64), side='right')


def per_sample(leaves, active, rand_idx, u_target, u_mix, usp):
  """Prioritized sampling given its random draws.

  leaves: exponentiated priorities by tree index; active: active tree
  indices (sampling order); rand_idx: randint draws into `active`;
  u_target / u_mix: uniform draws.  Returns (tree indices, probabilities).
  """
  leaves = np.asarray(leaves, np.float64)
  root = leaves.sum()
  uni = np.asarray([active[j] for j in rand_idx])
  if root == 0.0:
    pri = uni
  else:
    cum = np.cumsum(leaves)
    pri = np.searchsorted(cum, np.asarray(u_target) * root, side='right')
  idx = np.where(np.asarray(u_mix) < usp, uni, pri)
  n = len(active)
  pp = np.full(len(idx), 1.0 / n) if root == 0.0 else leaves[idx] / root
  return idx, (1.0 - usp) * pp + usp / n


def algorithm_r(n_items, capacity, draws):
  """Reservoir slot contents after n_items adds; draws[t] = randint(0, t)."""
  slots = []
  it = iter(draws)
  for t in range(n_items):
    if len(slots) < capacity:
      slots.append(t)
    else:
      j = next(it)
      if j < capacity:
        slots[j] = t
  return slots
