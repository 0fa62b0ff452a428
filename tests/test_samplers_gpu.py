"""GPU: device samplers vs the reference's golden vectors and the oracle.

* learned-logit buffers (replay_circular.py): logits after add / popleft /
  replace / setitem within 1e-6 (f32 log-sum-exp summation order differs);
  softmax-sampled indices bit-exact given the Generator's own uniforms;
  the exact mode's p bit for bit numpy's probabilities_from_logits and its
  draws Generator.choice's at up to 1M slots.
* fp64 sum tree: device storage bit-identical to the host SumTree after the
  same set() calls; device queries identical to host queries.
* device PER sampler: frequencies vs (1-usp) p^a/sum + usp/N (rtol as the
  reference's statistical test), weights = (1/N / prob)^beta / max; with the
  reference RandomState's draws injected, ids and probabilities equal the
  reference's golden vectors index for index (distribution level) and the
  device-resident prioritized replay reproduces the golden replay log (ids,
  stored items, importance weights) through add / sample / update.
"""

import ctypes
import json
import os

import numpy as np
import pytest
import torch

from oracle import replay_ref
from tests import helpers

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), 'golden',
                                     'replay_golden.json')))


def _frame_item(i, rng):
  s = rng.integers(0, 256, (84, 84, 4), dtype=np.uint8)
  from dqn_mgsc_zoo_amd import replay as replay_lib
  return replay_lib.Transition(s, i % 6, float(i), 0.99, s)


def _logits_match(got, want, exact):
  """Default mode: the running log-sum-exp sums in another order (1e-6);
  exact mode: the reference's float32 logsumexp, so the same bits."""
  if exact:
    np.testing.assert_array_equal(np.asarray(got, np.float32), np.asarray(want, np.float32))
  else:
    np.testing.assert_allclose(got, want, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize('exact', [False, True])
def test_circular_logit_buffer_golden(device, exact):
  from dqn_mgsc_zoo_amd import replay_circular as rc
  g = GOLDEN['circular']['logit_buffer']
  b = rc.CircularLogitBuffer(g['capacity'], np.random.default_rng(g['seed']), exact_sampling=exact)
  for op in g['ops']:
    if op[0] == 'add':
      b.add(op[1])
    elif op[0] == 'popleft':
      b.popleft()
    else:
      b[np.array(op[1][0])] = np.array(op[1][1], np.float32)
    _logits_match(b.logits.cpu().numpy(), op[2], exact)
  assert b._left_head == g['left_head']  # pylint: disable=protected-access
  if exact:  # as_probs = probabilities_from_logits, bit for bit
    want = replay_ref.softmax_f32(b.logits.cpu().numpy())
    assert (b.as_probs().cpu().numpy().view(np.uint32) == want.view(np.uint32)).all()
  assert b.sample(5).tolist() == g['sample']
  assert b.sample_uniform(4, replace=False).tolist() == g['sample_uniform']


@pytest.mark.parametrize('exact', [False, True])
def test_mgsc_fifo_replay_golden(device, exact):
  from dqn_mgsc_zoo_amd import replay_circular as rc
  g = GOLDEN['circular']['mgsc_fifo']
  r = rc.MGSCFiFoTransitionReplay(g['capacity'], rc.Transition(None, None, None, None, None),
                                  np.random.default_rng(g['seed']), exact_sampling=exact)
  for i in range(g['n_add']):
    r.add(rc.Transition(i, 0, 0.0, 1.0, i))
  assert r.sample(5).s_tm1.tolist() == g['sample_items']
  ind, tr, lg = r.batch_of_ids_transitions_and_logits(3)
  assert ind.tolist() == g['meta_indices']
  assert tr.s_tm1.tolist() == g['meta_items']
  _logits_match(lg, g['meta_logits'], exact)
  r.update_priorities(ind, np.array([0.5, -0.25, 1.0], np.float32))
  assert r.sample(4).s_tm1.tolist() == g['sample2_items']
  _logits_match(r.logits.cpu().numpy(), g['logits'], exact)


@pytest.mark.parametrize('exact', [False, True])
def test_mgsc_reservoir_replay_golden(device, exact):
  from dqn_mgsc_zoo_amd import replay_circular as rc
  g = GOLDEN['circular']['mgsc_reservoir']
  r = rc.MGSCReservoirTransitionReplay(g['capacity'], rc.Transition(None, None, None, None, None),
                                       np.random.default_rng(g['seed']), exact_sampling=exact)
  for i in range(g['n_add']):
    r.add(rc.Transition(i, 0, 0.0, 1.0, i))
  _logits_match(r.logits.cpu().numpy(), g['logits_after_adds'], exact)
  items = [int(x.s_tm1[0]) for x in r.get(range(g['capacity']))]
  assert items == g['slot_items']
  assert r.sample(5).s_tm1.tolist() == g['sample_items']
  ind, _, lg = r.batch_of_ids_transitions_and_logits(3)
  assert ind.tolist() == g['meta_indices']
  _logits_match(lg, g['meta_logits'], exact)
  r.update_priorities(ind, np.array([1.0, 0.0, -2.0], np.float32))
  assert r.sample(5).s_tm1.tolist() == g['sample2_items']
  _logits_match(r.logits.cpu().numpy(), g['logits'], exact)


def _choice_from_p(p, u):
  """numpy's choice given p (replay_circular.py:205-217): sequential float64
  cumsum, normalised by its last entry, searchsorted side='right'."""
  cdf = np.cumsum(np.asarray(p, np.float32).astype(np.float64))
  cdf /= cdf[-1]
  return np.searchsorted(cdf, np.asarray(u, np.float64), side='right')


def _check_chunk_sums(dev):
  """The buffer's chunk sums are exactly the canonical sums of its terms
  expf(x - c), and those terms are numpy's expf(x - c) to the last ulp."""
  t, csum, c = dev.terms()
  t = t.cpu().numpy()
  x = dev.logits.cpu().numpy()
  np.testing.assert_array_equal(csum.cpu().numpy(), helpers.canonical_chunk_sums(t))
  want = np.exp(x - np.float32(c.item()))
  assert _ulps(t, want).max() <= 4
  return t


def _ulps(a, b):
  a = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
  b = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
  return np.abs(a - b)


def test_softmax_choice_large_capacity(device):
  """1M logits (the MGSC capacity).

  Index work is bit-exact: given the terms expf(x - c) the device forms, its
  choice equals numpy's sequential-cumsum choice for every query, and the
  chunk sums it searches are the canonical sums of those terms.  The only
  gap to the numpy reference is in p itself (f32 rounding of the exponent
  about c instead of lse, and exp's last ulps), bounded below; a query can
  land on a different slot only when such an ulp moves a CDF boundary
  across it.
  """
  from dqn_mgsc_zoo_amd import replay_circular as rc
  cap = 1_000_000
  rng = np.random.default_rng(0)
  logits = rng.standard_normal(cap).astype(np.float32)
  logits[rng.integers(0, cap, 1000)] = -np.inf  # empty slots
  dev = rc._DeviceLogits(cap)  # pylint: disable=protected-access
  dev.logits.copy_(torch.from_numpy(logits))
  u = np.random.default_rng(5).random(512)
  got = dev.sample_abs(u).cpu().numpy()
  t_dev = _check_chunk_sums(dev)
  np.testing.assert_array_equal(got, _choice_from_p(t_dev, u))
  p_dev, lse_dev = dev.probs()
  p_dev = p_dev.cpu().numpy()
  # the gap in p to numpy (replay_ref.softmax_f32 = probabilities_from_logits)
  p_np = replay_ref.softmax_f32(logits)
  live = np.isfinite(logits)
  assert (p_dev[~live] == 0).all()
  assert _ulps(p_dev[live], p_np[live]).max() <= 64, _ulps(p_dev[live], p_np[live]).max()
  assert abs(float(lse_dev.item()) - float(replay_ref.logsumexp_f32(logits))) <= 4e-6
  want = replay_ref.softmax_choice(logits, u)
  assert (got != want).sum() <= 1
  # log-mean-exp default logit over the full capacity
  dev.add_default(write_pos=7, size=cap - 1000, clear_pos=7)
  lg = logits.copy()
  lg[7] = -np.inf
  ref = replay_ref.logits_logmeanexp(lg, cap - 1000)
  np.testing.assert_allclose(dev.logits[7].item(), ref, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize('cap', [1000, 8193, 100_003, 1_000_000])
def test_exact_mode_is_the_reference_draw(device, cap):
  """dqz_logits_sample_exact: p is numpy's probabilities_from_logits bit for
  bit (replay_ref.softmax_f32 calls numpy on this host), and every draw is
  Generator.choice's for the same uniforms (replay_ref.softmax_choice).  The
  restatement the device follows (oracle/numpy_f32.py) is checked against
  this host's numpy too, so a failure says which side moved."""
  from oracle import numpy_f32
  from dqn_mgsc_zoo_amd import replay_circular as rc
  rng = np.random.default_rng(cap)
  logits = (rng.standard_normal(cap) * 2).astype(np.float32)
  logits[rng.integers(0, cap, max(1, cap // 1000))] = -np.inf  # empty slots
  p_np = replay_ref.softmax_f32(logits)
  assert (numpy_f32.probabilities_f32(logits).view(np.uint32) == p_np.view(np.uint32)).all()
  dev = rc._DeviceLogits(cap, max_queries=1024)  # pylint: disable=protected-access
  dev.logits.copy_(torch.from_numpy(logits))
  u = np.random.default_rng(cap + 1).random(1024)
  got, p_dev = dev.sample_exact(u, probs=True)
  p_dev = p_dev.cpu().numpy()
  bad = int((p_dev.view(np.uint32) != p_np.view(np.uint32)).sum())
  assert bad == 0, (bad, _ulps(p_dev, p_np).max())
  np.testing.assert_array_equal(got.cpu().numpy(), replay_ref.softmax_choice(logits, u))


def test_exact_add_at_full_size(device):
  """dqz_logits_add_exact at 1M slots: the default logit of an add and of a
  reservoir replace (clear, then log-mean-exp over the full capacity) equal
  the reference's logsumexp(logits) - np.log(size) as stored float32."""
  from dqn_mgsc_zoo_amd import replay_circular as rc
  cap = 1_000_000
  rng = np.random.default_rng(21)
  logits = (rng.standard_normal(cap) * 1.5).astype(np.float32)
  logits[rng.integers(0, cap, 2000)] = -np.inf
  dev = rc._DeviceLogits(cap)  # pylint: disable=protected-access
  dev.logits.copy_(torch.from_numpy(logits))
  for pos, size, clear in ((17, cap - 3000, -1), (123_456, cap, 123_456), (999_999, 5, -1)):
    lg = dev.logits.cpu().numpy().copy()
    if clear >= 0:
      lg[clear] = -np.inf
    want = np.float32(replay_ref.logsumexp_f32(lg) - np.log(size))
    dev.add_default_exact(pos, size, clear_pos=clear)
    got = dev.logits[pos].item()
    assert np.float32(got).view(np.uint32) == want.view(np.uint32), (pos, got, want)
  dev.add_default_exact(3, 0)
  assert dev.logits[3].item() == 0.0


def test_exact_mode_wide_and_tied_logits(device):
  """Exact mode on logits spanning the float32 exp range (terms down to
  denormals and underflow) and on ties (every logit equal: numpy's uniform
  p, draws = floor(u C) up to float64 cumsum rounding at the steps)."""
  from dqn_mgsc_zoo_amd import replay_circular as rc
  cap = 300_000
  rng = np.random.default_rng(11)
  logits = rng.uniform(-110.0, 0.0, cap).astype(np.float32)
  logits[rng.integers(0, cap, 100)] = -np.inf
  dev = rc._DeviceLogits(cap, max_queries=512)  # pylint: disable=protected-access
  dev.logits.copy_(torch.from_numpy(logits))
  u = np.random.default_rng(12).random(512)
  got, p_dev = dev.sample_exact(u, probs=True)
  p_np = replay_ref.softmax_f32(logits)
  assert (p_dev.cpu().numpy().view(np.uint32) == p_np.view(np.uint32)).all()
  assert (p_np == 0).sum() > 0 and ((p_np > 0) & (p_np < np.finfo(np.float32).tiny)).sum() > 0
  np.testing.assert_array_equal(got.cpu().numpy(), replay_ref.softmax_choice(logits, u))
  flat = np.zeros(cap, np.float32)
  dev.logits.copy_(torch.from_numpy(flat))
  got, p_dev = dev.sample_exact(u, probs=True)
  assert (p_dev.cpu().numpy().view(np.uint32) == replay_ref.softmax_f32(flat).view(np.uint32)).all()
  np.testing.assert_array_equal(got.cpu().numpy(), replay_ref.softmax_choice(flat, u))


def test_softmax_choice_wide_logits(device):
  """Logits spanning ~90 nats: most p are far below ulp(total), so numpy's
  sequential cumsum rounds many adds that the device's blocked sums round
  differently; those differences are ulps of the total, far below the CDF
  gaps the draws land in, so every draw still matches numpy's given the
  same p."""
  from dqn_mgsc_zoo_amd import replay_circular as rc
  cap = 200_000
  rng = np.random.default_rng(3)
  logits = rng.uniform(-90.0, 0.0, cap).astype(np.float32)
  logits[rng.integers(0, cap, 50)] = -np.inf
  dev = rc._DeviceLogits(cap, max_queries=512)  # pylint: disable=protected-access
  dev.logits.copy_(torch.from_numpy(logits))
  u = np.random.default_rng(9).random(512)
  got = dev.sample_abs(u).cpu().numpy()
  p_dev = _check_chunk_sums(dev)
  nz = p_dev[p_dev > 0]
  total = np.float64(nz.astype(np.float64).sum())
  assert np.frexp(nz)[1].min() - 24 < np.frexp(total)[1] - 53  # numpy's cumsum does round here
  np.testing.assert_array_equal(got, _choice_from_p(p_dev, u))


def _tree_dev(tree):
  return torch.from_numpy(tree.storage.copy()).to('cuda')


def test_sumtree_device_set_and_query(device):
  from dqn_mgsc_zoo_amd import _native
  from dqn_mgsc_zoo_amd import replay as replay_lib
  lib = _native.lib()
  rng = np.random.default_rng(3)
  for size in (1, 3, 37, 1000, 4096 + 17):
    host = replay_lib.SumTree()
    host.set_all(np.abs(rng.standard_cauchy(size)))
    dev = _tree_dev(host)
    cap = host.capacity
    for _ in range(5):
      idx = rng.integers(0, size, 64)
      vals = np.abs(rng.standard_cauchy(64))
      vals[::7] = 0.0
      # the reference sets leaves in order; duplicates keep the last value
      host.set(idx, vals)
      last = {}
      for i, v in zip(idx, vals):
        last[int(i)] = v
      di = torch.tensor(list(last.keys()), dtype=torch.int64, device=device)
      dv = torch.tensor(list(last.values()), dtype=torch.float64, device=device)
      _native.check(lib.dqz_sumtree_set(_native.ptr(dev), cap, _native.ptr(di),
                                        _native.ptr(dv), len(last),
                                        _native.stream_handle()))
      np.testing.assert_array_equal(dev.cpu().numpy()[1:], host.storage[1:])
      if host.root() == 0.0:
        continue
      targets = rng.uniform(0, host.root(), 257)
      targets[0] = 0.0
      dt = torch.from_numpy(targets).to(device)
      out = torch.empty(257, dtype=torch.int64, device=device)
      _native.check(lib.dqz_sumtree_query(_native.ptr(dev), cap, _native.ptr(dt),
                                          257, _native.ptr(out),
                                          _native.stream_handle()))
      assert out.cpu().numpy().tolist() == list(host.query(targets))
  # out of range targets -> -1
  bad = torch.tensor([-1.0, host.root(), host.root() + 1], dtype=torch.float64,
                     device=device)
  out = torch.empty(3, dtype=torch.int64, device=device)
  _native.check(lib.dqz_sumtree_query(_native.ptr(dev), cap, _native.ptr(bad),
                                      3, _native.ptr(out), _native.stream_handle()))
  assert out.cpu().numpy().tolist() == [-1, -1, -1]


def test_per_device_sampler_distribution(device):
  from dqn_mgsc_zoo_amd import _native
  from dqn_mgsc_zoo_amd import replay as replay_lib
  lib = _native.lib()
  cap, alpha, usp, beta = 8, 0.8, 0.1, 0.4
  prios = np.array([1.0, 0.0, 3.0, 4.0, 0.5, 2.0, 0.0, 1.5])
  host = replay_lib.SumTree()
  host.resize(cap)
  host.set(np.arange(cap), replay_lib._power(prios, alpha))  # pylint: disable=protected-access
  dev = _tree_dev(host)
  counter = torch.zeros(1, dtype=torch.int64, device=device)
  n = 1000
  slots = torch.empty(n, dtype=torch.int32, device=device)
  w = torch.empty(n, dtype=torch.float32, device=device)
  probs = torch.empty(n, dtype=torch.float64, device=device)
  counts = np.zeros(cap)
  for _ in range(60):
    _native.check(lib.dqz_per_sample(
        _native.ptr(dev), cap, 0, cap, cap, n, usp, beta, 1, 77,
        _native.ptr(counter), None, None, None, None, _native.ptr(slots), _native.ptr(w),
        _native.ptr(probs), _native.stream_handle()))
    s = slots.cpu().numpy()
    counts += np.bincount(s, minlength=cap)
  p = replay_lib._power(prios, alpha)  # pylint: disable=protected-access
  expected = (1 - usp) * p / p.sum() + usp / cap
  np.testing.assert_allclose(counts / counts.sum(), expected, rtol=2e-2,
                             atol=2e-4)
  s = slots.cpu().numpy()
  np.testing.assert_allclose(probs.cpu().numpy(), expected[s], rtol=1e-12)
  want_w = replay_lib.importance_sampling_weights(expected[s], 1.0 / cap, beta, True)
  np.testing.assert_allclose(w.cpu().numpy(), want_w, rtol=1e-6)


def test_sumtree_query_large_tree_boundaries(device):
  """2^20-leaf tree (PER at capacity 1e6): the half-wave four-level descent
  returns the serial descent's leaf for random targets and for targets that
  sit exactly on left-subtree sums (where the compare flips)."""
  from dqn_mgsc_zoo_amd import _native
  from dqn_mgsc_zoo_amd import replay as replay_lib
  lib = _native.lib()
  rng = np.random.default_rng(11)
  host = replay_lib.SumTree()
  prios = rng.random(1_000_000) ** 3
  prios[rng.integers(0, prios.size, 5000)] = 0.0
  host.set_all(prios)
  dev = _tree_dev(host)
  st = host.storage
  targets = list(rng.uniform(0, host.root(), 300))
  # exact boundaries: cumulative sums along a few random root-to-leaf paths
  for _ in range(20):
    node, acc = 1, 0.0
    while node < host.capacity:
      targets.append(acc + st[2 * node])  # == left sum: must go right
      if rng.random() < 0.5:
        node = 2 * node
      else:
        acc += st[2 * node]
        node = 2 * node + 1
  targets = np.array([t for t in targets if 0.0 <= t < host.root()])
  dt = torch.from_numpy(targets).to(device)
  out = torch.empty(targets.size, dtype=torch.int64, device=device)
  _native.check(lib.dqz_sumtree_query(_native.ptr(dev), host.capacity,
                                      _native.ptr(dt), targets.size,
                                      _native.ptr(out), _native.stream_handle()))
  assert out.cpu().numpy().tolist() == list(host.query(targets))


def test_per_device_sampler_injected_matches_golden_distribution(device):
  """PrioritizedDistribution.sample (replay.py:680-716) on device, fed the
  reference RandomState(3)'s own draws: ids and probabilities bit-equal to
  the goldens recorded from the reference."""
  from dqn_mgsc_zoo_amd import _native
  from dqn_mgsc_zoo_amd import replay as replay_lib
  g = GOLDEN['prioritized']['distribution']
  rs = np.random.RandomState(g['seed'])
  d = replay_lib.PrioritizedDistribution(g['exponent'], g['usp'], rs, 0, None)
  for op, ids, prios in [o + [None] * (3 - len(o)) for o in g['ops']]:
    if op == 'add':
      d.add_priorities(ids, prios)
    elif op == 'update':
      d.update_priorities(ids, prios)
    else:
      d.remove_priorities(ids)
  n = len(g['ids'])
  host_tree = d.sum_tree
  d.to_device(device)
  tree = d.sum_tree
  assert np.array_equal(tree.storage[1:2 * host_tree.capacity],
                        host_tree.storage[1:])
  uniform_idx, u = d.draw(n)
  inj_i = torch.from_numpy(uniform_idx).to(device)
  inj_u = torch.from_numpy(u).to(device)
  idx = torch.empty(n, dtype=torch.int32, device=device)
  slots = torch.empty(n, dtype=torch.int32, device=device)
  w = torch.empty(n, dtype=torch.float32, device=device)
  probs = torch.empty(n, dtype=torch.float64, device=device)
  lib = _native.lib()
  _native.check(lib.dqz_per_sample(
      _native.ptr(tree.tree), tree.capacity, 0, d.size, tree.capacity, n,
      g['usp'], 0.5, 1, 0, None, _native.ptr(inj_i), _native.ptr(inj_u), None,
      _native.ptr(idx), _native.ptr(slots), _native.ptr(w), _native.ptr(probs),
      _native.stream_handle()))
  got_idx = idx.cpu().numpy()
  assert d.index_to_id(got_idx).tolist() == g['ids']
  assert slots.cpu().numpy().tolist() == got_idx.tolist()  # identity map
  assert probs.cpu().numpy().tolist() == g['probs']  # bit-exact fp64
  want_w = replay_lib.importance_sampling_weights(np.array(g['probs']),
                                                  1.0 / d.size, 0.5, True)
  np.testing.assert_allclose(w.cpu().numpy(), want_w.astype(np.float32),
                             rtol=2e-7)


def _frame(v):
  return np.full((84, 84, 4), v, dtype=np.uint8)


@pytest.mark.parametrize('case', [0, 1])
def test_device_prioritized_replay_reproduces_golden_log(device, case):
  """PrioritizedTransitionReplay (replay.py:1046-1160) with its sum tree in
  HBM: frame transitions, RandomState(seed) as in the golden run; every
  sample's ids, items and importance weights equal the reference's, and
  the device tree equals the host mirror's after the same operations."""
  from dqn_mgsc_zoo_amd import replay as replay_lib
  g = GOLDEN['prioritized']['replay'][case]
  structure = replay_lib.Transition(None, None, None, None, None)

  def make():
    return replay_lib.PrioritizedTransitionReplay(
        capacity=8, structure=structure, priority_exponent=0.6,
        importance_sampling_exponent=lambda t: 0.4,
        uniform_sample_probability=0.1, normalize_weights=True,
        random_state=np.random.RandomState(g['seed']))

  r = make()
  host = make()
  log = iter(g['log'])
  for i, p in enumerate(g['priorities']):
    tr = replay_lib.Transition(_frame(i), 0, 0.0, 1.0, _frame(i))
    r.add(tr, priority=p)
    host.add(replay_lib.Transition(i, 0, 0.0, 1.0, i), priority=p)
    assert r.on_device and r.distribution.on_device
    if i < 3:
      continue
    want = next(log)
    indices, slots, weights = r.sample_device(5)
    ids = r.distribution.index_to_id(indices.cpu().numpy())
    assert ids.tolist() == want['ids']
    assert (slots.cpu().numpy() == ids % 8).all()
    items = r.frame_store.gather_stacks(slots, 0).cpu().numpy()[:, 0, 0, 0]
    assert items.tolist() == want['items']
    np.testing.assert_allclose(weights.cpu().numpy(),
                               np.float32(want['weights']), rtol=2e-7)
    _, host_ids, _ = host.sample(5)
    assert host_ids.tolist() == want['ids']
    uids, uprios = want['update']
    r.update_priorities(uids, uprios)
    host.update_priorities(uids, uprios)
    np.testing.assert_array_equal(r.distribution.sum_tree.storage[1:],
                                  host.distribution.sum_tree.storage[1:])
  ok, msg = r.check_valid()
  assert ok, msg


def test_device_per_add_and_write_back(device):
  """dqz_per_add (evict -> 0, new leaf -> max_seen ** alpha, tree index ->
  slot) and dqz_per_write_back (|td| -> max_seen -> leaves) against the host
  SumTree arithmetic."""
  from dqn_mgsc_zoo_amd import learner as learner_lib
  from dqn_mgsc_zoo_amd import networks
  from dqn_mgsc_zoo_amd import replay as replay_lib
  from dqn_mgsc_zoo_amd import store as store_lib
  alpha = 0.6
  r = replay_lib.PrioritizedTransitionReplay(
      capacity=16, structure=replay_lib.Transition(None, None, None, None, None),
      priority_exponent=alpha, importance_sampling_exponent=lambda t: 0.4,
      uniform_sample_probability=1e-3, normalize_weights=True,
      random_state=np.random.RandomState(5))
  max_seen = torch.full((1,), 2.5, dtype=torch.float64, device=device)
  for i in range(40):  # wraps the FIFO twice: every add also evicts
    r.add(replay_lib.Transition(_frame(i), i % 6, 0.0, 0.99, _frame(i + 1)),
          priority=max_seen if i % 3 else 0.75)
  d = r.distribution
  live = list(r._order)  # pylint: disable=protected-access
  vals = d.get_exponentiated_priorities(live)
  want = [np.float64(0.75)**alpha if i % 3 == 0 else np.float64(2.5)**alpha for i in live]
  np.testing.assert_allclose(vals, want, rtol=1e-15)
  host = replay_lib.SumTree()
  host.resize(16)
  host.set(d.index_of(live), vals)
  np.testing.assert_array_equal(d.sum_tree.storage[1:], host.storage[1:])
  m = d.sum_tree.index_to_slot.cpu().numpy()
  assert [int(m[d.index_of([i])[0]]) for i in live] == [i % 16 for i in live]
  # write-back of a learner step's |td|
  net = networks.double_dqn_atari_network(6)
  lrn = learner_lib.Learner(net, 32, algo='per')
  lrn.set_params(net.init(3))
  indices, slots, w = r.sample_device(32)
  lrn.step(r.frame_store, slots, w)
  r.write_back(lrn, indices, max_seen)
  _, td, _ = lrn.fetch_outputs()
  p = np.abs(td.cpu().numpy().astype(np.float64))
  assert max_seen.item() == max(2.5, p.max())
  last = {}
  for k, v in zip(indices.cpu().numpy().tolist(), p.tolist()):
    last[k] = v
  host.set(list(last), replay_lib._power(np.array(list(last.values())), alpha))  # pylint: disable=protected-access
  np.testing.assert_allclose(d.sum_tree.storage[1:], host.storage[1:], rtol=1e-15)


def _ref_lse(x):
  return replay_ref.logsumexp_f32(x)


@pytest.mark.parametrize('reservoir', [False, True])
def test_running_logsumexp_matches_full_recompute(device, reservoir):
  """12k random add / popleft (replace) / set / hand-out operations on a
  3000-slot buffer: the running log-sum-exp adds (replay_circular.py:166-190,
  526-533) stay within 1e-5 of the reference's full float32 recompute, across
  the 4096-add re-seed, guard re-scans and invalidations."""
  from dqn_mgsc_zoo_amd import replay_circular as rc
  cap = 3000
  rng = np.random.default_rng(11)
  ref = np.full(cap, -np.inf, np.float32)
  if reservoir:
    buf = rc.MGSCReservoirDistribution(np.random.default_rng(0), cap)
  else:
    buf = rc.CircularLogitBuffer(cap, np.random.default_rng(0))
  size = left = right = 0
  worst = 0.0
  for step in range(12000):
    op = rng.random()
    if reservoir:
      if size < cap:
        item = np.float32(0.0) if size == 0 else np.float32(_ref_lse(ref) - np.log(size))
        ref[size] = item
        buf.add()
        size += 1
      elif op < 0.8:
        idx = int(rng.integers(0, cap))
        ref[idx] = -np.inf
        ref[idx] = np.float32(_ref_lse(ref) - np.log(size))
        buf.replace(idx)
      else:
        keys = rng.integers(0, cap, 5)
        vals = rng.normal(0, 2, 5).astype(np.float32)
        for k, v in zip(keys, vals):
          ref[k] = v
        buf[keys] = vals
    else:
      if size == cap or (size > 0 and op < 0.3):
        ref[left] = -np.inf
        buf.popleft(return_value=False)
        left = (left + 1) % cap
        size -= 1
      elif size > 0 and op < 0.38:
        keys = rng.integers(0, size, 5)
        vals = rng.normal(0, 2, 5).astype(np.float32)
        for k, v in zip(keys, vals):
          ref[(left + k) % cap] = v
        buf[keys] = vals
      else:
        item = np.float32(0.0) if size == 0 else np.float32(_ref_lse(ref) - np.log(size))
        ref[right] = item
        buf.add()
        right = (right + 1) % cap
        size += 1
    if step % 2500 == 1249:  # hand the tensor out (as to the meta-update): next add re-scans
      _ = buf.logits
    if step % 1000 == 999:
      got = buf._dev.logits.cpu().numpy()  # pylint: disable=protected-access
      live = np.isfinite(ref)
      assert (np.isfinite(got) == live).all()
      worst = max(worst, float(np.abs(got[live] - ref[live]).max()))
      np.testing.assert_allclose(got[live], ref[live], rtol=0, atol=1e-5)
      ref[live] = got[live]  # re-anchor so errors do not compound across checks
  assert worst < 1e-5


def test_chunk_sums_follow_every_write(device):
  """The per-chunk sums a draw searches stay the canonical sums of the
  current terms through every writer: running adds, reservoir replace,
  popleft, explicit writes (dirty chunks), a guard that re-seeds c inside
  the writer (an item far above c, a removal that cancels S), a hand-out and
  a checkpoint restore — over a ragged multi-chunk buffer.  Each draw then
  equals numpy's choice given the device's terms."""
  from dqn_mgsc_zoo_amd import replay_circular as rc
  cap = 3 * 4096 + 123
  rng = np.random.default_rng(21)
  buf = rc.MGSCReservoirDistribution(np.random.default_rng(1), cap)
  dev = buf.device_logits
  for _ in range(cap):
    buf.add()
  _check_chunk_sums(dev)
  for step in range(300):
    op = rng.random()
    if op < 0.5:
      buf.replace(int(rng.integers(0, cap)))
    elif op < 0.8:
      keys = rng.integers(0, cap, 7)
      buf[keys] = rng.normal(0, 2, 7).astype(np.float32)
    else:
      dev.put(int(rng.integers(0, cap)), float(rng.normal(0, 2)))
    if step % 50 == 49:
      _check_chunk_sums(dev)
  c0 = dev.run_state()['c']
  dev.put(5, c0 + 85.0)  # far above c: the put re-seeds c and every chunk
  st = dev.run_state()
  assert st['valid'] == 1 and st['c'] == np.float32(c0 + 85.0)
  _check_chunk_sums(dev)
  dev.put(5, -np.inf)  # removes almost all of S: re-seed again
  assert dev.run_state()['c'] < c0 + 85.0
  _check_chunk_sums(dev)
  keys = np.arange(0, cap, 997)
  buf[keys] = np.float32(c0 + 90.0)  # explicit writes that trip the guard
  t = _check_chunk_sums(dev)
  u = np.random.default_rng(4).random(64)
  got = dev.sample_abs(u).cpu().numpy()
  np.testing.assert_array_equal(got, _choice_from_p(t, u))
  state = buf.get_state()
  other = rc.MGSCReservoirDistribution(np.random.default_rng(2), cap)
  other.set_state(state)
  t2 = _check_chunk_sums(other.device_logits)
  np.testing.assert_array_equal(t, t2)
  got2 = other.device_logits.sample_abs(u).cpu().numpy()
  np.testing.assert_array_equal(got, got2)
  _ = buf.logits  # handed out: the next draw re-seeds
  _check_chunk_sums(dev)


def test_chunk_sums_follow_fifo_writes(device):
  """The same invariant through CircularLogitBuffer (MGSC FIFO): running adds,
  popleft (-inf puts), explicit writes through __setitem__, wrap-around past
  the capacity, a buffer emptied to nothing (S = 0 re-seeds) and refilled."""
  from dqn_mgsc_zoo_amd import replay_circular as rc
  cap = 2 * 4096 + 777
  rng = np.random.default_rng(22)
  buf = rc.CircularLogitBuffer(cap, np.random.default_rng(3))
  dev = buf._dev  # pylint: disable=protected-access
  for _ in range(cap):
    buf.add()
  _check_chunk_sums(dev)
  for step in range(400):
    op = rng.random()
    if op < 0.4 and buf.size > 0:
      buf.popleft(return_value=False)
    elif op < 0.55 and buf.size > 0:
      keys = rng.integers(0, buf.size, 5)
      buf[keys] = rng.normal(0, 2, 5).astype(np.float32)
    elif buf.size < cap:
      buf.add()
    if step % 100 == 99:
      _check_chunk_sums(dev)
  while buf.size > 0:  # empty: the last popleft leaves S = 0
    buf.popleft(return_value=False)
  _check_chunk_sums(dev)
  for _ in range(100):
    buf.add()
  t = _check_chunk_sums(dev)
  u = np.random.default_rng(6).random(32)
  got = dev.sample_abs(u).cpu().numpy()
  np.testing.assert_array_equal(got, _choice_from_p(t, u))


def test_fused_logit_sampler_equals_philox_then_choice(device):
  """dqz_logits_sample_slots (one launch: Philox uniforms + block sums + CDF
  search behind an in-launch hand-off) draws exactly what
  dqz_uniform_philox + dqz_logits_sample draw, as int32 slots, advances the
  counter once per call, and stays exact under hipGraph replay (the launch
  resets its own hand-off words)."""
  from dqn_mgsc_zoo_amd import _native
  from dqn_mgsc_zoo_amd import replay_circular as rc
  cap, n = 1_000_000, 32
  rng = np.random.default_rng(12)
  logits = rng.standard_normal(cap).astype(np.float32)
  logits[rng.integers(0, cap, 500)] = -np.inf
  dev = rc._DeviceLogits(cap, max_queries=n)  # pylint: disable=protected-access
  dev.load(logits)
  lib = _native.lib()
  c_fused = torch.zeros((1,), dtype=torch.int64, device=device)
  c_ref = torch.zeros((1,), dtype=torch.int64, device=device)
  slots = torch.empty((n,), dtype=torch.int32, device=device)
  idx = torch.empty((n,), dtype=torch.int64, device=device)
  uni = torch.empty((n,), dtype=torch.float64, device=device)
  seed = 99

  def ref_draw():
    _native.check(lib.dqz_uniform_philox(seed, _native.ptr(c_ref), n, _native.ptr(uni),
                                         _native.stream_handle()))
    return dev.sample_abs(uni.cpu().numpy()).clone()

  for _ in range(4):
    dev.sample_slots_philox(seed, c_fused, slots, idx)
    want = ref_draw()
    torch.cuda.synchronize()
    assert torch.equal(idx, want)
    assert torch.equal(slots.long(), want)
    assert int(c_fused.item()) == int(c_ref.item())
  # the choice is numpy's given the device's terms
  t = _check_chunk_sums(dev)
  np.testing.assert_array_equal(idx.cpu().numpy(), _choice_from_p(t, uni.cpu().numpy()))
  # graph replay: 5 captured draws, replayed twice
  side = torch.cuda.Stream(device)
  side.wait_stream(torch.cuda.current_stream(device))
  with torch.cuda.stream(side):
    dev.sample_slots_philox(seed, c_fused, slots, idx)
  torch.cuda.current_stream(device).wait_stream(side)
  ref_draw()
  g = torch.cuda.CUDAGraph()
  outs = [torch.empty((n,), dtype=torch.int64, device=device) for _ in range(5)]
  with torch.cuda.graph(g):
    for o in outs:
      dev.sample_slots_philox(seed, c_fused, slots, o)
  for _ in range(2):
    g.replay()
    torch.cuda.synchronize()
    for o in outs:
      assert torch.equal(o, ref_draw())
  assert int(c_fused.item()) == int(c_ref.item())


def test_device_per_all_zero_priorities_follow_the_reference_stream(device):
  """while every priority is 0 the reference skips the target
  draw (replay.py:689-697: prio_idx = uniform_idx, one uniform stream for
  the usp mix).  The device replay draws the same ids with probabilities
  1/N and leaves its RandomState exactly where the host replay's is; after
  a positive priority both draw both streams again."""
  from dqn_mgsc_zoo_amd import replay as replay_lib

  def make(seed=4):
    return replay_lib.PrioritizedTransitionReplay(
        capacity=8, structure=replay_lib.Transition(None, None, None, None, None),
        priority_exponent=0.6, importance_sampling_exponent=lambda t: 0.4,
        uniform_sample_probability=0.1, normalize_weights=True,
        random_state=np.random.RandomState(seed))

  dev, host = make(), make()
  for i in range(6):
    dev.add(replay_lib.Transition(_frame(i), 0, 0.0, 1.0, _frame(i)), priority=0.0)
    host.add(replay_lib.Transition(i, 0, 0.0, 1.0, i), priority=0.0)
  assert dev.on_device
  for _ in range(3):
    indices, _, weights = dev.sample_device(5)
    _, host_ids, host_w = host.sample(5)
    assert dev.distribution.index_to_id(indices.cpu().numpy()).tolist() == host_ids.tolist()
    np.testing.assert_allclose(weights.cpu().numpy(), host_w, rtol=1e-6)
    st_d, st_h = dev._random_state.get_state(), host._random_state.get_state()  # pylint: disable=protected-access
    assert st_d[2] == st_h[2] and np.array_equal(st_d[1], st_h[1])
  dev.update_priorities([2], [1.5])
  host.update_priorities([2], [1.5])
  indices, _, _ = dev.sample_device(5)
  _, host_ids, _ = host.sample(5)
  assert dev.distribution.index_to_id(indices.cpu().numpy()).tolist() == host_ids.tolist()
  assert dev._random_state.get_state()[2] == host._random_state.get_state()[2]  # pylint: disable=protected-access
