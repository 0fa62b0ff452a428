"""GPU parity: the HIP learner step vs the fp64 oracle on identical inputs.

Tolerances (BASELINE.json north_star: Q-values within 1e-4 fp32):
  q / td: atol 1e-4; loss: rtol 1e-4; updated params: atol 2e-6;
  RMSProp moments: rtol 1e-3, atol 1e-12.
"""

import numpy as np
import pytest
import torch

from oracle import learner_ref
from tests import helpers

pytestmark = pytest.mark.gpu

Q_ATOL = 1e-4
P_ATOL = 2e-6


def _setup(algo, batch, capacity=256, num_frames=640, num_actions=6, seed=0,
           nonzero_opt_state=False):
  from dqn_mgsc_zoo_amd import learner as learner_lib
  from dqn_mgsc_zoo_amd import networks
  from dqn_mgsc_zoo_amd import store as store_lib
  net = (networks.dqn_atari_network(num_actions) if algo == 'dqn' else
         networks.double_dqn_atari_network(num_actions))
  online = net.init(seed)
  target = helpers.perturbed_tree(online, seed + 1)
  lrn = learner_lib.Learner(net, batch, algo=algo)
  lrn.set_params(online, target)
  mu = learner_ref.zeros_like_tree(online)
  nu = learner_ref.zeros_like_tree(online)
  if nonzero_opt_state:
    rng = np.random.default_rng(seed + 7)
    mu = {m: {n: 1e-3 * rng.standard_normal(v.shape) for n, v in d.items()}
          for m, d in mu.items()}
    nu = {m: {n: mu[m][n]**2 + 1e-6 * rng.random(v.shape) for n, v in d.items()}
          for m, d in mu.items()}
    lrn.set_opt_state(
        {m: {n: v.astype(np.float32) for n, v in d.items()} for m, d in mu.items()},
        {m: {n: v.astype(np.float32) for n, v in d.items()} for m, d in nu.items()})
    # Use the f32-rounded state in the oracle too.
    mu = {m: {n: v.astype(np.float32).astype(np.float64) for n, v in d.items()}
          for m, d in mu.items()}
    nu = {m: {n: v.astype(np.float32).astype(np.float64) for n, v in d.items()}
          for m, d in nu.items()}
  frames, fidx, action, reward, discount = helpers.random_store_contents(
      capacity, num_frames, num_actions, seed + 3)
  st = store_lib.FrameStore(capacity, num_frames)
  st.frames.copy_(torch.from_numpy(frames))
  st.fidx.copy_(torch.from_numpy(fidx))
  st.action.copy_(torch.from_numpy(action))
  st.reward.copy_(torch.from_numpy(reward))
  st.discount.copy_(torch.from_numpy(discount))
  host = dict(frames=frames, fidx=fidx, action=action, reward=reward,
              discount=discount)
  return net, lrn, st, host, online, target, mu, nu


def _compare_tree(got, want, atol, rtol=0.0, what=''):
  for m in want:
    for n in want[m]:
      np.testing.assert_allclose(got[m][n], want[m][n], atol=atol, rtol=rtol,
                                 err_msg='%s %s/%s' % (what, m, n))


@pytest.mark.parametrize('algo', ['dqn', 'double', 'per'])
@pytest.mark.parametrize('nonzero', [False, True])
def test_learner_step_matches_oracle(device, algo, nonzero):
  batch = 32
  net, lrn, st, host, online, target, mu, nu = _setup(
      algo, batch, seed=11 if nonzero else 3, nonzero_opt_state=nonzero)
  rng = np.random.default_rng(5)
  slots = helpers.kink_free_slots(online, host, st.capacity, batch, rng)
  weights = None
  if algo == 'per':
    weights = rng.uniform(0.2, 1.0, size=batch).astype(np.float32)
    weights /= weights.max()
  s_tm1 = helpers.stacks_from(host['frames'], host['fidx'], slots, 0)
  s_t = helpers.stacks_from(host['frames'], host['fidx'], slots, 1)
  ref = learner_ref.learner_step(
      online, target, mu, nu, s_tm1, host['action'][slots],
      host['reward'][slots], host['discount'][slots], s_t, algo=algo,
      weights=weights)
  slots_d = torch.from_numpy(slots).to(device)
  w_d = None if weights is None else torch.from_numpy(weights).to(device)
  lrn.step(st, slots_d, w_d)
  q, td, loss = lrn.fetch_outputs()
  torch.cuda.synchronize()
  np.testing.assert_allclose(q.cpu().numpy(), ref['q_tm1'], atol=Q_ATOL)
  np.testing.assert_allclose(td.cpu().numpy(), ref['td'], atol=Q_ATOL)
  np.testing.assert_allclose(loss.cpu().numpy()[0], ref['loss'], rtol=1e-4,
                             atol=1e-7)
  _compare_tree(lrn.params_tree('online'), ref['params'], P_ATOL, what='params')
  _compare_tree(lrn.params_tree('mu'), ref['mu'], 1e-9, 1e-3, what='mu')
  _compare_tree(lrn.params_tree('nu'), ref['nu'], 1e-12, 2e-3, what='nu')
  # the target network is untouched by a learner step
  _compare_tree(lrn.params_tree('target'), target, 0.0, what='target')


def _rel_norm_err(got, want):
  worst = 0.0
  for m in want:
    for n in want[m]:
      w = np.asarray(want[m][n], np.float64)
      d = np.linalg.norm(np.asarray(got[m][n], np.float64) - w)
      worst = max(worst, d / max(np.linalg.norm(w), 1e-30))
  return worst


@pytest.mark.parametrize('algo', ['dqn', 'double'])
def test_learner_step_on_unfiltered_batches(device, algo):
  """Plain rng.integers batches (no kink filter, helpers.kink_free_slots):
  a ReLU pre-activation within f32 rounding of 0 may take the other branch
  than in fp64, which moves single gradient entries (not the forward), so
  q / td / loss keep their elementwise bars and the gradient (mu after one
  step from zero state is (1 - decay) g) and the update are held to a
  relative Frobenius-norm bar per leaf."""
  batch = 32
  for seed in (21, 22, 23, 24):
    net, lrn, st, host, online, target, mu, nu = _setup(algo, batch, seed=seed)
    slots = np.random.default_rng(seed).integers(
        0, st.capacity, size=batch).astype(np.int32)
    s_tm1 = helpers.stacks_from(host['frames'], host['fidx'], slots, 0)
    s_t = helpers.stacks_from(host['frames'], host['fidx'], slots, 1)
    ref = learner_ref.learner_step(
        online, target, mu, nu, s_tm1, host['action'][slots],
        host['reward'][slots], host['discount'][slots], s_t, algo=algo)
    lrn.step(st, torch.from_numpy(slots).to(device))
    q, td, loss = lrn.fetch_outputs()
    torch.cuda.synchronize()
    np.testing.assert_allclose(q.cpu().numpy(), ref['q_tm1'], atol=Q_ATOL)
    np.testing.assert_allclose(td.cpu().numpy(), ref['td'], atol=Q_ATOL)
    np.testing.assert_allclose(loss.cpu().numpy()[0], ref['loss'], rtol=1e-4,
                               atol=1e-7)
    g_err = _rel_norm_err(lrn.params_tree('mu'), ref['mu'])
    after = lrn.params_tree('online')
    delta_got = {m: {n: after[m][n] - online[m][n]
                     for n in online[m]} for m in online}
    delta_want = {m: {n: ref['params'][m][n] - online[m][n]
                      for n in online[m]} for m in online}
    u_err = _rel_norm_err(delta_got, delta_want)
    print('seed %d margin %.2e: gradient rel err %.2e, update rel err %.2e' % (
        seed, learner_ref.relu_margin(online, s_tm1), g_err, u_err))
    # measured (round 3, seeds 21-24, margins 1.3e-7 .. 6.4e-7 — inside the
    # 1e-6 band the filtered tests exclude): gradient <= 4.3e-7, update
    # <= 3.6e-5
    assert g_err <= 1e-5, g_err
    assert u_err <= 1e-3, u_err


def test_forward_q_values_direct_and_slots(device):
  batch = 16
  net, lrn, st, host, online, _, _, _ = _setup('dqn', batch, seed=21)
  rng = np.random.default_rng(1)
  slots = rng.integers(0, st.capacity, size=batch).astype(np.int32)
  s_t = helpers.stacks_from(host['frames'], host['fidx'], slots, 1)
  q_ref, _ = learner_ref.forward(online, s_t)
  q_direct = lrn.q_values(torch.from_numpy(s_t).to(device))
  q_slots = lrn.q_values_slots(st, torch.from_numpy(slots).to(device), 1)
  np.testing.assert_allclose(q_direct.cpu().numpy(), q_ref, atol=Q_ATOL)
  np.testing.assert_allclose(q_slots.cpu().numpy(), q_ref, atol=Q_ATOL)
  # n smaller than the batch (the actor's B=1 path)
  q1 = lrn.q_values(torch.from_numpy(s_t[:1]).to(device))
  np.testing.assert_allclose(q1.cpu().numpy(), q_ref[:1], atol=Q_ATOL)


def test_gather_stacks_bit_exact(device):
  _, _, st, host, _, _, _, _ = _setup('dqn', 8, seed=4)
  slots = np.arange(0, st.capacity, 3).astype(np.int32)
  for which in (0, 1):
    got = st.gather_stacks(torch.from_numpy(slots).to(device), which)
    want = helpers.stacks_from(host['frames'], host['fidx'], slots, which)
    np.testing.assert_array_equal(got.cpu().numpy(), want)


def test_multi_step_with_target_sync(device):
  batch = 32
  net, lrn, st, host, online, target, mu, nu = _setup('dqn', batch, seed=8)
  rng = np.random.default_rng(9)
  p, t = online, target
  for step in range(3):
    slots = helpers.kink_free_slots(p, host, st.capacity, batch, rng)
    s_tm1 = helpers.stacks_from(host['frames'], host['fidx'], slots, 0)
    s_t = helpers.stacks_from(host['frames'], host['fidx'], slots, 1)
    ref = learner_ref.learner_step(
        p, t, mu, nu, s_tm1, host['action'][slots], host['reward'][slots],
        host['discount'][slots], s_t)
    lrn.step(st, torch.from_numpy(slots).to(device))
    p, mu, nu = ref['params'], ref['mu'], ref['nu']
    if step == 1:
      lrn.sync_target()
      t = p
  torch.cuda.synchronize()
  _compare_tree(lrn.params_tree('online'), p, 5e-6, what='params')
  _compare_tree(lrn.params_tree('target'), t, 5e-6, what='target')


def test_sample_uniform_device(device):
  from dqn_mgsc_zoo_amd import learner as learner_lib
  counter = torch.zeros((1,), dtype=torch.int64, device=device)
  out = torch.empty((4096,), dtype=torch.int32, device=device)
  capacity, size, base = 1000, 600, 700  # FIFO window wraps the ring
  counts = np.zeros(capacity)
  for _ in range(20):
    learner_lib.sample_uniform(base, size, capacity, 4096, 1234, counter, out)
    counts += np.bincount(out.cpu().numpy(), minlength=capacity)
  live = (base + np.arange(size)) % capacity
  assert counts.sum() == counts[live].sum()  # never outside the live window
  assert int(counter.item()) == 20  # device counter advanced once per call
  expected = counts.sum() / size
  # chi-square-ish bound on the per-slot counts
  assert np.abs(counts[live] - expected).max() < 6 * np.sqrt(expected)
  # a base past the ring's end names the same window (base is taken mod capacity)
  ca = torch.zeros((1,), dtype=torch.int64, device=device)
  cb = torch.zeros((1,), dtype=torch.int64, device=device)
  oa = torch.empty((512,), dtype=torch.int32, device=device)
  ob = torch.empty((512,), dtype=torch.int32, device=device)
  learner_lib.sample_uniform(base, size, capacity, 512, 99, ca, oa)
  learner_lib.sample_uniform(base + 3 * capacity, size, capacity, 512, 99, cb, ob)
  assert torch.equal(oa, ob)


def test_fused_uniform_step_matches_sample_then_step(device):
  """dqz_learner_step_uniform == dqz_sample_uniform + dqz_learner_step, bit for bit."""
  from dqn_mgsc_zoo_amd import learner as learner_lib
  batch = 32
  net, lrn, st, host, online, target, mu, nu = _setup('dqn', batch, seed=13)
  _, lrn2, _, _, _, _, _, _ = _setup('dqn', batch, seed=13)
  c1 = torch.zeros((1,), dtype=torch.int64, device=device)
  c2 = torch.zeros((1,), dtype=torch.int64, device=device)
  s1 = torch.zeros((batch,), dtype=torch.int32, device=device)
  s2 = torch.zeros((batch,), dtype=torch.int32, device=device)
  for _ in range(3):
    learner_lib.sample_uniform(5, 200, st.capacity, batch, 77, c1, s1)
    lrn.step(st, s1)
    lrn2.step_uniform(st, 5, 200, st.capacity, 77, c2, s2)
    torch.cuda.synchronize()
    assert torch.equal(s1, s2)
  assert int(c1.item()) == int(c2.item()) == 3
  for which in ('online', 'mu', 'nu'):
    assert torch.equal(getattr(lrn, which), getattr(lrn2, which))


@pytest.mark.parametrize('algo,batch,num_actions', [
    ('dqn', 1, 6), ('dqn', 8, 6), ('double', 5, 6), ('dqn', 20, 18), ('double', 48, 4), ('per', 40, 18)])
def test_learner_step_odd_shapes(device, algo, batch, num_actions):
  """Batches that are not multiples of the 8-XCD / 16-row / 32-row tilings,
  the full 18-action set (head kernel AMAX 32 path), and launches of at most
  16 samples (Z x B: dqn 1 and 8, double 5), whose forward runs conv2 / conv3
  as 8 jobs per sample (fwd.hpp fwd_conv_jobs)."""
  net, lrn, st, host, online, target, mu, nu = _setup(
      algo, batch, capacity=96, num_frames=260, num_actions=num_actions,
      seed=31 + batch)
  rng = np.random.default_rng(batch)
  slots = helpers.kink_free_slots(online, host, st.capacity, batch, rng)
  weights = None
  if algo == 'per':
    weights = rng.uniform(0.2, 1.0, size=batch).astype(np.float32)
  s_tm1 = helpers.stacks_from(host['frames'], host['fidx'], slots, 0)
  s_t = helpers.stacks_from(host['frames'], host['fidx'], slots, 1)
  ref = learner_ref.learner_step(
      online, target, mu, nu, s_tm1, host['action'][slots],
      host['reward'][slots], host['discount'][slots], s_t, algo=algo,
      weights=weights)
  lrn.step(st, torch.from_numpy(slots).to(device),
           None if weights is None else torch.from_numpy(weights).to(device))
  q, td, loss = lrn.fetch_outputs()
  np.testing.assert_allclose(q.cpu().numpy(), ref['q_tm1'], atol=Q_ATOL)
  np.testing.assert_allclose(td.cpu().numpy(), ref['td'], atol=Q_ATOL)
  _compare_tree(lrn.params_tree('online'), ref['params'], P_ATOL, what='params')
  # actor path at the same odd batch: q-values of s_t through dqz_forward
  q_t = lrn.q_values(torch.from_numpy(s_t).to(device))
  q_ref, _ = learner_ref.forward(ref['params'], s_t, algo != 'dqn')
  np.testing.assert_allclose(q_t.cpu().numpy(), q_ref, atol=Q_ATOL)


@pytest.mark.parametrize('algo,batch', [('dqn', 32), ('per', 20), ('double', 64),
                                        ('dqn', 33), ('dqn', 8)])
def test_handoff_kernels_bit_reproducible(device, algo, batch):
  """The in-launch hand-offs (bwd_bc_kernel: conv3 dX -> conv2 dX / conv2 dW,
  conv2 dX -> conv1 dW) sum in fixed orders, whichever workgroup arrives
  last: two learners fed the same
  steps agree bit for bit, eagerly, under hipGraph replay and after
  profile-mode back-to-back launches; the hand-off words reset themselves
  (sync_status 0); and the result stays at the oracle."""
  _, ref, st, host, online, target, mu, nu = _setup(algo, batch, seed=21)
  _, lrn, _, _, _, _, _, _ = _setup(algo, batch, seed=21)
  rng = np.random.default_rng(22)
  w = torch.rand((batch,), device=device) + 0.5 if algo == 'per' else None
  for _ in range(12):
    slots = torch.from_numpy(
        rng.integers(0, st.capacity, size=batch).astype(np.int32)).to(device)
    ref.step(st, slots, w)
    lrn.step(st, slots, w)
  slots = torch.from_numpy(
      rng.integers(0, st.capacity, size=batch).astype(np.int32)).to(device)
  side = torch.cuda.Stream(device)
  side.wait_stream(torch.cuda.current_stream(device))
  with torch.cuda.stream(side):
    lrn.step(st, slots, w)
  torch.cuda.current_stream(device).wait_stream(side)
  ref.step(st, slots, w)
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    for _ in range(4):
      lrn.step(st, slots, w)
  for _ in range(3):
    g.replay()
  for _ in range(12):
    ref.step(st, slots, w)
  torch.cuda.synchronize()
  assert lrn.sync_status() == 0 and ref.sync_status() == 0
  for which in ('online', 'mu', 'nu'):
    assert torch.equal(getattr(lrn, which), getattr(ref, which)), which
  q1, td1, _ = lrn.fetch_outputs()
  q2, td2, _ = ref.fetch_outputs()
  assert torch.equal(q1, q2) and torch.equal(td1, td2)
  # profile mode repeats every launch back to back; the hand-off words must
  # reset themselves between launches.
  lrn.profile(st, slots, weights=w, iters=5)
  torch.cuda.synchronize()
  assert lrn.sync_status() == 0
  # one more step from the same state on both: still identical, still sane
  slots = torch.from_numpy(
      rng.integers(0, st.capacity, size=batch).astype(np.int32)).to(device)
  lrn.set_params(ref.params_tree('online'), ref.params_tree('target'))
  lrn.set_opt_state(ref.params_tree('mu'), ref.params_tree('nu'))
  ref.step(st, slots, w)
  lrn.step(st, slots, w)
  torch.cuda.synchronize()
  for which in ('online', 'mu', 'nu'):
    assert torch.equal(getattr(lrn, which), getattr(ref, which)), which


def test_per_write_back_device(device):
  """dqz_per_write_back == |td| -> max_seen, _power(|td|, alpha) -> SumTree.set
  (host mirror of replay.py:411-423), duplicates keeping the last draw."""
  from dqn_mgsc_zoo_amd import _native
  from dqn_mgsc_zoo_amd import replay as replay_lib
  batch, alpha = 32, 0.6
  _, lrn, st, _, _, _, _, _ = _setup('per', batch, seed=31)
  rng = np.random.default_rng(32)
  host = replay_lib.SumTree()
  host.set_all(rng.random(st.capacity))
  tree = torch.from_numpy(host.storage.copy()).to(device)
  slots_np = rng.integers(0, st.capacity, size=batch).astype(np.int32)
  slots_np[5] = slots_np[20]  # a duplicate draw
  slots = torch.from_numpy(slots_np).to(device)
  w = torch.rand((batch,), device=device) + 0.5
  lrn.step(st, slots, w)
  max_seen = torch.tensor([0.25], dtype=torch.float64, device=device)
  _native.check(_native.lib().dqz_per_write_back(
      lrn._h, _native.ptr(tree), host.capacity, _native.ptr(slots), alpha,  # pylint: disable=protected-access
      _native.ptr(max_seen), _native.stream_handle()))
  _, td, _ = lrn.fetch_outputs()
  torch.cuda.synchronize()
  p = np.abs(td.cpu().numpy().astype(np.float64))
  host.set(slots_np, replay_lib._power(p, alpha))  # pylint: disable=protected-access
  np.testing.assert_allclose(tree.cpu().numpy()[1:], host.storage[1:], rtol=4e-16, atol=0)
  assert max_seen.item() == max(0.25, p.max())


def test_nonfinite_loss_is_flagged(device):
  """NaN guard: a step whose mean loss is not finite sets bit 1 of the
  learner's health word (dqz_learner_sync_status); reading it clears it."""
  _, lrn, st, _, _, _, _, _ = _setup('dqn', 32, seed=5)
  rng = np.random.default_rng(6)
  slots = torch.from_numpy(rng.integers(0, st.capacity, size=32).astype(np.int32)).to(device)
  lrn.step(st, slots)
  assert lrn.sync_status() == 0
  st.reward[slots[0].long()] = float('nan')
  lrn.step(st, slots)
  assert lrn.sync_status() == 2
  assert lrn.sync_status() == 0


def test_handoff_timeout_is_reported_and_cleared(device):
  """A hand-off wait that runs out (one sample's dy2 counter poisoned, the
  bounded spin shortened) sets bit 0 of the health word; reading it clears
  every hand-off word, and the next step from the same state equals a clean
  learner's bit for bit."""
  _, lrn, st, _, _, _, _, _ = _setup('dqn', 32, seed=8)
  _, ref, _, _, _, _, _, _ = _setup('dqn', 32, seed=8)
  rng = np.random.default_rng(9)

  def slots():
    return torch.from_numpy(rng.integers(0, st.capacity, size=32).astype(np.int32)).to(device)

  s0 = slots()
  lrn.step(st, s0)
  ref.step(st, s0)
  lrn.debug_stall(3, spin_max=4096)
  lrn.step(st, slots())
  assert lrn.sync_status() & 1
  assert lrn.sync_status() == 0
  lrn.debug_stall(-1)  # default spin limit again
  for which in ('online', 'target', 'mu', 'nu'):
    getattr(lrn, which).copy_(getattr(ref, which))
  s1 = slots()
  lrn.step(st, s1)
  ref.step(st, s1)
  assert lrn.sync_status() == 0 and ref.sync_status() == 0
  for which in ('online', 'mu', 'nu'):
    assert torch.equal(getattr(lrn, which), getattr(ref, which)), which


def test_fused_per_write_back_equals_the_separate_launch(device):
  """dqz_learner_step_per (write-back folded into the backward launch) ==
  dqz_learner_step + dqz_per_write_back: same parameters, the same sum tree
  bit for bit (duplicate draws keep the last), the same running max, also
  under hipGraph replay."""
  from dqn_mgsc_zoo_amd import _native
  from dqn_mgsc_zoo_amd import replay as replay_lib
  batch, alpha = 32, 0.6
  _, a, st, _, _, _, _, _ = _setup('per', batch, seed=41)
  _, b, _, _, _, _, _, _ = _setup('per', batch, seed=41)
  rng = np.random.default_rng(42)
  host = replay_lib.SumTree()
  host.set_all(rng.random(1000))
  ta = torch.from_numpy(host.storage.copy()).to(device)
  tb = ta.clone()
  ma = torch.tensor([0.5], dtype=torch.float64, device=device)
  mb = ma.clone()
  w = torch.rand((batch,), device=device) + 0.5

  def draw():
    s = rng.integers(0, st.capacity, size=batch).astype(np.int32)
    s[3] = s[17]  # a repeated draw
    return torch.from_numpy(s).to(device)

  for _ in range(3):
    s = draw()
    a.step(st, s, w)
    _native.check(_native.lib().dqz_per_write_back(
        a._h, _native.ptr(ta), host.capacity, _native.ptr(s), alpha,  # pylint: disable=protected-access
        _native.ptr(ma), _native.stream_handle()))
    b.step(st, s, w, write_back=(tb, host.capacity, s, alpha, mb))
  torch.cuda.synchronize()
  assert torch.equal(ta, tb) and torch.equal(ma, mb)
  for which in ('online', 'mu', 'nu'):
    assert torch.equal(getattr(a, which), getattr(b, which))
  s = draw()
  g = torch.cuda.CUDAGraph()
  side = torch.cuda.Stream(device)
  side.wait_stream(torch.cuda.current_stream(device))
  with torch.cuda.stream(side):
    b.step(st, s, w, write_back=(tb, host.capacity, s, alpha, mb))
  torch.cuda.current_stream(device).wait_stream(side)
  a.step(st, s, w)
  _native.check(_native.lib().dqz_per_write_back(
      a._h, _native.ptr(ta), host.capacity, _native.ptr(s), alpha,  # pylint: disable=protected-access
      _native.ptr(ma), _native.stream_handle()))
  with torch.cuda.graph(g):
    b.step(st, s, w, write_back=(tb, host.capacity, s, alpha, mb))
  g.replay()
  a.step(st, s, w)
  _native.check(_native.lib().dqz_per_write_back(
      a._h, _native.ptr(ta), host.capacity, _native.ptr(s), alpha,  # pylint: disable=protected-access
      _native.ptr(ma), _native.stream_handle()))
  torch.cuda.synchronize()
  assert torch.equal(ta, tb) and torch.equal(ma, mb)
  assert a.sync_status() == 0 and b.sync_status() == 0


def test_fused_logit_draw_step_equals_sampler_then_step(device):
  """dqz_learner_step_logits (the learned-logit draw inside the forward
  launch) == dqz_logits_sample_slots / dqz_logits_sample + dqz_learner_step,
  bit for bit: slots, counter, parameters — Philox draws, the caller's
  uniforms, and under hipGraph replay (the in-launch words reset)."""
  from dqn_mgsc_zoo_amd import replay_circular as rc
  batch = 32
  _, a, st, _, _, _, _, _ = _setup('dqn', batch, seed=51)
  _, b, _, _, _, _, _, _ = _setup('dqn', batch, seed=51)
  rng = np.random.default_rng(52)
  logits = rng.standard_normal(st.capacity).astype(np.float32)
  logits[rng.integers(0, st.capacity, 20)] = -np.inf
  dl = rc._DeviceLogits(st.capacity, device, max_queries=batch)  # pylint: disable=protected-access
  dl.load(logits)
  ca = torch.zeros((1,), dtype=torch.int64, device=device)
  cb = torch.zeros((1,), dtype=torch.int64, device=device)
  sa = torch.zeros((batch,), dtype=torch.int32, device=device)
  sb = torch.zeros((batch,), dtype=torch.int32, device=device)
  for _ in range(3):
    dl.sample_slots_philox(9, ca, sa)
    a.step(st, sa)
    b.step_logits(st, dl, sb, seed=9, counter=cb)
    torch.cuda.synchronize()
    assert torch.equal(sa, sb)
  assert int(ca.item()) == int(cb.item()) == 3
  for _ in range(2):  # the replay Generator's own uniforms
    u = rng.random(batch)
    sa.copy_(dl.sample_abs(u).to(torch.int32))
    a.step(st, sa)
    b.step_logits(st, dl, sb, uniforms=torch.from_numpy(u).to(device))
    torch.cuda.synchronize()
    assert torch.equal(sa, sb)
  side = torch.cuda.Stream(device)
  side.wait_stream(torch.cuda.current_stream(device))
  with torch.cuda.stream(side):
    b.step_logits(st, dl, sb, seed=9, counter=cb)
  torch.cuda.current_stream(device).wait_stream(side)
  dl.sample_slots_philox(9, ca, sa)
  a.step(st, sa)
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    for _ in range(3):
      b.step_logits(st, dl, sb, seed=9, counter=cb)
  g.replay()
  for _ in range(3):
    dl.sample_slots_philox(9, ca, sa)
    a.step(st, sa)
  torch.cuda.synchronize()
  assert torch.equal(sa, sb) and int(ca.item()) == int(cb.item())
  for which in ('online', 'mu', 'nu'):
    assert torch.equal(getattr(a, which), getattr(b, which)), which
  assert a.sync_status() == 0 and b.sync_status() == 0


@pytest.mark.parametrize('injected', [False, True])
def test_fused_per_draw_step_equals_sampler_then_step(device, injected):
  """dqz_learner_step_per_draw (the PER draw in conv1, the IS weights in the
  head, the write-back in the backward) == dqz_per_sample +
  dqz_learner_step_per, bit for bit: indices, slots, probabilities,
  weights, parameters, sum tree, max_seen — Philox draws or the reference's
  RandomState draws injected, and under hipGraph replay."""
  from dqn_mgsc_zoo_amd import _native
  from dqn_mgsc_zoo_amd import replay as replay_lib
  batch, alpha, usp, beta = 32, 0.6, 0.05, 0.4
  _, a, st, _, _, _, _, _ = _setup('per', batch, seed=61)
  _, b, _, _, _, _, _, _ = _setup('per', batch, seed=61)
  rng = np.random.default_rng(62)
  host = replay_lib.SumTree()
  prios = rng.random(st.capacity) ** 2
  prios[::17] = 0.0
  host.set_all(prios)
  cap = host.capacity
  ta = torch.from_numpy(host.storage.copy()).to(device)
  tb = ta.clone()
  ma = torch.tensor([1.0], dtype=torch.float64, device=device)
  mb = ma.clone()
  ca = torch.zeros((1,), dtype=torch.int64, device=device)
  cb = torch.zeros((1,), dtype=torch.int64, device=device)
  i32 = lambda: torch.zeros((batch,), dtype=torch.int32, device=device)
  ia, sa, ib, sb = i32(), i32(), i32(), i32()
  wa = torch.zeros((batch,), dtype=torch.float32, device=device)
  wb = wa.clone()
  pa = torch.zeros((batch,), dtype=torch.float64, device=device)
  pb = pa.clone()
  lib = _native.lib()
  inj = {}

  def draws():
    if injected:
      inj['i'] = torch.from_numpy(rng.integers(0, st.capacity, batch).astype(np.int32)).to(device)
      inj['u'] = torch.from_numpy(rng.random(2 * batch)).to(device)

  def ref_step():
    _native.check(lib.dqz_per_sample(
        _native.ptr(ta), cap, 0, st.capacity, st.capacity, batch, usp, beta, 1, 7,
        None if injected else _native.ptr(ca), _native.ptr(inj.get('i')),
        _native.ptr(inj.get('u')), None, _native.ptr(ia), _native.ptr(sa),
        _native.ptr(wa), _native.ptr(pa), _native.stream_handle()))
    a.step(st, sa, wa, write_back=(ta, cap, ia, alpha, ma))

  def fused_draw():
    return _native.DqzPerDraw(
        tb.data_ptr(), cap, 0, st.capacity, st.capacity, usp, beta, 1, 7,
        None if injected else cb.data_ptr(),
        inj['i'].data_ptr() if injected else None,
        inj['u'].data_ptr() if injected else None, None, alpha, mb.data_ptr(),
        ib.data_ptr(), sb.data_ptr(), pb.data_ptr(), wb.data_ptr())

  for _ in range(3):
    draws()
    ref_step()
    b.step_per_draw(st, fused_draw())
    torch.cuda.synchronize()
    for x, y in ((ia, ib), (sa, sb), (pa, pb), (wa, wb)):
      assert torch.equal(x, y)
  if not injected:  # graph replay of the Philox form
    side = torch.cuda.Stream(device)
    side.wait_stream(torch.cuda.current_stream(device))
    d = fused_draw()
    with torch.cuda.stream(side):
      b.step_per_draw(st, d)
    torch.cuda.current_stream(device).wait_stream(side)
    ref_step()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
      for _ in range(3):
        b.step_per_draw(st, d)
    g.replay()
    for _ in range(3):
      ref_step()
    assert int(ca.item()) == int(cb.item())
  torch.cuda.synchronize()
  assert torch.equal(ta, tb) and torch.equal(ma, mb)
  for which in ('online', 'mu', 'nu'):
    assert torch.equal(getattr(a, which), getattr(b, which)), which
  assert a.sync_status() == 0 and b.sync_status() == 0
