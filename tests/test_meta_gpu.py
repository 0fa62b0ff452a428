"""GPU parity: learner gradients and the MGSC meta-update vs the fp64 oracle.

Tolerances: gradients atol 1e-6 + rtol 1e-3 of the leaf's max |g|; meta
probabilities rtol 1e-6; d meta-loss / d logits within 2e-5 of max |dlogits|
and meta loss rtol 2e-5 (f32 sums over 1.7M parameters against fp64;
measured 1e-6 / 3e-7 at worst); Adam first moment within 1e-5 of its max;
updated logits atol 1e-6 (the Adam step is lr-scaled).
"""

import numpy as np
import pytest
import torch

from oracle import learner_ref
from tests import helpers

pytestmark = pytest.mark.gpu


def _store(capacity, num_frames, num_actions, seed, device):
  from dqn_mgsc_zoo_amd import store as store_lib
  frames, fidx, action, reward, discount = helpers.random_store_contents(
      capacity, num_frames, num_actions, seed)
  st = store_lib.FrameStore(capacity, num_frames)
  for name, arr in (('frames', frames), ('fidx', fidx), ('action', action),
                    ('reward', reward), ('discount', discount)):
    getattr(st, name).copy_(torch.from_numpy(arr))
  host = dict(frames=frames, fidx=fidx, action=action, reward=reward,
              discount=discount)
  return st, host


def _rand_opt_state(tree, seed):
  rng = np.random.default_rng(seed)
  mu = {m: {n: (1e-3 * rng.standard_normal(np.shape(v))).astype(np.float32)
            for n, v in d.items()} for m, d in tree.items()}
  nu = {m: {n: (mu[m][n].astype(np.float64)**2 +
                1e-6 * rng.random(np.shape(v))).astype(np.float32)
            for n, v in d.items()} for m, d in mu.items()}
  return mu, nu


def _f64(tree):
  return {m: {n: np.asarray(v, np.float64) for n, v in d.items()}
          for m, d in tree.items()}


@pytest.mark.parametrize('algo', ['dqn', 'double'])
def test_learner_grad_matches_oracle(device, algo):
  from dqn_mgsc_zoo_amd import learner as learner_lib
  from dqn_mgsc_zoo_amd import networks
  net = (networks.dqn_atari_network(6) if algo == 'dqn' else
         networks.double_dqn_atari_network(6))
  online = net.init(5)
  target = helpers.perturbed_tree(online, 6)
  lrn = learner_lib.Learner(net, 32, algo=algo)
  lrn.set_params(online, target)
  st, host = _store(128, 320, 6, 7, device)
  slots = helpers.kink_free_slots(online, host, 128, 32, np.random.default_rng(8))
  s_tm1 = helpers.stacks_from(host['frames'], host['fidx'], slots, 0)
  s_t = helpers.stacks_from(host['frames'], host['fidx'], slots, 1)
  z = learner_ref.zeros_like_tree(online)
  ref = learner_ref.learner_step(online, target, z, z, s_tm1,
                                 host['action'][slots], host['reward'][slots],
                                 host['discount'][slots], s_t, algo=algo)
  before = lrn.online.clone()
  g = lrn.grad(st, torch.from_numpy(slots).to(device))
  assert torch.equal(before, lrn.online)  # gradient mode leaves params alone
  got = net.unflatten(g.cpu().numpy())
  for m in ref['grads']:
    for n in ref['grads'][m]:
      want = ref['grads'][m][n]
      np.testing.assert_allclose(got[m][n], want,
                                 atol=1e-6 + 1e-3 * np.abs(want).max(),
                                 err_msg='%s/%s' % (m, n))


@pytest.mark.parametrize('meta_batch', [8, 100, 300])
def test_meta_update_matches_oracle(device, meta_batch):
  from dqn_mgsc_zoo_amd import learner as learner_lib
  from dqn_mgsc_zoo_amd import networks
  from dqn_mgsc_zoo_amd import replay as replay_lib
  a = 6
  net = networks.dqn_atari_network(a)
  online = net.init(21)
  target = helpers.perturbed_tree(online, 22)
  mu, nu = _rand_opt_state(online, 23)
  lrn = learner_lib.Learner(net, 32, algo='dqn')
  lrn.set_params(online, target)
  lrn.set_opt_state(mu, nu)
  meta = learner_lib.MetaLearner(lrn, meta_batch, learner_lib.adam(2.5e-4))
  rng = np.random.default_rng(24)
  am = (1e-3 * rng.standard_normal(meta_batch)).astype(np.float32)
  av = (1e-6 * rng.random(meta_batch)).astype(np.float32)
  meta.set_state({'count': 2, 'mu': am, 'nu': av})

  capacity = max(256, 2 * meta_batch)  # 300: two chunks of 256, the second padded
  st, host = _store(capacity, 2 * capacity + 128, a, 25, device)
  slots = rng.choice(capacity, meta_batch, replace=False).astype(np.int32)
  cap_logits = 1000
  logits = rng.standard_normal(cap_logits).astype(np.float32)
  pos = rng.choice(cap_logits, meta_batch, replace=False).astype(np.int32)
  ot_tm1 = rng.integers(0, 256, (84, 84, 4), dtype=np.uint8)
  ot_t = rng.integers(0, 256, (84, 84, 4), dtype=np.uint8)
  ot_t[..., 3] = 0  # trailing zero padding
  ot = replay_lib.Transition(ot_tm1, 3, -1.0, 0.99, ot_t)

  mb = dict(s_tm1=helpers.stacks_from(host['frames'], host['fidx'], slots, 0),
            a_tm1=host['action'][slots], r_t=host['reward'][slots],
            discount_t=host['discount'][slots],
            s_t=helpers.stacks_from(host['frames'], host['fidx'], slots, 1))
  ref = learner_ref.meta_update(
      _f64(online), _f64(target), _f64(mu), _f64(nu), mb, logits[pos],
      dict(s_tm1=ot_tm1, a_tm1=3, r_t=-1.0, discount_t=0.99, s_t=ot_t),
      am, av, 2)

  meta.set_online_transition(ot)
  logits_d = torch.from_numpy(logits).to(device)
  p0 = [t.clone() for t in (lrn.online, lrn.target, lrn.mu, lrn.nu)]
  meta.update(st, torch.from_numpy(slots).to(device), logits_d,
              torch.from_numpy(pos).to(device))
  probs, dlogits, td, loss = [t.cpu().numpy() for t in meta.fetch_outputs()]
  for before, after in zip(p0, (lrn.online, lrn.target, lrn.mu, lrn.nu)):
    assert torch.equal(before, after)  # meta_update leaves theta / opt_state
  np.testing.assert_allclose(probs, ref['probs'], rtol=1e-5)
  np.testing.assert_allclose(td, ref['td'], atol=1e-4)
  scale = np.abs(ref['dlogits']).max()
  # measured (round 2): loss 1.5-2.3e-7 relative, dlogits 1.7-5.1e-7 of max
  np.testing.assert_allclose(loss[0], ref['loss'], rtol=2e-5)
  assert scale > 0
  np.testing.assert_allclose(dlogits, ref['dlogits'], atol=2e-5 * scale)
  new = logits_d.cpu().numpy()
  np.testing.assert_allclose(new[pos], ref['new_logits'], atol=1e-6)
  untouched = np.setdiff1d(np.arange(cap_logits), pos)
  np.testing.assert_array_equal(new[untouched], logits[untouched])
  state = meta.get_state()[0]
  assert state.count == 3
  # measured (round 2): 2.6e-10 against max |m| 2.8e-3
  np.testing.assert_allclose(state.mu, ref['adam_m'], atol=1e-5 * np.abs(ref['adam_m']).max())


@pytest.mark.parametrize('bound,meta_batch,a', [(5.0, 8, 6), (1.0 / 32, 8, 6), (5.0, 260, 6), (5.0, 8, 18)])
def test_second_order_meta_update_matches_oracle(device, bound, meta_batch, a):
  """dqn_mgsc_batched_reservoir: no stop_gradient on theta'' (HVP path);
  meta_batch 260 runs as two chunks (256 + 4 padded to 256).  A = 18 takes
  the HVP's other branches: b3 gathers Wdot2[:, a] instead of staging Wdot2
  in LDS (A > 16), and the fc2 / bias puts run in two batches (A + 1 > 9)."""
  from dqn_mgsc_zoo_amd import learner as learner_lib
  from dqn_mgsc_zoo_amd import networks
  from dqn_mgsc_zoo_amd import replay as replay_lib
  net = networks.dqn_atari_network(a)
  online = net.init(51)
  target = helpers.perturbed_tree(online, 52)
  mu, nu = _rand_opt_state(online, 53)
  lrn = learner_lib.Learner(net, 32, algo='dqn', grad_error_bound=bound)
  lrn.set_params(online, target)
  lrn.set_opt_state(mu, nu)
  meta = learner_lib.MetaLearner(lrn, meta_batch, learner_lib.adam(2.5e-4),
                                 second_order=True)
  rng = np.random.default_rng(54)
  capacity = max(128, 2 * meta_batch)
  st, host = _store(capacity, 2 * capacity + 64, a, 55, device)
  slots = rng.choice(capacity, meta_batch, replace=False).astype(np.int32)
  logits = rng.standard_normal(max(64, 2 * meta_batch)).astype(np.float32)
  pos = rng.choice(logits.size, meta_batch, replace=False).astype(np.int32)
  ot_tm1 = rng.integers(0, 256, (84, 84, 4), dtype=np.uint8)
  ot_t = rng.integers(0, 256, (84, 84, 4), dtype=np.uint8)
  oa = 2 if a == 6 else 13  # A = 18: the online action past the first put batch
  ot = replay_lib.Transition(ot_tm1, oa, 1.0, 0.99, ot_t)
  mb = dict(s_tm1=helpers.stacks_from(host['frames'], host['fidx'], slots, 0),
            a_tm1=host['action'][slots], r_t=host['reward'][slots],
            discount_t=host['discount'][slots],
            s_t=helpers.stacks_from(host['frames'], host['fidx'], slots, 1))
  ref = learner_ref.meta_update(
      _f64(online), _f64(target), _f64(mu), _f64(nu), mb, logits[pos],
      dict(s_tm1=ot_tm1, a_tm1=oa, r_t=1.0, discount_t=0.99, s_t=ot_t),
      np.zeros(meta_batch), np.zeros(meta_batch), 0, grad_error_bound=bound,
      stop_gradient=False)
  first = learner_ref.meta_update(
      _f64(online), _f64(target), _f64(mu), _f64(nu), mb, logits[pos],
      dict(s_tm1=ot_tm1, a_tm1=oa, r_t=1.0, discount_t=0.99, s_t=ot_t),
      np.zeros(meta_batch), np.zeros(meta_batch), 0, grad_error_bound=bound)
  meta.set_online_transition(ot)
  logits_d = torch.from_numpy(logits).to(device)
  meta.update(st, torch.from_numpy(slots).to(device), logits_d,
              torch.from_numpy(pos).to(device))
  probs, dlogits, td, loss = [t.cpu().numpy() for t in meta.fetch_outputs()]
  np.testing.assert_allclose(probs, ref['probs'], rtol=1e-5)
  scale = np.abs(ref['dlogits']).max()
  # measured (round 2): loss 1.4-3.1e-7 relative, dlogits 2.1e-7-1.3e-6 of max
  np.testing.assert_allclose(loss[0], ref['loss'], rtol=2e-5)
  np.testing.assert_allclose(dlogits, ref['dlogits'], atol=2e-5 * scale)
  # and the second-order answer is not the first-order one
  assert np.abs(ref['dlogits'] - first['dlogits']).max() > 0.05 * scale


@pytest.mark.parametrize('meta_lr', [2.5e-4, 200.0])
def test_meta_update_keeps_logit_buffer_state(device, meta_lr):
  """The meta-update on a logit buffer whose running state is known
  (meta_adam_chunks_kernel: Adam and the re-sums of the chunks it writes in
  one launch).  The written logits match the oracle's Adam step, the others
  are untouched, the running log-sum-exp equals a fresh fp64 scan and every
  chunk sum equals its canonical restatement bit for bit.  meta_lr = 200
  moves some logits ~200 above the running shift c: the guard trips and the
  last active block re-scans the buffer and re-sums every chunk
  (replay_circular.py:166-217 semantics are those of the plain write)."""
  from dqn_mgsc_zoo_amd import learner as learner_lib
  from dqn_mgsc_zoo_amd import networks
  from dqn_mgsc_zoo_amd import replay as replay_lib
  from dqn_mgsc_zoo_amd import replay_circular as rc
  a, m, cap_logits = 6, 100, 50_000  # 13 chunks, the last one partial
  net = networks.dqn_atari_network(a)
  online = net.init(71)
  target = helpers.perturbed_tree(online, 72)
  mu, nu = _rand_opt_state(online, 73)
  lrn = learner_lib.Learner(net, 32, algo='dqn')
  lrn.set_params(online, target)
  lrn.set_opt_state(mu, nu)
  meta = learner_lib.MetaLearner(lrn, m, learner_lib.adam(meta_lr))
  rng = np.random.default_rng(74)
  st, host = _store(256, 640, a, 75, device)
  slots = rng.choice(256, m, replace=False).astype(np.int32)
  logits = rng.standard_normal(cap_logits).astype(np.float32)
  # positions clustered in a few chunks, some chunks untouched
  pos = np.concatenate([rng.choice(np.arange(4096, 8192), 60, replace=False),
                        rng.choice(np.arange(40_000, cap_logits), 40, replace=False)]).astype(np.int32)
  rng.shuffle(pos)
  dev = rc._DeviceLogits(cap_logits, device, max_queries=32)  # pylint: disable=protected-access
  dev.load(logits)
  dev.sample_abs(rng.random(32))  # a draw re-seeds: the running state is known
  assert dev.run_state()['known'] == 1
  ot_tm1 = rng.integers(0, 256, (84, 84, 4), dtype=np.uint8)
  ot_t = rng.integers(0, 256, (84, 84, 4), dtype=np.uint8)
  ot = replay_lib.Transition(ot_tm1, 1, 1.0, 0.99, ot_t)
  mb = dict(s_tm1=helpers.stacks_from(host['frames'], host['fidx'], slots, 0),
            a_tm1=host['action'][slots], r_t=host['reward'][slots],
            discount_t=host['discount'][slots],
            s_t=helpers.stacks_from(host['frames'], host['fidx'], slots, 1))
  ref = learner_ref.meta_update(
      _f64(online), _f64(target), _f64(mu), _f64(nu), mb, logits[pos],
      dict(s_tm1=ot_tm1, a_tm1=1, r_t=1.0, discount_t=0.99, s_t=ot_t),
      np.zeros(m), np.zeros(m), 0, meta_lr=meta_lr)
  meta.set_online_transition(ot)
  pos_d = torch.from_numpy(pos).to(device)
  meta.update(st, torch.from_numpy(slots).to(device), dev.logits, pos_d,
              logit_buffer=dev)
  probs, dlogits, _, loss = [t.cpu().numpy() for t in meta.fetch_outputs()]
  np.testing.assert_allclose(probs, ref['probs'], rtol=1e-5)
  np.testing.assert_allclose(loss[0], ref['loss'], rtol=2e-5)
  scale = np.abs(ref['dlogits']).max()
  np.testing.assert_allclose(dlogits, ref['dlogits'], atol=2e-5 * scale)
  after = dev.logits.cpu().numpy()
  np.testing.assert_allclose(after[pos], ref['new_logits'], atol=1e-6 * max(1.0, meta_lr))
  keep = np.ones(cap_logits, bool)
  keep[pos] = False
  np.testing.assert_array_equal(after[keep], logits[keep])
  run = dev.run_state()
  assert run['valid'] == 1 and run['known'] == 1
  a64 = after.astype(np.float64)
  want_lse = a64.max() + np.log(np.exp(a64 - a64.max()).sum())
  assert abs(run['c'] + np.log(run['S']) - want_lse) < 1e-9 * max(1.0, abs(want_lse))
  if meta_lr > 1.0:
    assert after.max() > logits.max() + 80.0  # the guard's case was hit
    assert run['c'] == after.max()  # re-seeded about the new maximum
  t_dev, csum, _ = dev.terms()
  np.testing.assert_array_equal(csum.cpu().numpy(),
                                helpers.canonical_chunk_sums(t_dev.cpu().numpy()))
  # and the buffer samples from the new state (no re-seed needed first)
  assert dev.sample_abs(rng.random(32)).cpu().numpy().max() < cap_logits


def _meta_setup(device, m, second_order=False, a=6, seed=80):
  from dqn_mgsc_zoo_amd import learner as learner_lib
  from dqn_mgsc_zoo_amd import networks
  from dqn_mgsc_zoo_amd import replay as replay_lib
  net = networks.dqn_atari_network(a)
  online = net.init(seed)
  target = helpers.perturbed_tree(online, seed + 1)
  mu, nu = _rand_opt_state(online, seed + 2)
  lrn = learner_lib.Learner(net, 32, algo='dqn')
  lrn.set_params(online, target)
  lrn.set_opt_state(mu, nu)
  meta = learner_lib.MetaLearner(lrn, m, learner_lib.adam(2.5e-4),
                                 second_order=second_order)
  rng = np.random.default_rng(seed + 3)
  st, host = _store(256, 640, a, seed + 4, device)
  slots = rng.choice(256, m, replace=False).astype(np.int32)
  ot_tm1 = rng.integers(0, 256, (84, 84, 4), dtype=np.uint8)
  ot_t = rng.integers(0, 256, (84, 84, 4), dtype=np.uint8)
  ot = replay_lib.Transition(ot_tm1, 1, 1.0, 0.99, ot_t)
  meta.set_online_transition(ot)
  mb = dict(s_tm1=helpers.stacks_from(host['frames'], host['fidx'], slots, 0),
            a_tm1=host['action'][slots], r_t=host['reward'][slots],
            discount_t=host['discount'][slots],
            s_t=helpers.stacks_from(host['frames'], host['fidx'], slots, 1))
  trans = dict(s_tm1=ot_tm1, a_tm1=1, r_t=1.0, discount_t=0.99, s_t=ot_t)
  ref_args = (_f64(online), _f64(target), _f64(mu), _f64(nu), mb)
  return meta, st, slots, rng, ref_args, trans


def test_meta_adam_chunks_with_more_blocks_than_the_chip_holds(device):
  """the fused Adam's leader stores m, v, count and the
  running state that every active chunk block reads at entry.  With 2^26
  logits the launch has 16,384 chunk blocks, far more than are resident at
  once, the leader's chunk (pos[0]) comes first and the other active chunks
  are among the last blocks dispatched: every written logit must still be
  the oracle's single Adam step, the count must advance once and the running
  log-sum-exp must equal a fresh scan."""
  from dqn_mgsc_zoo_amd import replay_circular as rc
  m, cap_logits = 100, 1 << 26
  meta, st, slots, rng, ref_args, trans = _meta_setup(device, m, seed=90)
  logits = rng.standard_normal(cap_logits).astype(np.float32)
  nchunks = cap_logits // 4096
  pos = np.concatenate([
      [5], rng.choice(np.arange((nchunks - 40) * 4096, cap_logits), m - 1,
                      replace=False)]).astype(np.int32)
  am = (1e-3 * rng.standard_normal(m)).astype(np.float32)
  av = (1e-6 * rng.random(m)).astype(np.float32)
  meta.set_state({'count': 4, 'mu': am, 'nu': av})
  ref = learner_ref.meta_update(*ref_args, logits[pos], trans, am, av, 4)
  dev = rc._DeviceLogits(cap_logits, device, max_queries=32)  # pylint: disable=protected-access
  dev.load(logits)
  dev.sample_abs(rng.random(32))  # a draw re-seeds: the running state is known
  assert dev.run_state()['known'] == 1
  meta.update(st, torch.from_numpy(slots).to(device), dev.logits,
              torch.from_numpy(pos).to(device), logit_buffer=dev)
  assert meta.sync_status() == 0
  after = dev.logits[torch.from_numpy(pos.astype(np.int64)).to(device)].cpu().numpy()
  np.testing.assert_allclose(after, ref['new_logits'], atol=1e-6)
  state = meta.get_state()[0]
  assert state.count == 5
  np.testing.assert_allclose(state.mu, ref['adam_m'], atol=1e-5 * np.abs(ref['adam_m']).max())
  run = dev.run_state()
  assert run['valid'] == 1 and run['known'] == 1
  full = dev.logits.cpu().numpy().astype(np.float64)
  mx = full.max()
  want_lse = mx + np.log(np.exp(full - mx).sum())
  assert abs(run['c'] + np.log(run['S']) - want_lse) < 1e-9 * max(1.0, abs(want_lse))


def test_meta_sync_status_reports_and_clears_a_stalled_wait(device):
  """the second-order meta-update's in-launch waits
  (the HVP's ddot1 hand-off, the fused Adam's entry wait) report a timeout
  through dqz_meta_sync_status, which also clears the words, so the next
  meta-update is correct again."""
  from dqn_mgsc_zoo_amd import replay_circular as rc
  m, cap_logits = 8, 20_000
  meta, st, slots, rng, ref_args, trans = _meta_setup(device, m, second_order=True, seed=100)
  logits = rng.standard_normal(cap_logits).astype(np.float32)
  pos = rng.choice(cap_logits, m, replace=False).astype(np.int32)
  ref = learner_ref.meta_update(*ref_args, logits[pos], trans, np.zeros(m), np.zeros(m), 0,
                                stop_gradient=False)
  dev = rc._DeviceLogits(cap_logits, device, max_queries=32)  # pylint: disable=protected-access
  slots_d = torch.from_numpy(slots).to(device)
  pos_d = torch.from_numpy(pos).to(device)

  def fresh_run():
    dev.load(logits)
    dev.sample_abs(rng.random(32))
    meta.set_state({'count': 0, 'mu': np.zeros(m, np.float32), 'nu': np.zeros(m, np.float32)})
    meta.update(st, slots_d, dev.logits, pos_d, logit_buffer=dev)

  fresh_run()
  assert meta.sync_status() == 0
  meta.debug_stall(poison=True, spin_max=2000)
  fresh_run()
  assert meta.sync_status() & 1  # reported ...
  assert meta.sync_status() == 0  # ... and cleared by the read
  meta.debug_stall(poison=False, spin_max=0)
  fresh_run()
  assert meta.sync_status() == 0
  _, dlogits, _, loss = [t.cpu().numpy() for t in meta.fetch_outputs()]
  np.testing.assert_allclose(loss[0], ref['loss'], rtol=2e-5)
  np.testing.assert_allclose(dlogits, ref['dlogits'], atol=2e-5 * np.abs(ref['dlogits']).max())
  after = dev.logits.cpu().numpy()
  np.testing.assert_allclose(after[pos], ref['new_logits'], atol=1e-6)
