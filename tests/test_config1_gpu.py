"""GPU: BASELINE config 1 on HIP — the dqn agent with a 1M-capacity uniform
replay, driven by parts.run_loop through processors.atari.

The reference builds `TransitionReplay(capacity=1e6)` with a RandomState
(dqn/run_atari.py:204-206), the centered RMSProp of :208-213, batch 32,
learn period 16, and drives `agent.Dqn` with `parts.run_loop` over raw
210x160 RGB Atari frames through `processors.atari` (:252-294).  Here the
same objects run on the device path: the observation math of
processors.atari on device (dqz_atari_frame), every transition in the 1M
frame store, the learner step on the slots the replay's RandomState drew.
Checked: the replay's own invariants (`check_valid`), one learn step
through those slots against the fp64 oracle on host restacked transitions,
and the hard target copy at its period (dqn/agent.py:155-156).
Learning starts at a small `min_replay_capacity_fraction` (1e-4 of 1M =
100 transitions) so the test runs in seconds; the replay's capacity, and so
its frame pool, slot arithmetic and sampling range, is the config's 1M.
"""

import numpy as np
import pytest
import torch

from oracle import learner_ref

pytestmark = pytest.mark.gpu

LR, DECAY, EPS, BOUND = 2.5e-4, 0.95, 0.01 / 32**2, 1.0 / 32
CAPACITY = 1_000_000
LEARN_PERIOD = 16
TARGET_PERIOD = 640  # frames; 40,000 in the reference (learn period x 2,500)


def _params_host(tree):
  return {m: {n: v.astype(np.float64) for n, v in d.items()}
          for m, d in tree.items()}


def _make(seed=1, min_replay_fraction=1e-4, target_period=TARGET_PERIOD, eps_decay=20_000):
  from dqn_mgsc_zoo_amd import learner as learner_lib
  from dqn_mgsc_zoo_amd import networks
  from dqn_mgsc_zoo_amd import parts
  from dqn_mgsc_zoo_amd import processors
  from dqn_mgsc_zoo_amd import replay as replay_lib
  from dqn_mgsc_zoo_amd.dqn import agent as agent_lib
  random_state = np.random.RandomState(seed)
  replay = replay_lib.TransitionReplay(
      CAPACITY, replay_lib.Transition(None, None, None, None, None),
      random_state)
  agent = agent_lib.Dqn(
      preprocessor=processors.atari(),  # device observation frame
      sample_network_input=np.zeros((84, 84, 4), np.uint8),
      network=networks.dqn_atari_network(6),
      optimizer=learner_lib.rmsprop(LR, DECAY, EPS, centered=True),
      transition_accumulator=replay_lib.TransitionAccumulator(),
      replay=replay, batch_size=32,
      exploration_epsilon=parts.LinearSchedule(
          begin_t=0, decay_steps=eps_decay, begin_value=1.0, end_value=0.1),
      min_replay_capacity_fraction=min_replay_fraction, learn_period=LEARN_PERIOD,
      target_network_update_period=target_period, grad_error_bound=BOUND,
      rng_key=np.array([0, seed], np.uint32))
  return agent, replay


def test_config1_dqn_agent_1m_replay_run_loop(device):
  from dqn_mgsc_zoo_amd import parts
  from dqn_mgsc_zoo_amd import synthetic
  agent, replay = _make()
  assert replay.capacity == CAPACITY
  lrn = agent.learner
  learns, syncs = [], []
  orig_learn, orig_sync = agent._learn, lrn.sync_target  # pylint: disable=protected-access

  def learn():
    learns.append(agent._frame_t)  # pylint: disable=protected-access
    orig_learn()

  def sync(stream=None):
    orig_sync(stream)
    # the copy is a hard alias of the online parameters at this frame
    syncs.append((agent._frame_t, torch.equal(lrn.target, lrn.online)))  # pylint: disable=protected-access

  agent._learn = learn  # pylint: disable=protected-access
  lrn.sync_target = sync
  env = synthetic.SyntheticAtari(episode_len=700, seed=3)
  loop = parts.run_loop(agent, env, max_steps_per_episode=0)
  p0 = lrn.online.clone()
  for _ in range(1600):
    next(loop)
  torch.cuda.synchronize()

  # the replay: every emitted transition stored, invariants of replay.py
  assert replay.on_device and replay.frame_store is not None
  assert 100 <= replay.size < CAPACITY
  ok, msg = replay.check_valid()
  assert ok, msg
  # learning started once 100 transitions were in, every 16th frame after
  assert learns and all(f % LEARN_PERIOD == 0 for f in learns)
  assert len(learns) >= 60
  assert not torch.equal(p0, lrn.online) and torch.isfinite(lrn.online).all()
  # target copies at frames 640 and 1280 (after learning started), each a
  # copy of the online parameters of that frame
  assert [f for f, _ in syncs] == [640, 1280]
  assert all(eq for _, eq in syncs)
  assert agent.check_learner_health() == 0

  # one learn step through slots the replay's RandomState drew, against the
  # fp64 oracle on host restacks of those transitions
  online = _params_host(lrn.params_tree('online'))
  target = _params_host(lrn.params_tree('target'))
  mu = _params_host(lrn.params_tree('mu'))
  nu = _params_host(lrn.params_tree('nu'))
  ids, slots = replay.sample_slots(32)
  assert int(np.max(slots.cpu().numpy())) < CAPACITY
  host = list(replay.get(ids))
  s_tm1 = np.stack([h.s_tm1 for h in host])
  s_t = np.stack([h.s_t for h in host])
  a = np.array([h.a_tm1 for h in host])
  r = np.array([h.r_t for h in host], np.float32)
  d = np.array([h.discount_t for h in host], np.float32)
  ref = learner_ref.learner_step(online, target, mu, nu, s_tm1, a, r, d, s_t,
                                 algo='dqn', lr=LR, decay=DECAY, eps=EPS,
                                 grad_error_bound=BOUND)
  lrn.step(agent._store(), slots)  # pylint: disable=protected-access
  q, td, loss = lrn.fetch_outputs()
  np.testing.assert_allclose(q.cpu().numpy(), ref['q_tm1'], atol=1e-4)
  np.testing.assert_allclose(td.cpu().numpy(), ref['td'], atol=1e-4)
  assert float(loss.item()) == pytest.approx(ref['loss'], rel=1e-4)
  got = lrn.params_tree('online')
  for m in ref['params']:
    for n in ref['params'][m]:
      np.testing.assert_allclose(got[m][n], ref['params'][m][n], atol=2e-6,
                                 err_msg='%s/%s' % (m, n))
  # the device gather of those slots is the host restack, bit for bit
  st = agent._store()  # pylint: disable=protected-access
  np.testing.assert_array_equal(st.gather_stacks(slots, 0).cpu().numpy(), s_tm1)
  np.testing.assert_array_equal(st.gather_stacks(slots, 1).cpu().numpy(), s_t)


def test_config1_at_the_reference_schedule(device):
  """Config 1 at dqn/run_atari.py's own schedule:
  min_replay_capacity_fraction 0.05 of the 1M replay (learning starts once
  50,000 transitions are in, dqn/agent.py:149-150), learn period 16, target
  period 40,000 frames (dqn/run_atari.py:77-79; the copy only once learning
  runs, dqn/agent.py:155-156), epsilon 1 -> 0.1 over 4M frames from the
  start of learning.  processors.atari repeats each action 4 times
  (processors.py), so 50,000 transitions take ~200,000 frames: 241,000
  frames through parts.run_loop, no learn step before the replay holds
  50,000 transitions, then one every 16 frames, a target copy at every
  multiple of 40,000 frames once learning runs (240,000 among them), each
  equal to the online parameters of its frame, the replay's invariants, a
  finite loss and a clean health word."""
  from dqn_mgsc_zoo_amd import parts
  from dqn_mgsc_zoo_amd import synthetic
  min_frac, period = 0.05, 40_000
  agent, replay = _make(seed=7, min_replay_fraction=min_frac, target_period=period,
                        eps_decay=4_000_000)
  lrn = agent.learner
  learns, syncs, sizes = [], [], []
  orig_learn, orig_sync = agent._learn, lrn.sync_target  # pylint: disable=protected-access

  def learn():
    learns.append(agent._frame_t)  # pylint: disable=protected-access
    sizes.append(replay.size)
    orig_learn()

  def sync(stream=None):
    orig_sync(stream)
    syncs.append((agent._frame_t, torch.equal(lrn.target, lrn.online)))  # pylint: disable=protected-access

  agent._learn = learn  # pylint: disable=protected-access
  lrn.sync_target = sync
  env = synthetic.SyntheticAtari(episode_len=27_000, seed=8)
  loop = parts.run_loop(agent, env, max_steps_per_episode=108_000)
  for _ in range(241_000):
    next(loop)
  torch.cuda.synchronize()
  need = int(min_frac * CAPACITY)
  assert learns and min(sizes) >= need
  assert all(f % LEARN_PERIOD == 0 for f in learns)
  # one learn per 16 frames from the first frame the replay was full enough
  assert learns == list(range(learns[0], learns[-1] + 1, LEARN_PERIOD))
  assert len(learns) > 2_000
  assert 240_000 in [f for f, _ in syncs]
  assert all(f % period == 0 and f >= learns[0] and eq for f, eq in syncs)
  ok, msg = replay.check_valid()
  assert ok, msg
  _, _, loss = lrn.fetch_outputs()
  assert np.isfinite(float(loss.item()))
  assert torch.isfinite(lrn.online).all()
  assert agent.check_learner_health() == 0
