"""GPU: the actor path — device eps-greedy select_action (dqz_act) and the
one-launch replay add (dqz_store_put).

select_action (dqn/agent.py:121-131) draws from distrax.EpsilonGreedy with
JAX threefry keys, which cannot be reproduced here; the device draw is
checked for what the reference pins: v_t = max q exactly, the greedy action
at eps = 0, and the eps-greedy distribution (parts.epsilon_greedy_probs, the
host mirror of distrax.EpsilonGreedy, including ties).
"""

import ctypes

import numpy as np
import pytest
import torch

from tests import fake_env

pytestmark = pytest.mark.gpu


def _act_setup(batch=4, num_actions=6, seed=41):
  from dqn_mgsc_zoo_amd import learner as learner_lib
  from dqn_mgsc_zoo_amd import networks
  net = networks.dqn_atari_network(num_actions)
  params = net.init(seed)
  lrn = learner_lib.Learner(net, batch, algo='dqn')
  lrn.set_params(params)
  obs = np.random.default_rng(seed).integers(0, 256, (84, 84, 4), dtype=np.uint8)
  return net, params, lrn, obs


def test_act_matches_q_values_and_eps_greedy(device):
  from dqn_mgsc_zoo_amd import parts
  _, _, lrn, obs = _act_setup()
  q = lrn.q_values(torch.from_numpy(obs[None]).to(device))[0].cpu().numpy()
  a0, v0 = lrn.act(obs, 0.0, seed=3, counter=0)
  assert v0 == q.max() and a0 == int(np.argmax(q))
  for eps in (0.3, 1.0):
    n = 3000
    counts = np.zeros(6)
    for c in range(n):
      a, v = lrn.act(obs, eps, seed=5, counter=c)
      counts[a] += 1
      assert v == v0
    probs = parts.epsilon_greedy_probs(q, eps)
    np.testing.assert_allclose(counts / n, probs, atol=4 * np.sqrt(0.25 / n))
  # the draw is a function of (seed, counter) only
  assert lrn.act(obs, 0.5, 9, 17) == lrn.act(obs, 0.5, 9, 17)


def test_act_ties_spread_the_greedy_mass(device):
  _, params, lrn, obs = _act_setup()
  tied = {m: {n: v.copy() for n, v in d.items()} for m, d in params.items()}
  head = [m for m in tied if m.endswith('linear_1')]
  assert len(head) == 1
  tied[head[0]]['w'][...] = 0.0
  tied[head[0]]['b'][...] = 0.25  # every Q-value is exactly 0.25
  lrn.set_params(tied)
  n = 1800
  counts = np.zeros(6)
  for c in range(n):
    a, v = lrn.act(obs, 0.0, seed=1, counter=c)
    counts[a] += 1
    assert v == 0.25
  np.testing.assert_allclose(counts / n, np.full(6, 1 / 6), atol=4 * np.sqrt(0.25 / n))


def test_act_device_buffers_and_pageable_refusal(device):
  """Device input / output buffers give the same draw as the pinned ones;
  pageable host memory is refused before any kernel touches it."""
  from dqn_mgsc_zoo_amd import _native
  _, _, lrn, obs = _act_setup()
  st = torch.from_numpy(obs[None].copy()).to(device)
  out = torch.zeros((2,), dtype=torch.int32, device=device)
  _native.check(_native.lib().dqz_act(
      lrn._h, _native.ptr(lrn.online), _native.ptr(st), 1, 0.4, 7, 11,  # pylint: disable=protected-access
      _native.ptr(out), _native.stream_handle()))
  torch.cuda.synchronize()
  a, v = lrn.act(obs, 0.4, 7, 11)
  assert int(out[0].item()) == a and out.view(torch.float32)[1].item() == v
  pageable = np.ascontiguousarray(obs[None])
  with pytest.raises(_native.NativeLibraryError, match='pinned host memory'):
    _native.check(_native.lib().dqz_act(
        lrn._h, _native.ptr(lrn.online), ctypes.c_void_p(pageable.ctypes.data),  # pylint: disable=protected-access
        1, 0.4, 7, 11, _native.ptr(out), _native.stream_handle()))


def test_epsilon_greedy_actor(device):
  """parts.EpsilonGreedyActor (the evaluation actor) acts through dqz_act."""
  from dqn_mgsc_zoo_amd import networks
  from dqn_mgsc_zoo_amd import parts
  net = networks.dqn_atari_network(6)
  actor = parts.EpsilonGreedyActor(fake_env.FrameStacker(), net, 0.05,
                                   np.array([0, 3], np.uint32))
  actor.network_params = net.init(5)
  env = fake_env.FakeAtari(episode_len=9, seed=2)
  loop = parts.run_loop(actor, env, max_steps_per_episode=0)
  acts = [next(loop) for _ in range(30)]
  assert len(acts) == 30
  state = actor.get_state()
  assert state['act_count'] > 0


def test_store_put_device(device):
  """dqz_store_put: new frames from the pinned staging slots into their pool
  rows and the record at its slot, one launch per add (slots reused past
  the 64-slot ring)."""
  from dqn_mgsc_zoo_amd import store as store_lib
  st = store_lib.FrameStore(16, 40)
  rng = np.random.default_rng(3)
  frames = rng.integers(0, 256, (3, 84, 84), dtype=np.uint8)
  want = {}
  for rep in range(70):
    rows = [(5 * rep + i) % 40 for i in range(3)]
    fidx = [rows[0], rows[1], rows[2], -1, rows[1], rows[2], -1, -1]
    new = [(rows[i], frames[i] ^ np.uint8(rep)) for i in range(3)]
    st.put(rep % 16, fidx, rep % 6, -1.0 if rep % 2 else 0.5, 0.99, new)
    for r, f in new:
      want[r] = f.reshape(-1)
  torch.cuda.synchronize()
  for r, f in want.items():
    np.testing.assert_array_equal(st.frames[r].cpu().numpy(), f)
  rep = 69
  rows = [(5 * rep + i) % 40 for i in range(3)]
  assert st.fidx[rep % 16].cpu().tolist() == [rows[0], rows[1], rows[2], -1,
                                               rows[1], rows[2], -1, -1]
  assert int(st.action[rep % 16]) == rep % 6
  assert float(st.reward[rep % 16]) == -1.0
  assert float(st.discount[rep % 16]) == float(np.float32(0.99))
  with pytest.raises(Exception, match='out of range'):
    st.put(16, [0] * 8, 0, 0.0, 1.0)
