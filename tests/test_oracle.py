"""CPU: the fp64 oracle vs an independent torch autograd restatement.

The reference holds no Q-value / gradient golden vectors (networks_test.py
pins only shapes and the shared-bias output), so the oracle's network, loss
and optimizer math is cross-checked against torch.nn.functional +
autograd, written from the same reference call sites.
"""

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import learner_ref
from tests import helpers

_T = 'sequential/sequential'
_H = 'sequential/sequential_1'


def _init(num_actions, shared, seed):
  rng = np.random.default_rng(seed)
  shapes = {
      _T + '/conv2_d': ((8, 8, 4, 32), 256), _T + '/conv2_d_1': ((4, 4, 32, 64), 512),
      _T + '/conv2_d_2': ((3, 3, 64, 64), 576), _H + '/linear': ((3136, 512), 3136),
      _H + '/linear_1': ((512, num_actions), 512)}
  tree = {}
  for mod, (shape, fan) in shapes.items():
    bnd = 1 / np.sqrt(fan)
    tree[mod] = {'w': rng.uniform(-bnd, bnd, shape).astype(np.float32)}
    if not (shared and mod.endswith('linear_1')):
      tree[mod]['b'] = rng.uniform(-bnd, bnd, shape[-1:]).astype(np.float32)
  if shared:
    tree[_H] = {'b': rng.uniform(-0.04, 0.04, (1,)).astype(np.float32)}
  return tree


def _torch_q(tree, s, shared):
  x = torch.as_tensor(s).to(torch.float64).permute(0, 3, 1, 2) / 255.0
  for mod, stride in ((_T + '/conv2_d', 4), (_T + '/conv2_d_1', 2), (_T + '/conv2_d_2', 1)):
    w = tree[mod]['w'].permute(3, 2, 0, 1)  # HWIO -> OIHW
    x = F.relu(F.conv2d(x, w, tree[mod]['b'], stride=stride))
  flat = x.permute(0, 2, 3, 1).reshape(x.shape[0], -1)  # Haiku Flatten of NHWC
  h = F.relu(flat @ tree[_H + '/linear']['w'] + tree[_H + '/linear']['b'])
  b2 = tree[_H]['b'] if shared else tree[_H + '/linear_1']['b']
  return h @ tree[_H + '/linear_1']['w'] + b2


class _ClipGrad(torch.autograd.Function):
  @staticmethod
  def forward(ctx, x, lo, hi):
    ctx.lo, ctx.hi = lo, hi
    return x.clone()

  @staticmethod
  def backward(ctx, g):
    return g.clamp(ctx.lo, ctx.hi), None, None


@pytest.mark.parametrize('algo', ['dqn', 'double', 'per'])
def test_oracle_matches_torch_autograd(algo):
  shared = algo != 'dqn'
  a = 6
  online = _init(a, shared, 1)
  target = helpers.perturbed_tree(online, 2)
  rng = np.random.default_rng(3)
  b = 4
  s_tm1 = rng.integers(0, 256, (b, 84, 84, 4), dtype=np.uint8)
  s_t = rng.integers(0, 256, (b, 84, 84, 4), dtype=np.uint8)
  s_t[0, :, :, 2:] = 0  # trailing zero padding
  act = rng.integers(0, a, b)
  r = np.array([1.0, 0.0, -1.0, 0.0])
  d = np.array([0.99, 0.0, 0.99, 0.99])
  w = rng.uniform(0.3, 1.0, b) if algo == 'per' else None
  zeros = learner_ref.zeros_like_tree(online)
  # a large error bound exercises both sides of clip_gradient
  bound = 0.05
  ref = learner_ref.learner_step(online, target, zeros, zeros, s_tm1, act, r, d,
                                 s_t, algo=algo, weights=w,
                                 grad_error_bound=bound)

  tp = {m: {n: torch.tensor(v, dtype=torch.float64, requires_grad=True)
            for n, v in dd.items()} for m, dd in online.items()}
  tt = {m: {n: torch.tensor(v, dtype=torch.float64) for n, v in dd.items()}
        for m, dd in target.items()}
  q_tm1 = _torch_q(tp, s_tm1, shared)
  with torch.no_grad():
    q_tgt = _torch_q(tt, s_t, shared)
    if algo == 'dqn':
      v = q_tgt.max(dim=1).values
    else:
      sel = _torch_q(tp, s_t, shared).argmax(dim=1)
      v = q_tgt[torch.arange(b), sel]
    target_v = torch.as_tensor(r) + torch.as_tensor(d) * v
  td = target_v - q_tm1[torch.arange(b), torch.as_tensor(act)]
  td_c = _ClipGrad.apply(td, -bound, bound)
  losses = 0.5 * td_c**2
  if w is not None:
    losses = losses * torch.as_tensor(w)
  loss = losses.mean()
  loss.backward()

  np.testing.assert_allclose(ref['q_tm1'], q_tm1.detach().numpy(), atol=1e-10)
  np.testing.assert_allclose(ref['td'], td.detach().numpy(), atol=1e-10)
  np.testing.assert_allclose(ref['loss'], loss.item(), rtol=1e-10)
  for m in online:
    for n in online[m]:
      np.testing.assert_allclose(ref['grads'][m][n], tp[m][n].grad.numpy(),
                                 atol=1e-12, rtol=1e-8, err_msg=m + '/' + n)


def test_rmsprop_and_adam_formulas():
  p = {'l': {'w': np.array([1.0, -2.0, 0.5])}}
  g = {'l': {'w': np.array([0.1, -0.3, 0.0])}}
  z = learner_ref.zeros_like_tree(p)
  newp, mu, nu = learner_ref.rmsprop_centered(p, g, z, z, 0.1, 0.95, 1e-4)
  gg = g['l']['w']
  m = 0.05 * gg
  v = 0.05 * gg * gg
  np.testing.assert_allclose(mu['l']['w'], m)
  np.testing.assert_allclose(nu['l']['w'], v)
  np.testing.assert_allclose(newp['l']['w'],
                             p['l']['w'] - 0.1 * gg / np.sqrt(v - m * m + 1e-4))
  x, m1, v1, c = learner_ref.adam(np.zeros(2), np.array([1.0, -1.0]),
                                  np.zeros(2), np.zeros(2), 0, lr=0.01)
  # first bias-corrected Adam step moves by lr * g/|g| (up to eps)
  np.testing.assert_allclose(x, [-0.01, 0.01], rtol=1e-6)
  assert c == 1


def _torch_rms(p, g, mu, nu, lr, decay, eps):
  m = (1 - decay) * g + decay * mu
  v = (1 - decay) * g * g + decay * nu
  return p - lr * g * torch.rsqrt(v - m * m + eps), m, v


def test_oracle_meta_update_matches_torch_autograd():
  """MGSC meta_loss_fn (dqn_mgsc_batched/agent.py:160-199) restated in torch
  and differentiated by autograd w.r.t. the logits, vs the oracle's analytic
  chain (per-example dot products + softmax backward)."""
  a, m_size = 6, 4
  online = _init(a, False, 11)
  target = helpers.perturbed_tree(online, 12)
  rng = np.random.default_rng(13)
  meta = dict(s_tm1=rng.integers(0, 256, (m_size, 84, 84, 4), dtype=np.uint8),
              a_tm1=rng.integers(0, a, m_size),
              r_t=np.array([1.0, 0.0, -1.0, 0.0]),
              discount_t=np.array([0.99, 0.0, 0.99, 0.99]),
              s_t=rng.integers(0, 256, (m_size, 84, 84, 4), dtype=np.uint8))
  ot = dict(s_tm1=rng.integers(0, 256, (84, 84, 4), dtype=np.uint8), a_tm1=2,
            r_t=1.0, discount_t=0.99,
            s_t=rng.integers(0, 256, (84, 84, 4), dtype=np.uint8))
  mu = {m: {n: 1e-3 * rng.standard_normal(np.shape(v)) for n, v in d.items()}
        for m, d in online.items()}
  nu = {m: {n: mu[m][n]**2 + 1e-6 * rng.random(np.shape(v))
            for n, v in d.items()} for m, d in mu.items()}
  logits = rng.standard_normal(m_size).astype(np.float32)
  am, av = 0.1 * rng.standard_normal(m_size), 0.01 * rng.random(m_size)
  lr, decay, eps, bound = 2.5e-4, 0.95, 0.01 / 32**2, 0.05
  ref = learner_ref.meta_update(online, target, mu, nu, meta, logits, ot, am,
                                av, 3, lr=lr, decay=decay, eps=eps,
                                grad_error_bound=bound)

  keys = [(m, n) for m in online for n in online[m]]
  th = {k: torch.tensor(online[k[0]][k[1]], dtype=torch.float64) for k in keys}

  def tree(flat):
    out = {}
    for (m, n), v in flat.items():
      out.setdefault(m, {})[n] = v
    return out

  def single_grad(params, target_params, s_tm1, act, r, d, s_t):
    p = {k: v.detach().requires_grad_(True) for k, v in params.items()}
    q = _torch_q(tree(p), s_tm1[None], False)
    with torch.no_grad():
      v = _torch_q(tree(target_params), s_t[None], False).max(dim=1).values
    td = (r + d * v) - q[0, act]
    loss = (0.5 * _ClipGrad.apply(td, -bound, bound)**2).mean()
    gs = torch.autograd.grad(loss, [p[k] for k in keys])
    return dict(zip(keys, gs))

  x = torch.tensor(logits, dtype=torch.float64, requires_grad=True)
  c = x.max()
  probs = torch.exp(x - (c + torch.log(torch.sum(torch.exp(x - c)))))
  tt = {k: torch.tensor(target[k[0]][k[1]], dtype=torch.float64) for k in keys}
  per = [single_grad(th, tt, meta['s_tm1'][i], meta['a_tm1'][i], meta['r_t'][i],
                     meta['discount_t'][i], meta['s_t'][i]) for i in range(m_size)]
  big_g = {k: sum(probs[i] * per[i][k] for i in range(m_size)) for k in keys}
  tmu = {k: torch.tensor(mu[k[0]][k[1]]) for k in keys}
  tnu = {k: torch.tensor(nu[k[0]][k[1]]) for k in keys}
  th_p, mu_p, nu_p = {}, {}, {}
  for k in keys:
    th_p[k], mu_p[k], nu_p[k] = _torch_rms(th[k], big_g[k], tmu[k], tnu[k], lr,
                                           decay, eps)
  g2 = single_grad(th_p, th, ot['s_tm1'], ot['a_tm1'], ot['r_t'],
                   ot['discount_t'], ot['s_t'])
  loss = 0.0
  for k in keys:
    th_pp, _, _ = _torch_rms(th_p[k].detach(), g2[k], mu_p[k].detach(),
                             nu_p[k].detach(), lr, decay, eps)
    loss = loss + torch.sum((th_p[k] - th_pp.detach())**2)
  loss.backward()
  np.testing.assert_allclose(ref['probs'], probs.detach().numpy(), rtol=1e-12)
  np.testing.assert_allclose(ref['loss'], loss.item(), rtol=1e-9)
  np.testing.assert_allclose(ref['dlogits'], x.grad.numpy(), rtol=1e-6,
                             atol=1e-6 * np.abs(x.grad.numpy()).max())
  assert np.abs(ref['dlogits']).max() > 0
  # adam on the logits, optax 0.1.2 bias-corrected, count 3 -> 4
  b1, b2 = 0.9, 0.999
  mm = b1 * am + (1 - b1) * ref['dlogits']
  vv = b2 * av + (1 - b2) * ref['dlogits']**2
  want = logits - 2.5e-4 * (mm / (1 - b1**4)) / (np.sqrt(vv / (1 - b2**4)) + 1e-8)
  np.testing.assert_allclose(ref['new_logits'], want, rtol=1e-12)
  assert ref['adam_count'] == 4


def test_oracle_hvp_matches_torch_double_backward():
  a = 6
  params = _init(a, False, 31)
  rng = np.random.default_rng(32)
  s = rng.integers(0, 256, (1, 84, 84, 4), dtype=np.uint8)
  tangent = {m: {n: rng.standard_normal(np.shape(v)) for n, v in d.items()}
             for m, d in params.items()}
  q, cache = learner_ref.forward(params, s)
  e = np.zeros_like(q)
  e[0, 4] = 1.0
  got = learner_ref.hvp(params, cache, e, tangent)
  keys = [(m, n) for m in params for n in params[m]]
  tp = {k: torch.tensor(params[k[0]][k[1]], dtype=torch.float64, requires_grad=True) for k in keys}
  tree = {}
  for (m, n), v in tp.items():
    tree.setdefault(m, {})[n] = v
  qt = _torch_q(tree, s, False)[0, 4]
  gs = torch.autograd.grad(qt, [tp[k] for k in keys], create_graph=True)
  dot = sum((g * torch.tensor(tangent[k[0]][k[1]])).sum() for g, k in zip(gs, keys))
  hs = torch.autograd.grad(dot, [tp[k] for k in keys], allow_unused=True)
  for h, k in zip(hs, keys):
    want = np.zeros(np.shape(params[k[0]][k[1]])) if h is None else h.numpy()
    np.testing.assert_allclose(got[k[0]][k[1]], want, rtol=1e-8,
                               atol=1e-10 * (1 + np.abs(want).max()), err_msg=str(k))


def test_oracle_second_order_meta_update_matches_torch_autograd():
  """dqn_mgsc_batched_reservoir/agent.py: meta_loss_fn without stop_gradient
  on theta'' -- autograd differentiates through g'(theta') (double backward)."""
  a, m_size = 6, 3
  online = _init(a, False, 41)
  target = helpers.perturbed_tree(online, 42)
  rng = np.random.default_rng(43)
  meta = dict(s_tm1=rng.integers(0, 256, (m_size, 84, 84, 4), dtype=np.uint8),
              a_tm1=rng.integers(0, a, m_size),
              r_t=np.array([1.0, 0.0, -1.0]),
              discount_t=np.array([0.99, 0.99, 0.0]),
              s_t=rng.integers(0, 256, (m_size, 84, 84, 4), dtype=np.uint8))
  ot = dict(s_tm1=rng.integers(0, 256, (84, 84, 4), dtype=np.uint8), a_tm1=1,
            r_t=0.5, discount_t=0.99,
            s_t=rng.integers(0, 256, (84, 84, 4), dtype=np.uint8))
  mu = {m: {n: 1e-3 * rng.standard_normal(np.shape(v)) for n, v in d.items()}
        for m, d in online.items()}
  nu = {m: {n: mu[m][n]**2 + 1e-6 * rng.random(np.shape(v))
            for n, v in d.items()} for m, d in mu.items()}
  logits = rng.standard_normal(m_size).astype(np.float32)
  lr, decay, eps = 2.5e-4, 0.95, 0.01 / 32**2
  for bound in (5.0, 1e-3):  # online TD inside / outside the clip bound
    ref = learner_ref.meta_update(online, target, mu, nu, meta, logits, ot,
                                  np.zeros(m_size), np.zeros(m_size), 0, lr=lr,
                                  decay=decay, eps=eps, grad_error_bound=bound,
                                  stop_gradient=False)
    keys = [(m, n) for m in online for n in online[m]]

    def tree(flat):
      out = {}
      for (m, n), v in flat.items():
        out.setdefault(m, {})[n] = v
      return out

    th = {k: torch.tensor(online[k[0]][k[1]], dtype=torch.float64) for k in keys}
    tt = {k: torch.tensor(target[k[0]][k[1]], dtype=torch.float64) for k in keys}

    def loss_of(params, tparams, s_tm1, act, r, d, s_t):
      q = _torch_q(tree(params), s_tm1[None], False)
      with torch.no_grad():
        v = _torch_q(tree(tparams), s_t[None], False).max(dim=1).values
      td = (r + d * v) - q[0, act]
      return (0.5 * _ClipGrad.apply(td, -bound, bound)**2).mean()

    x = torch.tensor(logits, dtype=torch.float64, requires_grad=True)
    c = x.max()
    probs = torch.exp(x - (c + torch.log(torch.sum(torch.exp(x - c)))))
    per = []
    for i in range(m_size):
      p = {k: v.clone().requires_grad_(True) for k, v in th.items()}
      li = loss_of(p, tt, meta['s_tm1'][i], meta['a_tm1'][i], meta['r_t'][i],
                   meta['discount_t'][i], meta['s_t'][i])
      per.append(dict(zip(keys, torch.autograd.grad(li, [p[k] for k in keys]))))
    big_g = {k: sum(probs[i] * per[i][k] for i in range(m_size)) for k in keys}
    th_p, mu_p, nu_p = {}, {}, {}
    for k in keys:
      th_p[k], mu_p[k], nu_p[k] = _torch_rms(th[k], big_g[k], torch.tensor(mu[k[0]][k[1]]),
                                             torch.tensor(nu[k[0]][k[1]]), lr, decay, eps)
    l2 = loss_of(th_p, th, ot['s_tm1'], ot['a_tm1'], ot['r_t'], ot['discount_t'], ot['s_t'])
    g2 = dict(zip(keys, torch.autograd.grad(l2, [th_p[k] for k in keys], create_graph=True)))
    loss = 0.0
    for k in keys:
      th_pp, _, _ = _torch_rms(th_p[k], g2[k], mu_p[k], nu_p[k], lr, decay, eps)
      loss = loss + torch.sum((th_p[k] - th_pp)**2)
    loss.backward()
    np.testing.assert_allclose(ref['loss'], loss.item(), rtol=1e-9)
    want = x.grad.numpy()
    np.testing.assert_allclose(ref['dlogits'], want, rtol=1e-6,
                               atol=1e-6 * np.abs(want).max(), err_msg='bound=%g' % bound)
    assert np.abs(want).max() > 0


@pytest.mark.parametrize('algo', ['dqn', 'double', 'per'])
def test_torch_cpu_baseline_matches_oracle(algo):
  """bench.py's CPU baseline (oracle/torch_cpu.py) computes the same update."""
  from oracle import torch_cpu
  shared = algo != 'dqn'
  a = 6
  online = _init(a, shared, 11)
  target = helpers.perturbed_tree(online, 12)
  rng = np.random.default_rng(13)
  b = 8
  s_tm1 = rng.integers(0, 256, (b, 84, 84, 4), dtype=np.uint8)
  s_t = rng.integers(0, 256, (b, 84, 84, 4), dtype=np.uint8)
  act = rng.integers(0, a, b)
  r = rng.choice([-1.0, 0.0, 1.0], b)
  d = np.where(rng.random(b) < 0.2, 0.0, 0.99)
  w = rng.uniform(0.3, 1.0, b) if algo == 'per' else None
  lrn = torch_cpu.TorchCpuLearner(online, target, algo=algo)
  mu = learner_ref.zeros_like_tree(online)
  nu = learner_ref.zeros_like_tree(online)
  params = online
  for _ in range(2):
    ref = learner_ref.learner_step(params, target, mu, nu, s_tm1, act, r, d,
                                   s_t, algo=algo, weights=w)
    q, td, loss = lrn.step(
        torch.from_numpy(s_tm1), torch.from_numpy(act), torch.from_numpy(r).float(),
        torch.from_numpy(d).float(), torch.from_numpy(s_t),
        None if w is None else torch.from_numpy(w).float())
    np.testing.assert_allclose(q.numpy(), ref['q_tm1'], atol=1e-4)
    np.testing.assert_allclose(td.numpy(), ref['td'], atol=1e-4)
    np.testing.assert_allclose(float(loss), ref['loss'], rtol=1e-4)
    params, mu, nu = ref['params'], ref['mu'], ref['nu']
  got = lrn.params_tree()
  for m in params:
    for n in params[m]:
      np.testing.assert_allclose(got[m][n], params[m][n], atol=2e-6,
                                 err_msg=m + '/' + n)
