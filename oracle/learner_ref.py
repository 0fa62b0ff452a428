"""ORACLE — test infrastructure only.  Never imported by the product.

fp64 numpy restatement of the DQN learner step that the HIP path must match
(BASELINE.json north_star: Q-values / TD errors within 1e-4 fp32).  Only
`tests/`, `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline leg may
use it, and only as the checker / CPU baseline.

What it restates (reference file:line; the arithmetic itself lives in
un-vendored dependencies pinned at docker_requirements.txt:6-26):
  * networks.dqn_torso / dqn_value_head (networks.py:181-221): x/255,
    Haiku Conv2D NHWC/HWIO VALID + bias + ReLU x3, Flatten (h,w,c), Linear +
    ReLU, Linear; shared-bias head (networks.py:120-134) -- dm-haiku 0.0.6.
  * rlax 0.1.2 q_learning / double_q_learning / clip_gradient / l2_loss as
    called at dqn/agent.py:85-107, double_q/agent.py:85-107,
    prioritized/agent.py:86-113.  clip_gradient is identity forward and clips
    the incoming cotangent backward.
  * optax 0.1.2 rmsprop(centered=True) = scale_by_stddev + scale(-lr)
    (dqn/run_atari.py:208-213): mu=(1-d)g+d mu, nu=(1-d)g^2+d nu,
    u = -lr g rsqrt(nu - mu^2 + eps).
  * optax 0.1.2 adam (dqn_mgsc_batched/run_atari.py:241-243).

Parity status: the reference's own tests pin only parameter names/shapes and
the shared-bias output (networks_test.py:36-103); no Q-value, gradient or
optimizer golden vector exists in the reference, and JAX is not installable
here, so this restatement is *parity unpinned* against the reference's
numbers.  It is cross-checked against an independent torch-CPU autograd
implementation in tests/test_oracle.py.
"""

import numpy as np

CONV_SPECS = (  # (kernel, stride, c_in, c_out)
    (8, 4, 4, 32),
    (4, 2, 32, 64),
    (3, 1, 64, 64),
)
_TORSO = 'sequential/sequential'
_HEAD = 'sequential/sequential_1'
CONV_NAMES = (_TORSO + '/conv2_d', _TORSO + '/conv2_d_1', _TORSO + '/conv2_d_2')


def _im2col(x, k, s):
  """x [B,H,W,C] -> [B,OH,OW,k*k*C] ordered (kh, kw, c) like HWIO."""
  b, h, w, c = x.shape
  oh, ow = (h - k) // s + 1, (w - k) // s + 1
  cols = np.empty((b, oh, ow, k, k, c), dtype=x.dtype)
  for kh in range(k):
    for kw in range(k):
      cols[:, :, :, kh, kw, :] = x[:, kh:kh + s * (oh - 1) + 1:s,
                                   kw:kw + s * (ow - 1) + 1:s, :]
  return cols.reshape(b, oh, ow, k * k * c)


def _col2im(dcols, x_shape, k, s):
  b, h, w, c = x_shape
  oh, ow = dcols.shape[1], dcols.shape[2]
  dcols = dcols.reshape(b, oh, ow, k, k, c)
  dx = np.zeros(x_shape, dtype=dcols.dtype)
  for kh in range(k):
    for kw in range(k):
      dx[:, kh:kh + s * (oh - 1) + 1:s, kw:kw + s * (ow - 1) + 1:s, :] += (
          dcols[:, :, :, kh, kw, :])
  return dx


def head_params(params, shared_bias):
  w2 = np.asarray(params[_HEAD + '/linear_1']['w'], np.float64)
  if shared_bias:
    b2 = np.asarray(params[_HEAD]['b'], np.float64)
  else:
    b2 = np.asarray(params[_HEAD + '/linear_1']['b'], np.float64)
  return w2, b2


def forward(params, s, shared_bias=False):
  """Q-values and intermediates for uint8 states s [B,84,84,4]."""
  x = np.asarray(s).astype(np.float32).astype(np.float64) / 255.0
  cache = {'x0': x}
  for i, ((k, st, _, co), name) in enumerate(zip(CONV_SPECS, CONV_NAMES)):
    w = np.asarray(params[name]['w'], np.float64)
    b = np.asarray(params[name]['b'], np.float64)
    cols = _im2col(x, k, st)
    z = cols @ w.reshape(-1, co) + b
    x = np.maximum(z, 0.0)
    cache['cols%d' % i] = cols
    cache['y%d' % i] = x
  flat = x.reshape(x.shape[0], -1)
  w1 = np.asarray(params[_HEAD + '/linear']['w'], np.float64)
  b1 = np.asarray(params[_HEAD + '/linear']['b'], np.float64)
  h1 = np.maximum(flat @ w1 + b1, 0.0)
  w2, b2 = head_params(params, shared_bias)
  q = h1 @ w2 + b2
  cache.update(flat=flat, h1=h1)
  return q, cache


def relu_margin(params, s):
  """Smallest |pre-activation| / largest |pre-activation| over the four ReLU
  layers of the forward on uint8 states s.  The ReLU derivative jumps at 0,
  so an f32 implementation can take the other side of the kink than fp64 for
  a pre-activation within its rounding of 0 (~1e-7 of the layer's scale) and
  move a whole unit's gradient contribution: gradient parity tests draw
  inputs that keep this margin (tests/helpers.kink_free_slots)."""
  x = np.asarray(s).astype(np.float64) / 255.0
  margin = np.inf
  for (k, st, _, co), name in zip(CONV_SPECS, CONV_NAMES):
    z = _im2col(x, k, st) @ np.asarray(params[name]['w'], np.float64).reshape(-1, co) + \
        np.asarray(params[name]['b'], np.float64)
    margin = min(margin, np.abs(z).min() / np.abs(z).max())
    x = np.maximum(z, 0.0)
  z = x.reshape(x.shape[0], -1) @ np.asarray(params[_HEAD + '/linear']['w'], np.float64) + \
      np.asarray(params[_HEAD + '/linear']['b'], np.float64)
  return min(margin, np.abs(z).min() / np.abs(z).max())


def backward(params, cache, dq, shared_bias=False):
  """Gradient tree of sum(dq * q) w.r.t. the online parameters."""
  grads = {}
  h1, flat = cache['h1'], cache['flat']
  w2, _ = head_params(params, shared_bias)
  grads[_HEAD + '/linear_1'] = {'w': h1.T @ dq}
  if shared_bias:
    grads[_HEAD] = {'b': np.array([dq.sum()])}
  else:
    grads[_HEAD + '/linear_1']['b'] = dq.sum(axis=0)
  dh1 = (dq @ w2.T) * (h1 > 0)
  w1 = np.asarray(params[_HEAD + '/linear']['w'], np.float64)
  grads[_HEAD + '/linear'] = {'w': flat.T @ dh1, 'b': dh1.sum(axis=0)}
  dflat = dh1 @ w1.T
  dy = dflat.reshape(cache['y2'].shape)
  for i in (2, 1, 0):
    k, st, _, co = CONV_SPECS[i]
    y = cache['y%d' % i]
    dz = dy * (y > 0)
    cols = cache['cols%d' % i]
    grads[CONV_NAMES[i]] = {
        'w': (cols.reshape(-1, cols.shape[-1]).T @ dz.reshape(-1, co)).reshape(
            np.asarray(params[CONV_NAMES[i]]['w']).shape),
        'b': dz.reshape(-1, co).sum(axis=0),
    }
    if i > 0:
      w = np.asarray(params[CONV_NAMES[i]]['w'], np.float64).reshape(-1, co)
      dcols = dz @ w.T
      x_shape = cache['y%d' % (i - 1)].shape
      dy = _col2im(dcols, x_shape, k, st)
  return grads


def td_loss(q_tm1, a_tm1, r_t, discount_t, q_target_t, q_selector_t=None,
            weights=None, grad_error_bound=1.0 / 32):
  """TD errors, mean loss and d loss / d q_tm1.

  q_learning: target = r + d * max_a q_target_t; double_q_learning: target =
  r + d * q_target_t[argmax q_selector_t] (first maximum).  loss =
  mean(0.5 td^2 [* w]).  The cotangent at td is clip(w td / B, +-bound)
  because rlax.clip_gradient sits between td and l2_loss.
  """
  b = q_tm1.shape[0]
  idx = np.arange(b)
  a_tm1 = np.asarray(a_tm1, np.int64)
  if q_selector_t is None:
    v = q_target_t.max(axis=1)
  else:
    v = q_target_t[idx, np.argmax(q_selector_t, axis=1)]
  target = np.asarray(r_t, np.float64) + np.asarray(discount_t, np.float64) * v
  td = target - q_tm1[idx, a_tm1]
  w = np.ones(b) if weights is None else np.asarray(weights, np.float64)
  loss = np.mean(0.5 * td * td * w)
  g_td = np.clip(w * td / b, -grad_error_bound, grad_error_bound)
  dq = np.zeros_like(q_tm1)
  dq[idx, a_tm1] = -g_td
  return td, loss, dq


def rmsprop_centered(params, grads, mu, nu, lr, decay, eps):
  """optax 0.1.2 rmsprop(centered=True); returns new (params, mu, nu)."""
  new_p, new_mu, new_nu = {}, {}, {}
  for mod in params:
    new_p[mod], new_mu[mod], new_nu[mod] = {}, {}, {}
    for name in params[mod]:
      g = np.asarray(grads[mod][name], np.float64)
      m = (1.0 - decay) * g + decay * np.asarray(mu[mod][name], np.float64)
      v = (1.0 - decay) * g * g + decay * np.asarray(nu[mod][name], np.float64)
      new_mu[mod][name] = m
      new_nu[mod][name] = v
      new_p[mod][name] = (np.asarray(params[mod][name], np.float64) -
                          lr * g / np.sqrt(v - m * m + eps))
  return new_p, new_mu, new_nu


def adam(params, grads, m, v, count, lr, b1=0.9, b2=0.999, eps=1e-8):
  """optax 0.1.2 adam on a flat array; returns (params, m, v, count)."""
  g = np.asarray(grads, np.float64)
  m = b1 * np.asarray(m, np.float64) + (1 - b1) * g
  v = b2 * np.asarray(v, np.float64) + (1 - b2) * g * g
  count = count + 1
  m_hat = m / (1 - b1**count)
  v_hat = v / (1 - b2**count)
  return np.asarray(params, np.float64) - lr * m_hat / (np.sqrt(v_hat) + eps), m, v, count


def learner_step(online, target, mu, nu, s_tm1, a_tm1, r_t, discount_t, s_t,
                 algo='dqn', weights=None, lr=2.5e-4, decay=0.95,
                 eps=0.01 / 32**2, grad_error_bound=1.0 / 32):
  """One `update` (dqn/agent.py:109-119; prioritized/agent.py:115-127).

  algo: 'dqn' (q_learning, per-action bias), 'double' or 'per'
  (double_q_learning, shared-bias head; 'per' weights the loss).
  Returns dict(q_tm1, td, loss, params, mu, nu, grads).
  """
  shared = algo != 'dqn'
  q_tm1, cache = forward(online, s_tm1, shared)
  q_target_t, _ = forward(target, s_t, shared)
  q_sel = None
  if algo != 'dqn':
    q_sel, _ = forward(online, s_t, shared)
  td, loss, dq = td_loss(q_tm1, a_tm1, r_t, discount_t, q_target_t, q_sel,
                         weights if algo == 'per' else None, grad_error_bound)
  grads = backward(online, cache, dq, shared)
  new_p, new_mu, new_nu = rmsprop_centered(online, grads, mu, nu, lr, decay,
                                           eps)
  return dict(q_tm1=q_tm1, q_target_t=q_target_t, td=td, loss=loss,
              params=new_p, mu=new_mu, nu=new_nu, grads=grads)


def zeros_like_tree(tree):
  return {m: {n: np.zeros_like(np.asarray(v, np.float64)) for n, v in d.items()}
          for m, d in tree.items()}


def _tree_map(f, *trees):
  return {m: {n: f(*(t[m][n] for t in trees)) for n in trees[0][m]}
          for m in trees[0]}


def _tree_dot(a, b):
  return sum(float(np.sum(np.asarray(a[m][n], np.float64) *
                          np.asarray(b[m][n], np.float64)))
             for m in a for n in a[m])


def softmax_logsumexp(logits):
  """replay_circular.JNPprobabilities_from_logits (replay_circular.py:79-86)."""
  x = np.asarray(logits, np.float64)
  c = x.max()
  return np.exp(x - (c + np.log(np.sum(np.exp(x - c)))))


def rmsprop_update_jacobian(g, mu, nu, lr, decay, eps):
  """d u / d g of the centered RMSProp update u = -lr g rsqrt(D) (diagonal).

  mu' = d mu + c g, nu' = d nu + c g^2, D = nu' - mu'^2 + eps (c = 1 - d):
  du/dg = -lr D^{-3/2} (D - c g (g - mu')).
  """
  c = 1.0 - decay
  m = c * g + decay * mu
  v = c * g * g + decay * nu
  dd = v - m * m + eps
  return -lr * (dd - c * g * (g - m)) / dd**1.5


def hvp(params, cache, dq, tangent, shared_bias=False):
  """Hessian-vector product of sum(dq * q(theta)) along `tangent` (a tree).

  Forward-over-reverse restatement of `forward`/`backward`: tangents of every
  pre-activation with the ReLU masks held fixed, then the tangent of each
  backward signal and of each weight gradient (product rule).  Used for the
  second-order meta-gradient of dqn_mgsc_batched_reservoir/agent.py (no
  stop_gradient on theta'').
  """
  def tw(name, leaf='w'):
    return np.asarray(tangent[name][leaf], np.float64)

  def pw(name, leaf='w'):
    return np.asarray(params[name][leaf], np.float64)

  # tangent forward
  ydot = [None, None, None]
  colsdot = [None, None, None]
  prev = None
  for i, ((k, st, _, co), name) in enumerate(zip(CONV_SPECS, CONV_NAMES)):
    cols = cache['cols%d' % i]
    zdot = cols @ tw(name).reshape(-1, co) + tw(name, 'b')
    if prev is not None:
      colsdot[i] = _im2col(prev, k, st)
      zdot = zdot + colsdot[i] @ pw(name).reshape(-1, co)
    ydot[i] = zdot * (cache['y%d' % i] > 0)
    prev = ydot[i]
  flat, h1 = cache['flat'], cache['h1']
  flatdot = ydot[2].reshape(flat.shape)
  w1 = pw(_HEAD + '/linear')
  h1dot = (flat @ tw(_HEAD + '/linear') + flatdot @ w1 + tw(_HEAD + '/linear', 'b')) * (h1 > 0)
  w2, _ = head_params(params, shared_bias)
  w2dot = tw(_HEAD + '/linear_1')
  out = {}
  out[_HEAD + '/linear_1'] = {'w': h1dot.T @ dq}
  if shared_bias:
    out[_HEAD] = {'b': np.zeros(1)}
  else:
    out[_HEAD + '/linear_1']['b'] = np.zeros(dq.shape[1])
  dh1 = (dq @ w2.T) * (h1 > 0)
  dh1dot = (dq @ w2dot.T) * (h1 > 0)
  out[_HEAD + '/linear'] = {'w': flatdot.T @ dh1 + flat.T @ dh1dot,
                            'b': dh1dot.sum(axis=0)}
  dflat = dh1 @ w1.T
  dflatdot = dh1dot @ w1.T + dh1 @ tw(_HEAD + '/linear').T
  dy = dflat.reshape(cache['y2'].shape)
  dydot = dflatdot.reshape(cache['y2'].shape)
  for i in (2, 1, 0):
    k, st, _, co = CONV_SPECS[i]
    mask = cache['y%d' % i] > 0
    dz, dzdot = dy * mask, dydot * mask
    cols = cache['cols%d' % i].reshape(-1, cache['cols%d' % i].shape[-1])
    gw = cols.T @ dzdot.reshape(-1, co)
    if colsdot[i] is not None:
      gw = gw + colsdot[i].reshape(-1, cols.shape[-1]).T @ dz.reshape(-1, co)
    out[CONV_NAMES[i]] = {'w': gw.reshape(np.asarray(params[CONV_NAMES[i]]['w']).shape),
                          'b': dzdot.reshape(-1, co).sum(axis=0)}
    if i > 0:
      w = pw(CONV_NAMES[i]).reshape(-1, co)
      wdot = tw(CONV_NAMES[i]).reshape(-1, co)
      x_shape = cache['y%d' % (i - 1)].shape
      dy = _col2im(dz @ w.T, x_shape, k, st)
      dydot = _col2im(dzdot @ w.T + dz @ wdot.T, x_shape, k, st)
  return out


def meta_update(online, target, mu, nu, meta, logits, online_transition,
                adam_m, adam_v, adam_count, lr=2.5e-4, decay=0.95,
                eps=0.01 / 32**2, grad_error_bound=1.0 / 32, meta_lr=2.5e-4,
                stop_gradient=True):
  """MGSCDqn.meta_update (dqn_mgsc_batched/agent.py:104-220), fp64.

  meta: dict(s_tm1 [M,84,84,4], a_tm1, r_t, discount_t, s_t) — the meta batch.
  online_transition: the same keys for one transition (no batch axis).
  Follows the reference literally: per-example gradients g_i of
  loss_fn on a single transition (:152-158), G = sum_i p_i g_i (:171-172),
  theta' = theta + RMSProp(G; s) (:178-179), g' = grad loss_fn(theta',
  target=theta, online transition) (:183-185), theta'' =
  stop_gradient(theta' + RMSProp(g'; s')) (:189-191), loss =
  sum ||theta' - theta''||^2 (:104-110, :195).  The gradient w.r.t. the
  logits is taken analytically: dL/dtheta' = -2 u', dtheta'/dG = diag(du/dG),
  dL/dp_i = v . g_i with v = dL/dG; softmax backward; optax adam.
  Returns dict(probs, td, G, theta_p, g_p, loss, v, dlogits, new_logits,
  adam_m, adam_v, adam_count).
  """
  s_tm1 = np.asarray(meta['s_tm1'])
  m_size = s_tm1.shape[0]
  p = softmax_logsumexp(logits)
  q_tm1, _ = forward(online, s_tm1)
  q_t, _ = forward(target, np.asarray(meta['s_t']))
  td, _, _ = td_loss(q_tm1, meta['a_tm1'], meta['r_t'], meta['discount_t'], q_t,
                     None, None, grad_error_bound)
  per_example = []
  for i in range(m_size):
    qi, cache = forward(online, s_tm1[i:i + 1])
    _, _, dq = td_loss(qi, np.asarray(meta['a_tm1'])[i:i + 1],
                       np.asarray(meta['r_t'])[i:i + 1],
                       np.asarray(meta['discount_t'])[i:i + 1],
                       q_t[i:i + 1], None, None, grad_error_bound)
    per_example.append(backward(online, cache, dq))
  big_g = _tree_map(lambda *gs: sum(pi * g for pi, g in zip(p, gs)),
                    *per_example)
  theta_p, mu_p, nu_p = rmsprop_centered(online, big_g, mu, nu, lr, decay, eps)
  ot = {k: np.asarray(v)[None, ...] for k, v in online_transition.items()}
  step2 = learner_step(theta_p, online, mu_p, nu_p, ot['s_tm1'], ot['a_tm1'],
                       ot['r_t'], ot['discount_t'], ot['s_t'], lr=lr,
                       decay=decay, eps=eps, grad_error_bound=grad_error_bound)
  theta_pp = step2['params']
  u_p = _tree_map(lambda a, b: a - b, theta_pp, theta_p)
  loss = _tree_dot(u_p, u_p)
  jac = _tree_map(lambda g, m, n: rmsprop_update_jacobian(g, m, n, lr, decay,
                                                          eps),
                  big_g, _tree_map(np.asarray, mu), _tree_map(np.asarray, nu))
  if stop_gradient:
    # dL/dtheta' = -2 u' (theta'' is a constant): v = -2 u' dtheta'/dG
    v = _tree_map(lambda u, j: -2.0 * u * j, u_p, jac)
  else:
    # dqn_mgsc_batched_reservoir: L = sum u'^2 with u' = F(g'(theta'), mu', nu')
    # and mu' = d mu + c G, nu' = d nu + c G^2 (theta' cancels in theta' - theta'').
    #   dL/dG = 2u' (c dF/dmu' + 2 c G dF/dnu') + J (H w),  w = 2u' dF/dg',
    #   dF/dg' = -lr D^{-3/2} (D - c g' (g' - mu'')),  D = nu'' - mu''^2 + eps,
    #   c dF/dmu' + 2cG dF/dnu' = c d lr g' D^{-3/2} (G - mu''),
    #   H = alpha grad q grad q^T - clip(td') hess q  (the online transition's
    #   loss at theta', target theta; alpha = 1 inside the clip bound).
    c, d = 1.0 - decay, decay
    g_p = step2['grads']
    mu_pp, nu_pp = step2['mu'], step2['nu']
    dd = _tree_map(lambda m, n: n - m * m + eps, mu_pp, nu_pp)
    v_dir = _tree_map(lambda u, g, dv, gg, m: 2.0 * u * c * d * lr * g * dv**-1.5 * (gg - m),
                      u_p, g_p, dd, big_g, mu_pp)
    w = _tree_map(lambda u, g, dv, m: 2.0 * u * (-lr) * dv**-1.5 * (dv - c * g * (g - m)),
                  u_p, g_p, dd, mu_pp)
    q1, cache1 = forward(theta_p, ot['s_tm1'])
    e_a = np.zeros_like(q1)
    e_a[0, int(np.asarray(ot['a_tm1']).reshape(-1)[0])] = 1.0
    grad_q = backward(theta_p, cache1, e_a)
    hess_q_w = hvp(theta_p, cache1, e_a, w)
    td_p = float(np.asarray(step2['td']).reshape(-1)[0])
    alpha = 1.0 if abs(td_p) < grad_error_bound else 0.0
    clip_td = float(np.clip(td_p, -grad_error_bound, grad_error_bound))
    s1 = _tree_dot(grad_q, w)
    h_w = _tree_map(lambda gq, hq: alpha * s1 * gq - clip_td * hq, grad_q, hess_q_w)
    v = _tree_map(lambda vd, j, hw: vd + j * hw, v_dir, jac, h_w)
  dp = np.array([_tree_dot(v, g) for g in per_example])
  dlogits = p * (dp - np.dot(p, dp))
  new_logits, m, vv, count = adam(np.asarray(logits, np.float64), dlogits,
                                  adam_m, adam_v, adam_count, meta_lr)
  return dict(probs=p, td=td, G=big_g, theta_p=theta_p, g_p=step2['grads'],
              loss=loss, v=v, dp=dp, dlogits=dlogits, new_logits=new_logits,
              adam_m=m, adam_v=vv, adam_count=count)
