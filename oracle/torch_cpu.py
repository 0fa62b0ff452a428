"""ORACLE — test infrastructure only.  Never imported by the product.

torch-CPU fp32 restatement of the DQN learner step, used as `bench.py`'s
CPU baseline (SURVEY.md §8(d) "CPU baseline": the reference's
`--jax_platform_name=cpu` path cannot run without JAX, so the same learner
step is timed in torch fp32 on the host cores at N = all allotted threads
and N = 2, the reference's `--cpus-per-task=2`, run_dqn_normal.sh:9).

Same math as `learner_ref.learner_step` (and so as the reference's jitted
`update`, dqn/agent.py:85-119): x/255, three VALID convs + ReLU, Haiku
(h, w, c) flatten, fc1 + ReLU, fc2; rlax q_learning (or double_q_learning)
with clip_gradient on the TD cotangent (±1/32), loss mean(0.5·td²); optax
0.1.2 centered RMSProp (eps inside the sqrt).  Convolutions run NCHW with
OIHW weights (torch's native CPU layout) — a layout choice, not a different
computation: `tests/test_oracle.py` checks the step against the fp64 oracle.
"""

import numpy as np
import torch
import torch.nn.functional as F

_T = 'sequential/sequential'
_H = 'sequential/sequential_1'
_CONVS = ((_T + '/conv2_d', 4), (_T + '/conv2_d_1', 2), (_T + '/conv2_d_2', 1))


class _ClipGrad(torch.autograd.Function):
  """rlax.clip_gradient: identity forward, clipped cotangent backward."""

  @staticmethod
  def forward(ctx, x, lo, hi):
    ctx.lo, ctx.hi = lo, hi
    return x.view_as(x)

  @staticmethod
  def backward(ctx, g):
    return g.clamp(ctx.lo, ctx.hi), None, None


class TorchCpuLearner:
  """Params / RMSProp moments as fp32 torch CPU tensors; `step` is one update.

  Parameters are held in torch layout (OIHW convs; fc1 rows permuted from
  Haiku's (h, w, c) flatten to NCHW's (c, h, w)); `params_tree()` converts
  back to the Haiku tree.
  """

  def __init__(self, tree, target_tree=None, algo='dqn', lr=2.5e-4,
               decay=0.95, eps=0.01 / 32**2, grad_error_bound=1.0 / 32):
    self.algo = algo
    self.shared = algo != 'dqn'
    self.lr, self.decay, self.eps = lr, decay, eps
    self.bound = grad_error_bound
    self.params = self._to_torch(tree)
    self.target = self._to_torch(target_tree if target_tree is not None else tree)
    for p in self.params:
      p.requires_grad_(True)
    self.mu = [torch.zeros_like(p) for p in self.params]
    self.nu = [torch.zeros_like(p) for p in self.params]

  def _to_torch(self, tree):
    out = []
    for mod, _ in _CONVS:
      out.append(torch.as_tensor(np.asarray(tree[mod]['w'], np.float32)).permute(3, 2, 0, 1).contiguous())
      out.append(torch.as_tensor(np.asarray(tree[mod]['b'], np.float32)).clone())
    w1 = np.asarray(tree[_H + '/linear']['w'], np.float32).reshape(7, 7, 64, 512)
    out.append(torch.as_tensor(w1).permute(2, 0, 1, 3).reshape(3136, 512).contiguous())
    out.append(torch.as_tensor(np.asarray(tree[_H + '/linear']['b'], np.float32)).clone())
    out.append(torch.as_tensor(np.asarray(tree[_H + '/linear_1']['w'], np.float32)).clone())
    b2 = tree[_H]['b'] if self.shared else tree[_H + '/linear_1']['b']
    out.append(torch.as_tensor(np.asarray(b2, np.float32)).clone())
    return out

  def params_tree(self):
    p = [t.detach() for t in self.params]
    tree = {}
    for i, (mod, _) in enumerate(_CONVS):
      tree[mod] = {'w': p[2 * i].permute(2, 3, 1, 0).numpy().copy(),
                   'b': p[2 * i + 1].numpy().copy()}
    w1 = p[6].reshape(64, 7, 7, 512).permute(1, 2, 0, 3).reshape(3136, 512)
    tree[_H + '/linear'] = {'w': w1.numpy().copy(), 'b': p[7].numpy().copy()}
    if self.shared:
      tree[_H + '/linear_1'] = {'w': p[8].numpy().copy()}
      tree[_H] = {'b': p[9].numpy().copy()}
    else:
      tree[_H + '/linear_1'] = {'w': p[8].numpy().copy(), 'b': p[9].numpy().copy()}
    return tree

  @staticmethod
  def q_values(params, s):
    """s: uint8 [B,84,84,4] NHWC torch tensor."""
    x = s.permute(0, 3, 1, 2).to(torch.float32) / 255.0
    for i, (_, stride) in enumerate(_CONVS):
      x = F.relu(F.conv2d(x, params[2 * i], params[2 * i + 1], stride=stride))
    h = F.relu(x.reshape(x.shape[0], -1) @ params[6] + params[7])
    return h @ params[8] + params[9]

  def step(self, s_tm1, a_tm1, r_t, discount_t, s_t, weights=None):
    """One learner update in place; returns (q_tm1, td, loss)."""
    with torch.no_grad():
      q_t = self.q_values(self.target, s_t)
      if self.shared:
        sel = self.q_values(self.params, s_t).argmax(dim=1)
        v_t = q_t.gather(1, sel[:, None])[:, 0]
      else:
        v_t = q_t.max(dim=1).values
      target = r_t + discount_t * v_t
    q_tm1 = self.q_values(self.params, s_tm1)
    qa = q_tm1.gather(1, a_tm1[:, None])[:, 0]
    td = _ClipGrad.apply(target - qa, -self.bound, self.bound)
    losses = 0.5 * td * td
    if weights is not None:
      losses = losses * weights
    loss = losses.mean()
    grads = torch.autograd.grad(loss, self.params)
    d = self.decay
    with torch.no_grad():
      for p, g, m, v in zip(self.params, grads, self.mu, self.nu):
        m.mul_(d).add_(g, alpha=1.0 - d)
        v.mul_(d).addcmul_(g, g, value=1.0 - d)
        p.sub_(self.lr * g / torch.sqrt(v - m * m + self.eps))
    return q_tm1.detach(), td.detach(), loss.detach()
