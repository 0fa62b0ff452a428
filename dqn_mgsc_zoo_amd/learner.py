"""Device learner: owns params / optimizer state and drives libdqz.

`Learner.step(store, slots)` is the jitted `update` of the reference
(dqn/agent.py:109-119, double_q/agent.py, prioritized/agent.py:115-127):
forward of online(s_tm1) and target(s_t) [and online(s_t)], TD loss with
clip_gradient, backward and centered RMSProp, in place.  Everything runs in
libdqz.so on the current HIP stream; there is no host fallback.
"""

import ctypes

import numpy as np
import torch

from dqn_mgsc_zoo_amd import _native
from dqn_mgsc_zoo_amd import networks as networks_lib
from dqn_mgsc_zoo_amd import optim_state

ALGOS = {'dqn': _native.ALGO_DQN, 'double': _native.ALGO_DOUBLE,
         'per': _native.ALGO_PER}


class RMSPropConfig:
  """optax.rmsprop(learning_rate, decay, eps, centered=True) stand-in."""

  def __init__(self, learning_rate, decay=0.9, eps=1e-8, centered=False):
    if not centered:
      raise NotImplementedError(
          'only centered RMSProp is on the hot path (dqn/run_atari.py:208-213)')
    self.learning_rate = float(learning_rate)
    self.decay = float(decay)
    self.eps = float(eps)
    self.centered = True


def rmsprop(learning_rate, decay=0.9, eps=1e-8, centered=False):
  return RMSPropConfig(learning_rate, decay, eps, centered)


class Learner:
  """Online/target params + RMSProp moments in HBM and a libdqz handle."""

  def __init__(self, network: networks_lib.NetworkSpec, batch_size, algo='dqn',
               optimizer=None, grad_error_bound=1.0 / 32, device='cuda'):
    if algo not in ALGOS:
      raise ValueError('algo must be one of %s' % sorted(ALGOS))
    if (algo == 'dqn') == network.shared_bias:
      raise ValueError(
          "algo 'dqn' uses dqn_atari_network; 'double'/'per' use "
          'double_dqn_atari_network (shared bias)')
    optimizer = optimizer or rmsprop(2.5e-4, 0.95, 0.01 / 32**2, True)
    self.network = network
    self.algo = algo
    self.batch_size = int(batch_size)
    self.optimizer = optimizer
    self.grad_error_bound = float(grad_error_bound)
    self.device = torch.device(device)
    self.offsets, self.sizes, self.total = network.layout()
    self.online = torch.zeros((self.total,), dtype=torch.float32, device=self.device)
    self.target = torch.zeros_like(self.online)
    self.mu = torch.zeros_like(self.online)
    self.nu = torch.zeros_like(self.online)
    self.q_tm1 = torch.zeros((self.batch_size, network.num_actions),
                             dtype=torch.float32, device=self.device)
    self.td = torch.zeros((self.batch_size,), dtype=torch.float32, device=self.device)
    self.loss = torch.zeros((1,), dtype=torch.float32, device=self.device)
    cfg = _native.DqzLearnerConfig(
        self.batch_size, network.num_actions, ALGOS[algo],
        optimizer.learning_rate, optimizer.decay, optimizer.eps,
        float(grad_error_bound))
    handle = ctypes.c_void_p()
    _native.check(_native.lib().dqz_learner_create(ctypes.byref(cfg),
                                                   ctypes.byref(handle)))
    self._h = handle
    self._params_c = _native.DqzParams(
        self.online.data_ptr(), self.target.data_ptr(), self.mu.data_ptr(),
        self.nu.data_ptr())

  def __del__(self):
    h = getattr(self, '_h', None)
    if h is not None and h.value and _native is not None and _native._lib is not None:  # pylint: disable=protected-access
      _native.lib().dqz_learner_destroy(h)
      self._h = None

  # -- state -------------------------------------------------------------

  def set_params(self, tree, target_tree=None):
    flat = torch.from_numpy(self.network.flatten(tree))
    self.online.copy_(flat)
    if target_tree is None:
      self.target.copy_(flat)
    else:
      self.target.copy_(torch.from_numpy(self.network.flatten(target_tree)))

  def set_opt_state(self, mu_tree, nu_tree):
    self.mu.copy_(torch.from_numpy(self.network.flatten(mu_tree)))
    self.nu.copy_(torch.from_numpy(self.network.flatten(nu_tree)))

  def params_tree(self, which='online'):
    t = {'online': self.online, 'target': self.target, 'mu': self.mu,
         'nu': self.nu}[which]
    return self.network.unflatten(t.detach().cpu().numpy())

  def sync_target(self, stream=None):
    """target <- online (dqn/agent.py:155-156)."""
    _native.check(_native.lib().dqz_target_copy(
        _native.ptr(self.target), _native.ptr(self.online), self.total,
        _native.stream_handle(stream)))

  # -- hot path ------------------------------------------------------------

  def step(self, store, slots, weights=None, stream=None, write_back=None):
    """One learner step on replay `slots` (device int32 [B]).

    write_back (PER only): (tree, cap, indices, alpha, max_seen_dev) — the
    priority write-back of this step's |td| (dqz_per_write_back's arguments)
    folded into the backward launch (dqz_learner_step_per)."""
    if slots.dtype != torch.int32 or slots.numel() != self.batch_size:
      raise ValueError('slots must be a device int32 tensor of batch size')
    if self.algo == 'per' and weights is None:
      raise ValueError('PER step needs importance weights')
    if write_back is not None:
      tree, cap, indices, alpha, max_seen = write_back
      _native.check(_native.lib().dqz_learner_step_per(
          self._h, ctypes.byref(self._params_c), store.c_ref(),
          _native.ptr(slots), _native.ptr(weights), _native.ptr(tree), int(cap),
          _native.ptr(indices), float(alpha), _native.ptr(max_seen),
          _native.stream_handle(stream)))
      return
    _native.check(_native.lib().dqz_learner_step(
        self._h, ctypes.byref(self._params_c), store.c_ref(),
        _native.ptr(slots), _native.ptr(weights), _native.stream_handle(stream)))

  def step_uniform(self, store, base, size, capacity, seed, counter, slots_out,
                   stream=None):
    """Uniform sample + learner step in one pass (sampler fused into conv1).

    Draws exactly what `sample_uniform(base, size, capacity, B, seed,
    counter, ...)` would, writes them to `slots_out` and advances `counter`.
    """
    if slots_out.dtype != torch.int32 or slots_out.numel() != self.batch_size:
      raise ValueError('slots_out must be a device int32 tensor of batch size')
    _native.check(_native.lib().dqz_learner_step_uniform(
        self._h, ctypes.byref(self._params_c), store.c_ref(), int(base),
        int(size), int(capacity), int(seed) & (2**64 - 1), _native.ptr(counter),
        _native.ptr(slots_out), _native.stream_handle(stream)))

  def step_logits(self, store, logit_buffer, slots_out, seed=0, counter=None,
                  uniforms=None, stream=None):
    """Learned-logit sample + learner step, the draw inside the forward
    launch (dqz_learner_step_logits): draws what
    logit_buffer.sample_slots_philox(seed, counter, slots_out) — or, given
    device f64 `uniforms` [B] (a Generator's draws), sample_abs(uniforms) —
    would, writes them to `slots_out` and (Philox) advances `counter`."""
    if slots_out.dtype != torch.int32 or slots_out.numel() != self.batch_size:
      raise ValueError('slots_out must be a device int32 tensor of batch size')
    if (counter is None) == (uniforms is None):
      raise ValueError('pass exactly one of counter (Philox) and uniforms')
    _native.check(_native.lib().dqz_learner_step_logits(
        self._h, ctypes.byref(self._params_c), store.c_ref(),
        logit_buffer.handle, _native.ptr(logit_buffer.logits),
        int(seed) & (2**64 - 1), _native.ptr(counter), _native.ptr(uniforms),
        _native.ptr(slots_out), _native.stream_handle(stream)))

  def step_per_draw(self, store, draw, stream=None):
    """A whole prioritized learn in one learner step
    (dqz_learner_step_per_draw): the PER draw inside the forward launch, the
    IS weights in the head, the write-back inside the backward launch.
    `draw` is a _native.DqzPerDraw (see
    replay.PrioritizedTransitionReplay.per_draw)."""
    if self.algo != 'per':
      raise ValueError('step_per_draw needs a PER learner')
    _native.check(_native.lib().dqz_learner_step_per_draw(
        self._h, ctypes.byref(self._params_c), store.c_ref(), ctypes.byref(draw),
        _native.stream_handle(stream)))

  def grad(self, store, slots, weights=None, out=None, stream=None):
    """jax.grad(loss_fn) of the same step into a flat tensor (no update)."""
    if slots.dtype != torch.int32 or slots.numel() != self.batch_size:
      raise ValueError('slots must be a device int32 tensor of batch size')
    out = torch.zeros_like(self.online) if out is None else out
    _native.check(_native.lib().dqz_learner_grad(
        self._h, ctypes.byref(self._params_c), store.c_ref(),
        _native.ptr(slots), _native.ptr(weights), _native.ptr(out),
        _native.stream_handle(stream)))
    return out

  def profile(self, store, slots, weights=None, iters=20, stream=None):
    """Average ms per phase (HIP events on the launch stream), dict."""
    out = (ctypes.c_float * _native.NUM_PHASES)()
    _native.check(_native.lib().dqz_learner_profile(
        self._h, ctypes.byref(self._params_c), store.c_ref(),
        _native.ptr(slots), _native.ptr(weights), int(iters), out,
        _native.stream_handle(stream)))
    ms = [float(x) for x in out]
    names = list(_native.PHASE_NAMES)
    # phases merged into another launch report 0 and are left out
    return {n: t for n, t in zip(names, ms) if t > 0.0}

  def fetch_outputs(self, stream=None):
    """Copies (q_tm1, td, loss) of the last step into self tensors."""
    _native.check(_native.lib().dqz_learner_outputs(
        self._h, _native.ptr(self.q_tm1), _native.ptr(self.td),
        _native.ptr(self.loss), _native.stream_handle(stream)))
    return self.q_tm1, self.td, self.loss

  def sync_status(self):
    """0 if every in-launch backward hand-off completed (synchronises)."""
    st = ctypes.c_int(0)
    _native.check(_native.lib().dqz_learner_sync_status(self._h, ctypes.byref(st)))
    return st.value

  def debug_stall(self, sample, spin_max=0):
    """Test hook (dqz_learner_debug_stall): poison `sample`'s dy2 hand-off
    counter (sample >= 0) and cap the bounded spin at `spin_max` polls."""
    _native.check(_native.lib().dqz_learner_debug_stall(self._h, int(sample), int(spin_max)))

  def q_values(self, states, params=None, stream=None):
    """network.apply(params, s).q_values for uint8 [n,84,84,4] device states."""
    params = self.online if params is None else params
    states = states.contiguous()
    n = int(states.shape[0])
    out = torch.empty((n, self.network.num_actions), dtype=torch.float32,
                      device=self.device)
    for i in range(0, n, self.batch_size):
      j = min(n, i + self.batch_size)
      _native.check(_native.lib().dqz_forward(
          self._h, _native.ptr(params), _native.ptr(states[i:j]), j - i,
          _native.ptr(out[i:j]), _native.stream_handle(stream)))
    return out

  def _params_tensor(self, params):
    """Flat device parameters from None (online), a flat tensor, a device
    tree of views (agent.online_params: no copy) or a host tree."""
    if params is None:
      return self.online
    if isinstance(params, torch.Tensor):
      return params
    leaf = next(iter(next(iter(params.values())).values()))
    if isinstance(leaf, torch.Tensor):
      flat = self.network.flat_of_device_tree(params)
      if flat is not None:
        return flat
      params = {m: {n: v.detach().cpu().numpy() for n, v in d.items()}
                for m, d in params.items()}
    return torch.from_numpy(self.network.flatten(params)).to(self.device)

  def q_values_host(self, observation, params=None):
    """Q-values of one host uint8 [84,84,4] state (the actor's select_action)."""
    obs = np.ascontiguousarray(observation, dtype=np.uint8)
    if obs.ndim == 3:
      obs = obs[None]
    if getattr(self, '_obs_buf', None) is None or self._obs_buf.shape[0] < obs.shape[0]:
      self._obs_buf = torch.empty((max(obs.shape[0], 1), 84, 84, 4),
                                  dtype=torch.uint8, device=self.device)
    buf = self._obs_buf[:obs.shape[0]]
    buf.copy_(torch.from_numpy(obs))
    q = self.q_values(buf, self._params_tensor(params))
    out = q.cpu().numpy()
    return out[0] if observation.ndim == 3 else out

  def act(self, observation, epsilon, seed, counter, params=None):
    """select_action on device (dqn/agent.py:121-131): (action, max_a q) for
    one host uint8 [84,84,4] observation, the eps-greedy draw being number
    `counter` of the Philox stream `seed` (dqz_act).  The observation is
    read and the result written in place in pinned host buffers: one launch
    chain and one stream synchronisation per call, no staging copies."""
    if getattr(self, '_act_in', None) is None:
      self._act_in = torch.empty((1, 84, 84, 4), dtype=torch.uint8,
                                 pin_memory=True)
      self._act_in_np = self._act_in.numpy()
      self._act_out = torch.zeros((2,), dtype=torch.int32, pin_memory=True)
      self._act_out_np = self._act_out.numpy()
    self._act_in_np[0] = observation
    _native.check(_native.lib().dqz_act(
        self._h, _native.ptr(self._params_tensor(params)),
        ctypes.c_void_p(self._act_in.data_ptr()), 1, float(epsilon),
        int(seed) & (2**64 - 1), int(counter) & (2**64 - 1),
        ctypes.c_void_p(self._act_out.data_ptr()), _native.stream_handle()))
    torch.cuda.current_stream(self.device).synchronize()
    return int(self._act_out_np[0]), float(self._act_out_np.view(np.float32)[1])

  def q_values_slots(self, store, slots, which, params=None, stream=None):
    params = self.online if params is None else params
    n = int(slots.numel())
    out = torch.empty((n, self.network.num_actions), dtype=torch.float32,
                      device=self.device)
    _native.check(_native.lib().dqz_forward_slots(
        self._h, _native.ptr(params), store.c_ref(), _native.ptr(slots), n,
        int(which), _native.ptr(out), _native.stream_handle(stream)))
    return out


def sample_uniform(base, size, capacity, n, seed, counter, out, stream=None):
  """Device Philox uniform sampler (replay.py:119-125 distribution)."""
  _native.check(_native.lib().dqz_sample_uniform(
      int(base), int(size), int(capacity), int(n), int(seed) & (2**64 - 1),
      _native.ptr(counter), _native.ptr(out), _native.stream_handle(stream)))
  return out


class AdamConfig:
  """optax.adam(learning_rate, b1, b2, eps) stand-in (eps_root = 0)."""

  def __init__(self, learning_rate, b1=0.9, b2=0.999, eps=1e-8, eps_root=0.0):
    if eps_root != 0.0:
      raise NotImplementedError('eps_root is not used by the reference')
    self.learning_rate = float(learning_rate)
    self.b1 = float(b1)
    self.b2 = float(b2)
    self.eps = float(eps)


def adam(learning_rate, b1=0.9, b2=0.999, eps=1e-8, eps_root=0.0):
  return AdamConfig(learning_rate, b1, b2, eps, eps_root)


class MetaLearner:
  """MGSC meta-update on device (dqn_mgsc_batched/agent.py:104-220, 302-334).

  second_order=True is the reservoir agent's meta_loss_fn (no stop_gradient
  on theta'', dqn_mgsc_batched_reservoir/agent.py): the gradient also flows
  through the online transition's gradient at theta' (a Hessian-vector
  product, hvp.hpp).

  Holds the meta optimizer state (optax ScaleByAdamState(count, mu, nu) over
  the M meta-batch logits, shared across calls exactly as the reference's
  `self._meta_opt_state`) and a one-slot frame store for the newest
  transition.  `update` reads the learner's online/target params and RMSProp
  state, never modifies them, and writes the Adam-updated logits back into
  the replay's device logit buffer at the meta batch's positions
  (replay.update_priorities(indices, new_meta_params)).
  """

  def __init__(self, learner: Learner, meta_batch_size, meta_optimizer=None,
               second_order=False):
    from dqn_mgsc_zoo_amd import store as store_lib  # pylint: disable=g-import-not-at-top
    if learner.algo != 'dqn':
      raise ValueError('the MGSC agents use q_learning on dqn_atari_network')
    meta_optimizer = meta_optimizer or adam(2.5e-4)
    self.learner = learner
    self.meta_batch_size = int(meta_batch_size)
    self.meta_optimizer = meta_optimizer
    self.second_order = bool(second_order)
    dev = learner.device
    m = self.meta_batch_size
    self.adam_mu = torch.zeros((m,), dtype=torch.float32, device=dev)
    self.adam_nu = torch.zeros((m,), dtype=torch.float32, device=dev)
    self.adam_count = torch.zeros((1,), dtype=torch.int32, device=dev)
    self.probs = torch.zeros((m,), dtype=torch.float32, device=dev)
    self.dlogits = torch.zeros((m,), dtype=torch.float32, device=dev)
    self.td = torch.zeros((m,), dtype=torch.float32, device=dev)
    self.loss = torch.zeros((1,), dtype=torch.float32, device=dev)
    self.online_store = store_lib.FrameStore(1, 8, device=dev)
    self.online_store.fidx[0].copy_(torch.arange(8, dtype=torch.int32))
    self.online_slot = torch.zeros((1,), dtype=torch.int32, device=dev)
    opt = learner.optimizer
    cfg = _native.DqzMetaConfig(
        m, learner.network.num_actions, opt.learning_rate, opt.decay, opt.eps,
        learner.grad_error_bound, meta_optimizer.learning_rate,
        meta_optimizer.b1, meta_optimizer.b2, meta_optimizer.eps,
        int(bool(second_order)))
    handle = ctypes.c_void_p()
    _native.check(_native.lib().dqz_meta_create(ctypes.byref(cfg),
                                                ctypes.byref(handle)))
    self._h = handle

  def __del__(self):
    h = getattr(self, '_h', None)
    if h is not None and h.value and _native is not None and _native._lib is not None:  # pylint: disable=protected-access
      _native.lib().dqz_meta_destroy(h)
      self._h = None

  def set_online_transition(self, transition):
    """Uploads the newest host transition (uint8 [84,84,4] stacks): its eight
    channel frames (s_tm1 0..3, s_t 4..7) as pool rows 0..7 of the one-slot
    store plus its {a, r, d} record, in one launch that reads pinned staging
    in place (FrameStore.put / dqz_store_put): no host wait on queued work."""
    s_tm1 = np.asarray(transition.s_tm1, np.uint8)
    s_t = np.asarray(transition.s_t, np.uint8)
    frames = [(c, s_tm1[..., c]) for c in range(4)] + [(4 + c, s_t[..., c]) for c in range(4)]
    self.online_store.put(0, range(8), int(transition.a_tm1), float(transition.r_t),
                          float(transition.discount_t), frames)

  def update(self, store, slots, logits, positions, stream=None,
             logit_buffer=None):
    """One meta_update on replay `slots` (device int32 [M]); logits updated
    in place at `positions` (device int32 [M], distinct).  `logit_buffer`
    (the replay's device logit buffer, replay_circular._DeviceLogits) keeps
    its running log-sum-exp and chunk sums current through the write; when
    it is omitted and `logits` is a live buffer's tensor, that buffer is
    used (a raw tensor kept from `replay.logits` must not bypass the state
    its samplers read)."""
    m = self.meta_batch_size
    if slots.dtype != torch.int32 or slots.numel() != m:
      raise ValueError('slots must be a device int32 tensor of meta batch size')
    if positions.dtype != torch.int32 or positions.numel() != m:
      raise ValueError('positions must be a device int32 tensor [M]')
    if logits.dtype != torch.float32:
      raise ValueError('logits must be float32')
    if logit_buffer is not None and logits.data_ptr() != logit_buffer.logits.data_ptr():
      raise ValueError('logit_buffer does not own these logits')
    if logit_buffer is None:
      from dqn_mgsc_zoo_amd import replay_circular  # pylint: disable=g-import-not-at-top
      logit_buffer = replay_circular.logit_buffer_of(logits)
    lrn = self.learner
    _native.check(_native.lib().dqz_meta_update(
        self._h, ctypes.byref(lrn._params_c), store.c_ref(),  # pylint: disable=protected-access
        _native.ptr(slots), self.online_store.c_ref(),
        _native.ptr(self.online_slot), _native.ptr(logits),
        _native.ptr(positions), _native.ptr(self.adam_mu),
        _native.ptr(self.adam_nu), _native.ptr(self.adam_count),
        None if logit_buffer is None else logit_buffer.handle,
        _native.stream_handle(stream)))

  def fetch_outputs(self, stream=None):
    """(probs [M], dL/dlogits [M], meta-batch td [M], meta loss [1])."""
    _native.check(_native.lib().dqz_meta_outputs(
        self._h, _native.ptr(self.probs), _native.ptr(self.dlogits),
        _native.ptr(self.td), _native.ptr(self.loss),
        _native.stream_handle(stream)))
    return self.probs, self.dlogits, self.td, self.loss

  def sync_status(self):
    """0 if every bounded wait of the meta-update completed and every loss
    was finite since the previous check (dqz_meta_sync_status: the batch
    and one-transition learners' health words and the meta handle's own;
    synchronises; a non-zero word also clears every hand-off word)."""
    st = ctypes.c_int(0)
    _native.check(_native.lib().dqz_meta_sync_status(self._h, ctypes.byref(st)))
    return st.value

  def debug_stall(self, poison=True, spin_max=0):
    """Test hook (dqz_meta_debug_stall): cap every bounded wait of the
    meta handle at `spin_max` polls (0 restores the default) and, with
    `poison`, make the next update's HVP ddot1 and Adam entry waits run out."""
    _native.check(_native.lib().dqz_meta_debug_stall(self._h, int(bool(poison)), int(spin_max)))

  def get_state(self):
    """optax.adam's state, (ScaleByAdamState(count, mu, nu), EmptyState()),
    with host arrays (dqn_mgsc_batched/agent.py:80,390)."""
    return optim_state.adam_state(int(self.adam_count.item()),
                                  self.adam_mu.cpu().numpy(),
                                  self.adam_nu.cpu().numpy())

  def set_state(self, state):
    count, mu, nu = optim_state.adam_moments(state)
    self.adam_count.fill_(count)
    self.adam_mu.copy_(torch.as_tensor(np.asarray(mu, np.float32)))
    self.adam_nu.copy_(torch.as_tensor(np.asarray(nu, np.float32)))
