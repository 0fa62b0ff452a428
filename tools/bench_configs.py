"""Per-config device timings beside bench.py's headline line.

usage (GPU box): python tools/bench_configs.py [--steps K] [--capacity C] > out.json

Prints one JSON object with, for B = 32 and a synthetic replay pre-filled to
C transitions:
  double_uniform  double_q learner step + fused uniform draw (hipGraph)
  per_double      prioritized config (3): device PER sample over a 2^20-leaf
                  fp64 sum tree (alpha-exponentiated random priorities, usp
                  1e-3, beta 0.4, normalised weights) + double-Q learner step
                  with IS weights + |td|^alpha priority write-back (hipGraph)
  mgsc_learn      MGSC config (3) learner part: one-launch softmax sample over
                  C logits (N(0,1), Philox uniforms, int32 slots) + DQN
                  learner step (hipGraph)
  mgsc_meta_*     one meta_update (M = 100 and M = 300, first / second
                  order) on a fixed meta batch (stream-timed, not captured)
Times are device time from HIP events around K steps on one stream.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from dqn_mgsc_zoo_amd import _native, learner as learner_lib, networks, synthetic  # noqa: E402

B, A = 32, 6


def timed(fn, steps, warmup, dev, graph_steps=0):
  """Device ms per call of fn (optionally replayed from a hipGraph)."""
  for _ in range(warmup):
    fn()
  torch.cuda.synchronize(dev)
  if graph_steps:
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
      fn()
    torch.cuda.current_stream(dev).wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
      for _ in range(graph_steps):
        fn()
    run = g.replay
    reps = max(1, steps // graph_steps)
    n = reps * graph_steps
  else:
    run, reps, n = fn, steps, steps
  e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  torch.cuda.synchronize(dev)
  e0.record()
  for _ in range(reps):
    run()
  e1.record()
  torch.cuda.synchronize(dev)
  ms = e0.elapsed_time(e1) / n
  return {'ms_per_step': round(ms, 5), 'steps_per_s': round(1e3 / ms, 1), 'steps': n}


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument('--steps', type=int, default=2000)
  ap.add_argument('--capacity', type=int, default=1_000_000)
  args = ap.parse_args()
  dev = torch.device('cuda:0')
  lib = _native.lib()
  cap = args.capacity
  store = synthetic.fill_episodic(cap, A, seed=0, device=dev)
  out = {'batch': B, 'num_actions': A, 'capacity': cap}

  # ---- double_q, uniform -------------------------------------------------
  net_d = networks.double_dqn_atari_network(A)
  lrn_d = learner_lib.Learner(net_d, B, algo='double', device=dev)
  lrn_d.set_params(net_d.init(seed=1))
  slots = torch.zeros((B,), dtype=torch.int32, device=dev)
  ctr = torch.zeros((1,), dtype=torch.int64, device=dev)
  print('double_uniform ...', file=sys.stderr, flush=True)
  out['double_uniform'] = timed(
      lambda: lrn_d.step_uniform(store, 0, cap, cap, 7, ctr, slots),
      args.steps, 20, dev, graph_steps=50)

  # ---- prioritized double-Q ------------------------------------------------
  tcap = 1 << max(1, (cap - 1).bit_length())
  rng = np.random.default_rng(0)
  tree = torch.zeros((2 * tcap,), dtype=torch.float64, device=dev)
  idx_all = torch.arange(cap, dtype=torch.int64, device=dev)
  pri = torch.from_numpy(rng.uniform(0.01, 2.0, cap) ** 0.6).to(dev)
  for s0 in range(0, cap, 65536):  # dqz_sumtree_set takes <= 65536 leaves per call
    n = min(65536, cap - s0)
    _native.check(lib.dqz_sumtree_set(_native.ptr(tree), tcap, _native.ptr(idx_all[s0:s0 + n]),
                                      _native.ptr(pri[s0:s0 + n]), n, _native.stream_handle()))
  lrn_p = learner_lib.Learner(net_d, B, algo='per', device=dev)
  lrn_p.set_params(net_d.init(seed=2))
  p_slots = torch.zeros((B,), dtype=torch.int32, device=dev)
  p_w = torch.zeros((B,), dtype=torch.float32, device=dev)
  p_ctr = torch.zeros((1,), dtype=torch.int64, device=dev)
  max_seen = torch.ones((1,), dtype=torch.float64, device=dev)

  def per_step():
    _native.check(lib.dqz_per_sample(
        _native.ptr(tree), tcap, 0, cap, cap, B, ctypes.c_double(1e-3), ctypes.c_double(0.4), 1, 11,
        _native.ptr(p_ctr), None, None, None, None, _native.ptr(p_slots), _native.ptr(p_w), None,
        _native.stream_handle()))
    # write-back folded into the backward launch (dqz_learner_step_per)
    lrn_p.step(store, p_slots, p_w, write_back=(tree, tcap, p_slots, 0.6, max_seen))
  print('per_double ...', file=sys.stderr, flush=True)
  out['per_double'] = timed(per_step, args.steps, 20, dev, graph_steps=50)

  # ---- MGSC learner part: softmax sample over the logits + DQN step -------
  net = networks.dqn_atari_network(A)
  lrn = learner_lib.Learner(net, B, algo='dqn', device=dev)
  lrn.set_params(net.init(seed=3))
  from dqn_mgsc_zoo_amd import replay_circular as rc  # pylint: disable=g-import-not-at-top
  lbuf = rc._DeviceLogits(cap, dev, max_queries=B)  # pylint: disable=protected-access
  lbuf.load(rng.standard_normal(cap).astype(np.float32))
  logits = lbuf.logits
  u_ctr = torch.zeros((1,), dtype=torch.int64, device=dev)
  m_slots = torch.zeros((B,), dtype=torch.int32, device=dev)

  def mgsc_learn():
    lbuf.sample_slots_philox(13, u_ctr, m_slots)  # one launch: draws + choice + int32 slots
    lrn.step(store, m_slots)
  print('mgsc_learn ...', file=sys.stderr, flush=True)
  out['mgsc_learn'] = timed(mgsc_learn, args.steps, 20, dev, graph_steps=50)

  # ---- MGSC meta_update ----------------------------------------------------
  from dqn_mgsc_zoo_amd import replay as replay_lib  # pylint: disable=g-import-not-at-top
  ot = replay_lib.Transition(rng.integers(0, 256, (84, 84, 4), dtype=np.uint8), 2, 1.0, 0.99,
                             rng.integers(0, 256, (84, 84, 4), dtype=np.uint8))
  for m_batch in (100, 300):
    for order in (0, 1):
      meta = learner_lib.MetaLearner(lrn, m_batch, learner_lib.adam(2.5e-4), second_order=bool(order))
      meta.set_online_transition(ot)
      ms = torch.from_numpy(rng.choice(cap, m_batch, replace=False).astype(np.int32)).to(dev)
      mp = ms.clone()
      t = timed(lambda: meta.update(store, ms, logits, mp, logit_buffer=lbuf), max(20, args.steps // 20), 3, dev)
      out['mgsc_meta_M%d_%s' % (m_batch, 'second' if order else 'first')] = t
      print('mgsc_meta M=%d order=%d %s' % (m_batch, order, t), file=sys.stderr, flush=True)
      del meta
  print(json.dumps(out))


if __name__ == '__main__':
  main()
