"""Micro-timings of the learned-logit and PER sampler pieces (GPU box).

usage: python tools/sampler_bench.py > out.json
Back-to-back HIP-event timings (ms per launch) at 1M logits / 2^20 leaves:
  probs          dqz_logits_probs (the producers' block-sum pass + p out)
  sample_slots   dqz_logits_sample_slots (one launch: producers + 32 queries)
  sample_inj     dqz_logits_sample (same, caller's uniforms)
  per_sample     dqz_per_sample (Philox)
and 50-step graph replays of the learner step three ways: uniform draw in
conv1 (config 2), the learned-logit draw in the forward launch
(dqz_learner_step_logits) and the stand-alone sampler + step.
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dqn_mgsc_zoo_amd import _native, learner as learner_lib, networks, synthetic  # noqa: E402
from dqn_mgsc_zoo_amd import replay_circular as rc  # noqa: E402


def b2b(fn, iters=200):
  fn()
  torch.cuda.synchronize()
  e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  e0.record()
  for _ in range(iters):
    fn()
  e1.record()
  e1.synchronize()
  return round(e0.elapsed_time(e1) / iters, 5)


def graph_rate(fn, steps=50, reps=40):
  side = torch.cuda.Stream()
  side.wait_stream(torch.cuda.current_stream())
  with torch.cuda.stream(side):
    for _ in range(3):
      fn()
  torch.cuda.current_stream().wait_stream(side)
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    for _ in range(steps):
      fn()
  g.replay()
  torch.cuda.synchronize()
  e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  e0.record()
  for _ in range(reps):
    g.replay()
  e1.record()
  e1.synchronize()
  return round(e0.elapsed_time(e1) / (steps * reps), 5)


def main():
  dev = torch.device('cuda:0')
  cap, B = 1_000_000, 32
  lib = _native.lib()
  out = {}
  dl = rc._DeviceLogits(cap, dev, max_queries=B)  # pylint: disable=protected-access
  dl.load(np.random.default_rng(0).standard_normal(cap).astype(np.float32))
  p = torch.empty_like(dl.logits)
  lse = torch.empty((1,), device=dev)
  ctr = torch.zeros((1,), dtype=torch.int64, device=dev)
  slots = torch.zeros((B,), dtype=torch.int32, device=dev)
  idx = torch.zeros((B,), dtype=torch.int64, device=dev)
  u = torch.rand((B,), dtype=torch.float64, device=dev)
  out['probs'] = b2b(lambda: _native.check(lib.dqz_logits_probs(
      dl.handle, _native.ptr(dl.logits), _native.ptr(p), _native.ptr(lse), _native.stream_handle())))
  out['sample_slots'] = b2b(lambda: dl.sample_slots_philox(1, ctr, slots))
  out['sample_inj'] = b2b(lambda: _native.check(lib.dqz_logits_sample(
      dl.handle, _native.ptr(dl.logits), _native.ptr(u), B, _native.ptr(idx), _native.stream_handle())))
  run = dl.run_state()
  out['run_state'] = run
  tcap = 1 << 20
  tree = torch.zeros((2 * tcap,), dtype=torch.float64, device=dev)
  pri = torch.rand((cap,), dtype=torch.float64, device=dev) + 0.01
  ia = torch.arange(cap, dtype=torch.int64, device=dev)
  for s0 in range(0, cap, 65536):
    n = min(65536, cap - s0)
    _native.check(lib.dqz_sumtree_set(_native.ptr(tree), tcap, _native.ptr(ia[s0:s0 + n]),
                                      _native.ptr(pri[s0:s0 + n]), n, _native.stream_handle()))
  w = torch.zeros((B,), dtype=torch.float32, device=dev)
  pc = torch.zeros((1,), dtype=torch.int64, device=dev)
  out['per_sample'] = b2b(lambda: _native.check(lib.dqz_per_sample(
      _native.ptr(tree), tcap, 0, cap, cap, B, 1e-3, 0.4, 1, 3, _native.ptr(pc), None, None, None, None,
      _native.ptr(slots), _native.ptr(w), None, _native.stream_handle())))
  store = synthetic.fill_episodic(cap, 6, seed=0, device=dev)
  net = networks.dqn_atari_network(6)
  lrn = learner_lib.Learner(net, B, algo='dqn', device=dev)
  lrn.set_params(net.init(0))
  c2 = torch.zeros((1,), dtype=torch.int64, device=dev)
  out['step_uniform_graph'] = graph_rate(lambda: lrn.step_uniform(store, 0, cap, cap, 5, c2, slots))
  out['step_logits_graph'] = graph_rate(lambda: lrn.step_logits(store, dl, slots, seed=5, counter=c2))

  def sep():
    dl.sample_slots_philox(5, c2, slots)
    lrn.step(store, slots)
  out['sampler_then_step_graph'] = graph_rate(sep)
  out['step_graph'] = graph_rate(lambda: lrn.step(store, slots))
  print(json.dumps(out))


if __name__ == '__main__':
  main()
