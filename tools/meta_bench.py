"""MGSC meta-update timing (M = 100, timed apart
from the learner step): eager calls and hipGraph replays of
MetaLearner.update, first and second order.

usage (GPU box): python tools/meta_bench.py [--m 100] [--steps 200] > out.json
Under rocprofv3 --kernel-trace --stats the per-kernel split of the same calls.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from dqn_mgsc_zoo_amd import learner as learner_lib, networks, replay as replay_lib, synthetic  # noqa: E402
from dqn_mgsc_zoo_amd import replay_circular as rc  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, 'tools'))
from bench_configs import timed  # noqa: E402  pylint: disable=g-import-not-at-top

B, A = 32, 6


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument('--m', type=int, nargs='+', default=[100])
  ap.add_argument('--steps', type=int, default=200)
  ap.add_argument('--capacity', type=int, default=1_000_000)
  ap.add_argument('--orders', type=int, nargs='+', default=[0, 1])
  ap.add_argument('--graph', type=int, default=10, help='meta updates per captured graph (0: eager only)')
  args = ap.parse_args()
  dev = torch.device('cuda:0')
  cap = args.capacity
  store = synthetic.fill_episodic(cap, A, seed=0, device=dev)
  rng = np.random.default_rng(0)
  net = networks.dqn_atari_network(A)
  lrn = learner_lib.Learner(net, B, algo='dqn', device=dev)
  lrn.set_params(net.init(seed=3))
  lbuf = rc._DeviceLogits(cap, dev, max_queries=B)  # pylint: disable=protected-access
  lbuf.load(rng.standard_normal(cap).astype(np.float32))
  # one draw re-seeds the running log-sum-exp, as the agent loop's samples
  # and adds keep it: the meta-update then maintains it and re-sums the
  # chunks it writes (the path config 3's agent takes)
  lbuf.sample_abs(rng.random(B))
  ot = replay_lib.Transition(rng.integers(0, 256, (84, 84, 4), dtype=np.uint8), 2, 1.0, 0.99,
                             rng.integers(0, 256, (84, 84, 4), dtype=np.uint8))
  out = {'capacity': cap, 'num_actions': A, 'steps': args.steps}
  for m in args.m:
    for order in args.orders:
      meta = learner_lib.MetaLearner(lrn, m, learner_lib.adam(2.5e-4), second_order=bool(order))
      meta.set_online_transition(ot)
      ms = torch.from_numpy(rng.choice(cap, m, replace=False).astype(np.int32)).to(dev)
      fn = lambda: meta.update(store, ms, lbuf.logits, ms, logit_buffer=lbuf)  # pylint: disable=cell-var-from-loop
      key = 'meta_M%d_%s' % (m, 'second' if order else 'first')
      out[key + '_eager'] = timed(fn, args.steps, 3, dev)
      if args.graph:
        out[key + '_graph'] = timed(fn, args.steps, 3, dev, graph_steps=args.graph)
      print(key, out[key + '_eager'], out.get(key + '_graph'), file=sys.stderr, flush=True)
      del meta
  print(json.dumps(out))


if __name__ == '__main__':
  main()
