"""Probe: forward launches at Z = 1 (one network copy) against the learner
step's Z = 2, to bound what taking the target forward off the step's
critical path could save.  Run under rocprofv3 --kernel-trace --stats:
500 fused learner steps (eager), then 500 one-copy forwards of the same
32-sample batch (dqz_forward_slots: the conv hand-off launch, fc1, head).
usage (GPU box): rocprofv3 --kernel-trace --stats -d DIR -o run -- python tools/z1_probe.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from dqn_mgsc_zoo_amd import learner as learner_lib  # noqa: E402
from dqn_mgsc_zoo_amd import networks  # noqa: E402
from dqn_mgsc_zoo_amd import synthetic  # noqa: E402


def main():
  dev = torch.device('cuda:0')
  net = networks.dqn_atari_network(6)
  lrn = learner_lib.Learner(net, 32, algo='dqn', device=dev)
  lrn.set_params(net.init(0))
  cap = 1_000_000
  st = synthetic.fill_episodic(cap, 6, seed=0, device=dev)
  counter = torch.zeros((1,), dtype=torch.int64, device=dev)
  slots = torch.zeros((32,), dtype=torch.int32, device=dev)
  for _ in range(500):
    lrn.step_uniform(st, 0, cap, cap, 1, counter, slots)
  torch.cuda.synchronize()
  for _ in range(500):
    lrn.q_values_slots(st, slots, 1, params=lrn.target)
  torch.cuda.synchronize()
  print('ok')


if __name__ == '__main__':
  main()
