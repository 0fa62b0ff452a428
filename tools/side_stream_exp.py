"""Experiment (GPU box): cost to the learner chain of a concurrent batched
target forward on a side stream, forked once per 50-step hipGraph.

Prints us/step for: the plain 50-step graph; the same graph with a side
branch running `chunks` forwards of n samples (the next chunk's target
network outputs, 1,600 samples at the defaults); and the side work alone.
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dqn_mgsc_zoo_amd import learner as learner_lib, networks, synthetic  # noqa: E402

dev = torch.device('cuda:0')
net = networks.dqn_atari_network(6)
lrn = learner_lib.Learner(net, 32, algo='dqn', device=dev)
lrn.set_params(net.init(0))
side_lrn = learner_lib.Learner(net, 256, algo='dqn', device=dev)
side_lrn.set_params(net.init(0))
cap = 200000
store = synthetic.fill_episodic(cap, 6, seed=0, device=dev)
slots = torch.zeros((32,), dtype=torch.int32, device=dev)
counter = torch.zeros((1,), dtype=torch.int64, device=dev)
NCH = int(os.environ.get('NCH', '7'))
NS = int(os.environ.get('NS', '229'))
side_slots = torch.randint(0, cap, (NS,), dtype=torch.int32, device=dev)
main = torch.cuda.Stream(dev)
side = torch.cuda.Stream(dev)
G = 50


def step():
  lrn.step_uniform(store, 0, cap, cap, 1, counter, slots)


def side_work():
  for _ in range(NCH):
    side_lrn.q_values_slots(store, side_slots, 1, params=side_lrn.target)


def body(fork):
  if fork:
    e = torch.cuda.Event()
    e.record(main)
    side.wait_event(e)
    with torch.cuda.stream(side):
      side_work()
    e2 = torch.cuda.Event()
    e2.record(side)
  for _ in range(G):
    step()
  if fork:
    main.wait_event(e2)


def run(fork, reps=20):
  with torch.cuda.stream(main):
    body(fork)
  torch.cuda.synchronize()
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g, stream=main):
    body(fork)
  for _ in range(3):
    g.replay()
  torch.cuda.synchronize()
  t = time.perf_counter()
  for _ in range(reps):
    g.replay()
  torch.cuda.synchronize()
  return (time.perf_counter() - t) / (reps * G) * 1e6


def run_side(reps=20):
  with torch.cuda.stream(side):
    side_work()
  torch.cuda.synchronize()
  t = time.perf_counter()
  with torch.cuda.stream(side):
    for _ in range(reps):
      side_work()
  torch.cuda.synchronize()
  return (time.perf_counter() - t) / reps * 1e6


for r in range(2):
  print('plain %.2f us/step | fork+side %.2f us/step | side alone %.1f us per chunk (%d x %d samples)' % (
      run(False), run(True), run_side(), NCH, NS), flush=True)
