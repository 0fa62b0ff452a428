"""Fixed cost of a short timed region (the driver's `--steps 20`): host time
of K = 20 learner steps replayed as one 20-step graph or as smaller graph
chunks, against the same steps' GPU time (HIP events on the stream) and an
empty sync round trip.  usage (GPU box): python tools/overhead_probe.py
Prints one JSON line: per plan, the median host ms and event ms over N reps."""
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

K, REPS = 20, 25
dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)
wl = bench.Workload('dqn', 1_000_000, 0, dev)
one_step = wl.one_step
for _ in range(5):
  one_step()
torch.cuda.synchronize()
plans = {'20': [20], '10+10': [10, 10], '5x4': [5] * 4, '2+18': [2, 18], '4+16': [4, 16], '1+19': [1, 19]}
graphs = {}
for k in sorted({k for p in plans.values() for k in p}):
  if k == 1:
    continue
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    for _ in range(k):
      one_step()
  graphs[k] = g
  for _ in range(2):
    g.replay()
torch.cuda.synchronize()


def run(plan):
  for k in plan:
    if k == 1:
      one_step()
    else:
      graphs[k].replay()


from dqn_mgsc_zoo_amd import replicas as replicas_lib  # noqa: E402
reps_nccl = replicas_lib.Replicas('nccl')  # a world-1 RCCL group, as bench.py forms
import torch.distributed as dist  # noqa: E402
gloo = dist.new_group(backend='gloo')


def barrier_nccl():
  dist.barrier()


def barrier_gloo():
  dist.barrier(group=gloo)


out = {}
t = []
for _ in range(REPS):
  torch.cuda.synchronize()
  t0 = time.perf_counter()
  torch.cuda.synchronize()
  t.append(time.perf_counter() - t0)
out['empty_sync_ms'] = round(1e3 * statistics.median(t), 4)
cases = [(name, plan, None) for name, plan in plans.items()]
cases += [('20+rccl_barrier', [20], barrier_nccl), ('20+gloo_barrier', [20], barrier_gloo)]
for name, plan, bar in cases:
  host, ev = [], []
  for _ in range(REPS):
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    if bar is not None:
      bar()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record()
    run(plan)
    e1.record()
    torch.cuda.synchronize()
    host.append(time.perf_counter() - t0)
    ev.append(e0.elapsed_time(e1) * 1e-3)
  out[name] = {'host_ms': round(1e3 * statistics.median(host), 4), 'event_ms': round(1e3 * statistics.median(ev), 4),
               'host_steps_per_s': round(K / statistics.median(host), 1)}
  print(name, out[name], file=sys.stderr, flush=True)
print(json.dumps(out))
