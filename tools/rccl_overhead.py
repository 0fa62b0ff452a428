"""Does an idle RCCL communicator slow the learner's graph replays?

usage (GPU box): python tools/rccl_overhead.py
Times the bench's 50-step graph replays, then creates a world-1 NCCL group
in stages (init_process_group, first collective), re-timing after each, and
prints the host thread's CPU affinity at each stage.
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _free_port():
  import socket  # pylint: disable=g-import-not-at-top
  with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
    s.bind(('127.0.0.1', 0))
    return s.getsockname()[1]


def main():
  dev = torch.device('cuda:0')
  torch.cuda.set_device(dev)
  out = {}
  before = len(sys.argv) > 1 and sys.argv[1] == 'before'
  import torch.distributed as dist  # pylint: disable=g-import-not-at-top
  os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
  os.environ.setdefault('MASTER_PORT', str(_free_port()))
  if before:  # the group exists while the workload is built and captured
    dist.init_process_group('nccl', rank=0, world_size=1)
  wl = bench.Workload('dqn', 1_000_000, 0, dev)
  side = torch.cuda.Stream(dev)
  side.wait_stream(torch.cuda.current_stream(dev))
  with torch.cuda.stream(side):
    for _ in range(3):
      wl.one_step()
  torch.cuda.current_stream(dev).wait_stream(side)
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    for _ in range(50):
      wl.one_step()

  def rate(reps=200):
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
      g.replay()
    torch.cuda.synchronize()
    return 50 * reps / (time.perf_counter() - t0)

  out['mode'] = 'group before capture' if before else 'group after capture'
  out['first'] = (rate(), len(os.sched_getaffinity(0)))
  if not before:
    dist.init_process_group('nccl', rank=0, world_size=1)
  out['after_init'] = (rate(), len(os.sched_getaffinity(0)))
  t = torch.ones((2,), device=dev)
  dist.all_reduce(t)
  torch.cuda.synchronize()
  out['after_first_collective'] = (rate(), len(os.sched_getaffinity(0)))
  out['again'] = (rate(), len(os.sched_getaffinity(0)))
  dist.destroy_process_group()
  out['after_destroy'] = (rate(), len(os.sched_getaffinity(0)))
  print(json.dumps(out))


if __name__ == '__main__':
  main()
