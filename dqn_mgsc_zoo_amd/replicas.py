"""Independent-seed replicas, one process per GPU.

The learner step is sequentially dependent and the reference never shares
gradients (its SLURM arrays run one seed per job), so multi-GPU here is
replicas only: each rank owns its own replay, learner and RNG streams.  The
only collectives are a MAX of the timed-region wall clock and an all-gather
of a small float64 statistics vector, both after the timed region — over
RCCL ("nccl") on the GPU box, gloo in the CPU tests.
"""

import os

import numpy as np
import torch


class Replicas:
  """Rank bookkeeping + the two reporting collectives."""

  def __init__(self, backend=None):
    self.world = int(os.environ.get('WORLD_SIZE', '1'))
    self.rank = int(os.environ.get('RANK', '0'))
    self.local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    self.dist = None
    if self.world > 1:
      import torch.distributed as dist  # pylint: disable=g-import-not-at-top
      if not dist.is_initialized():
        dist.init_process_group(backend or 'nccl')
      self.dist = dist

  def seed(self, base=0):
    """Per-rank seed: rank r runs seed base + r."""
    return base + self.rank

  def barrier(self):
    if self.dist is not None:
      self.dist.barrier()

  def max_over_ranks(self, value, device='cpu'):
    """MAX of a python float over ranks (the timed-region wall clock)."""
    if self.dist is None:
      return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
    return float(t.item())

  def gather_stats(self, values, device='cpu'):
    """All-gather a float64 vector from every rank -> numpy [world, k]."""
    v = torch.as_tensor(np.asarray(values, np.float64), device=device)
    if self.dist is None:
      return v.cpu().numpy()[None, :]
    out = [torch.zeros_like(v) for _ in range(self.world)]
    self.dist.all_gather(out, v)
    return torch.stack(out).cpu().numpy()

  def close(self):
    if self.dist is not None and self.dist.is_initialized():
      self.dist.destroy_process_group()
