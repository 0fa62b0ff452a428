"""Independent-seed replicas, one process per GPU.

The learner step is sequentially dependent and the reference never shares
gradients (its SLURM arrays run one seed per job), so multi-GPU here is
replicas only: each rank owns its own replay, learner and RNG streams.  The
collectives are a small float64 statistics all-gather every
`--stats-every` steps inside bench.py's timed loop (enqueued, consumed after
it), and a MAX of the timed-region wall clock plus a final statistics gather
after it — over RCCL ("nccl") on the GPU box, gloo in the CPU tests.  The
process group is initialised at every world size, 1 included, so a 1-GPU
run goes through the same RCCL calls as an 8-GPU one (run_dqn_normal.sh:5,47
runs one seed per job; here the seeds report through one group).
"""

import os

import numpy as np
import torch

# Environment variable naming the rendezvous file of ranks started by
# bench.spawn_ranks (a torch.distributed.FileStore).
STORE_FILE_ENV = 'DQZ_STORE_FILE'


def device_identity(local_rank, stand_in=None):
  """What a rank's device is: name, PCI location and UUID.

  `stand_in` (a string) replaces the hardware query in the CPU self-test,
  where there is no device to ask.
  """
  if stand_in is not None:
    return {'name': 'cpu stand-in', 'pci': stand_in, 'uuid': stand_in}
  p = torch.cuda.get_device_properties(local_rank)
  pci = '%04x:%02x:%02x' % (int(p.pci_domain_id), int(p.pci_bus_id),
                            int(p.pci_device_id))
  return {'name': p.name, 'pci': pci, 'uuid': str(p.uuid)}


def check_devices(identities, expected_world):
  """Errors of an N-rank run's device set: every rank on its own device.

  identities: one device_identity() per rank, in rank order.  Returns a list
  of messages (empty when the world is the expected size and no two ranks
  share a PCI location or a UUID).
  """
  errors = []
  if len(identities) != expected_world:
    errors.append('world %d != --gpus %d' % (len(identities), expected_world))
  for key in ('pci', 'uuid'):
    seen = {}
    for r, ident in enumerate(identities):
      v = ident.get(key)
      if v in seen:
        errors.append('ranks %d and %d report the same device (%s %s)'
                      % (seen[v], r, key, v))
      else:
        seen[v] = r
  return errors


class Replicas:
  """Rank bookkeeping + the two reporting collectives."""

  def __init__(self, backend=None):
    self.world = int(os.environ.get('WORLD_SIZE', '1'))
    self.rank = int(os.environ.get('RANK', '0'))
    self.local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    self.dist = None
    self.backend = None
    if self.world == 1 and os.environ.get('DQZ_BENCH_NO_GROUP') == '1':
      return  # diagnostic A/B only: a lone rank without a process group
    import torch.distributed as dist  # pylint: disable=g-import-not-at-top
    backend = backend or 'nccl'
    if not dist.is_initialized():
      kw = {}
      if backend == 'nccl':
        # bind the communicator to this rank's GPU up front (without it
        # torch guesses the device from the global rank)
        kw['device_id'] = torch.device('cuda', self.local_rank)
      store_file = os.environ.get(STORE_FILE_ENV)
      if store_file:
        # ranks started by bench.spawn_ranks meet in a file store the parent
        # named: no port is probed and later bound (a probed loopback port
        # was once taken by another process before the bind, EADDRINUSE)
        store = dist.FileStore(store_file, self.world)
        dist.init_process_group(backend, store=store, rank=self.rank,
                                world_size=self.world, **kw)
      elif self.world == 1 and 'MASTER_ADDR' not in os.environ:
        # a lone rank still forms a group, over an in-process store
        dist.init_process_group(backend, store=dist.HashStore(), rank=0,
                                world_size=1, **kw)
      else:  # torch.distributed.run: the launcher's env:// rendezvous
        dist.init_process_group(backend, rank=self.rank, world_size=self.world,
                                **kw)
    self.dist = dist
    self.backend = dist.get_backend()

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

  def gather_objects(self, obj):
    """All-gather a picklable python object from every rank -> list."""
    if self.dist is None:
      return [obj]
    out = [None] * self.world
    self.dist.all_gather_object(out, obj)
    return out

  def close(self):
    if self.dist is not None and self.dist.is_initialized():
      self.dist.destroy_process_group()
