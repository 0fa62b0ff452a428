"""CPU: the replicas-only multi-process path over gloo, world_size 2."""

import os
import socket

import numpy as np
import torch.multiprocessing as mp


def _free_port():
  with socket.socket() as s:
    s.bind(('127.0.0.1', 0))
    return s.getsockname()[1]


def _worker(rank, world, port, q):
  os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port),
                    WORLD_SIZE=str(world), RANK=str(rank), LOCAL_RANK=str(rank))
  from dqn_mgsc_zoo_amd import replicas  # pylint: disable=g-import-not-at-top
  r = replicas.Replicas(backend='gloo')
  r.barrier()
  elapsed = 1.0 + r.rank  # rank 1 is the slow one
  mx = r.max_over_ranks(elapsed)
  stats = r.gather_stats([100.0 * (r.rank + 1), elapsed, r.seed(7)])
  q.put((rank, mx, stats.tolist()))
  r.close()


def test_replicas_gloo_world2():
  ctx = mp.get_context('spawn')
  q = ctx.Queue()
  port = _free_port()
  procs = [ctx.Process(target=_worker, args=(i, 2, port, q)) for i in range(2)]
  for p in procs:
    p.start()
  out = [q.get(timeout=120) for _ in procs]
  for p in procs:
    p.join(timeout=60)
    assert p.exitcode == 0
  for rank, mx, stats in out:
    assert mx == 2.0  # max over ranks
    np.testing.assert_array_equal(stats, [[100.0, 1.0, 7.0], [200.0, 2.0, 8.0]])


def test_replicas_single_process():
  """World 1 still forms a process group (bench.py's 1-GPU run goes
  through the same collectives as an N-GPU one)."""
  from dqn_mgsc_zoo_amd import replicas  # pylint: disable=g-import-not-at-top
  for k in ('WORLD_SIZE', 'RANK', 'MASTER_ADDR', 'MASTER_PORT'):
    os.environ.pop(k, None)
  r = replicas.Replicas(backend='gloo')
  try:
    assert r.dist.is_initialized() and r.dist.get_world_size() == 1
    assert r.backend == 'gloo'
    assert r.world == 1 and r.max_over_ranks(3.5) == 3.5
    np.testing.assert_array_equal(r.gather_stats([1.0, 2.0]), [[1.0, 2.0]])
  finally:
    r.close()


def _file_store_worker(rank, world, path, q):
  os.environ.update(WORLD_SIZE=str(world), RANK=str(rank), LOCAL_RANK=str(rank))
  for k in ('MASTER_ADDR', 'MASTER_PORT'):
    os.environ.pop(k, None)
  from dqn_mgsc_zoo_amd import replicas  # pylint: disable=g-import-not-at-top
  os.environ[replicas.STORE_FILE_ENV] = path
  r = replicas.Replicas(backend='gloo')
  mx = r.max_over_ranks(float(rank))
  stats = r.gather_stats([float(rank)])
  q.put((rank, mx, stats.tolist()))
  r.close()


def test_replicas_file_store_rendezvous(tmp_path):
  """Ranks spawned by bench.spawn_ranks meet in a FileStore the parent
  names (no probed port)."""
  ctx = mp.get_context('spawn')
  q = ctx.Queue()
  path = str(tmp_path / 'store')
  procs = [ctx.Process(target=_file_store_worker, args=(i, 2, path, q))
           for i in range(2)]
  for p in procs:
    p.start()
  out = [q.get(timeout=120) for _ in procs]
  for p in procs:
    p.join(timeout=60)
    assert p.exitcode == 0
  for _, mx, stats in out:
    assert mx == 1.0
    np.testing.assert_array_equal(stats, [[0.0], [1.0]])
