"""CPU: bench.py's step arithmetic and rank orchestration (no GPU).

The driver runs `bench.py --gpus N --steps K --warmup W` for N in 1,2,4,8;
round 1's bench rounded K down to a multiple of the graph size and timed 0
steps at K = 20.  These tests pin that exactly K steps are timed for any K,
that target syncs / stats gathers fire at their step boundaries, and that
`--gpus 2` starts two ranks by itself (gloo stand-in step, no GPU).
"""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # pylint: disable=g-import-not-at-top,wrong-import-position


@pytest.mark.parametrize('steps', [1, 20, 49, 50, 51, 5000])
@pytest.mark.parametrize('graph_steps', [1, 50])
def test_exact_step_count(steps, graph_steps):
  g, rem = bench.plan_chunks(steps, graph_steps, True)
  assert 1 <= g <= graph_steps and 0 <= rem < g
  assert (steps // g) * g + rem == steps
  calls = []

  class G:
    def __init__(self, k):
      self.k = k

    def replay(self):
      calls.append(self.k)

  graphs = {k: G(k) for k in (g, rem) if k > 1}
  runner = bench.StepRunner(lambda: calls.append(1), graphs, 10**9,
                            lambda: None)
  assert runner.run(steps, g, rem) == steps
  assert sum(calls) == steps
  # at most one eager / remainder chunk after the full graphs
  assert len(calls) <= steps // g + max(rem, 1)


def test_eager_and_invalid():
  assert bench.plan_chunks(20, 50, False) == (1, 0)
  with pytest.raises(ValueError):
    bench.plan_chunks(0, 50, True)


@pytest.mark.parametrize('g', [1, 7, 50])
def test_target_sync_and_stats_boundaries(g):
  syncs, stats = [], []
  rem = 1000 % g
  graph = type('G', (), {'replay': lambda self: None})()
  runner = bench.StepRunner(lambda: None, {g: graph, rem: graph}, 100,
                            lambda: syncs.append(runner.done), 250,
                            stats.append)
  runner.run(1000, g, rem)
  # every crossing of a period boundary syncs once, right after that chunk
  assert len(syncs) == 10
  assert all(0 <= s - 100 * (i + 1) < max(g, 1) for i, s in enumerate(syncs))
  assert len(stats) == 4


def _run_bench(args, env=None, timeout=240):
  e = dict(os.environ)
  for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT'):
    e.pop(k, None)
  e.update(env or {})
  return subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py')] + args,
                        capture_output=True, text=True, timeout=timeout, env=e,
                        cwd=ROOT)


def test_gpus2_spawns_two_ranks_gloo():
  p = _run_bench(['--gpus', '2', '--steps', '20', '--warmup', '5',
                  '--stats-every', '8', '--target-period', '10',
                  '--graph-steps', '6', '--selftest-cpu'])
  assert p.returncode == 0, p.stderr[-2000:]
  lines = [l for l in p.stdout.splitlines() if l.startswith('{')]
  assert len(lines) == 1  # rank 0 only
  out = json.loads(lines[0])
  assert out['n_gpus'] == 2 and out['steps'] == 20
  assert out['per_rank_steps'] == [20, 20]
  assert out['chunks'] == [6, 2]
  # warmup 5 + 20 timed: target-period 10 crossed at 10 and 20 (and 25 is
  # not a multiple), stats-every 8 crossed at 8, 16, 24
  assert out['per_rank_target_syncs'] == [2, 2]
  assert out['per_rank_stats_gathers'] == [3, 3]
  assert out['value'] > 0
  # the gathered statistics are read back: every rank's step count at the
  # last in-loop gather (the chunk that crossed step 24 ends at 25)
  assert out['rccl']['backend'] == 'gloo' and out['rccl']['world'] == 2
  assert out['rccl']['last_in_loop_gather']['steps_done'] == [25, 25]
  assert len(out['rccl']['last_in_loop_gather']['value']) == 2
  # each rank's device identity (stand-ins on CPU), all distinct
  assert [d['pci'] for d in out['devices']] == ['stand-in-0', 'stand-in-1']


def test_gpus2_same_device_fails():
  """Two ranks reporting one device make the line invalid (exit 4)."""
  p = _run_bench(['--gpus', '2', '--steps', '4', '--warmup', '0',
                  '--selftest-cpu'], env={'DQZ_SELFTEST_DEVICE': 'dup'})
  assert p.returncode == 4, p.stderr[-2000:]
  assert 'report the same device' in p.stderr
  assert not [l for l in p.stdout.splitlines() if l.startswith('{')]


def test_check_devices():
  from dqn_mgsc_zoo_amd import replicas  # pylint: disable=g-import-not-at-top
  ids = [{'pci': '0000:%02x:00' % i, 'uuid': 'u%d' % i} for i in range(4)]
  assert replicas.check_devices(ids, 4) == []
  assert replicas.check_devices(ids, 8) == ['world 4 != --gpus 8']
  ids[3] = dict(ids[1])
  errs = replicas.check_devices(ids, 4)
  assert len(errs) == 2 and all('ranks 1 and 3' in e for e in errs)


def test_gpus1_forms_a_process_group():
  """World 1 goes through the same collectives (a group of one)."""
  p = _run_bench(['--gpus', '1', '--steps', '10', '--warmup', '0',
                  '--stats-every', '5', '--selftest-cpu'])
  assert p.returncode == 0, p.stderr[-2000:]
  out = json.loads([l for l in p.stdout.splitlines() if l.startswith('{')][0])
  assert out['rccl']['world'] == 1
  assert out['rccl']['last_in_loop_gather']['steps_done'] == [10]


def test_lead_eager_steps_keep_the_timed_count():
  """--lead-eager L: L eager steps, then graphs over the other K - L."""
  p = _run_bench(['--gpus', '1', '--steps', '20', '--warmup', '0',
                  '--graph-steps', '6', '--lead-eager', '3', '--stats-every', '5',
                  '--selftest-cpu'])
  assert p.returncode == 0, p.stderr[-2000:]
  out = json.loads([l for l in p.stdout.splitlines() if l.startswith('{')][0])
  assert out['steps'] == 20 and out['per_rank_steps'] == [20]
  assert out['chunks'] == [6, 5]  # 17 = 2 x 6 + 5
  bad = _run_bench(['--gpus', '1', '--steps', '4', '--lead-eager', '4',
                    '--selftest-cpu'], timeout=120)
  assert bad.returncode != 0 and '--lead-eager' in bad.stderr


def test_world_mismatch_fails():
  p = _run_bench(['--gpus', '2', '--steps', '4', '--warmup', '0',
                  '--selftest-cpu'], env={'WORLD_SIZE': '1'}, timeout=120)
  assert p.returncode != 0
  assert 'WORLD_SIZE=1' in p.stderr


def _json_line(p):
  lines = [l for l in p.stdout.splitlines() if l.startswith('{')]
  assert len(lines) == 1, p.stdout[-2000:]  # rank 0 only
  return json.loads(lines[0])


def test_gpus8_spawns_eight_ranks_gloo():
  """World-8 readiness (config 5: 8 independent seeds, one per GPU,
  run_dqn_normal.sh:5,47): bench.py starts 8 ranks itself, every rank times
  exactly K steps, the line carries 8 distinct device identities and 8
  per-rank rates, and value = world x K / max-over-ranks time."""
  p = _run_bench(['--gpus', '8', '--steps', '20', '--warmup', '5',
                  '--stats-every', '8', '--target-period', '10',
                  '--graph-steps', '6', '--selftest-cpu'], timeout=400)
  assert p.returncode == 0, p.stderr[-3000:]
  out = _json_line(p)
  assert out['n_gpus'] == 8 and out['rccl']['world'] == 8
  assert out['per_rank_steps'] == [20] * 8
  assert out['per_rank_target_syncs'] == [2] * 8
  assert out['per_rank_stats_gathers'] == [3] * 8
  assert out['rccl']['last_in_loop_gather']['steps_done'] == [25] * 8
  assert len(out['per_rank_steps_per_s']) == 8
  assert all(v > 0 for v in out['per_rank_steps_per_s'])
  assert out['per_gpu_min_steps_per_s'] == min(out['per_rank_steps_per_s'])
  ids = [d['pci'] for d in out['devices']]
  assert ids == ['stand-in-%d' % r for r in range(8)] and len(set(ids)) == 8
  # value is the whole-job aggregate over the slowest rank's time
  assert abs(out['value'] - 8 * 20 / (out['ms_per_step'] * 20 / 1e3)) < 1e-6 * out['value'] + 0.02


def test_gpus8_two_ranks_on_one_device_fail():
  """check_devices' failure path at world 8: rank 5 reporting rank 2's
  device makes the line invalid (exit 4, no JSON line)."""
  p = _run_bench(['--gpus', '8', '--steps', '4', '--warmup', '0',
                  '--selftest-cpu'], env={'DQZ_SELFTEST_DEVICE': '5=stand-in-2'},
                 timeout=400)
  assert p.returncode == 4, p.stderr[-3000:]
  assert 'ranks 2 and 5 report the same device' in p.stderr
  assert not [l for l in p.stdout.splitlines() if l.startswith('{')]


def test_gpus8_under_torch_distributed_run():
  """The driver's own launch: python -m torch.distributed.run
  --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8 (env://
  rendezvous, WORLD_SIZE set by the launcher, no ranks spawned here)."""
  import socket  # pylint: disable=g-import-not-at-top
  with socket.socket() as s:
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
  e = dict(os.environ)
  for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT'):
    e.pop(k, None)
  e['OMP_NUM_THREADS'] = '1'
  p = subprocess.run(
      [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
       '--nproc-per-node', '8', '--master-addr', '127.0.0.1', '--master-port',
       str(port), os.path.join(ROOT, 'bench.py'), '--gpus', '8', '--steps', '12',
       '--warmup', '2', '--graph-steps', '5', '--selftest-cpu'],
      capture_output=True, text=True, timeout=400, env=e, cwd=ROOT)
  assert p.returncode == 0, p.stderr[-3000:]
  out = _json_line(p)
  assert out['n_gpus'] == 8 and out['per_rank_steps'] == [12] * 8
  assert len({d['pci'] for d in out['devices']}) == 8
  assert len(out['per_rank_steps_per_s']) == 8
