"""Learner grad-steps/s at batch 32 on synthetic 84x84x4 uint8 replay.

`python bench.py --gpus N --steps K --warmup W`: one process per GPU.  Under
torch.distributed.run (WORLD_SIZE set) each process is one rank; without it
and N > 1, this process starts the N rank processes itself (before touching
the GPU) and exits with the worst of their exit codes.  A *step* is one pass of the
hot path on device: uniform sample of 32 slots from a 1M-transition frame
replay (Philox on device) -> frame gather + /255 fused into conv1 ->
NatureQNetwork forward of online(s_tm1) and target(s_t) -> q_learning TD
loss with clip_gradient -> backward -> centered RMSProp; the target copy
runs every 2,500 steps (40,000 frames / learn_period 16) inside the timed
loop.  Replicas are independent seeds (no gradient all-reduce); RCCL only
all-gathers a per-rank statistics vector every 1,000 steps (SURVEY.md §8(d)
config 4) and after the timed region.  The process group exists at every
world size, so the 1-GPU line goes through the same RCCL calls.

`--algo` picks the BASELINE config the step follows: dqn (config 2, the
default and the headline line), double (double-Q on the same uniform
replay), per (config 4: device PER sample over a 2^20-leaf fp64 sum tree +
double-Q step with IS weights + |td|^alpha write-back), mgsc (config 3's
learner part: softmax-CDF sample over 1M learned f32 logits + DQN step) or
agent (config 1: the whole dqn agent, parts.run_loop over raw 210x160 RGB
frames through processors.atari, a 1M TransitionReplay, learning every 16
frames once 5 % of it is full; K learner steps are timed, 16 K frames).

Prints ONE JSON line on rank 0.
"""

import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
  sys.path.insert(0, ROOT)

METRIC = ('learner grad-steps/sec at batch=32, 84×84×4 uint8, '
          '1/2/4/8 MI355X')
# --algo agent (config 1): learner steps/s of the whole agent loop (acting,
# preprocessing and replay adds inside the timed region) -- not the headline
# learner-only quantity, so it carries a metric name of its own
AGENT_METRIC = ('agent-loop learner steps/sec (act + preprocess + add + learn), '
                'batch=32, 84×84×4 uint8, MI355X')
BATCH = 32
META_BATCH = 100  # the meta-update timed apart at M = 100
NUM_ACTIONS = 6  # Pong minimal action set (gym_atari.py:52-54)
F32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32 = f32 vector peak
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
STEP_FLOP = {'dqn': 2182873088, 'double': 2781020160,
             'per': 2781020160, 'mgsc': 2182873088}
# SURVEY.md §8(d); an MGSC draw adds, per sample, one read of the chunk sums
# (245 f64) and of one chunk of 4096 f32 logits: 32 x 18,344 B
STEP_BYTES = {'dqn': 49048488, 'double': 49048488, 'per': 49048488,
              'mgsc': 49048488 + 32 * (4096 * 4 + 245 * 8)}
LEARNER_ALGO = {'dqn': 'dqn', 'double': 'double', 'per': 'per', 'mgsc': 'dqn'}
WORKLOAD = {
    'dqn': 'BASELINE config 2: dqn agent learner-only loop',
    'double': 'double_q learner-only loop (uniform replay, shared-bias head)',
    'per': 'BASELINE config 4: prioritized (PER sum-tree sample + IS weights, '
           'double-Q, |td|^alpha write-back) learner-only loop',
    'mgsc': 'BASELINE config 3 learner part: dqn_mgsc_batched reservoir, '
            'softmax sample over N(0,1) learned logits + DQN step',
}
PER_ALPHA, PER_BETA, PER_USP = 0.6, 0.4, 1e-3  # prioritized/run_atari.py:104-114
# Algorithmic FLOP of one MGSC meta-update at M = META_BATCH
# (dqn_mgsc_batched/agent.py:152-220; DESIGN.md §4 "MGSC meta-update"):
#   the p-weighted loss gradient over the M meta transitions (2 forwards +
#   backward per sample, SURVEY §8(d)'s 34,107,392 MAC), the one-transition
#   gradient at theta', the tangent forward V * y of conv1..fc1 (and fc2's
#   h1 . V2[:, a]) over the M samples, and the per-sample dot products
#   <dz, V y + vb> (21,632 MAC); the second order (the reservoir agent's
#   Hessian-vector product of the online transition's q) adds a tangent
#   forward and a tangent backward of that one sample (2 x (fwd + bwd) MAC).
#   Elementwise stages (RMSProp tangents, Adam) are counted as bytes, not FLOP.
_FWD_MAC = 9346048
_BWD_MAC = 15415296
META_FLOP = {
    'first': 2 * (META_BATCH * 34107392 + 34107392 + META_BATCH * (_FWD_MAC - 3072 + 512)
                  + META_BATCH * 21632),
}
META_FLOP['second'] = META_FLOP['first'] + 2 * 2 * (_FWD_MAC + _BWD_MAC)
STATS_LEN = 3  # the in-loop RCCL statistics vector: steps, loss, seconds

ALL_BWD = 'conv3_dx+conv2_dx+fc1_dw+conv3_dw+conv2_dw+conv1_dw'

# Algorithmic MACs per sample of each forward layer.
MAC = dict(conv1=400 * 256 * 32, conv2=81 * 512 * 64, conv3=49 * 576 * 64,
           fc1=3136 * 512, fc2=512 * NUM_ACTIONS)


def phase_flops(algo, batch):
  """Algorithmic FLOPs of each libdqz phase (one launch each)."""
  algo = LEARNER_ALGO.get(algo, algo)
  z = 2 if algo == 'dqn' else 3
  b = batch
  return {
      'conv1_fwd': 2 * z * b * MAC['conv1'],
      'conv2_fwd': 2 * z * b * MAC['conv2'],
      'conv3_fwd': 2 * z * b * MAC['conv3'],
      'conv_fwd': 2 * z * b * (MAC['conv1'] + MAC['conv2'] + MAC['conv3']),
      'fc1_fwd': 2 * z * b * MAC['fc1'],
      # fc2 forward + fc2 dX (dz1 = dq W2^T)
      'head': 2 * z * b * MAC['fc2'] + 2 * b * MAC['fc2'],
      'fc1_dx': 2 * b * MAC['fc1'],
      ALL_BWD: 2 * b * (2 * MAC['conv3'] + MAC['fc1'] + 2 * MAC['conv2'] + MAC['conv1']),
      'update': 2 * b * MAC['fc2'],  # fc2 dW (the rest is the optimizer)
  }


# f32 bytes of one sample's activations / uint8 bytes of one stacked state.
ACT = dict(state=84 * 84 * 4, y1=4 * 32 * 20 * 20, y2=4 * 64 * 9 * 9,
           y3=4 * 64 * 7 * 7, h=4 * 512)
PARAM = dict(conv1=4 * (8 * 8 * 4 * 32 + 32), conv2=4 * (4 * 4 * 32 * 64 + 64),
             conv3=4 * (3 * 3 * 64 * 64 + 64), fc1=4 * (3136 * 512 + 512),
             fc2=4 * (512 * NUM_ACTIONS + NUM_ACTIONS))


def phase_bytes(algo, batch):
  """Algorithmic HBM bytes of each libdqz phase (one launch each).

  Every tensor the phase consumes is read once and every tensor it produces
  is written once; implementation scratch (split-K partials, per-sample dW
  partials, hand-off payloads) is excluded.  Centered RMSProp reads and
  writes theta, mu, nu (6 x 4 B per parameter); fc1's update runs inside the
  merged backward launch.
  """
  algo = LEARNER_ALGO.get(algo, algo)
  z = 2 if algo == 'dqn' else 3
  b = batch
  rms = 6 * (sum(PARAM.values()) - PARAM['fc1'])
  return {
      'conv1_fwd': z * b * (ACT['state'] + ACT['y1']) + z * PARAM['conv1'],
      'conv2_fwd': z * b * (ACT['y1'] + ACT['y2']) + z * PARAM['conv2'],
      'conv3_fwd': z * b * (ACT['y2'] + ACT['y3']) + z * PARAM['conv3'],
      # conv1 -> conv2 -> conv3 as one hand-off launch: y1 / y2 stay inside it
      'conv_fwd': z * b * (ACT['state'] + ACT['y3']) + z * (PARAM['conv1'] + PARAM['conv2'] + PARAM['conv3']),
      'fc1_fwd': z * b * (ACT['y3'] + ACT['h']) + z * PARAM['fc1'],
      # fc1 reduce -> h1 (read once as the split sum, written), W2, dz1 out
      'head': z * b * ACT['h'] + z * PARAM['fc2'] + b * ACT['h'],
      'fc1_dx': b * (ACT['h'] + 2 * ACT['y3']) + PARAM['fc1'],
      # the whole backward after fc1 dX in one launch: dy2 and dy1 are handed
      # off inside it; dy3, y2, y1 and the state are read once
      ALL_BWD: (b * (ACT['y3'] + ACT['y2'] + ACT['y1'] + ACT['state']) +
                2 * PARAM['conv3'] + 2 * PARAM['conv2'] + PARAM['conv1'] +
                b * (ACT['y3'] + ACT['h']) + 6 * PARAM['fc1']),
      'update': rms,
  }


# libdqz phase -> kernel symbol (rocprofv3 names, template args stripped).
PHASE_KERNEL = {
    'conv1_fwd': 'conv1_fwd_kernel', 'conv2_fwd': 'conv2_fwd_kernel',
    'conv3_fwd': 'conv3_fwd_kernel', 'conv_fwd': 'fwd_conv_kernel', 'fc1_fwd': 'fc1_fwd32_kernel',
    'head': 'head_kernel',
    'fc1_dx': 'fc1_dx_kernel', ALL_BWD: 'bwd_bc_kernel',
    'update': 'update_kernel'}
PMC_JSON = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')


def pmc_traffic(phase):
  """Measured fabric bytes per launch of `phase`'s kernel, or None.

  From the committed rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes
  (profiles/run_pmc.sh + pmc_summary.py, gfx950 FETCH_SIZE doubled).
  """
  try:
    with open(PMC_JSON) as f:
      rec = json.load(f).get(PHASE_KERNEL[phase], {})
  except (OSError, ValueError):
    return None
  t = rec.get('traffic_bytes')
  return None if t is None else int(t)


def cpu_baseline(seconds, algo):
  """torch-CPU fp32 learner step on this host's cores.

  The reference's --jax_platform_name=cpu path cannot run (no JAX stack), so
  the same update is timed as an fp32 torch-CPU port (`oracle/torch_cpu.py`,
  pinned to the fp64 oracle by tests/test_oracle.py) at every thread this
  process is allotted and at 2 threads (run_dqn_normal.sh:9
  --cpus-per-task=2), about seconds/2 each.
  """
  from oracle import torch_cpu  # pylint: disable=g-import-not-at-top
  from dqn_mgsc_zoo_amd import networks  # pylint: disable=g-import-not-at-top
  algo = LEARNER_ALGO[algo]
  net = (networks.dqn_atari_network(NUM_ACTIONS) if algo == 'dqn' else
         networks.double_dqn_atari_network(NUM_ACTIONS))
  allotted = int(os.environ.get('OMP_NUM_THREADS', '0') or 0)
  if allotted <= 0:
    allotted = len(os.sched_getaffinity(0))
  prev = torch.get_num_threads()
  gen = torch.Generator().manual_seed(0)
  rates = {}
  samples = {}
  for threads in (allotted, 2):
    torch.set_num_threads(threads)
    lrn = torch_cpu.TorchCpuLearner(net.init(0), algo=algo)
    n, t0 = 0, None
    while True:
      s_tm1 = torch.randint(0, 256, (BATCH, 84, 84, 4), generator=gen, dtype=torch.uint8)
      s_t = torch.randint(0, 256, (BATCH, 84, 84, 4), generator=gen, dtype=torch.uint8)
      a = torch.randint(0, NUM_ACTIONS, (BATCH,), generator=gen)
      r = torch.zeros(BATCH)
      d = torch.full((BATCH,), 0.99)
      w = torch.rand((BATCH,), generator=gen) if algo == 'per' else None
      lrn.step(s_tm1, a, r, d, s_t, weights=w)
      if t0 is None:  # the first step pays one-off allocation; not timed
        t0 = time.perf_counter()
        continue
      n += 1
      dt = time.perf_counter() - t0
      if dt >= seconds / 2 and n >= 2:
        break
    rates[threads] = n / dt
    samples[threads] = '%d steps in %.1f s' % (n, dt)
  torch.set_num_threads(prev)
  return {'value': round(rates[allotted], 3), 'unit': 'steps/s',
          'cores': allotted, 'kind': 'port',
          'value_2_threads': round(rates[2], 3),
          'sample': 'torch-CPU fp32 learner update (oracle/torch_cpu.py: %s, '
                    'B=32, 84x84x4 uint8, A=%d, centered RMSProp), one '
                    'untimed step then %s at %d threads; %s at 2 threads '
                    '(run_dqn_normal.sh:9 --cpus-per-task=2)' % (
                        algo, NUM_ACTIONS, samples[allotted], allotted,
                        samples[2])}


def plan_chunks(steps, graph_steps, use_graph):
  """Graph sizes (g, rem) so that the timed steps are EXACTLY `steps`.

  `steps // g` replays of a g-step graph then, if rem > 0, one replay of a
  rem-step graph; g = 1 and rem = 0 means eager launches.
  """
  if steps < 1:
    raise ValueError('--steps must be >= 1, got %d' % steps)
  if not use_graph:
    return 1, 0
  if graph_steps < 1:
    raise ValueError('--graph-steps must be >= 1')
  g = min(graph_steps, steps)
  return g, steps % g


class StepRunner:
  """Runs `n` learner steps through the captured graphs (or eagerly).

  Host-side bookkeeping between replays: the target hard copy whenever the
  global step count crosses a multiple of target_period (dqn/agent.py:155-156:
  the copy follows the learn of that step) and the statistics gather every
  stats_every steps.
  """

  def __init__(self, one_step, graphs, target_period, sync_target,
               stats_every=0, on_stats=None):
    self.one_step = one_step
    self.graphs = graphs  # {size: graph}
    self.target_period = target_period
    self.sync_target = sync_target
    self.stats_every = stats_every
    self.on_stats = on_stats
    self.done = 0

  def _advance(self, k):
    before, self.done = self.done, self.done + k
    if self.done // self.target_period > before // self.target_period:
      self.sync_target()
    if self.stats_every and self.on_stats is not None and (
        self.done // self.stats_every > before // self.stats_every):
      self.on_stats(self.done)

  def run(self, n, g, rem):
    """n == reps * g + rem steps: full graphs first, then the remainder."""
    i = 0
    while i < n:
      left = n - i
      if g > 1 and left >= g:
        self.graphs[g].replay()
        k = g
      elif rem > 1 and left == rem:
        self.graphs[rem].replay()
        k = rem
      else:
        self.one_step()
        k = 1
      i += k
      self._advance(k)
    return i


def spawn_ranks(n, argv, script=None):
  """Starts n rank processes of `script` (default: this one) with
  RANK/LOCAL_RANK/WORLD_SIZE set and returns the worst exit code.  The ranks
  rendezvous in a torch.distributed.FileStore whose path this parent names
  (replicas.STORE_FILE_ENV): no loopback port is probed here and bound later
  by a child, so nothing else can take it in between.  Called before
  anything touches the GPU; children are started, never exec'd into."""
  from dqn_mgsc_zoo_amd import replicas as replicas_lib  # pylint: disable=g-import-not-at-top
  tmp = tempfile.mkdtemp(prefix='dqz_ranks_')
  try:
    return _run_ranks(n, argv, os.path.join(tmp, 'store'),
                      script or os.path.abspath(__file__),
                      replicas_lib.STORE_FILE_ENV)
  finally:
    shutil.rmtree(tmp, ignore_errors=True)


def _run_ranks(n, argv, store_file, script, store_env):
  procs = []
  for r in range(n):
    env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
               LOCAL_WORLD_SIZE=str(n), **{store_env: store_file})
    env.pop('MASTER_ADDR', None)
    env.pop('MASTER_PORT', None)
    procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env))
  rcs = [None] * n
  own = []  # exit codes of ranks that failed by themselves (not terminated here)
  while any(rc is None for rc in rcs):
    for i, p in enumerate(procs):
      if rcs[i] is None:
        rcs[i] = p.poll()
    own = [rc for rc in rcs if rc not in (None, 0)]
    if own:  # one rank failed: the others would wait forever at a collective
      for i, p in enumerate(procs):
        if rcs[i] is None:
          p.terminate()
      for i, p in enumerate(procs):
        if rcs[i] is None:
          try:
            rcs[i] = p.wait(timeout=30)
          except subprocess.TimeoutExpired:
            p.kill()
            rcs[i] = p.wait()
      break
    time.sleep(0.05)
  # the code of the first rank that failed by itself (a rank this parent
  # terminated after it reports -SIGTERM, which says nothing of the cause)
  for rc in own + rcs:
    if rc != 0:
      return rc if rc > 0 else 1
  return 0


def parse_args(argv=None):
  ap = argparse.ArgumentParser()
  ap.add_argument('--gpus', type=int, default=1)
  ap.add_argument('--steps', type=int, default=5000)
  ap.add_argument('--warmup', type=int, default=200)
  ap.add_argument('--algo', default='dqn',
                  choices=['dqn', 'double', 'per', 'mgsc', 'agent'])
  ap.add_argument('--min-replay-fraction', type=float, default=0.05,
                  help='--algo agent: min_replay_capacity_fraction '
                       '(dqn/run_atari.py default 0.05)')
  ap.add_argument('--capacity', type=int, default=1_000_000)
  ap.add_argument('--graph', type=int, default=1, help='hipGraph-replay steps')
  ap.add_argument('--graph-steps', type=int, default=50)
  ap.add_argument('--lead-eager', type=int, default=0,
                  help='timed steps launched eagerly ahead of the graph '
                       'replays (the first kernels start without waiting '
                       'for a graph submission)')
  ap.add_argument('--target-period', type=int, default=2500)
  ap.add_argument('--stats-every', type=int, default=1000)
  ap.add_argument('--profile-iters', type=int, default=100)
  ap.add_argument('--cpu-seconds', type=float, default=20.0)
  ap.add_argument('--selftest-cpu', action='store_true',
                  help='orchestration self-test on CPU (gloo, no GPU, a '
                       'stand-in step): exercises rank launch, timing and '
                       'the statistics gathers only')
  return ap.parse_args(argv)


def main(argv=None):
  argv = sys.argv[1:] if argv is None else argv
  args = parse_args(argv)
  if args.gpus < 1:
    print('--gpus must be >= 1', file=sys.stderr)
    return 2
  if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
    return spawn_ranks(args.gpus, argv)
  world_env = int(os.environ.get('WORLD_SIZE', '1'))
  if world_env != args.gpus:
    print('bench.py: --gpus %d but WORLD_SIZE=%d' % (args.gpus, world_env),
          file=sys.stderr)
    return 2
  try:
    if not 0 <= args.lead_eager < args.steps:
      raise ValueError('--lead-eager must be in [0, --steps)')
    g, rem = plan_chunks(args.steps - args.lead_eager, args.graph_steps,
                         bool(args.graph))
  except ValueError as e:
    print('bench.py: %s' % e, file=sys.stderr)
    return 2
  if args.selftest_cpu:
    return selftest_cpu(args, g, rem)
  if args.algo == 'agent':
    return run_agent(args)
  return run_gpu(args, g, rem)


def _barrier(reps):
  mode = os.environ.get('DQZ_BENCH_BARRIER', 'barrier')  # diagnostic A/B only
  if mode == 'none' or reps.dist is None:
    return
  if mode == 'allreduce':
    t = torch.zeros((1,), device=torch.device('cuda', torch.cuda.current_device()))
    reps.dist.all_reduce(t)
    torch.cuda.synchronize()
    return
  reps.barrier()


def _timed(reps, runner, steps, g, rem, sync, lead=0):
  _barrier(reps)
  sync()
  t0 = time.perf_counter()
  n = runner.run(lead, 1, 0) if lead else 0
  n += runner.run(steps - lead, g, rem)
  sync()
  elapsed = time.perf_counter() - t0
  _barrier(reps)
  if n != steps:
    raise RuntimeError('timed %d steps, asked for %d' % (n, steps))
  return elapsed


def selftest_cpu(args, g, rem):
  """The orchestration of run_gpu with a CPU stand-in step (tests only)."""
  from dqn_mgsc_zoo_amd import replicas as replicas_lib  # pylint: disable=g-import-not-at-top
  reps = replicas_lib.Replicas('gloo')
  x = torch.ones((64, 64))
  counters = {'steps': 0, 'syncs': 0, 'gathers': 0}

  def one_step():
    x.copy_(torch.tanh(x @ x / 64.0))
    counters['steps'] += 1

  class _Graph:  # stand-in for a captured k-step graph
    def __init__(self, k):
      self.k = k

    def replay(self):
      for _ in range(self.k):
        one_step()

  def sync_target():
    counters['syncs'] += 1

  last = {}

  def on_stats(done):
    last['stats'] = reps.gather_stats([float(done), float(x[0, 0])])
    counters['gathers'] += 1

  graphs = {k: _Graph(k) for k in (g, rem) if k > 1}
  runner = StepRunner(one_step, graphs, args.target_period, sync_target,
                      args.stats_every, on_stats)
  # the timed gathers are collectives: every rank runs the same step counts
  runner.run(args.warmup, 1, 0)
  warm = counters['steps']
  elapsed = _timed(reps, runner, args.steps, g, rem, lambda: None,
                   lead=args.lead_eager)
  elapsed_max = reps.max_over_ranks(elapsed)
  per_rank = reps.gather_stats([counters['steps'] - warm, elapsed,
                                counters['syncs'], counters['gathers']])
  # device identities: stand-ins here.  DQZ_SELFTEST_DEVICE overrides the
  # per-rank default so a test can make ranks collide: a plain name applies
  # to every rank, 'r=name,...' to the ranks it lists
  stand_in = 'stand-in-%d' % reps.rank
  spec = os.environ.get('DQZ_SELFTEST_DEVICE')
  if spec and '=' not in spec:
    stand_in = spec
  elif spec:
    stand_in = dict(kv.split('=', 1) for kv in spec.split(',')).get(str(reps.rank), stand_in)
  devices = reps.gather_objects(
      dict(replicas_lib.device_identity(reps.local_rank, stand_in=stand_in),
           fill_s=0.0))
  errors = replicas_lib.check_devices(devices, args.gpus)
  if errors:
    if reps.rank == 0:
      print('bench.py: %s' % '; '.join(errors), file=sys.stderr)
    reps.close()
    return 4
  if reps.rank == 0:
    print(json.dumps({
        'metric': METRIC + ' [CPU orchestration self-test]',
        'value': round(reps.world * args.steps / elapsed_max, 2),
        'unit': 'steps/s', 'n_gpus': reps.world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': 1e3 * elapsed_max / args.steps,
        'chunks': [g, rem],
        'per_rank_steps': [int(v) for v in per_rank[:, 0]],
        # the fields the GPU line carries per rank (the stand-in step's rate)
        'per_rank_steps_per_s': [round(float(v[0] / v[1]), 2) for v in per_rank],
        'per_gpu_min_steps_per_s': round(float((per_rank[:, 0] / per_rank[:, 1]).min()), 2),
        'per_rank_target_syncs': [int(v) for v in per_rank[:, 2]],
        'per_rank_stats_gathers': [int(v) for v in per_rank[:, 3]],
        'devices': devices,
        'rccl': {'backend': reps.backend, 'world': reps.world,
                 'last_in_loop_gather': None if 'stats' not in last else {
                     'steps_done': [int(v) for v in last['stats'][:, 0]],
                     'value': [float(v) for v in last['stats'][:, 1]]}}}),
          flush=True)
  reps.close()
  return 0


class Workload:
  """One BASELINE config's step on device: the learner, the replay it reads,
  `one_step()` (everything a step launches, capturable in a hipGraph) and
  the sampler launches to time apart from the learner phases."""

  def __init__(self, algo, capacity, rank, dev):
    from dqn_mgsc_zoo_amd import _native  # pylint: disable=g-import-not-at-top
    from dqn_mgsc_zoo_amd import learner as learner_lib  # pylint: disable=g-import-not-at-top
    from dqn_mgsc_zoo_amd import networks  # pylint: disable=g-import-not-at-top
    from dqn_mgsc_zoo_amd import synthetic  # pylint: disable=g-import-not-at-top
    self.algo = algo
    la = LEARNER_ALGO[algo]
    net = (networks.dqn_atari_network(NUM_ACTIONS) if la == 'dqn' else
           networks.double_dqn_atari_network(NUM_ACTIONS))
    self.lrn = lrn = learner_lib.Learner(net, BATCH, algo=la, device=dev)
    lrn.set_params(net.init(seed=rank))
    t_fill = time.perf_counter()
    self.store = store = synthetic.fill_episodic(capacity, NUM_ACTIONS,
                                                 seed=rank, device=dev)
    self.slots = slots = torch.zeros((BATCH,), dtype=torch.int32, device=dev)
    self.weights = None
    self.counter = counter = torch.zeros((1,), dtype=torch.int64, device=dev)
    seed = 1 + rank
    lib, ptr, stream = _native.lib(), _native.ptr, _native.stream_handle
    self.samplers = {}  # name -> launch fn (timed apart, HIP events)
    self.sampler_bytes = {}  # name -> algorithmic bytes per launch

    if algo in ('dqn', 'double'):
      def one_step():
        # FIFO replay full: live ids [t - size, t) = slots [0, capacity).
        # The uniform draw is fused into the step's conv1 kernel.
        lrn.step_uniform(store, 0, capacity, capacity, seed, counter, slots)
    elif algo == 'per':
      # 2^20-leaf fp64 sum tree over alpha-exponentiated random priorities
      tcap = 1 << max(1, (capacity - 1).bit_length())
      gen = torch.Generator(device=dev)
      gen.manual_seed(100 + rank)
      self.tree = tree = torch.zeros((2 * tcap,), dtype=torch.float64, device=dev)
      pri = torch.rand((capacity,), generator=gen, dtype=torch.float64,
                       device=dev) * 1.99 + 0.01
      idx_all = torch.arange(capacity, dtype=torch.int64, device=dev)
      pri = pri ** PER_ALPHA
      for s0 in range(0, capacity, 65536):  # <= 65536 leaves per call
        n = min(65536, capacity - s0)
        _native.check(lib.dqz_sumtree_set(
            ptr(tree), tcap, ptr(idx_all[s0:s0 + n]), ptr(pri[s0:s0 + n]), n,
            stream()))
      self.weights = w = torch.zeros((BATCH,), dtype=torch.float32, device=dev)
      self.max_seen = max_seen = torch.ones((1,), dtype=torch.float64, device=dev)

      def per_write_back():
        _native.check(lib.dqz_per_write_back(
            lrn._h, ptr(tree), tcap, ptr(slots), PER_ALPHA, ptr(max_seen),  # pylint: disable=protected-access
            stream()))

      self.per_idx = idx = torch.zeros((BATCH,), dtype=torch.int32, device=dev)
      self.per_probs = probs = torch.zeros((BATCH,), dtype=torch.float64, device=dev)
      self.draw = _native.DqzPerDraw(
          tree.data_ptr(), tcap, 0, capacity, capacity, PER_USP, PER_BETA, 1,
          seed, counter.data_ptr(), None, None, None, PER_ALPHA,
          max_seen.data_ptr(), idx.data_ptr(), slots.data_ptr(),
          probs.data_ptr(), w.data_ptr())
      self.sampler_counter = sc = torch.zeros((1,), dtype=torch.int64, device=dev)

      def per_sample_standalone():
        _native.check(lib.dqz_per_sample(
            ptr(tree), tcap, 0, capacity, capacity, BATCH, PER_USP, PER_BETA,
            1, seed, ptr(sc), None, None, None, None, ptr(slots), ptr(w),
            None, stream()))

      def one_step():
        # one call: the draw in the forward's conv1 workgroups, the IS
        # weights in the head, the |td|^alpha write-back in the backward
        lrn.step_per_draw(store, self.draw)
      # the stand-alone sampler and write-back launches, timed for reference
      self.samplers = {'per_sample_standalone': per_sample_standalone,
                       'per_write_back_standalone': per_write_back}
    elif algo == 'mgsc':
      from dqn_mgsc_zoo_amd import replay_circular as rc  # pylint: disable=g-import-not-at-top
      gen = torch.Generator(device=dev)
      gen.manual_seed(200 + rank)
      self.logit_buf = lb = rc._DeviceLogits(capacity, dev, max_queries=BATCH)  # pylint: disable=protected-access
      lb.logits.copy_(torch.randn((capacity,), generator=gen, device=dev))
      lb.invalidate()

      self.sampler_counter = sc = torch.zeros((1,), dtype=torch.int64, device=dev)

      def mgsc_sample():  # the stand-alone one-launch sampler, timed for reference
        lb.sample_slots_philox(seed, sc, slots)

      def one_step():
        # the draw runs inside the learner's forward launch
        lrn.step_logits(store, lb, slots, seed=seed, counter=counter)
      self.samplers = {'logits_sample_standalone': mgsc_sample}
      # The meta-update the agent runs once per learn step
      # (dqn_mgsc_batched/agent.py:253), M = 100, timed apart:
      # first order (dqn_mgsc_batched) and second order (the reservoir
      # variant), on a fixed meta batch and online transition.
      from dqn_mgsc_zoo_amd import replay as replay_lib  # pylint: disable=g-import-not-at-top
      rng = np.random.default_rng(300 + rank)
      self.meta_online = replay_lib.Transition(
          rng.integers(0, 256, (84, 84, 4), dtype=np.uint8), 2, 1.0, 0.99,
          rng.integers(0, 256, (84, 84, 4), dtype=np.uint8))
      self.meta_slots = torch.from_numpy(
          rng.choice(capacity, META_BATCH, replace=False).astype(np.int32)).to(dev)
    else:
      raise ValueError(algo)
    self.one_step = one_step
    torch.cuda.synchronize(dev)
    self.fill_s = time.perf_counter() - t_fill

  def time_meta(self, iters):
    """MGSC only: average ms per M = 100 meta-update, first and second order
    (HIP events around `iters` back-to-back calls after 3 untimed ones)."""
    if self.algo != 'mgsc':
      return {}
    from dqn_mgsc_zoo_amd import learner as learner_lib  # pylint: disable=g-import-not-at-top
    out = {}
    for order in (0, 1):
      meta = learner_lib.MetaLearner(self.lrn, META_BATCH, learner_lib.adam(2.5e-4),
                                     second_order=bool(order))
      meta.set_online_transition(self.meta_online)
      lb, ms = self.logit_buf, self.meta_slots
      fn = lambda: meta.update(self.store, ms, lb.logits, ms, logit_buffer=lb)  # pylint: disable=cell-var-from-loop
      for _ in range(3):
        fn()
      e0 = torch.cuda.Event(enable_timing=True)
      e1 = torch.cuda.Event(enable_timing=True)
      e0.record()
      for _ in range(iters):
        fn()
      e1.record()
      e1.synchronize()
      out['M%d_%s_order' % (META_BATCH, 'second' if order else 'first')] = e0.elapsed_time(e1) / iters
      del meta
    return out

  def time_mgsc_learn(self, graph_steps=20, reps=10):
    """MGSC only: config 3's whole learn step as the reference runs it on a
    learn frame (dqn_mgsc_batched/agent.py:253-275, 302-357): the M = 100
    meta-update (a fresh meta batch each step: uniform without replacement,
    positions = slots as in the reservoir buffer; the meta batch's logits
    written back, the running log-sum-exp kept), then the learned-logit draw
    of 32 slots and the DQN step (one call, the draw inside the forward
    launch).  A hipGraph of `graph_steps` such steps is replayed `reps`
    times between HIP events on the capture stream; first and second order
    (the batched and the reservoir agent).  The per-frame replay add
    (running log-mean-exp, 14 us per add at 1M) and the host's
    meta-batch draw are outside the timed graph."""
    if self.algo != 'mgsc':
      return {}
    from dqn_mgsc_zoo_amd import learner as learner_lib  # pylint: disable=g-import-not-at-top
    dev = self.slots.device
    rng = np.random.default_rng(400)
    cap = self.logit_buf.logits.numel()
    sets = torch.from_numpy(np.stack([
        rng.choice(cap, META_BATCH, replace=False).astype(np.int32)
        for _ in range(graph_steps)])).to(dev)
    lrn, lb, store = self.lrn, self.logit_buf, self.store
    out = {}
    for order in (0, 1):
      meta = learner_lib.MetaLearner(lrn, META_BATCH, learner_lib.adam(2.5e-4),
                                     second_order=bool(order))
      meta.set_online_transition(self.meta_online)
      counter = torch.zeros((1,), dtype=torch.int64, device=dev)

      def learn_step(k, meta=meta, counter=counter):
        ms = sets[k]
        meta.update(store, ms, lb.logits, ms, logit_buffer=lb)
        lrn.step_logits(store, lb, self.slots, seed=7, counter=counter)

      side = torch.cuda.Stream(dev)
      side.wait_stream(torch.cuda.current_stream(dev))
      with torch.cuda.stream(side):
        for k in range(3):  # eager warm-up: the buffer's running state is known
          learn_step(k)
      torch.cuda.current_stream(dev).wait_stream(side)
      graph = torch.cuda.CUDAGraph()
      with torch.cuda.graph(graph):
        for k in range(graph_steps):
          learn_step(k)
      graph.replay()
      graph.replay()
      e0 = torch.cuda.Event(enable_timing=True)
      e1 = torch.cuda.Event(enable_timing=True)
      e0.record()
      for _ in range(reps):
        graph.replay()
      e1.record()
      e1.synchronize()
      us = 1e3 * e0.elapsed_time(e1) / (reps * graph_steps)
      status = lrn.sync_status() | meta.sync_status()
      key = '%s_order' % ('second' if order else 'first')
      out[key] = {'us_per_learn_step': round(us, 2),
                  'learn_steps_per_s': round(1e6 / us, 1),
                  'meta_batch': META_BATCH, 'batch': BATCH,
                  'steps_timed': reps * graph_steps, 'health': int(status)}
      del graph, meta
    return out

  def time_samplers(self, iters):
    """Average ms per launch of each sampler call, back to back on the
    launch stream (HIP events on that stream)."""
    out = {}
    for name, fn in self.samplers.items():
      fn()
      e0 = torch.cuda.Event(enable_timing=True)
      e1 = torch.cuda.Event(enable_timing=True)
      e0.record()
      for _ in range(iters):
        fn()
      e1.record()
      e1.synchronize()
      out[name] = e0.elapsed_time(e1) / iters
    return out


def _json_stdout():
  """A private handle on the real stdout for the one JSON line; fd 1 itself
  goes to stderr, so whatever RCCL / HIP print at communicator creation
  cannot land on the line the driver parses."""
  out = os.fdopen(os.dup(1), 'w')
  sys.stdout.flush()
  os.dup2(2, 1)
  return out


def run_gpu(args, g, rem):
  from dqn_mgsc_zoo_amd import replicas as replicas_lib  # pylint: disable=g-import-not-at-top
  json_out = _json_stdout()
  local_rank = int(os.environ.get('LOCAL_RANK', '0'))
  torch.cuda.set_device(local_rank)
  rank = int(os.environ.get('RANK', '0'))
  dev = torch.device('cuda', local_rank)

  algo = args.algo
  wl = Workload(algo, args.capacity, rank, dev)
  lrn, store, slots, one_step = wl.lrn, wl.store, wl.slots, wl.one_step

  graphs = {}
  if args.graph:
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
      for _ in range(3):
        one_step()
    torch.cuda.current_stream(dev).wait_stream(side)
    for k in sorted({g, rem}):
      if k > 1:
        graphs[k] = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graphs[k]):
          for _ in range(k):
            one_step()

  # The RCCL group (replicas only, no gradient exchange).  Its communicator
  # is created by the first collective, here, before the warm-up steps: the
  # first graph replays after communicator creation are slow, and with the
  # driver's --steps 20 that one-off cost landed inside the timed region
  # (13,980 against 15,555 steps/s at 5,000 steps).
  reps = replicas_lib.Replicas('nccl')
  world = reps.world
  if world != args.gpus or reps.rank != rank:
    print('bench.py: world %d != --gpus %d' % (world, args.gpus), file=sys.stderr)
    return 2
  _barrier(reps)

  # Statistics vector [steps done, last loss, seconds since the timed region
  # began], all-gathered over RCCL every stats_every steps: enqueued on the
  # stream, never waited for inside the timed region, read after it.
  stats_vec = torch.zeros((STATS_LEN,), dtype=torch.float64, device=dev)
  gathered = torch.zeros((world, STATS_LEN), dtype=torch.float64, device=dev)
  pending = []
  clock = {'t0': time.perf_counter()}

  stats_mode = os.environ.get('DQZ_BENCH_STATS', 'sync')  # diagnostic A/B: sync | async

  def on_stats(done):
    lrn.fetch_outputs()
    stats_vec[0].fill_(float(done))
    stats_vec[1].copy_(lrn.loss[0])
    stats_vec[2].fill_(time.perf_counter() - clock['t0'])
    if reps.dist is None:
      return
    if stats_mode == 'async':
      pending.append(reps.dist.all_gather_into_tensor(gathered, stats_vec,
                                                      async_op=True))
      return
    # Drain the learner's queue first, then gather on an idle device: an
    # async gather enqueued behind the replayed graphs cost ~7 ms each
    # (13,200 against 14,630 steps/s over 20,000 steps, tools/ab_rccl.sh);
    # draining costs one pipeline refill per stats interval.
    torch.cuda.synchronize(dev)
    pending.append(reps.dist.all_gather_into_tensor(gathered, stats_vec,
                                                    async_op=True))
    pending[-1].wait()

  runner = StepRunner(one_step, graphs, args.target_period, lrn.sync_target,
                      args.stats_every, on_stats)
  runner.run(args.warmup, 1, 0)
  for k in graphs:  # first replays of each graph upload it: keep them untimed
    runner.run(2 * k, k, 0)
  warm_steps = runner.done
  pending.clear()  # warm-up gathers are not reported
  torch.cuda.synchronize(dev)
  clock['t0'] = time.perf_counter()
  elapsed = _timed(reps, runner, args.steps, g, rem,
                   lambda: torch.cuda.synchronize(dev), lead=args.lead_eager)
  steps = args.steps
  for w in pending:
    w.wait()
  in_loop = gathered.cpu().numpy() if pending else None
  status = lrn.sync_status()  # in-launch hand-off health over every step run
  elapsed_max = reps.max_over_ranks(elapsed, device=dev)
  status_max = reps.max_over_ranks(float(status), device=dev)
  lrn.fetch_outputs()
  per_rank = reps.gather_stats([steps / elapsed, elapsed, float(steps),
                                float(lrn.loss[0].item())], device=dev)
  # which device each rank ran on, and its replay fill time: a line from N
  # ranks is only valid with N distinct devices (SCALE runs, config 5)
  devices = reps.gather_objects(
      dict(replicas_lib.device_identity(local_rank), fill_s=round(wl.fill_s, 2)))
  dev_errors = replicas_lib.check_devices(devices, args.gpus)
  if dev_errors:
    if rank == 0:
      print('bench.py: %s: the line is invalid' % '; '.join(dev_errors),
            file=sys.stderr)
    reps.close()
    return 4

  # Per-phase device time (HIP events on the launch stream) for the roofline.
  phases = lrn.profile(store, slots, weights=wl.weights, iters=args.profile_iters)
  if 'conv1_fwd' in phases and 'conv2_fwd' not in phases:  # the one conv1..conv3 launch
    phases = {('conv_fwd' if k == 'conv1_fwd' else k): v for k, v in phases.items()}
  sampler_ms = wl.time_samplers(args.profile_iters)
  meta_ms = wl.time_meta(max(20, args.profile_iters // 10))
  mgsc_learn = wl.time_mgsc_learn()
  q_tm1, td, loss = lrn.fetch_outputs()
  torch.cuda.synchronize(dev)
  finite = bool(torch.isfinite(lrn.online).all().item())
  status_after = lrn.sync_status()

  if rank != 0:
    reps.close()
    return 0 if (status == 0 and status_after == 0) else 3

  value = world * steps / elapsed_max
  flops = phase_flops(algo, BATCH)
  nbytes = phase_bytes(algo, BATCH)
  timed_phases = dict(phases)
  for k, v in sampler_ms.items():
    if k in wl.sampler_bytes:  # HBM-bound samplers compete for the roofline
      timed_phases[k] = v
      flops[k] = 0
      nbytes[k] = wl.sampler_bytes[k]
  dom = max(timed_phases, key=timed_phases.get)
  dom_ms = timed_phases[dom]
  # The bound is whichever roof the kernel sits closer to.
  tflops = flops[dom] / (dom_ms * 1e-3) / 1e12
  gbs = nbytes[dom] / (dom_ms * 1e-3) / 1e9
  mfma_frac = tflops / F32_MFMA_PEAK_TFLOPS
  hbm_frac = gbs / HBM_PEAK_GBS
  if mfma_frac >= hbm_frac:
    roof = {'bound': 'mfma', 'achieved': round(tflops, 3),
            'peak': F32_MFMA_PEAK_TFLOPS, 'unit': 'TFLOP/s',
            'frac': round(mfma_frac, 4)}
  else:
    roof = {'bound': 'hbm', 'achieved': round(gbs, 1), 'peak': HBM_PEAK_GBS,
            'unit': 'GB/s', 'frac': round(hbm_frac, 4)}
  roof.update({
      'traffic': pmc_traffic(dom) if algo == 'dqn' else None,
      'kernel': PHASE_KERNEL.get(dom, dom) + ' (' + dom + ')',
      'kernel_ms': round(dom_ms, 5),
      'algorithmic_flop_per_launch': flops[dom],
      'algorithmic_bytes_per_launch': nbytes[dom],
      'mfma_frac': round(mfma_frac, 4), 'hbm_frac': round(hbm_frac, 4),
      'flop_basis': 'algorithmic f32-equivalent FLOP over the exact-f32 MFMA '
                    'peak; conv1 fwd / dW issue three bf16 piece products per '
                    'multiply on bf16 MFMA, counted once here'})
  per_gpu = steps / elapsed
  step_tflops = STEP_FLOP[algo] * per_gpu / 1e12
  step_gbs = STEP_BYTES[algo] * per_gpu / 1e9
  rccl = {'backend': reps.backend, 'world': world, 'devices': devices,
          'in_loop_gathers': len(pending), 'stats_every': args.stats_every,
          'final_gather': {'steps_per_s': [round(float(x), 2) for x in per_rank[:, 0]],
                           'steps': [int(x) for x in per_rank[:, 2]],
                           'last_loss': [float(x) for x in per_rank[:, 3]],
                           'loss_mean': float(per_rank[:, 3].mean())}}
  if in_loop is not None:
    rccl['last_in_loop_gather'] = {
        'steps_done': [int(x) for x in in_loop[:, 0]],
        'loss': [float(x) for x in in_loop[:, 1]],
        'loss_mean': float(in_loop[:, 1].mean()),
        'seconds': [round(float(x), 4) for x in in_loop[:, 2]]}
  out = {
      'metric': METRIC,
      'value': round(value, 2),
      'unit': 'steps/s',
      'n_gpus': world,
      'steps': steps,
      'warmup': args.warmup,
      'ms_per_step': round(1e3 * elapsed_max / steps, 5),
      'higher_is_better': True,
      'scaling': 'weak',
      'vs_baseline': None,
      'dtype': 'f32',
      'numerics': 'f32 everywhere; conv1 fwd / dW on bf16 MFMA with exact operands '
                  '(integer pixels x three-piece exact bf16 splits of the f32 weights / dy1: '
                  'every product exact, f32 accumulation)',
      'data': 'synthetic (uint8 U{0..255} frames, 1000-transition episodes, '
              'random-init NatureQNetwork)',
      'config': {'workload': '%s, synthetic 84x84x4 uint8 replay pre-filled to '
                             '%d, batch=32, A=%d, algo=%s' % (
                                 WORKLOAD[algo], args.capacity, NUM_ACTIONS, algo),
                 'global_batch': BATCH * world, 'replay_capacity': args.capacity,
                 'parallelism': 'independent-seed replicas x%d' % world,
                 'hipgraph_chunks': [g, rem],
                 'lead_eager_steps': args.lead_eager,
                 'warmup_steps_run': warm_steps},
      'roofline': roof,
      'step_roofline': {
          'achieved_tflops': round(step_tflops, 3),
          'frac_f32_mfma': round(step_tflops / F32_MFMA_PEAK_TFLOPS, 4),
          'achieved_gbs': round(step_gbs, 1),
          'frac_hbm': round(step_gbs / HBM_PEAK_GBS, 4),
          'flop_per_step': STEP_FLOP[algo], 'bytes_per_step': STEP_BYTES[algo]},
      'phase_ms': {k: round(v, 5) for k, v in phases.items()},
      'sampler_us': {k: round(1e3 * v, 3) for k, v in sampler_ms.items()},
      'per_rank_steps_per_s': [round(float(x), 2) for x in per_rank[:, 0]],
      'per_gpu_min_steps_per_s': round(float(per_rank[:, 0].min()), 2),
      'rccl': rccl,
      # learner health word (dqz_learner_sync_status): bit 0 a hand-off wait
      # gave up, bit 1 a step's mean loss was not finite
      'handoff_status': int(max(status_max, status_after)) & 1,
      'nonfinite_loss': bool(int(max(status_max, status_after)) & 2),
      'fill_s': round(wl.fill_s, 2),
      'last_loss': float(loss.item()),
      'params_finite': finite,
  }
  if algo == 'mgsc':
    # the reference's own per-call timings of this agent (V100 + JAX):
    # dqn_mgsc_batched/run_atari.py:308-315
    out['reference_per_call_ms'] = {'update': 12.24, 'replay_sample_batch': 57.1,
                                    # 206.19 s / 49,924 calls, --meta_batch_size=5
                                    # (run_mgscdqnbatched_normal_timing.sh:50)
                                    'meta_update_M5': 4.13,
                                    'replay_sample_meta_batch': 55.6}
    out['meta_update_us'] = {k: round(1e3 * v, 2) for k, v in meta_ms.items()}
    meta_roof = {}
    for order in ('first', 'second'):
      ms = meta_ms.get('M%d_%s_order' % (META_BATCH, order))
      if ms:
        tf = META_FLOP[order] / (ms * 1e-3) / 1e12
        meta_roof[order] = {'algorithmic_flop': META_FLOP[order], 'us': round(1e3 * ms, 2),
                            'achieved_tflops': round(tf, 3), 'peak': F32_MFMA_PEAK_TFLOPS,
                            'frac': round(tf / F32_MFMA_PEAK_TFLOPS, 4)}
    out['meta_roofline'] = meta_roof
    # config 3 as one learn frame of the reference: meta-update (M = 100),
    # then the learned-logit draw and the DQN step, in one captured graph;
    # `value` above stays the learner part alone
    out['mgsc_learn_step'] = mgsc_learn
  if world == 1 and args.cpu_seconds > 0:
    out['cpu_baseline'] = cpu_baseline(args.cpu_seconds, algo)
  else:
    out['cpu_baseline'] = None
  print(json.dumps(out), file=json_out, flush=True)
  reps.close()
  if out['handoff_status'] != 0 or out['nonfinite_loss'] or not finite:
    print('bench.py: hand-off status %d, non-finite loss %s, params finite %s: '
          'the timed steps are invalid' % (out['handoff_status'], out['nonfinite_loss'],
                                           finite), file=sys.stderr)
    return 3
  return 0


# The reference's own training frame rate of this agent: median
# train_frame_rate of results/dqn/seed_0.csv (iterations 1-50, 1,103-1,168;
# Pong, its cluster's GPU + JAX, the ALE emulator inside the loop).
REFERENCE_TRAIN_FRAMES_PER_S = 1136.0


def run_agent(args):
  """BASELINE config 1: the dqn agent (dqn/run_atari.py:204-294) on device.

  parts.run_loop drives agent.Dqn over raw Atari-shaped RGB frames
  (synthetic.SyntheticAtari: no ALE here) through processors.atari (the
  observation math on device), a TransitionReplay(capacity) with the
  RandomState, batch 32, learn period 16, target period 40,000 frames,
  centered RMSProp.  Frames are stepped until learning has begun and
  `--warmup` learner steps ran; then exactly `--steps` learner steps (16
  frames each) are timed, act + preprocess + add + learn included."""
  from dqn_mgsc_zoo_amd import learner as learner_lib  # pylint: disable=g-import-not-at-top
  from dqn_mgsc_zoo_amd import networks  # pylint: disable=g-import-not-at-top
  from dqn_mgsc_zoo_amd import parts  # pylint: disable=g-import-not-at-top
  from dqn_mgsc_zoo_amd import processors  # pylint: disable=g-import-not-at-top
  from dqn_mgsc_zoo_amd import replay as replay_lib  # pylint: disable=g-import-not-at-top
  from dqn_mgsc_zoo_amd import replicas as replicas_lib  # pylint: disable=g-import-not-at-top
  from dqn_mgsc_zoo_amd import synthetic  # pylint: disable=g-import-not-at-top
  from dqn_mgsc_zoo_amd.dqn import agent as agent_lib  # pylint: disable=g-import-not-at-top
  json_out = _json_stdout()
  local_rank = int(os.environ.get('LOCAL_RANK', '0'))
  torch.cuda.set_device(local_rank)
  rank = int(os.environ.get('RANK', '0'))
  dev = torch.device('cuda', local_rank)
  learn_period = 16
  random_state = np.random.RandomState(1 + rank)
  replay = replay_lib.TransitionReplay(
      args.capacity, replay_lib.Transition(None, None, None, None, None),
      random_state)
  agent = agent_lib.Dqn(
      preprocessor=processors.atari(),
      sample_network_input=np.zeros((84, 84, 4), np.uint8),
      network=networks.dqn_atari_network(NUM_ACTIONS),
      optimizer=learner_lib.rmsprop(2.5e-4, 0.95, 0.01 / 32**2, centered=True),
      transition_accumulator=replay_lib.TransitionAccumulator(),
      replay=replay, batch_size=BATCH,
      # dqn/run_atari.py: epsilon 1 -> 0.1 over 0.02 x 200 iterations x 1M frames
      exploration_epsilon=parts.LinearSchedule(
          begin_t=int(args.min_replay_fraction * args.capacity * 4),
          decay_steps=4_000_000, begin_value=1.0, end_value=0.1),
      min_replay_capacity_fraction=args.min_replay_fraction,
      learn_period=learn_period, target_network_update_period=40_000,
      grad_error_bound=1.0 / 32, rng_key=np.array([0, 1 + rank], np.uint32),
      device=dev)
  counts = {'learn': 0}
  orig_learn = agent._learn  # pylint: disable=protected-access

  def learn():
    counts['learn'] += 1
    orig_learn()

  agent._learn = learn  # pylint: disable=protected-access
  counts['target_syncs'] = 0
  orig_sync = agent._learner.sync_target  # pylint: disable=protected-access

  def sync_target():
    counts['target_syncs'] += 1
    orig_sync()

  agent._learner.sync_target = sync_target  # pylint: disable=protected-access
  env = synthetic.SyntheticAtari(episode_len=27_000, seed=1 + rank,
                                 num_actions=NUM_ACTIONS)
  loop = parts.run_loop(agent, env, max_steps_per_episode=108_000)
  t_fill = time.perf_counter()
  fill_frames = 0
  while counts['learn'] < max(1, args.warmup):
    next(loop)
    fill_frames += 1
  torch.cuda.synchronize(dev)
  fill_s = time.perf_counter() - t_fill
  reps = replicas_lib.Replicas('nccl')
  _barrier(reps)
  torch.cuda.synchronize(dev)
  start = counts['learn']
  syncs0 = counts['target_syncs']
  frames = 0
  t0 = time.perf_counter()
  while counts['learn'] - start < args.steps:
    next(loop)
    frames += 1
  torch.cuda.synchronize(dev)
  elapsed = time.perf_counter() - t0
  _barrier(reps)
  status = agent.check_learner_health()
  ok, msg = replay.check_valid()
  elapsed_max = reps.max_over_ranks(elapsed, device=dev)
  per_rank = reps.gather_stats([args.steps / elapsed, frames / elapsed,
                                float(frames)], device=dev)
  devices = reps.gather_objects(
      dict(replicas_lib.device_identity(dev.index), fill_s=round(fill_s, 2)))
  dev_errors = replicas_lib.check_devices(devices, args.gpus)
  if dev_errors:
    if rank == 0:
      print('bench.py: %s: the line is invalid' % '; '.join(dev_errors),
            file=sys.stderr)
    reps.close()
    return 4
  finite = bool(torch.isfinite(agent.learner.online).all().item())
  if rank != 0:
    reps.close()
    return 0 if (status == 0 and ok and finite) else 3
  world = reps.world
  out = {
      'metric': AGENT_METRIC,
      'value': round(world * args.steps / elapsed_max, 2),
      'unit': 'steps/s',
      'n_gpus': world,
      'steps': args.steps,
      'warmup': args.warmup,
      'ms_per_step': round(1e3 * elapsed_max / args.steps, 5),
      'higher_is_better': True,
      'scaling': 'weak',
      'vs_baseline': None,
      'dtype': 'f32',
      'data': 'synthetic (Atari-shaped 210x160x3 uint8 RGB frames from a seeded '
              'pool, lives, rewards; random-init NatureQNetwork)',
      'config': {'workload': 'BASELINE config 1: dqn agent, parts.run_loop over '
                             'raw frames through processors.atari (device '
                             'observation math), TransitionReplay(capacity=%d, '
                             'RandomState), batch=32, learn_period=16, '
                             'min_replay_capacity_fraction=%g, '
                             'target_network_update_period=40000 frames, '
                             'A=%d' % (args.capacity, args.min_replay_fraction,
                                       NUM_ACTIONS),
                 'target_update_period_frames': 40_000,
                 'min_replay_capacity_fraction': args.min_replay_fraction,
                 'global_batch': BATCH * world, 'replay_capacity': args.capacity,
                 'parallelism': 'independent-seed replicas x%d' % world},
      'frames': frames,
      'frames_per_s': round(world * frames / elapsed_max, 1),
      'learner_steps_per_s': round(world * args.steps / elapsed_max, 2),
      'per_rank_frames_per_s': [round(float(x), 1) for x in per_rank[:, 1]],
      'reference_train_frames_per_s': REFERENCE_TRAIN_FRAMES_PER_S,
      'reference_note': 'median train_frame_rate of results/dqn/seed_0.csv '
                        '(Pong, ALE emulator inside the loop); this loop steps '
                        'a synthetic environment',
      'replay_size': replay.size,
      'replay_valid': bool(ok),
      'fill_frames': fill_frames,
      'target_syncs_timed': counts['target_syncs'] - syncs0,
      'fill_s': round(fill_s, 2),
      'handoff_status': int(status) & 1,
      'params_finite': finite,
      'roofline': None,
      'cpu_baseline': None,
  }
  print(json.dumps(out), file=json_out, flush=True)
  reps.close()
  if status & 1 or not ok or not finite:
    print('bench.py: agent run invalid (status %d, replay %s, finite %s)' % (
        status, msg, finite), file=sys.stderr)
    return 3
  return 0


if __name__ == '__main__':
  sys.exit(main())
