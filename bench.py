"""Learner grad-steps/s at batch 32 on synthetic 84x84x4 uint8 replay.

`python bench.py --gpus N --steps K --warmup W` (N>1 under
torch.distributed.run, one process per GPU).  A *step* is one pass of the
hot path on device: uniform sample of 32 slots from a 1M-transition frame
replay (Philox on device) -> frame gather + /255 fused into conv1 ->
NatureQNetwork forward of online(s_tm1) and target(s_t) -> q_learning TD
loss with clip_gradient -> backward -> centered RMSProp; the target copy
runs every 2,500 steps (40,000 frames / learn_period 16) inside the timed
loop.  Replicas are independent seeds (no gradient all-reduce); RCCL only
all-gathers per-rank statistics after the timed region.

Prints ONE JSON line on rank 0.
"""

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
  sys.path.insert(0, ROOT)

METRIC = ('learner grad-steps/sec at batch=32, 84×84×4 uint8, '
          '1/2/4/8 MI355X')
BATCH = 32
NUM_ACTIONS = 6  # Pong minimal action set (gym_atari.py:52-54)
F32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32 = f32 vector peak
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
STEP_FLOP = {'dqn': 2182873088, 'double': 2781020160}
STEP_BYTES = {'dqn': 49048488, 'double': 49048488}

ALL_BWD = 'conv3_dx+conv2_dx+fc1_dw+conv3_dw+conv2_dw+conv1_dw'

# Algorithmic MACs per sample of each forward layer.
MAC = dict(conv1=400 * 256 * 32, conv2=81 * 512 * 64, conv3=49 * 576 * 64,
           fc1=3136 * 512, fc2=512 * NUM_ACTIONS)


def phase_flops(algo, batch):
  """Algorithmic FLOPs of each libdqz phase (one launch each)."""
  z = 2 if algo == 'dqn' else 3
  b = batch
  return {
      'conv1_fwd': 2 * z * b * MAC['conv1'],
      'conv2_fwd': 2 * z * b * MAC['conv2'],
      'conv3_fwd': 2 * z * b * MAC['conv3'],
      'fc1_fwd': 2 * z * b * MAC['fc1'],
      'head': 2 * z * b * MAC['fc2'],
      'fc1_dx': 2 * b * MAC['fc1'],
      'head+fc1_dx': 2 * z * b * MAC['fc2'] + 2 * b * MAC['fc1'],
      'conv3_dx+fc1_dw': 2 * b * (MAC['conv3'] + MAC['fc1']),
      'conv2_dx+conv3_dw': 2 * b * (MAC['conv2'] + MAC['conv3']),
      'conv3_dx+conv2_dx+fc1_dw+conv3_dw': 2 * b * (2 * MAC['conv3'] + MAC['fc1'] +
                                                   MAC['conv2']),
      'conv1_dw+conv2_dw': 2 * b * (MAC['conv1'] + MAC['conv2']),
      ALL_BWD: 2 * b * (2 * MAC['conv3'] + MAC['fc1'] + 2 * MAC['conv2'] + MAC['conv1']),
      'update': 0,
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
  partials) is excluded.  Centered RMSProp reads and writes theta, mu, nu
  (6 x 4 B per parameter); fc1's update runs inside conv3_dx+fc1_dw.
  """
  z = 2 if algo == 'dqn' else 3
  b = batch
  rms = 6 * (sum(PARAM.values()) - PARAM['fc1'])
  return {
      'conv1_fwd': z * b * (ACT['state'] + ACT['y1']) + z * PARAM['conv1'],
      'conv2_fwd': z * b * (ACT['y1'] + ACT['y2']) + z * PARAM['conv2'],
      'conv3_fwd': z * b * (ACT['y2'] + ACT['y3']) + z * PARAM['conv3'],
      'fc1_fwd': z * b * (ACT['y3'] + ACT['h']) + z * PARAM['fc1'],
      'head': z * b * ACT['h'] + z * PARAM['fc2'],
      'fc1_dx': b * (ACT['h'] + 2 * ACT['y3']) + PARAM['fc1'],
      # one launch (head_dx_kernel): dz1 is handed off inside it
      'head+fc1_dx': (z * b * ACT['h'] + z * PARAM['fc2'] + 2 * b * ACT['y3'] +
                      PARAM['fc1']),
      'conv3_dx+fc1_dw': (b * (ACT['y3'] + 2 * ACT['y2']) + PARAM['conv3'] +
                          b * (ACT['y3'] + ACT['h']) + 6 * PARAM['fc1']),
      'conv2_dx+conv3_dw': (b * (ACT['y2'] + 2 * ACT['y1']) + PARAM['conv2'] +
                            b * (ACT['y2'] + ACT['y3']) + PARAM['conv3']),
      # one launch (bwd_bc_kernel): dy2 is handed off inside it, dy3 and y2
      # are read once
      'conv3_dx+conv2_dx+fc1_dw+conv3_dw': (
          b * (ACT['y3'] + ACT['y2'] + 2 * ACT['y1']) + 2 * PARAM['conv3'] +
          PARAM['conv2'] + b * (ACT['y3'] + ACT['h']) + 6 * PARAM['fc1']),
      'conv1_dw+conv2_dw': (b * (ACT['state'] + ACT['y1']) + PARAM['conv1'] +
                            b * (ACT['y1'] + ACT['y2']) + PARAM['conv2']),
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
    'conv3_fwd': 'conv3_fwd_kernel', 'fc1_fwd': 'fc1_fwd_kernel',
    'head': 'head_kernel', 'fc1_dx': 'fc1_dx_kernel',
    'head+fc1_dx': 'head_dx_kernel',
    'conv3_dx+fc1_dw': 'bwd_b_kernel', 'conv2_dx+conv3_dw': 'bwd_c_kernel',
    'conv3_dx+conv2_dx+fc1_dw+conv3_dw': 'bwd_bc_kernel',
    'conv1_dw+conv2_dw': 'bwd_d_kernel', ALL_BWD: 'bwd_bc_kernel',
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
  """Times the oracle's fp64 learner step (a CPU *port*) on this host."""
  from threadpoolctl import threadpool_info, threadpool_limits  # pylint: disable=g-import-not-at-top
  from oracle import learner_ref  # pylint: disable=g-import-not-at-top
  from dqn_mgsc_zoo_amd import networks  # pylint: disable=g-import-not-at-top
  threads = min(16, os.cpu_count() or 1)
  net = (networks.dqn_atari_network(NUM_ACTIONS) if algo == 'dqn' else
         networks.double_dqn_atari_network(NUM_ACTIONS))
  rng = np.random.default_rng(0)
  params = net.init(0)
  mu = learner_ref.zeros_like_tree(params)
  nu = learner_ref.zeros_like_tree(params)
  with threadpool_limits(limits=threads):
    blas = [i.get('num_threads') for i in threadpool_info()]
    used = max([t for t in blas if t] + [1])
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
      s_tm1 = rng.integers(0, 256, (BATCH, 84, 84, 4), dtype=np.uint8)
      s_t = rng.integers(0, 256, (BATCH, 84, 84, 4), dtype=np.uint8)
      a = rng.integers(0, NUM_ACTIONS, BATCH)
      r = rng.choice([-1.0, 0.0, 1.0], BATCH, p=[0.01, 0.98, 0.01])
      d = np.full(BATCH, 0.99)
      out = learner_ref.learner_step(params, params, mu, nu, s_tm1, a, r, d,
                                     s_t, algo=algo)
      params, mu, nu = out['params'], out['mu'], out['nu']
      n += 1
    dt = time.perf_counter() - t0
  return {'value': n / dt, 'unit': 'steps/s', 'cores': used, 'kind': 'port',
          'sample': '%d oracle fp64 numpy learner steps (B=32, 84x84x4 uint8, '
                    '%s) in %.1f s, BLAS threads=%d' % (n, algo, dt, used)}


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument('--gpus', type=int, default=1)
  ap.add_argument('--steps', type=int, default=5000)
  ap.add_argument('--warmup', type=int, default=200)
  ap.add_argument('--algo', default='dqn', choices=['dqn', 'double'])
  ap.add_argument('--capacity', type=int, default=1_000_000)
  ap.add_argument('--graph', type=int, default=1, help='hipGraph-replay steps')
  ap.add_argument('--graph-steps', type=int, default=50)
  ap.add_argument('--target-period', type=int, default=2500)
  ap.add_argument('--profile-iters', type=int, default=100)
  ap.add_argument('--cpu-seconds', type=float, default=15.0)
  args = ap.parse_args()

  from dqn_mgsc_zoo_amd import replicas as replicas_lib  # pylint: disable=g-import-not-at-top
  local_rank = int(os.environ.get('LOCAL_RANK', '0'))
  torch.cuda.set_device(local_rank)
  reps = replicas_lib.Replicas('nccl')  # RCCL; replicas only, no grad exchange
  world, rank = reps.world, reps.rank
  dev = torch.device('cuda', local_rank)

  from dqn_mgsc_zoo_amd import learner as learner_lib  # pylint: disable=g-import-not-at-top
  from dqn_mgsc_zoo_amd import networks  # pylint: disable=g-import-not-at-top
  from dqn_mgsc_zoo_amd import synthetic  # pylint: disable=g-import-not-at-top

  algo = args.algo
  net = (networks.dqn_atari_network(NUM_ACTIONS) if algo == 'dqn' else
         networks.double_dqn_atari_network(NUM_ACTIONS))
  lrn = learner_lib.Learner(net, BATCH, algo=algo, device=dev)
  lrn.set_params(net.init(seed=rank))
  t_fill = time.perf_counter()
  store = synthetic.fill_episodic(args.capacity, NUM_ACTIONS, seed=rank,
                                  device=dev)
  torch.cuda.synchronize(dev)
  t_fill = time.perf_counter() - t_fill
  slots = torch.zeros((BATCH,), dtype=torch.int32, device=dev)
  counter = torch.zeros((1,), dtype=torch.int64, device=dev)
  seed = 1 + rank

  def one_step():
    # FIFO replay full: live ids [t - size, t) = slots [0, capacity).  The
    # uniform draw is fused into the step's conv1 kernel.
    lrn.step_uniform(store, 0, args.capacity, args.capacity, seed, counter,
                     slots)

  g = args.graph_steps if args.graph else 1
  graph = None
  if args.graph:
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
      for _ in range(3):
        one_step()
    torch.cuda.current_stream(dev).wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
      for _ in range(g):
        one_step()

  def run(n_steps, done):
    i = 0
    while i < n_steps:
      if graph is not None and n_steps - i >= g:
        graph.replay()
        k = g
      else:
        one_step()
        k = 1
      before = done + i
      i += k
      # target sync each time the step count crosses a period boundary
      if (done + i) // args.target_period > before // args.target_period:
        lrn.sync_target()
    return done + i

  done = run(args.warmup, 0)
  steps = (args.steps // g) * g if graph is not None else args.steps
  reps.barrier()
  torch.cuda.synchronize(dev)
  ev0 = torch.cuda.Event(enable_timing=True)
  ev1 = torch.cuda.Event(enable_timing=True)
  t0 = time.perf_counter()
  ev0.record()
  done = run(steps, done)
  ev1.record()
  torch.cuda.synchronize(dev)
  elapsed = time.perf_counter() - t0
  reps.barrier()
  gpu_ms = ev0.elapsed_time(ev1)
  elapsed_max = reps.max_over_ranks(elapsed, device=dev)
  per_rank = reps.gather_stats([steps / elapsed, elapsed, gpu_ms / 1e3],
                               device=dev)

  # Per-phase device time (HIP events on the launch stream) for the roofline.
  phases = lrn.profile(store, slots, iters=args.profile_iters)
  q_tm1, td, loss = lrn.fetch_outputs()
  torch.cuda.synchronize(dev)
  finite = bool(torch.isfinite(lrn.online).all().item())

  if rank != 0:
    reps.close()
    return

  value = world * steps / elapsed_max
  flops = phase_flops(algo, BATCH)
  nbytes = phase_bytes(algo, BATCH)
  dom = max(phases, key=phases.get)
  dom_ms = phases[dom]
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
      'kernel': PHASE_KERNEL[dom] + ' (' + dom + ')',
      'kernel_ms': round(dom_ms, 5),
      'algorithmic_flop_per_launch': flops[dom],
      'algorithmic_bytes_per_launch': nbytes[dom],
      'mfma_frac': round(mfma_frac, 4), 'hbm_frac': round(hbm_frac, 4)})
  per_gpu = steps / elapsed
  step_tflops = STEP_FLOP[algo] * per_gpu / 1e12
  step_gbs = STEP_BYTES[algo] * per_gpu / 1e9
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
      'data': 'synthetic (uint8 U{0..255} frames, 1000-transition episodes, '
              'random-init NatureQNetwork)',
      'config': {'workload': 'dqn agent learner-only loop, synthetic 84x84x4 '
                             'uint8 replay pre-filled to %d, batch=32, A=%d, '
                             'algo=%s' % (args.capacity, NUM_ACTIONS, algo),
                 'global_batch': BATCH * world, 'replay_capacity': args.capacity,
                 'parallelism': 'independent-seed replicas x%d' % world,
                 'hipgraph_steps': g},
      'roofline': roof,
      'step_roofline': {
          'achieved_tflops': round(step_tflops, 3),
          'frac_f32_mfma': round(step_tflops / F32_MFMA_PEAK_TFLOPS, 4),
          'achieved_gbs': round(step_gbs, 1),
          'frac_hbm': round(step_gbs / HBM_PEAK_GBS, 4),
          'flop_per_step': STEP_FLOP[algo], 'bytes_per_step': STEP_BYTES[algo]},
      'phase_ms': {k: round(v, 5) for k, v in phases.items()},
      'per_rank_steps_per_s': [round(float(x), 2) for x in per_rank[:, 0]],
      'gpu_event_s': round(gpu_ms / 1e3, 4),
      'fill_s': round(t_fill, 2),
      'last_loss': float(loss.item()),
      'params_finite': finite,
  }
  if world == 1 and args.cpu_seconds > 0:
    out['cpu_baseline'] = cpu_baseline(args.cpu_seconds, algo)
  else:
    out['cpu_baseline'] = None
  print(json.dumps(out), flush=True)
  reps.close()


if __name__ == '__main__':
  main()
