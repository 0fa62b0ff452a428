"""Full agent loop throughput: parts.run_loop over a synthetic Atari-like env.

usage (GPU box): python tools/agent_loop_bench.py [--frames N] [--kind dqn|double|mgsc|mgsc_reservoir]

Drives the DQN agent as run_atari does: one agent.step per environment
frame, the processor returning a stacked observation every 4th frame
(action repeat 4, processors.py:453-505; the other frames repeat the last
action), act + add on those, learn every 16 frames once the replay holds 5 %
of its capacity, hard target copy every 40,000 frames.  Frames are seeded
random 84x84 uint8 (FakeAtari).  Reports frames/s and learner steps/s after
a warm-up past the learning threshold, and host time per act / add / learn
(perf_counter brackets around the agent's own methods).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from dqn_mgsc_zoo_amd import learner as learner_lib  # noqa: E402
from dqn_mgsc_zoo_amd import networks, parts  # noqa: E402
from dqn_mgsc_zoo_amd import replay as replay_lib  # noqa: E402
from dqn_mgsc_zoo_amd import synthetic  # noqa: E402
from tests import fake_env  # noqa: E402


FakeRGBAtari = synthetic.SyntheticAtari


def host_atari_frame(obs):
  """The reference's host observation math (processors.py:488-497)."""
  from PIL import Image  # pylint: disable=g-import-not-at-top
  pooled = np.max(np.stack(list(obs)[-2:], axis=0), axis=0)
  y = np.tensordot(pooled, [0.299, 0.587, 1 - (0.299 + 0.587)], (-1, 0)).astype(np.uint8)
  return np.array(Image.fromarray(y).resize((84, 84), Image.Resampling.BILINEAR), dtype=np.uint8)


class RepeatStacker(fake_env.FrameStacker):
  """FrameStacker that emits every `repeat`-th frame (None in between)."""

  def __init__(self, repeat=4):
    super().__init__()
    self._repeat = repeat
    self._k = 0

  def __call__(self, timestep):
    if timestep.first():
      self._k = 0
    self._k += 1
    if not (timestep.first() or timestep.last()) and self._k % self._repeat:
      return None
    return super().__call__(timestep)


def make_mgsc_agent(kind, capacity, seed=0, preprocessor=None, meta_batch=100):
  """dqn_mgsc_batched (FIFO logits, first-order meta-gradient) or
  dqn_mgsc_batched_reservoir (reservoir logits, second order), with the
  reference's training settings (run_mgscdqnbatched_normal.sh /
  run_mgscdqnbatched_reservoir.sh: meta batch 100, learn period 16)."""
  from dqn_mgsc_zoo_amd import replay_circular as rc  # pylint: disable=g-import-not-at-top
  if kind == 'mgsc':
    from dqn_mgsc_zoo_amd.dqn_mgsc_batched import agent as agent_lib  # pylint: disable=g-import-not-at-top
    replay = rc.MGSCFiFoTransitionReplay(capacity, rc.Transition(None, None, None, None, None),
                                         np.random.default_rng(seed))
  else:
    from dqn_mgsc_zoo_amd.dqn_mgsc_batched_reservoir import agent as agent_lib  # pylint: disable=g-import-not-at-top
    replay = rc.MGSCReservoirTransitionReplay(capacity, rc.Transition(None, None, None, None, None),
                                              np.random.default_rng(seed))
  return agent_lib.MGSCDqn(
      preprocessor=preprocessor or RepeatStacker(),
      sample_network_input=np.zeros((84, 84, 4), np.uint8),
      network=networks.dqn_atari_network(6),
      optimizer=learner_lib.rmsprop(2.5e-4, 0.95, 0.01 / 32**2, centered=True),
      transition_accumulator=rc.TransitionAccumulator(), replay=replay, batch_size=32,
      exploration_epsilon=parts.LinearSchedule(
          begin_t=0, decay_steps=1_000_000, begin_value=1.0, end_value=0.1),
      min_replay_capacity_fraction=0.05, learn_period=16,
      target_network_update_period=40_000, grad_error_bound=1.0 / 32,
      rng_key=np.array([0, seed], np.uint32),
      meta_optimizer=learner_lib.adam(2.5e-4), meta_batch_size=meta_batch)


def make_agent(kind, capacity, seed=0, preprocessor=None):
  if kind in ('mgsc', 'mgsc_reservoir'):
    return make_mgsc_agent(kind, capacity, seed, preprocessor)
  rs = np.random.RandomState(seed)
  structure = replay_lib.Transition(None, None, None, None, None)
  if kind == 'double':
    from dqn_mgsc_zoo_amd.double_q import agent as agent_lib  # pylint: disable=g-import-not-at-top
    cls, net = agent_lib.DoubleDqn, networks.double_dqn_atari_network(6)
  else:
    from dqn_mgsc_zoo_amd.dqn import agent as agent_lib  # pylint: disable=g-import-not-at-top
    cls, net = agent_lib.Dqn, networks.dqn_atari_network(6)
  replay = replay_lib.TransitionReplay(capacity, structure, rs)
  return cls(
      preprocessor=preprocessor or RepeatStacker(),
      sample_network_input=np.zeros((84, 84, 4), np.uint8),
      network=net,
      optimizer=learner_lib.rmsprop(2.5e-4, 0.95, 0.01 / 32**2, centered=True),
      transition_accumulator=replay_lib.TransitionAccumulator(),
      replay=replay, batch_size=32,
      exploration_epsilon=parts.LinearSchedule(
          begin_t=0, decay_steps=1_000_000, begin_value=1.0, end_value=0.1),
      min_replay_capacity_fraction=0.05, learn_period=16,
      target_network_update_period=40_000, grad_error_bound=1.0 / 32,
      rng_key=np.array([0, seed], np.uint32))


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument('--frames', type=int, default=8000)
  ap.add_argument('--capacity', type=int, default=20_000)
  ap.add_argument('--kind', default='dqn', choices=['dqn', 'double', 'mgsc', 'mgsc_reservoir'])
  ap.add_argument('--env', default='stacked', choices=['stacked', 'atari-device', 'atari-host'],
                  help='stacked: pre-stacked 84x84 frames; atari-*: raw RGB frames through '
                       'processors.atari with the observation math on device or on the host')
  args = ap.parse_args()
  pre = None
  if args.env != 'stacked':
    from dqn_mgsc_zoo_amd import processors  # pylint: disable=g-import-not-at-top
    pre = processors.atari(observation_frame=host_atari_frame if args.env == 'atari-host' else None)
  agent = make_agent(args.kind, args.capacity, preprocessor=pre)
  times = {'act': 0.0, 'add': 0.0, 'learn': 0.0}
  counts = {'act': 0, 'add': 0, 'learn': 0}
  mgsc = args.kind.startswith('mgsc')
  if mgsc:
    times['meta'], counts['meta'] = 0.0, 0

  def wrap(name, fn):
    def inner(*a, **k):
      t0 = time.perf_counter()
      out = fn(*a, **k)
      times[name] += time.perf_counter() - t0
      counts[name] += 1
      return out
    return inner

  agent._act = wrap('act', agent._act)  # pylint: disable=protected-access
  agent._add = wrap('add', agent._add)  # pylint: disable=protected-access
  agent._learn = wrap('learn', agent._learn)  # pylint: disable=protected-access
  if mgsc:  # these agents add through the replay directly (agent.py:268-270)
    agent._meta_prioritization_learn = wrap('meta', agent._meta_prioritization_learn)  # pylint: disable=protected-access
    agent._replay.add = wrap('add', agent._replay.add)  # pylint: disable=protected-access
    # the meta step's host pieces (inside 'meta')
    for name, obj, attr in (('meta_batch', agent._replay, 'meta_batch_slots'),  # pylint: disable=protected-access
                            ('meta_online', agent.meta_learner, 'set_online_transition'),
                            ('meta_update', agent.meta_learner, 'update')):
      times[name], counts[name] = 0.0, 0
      setattr(obj, attr, wrap(name, getattr(obj, attr)))
  env = (fake_env.FakeAtari(episode_len=2000, seed=1) if args.env == 'stacked' else
         FakeRGBAtari(episode_len=2000, seed=1))
  loop = parts.run_loop(agent, env, max_steps_per_episode=0)
  warm = 4 * int(0.05 * args.capacity) + 256
  for _ in range(warm):
    next(loop)
  torch.cuda.synchronize()
  for k in times:
    times[k], counts[k] = 0.0, 0
  t0 = time.perf_counter()
  for _ in range(args.frames):
    next(loop)
  torch.cuda.synchronize()
  dt = time.perf_counter() - t0
  out = {'kind': args.kind, 'env': args.env, 'frames': args.frames, 'seconds': round(dt, 3),
         'frames_per_s': round(args.frames / dt, 1),
         'learner_steps_per_s': round(counts['learn'] / dt, 1),
         'us_per_frame': round(1e6 * dt / args.frames, 1)}
  for k in times:
    out['us_per_%s' % k] = round(1e6 * times[k] / max(1, counts[k]), 1)
    out['n_%s' % k] = counts[k]
  out['us_per_frame_outside'] = round(
      1e6 * (dt - sum(v for k, v in times.items() if not k.startswith('meta_'))) / args.frames, 1)
  print(json.dumps(out))


if __name__ == '__main__':
  main()
