"""Atari observation preprocessing per emitted step: the reference's host
path (np.stack + np.max + rgb2y tensordot + PIL BILINEAR resize,
processors.py:488-497) vs dqz_atari_frame (one launch, pinned in/out).

usage (GPU box): python tools/preprocess_bench.py [--iters N]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from dqn_mgsc_zoo_amd import processors  # noqa: E402


def host_frame(obs):
  pooled = np.max(np.stack(obs[-2:], axis=0), axis=0)
  y = np.tensordot(pooled, [0.299, 0.587, 1 - (0.299 + 0.587)], (-1, 0)).astype(np.uint8)
  return np.array(Image.fromarray(y).resize((84, 84), Image.Resampling.BILINEAR), dtype=np.uint8)


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument('--iters', type=int, default=2000)
  args = ap.parse_args()
  rng = np.random.default_rng(0)
  obs = [rng.integers(0, 256, (210, 160, 3), dtype=np.uint8) for _ in range(4)]
  dev = processors.DeviceAtariFrame(2)
  assert np.array_equal(dev(obs), host_frame(obs))
  out = {}
  for name, fn in (('host_numpy_pil', host_frame), ('device', dev)):
    for _ in range(50):
      fn(obs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.iters):
      fn(obs)
    torch.cuda.synchronize()
    out['us_per_frame_' + name] = round(1e6 * (time.perf_counter() - t0) / args.iters, 2)
  print(json.dumps(out))


if __name__ == '__main__':
  main()
