"""processors.atari against the reference's own outputs (tests/golden/
processors_golden.json, recorded from dqn_zoo/processors.py by
tests/golden/make_processors_golden.py on synthetic (rgb, lives) episodes).

CPU: the control flow (action-repeat buffer, subsampling, reward / discount
aggregation, life loss, stacking) with the oracle's observation restatement
plugged in.  GPU: the default device observation path (dqz_atari_frame).
Observations are compared by SHA-256 of their bytes: bit-exact.
"""

import hashlib
import json
import os

import numpy as np
import pytest

from oracle import preprocess_ref
from tests.golden import make_processors_golden as gen

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden',
                      'processors_golden.json')


def _replay_case(processors, case, frame_fn):
  kw = {} if frame_fn is None else {'observation_frame': frame_fn}
  p = processors.atari(**kw)
  got = []
  for kind, ts in gen.episode_stream(case['seed'], case['episodes'], tuple(case['shape'])):
    if kind == 'reset':
      processors.reset(p)
      got.append('reset')
      continue
    o = p(ts)
    if o is None:
      got.append(None)
      continue
    got.append({'step_type': int(o.step_type),
                'reward': None if o.reward is None else float(o.reward),
                'discount': None if o.discount is None else float(o.discount),
                'shape': list(o.observation.shape), 'dtype': str(o.observation.dtype),
                'sha256': hashlib.sha256(np.ascontiguousarray(o.observation).tobytes()).hexdigest()})
  return got


def _check(frame_fn):
  from dqn_mgsc_zoo_amd import processors
  golden = json.load(open(GOLDEN))
  for case in golden['cases']:
    got = _replay_case(processors, case, frame_fn)
    assert len(got) == len(case['outputs'])
    for i, (g, w) in enumerate(zip(got, case['outputs'])):
      assert g == w, 'seed %d record %d: %s != %s' % (case['seed'], i, g, w)


def test_atari_processor_control_flow_matches_reference():
  _check(lambda obs: preprocess_ref.atari_frame(list(obs)[-2:]))


@pytest.mark.gpu
def test_atari_processor_device_matches_reference(device):
  _check(None)


@pytest.mark.gpu
def test_device_atari_frame_matches_pil(device):
  """dqz_atari_frame vs the oracle (itself pinned to PIL) on random frames,
  one and two pooled frames, Atari and odd sizes (byte path)."""
  from dqn_mgsc_zoo_amd import processors
  rng = np.random.default_rng(5)
  for shape in ((210, 160), (250, 160), (37, 53), (84, 84)):
    dev = processors.DeviceAtariFrame(2)
    for n in (1, 2):
      frames = [rng.integers(0, 256, shape + (3,), dtype=np.uint8) for _ in range(n)]
      np.testing.assert_array_equal(dev(frames), preprocess_ref.atari_frame(frames),
                                    err_msg='%s n=%d' % (shape, n))
    # extremes: all-zero and all-255 frames
    for v in (0, 255):
      frames = [np.full(shape + (3,), v, np.uint8)] * 2
      np.testing.assert_array_equal(dev(frames), preprocess_ref.atari_frame(frames))
