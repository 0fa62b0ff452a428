"""CPU: the oracle's Atari observation restatement against its own sources.

rgb2y against numpy's tensordot (processors.py:367-371) and the BILINEAR
resize against PIL itself (processors.py:374-387) — the reference's
algorithm lives in those two dependencies, so they pin the oracle.
"""

import numpy as np
import pytest

from oracle import preprocess_ref

PIL = pytest.importorskip('PIL')
from PIL import Image  # noqa: E402  pylint: disable=g-import-not-at-top


def _pil_resize(img, h, w):
  return np.array(Image.fromarray(img).resize((w, h), Image.Resampling.BILINEAR),
                  dtype=np.uint8)


def test_rgb2y_matches_numpy_tensordot():
  rng = np.random.default_rng(0)
  rgb = rng.integers(0, 256, (1 << 20, 3), dtype=np.uint8)
  rgb[:4] = [[0, 0, 0], [255, 255, 255], [255, 0, 0], [0, 255, 255]]
  want = np.tensordot(rgb, [0.299, 0.587, 1 - (0.299 + 0.587)], (-1, 0)).astype(np.uint8)
  np.testing.assert_array_equal(preprocess_ref.rgb2y(rgb), want)


@pytest.mark.parametrize('shape', [(210, 160), (250, 160), (84, 84), (100, 300), (37, 53)])
def test_resize_matches_pil(shape):
  rng = np.random.default_rng(shape[0] * 1000 + shape[1])
  for _ in range(3):
    img = rng.integers(0, 256, shape, dtype=np.uint8)
    np.testing.assert_array_equal(preprocess_ref.resize_bilinear_u8(img, 84, 84),
                                  _pil_resize(img, 84, 84))
  # flat and saturated images hit the clip at both ends
  for v in (0, 255):
    img = np.full(shape, v, np.uint8)
    np.testing.assert_array_equal(preprocess_ref.resize_bilinear_u8(img, 84, 84),
                                  _pil_resize(img, 84, 84))


def test_atari_frame_pipeline():
  rng = np.random.default_rng(7)
  a = rng.integers(0, 256, (210, 160, 3), dtype=np.uint8)
  b = rng.integers(0, 256, (210, 160, 3), dtype=np.uint8)
  pooled = np.max(np.stack([a, b]), axis=0)
  y = np.tensordot(pooled, [0.299, 0.587, 1 - (0.299 + 0.587)], (-1, 0)).astype(np.uint8)
  np.testing.assert_array_equal(preprocess_ref.atari_frame([a, b]), _pil_resize(y, 84, 84))
