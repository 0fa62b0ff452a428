"""CPU checks of the arithmetic behind conv1's bf16 MFMA path (csrc/conv1.hpp).

* split3_bf16: w == hi + mid + lo exactly, each piece a bf16 (low 16 bits of
  its f32 pattern zero), for f32 values across the weight / gradient range;
* a pixel (integer 0..255) times a piece is exact in f32 (8 x 8 significant
  bits), so the MFMA sums exact products;
* div255 (reciprocal product + one FMA residual) is within one ulp of the
  IEEE quotient x / 255 (and equal to it for nearly all x).

The device code is restated here with numpy float32 / float64 (an f32 FMA is
the float64 value of a*b + c rounded once to f32: the products involved have
at most 48 significant bits).
"""

import numpy as np

MASK = np.uint32(0xFFFF0000)


def _split3(w):
  w = np.asarray(w, np.float32)
  hi = (w.view(np.uint32) & MASK).view(np.float32)
  r1 = (w - hi).astype(np.float32)
  mid = (r1.view(np.uint32) & MASK).view(np.float32)
  lo = (r1 - mid).astype(np.float32)
  return hi, mid, lo


def _values(n, seed):
  rng = np.random.default_rng(seed)
  mag = 10.0 ** rng.uniform(-30, 3, n)
  return (rng.choice([-1.0, 1.0], n) * mag).astype(np.float32)


def test_split3_is_exact_and_bf16():
  w = np.concatenate([_values(200000, 0), np.float32([0.0, 1.0, -1.0, 3.1415927, 1e-30])])
  hi, mid, lo = _split3(w)
  for piece in (hi, mid, lo):
    assert not np.any(piece.view(np.uint32) & np.uint32(0xFFFF))  # a bf16 value
  total = hi.astype(np.float64) + mid.astype(np.float64) + lo.astype(np.float64)
  np.testing.assert_array_equal(total, w.astype(np.float64))
  # piece magnitudes (truncated pieces: |mid| < 2^-7 |w|, |lo| < 2^-15 |w|)
  nz = w != 0
  assert np.all(np.abs(mid[nz]) < 2.0 ** -7 * np.abs(w[nz]))
  assert np.all(np.abs(lo[nz]) < 2.0 ** -15 * np.abs(w[nz]))


def test_pixel_times_piece_is_exact_in_f32():
  pix = np.arange(256, dtype=np.float32)
  for piece in _split3(_values(4096, 1)):
    prod32 = (pix[:, None] * piece[None, :]).astype(np.float32)
    prod64 = pix[:, None].astype(np.float64) * piece[None, :].astype(np.float64)
    np.testing.assert_array_equal(prod32.astype(np.float64), prod64)


def _f32_fma(a, b, c):
  return (np.float64(a) * np.float64(b) + np.float64(c)).astype(np.float32)


def test_div255_within_one_ulp():
  rng = np.random.default_rng(2)
  s = np.concatenate([rng.uniform(-3e4, 3e4, 200000), rng.integers(-65280, 65280, 20000)]).astype(np.float32)
  r = np.float32(1.0) / np.float32(255.0)
  q = (s * r).astype(np.float32)
  e = _f32_fma(-q, np.float32(255.0), s)
  got = _f32_fma(e, r, q)
  want = (s.astype(np.float64) / 255.0).astype(np.float32)  # the IEEE f32 quotient
  ulp = np.spacing(np.abs(want))
  assert np.all(np.abs(got.astype(np.float64) - want.astype(np.float64)) <= ulp)
  assert np.mean(got == want) > 0.999
