"""CPU restatement of the Atari observation pipeline (test infrastructure).

Checker for the device kernel `dqz_atari_frame`.  Only tests/ may import it.
Follows processors.atari's observation branch (processors.py:488-505):

  np.max(stack of the last 2 RGB frames)   max-pool
  rgb2y                                    processors.py:367-371
  resize((84, 84))                         processors.py:374-387 (PIL BILINEAR)

rgb2y is `np.tensordot(rgb, [0.299, 0.587, 1 - (0.299 + 0.587)], (-1, 0))`
then `.astype(np.uint8)`.  numpy evaluates that dot with OpenBLAS; on this
image its result equals fma(b, w2, fma(r, w0, g * w1)) in float64 for all
2^24 RGB triples (checked exhaustively when this file was written; the
reference pins numpy 1.21.5 / its own OpenBLAS, docker_requirements.txt:24,
whose dot may round ~500 of the 2^24 triples differently — parity is pinned
to the numpy of this image).

PIL's BILINEAR resize of an 8-bit image ('L') is Pillow's two-pass
fixed-point resampler (libImaging/Resample.c; Pillow 10.0.0 in the
reference, docker_requirements.txt:25; 12.2.0 here, same algorithm):
per output coordinate a triangle filter of support 1 scaled by the
reduction factor, normalised double weights converted to int32 with 22
fractional bits (round half away from zero), accumulation from 2^21 and an
arithmetic shift + clip to [0, 255]; the horizontal pass runs first over
the source rows the vertical pass needs.  `resize_bilinear_u8` restates it;
tests/test_preprocess.py checks it against PIL itself.
"""

import math

import numpy as np

PRECISION_BITS = 32 - 8 - 2
RGB2Y_W = (0.299, 0.587, 1 - (0.299 + 0.587))


def _fma(a, x, c):
  # a: small non-negative integers (exact in float64), x, c float64: the
  # product a*x fits the 64-bit long-double mantissa exactly, so one
  # long-double add + rounding to float64 is the fused multiply-add.
  return (np.asarray(a, np.longdouble) * np.longdouble(x) +
          np.asarray(c, np.longdouble)).astype(np.float64)


def rgb2y(rgb):
  """uint8 [..., 3] -> uint8 [...] as numpy's tensordot rounds it here."""
  rgb = np.asarray(rgb)
  r, g, b = (rgb[..., i].astype(np.float64) for i in range(3))
  w0, w1, w2 = RGB2Y_W
  return _fma(b, w2, _fma(r, w0, g * w1)).astype(np.uint8)


def precompute_coeffs(in_size, out_size):
  """(bounds [out][2] = (first, count), int32 coefficients [out][ksize]) of
  Pillow's BILINEAR filter for one axis (box = (0, in_size))."""
  scale = float(in_size) / out_size
  filterscale = max(scale, 1.0)
  support = 1.0 * filterscale
  ksize = int(math.ceil(support)) * 2 + 1
  bounds = np.zeros((out_size, 2), np.int64)
  kk = np.zeros((out_size, ksize), np.float64)
  ss = 1.0 / filterscale
  for xx in range(out_size):
    center = (xx + 0.5) * scale
    xmin = max(int(center - support + 0.5), 0)
    xmax = min(int(center + support + 0.5), in_size) - xmin
    ws = []
    for x in range(xmax):
      t = abs((x + xmin - center + 0.5) * ss)
      ws.append(1.0 - t if t < 1.0 else 0.0)
    ww = 0.0
    for w in ws:
      ww += w
    for x, w in enumerate(ws):
      kk[xx, x] = w / ww if ww != 0.0 else w
    bounds[xx] = (xmin, xmax)
  one = float(1 << PRECISION_BITS)
  ik = np.where(kk < 0, np.trunc(-0.5 + kk * one), np.trunc(0.5 + kk * one)).astype(np.int64)
  return bounds, ik


def _clip8(acc):
  return np.clip(acc >> PRECISION_BITS, 0, 255).astype(np.uint8)


def resize_bilinear_u8(img, out_h, out_w):
  """Image.fromarray(img).resize((out_w, out_h), BILINEAR) for uint8 [h, w]."""
  img = np.asarray(img, np.uint8)
  in_h, in_w = img.shape
  hb, hk = precompute_coeffs(in_w, out_w)
  vb, vk = precompute_coeffs(in_h, out_h)
  y_first = int(vb[0, 0])
  y_last = int(vb[-1, 0] + vb[-1, 1])
  rows = img[y_first:y_last].astype(np.int64)
  tmp = np.empty((y_last - y_first, out_w), np.uint8)
  for xx in range(out_w):
    x0, n = hb[xx]
    acc = np.full(rows.shape[0], 1 << (PRECISION_BITS - 1), np.int64)
    for x in range(n):
      acc += rows[:, x0 + x] * hk[xx, x]
    tmp[:, xx] = _clip8(acc)
  t = tmp.astype(np.int64)
  out = np.empty((out_h, out_w), np.uint8)
  for yy in range(out_h):
    y0, n = vb[yy]
    y0 -= y_first
    acc = np.full(out_w, 1 << (PRECISION_BITS - 1), np.int64)
    for y in range(n):
      acc += t[y0 + y] * vk[yy, y]
    out[yy] = _clip8(acc)
  return out


def atari_frame(rgb_frames, out_h=84, out_w=84):
  """max-pool of the given RGB frames -> rgb2y -> BILINEAR resize."""
  pooled = np.max(np.stack(rgb_frames, axis=0), axis=0)
  return resize_bilinear_u8(rgb2y(pooled), out_h, out_w)
