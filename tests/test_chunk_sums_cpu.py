"""The numpy restatement of the device's chunk sums (sampling.hpp chunk_sum,
used by the GPU tests as the exact reference) checked on the CPU: it is a sum
of every chunk's terms (against float64 sums), exact when no partial sum
rounds (small integers), and zero-padded past the buffer's end."""
import numpy as np

from tests import helpers


def test_canonical_chunk_sums_are_the_chunk_totals():
  rng = np.random.default_rng(0)
  t = np.exp(rng.standard_normal(3 * 4096 + 123)).astype(np.float32)
  got = helpers.canonical_chunk_sums(t)
  assert got.shape == (4,)
  want = np.add.reduceat(t.astype(np.float64), np.arange(0, t.size, 4096))
  np.testing.assert_allclose(got, want, rtol=1e-13)


def test_canonical_chunk_sums_exact_on_integers_and_empty_slots():
  t = np.arange(2 * 4096, dtype=np.float32) % 7
  t[::5] = 0.0  # empty slots contribute exactly zero
  got = helpers.canonical_chunk_sums(t)
  want = [float(t[:4096].astype(np.int64).sum()), float(t[4096:].astype(np.int64).sum())]
  assert got.tolist() == want


def _dpp_fold63(v):
  """sampling.hpp block_total_f64's wave step (common.hpp wave_fold63_f64):
  row_shr 1/2/4/8 inside 16-lane rows (lanes whose source leaves the row
  read 0), then row_bcast 15 into rows 1 and 3 and row_bcast 31 into rows 2
  and 3; lane 63's value."""
  v = v.copy()
  pos = np.arange(64)
  for o in (1, 2, 4, 8):
    ok = (pos % 16) >= o
    v = v + np.where(ok, v[np.clip(pos - o, 0, 63)], 0.0)
  rows = pos // 16
  m = (rows == 1) | (rows == 3)
  d = np.zeros(64)
  d[m] = v[16 * rows[m] - 1]
  v = np.where(m, v + d, v)
  m = rows >= 2
  d = np.zeros(64)
  d[m] = v[31]
  v = np.where(m, v + d, v)
  return v[63]


def test_dpp_fold_has_the_scan_last_lane_bits():
  """The chunk totals are formed by a DPP fold (no scan) and must keep the
  bits of the Hillis-Steele scan's last lane that canonical_chunk_sums (and
  the sampler's in-chunk scan) use: the same additions happen in lane 63."""
  rng = np.random.default_rng(1)
  for _ in range(300):
    lanes = (rng.random(256) * np.exp(rng.normal(0.0, 6.0, 256))).astype(np.float32)
    lanes[rng.random(256) < 0.3] = 0.0
    lanes = lanes.astype(np.float64)
    w = [_dpp_fold63(lanes[64 * k:64 * k + 64]) for k in range(4)]
    got = w[3] + ((w[0] + w[1]) + w[2])
    t = np.zeros(4096, np.float32)  # lane l's 16 terms: its value, then zeros
    t[::16] = lanes
    assert got == helpers.canonical_chunk_sums(t)[0]
