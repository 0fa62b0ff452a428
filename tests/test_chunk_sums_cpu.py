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
