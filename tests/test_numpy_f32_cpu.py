"""oracle/numpy_f32.py against numpy itself, bit for bit: the float32 exp,
log and sum numpy runs in the reference's probabilities_from_logits /
logsumexp (replay_circular.py:69-76), and the probabilities and choices of
whole learned-logit buffers (the exact sampling mode's reference)."""
import numpy as np
import pytest

from oracle import numpy_f32 as nf
from oracle import replay_ref


def _eq(a, b):
  a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
  assert a.shape == b.shape
  assert (a.view(np.uint32) == b.view(np.uint32)).all(), int((a.view(np.uint32) != b.view(np.uint32)).sum())


def test_fma_is_the_rounded_exact_product_sum():
  rng = np.random.default_rng(0)
  a = rng.standard_normal(20000).astype(np.float32)
  b = rng.standard_normal(20000).astype(np.float32)
  c = rng.standard_normal(20000).astype(np.float32)
  from fractions import Fraction
  got = nf.fma(a, b, c)
  for i in range(0, 20000, 97):
    exact = Fraction(float(a[i])) * Fraction(float(b[i])) + Fraction(float(c[i]))
    lo = np.float32(float(exact))
    # nearest float32 to the exact value (ties to even)
    cands = [np.nextafter(lo, np.float32(-np.inf)), lo, np.nextafter(lo, np.float32(np.inf))]
    best = min(cands, key=lambda v: (abs(Fraction(float(v)) - exact), int(np.float32(v).view(np.uint32)) & 1))
    assert got[i] == best


def test_exp_matches_numpy():
  rng = np.random.default_rng(1)
  x = np.concatenate([rng.uniform(-110, 0, 1_000_000), rng.uniform(-1, 1, 200_000),
                      rng.uniform(-104.5, -86, 200_000), [0.0, -0.0, -np.inf, -103.97208404541015625,
                                                         -103.97207, 88.7228, -87.33654]]).astype(np.float32)
  _eq(nf.exp_f32(x), np.exp(x))


def test_log_matches_numpy():
  rng = np.random.default_rng(2)
  x = np.concatenate([np.exp(rng.uniform(-80, 80, 1_000_000)), rng.uniform(1, 2e6, 500_000),
                      [1.0, 2.0, 0.5, 0.70710677, 0.7071068, 1e6]]).astype(np.float32)
  _eq(nf.log_f32(x), np.log(x))


@pytest.mark.parametrize('n', [1, 7, 8, 100, 128, 129, 1000, 8192, 8193, 50_003, 1_000_000])
def test_sum_matches_numpy(n):
  rng = np.random.default_rng(n)
  a = np.exp(rng.standard_normal(n) * 3).astype(np.float32)
  a[rng.random(n) < 0.2] = 0.0
  _eq(nf.sum_f32(a), np.sum(a))


@pytest.mark.parametrize('n', [1000, 8193, 100_003, 1_000_000])
def test_probabilities_and_choice_match_numpy(n):
  rng = np.random.default_rng(7)
  x = (rng.standard_normal(n) * 2).astype(np.float32)
  x[rng.random(n) < 0.05] = -np.inf  # empty slots
  p = nf.probabilities_f32(x)
  _eq(p, replay_ref.softmax_f32(x))
  u = rng.random(64)
  p64 = p.astype(np.float64)
  cdf = np.cumsum(p64)
  cdf /= cdf[-1]
  np.testing.assert_array_equal(np.searchsorted(cdf, u, side='right'), replay_ref.softmax_choice(x, u))
