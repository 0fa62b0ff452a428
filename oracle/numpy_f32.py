"""ORACLE — test infrastructure only.  Never imported by the product.

Restatement of the float32 arithmetic numpy performs in the reference's
learned-logit sampling (replay_circular.py:69-76 probabilities_from_logits /
logsumexp; :205-217 and :540-545 Generator.choice(C, n, p=...)), written out
operation by operation so that libdqz's exact sampling mode
(sampling.hpp np_expf / np_logf / npx_* kernels) can follow the same
operations and the tests can pin both:

  * exp_f32: numpy's SIMD float32 exp (AVX2 / AVX512F loops of
    numpy/_core/src/umath/loops_exponent_log.dispatch.c.src): Cody-Waite
    range reduction x = q ln2 + r, q = rint(x log2 e) by the 1.5 * 2^23
    magic add, exp(r) = P(r) / Q(r) (degree 5 / 2, fused multiply-adds),
    times 2^q; x >= 88.7228... -> inf, x <= -103.972... -> 0.
  * log_f32: numpy's SIMD float32 log: x = m 2^e, m in [0.5, 1); m <=
    sqrt(0.5) -> (2m, e) else (m, e + 1); log = P(m - 1) / Q(m - 1) (degree
    5 / 5) + e ln 2, fused.
  * sum_f32: np.sum of a contiguous float32 array: the reduction runs over
    8192-element buffers (np.getbufsize()), each summed by numpy's pairwise
    summation (8 accumulators below 128 elements, halves rounded down to a
    multiple of 8 above), the buffer sums added in order.

The polynomial constants are the float32 values in numpy's compiled
_multiarray_umath (numpy 2.2.6 here); tests/test_numpy_f32_cpu.py checks
every function against numpy itself, bit for bit, on millions of inputs.
numpy on a CPU without AVX2 uses libm instead, so "the reference's draws"
are those of an x86-64 host with AVX2 or AVX-512 (every host here).
"""

import numpy as np

f32 = np.float32

EXP_P = [f32(1.0), f32(7.257664613233124478488e-01), f32(2.473615434895520810817e-01),
         f32(5.114512081637298353406e-02), f32(6.757896990527504603057e-03), f32(5.082762527590693718096e-04)]
EXP_Q = [f32(1.0), f32(-2.742335390411667452936e-01), f32(2.159509375685829852307e-02)]
EXP_C1 = f32(-6.93145752e-1)
EXP_C2 = f32(-1.42860677e-6)
EXP_MAGIC = f32(12582912.0)  # 1.5 * 2^23
LOG2E = f32(1.442695040888963407359924681001892137)
EXP_XMAX = f32(88.72283935546875)
EXP_XMIN = f32(-103.97208404541015625)

LOG_P = [f32(0.0), f32(9.999999999999998702752e-01), f32(2.112677543073053063722e+00),
         f32(1.480000633576506585156e+00), f32(3.808837741388407920751e-01), f32(2.589979117907922693523e-02)]
LOG_Q = [f32(1.0), f32(2.612677543073109236779e+00), f32(2.453006071784736363091e+00),
         f32(9.864942958519418960339e-01), f32(1.546476374983906719538e-01),
         np.array([0x3bc083df], np.uint32).view(np.float32)[0]]
LN2 = f32(0.693147180559945309417232121458176568)
SQRT_HALF = np.array([0x3f3504f3], np.uint32).view(np.float32)[0]

PW_BLOCK = 128   # numpy's PW_BLOCKSIZE
BUFSIZE = 8192   # np.getbufsize()


def fma(a, b, c):
  """float32 fused multiply-add, exact: a*b is exact in float64; a + b's
  float64 rounding can only matter when it lands exactly on a float32
  rounding midpoint, where the TwoSum error term breaks the tie."""
  a = np.asarray(a, np.float32).astype(np.float64)
  b = np.asarray(b, np.float32).astype(np.float64)
  c = np.asarray(c, np.float32).astype(np.float64)
  p = a * b
  s = p + c
  bb = s - p
  err = (p - (s - bb)) + (c - bb)
  r = s.astype(np.float32)
  r64 = r.astype(np.float64)
  with np.errstate(all='ignore'):
    other = np.where(r64 > s, np.nextafter(r, np.float32(-np.inf)),
                     np.nextafter(r, np.float32(np.inf))).astype(np.float64)
    mid = (s - r64) == (other - s)  # s exactly between r and its neighbour
  pick = mid & (((other > r64) & (err > 0)) | ((other < r64) & (err < 0)))
  out = np.where(pick, other, r64)
  return out.astype(np.float32)


def exp_f32(x):
  x = np.asarray(x, np.float32)
  with np.errstate(all='ignore'):
    nan = np.isnan(x)
    xs = np.where(nan, f32(0), x).astype(np.float32)
    q = (xs * LOG2E).astype(np.float32)
    q = ((q + EXP_MAGIC).astype(np.float32) - EXP_MAGIC).astype(np.float32)
    r = fma(q, EXP_C1, xs)
    r = fma(q, EXP_C2, r)
    r = fma(q, f32(0), r)
    num = fma(EXP_P[5], r, EXP_P[4])
    for c in (EXP_P[3], EXP_P[2], EXP_P[1], EXP_P[0]):
      num = fma(num, r, c)
    den = fma(EXP_Q[2], r, EXP_Q[1])
    den = fma(den, r, EXP_Q[0])
    v = (num / den).astype(np.float32)
    out = np.ldexp(v, np.where(np.isfinite(q), q, 0).astype(np.int32)).astype(np.float32)
    out = np.where(xs <= EXP_XMIN, f32(0), out)
    out = np.where(xs >= EXP_XMAX, f32(np.inf), out)
    out = np.where(nan, x, out)
  return out.astype(np.float32)


def log_f32(x):
  """Positive normal inputs (a sum of exponentials is >= 1 here)."""
  x = np.asarray(x, np.float32)
  bits = x.view(np.uint32)
  e = ((bits >> 23) & 0xFF).astype(np.float32) - f32(127)
  m = ((bits & 0x7FFFFF) | (126 << 23)).astype(np.uint32).view(np.float32)
  small = m <= SQRT_HALF
  y = np.where(small, (m + m).astype(np.float32), m).astype(np.float32)
  e = np.where(small, e, (e + f32(1)).astype(np.float32)).astype(np.float32)
  y = (y - f32(1)).astype(np.float32)
  num = fma(LOG_P[5], y, LOG_P[4])
  for c in (LOG_P[3], LOG_P[2], LOG_P[1], LOG_P[0]):
    num = fma(num, y, c)
  den = fma(LOG_Q[5], y, LOG_Q[4])
  for c in (LOG_Q[3], LOG_Q[2], LOG_Q[1], LOG_Q[0]):
    den = fma(den, y, c)
  p = (num / den).astype(np.float32)
  return fma(e, LN2, p)


def pairwise_f32(a):
  """numpy's pairwise summation of a float32 vector (one buffer)."""
  a = np.asarray(a, np.float32)
  n = len(a)
  if n < 8:
    r = f32(0)
    for v in a:
      r = f32(r + v)
    return r
  if n <= PW_BLOCK:
    r = a[:8].copy()
    i = 8
    while i < n - n % 8:
      r = (r + a[i:i + 8]).astype(np.float32)
      i += 8
    res = f32(f32(f32(r[0] + r[1]) + f32(r[2] + r[3])) + f32(f32(r[4] + r[5]) + f32(r[6] + r[7])))
    for v in a[i:]:
      res = f32(res + v)
    return res
  n2 = n // 2
  n2 -= n2 % 8
  return f32(pairwise_f32(a[:n2]) + pairwise_f32(a[n2:]))


def sum_f32(a):
  a = np.asarray(a, np.float32)
  res = f32(0)
  for lo in range(0, len(a), BUFSIZE):
    res = f32(res + pairwise_f32(a[lo:lo + BUFSIZE]))
  return res


def logsumexp_f32(x):
  """replay_circular.py:73-76 in numpy's float32 operations."""
  x = np.asarray(x, np.float32)
  c = x.max()
  return f32(c + log_f32(np.array([sum_f32(exp_f32((x - c).astype(np.float32)))], np.float32))[0])


def probabilities_f32(x):
  """replay_circular.py:69-71."""
  x = np.asarray(x, np.float32)
  return exp_f32((x - logsumexp_f32(x)).astype(np.float32))
